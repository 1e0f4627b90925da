"""Instruction mix per basic block of one kernel in a hipcc --save-temps .s file.

    python tools/isa_mix.py file.s kernel_substring
"""
import collections
import re
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    lines = open(path).read().split('\n')
    start = next(i for i, l in enumerate(lines) if re.match(r'^_Z\S*' + re.escape(key) + r'\S*:', l))
    blocks, cur = [], None
    for l in lines[start + 1:]:
        t = l.strip()
        if t.startswith('.Lfunc_end'):
            break
        if re.match(r'^\.LBB\d+_\d+:', t):
            cur = [t[:-1], collections.Counter(), 0]
            blocks.append(cur)
            continue
        if not t or t.startswith(';') or t.startswith('.'):
            continue
        if cur is None:
            cur = ['entry', collections.Counter(), 0]
            blocks.append(cur)
        op = t.split()[0]
        cur[1][op] += 1
        cur[2] += 1
    tot = collections.Counter()
    for name, c, n in blocks:
        tot.update(c)
        f64 = sum(v for k, v in c.items() if k.endswith('_f64'))
        dpp = sum(v for k, v in c.items() if 'dpp' in k)
        ds = sum(v for k, v in c.items() if k.startswith('ds_'))
        valu = sum(v for k, v in c.items() if k.startswith('v_'))
        scr = sum(v for k, v in c.items() if k.startswith('scratch') or k.startswith('buffer_st') or k.startswith('buffer_lo'))
        print(f"{name:14s} n={n:5d} valu={valu:5d} f64={f64:4d} dpp={dpp:4d} ds={ds:4d} scratch={scr:3d} wait={c['s_waitcnt']:3d}")
    if '-v' in sys.argv:
        for k, v in tot.most_common():
            print(f"  {k:32s} {v}")


if __name__ == '__main__':
    main()
