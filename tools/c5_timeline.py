"""Timeline of the last areas solve in a rocprofv3 kernel + memory-copy trace of
tools/c5_leg.py (tools/runs/gpu_c5.sh): every kernel and copy from the last
host-to-device copy of the batch on, with its start relative to that copy, its
duration and the gap before it."""
import csv
import sys

d = sys.argv[1]
ev = []
for r in csv.DictReader(open(f"{d}/kt_kernel_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:48], r["Queue_Id"]))
for r in csv.DictReader(open(f"{d}/kt_memory_copy_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"].replace("MEMORY_COPY_", ""), "copy"))
ev.sort()
h2d = [e for e in ev if e[2] == "HOST_TO_DEVICE" and e[1] - e[0] > 100000]
t0 = h2d[-1][0]
prev_end = t0
busy = 0
for s, e, name, q in ev:
    if s < t0:
        continue
    print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:7.1f} us  gap {(s - prev_end) / 1e3:7.1f}  q{q:>4}  {name}")
    busy += e - s
    prev_end = max(prev_end, e)
print(f"span {(prev_end - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
