// fpf_lane.hip -- the lane kernel (fast mode, fpf_opts.exact = 0): every sweep
// of DPF_return7 (Broker/src/vvc/DPF_return7.cpp:104-217) with ONE LANE PER
// SCENARIO, 64 scenarios per workgroup of LANE_NW = 8 wavefronts.
//
// The wave kernel (fpf_wave.hip) spreads one scenario over 32 lanes and pays for
// it in the sweep: a fp64 DPP scan moves every double as two 32-bit halves (31 %
// of its VALU), and ~100 LDS round trips per wave-sweep sit on the dependency
// chain.  Here a scenario's nodes are spread over the eight
// WAVES of a workgroup instead, and the 64 lanes of every wave are 64 scenarios:
//   * the depth-first order of the wave kernel (in-block child first, so every
//     subtree and every block is a contiguous range of positions) is dealt to the
//     waves in contiguous runs; position q of wave w lives in slot i = q - first_w,
//     its V (then its scan values) in that wave's registers for the whole solve --
//     x[16][3] complex, 192 VGPRs, two waves per SIMD;
//   * all of a slot's arithmetic is per lane: the load current, a sequential
//     prefix over the wave's slots, the branch drop -- no cross-lane moves at all;
//   * what differs between the waves (rows, TEMP, which scan values to publish or
//     gather) is wave-uniform data, read with scalar loads: every wave runs the
//     same code (one code body, instruction-cache friendly, no per-feeder build);
//   * the waves meet in LDS, in per-lane columns (lane l of every wave is
//     scenario l): the backward sweep is the prefix scan E of IL, Ib(q) =
//     E[last(q)] - E[q - 1], with the wave totals giving each wave its carry and
//     the subtree ends published; the forward sweep is the prefix scan G of the
//     drops, V(q) = V0 - off(block) - G[q], off(b) = sum over b's block-ancestor
//     chain of G[tap] - G[first - 1] (the wave kernel's algebra, fpf_wave.hip).
//     Four barriers per sweep: wave totals of E, published E, wave totals of G,
//     published G.
// The loads (P, Q) are read from the caller's scenario-fastest batch every sweep
// (64 consecutive doubles per load instruction, one slot ahead; FPF_LANE_DMA=1:
// through an LDS-DMA ring three slots ahead) -- 3.2x the algorithmic bytes beyond
// L2 (profiles/r06_c4lane), the design's bound.  A lane whose
// scenario has finished is frozen -- every update of a
// sweep runs under a divergent !done branch -- so its registers keep the V of its
// last sweep until the workgroup's last scenario is done; then every lane's V
// leaves in whole 512-byte rows (stored in the sweep each scenario finished, the
// rows went out in part-lines twice: +0.2 ms on config 4, profiles/r06_lane).
//
// Scope (fpf_api.cpp: analyse_lane): well-formed tree-order feeders of at most
// LANE_NW * LANE_NS = 128 branches, no zeroed phases, every branch's TEMP with one
// common off-diagonal value, light outputs (V, iters, status, loss, vmin, vmax,
// errmx, guard), scenario-fastest batches, the feeder's own source.  Everything
// else runs the wave kernel.
//
// Arithmetic: the wave kernel's quantities (refined-reciprocal load currents,
// symmetric-TEMP FMA drops, prefix-sum differences, the loss as s3 sum
// Re(drop conj(Ib))) in another association; checked at the north-star bar
// against the oracle (tests/test_gpu_lane.py).  The convergence guard's band
// covers this kernel's order of Ib(0): a sequential sum over <= 16 slots, then 8
// wave totals (<= 24 u sum |IL| against the band's 2 (Nb + 24) u).
#include <array>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <set>

#include "fpf_internal.h"
#include "fpf_math.hpp"
#include "fpf_wave_common.h"
#include "fpf_generic_body.h"

namespace fpf {

// diagnostic ablation builds (tools/runs: FPF_LANE_ABL bits; results are wrong
// when set): 1 the loads come from a constant instead of memory, 2 the backward
// gathers read the slot's own value instead of LDS, 4 every scenario takes
// exactly 5 sweeps (so that the other bits compare at equal work), 8 no
// reciprocal in the load currents.  The other switches are the measured
// alternatives of profiles/r06_lane (the defaults are the faster ones)
#ifndef FPF_LANE_ABL
#define FPF_LANE_ABL 0
#endif
// the carry loops' three reads issued together (measured slower: 1.151 vs 1.114 ms)
#ifndef FPF_LANE_LD3
#define FPF_LANE_LD3 0
#endif
#ifndef FPF_LANE_IL3
#define FPF_LANE_IL3 0   // (measured: no faster, and the register-load variant spills; profiles/r06_lane)
#endif
#ifndef FPF_LANE_SB
#define FPF_LANE_SB 1   // (bit 1: a scheduling barrier between the load currents' slots)
#endif
// slots of loads in flight ahead of the load currents (registers: 12 per slot;
// 2 and 3 spill)
#ifndef FPF_LANE_PF
#define FPF_LANE_PF 1
#endif

namespace {

#ifdef FPF_LANE_STAMPS
// diagnostic build only (tools/lane_stamps.py): lane 0 of each wave of the eight
// workgroups from fpf_lane_stamp_base on records s_memtime, [64][128]: 0 entry,
// 1 loop start, 4 + 10 it + k in sweep it < 12 (k: 0 top, 1 currents, 2 B1, 3
// carry + E published, 4 B2, 5 drops, 6 B3, 7 G published, 8 B4, 9 voltages),
// 120 after the loop, 121 V out, 122 end
__device__ unsigned long long *fpf_lane_stamp_buf = nullptr;
__device__ unsigned fpf_lane_stamp_base = 0;
#define LSTAMP(idx)                                                                                    \
    do {                                                                                               \
        const unsigned g_ = (blockIdx.x - fpf_lane_stamp_base) * LANE_NW + (threadIdx.x >> 6);        \
        if (fpf_lane_stamp_buf && (threadIdx.x & 63) == 0 && blockIdx.x >= fpf_lane_stamp_base &&     \
            g_ < 64u && (idx) < 128)                                                                   \
            fpf_lane_stamp_buf[g_ * 128 + (idx)] = __builtin_amdgcn_s_memtime();                       \
    } while (0)
#define LSTAMP_IT(k) LSTAMP(it < 12 ? 4 + 10 * it + (k) : 999)
#else
#define LSTAMP(idx) ((void)0)
#define LSTAMP_IT(k) ((void)0)
#endif

typedef const __attribute__((address_space(4))) double cdbl;      // constant address space:
typedef const __attribute__((address_space(4))) int32_t cint;     // scalar loads


// every wave's LDS stores before it, every wave's LDS reads after it; the vector
// memory loads in flight (the next slots' P, Q) are not waited for
__device__ __forceinline__ void lane_barrier() { __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// a slot's new values stay where they are computed: without it the compiler
// sinks each slot's V = cb - G to the loop latch (its only other use), keeping
// every slot's block constant alive across the phase (12 registers per slot)
__device__ __forceinline__ void pin(cx (&v)[3]) {
    __asm__ volatile("" : "+v"(v[0].re), "+v"(v[0].im), "+v"(v[1].re), "+v"(v[1].im), "+v"(v[2].re), "+v"(v[2].im));
}

__device__ __forceinline__ cx ldc(const double2 *a, int i) {
    const double2 v = a[i];
    return mk(v.x, v.y);
}
// a wave's three phase entries (stride 64): the three reads issued together, one
// wait (else the compiler reuses one register quad and waits after each)
__device__ __forceinline__ void ld3(cx (&t)[3], const double2 *a, int i) {
#pragma unroll
    for (int p = 0; p < 3; ++p) t[p] = ldc(a, i + p * 64);
    if (FPF_LANE_LD3)
        __asm__ volatile("" : "+v"(t[0].re), "+v"(t[0].im), "+v"(t[1].re), "+v"(t[1].im), "+v"(t[2].re), "+v"(t[2].im));
}
__device__ __forceinline__ void stc(double2 *a, int i, cx v) { a[i] = make_double2(v.re, v.im); }

// buffer resources on wave-uniform bases (scalar registers) with the lane's
// 32-bit offset: no 64-bit address per load or store lives in vector registers.
// The loads [6][Nl][B]: one resource on the batch, element (f, row) of this
// lane's scenario at byte ((f Nl + row) B + s) 8 = a scalar offset (f Nl + row)
// 8B plus the lane's 8s (the host keeps the batch below 4 GiB, fpf_api.cpp)
__device__ __forceinline__ __attribute__((ext_vector_type(2))) unsigned bits2(double v) {
    return __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v);
}
// a wave-uniform pointer parked in LDS (read where it is used, into scalar registers)
__device__ __forceinline__ double *lds_ptr(const uint64_t *a, int k) {
    const uint64_t v = a[k];
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return (double *)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ void load_pq(double (&d)[6], __amdgpu_buffer_rsrc_t rp, int row, unsigned plane,
                                        unsigned bb, unsigned vo) {
    const unsigned ro = (unsigned)row * bb;
#pragma unroll
    for (int f = 0; f < 6; ++f) {
        if (FPF_LANE_ABL & 1) d[f] = 1e-3 * (f + 1) + 1e-6 * row + 1e-9 * vo;
        else d[f] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rp, vo, ro + f * plane, 0));
    }
}

// ---- the loads through LDS-DMA (the DMA variant: no VGPR holds a load in flight,
// so they run three slots ahead).  A wave's ring has two entries of [6][64]
// doubles (one slot's P1 Q1 P2 Q2 P3 Q3 of its 64 scenarios); a slot is three
// 16-byte pieces per lane -- lanes 0-31 field 2k, lanes 32-63 field 2k + 1, lane
// l scenarios s0 + 2 (l % 32) and + 1 -- each piece one wave instruction writing
// 1 KiB of LDS at M0 + 16 lane.  hipcc does not count these loads: the waits for
// them are explicit (vm_wait) and the ring entry is overwritten only after the
// wave's own reads of it are done (lgkmcnt(0) in the same statement).
typedef unsigned __attribute__((ext_vector_type(4))) u4;
// (issued with every lane on: a lane's piece carries its neighbours' scenarios,
// and the load currents run under the divergent !done branch)
__device__ __forceinline__ void dma_piece(u4 rsrc, unsigned vo, unsigned so, unsigned lds_addr) {
    unsigned keep;
    unsigned long long ex;
    __asm__ volatile(
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_mov_b64 %1, exec\n\t"
        "s_mov_b64 exec, -1\n\t"
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %4\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %2, %3, %5 offen lds\n\t"
        "s_mov_b32 m0, %0\n\t"
        "s_mov_b64 exec, %1"
        : "=&s"(keep), "=&s"(ex)
        : "v"(vo), "s"(rsrc), "s"(lds_addr), "s"(so)
        : "memory");
}
// one slot's three pieces: row offset row B 8, field pair k at + 2 k plane
__device__ __forceinline__ void dma_slot(u4 rsrc, unsigned vo, int row, unsigned bb, unsigned plane2, unsigned lds_addr) {
    if (FPF_LANE_ABL & 1) return;
    int r = row;
    __asm__ volatile("" : "+s"(r));   // (the offsets here, not hoisted)
    const unsigned ro = (unsigned)r * bb;
#pragma unroll
    for (int k = 0; k < 3; ++k) dma_piece(rsrc, vo, ro + k * plane2, lds_addr + k * 1024);
}
// every vector memory operation but the newest three (one slot's pieces) done, or all
__device__ __forceinline__ void vm_wait(bool leave3) {
    if (leave3) __asm__ volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// a slot's six values of this lane's scenario from a ring entry
__device__ __forceinline__ void ring_read(double (&d)[6], const double *e, int lane, int row, unsigned vo) {
#pragma unroll
    for (int f = 0; f < 6; ++f) d[f] = (FPF_LANE_ABL & 1) ? 1e-3 * (f + 1) + 1e-6 * row + 1e-9 * vo : e[f * 64 + lane];
}

}  // namespace

// one sweep's phases on the wave's NS slots (every slot is live: a wave's run of
// positions is padded with dummy slots whose loads scale by 0 and whose TEMP is 0,
// so their IL, Ib and drop are exactly 0 and no slot needs a branch)
template <int NS>
struct LaneSweep {
    // a slot's load currents IL = conj(S/V) = conj(S) V / |V|^2 (one refined
    // reciprocal per phase) added to the wave's local prefix.  FPF_LANE_IL3: the
    // three phases' chains in lockstep, stage by stage (the scheduler otherwise
    // runs them one after another at this register pressure: ~11 dependent fp64
    // steps each)
    __device__ __forceinline__ static void slot_currents(cx (&x)[NS][3], int i, const double (&sc)[6], double isc) {
        double d2[3], r[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) d2[p] = fma(x[i][p].re, x[i][p].re, x[i][p].im * x[i][p].im);
        if (FPF_LANE_IL3) __asm__ volatile("" : "+v"(d2[0]), "+v"(d2[1]), "+v"(d2[2]));
#pragma unroll
        for (int p = 0; p < 3; ++p) r[p] = (FPF_LANE_ABL & 8) ? d2[p] : __builtin_amdgcn_rcp(d2[p]);
        if (FPF_LANE_IL3) __asm__ volatile("" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]));
#pragma unroll
        for (int p = 0; p < 3; ++p) r[p] = fma(r[p], fma(-d2[p], r[p], 1.0), r[p]) * isc;
        if (FPF_LANE_IL3) __asm__ volatile("" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]));
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const double P = sc[2 * p], Q = sc[2 * p + 1];
            const cx v = x[i][p];
            const cx il = mk(fma(P, v.re, Q * v.im) * r[p], fma(P, v.im, -(Q * v.re)) * r[p]);
            x[i][p] = i == 0 ? il : cadd(x[i - 1][p], il);
        }
    }
    // ---- load currents (:106-130) and the wave's local prefix E of IL; the flat
    // start's first sweep is the same arithmetic on x = V0 (DPF_return7.cpp:92-96),
    // plus the guard's sum |S|_1 (a branch on one register only).  The loads run
    // FPF_LANE_PF slots ahead (sn[k]: slot i + 1 + k); the rows come from the
    // wave's row table, read once per phase
    __device__ __forceinline__ static void currents(cx (&x)[NS][3], double &sabs, bool flat, double (&sn)[FPF_LANE_PF][6],
                                                    __amdgpu_buffer_rsrc_t rp, cint *tab, unsigned plane, unsigned bb,
                                                    unsigned so, double inv_s3) {
        int row[NS], ei[NS];
#pragma unroll
        for (int i = 0; i < NS; ++i) row[i] = tab[i];
#pragma unroll
        for (int i = 0; i < NS; ++i) ei[i] = tab[2 * NS + i];
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            double sc[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) sc[k] = sn[0][k];
#pragma unroll
            for (int j = 0; j + 1 < FPF_LANE_PF; ++j)
#pragma unroll
                for (int k = 0; k < 6; ++k) sn[j][k] = sn[j + 1][k];
            if (i + FPF_LANE_PF < NS) {
                // (the row opaque here: else all NS x 6 load offsets are computed up
                // front, in scalar registers that spill)
                int r = row[i + FPF_LANE_PF];
                __asm__ volatile("" : "+s"(r));
                load_pq(sn[FPF_LANE_PF - 1], rp, r, plane, bb, so);
            }
            const double isc = (ei[i] & 1) ? inv_s3 : 0.0;   // (uniform) 0 on a dummy slot
            if (flat) {
#pragma unroll
                for (int k = 0; k < 6; ++k) sabs = fma(fabs(sc[k]), isc, sabs);
            }
            __asm__ volatile("" : "+v"(sabs));
            slot_currents(x, i, sc, isc);
            pin(x[i]);
            if (FPF_LANE_SB & 1) __builtin_amdgcn_sched_barrier(0);
        }
    }

    // ---- the same on the DMA ring: on entry slots 0 and 1 are in flight (entries 0
    // and 1); slot j + 3 is issued in slot j into the entry slot j + 1 was read from
    __device__ __forceinline__ static void currents_dma(cx (&x)[NS][3], double &sabs, bool flat, u4 rsrc, unsigned vo,
                                                        cint *tab, unsigned bb, unsigned plane2, unsigned ring_lds,
                                                        const double *ring, int lane, double inv_s3) {
        int row[NS], ei[NS];
#pragma unroll
        for (int i = 0; i < NS; ++i) row[i] = tab[i];
#pragma unroll
        for (int i = 0; i < NS; ++i) ei[i] = tab[2 * NS + i];
        double sn[6];
        vm_wait(NS > 1);   // slot 0 landed (slot 1 may not have)
        ring_read(sn, ring, lane, row[0], vo);
        if (NS > 2) dma_slot(rsrc, vo, row[2], bb, plane2, ring_lds);   // (waits for the reads of entry 0)
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            double sc[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) sc[k] = sn[k];
            if (i + 1 < NS) {
                vm_wait(i + 2 < NS);   // slot i + 1 landed (slot i + 2 may not have)
                ring_read(sn, ring + ((i + 1) & 1) * 384, lane, row[i + 1], vo);
            }
            __builtin_amdgcn_sched_barrier(0);
            const double isc = (ei[i] & 1) ? inv_s3 : 0.0;   // (uniform) 0 on a dummy slot
            if (flat) {
#pragma unroll
                for (int k = 0; k < 6; ++k) sabs = fma(fabs(sc[k]), isc, sabs);
            }
            __asm__ volatile("" : "+v"(sabs));
            slot_currents(x, i, sc, isc);
            pin(x[i]);
            __builtin_amdgcn_sched_barrier(0);
            if (i + 3 < NS) dma_slot(rsrc, vo, row[i + 3], bb, plane2, ring_lds + ((i + 1) & 1) * 3072);
        }
    }

    // ---- backward sweep (:134-160) Ib = E[last] - E[q - 1] on the globalised E
    // (x = carry + local prefix), slots in descending order so that E[q - 1] is
    // still in place; the branch drops lng (Ib . Zl) (:163-178) over it; then their
    // local prefix G in ascending order; also the lane's part of the loss, sum
    // Re(drop conj(Ib)) (s3 times it is PQb(0).re - sum_k PQL(k).re on a feeder
    // without zeroed phases, fpf_wave_body.h), kept in the sweep a scenario finishes
    __device__ __forceinline__ static void drops(cx (&x)[NS][3], double &lp, const double2 *cw,
                                                 const double2 *EG, cint *tab, cdbl *tmp, int lane) {
        int ei[NS];
#pragma unroll
        for (int i = 0; i < NS; ++i) ei[i] = tab[2 * NS + i];
        // the next slot's gathers (LDS) and TEMP (scalar loads) are issued at the top
        // of a slot and first used in the next one: one wait (lgkmcnt(0): scalar
        // loads return out of order, so any wait on them waits for every LDS read as
        // well) per slot, after the slot's arithmetic instead of before it
        cx el[3], en[3];
        double tc[LANE_TW], tn[LANE_TW];
        {
            const int li = (ei[NS - 1] >> 16) & 0xffff;
#pragma unroll
            for (int p = 0; p < 3; ++p) en[p] = ldc(EG, (li * 3 + p) * 64 + lane);
#pragma unroll
            for (int k = 0; k < LANE_TW; ++k) tn[k] = tmp[(NS - 1) * LANE_TW + k];
        }
#pragma unroll
        for (int i = NS - 1; i >= 0; --i) {
#pragma unroll
            for (int p = 0; p < 3; ++p) el[p] = en[p];
#pragma unroll
            for (int k = 0; k < LANE_TW; ++k) tc[k] = tn[k];
            // (consumed here: the wait for them comes before the next slot's loads)
            __asm__ volatile("" : "+s"(tc[0]), "+s"(tc[1]), "+s"(tc[2]), "+s"(tc[3]), "+s"(tc[4]), "+s"(tc[5]),
                             "+s"(tc[6]), "+s"(tc[7]));
            pin(el);
            __builtin_amdgcn_sched_barrier(0);
            if (i > 0) {
                const int li = (ei[i - 1] >> 16) & 0xffff;
#pragma unroll
                for (int p = 0; p < 3; ++p) en[p] = (FPF_LANE_ABL & 2) ? x[i - 1][p] : ldc(EG, (li * 3 + p) * 64 + lane);
                cdbl *tq = tmp + (i - 1) * LANE_TW;
                __asm__ volatile("" : "+s"(tq));   // (issued here, not hoisted to the phase start)
#pragma unroll
                for (int k = 0; k < LANE_TW; ++k) tn[k] = tq[k];
            }
            __builtin_amdgcn_sched_barrier(0);   // (the loads first)
            cx ib[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) ib[p] = csub(el[p], i > 0 ? x[i - 1][p] : ldc(cw, p * 64 + lane));   // (E[-1] = the carry)
            const cx zm = mk(tc[6], tc[7]);
            const cx sm = cadd(cadd(ib[0], ib[1]), ib[2]);
            const cx ms = mk(fma(zm.re, sm.re, -(zm.im * sm.im)), fma(zm.re, sm.im, zm.im * sm.re));
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                const cx d = mk(tc[2 * p], tc[2 * p + 1]);
                const cx b = ib[p];
                const cx g = mk(fma(d.re, b.re, fma(-d.im, b.im, ms.re)), fma(d.re, b.im, fma(d.im, b.re, ms.im)));
                x[i][p] = g;
            }
#pragma unroll
            for (int p = 0; p < 3; ++p) lp = fma(x[i][p].re, ib[p].re, fma(x[i][p].im, ib[p].im, lp));
            pin(x[i]);
            __asm__ volatile("" : "+v"(lp));   // (else summed where it is stored, keeping every Ib alive)
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int i = 1; i < NS; ++i) {
#pragma unroll
            for (int p = 0; p < 3; ++p) x[i][p] = cadd(x[i - 1][p], x[i][p]);
            pin(x[i]);
        }
    }

    // ---- forward sweep (:163-195): V = (V0 - off(block) - carry) - G, the block
    // offset resolved where a block starts (and at the wave's first slot)
    __device__ __forceinline__ static void voltages(cx (&x)[NS][3], const double2 *vw, const double2 *EG, cint *tab,
                                                    cint *blk, int lane) {
        int gv[NS];
#pragma unroll
        for (int i = 0; i < NS; ++i) gv[i] = tab[3 * NS + i];
        cx cb[3];
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            const int gi = gv[i];
            if (gi & (1 << 30)) {   // (uniform; always at slot 0)
                cint *const bt = blk + ((gi >> 16) & 0x3fff) * (1 + 2 * LANE_BD);
                const int dep = bt[0];
#pragma unroll
                for (int p = 0; p < 3; ++p) cb[p] = ldc(vw, p * 64 + lane);   // V0 - the carry of G
#pragma nounroll
                for (int j = 0; j < dep; ++j) {
                    const int ta = bt[1 + 2 * j], fm = bt[2 + 2 * j];
#pragma unroll
                    for (int p = 0; p < 3; ++p) cb[p] = cadd(cb[p], ldc(EG, (fm * 3 + p) * 64 + lane));
#pragma unroll
                    for (int p = 0; p < 3; ++p) cb[p] = csub(cb[p], ldc(EG, (ta * 3 + p) * 64 + lane));
                }
            }
#pragma unroll
            for (int p = 0; p < 3; ++p) x[i][p] = csub(cb[p], x[i][p]);
            pin(x[i]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }

    // ---- after the loop: V out (node rows of [3][Nn][B]) and the
    // extremes of the wave's slots (V_abc_list.cpp:7-81 with every row kept).  The
    // output bases come from LDS (optr) as buffer resources, each row's offset
    // (p Nn + node) 8B a scalar: the kernel's arguments are not kept in scalar
    // registers across the loop (they were spilled and reloaded per store)
    __device__ __forceinline__ static void finish(const cx (&x)[NS][3], double &mn, double &mx, bool fin, cint *tab,
                                                  const uint64_t *optr, unsigned nn, unsigned bb, unsigned so) {
#pragma unroll
        for (int i = 0; i < NS; ++i) {
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                const double m2 = fma(x[i][p].re, x[i][p].re, x[i][p].im * x[i][p].im);
                mn = fmin(mn, m2);
                mx = fmax(mx, m2);
            }
        }
        double *const vre = lds_ptr(optr, 0), *const vim = lds_ptr(optr, 1);
        const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void *)vre, 0, (int)0xffffffffu, 0x00020000);
        const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void *)vim, 0, (int)0xffffffffu, 0x00020000);
        if (!fin || !vre) return;   // (the host passes both planes or neither)
        const unsigned ps = nn * bb;   // bytes per phase plane
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            const int node = tab[NS + i];
            if (node >= 0) {
                unsigned ro = (unsigned)node * bb;
#pragma unroll
                for (int p = 0; p < 3; ++p, ro += ps) {
                    __builtin_amdgcn_raw_buffer_store_b64(bits2(x[i][p].re), rr, so, ro, 0);
                    __builtin_amdgcn_raw_buffer_store_b64(bits2(x[i][p].im), ri, so, ro, 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
};

template <int NS, bool DMA>
__global__ __launch_bounds__(LANE_NW * 64, 2) void dpf_lane_kernel(LaneDev f, int B, const double *__restrict__ pq,
                                                                   OutDev o) {
    constexpr int NW = LANE_NW;
    typedef LaneSweep<NS> SW;
    extern __shared__ double2 lds[];
    // DMA: [NW][2][6][64] the waves' load rings (48 KiB, first: M0 addresses stay
    // small), after the loop [NW][2][64] min / max |V|^2; else only the latter
    double *const MM = (double *)lds;
    double2 *const WT = (double2 *)(MM + (DMA ? NW * 2 * 384 : NW * 2 * 64));   // [NW][3][64] wave totals (E, then G)
    double2 *const IBO = WT + NW * 3 * 64;                 // [3][64] Ib(0) of the last sweep
    double *const LS = (double *)(IBO + 3 * 64);           // [NW][2][64] per wave: loss part, sum |S|_1
    double2 *const EG = (double2 *)(LS + NW * 2 * 64);     // [max(nE, nG) + 1][3][64] published E, then G; last: 0
    __shared__ int fix_n, fix_ids[64];
    __shared__ double res[64][4];
    __shared__ int last_wg;
    __shared__ uint64_t optr[5];   // v_re, v_im, iters, status, errmx (read where used)
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int s = (int)blockIdx.x * 64 + lane;
    const bool live = s < B;
    const unsigned so = 8u * (unsigned)(live ? s : B - 1);   // byte offset (lanes past the batch read its last scenario)
    const unsigned bb = 8u * (unsigned)B;                     // bytes per Dl row of a field plane
    const int nl = f.nl, nn = f.nn;
    cint *const tab0 = (cint *)f.slot + 4 * w * NS;   // [4][NS]: rows, nodes, backward, forward info
    cdbl *const tmp0 = (cdbl *)f.temp + (size_t)w * NS * LANE_TW;
    // one buffer resource on the batch [6][Nl][B] (P1 Q1 P2 Q2 P3 Q3 planes)
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc((void *)pq, 0, (int)0xffffffffu, 0x00020000);
    const unsigned plane = (unsigned)nl * bb;   // bytes per field plane
    const double inv_s3 = 1.0 / f.s3;
    const double eps2 = f.eps * f.eps;
    cx v0[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) v0[p] = mk(f.V0[2 * p], f.V0[2 * p + 1]);

    LSTAMP(0);
    if (f.stagger > 0 && blockIdx.x < 256u && ((blockIdx.x >> 3) & 1u)) {
        // every other CU of each XCD (blocks go round robin over the 8 XCDs) starts
        // its first workgroup late, its later ones follow on: the CUs' load-current
        // phases -- each workgroup's 377 KB of loads re-read in a burst -- then
        // fall at different times instead of all at once (FPF_LANE_STAGGER)
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        while (__builtin_amdgcn_s_memtime() - t0 < (unsigned long long)f.stagger) __builtin_amdgcn_s_sleep(8);
    }
    if (threadIdx.x == 0) fix_n = 0;
    if (threadIdx.x == 0) {
        optr[0] = (uint64_t)o.v_re;
        optr[1] = (uint64_t)o.v_im;
        optr[2] = (uint64_t)o.iters;
        optr[3] = (uint64_t)o.status;
        optr[4] = (uint64_t)o.errmx;
    }
    const bool guard_on = o.flag_count != nullptr;
    if ((int)threadIdx.x < 3 * 64) {
        IBO[threadIdx.x] = make_double2(0.0, 0.0);
        EG[max(f.nE, f.nG) * 3 * 64 + threadIdx.x] = make_double2(0.0, 0.0);   // the permanent zero entry
    }
    for (int i = threadIdx.x; i < NW * 2 * 64; i += NW * 64) LS[i] = 0.0;

    cx x[NS][3];   // the slots' state: V, then E, Ib -> G, then V again
#pragma unroll
    for (int i = 0; i < NS; ++i)
#pragma unroll
        for (int p = 0; p < 3; ++p) x[i][p] = v0[p];
    bool done = !live;
    double gmin = INFINITY;   // (wave 0) closest |errmx^2 - eps^2| of a decision in the coarse band
    int stat = 1;             // (wave 0) the scenario's status
    double sn[FPF_LANE_PF][6];   // (no DMA) the next slots' P, Q
    // (DMA) the batch resource with its exact size (pieces past the batch read 0),
    // this lane's piece offset, this wave's ring
    const u4 rq = {(unsigned)(uintptr_t)pq, (unsigned)((uintptr_t)pq >> 32), 6u * plane, 0x00020000u};
    const unsigned vdma = (lane >= 32 ? plane : 0u) + 8u * (unsigned)(blockIdx.x * 64 + 2 * (lane & 31));
    const unsigned ring_lds =
        (unsigned)(uintptr_t)(__attribute__((address_space(3))) double *)MM + (unsigned)w * 2u * 3072u;
    const double *const ring = MM + w * 2 * 384;
    if (DMA) {
        dma_slot(rq, vdma, tab0[0], bb, 2 * plane, ring_lds);
        dma_slot(rq, vdma, tab0[1], bb, 2 * plane, ring_lds + 3072);
    } else {
#pragma unroll
        for (int j = 0; j < FPF_LANE_PF; ++j) load_pq(sn[j], rp, tab0[j], plane, bb, so);
    }
    LSTAMP(1);
    for (int it = 0;; ++it) {
        LSTAMP_IT(0);
        // the slot tables' base opaque per sweep: their scalar loads stay inside the
        // loop instead of hundreds of scalar registers hoisted (and spilled) across it
        cint *tab = tab0;
        cdbl *tmp = tmp0;
        cint *blk = (cint *)f.blk;
        __asm__ volatile("" : "+s"(tab), "+s"(tmp), "+s"(blk));
        // a finished lane's state is frozen (every update below is under !done, a
        // divergent branch: its registers keep the V of its last sweep until the
        // loop ends, when every lane's V leaves in whole lines)
        if (!done) {
            double sabs = 0.0;
            if (DMA) SW::currents_dma(x, sabs, it == 0, rq, vdma, tab, bb, 2 * plane, ring_lds, ring, lane, inv_s3);
            else SW::currents(x, sabs, it == 0, sn, rp, tab, plane, bb, so, inv_s3);
            if (it == 0) LS[(w * 2 + 1) * 64 + lane] = sabs;
#pragma unroll
            for (int p = 0; p < 3; ++p) stc(WT, (w * 3 + p) * 64 + lane, x[NS - 1][p]);
        }
        LSTAMP_IT(1);
        lane_barrier();   // B1: the wave totals of E
        LSTAMP_IT(2);

        // ---- the carry of this wave and Ib(0) = the total, summed in wave order (the
        // same association in every wave, so every wave takes the same decisions)
        cx carry[3] = {mk(0, 0), mk(0, 0), mk(0, 0)};
#pragma nounroll
        for (int u = 0; u < w; ++u) {
            cx t[3];
            ld3(t, WT, u * 3 * 64 + lane);
#pragma unroll
            for (int p = 0; p < 3; ++p) carry[p] = cadd(carry[p], t[p]);
        }
        cx tot[3] = {carry[0], carry[1], carry[2]};
#pragma nounroll
        for (int u = w; u < NW; ++u) {
            cx t[3];
            ld3(t, WT, u * 3 * 64 + lane);
#pragma unroll
            for (int p = 0; p < 3; ++p) tot[p] = cadd(tot[p], t[p]);
        }
        // ---- convergence on the substation branch (:199-217)
        double err2 = 0.0;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const cx io = ldc(IBO, p * 64 + lane);
            const double dr = tot[p].re - io.re, di = tot[p].im - io.im;
            err2 = fmax(err2, fma(dr, dr, di * di));
        }
        const bool conv = (FPF_LANE_ABL & 4) ? false : err2 < eps2;
        const bool fin = !done && (conv || it == ((FPF_LANE_ABL & 4) ? 4 : f.mxitr - 1));
        if (w == 0 && guard_on) {
            // the guard record (fpf_wave_body.h): decisions within 2^-9 of eps^2
            const double dd = fabs(err2 - eps2);
            if (!done && dd <= 0x1p-9 * eps2) gmin = fmin(gmin, dd);
        }
        // E made global (x = carry + the local prefix) and published at the subtree
        // ends (the leaves; every slot gathers one)
        if (!done) {
            int ev[NS];
#pragma unroll
            for (int i = 0; i < NS; ++i) ev[i] = tab[2 * NS + i];
#pragma unroll
            for (int i = 0; i < NS; ++i) {
#pragma unroll
                for (int p = 0; p < 3; ++p) x[i][p] = cadd(carry[p], x[i][p]);
                pin(x[i]);
                const int pe = ((ev[i] >> 1) & 0x7fff) - 1;
                if (pe >= 0) {
#pragma unroll
                    for (int p = 0; p < 3; ++p) stc(EG, (pe * 3 + p) * 64 + lane, x[i][p]);
                }
            }
        }
        LSTAMP_IT(3);
        lane_barrier();   // B2: published E (every wave has read IBO and the wave totals)
        LSTAMP_IT(4);
        if (w == 0) {
#pragma unroll
            for (int p = 0; p < 3; ++p) stc(IBO, p * 64 + lane, tot[p]);
        }
        // the wave's carry parked in its WT entry for the backward sweep's slot 0
        // (12 registers fewer through it)
        double2 *const cw = WT + w * 3 * 64;
#pragma unroll
        for (int p = 0; p < 3; ++p) stc(cw, p * 64 + lane, carry[p]);

        if (!done) {
            double lp = 0.0;
            SW::drops(x, lp, cw, EG, tab, tmp, lane);
            // WT is free again (every wave read it before B2)
#pragma unroll
            for (int p = 0; p < 3; ++p) stc(WT, (w * 3 + p) * 64 + lane, x[NS - 1][p]);
            if (fin) LS[(w * 2 + 0) * 64 + lane] = lp;
        }
        // the next sweep's first loads, in flight across the barriers (DMA: slots 0
        // and 1 into the ring, free since the last slots' reads)
        if (DMA) {
            dma_slot(rq, vdma, tab[0], bb, 2 * plane, ring_lds);
            dma_slot(rq, vdma, tab[1], bb, 2 * plane, ring_lds + 3072);
        } else {
#pragma unroll
            for (int j = 0; j < FPF_LANE_PF; ++j) load_pq(sn[j], rp, tab[j], plane, bb, so);
        }
        LSTAMP_IT(5);
        lane_barrier();   // B3: the wave totals of G (every wave has read its gathered E)
        LSTAMP_IT(6);

        cx carryg[3] = {mk(0, 0), mk(0, 0), mk(0, 0)};
#pragma nounroll
        for (int u = 0; u < w; ++u) {
            cx t[3];
            ld3(t, WT, u * 3 * 64 + lane);
#pragma unroll
            for (int p = 0; p < 3; ++p) carryg[p] = cadd(carryg[p], t[p]);
        }
        // publish G at the taps and before the lateral blocks
        int gv[NS];
#pragma unroll
        for (int i = 0; i < NS; ++i) gv[i] = tab[3 * NS + i];
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            const int pg = (gv[i] & 0xffff) - 1;
            if (pg >= 0) {
#pragma unroll
                for (int p = 0; p < 3; ++p) stc(EG, (pg * 3 + p) * 64 + lane, cadd(carryg[p], x[i][p]));
            }
        }
        LSTAMP_IT(7);
        lane_barrier();   // B4: published G
        LSTAMP_IT(8);

        // V0 - the carry of G, parked in the wave's WT entry (every wave has read the
        // G totals before B4)
#pragma unroll
        for (int p = 0; p < 3; ++p) stc(cw, p * 64 + lane, csub(v0[p], carryg[p]));
        if (!done) SW::voltages(x, cw, EG, tab, blk, lane);
        LSTAMP_IT(9);
        if (fin) {
            if (w == 0) {
                stat = conv ? FPF_CONVERGED : FPF_NONCONVERGED;
                int32_t *const pit = (int32_t *)lds_ptr(optr, 2);
                int8_t *const pst = (int8_t *)lds_ptr(optr, 3);
                double *const per = lds_ptr(optr, 4);
                if (pit) pit[s] = it + 1;
                if (pst) pst[s] = (int8_t)stat;
                if (per) per[s] = sqrt(err2);
            }
        }
        done = done || fin;
        if (__ballot(!done) == 0) break;   // (the same in every wave)
    }
    LSTAMP(120);
    if (DMA) vm_wait(false);   // (the ring's last pieces, issued for a sweep that did not come)
    {
        // every lane's V (frozen at its last sweep) out in whole lines, and the
        // extremes of the wave's slots
        double mn = INFINITY, mx = -INFINITY;
        cint *tab = tab0;
        __asm__ volatile("" : "+s"(tab));
        SW::finish(x, mn, mx, live, tab, optr, (unsigned)nn, bb, so);
        MM[(w * 2 + 0) * 64 + lane] = mn;
        MM[(w * 2 + 1) * 64 + lane] = mx;
    }
    LSTAMP(121);
    lane_barrier();   // MM, LS complete

    // ---- per scenario (wave 0): loss (VoltVarCtrl.cpp:1152-1161), Vmin / Vmax
    // (V_abc_list.cpp:7-81 with every row kept, VoltVarCtrl.cpp:1201-1207), the
    // guard band, the substation row of V
    const int nsb = min(64, B - (int)blockIdx.x * 64);
    if (w == 0) {
        double ls = 0.0, sa = 0.0, mn = INFINITY, mx = -INFINITY;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const double m2 = fma(v0[p].re, v0[p].re, v0[p].im * v0[p].im);
            mn = fmin(mn, m2);
            mx = fmax(mx, m2);
        }
        for (int u = 0; u < NW; ++u) {
            ls += LS[(u * 2 + 0) * 64 + lane];
            mn = fmin(mn, MM[(u * 2 + 0) * 64 + lane]);
            mx = fmax(mx, MM[(u * 2 + 1) * 64 + lane]);
            sa += LS[(u * 2 + 1) * 64 + lane];
        }
        const double loss = f.s3 * ls, vmin = sqrt(mn), vmax = sqrt(mx);
        if (live) {
            if (o.loss) o.loss[s] = loss;
            if (o.vmin) o.vmin[s] = vmin;
            if (o.vmax) o.vmax[s] = vmax;
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                const size_t r = (size_t)p * nn * (unsigned)B + (unsigned)s;
                if (o.v_re) __builtin_nontemporal_store(v0[p].re, o.v_re + r);
                if (o.v_im) __builtin_nontemporal_store(v0[p].im, o.v_im + r);
            }
        }
        res[lane][0] = loss;
        res[lane][1] = vmin;
        res[lane][2] = vmax;
        res[lane][3] = stat == FPF_CONVERGED ? 0.0 : 1.0;
        // the guard band (fpf_wave_body.h): errmx within tau = guard_k sum_k |IL_k|_1
        // of eps at a decision, sum_k |IL_k|_1 <= 1.25 sqrt2 sum_k |S_k|_1 / min_k |V_k|
        if (o.flag_count && live) {
            const bool cand = gmin < INFINITY;
            const double tau = 1.25 * f.guard_k * 1.4142135623730951 * sa / sqrt(mn);
            const bool near = cand && gmin <= 2.0 * f.eps * (1.0 + 0x1p-9) * tau;
            if (near) guard_flag(o, s, &fix_n, fix_ids);
            if (o.guard) o.guard[s] = near ? 1 : 0;
        } else if (live && o.guard) {
            o.guard[s] = 0;
        }
    }

    // ---- fused batch aggregate (the wave kernel's: per-workgroup partial in
    // scenario order, ticket, the last workgroup folds in workgroup order)
    constexpr int NT = NW * 64;
    const bool agg = o.agg != nullptr;
    if (agg) {
        __syncthreads();
        if (threadIdx.x == 0) {
            double ls = 0, mn = INFINITY, mx = -INFINITY, nc = 0, nnc = 0, no = 0, nu = 0;
            for (int j = 0; j < nsb; ++j) {
                if (res[j][3] == 0.0) {
                    ls += res[j][0];
                    mn = fmin(mn, res[j][1]);
                    mx = fmax(mx, res[j][2]);
                    nc += 1;
                    if (res[j][2] > f.ub_v) no += 1;
                    if (res[j][1] < f.lb_v) nu += 1;
                } else {
                    nnc += 1;
                }
            }
            const double part[8] = {ls, mn, mx, nc, nnc, no, nu, (double)nsb};
            double *dst = o.partials + 8 * (size_t)blockIdx.x;
            for (int q = 0; q < 8; ++q) __hip_atomic_store(dst + q, part[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned t = __hip_atomic_fetch_add(o.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last_wg = t == gridDim.x - 1;
        }
        __syncthreads();
        if (last_wg) {
            double a[8] = {0, INFINITY, -INFINITY, 0, 0, 0, 0, 0};
            for (unsigned b = threadIdx.x; b < gridDim.x; b += NT) {
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const double r = __hip_atomic_load(o.partials + 8 * (size_t)b + q, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
                    a[q] = q == 1 ? fmin(a[q], r) : (q == 2 ? fmax(a[q], r) : a[q] + r);
                }
            }
            double *sh = (double *)lds;   // [8][NT] (the sweep's LDS is dead)
#pragma unroll
            for (int q = 0; q < 8; ++q) sh[q * NT + threadIdx.x] = a[q];
            __syncthreads();
            for (int h = NT / 2; h > 0; h >>= 1) {
                if ((int)threadIdx.x < h) {
                    const int t = threadIdx.x;
                    sh[0 * NT + t] += sh[0 * NT + t + h];
                    sh[1 * NT + t] = fmin(sh[1 * NT + t], sh[1 * NT + t + h]);
                    sh[2 * NT + t] = fmax(sh[2 * NT + t], sh[2 * NT + t + h]);
#pragma unroll
                    for (int q = 3; q < 8; ++q) sh[q * NT + t] += sh[q * NT + t + h];
                }
                __syncthreads();
            }
            if (threadIdx.x < 8) o.agg[threadIdx.x] = sh[threadIdx.x * NT];
            if (threadIdx.x == 0) __hip_atomic_store(o.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (threadIdx.x == 0 && o.flag_out)
                *o.flag_out = __hip_atomic_load(o.flag_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    LSTAMP(122);
    if (o.fix_dev) {
        // the guard's local mode (a solve without an aggregate): the scenarios this
        // workgroup flagged are re-solved on the exact body by its first wave, after
        // every store of the fast results has landed (fpf_wave_body.h)
        __shared__ OutDev osh;
        __syncthreads();
        if (fix_n > 0) {
            __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (threadIdx.x == 0) osh = o;
            __syncthreads();
            if (w == 0) g3::g3_fixup_local(o.fix_dev, B, pq, (double *)lds, &osh, fix_ids, fix_n);
        }
    }
}

#ifdef FPF_LANE_STAMPS
extern "C" int fpf_debug_set_lane_stamp_buffer(void *dptr, unsigned base) {
    unsigned long long *p = (unsigned long long *)dptr;
    if (hipMemcpyToSymbol(HIP_SYMBOL(fpf_lane_stamp_base), &base, sizeof(base)) != hipSuccess) return -3;
    return hipMemcpyToSymbol(HIP_SYMBOL(fpf_lane_stamp_buf), &p, sizeof(p)) == hipSuccess ? 0 : -3;
}
#endif

size_t lane_lds_bytes(const LaneDev &l, bool dma) {
    const size_t col = 3 * 64 * 16;   // one published entry: 3 phases x 64 lanes x complex
    const size_t first = dma ? (size_t)LANE_NW * 2 * 384 * 8 : (size_t)LANE_NW * 2 * 64 * 8;   // rings / extremes
    return first + (size_t)LANE_NW * col + 3 * 64 * 16 + (size_t)LANE_NW * 2 * 64 * 8 +
           (size_t)(std::max(l.nE, l.nG) + 1) * col;
}

int lane_min_scen() {
    const char *e = getenv("FPF_LANE");
    if (!e) return 1 << 30;   // (until measured: off by default)
    const int v = atoi(e);
    return v <= 0 ? (1 << 30) : v;
}

static std::atomic<int> g_lane_launches{0}, g_lane_dma_launches{0};
extern "C" int fpf_lane_launches(void) { return g_lane_launches.load(); }
extern "C" int fpf_lane_dma_launches(void) { return g_lane_dma_launches.load(); }

// FPF_LANE_DMA=1: the loads through the LDS-DMA ring (read per call).  Off by
// default: config 4 0.920 ms with it against 0.913 ms without (profiles/r06_lane:
// the ring hides the loads' latency, but the load-current phase takes as long --
// its time is not the loads' latency)
static bool lane_dma_allowed() {
    const char *e = getenv("FPF_LANE_DMA");
    return e && *e && atoi(e) != 0;
}

hipError_t launch_lane(const LaneDev &l, int n_scen, const double *pq, const OutDev &o, hipStream_t st) {
    typedef void (*KFn)(LaneDev, int, const double *, OutDev);
    KFn kr = nullptr, kd = nullptr;
    switch (l.ns) {
        case 4: kr = dpf_lane_kernel<4, false>; kd = dpf_lane_kernel<4, true>; break;
        case 8: kr = dpf_lane_kernel<8, false>; kd = dpf_lane_kernel<8, true>; break;
        case 12: kr = dpf_lane_kernel<12, false>; kd = dpf_lane_kernel<12, true>; break;
        case 16: kr = dpf_lane_kernel<16, false>; kd = dpf_lane_kernel<16, true>; break;
        default: return hipErrorInvalidValue;
    }
    static std::mutex mu;
    static std::map<std::array<int, 3>, int> static_lds;   // (device, ns, dma) -> the kernel's static LDS
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidDevice;
    auto prepare = [&](KFn k, int dma, int *stat) -> hipError_t {
        std::lock_guard<std::mutex> lk(mu);
        auto it = static_lds.find({dev, l.ns, dma});
        if (it == static_lds.end()) {
            hipFuncAttributes fa{};
            hipError_t e = hipFuncGetAttributes(&fa, (const void *)k);
            if (e == hipSuccess)
                e = hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        160 * 1024 - (int)fa.sharedSizeBytes);
            if (e != hipSuccess) return e;
            it = static_lds.emplace(std::array<int, 3>{dev, l.ns, dma}, (int)fa.sharedSizeBytes).first;
        }
        *stat = it->second;
        return hipSuccess;
    };
    // the DMA ring when it fits beside the kernel's static LDS and the batch has an
    // even number of scenarios (a lane's 16-byte piece is two scenarios: an odd
    // batch's last piece would reach past the end of the buffer)
    KFn k = kr;
    size_t lds = lane_lds_bytes(l, false);
    int stat = 0;
    if (lane_dma_allowed() && n_scen % 2 == 0) {
        if (prepare(kd, 1, &stat) == hipSuccess && lane_lds_bytes(l, true) + (size_t)stat <= (size_t)160 * 1024) {
            k = kd;
            lds = lane_lds_bytes(l, true);
        }
    }
    if (k == kr) {
        const hipError_t e = prepare(kr, 0, &stat);
        if (e != hipSuccess) return e;
    }
    const unsigned grid = (unsigned)((n_scen + 63) / 64);
    LaneDev la = l;
    {
        const char *e = getenv("FPF_LANE_STAGGER");   // (read per call)
        la.stagger = e && *e ? std::max(0, atoi(e)) : 0;
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(LANE_NW * 64), lds, st, la, n_scen, pq, o);
    const hipError_t e = hipGetLastError();
    if (e == hipSuccess) {
        g_lane_launches.fetch_add(1);
        if (k == kd) g_lane_dma_launches.fetch_add(1);
    }
    return e;
}

}  // namespace fpf
