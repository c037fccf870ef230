// Systolic exact first fit of one 64-node group with the node rotation folded into the step's
// own reads (variant of fp_pipe_sysv.h; same contract as fpp_sysv_group).
//
// fp_pipe_sysv.h rotates the four node records with four v_mov_dpp at the end of every step
// (21 VALU instructions, ~126 cycles per step on gfx950, tools/ubench/systolic.hip).  Here the
// rotation is the DPP modifier of the first instruction that reads each record in the next step:
// the tests read rot(x) (v_sub_co_u32_dpp / v_and_b32_dpp / v_or_b32_dpp) and the update writes
// back x = fits ? new : rot(x) (v_cndmask_b32_dpp), so the registers hold the state one rotation
// behind the step that reads them.  Only the labels (never updated) keep a plain v_mov_dpp.
// Liveness is folded into the conflict word instead of three chained v_cndmask:
//   t = (rot(xl) & kr) | (rot(xu) & kx) | dead        dead = -1 unless the lane's container runs
//   t |= borrow(rot(xc) - kc) ? -1 : 0 ; t |= borrow(rot(xm) - km) ? -1 : 0 ; fits = (t == 0)
// 18 VALU instructions per step.  Layout: at the start of step tau, position p is at lane
// (tau - 1 - p) & 63; the lane-t container tests position tau - t (k counts it; k < L = running,
// a placement sets k = PLACED).  Exactness as fp_pipe_sys.h: every position meets the containers
// in FFD order and every container the positions in node order.
#pragma once
#include <stdint.h>

// included by fp_pipe_sys.h after its helpers, SysOut and fp_pipe_sysv.h

namespace fpp {

// steps per exit check (one ballot + two branches): 16 (round 6: config 3 on the u32 kernels 55.9 ->
// 54.4-54.8 ms, config 2 0.77 -> 0.75 ms against 8, profiles/r07h_u32_unroll16_ab.jsonl; round 5: 8
// against 4, patterns 0-3 of tools/ubench/systolic.hip 109-138 vs 122-156 cycles per container)
#ifndef FPP_SD_UNROLL
#define FPP_SD_UNROLL 16
#endif

#define FPP_SD_DPP " wave_ror:1 row_mask:0xf bank_mask:0xf\n\t"
// one step; operands: records xc xm xu xl, container kc km kr kx, k, apos, L, kpl (PLACED);
// temps dv ta tb t d1 d2 tu k1
#ifndef FPP_SD_ORDER
#define FPP_SD_ORDER 1
#endif
#if FPP_SD_ORDER == 0
#define FPP_SD_STEP                                                   \
    "v_cmp_gt_u32_e32 vcc, %[L], %[k]\n\t"                           \
    "v_cndmask_b32_e64 %[dv], -1, 0, vcc\n\t"                        \
    "v_and_b32_dpp %[ta], %[xl], %[kr]" FPP_SD_DPP                   \
    "v_and_b32_dpp %[tb], %[xu], %[kx]" FPP_SD_DPP                   \
    "v_or3_b32 %[t], %[ta], %[tb], %[dv]\n\t"                        \
    "v_sub_co_u32_dpp %[d1], vcc, %[xc], %[kc]" FPP_SD_DPP           \
    "v_cndmask_b32_e64 %[t], %[t], -1, vcc\n\t"                      \
    "v_sub_co_u32_dpp %[d2], vcc, %[xm], %[km]" FPP_SD_DPP           \
    "v_cndmask_b32_e64 %[t], %[t], -1, vcc\n\t"                      \
    "v_or_b32_dpp %[tu], %[xu], %[kx]" FPP_SD_DPP                    \
    "v_add_u32_e32 %[k1], 1, %[k]\n\t"                               \
    "v_cmp_eq_u32_e32 vcc, 0, %[t]\n\t"                              \
    "v_cndmask_b32_dpp %[xc], %[xc], %[d1], vcc" FPP_SD_DPP          \
    "v_cndmask_b32_dpp %[xm], %[xm], %[d2], vcc" FPP_SD_DPP          \
    "v_cndmask_b32_dpp %[xu], %[xu], %[tu], vcc" FPP_SD_DPP          \
    "v_mov_b32_dpp %[xl], %[xl]" FPP_SD_DPP                          \
    "v_cndmask_b32_e32 %[apos], %[apos], %[k], vcc\n\t"              \
    "v_cndmask_b32_e32 %[k], %[k1], %[kpl], vcc\n\t"
#else
// the same instructions, scheduled so that independent work sits between each VCC write and its
// reader (the VCC hand-offs are the step's dependency chain)
#define FPP_SD_STEP                                                   \
    "v_cmp_gt_u32_e32 vcc, %[L], %[k]\n\t"                           \
    "v_and_b32_dpp %[ta], %[xl], %[kr]" FPP_SD_DPP                   \
    "v_and_b32_dpp %[tb], %[xu], %[kx]" FPP_SD_DPP                   \
    "v_cndmask_b32_e64 %[dv], -1, 0, vcc\n\t"                        \
    "v_sub_co_u32_dpp %[d1], vcc, %[xc], %[kc]" FPP_SD_DPP           \
    "v_or3_b32 %[t], %[ta], %[tb], %[dv]\n\t"                        \
    "v_or_b32_dpp %[tu], %[xu], %[kx]" FPP_SD_DPP                    \
    "v_cndmask_b32_e64 %[t], %[t], -1, vcc\n\t"                      \
    "v_sub_co_u32_dpp %[d2], vcc, %[xm], %[km]" FPP_SD_DPP           \
    "v_add_u32_e32 %[k1], 1, %[k]\n\t"                               \
    "v_mov_b32_dpp %[xl], %[xl]" FPP_SD_DPP                          \
    "v_cndmask_b32_e64 %[t], %[t], -1, vcc\n\t"                      \
    "v_cmp_eq_u32_e32 vcc, 0, %[t]\n\t"                              \
    "v_cndmask_b32_dpp %[xc], %[xc], %[d1], vcc" FPP_SD_DPP          \
    "v_cndmask_b32_dpp %[xm], %[xm], %[d2], vcc" FPP_SD_DPP          \
    "v_cndmask_b32_dpp %[xu], %[xu], %[tu], vcc" FPP_SD_DPP          \
    "v_cndmask_b32_e32 %[apos], %[apos], %[k], vcc\n\t"              \
    "v_cndmask_b32_e32 %[k], %[k1], %[kpl], vcc\n\t"
#endif

// Runs steps until no queued container is running or `cap` steps (rounded up to FPP_SD_UNROLL)
// have run; returns the steps taken (= rotations applied).
__device__ __forceinline__ uint32_t fpp_sysd_steps(uint32_t &xc, uint32_t &xm, uint32_t &xu, uint32_t &xl,
                                                   uint32_t kc, uint32_t km, uint32_t kr, uint32_t kx, uint32_t &k,
                                                   uint32_t &apos, uint32_t L, uint32_t cap) {
    uint32_t tau = 0;
    const uint32_t kpl = 0x80000000u;
    while (true) {
        uint32_t dv, ta, tb, t, d1, d2, tu, k1;
        asm volatile(
#if FPP_SD_UNROLL >= 1
            FPP_SD_STEP
#endif
#if FPP_SD_UNROLL >= 2
            FPP_SD_STEP
#endif
#if FPP_SD_UNROLL >= 3
            FPP_SD_STEP
#endif
#if FPP_SD_UNROLL >= 4
            FPP_SD_STEP
#endif
#if FPP_SD_UNROLL >= 8
            FPP_SD_STEP FPP_SD_STEP FPP_SD_STEP FPP_SD_STEP
#endif
#if FPP_SD_UNROLL >= 16
            FPP_SD_STEP FPP_SD_STEP FPP_SD_STEP FPP_SD_STEP FPP_SD_STEP FPP_SD_STEP FPP_SD_STEP FPP_SD_STEP
#endif
            "s_nop 1"
            : [xc] "+v"(xc), [xm] "+v"(xm), [xu] "+v"(xu), [xl] "+v"(xl), [k] "+v"(k), [apos] "+v"(apos),
              [dv] "=&v"(dv), [ta] "=&v"(ta), [tb] "=&v"(tb), [t] "=&v"(t), [d1] "=&v"(d1), [d2] "=&v"(d2),
              [tu] "=&v"(tu), [k1] "=&v"(k1)
            : [kc] "v"(kc), [km] "v"(km), [kr] "v"(kr), [kx] "v"(kx), [L] "s"(L), [kpl] "v"(kpl)
            : "vcc");
        tau += FPP_SD_UNROLL;
        if (tau >= cap) break;
        if (!__builtin_amdgcn_ballot_w64(k < L)) break;  // nothing running (placed: PLACED; done: >= L)
    }
    return tau;
}

// fpp_sys_group with the DPP-folded step loop (same contract).  TOUCHED = false: `touched` is left
// alone (one-group stages derive their used nodes from the final records, k_ffd_pipe).
template <bool TOUCHED = true>
__device__ __forceinline__ SysOut fpp_sysd_group(uint64_t q, uint64_t &touched, uint32_t &asg, uint32_t &rcf,
                                                 uint32_t &rmf, uint32_t &rcu, uint32_t rlab, uint32_t cpu,
                                                 uint32_t mem, uint32_t req, uint32_t conf, uint32_t gbg, uint32_t qc,
                                                 uint32_t qm, uint32_t max_steps) {
    const uint32_t lane = __lane_id();
    SysOut out{0};
    const uint64_t lm = (__builtin_amdgcn_ballot_w64(rcf >= qc) & __builtin_amdgcn_ballot_w64(rmf >= qm));
    const uint32_t L = (uint32_t)__builtin_popcountll(lm);
    if (L == 0) {
        if ((q >> lane) & 1ull) asg = 0xFFFFFFFFu;
        return out;
    }
    const bool inq = (q >> lane) & 1ull;
    const uint32_t Q = (uint32_t)__builtin_popcountll(q);
    // a queue that is lanes 0..Q-1 (a batch arriving whole at a filling group) is compacted already,
    // and a group whose nodes are all live needs no position map: no permutes for either.  The ranks
    // are branch-free (v_mbcnt + one select): per-lane ternaries over two popcounts compiled to
    // divergent branches
    const bool qpre = (q & (q + 1ull)) == 0ull, lfull = lm == ~0ull;
    const uint32_t qa = __builtin_amdgcn_mbcnt_hi((uint32_t)(q >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)q, 0u));
    const uint32_t rq = qpre ? lane : inq ? qa : Q + lane - qa;
    uint32_t kc = cpu, km = mem, kr = req, kx = conf;
    if (!qpre) { kc = sys_push(rq, cpu); km = sys_push(rq, mem); kr = sys_push(rq, req); kx = sys_push(rq, conf); }
    const bool live = (lm >> lane) & 1ull;
    const uint32_t la = __builtin_amdgcn_mbcnt_hi((uint32_t)(lm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)lm, 0u));
    const uint32_t pos = live ? la : L + lane - la;
    // position p starts at lane (63 - p) & 63: one rotation behind the first step (see above)
    const uint32_t at0 = (63u - pos) & 63u;
    uint32_t xc = sys_push(at0, rcf), xm = sys_push(at0, rmf), xu = sys_push(at0, rcu), xl = sys_push(at0, rlab);
    const uint32_t pmap = lfull ? lane : sys_push(pos, lane);
    const bool filler = ((63u - lane) & 63u) >= L;  // filler positions fit nothing
    xc = filler ? 0u : xc;
    xm = filler ? 0u : xm;
    xu = filler ? 0xFFFFFFFFu : xu;
    xl = filler ? 0xFFFFFFFFu : xl;
    uint32_t k = lane < Q ? (0u - lane) : 0x80000000u;
    uint32_t apos = 0xFFFFFFFFu;
    const uint32_t cap = max_steps < Q + L ? max_steps : Q + L;
    const uint32_t tau = fpp_sysd_steps(xc, xm, xu, xl, kc, km, kr, kx, k, apos, L, cap);
    // after tau steps position p is at lane (tau - 1 - p) & 63
    const uint32_t src = (tau - 1u - pos) & 63u;
    const uint32_t ncf = sys_pull(src, xc), nmf = sys_pull(src, xm), ncu = sys_pull(src, xu);
    rcf = live ? ncf : rcf;
    rmf = live ? nmf : rmf;
    rcu = live ? ncu : rcu;
    const uint32_t nl = lfull ? (apos & 63u) : sys_pull(apos & 63u, pmap);
    const uint32_t cnode = apos != 0xFFFFFFFFu ? gbg + nl : 0xFFFFFFFFu;
    const uint32_t back = qpre ? cnode : sys_pull(rq, cnode);
    const uint32_t open = k < L ? 1u : 0u;
    const uint32_t open_here = qpre ? open : sys_pull(rq, open);
    asg = inq ? back : asg;
    out.left = __builtin_amdgcn_ballot_w64(inq && open_here != 0);
    if (TOUCHED) {
        const uint32_t bl = apos != 0xFFFFFFFFu && nl < 32 ? 1u << nl : 0u;
        const uint32_t bh = apos != 0xFFFFFFFFu && nl >= 32 ? 1u << (nl - 32) : 0u;
        touched |= ((uint64_t)sys_wave_or(bh) << 32) | sys_wave_or(bl);
    }
    return out;
}

#undef FPP_SD_STEP
#undef FPP_SD_DPP

}  // namespace fpp
