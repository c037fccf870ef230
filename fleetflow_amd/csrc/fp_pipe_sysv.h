// Systolic exact first fit of one 64-node group, VALU-only step (variant of fp_pipe_sys.h).
//
// fpp_sys_steps (fp_pipe_sys.h) narrows EXEC with v_cmpx and keeps the pending set on the
// SALU: every step crosses VALU -> SALU -> EXEC -> VALU, ~50 cycles per crossing on gfx950
// (tools/ubench/isa.hip), ~130 cycles per step.  Here a step never leaves the VALU:
//   * a lane's container state is one counter k = (step - lane) while it runs: it tests
//     position k this step, it is live while k < L (unsigned: not started = negative = huge),
//     and a placement sets bit 31 (never live again);
//   * the three tests leave borrows / a conflict word; v_cndmask folds them into one word
//     that is 0 iff the container fits the position it holds, and VCC = (word == 0) selects
//     the new records (v_cndmask, no EXEC change);
//   * the node records rotate one lane (DPP wave_ror:1).
// The step count is fixed before the loop (the caller's cap); the loop checks once every
// FPP_SV_UNROLL steps (one ballot) whether any queued container is still running, so the
// VALU -> SALU crossing is paid once per FPP_SV_UNROLL steps.  Exactness is fp_pipe_sys.h's
// argument: at step tau lane t holds position tau - t, so every position meets the
// containers in FFD order and every container the positions in node order.
#pragma once
#include <stdint.h>

// included by fp_pipe_sys.h after its helpers and SysOut

namespace fpp {

#ifndef FPP_SV_UNROLL
#define FPP_SV_UNROLL 4
#endif

// one step; operands: xc xm xu xl (records), kc km kr kx (container), k, apos, L; temps
#define FPP_SV_STEP                                                        \
    "v_sub_co_u32 %[d1], %[b1], %[xc], %[kc]\n\t"                          \
    "v_sub_co_u32 %[d2], %[b2], %[xm], %[km]\n\t"                          \
    "v_cmp_le_u32 %[b3], %[L], %[k]\n\t"                                   \
    "v_and_b32 %[t], %[xl], %[kr]\n\t"                                     \
    "v_and_or_b32 %[t], %[xu], %[kx], %[t]\n\t"                            \
    "v_or_b32 %[tu], %[xu], %[kx]\n\t"                                     \
    "v_cndmask_b32 %[t], %[t], -1, %[b1]\n\t"                              \
    "v_cndmask_b32 %[t], %[t], -1, %[b2]\n\t"                              \
    "v_cndmask_b32 %[t], %[t], -1, %[b3]\n\t"                              \
    "v_or_b32 %[tk], %[bit31], %[k]\n\t"                                   \
    "v_cmp_eq_u32 vcc, 0, %[t]\n\t"                                        \
    "v_cndmask_b32 %[xc], %[xc], %[d1], vcc\n\t"                           \
    "v_cndmask_b32 %[xm], %[xm], %[d2], vcc\n\t"                           \
    "v_cndmask_b32 %[xu], %[xu], %[tu], vcc\n\t"                           \
    "v_cndmask_b32 %[apos], %[apos], %[k], vcc\n\t"                        \
    "v_cndmask_b32 %[k], %[k], %[tk], vcc\n\t"                             \
    "v_mov_b32_dpp %[xl], %[xl] wave_ror:1 row_mask:0xf bank_mask:0xf\n\t" \
    "v_add_u32 %[k], 1, %[k]\n\t"                                          \
    "v_mov_b32_dpp %[xc], %[xc] wave_ror:1 row_mask:0xf bank_mask:0xf\n\t" \
    "v_mov_b32_dpp %[xm], %[xm] wave_ror:1 row_mask:0xf bank_mask:0xf\n\t" \
    "v_mov_b32_dpp %[xu], %[xu] wave_ror:1 row_mask:0xf bank_mask:0xf\n\t"

// Runs steps until no queued container is live or `cap` steps (rounded up to FPP_SV_UNROLL)
// have run; returns the steps taken (= rotations applied).  k / apos as described above.
__device__ __forceinline__ uint32_t fpp_sysv_steps(uint32_t &xc, uint32_t &xm, uint32_t &xu, uint32_t &xl,
                                                   uint32_t kc, uint32_t km, uint32_t kr, uint32_t kx, uint32_t &k,
                                                   uint32_t &apos, uint32_t L, uint32_t cap) {
    uint32_t tau = 0;
    const uint32_t bit31 = 0x80000000u;
    while (true) {
        uint32_t d1, d2, t, tu, tk;
        uint64_t b1, b2, b3;
        asm volatile(
#if FPP_SV_UNROLL >= 1
            FPP_SV_STEP
#endif
#if FPP_SV_UNROLL >= 2
            FPP_SV_STEP
#endif
#if FPP_SV_UNROLL >= 3
            FPP_SV_STEP
#endif
#if FPP_SV_UNROLL >= 4
            FPP_SV_STEP
#endif
#if FPP_SV_UNROLL >= 5
            FPP_SV_STEP FPP_SV_STEP FPP_SV_STEP FPP_SV_STEP
#endif
            "s_nop 1"
            : [xc] "+v"(xc), [xm] "+v"(xm), [xu] "+v"(xu), [xl] "+v"(xl), [k] "+v"(k), [apos] "+v"(apos),
              [d1] "=&v"(d1), [d2] "=&v"(d2), [t] "=&v"(t), [tu] "=&v"(tu), [tk] "=&v"(tk), [b1] "=&s"(b1),
              [b2] "=&s"(b2), [b3] "=&s"(b3)
            : [kc] "v"(kc), [km] "v"(km), [kr] "v"(kr), [kx] "v"(kx), [L] "v"(L), [bit31] "v"(bit31)
            : "vcc");
        tau += FPP_SV_UNROLL >= 5 ? 8 : FPP_SV_UNROLL;
        if (tau >= cap) break;
        if (!__builtin_amdgcn_ballot_w64(k < L)) break;  // nothing live (placed: bit 31; done: >= L)
    }
    return tau;
}

// fpp_sys_group with the VALU-only step loop (same contract).
__device__ __forceinline__ SysOut fpp_sysv_group(uint64_t q, uint64_t &touched, uint32_t &asg, uint32_t &rcf,
                                                 uint32_t &rmf, uint32_t &rcu, uint32_t rlab, uint32_t cpu,
                                                 uint32_t mem, uint32_t req, uint32_t conf, uint32_t gbg, uint32_t qc,
                                                 uint32_t qm, uint32_t max_steps) {
    const uint32_t lane = __lane_id();
    const uint64_t below = (1ull << lane) - 1ull;
    SysOut out{0};
    const uint64_t lm = (__builtin_amdgcn_ballot_w64(rcf >= qc) & __builtin_amdgcn_ballot_w64(rmf >= qm));
    const uint32_t L = (uint32_t)__builtin_popcountll(lm);
    if (L == 0) {
        if ((q >> lane) & 1ull) asg = 0xFFFFFFFFu;
        return out;
    }
    const bool inq = (q >> lane) & 1ull;
    const uint32_t Q = (uint32_t)__builtin_popcountll(q);
    const uint32_t rq = inq ? (uint32_t)__builtin_popcountll(q & below) : Q + (uint32_t)__builtin_popcountll(~q & below);
    const uint32_t kc = sys_push(rq, cpu), km = sys_push(rq, mem), kr = sys_push(rq, req), kx = sys_push(rq, conf);
    const bool live = (lm >> lane) & 1ull;
    const uint32_t pos = live ? (uint32_t)__builtin_popcountll(lm & below) : L + (uint32_t)__builtin_popcountll(~lm & below);
    const uint32_t at0 = (64u - pos) & 63u;
    uint32_t xc = sys_push(at0, rcf), xm = sys_push(at0, rmf), xu = sys_push(at0, rcu), xl = sys_push(at0, rlab);
    const uint32_t pmap = sys_push(pos, lane);
    if (((64u - lane) & 63u) >= L) {
        xc = 0u; xm = 0u; xu = 0xFFFFFFFFu; xl = 0xFFFFFFFFu;
    }
    // compacted lane t < Q: k = -t (starts at step t); the rest never run
    uint32_t k = lane < Q ? (0u - lane) : 0x80000000u;
    uint32_t apos = 0xFFFFFFFFu;  // position of the placement
    const uint32_t cap = max_steps < Q + L ? max_steps : Q + L;
    const uint32_t tau = fpp_sysv_steps(xc, xm, xu, xl, kc, km, kr, kx, k, apos, L, cap);
    const uint32_t src = (tau - pos) & 63u;
    const uint32_t ncf = sys_pull(src, xc), nmf = sys_pull(src, xm), ncu = sys_pull(src, xu);
    if (live) { rcf = ncf; rmf = nmf; rcu = ncu; }
    const uint32_t nl = sys_pull(apos & 63u, pmap);
    const uint32_t cnode = apos != 0xFFFFFFFFu ? gbg + nl : 0xFFFFFFFFu;
    const uint32_t back = sys_pull(rq, cnode);
    // still running (not placed, not past the last position): the serial finish takes it
    const uint32_t open = k < L ? 1u : 0u;
    const uint32_t open_here = sys_pull(rq, open);
    if (inq) asg = back;
    out.left = __builtin_amdgcn_ballot_w64(inq && open_here != 0);
    const uint32_t bl = apos != 0xFFFFFFFFu && nl < 32 ? 1u << nl : 0u;
    const uint32_t bh = apos != 0xFFFFFFFFu && nl >= 32 ? 1u << (nl - 32) : 0u;
    touched |= ((uint64_t)sys_wave_or(bh) << 32) | sys_wave_or(bl);
    return out;
}

}  // namespace fpp
