// Hand-scheduled serial group loop of k_ffd_pipe (one group's queue, one stage): exact first
// fit, container by container in FFD order, as an inline-asm block with one branch per container
// (fpp_asm_group_x), the re-test of a queue after its first miss (fpp_refilter_loop) and the
// per-group epilogue (fpp_group_x).  gfx950 (GFX9 encoding): one SGPR per VALU op, lane selects
// come from SALU results or M0; M0 is restored on exit (the compiler treats it as reserved).
// (Round 1's container-major loop and round 2's readlane / writelane group loop are in git
// history; DESIGN.md 7 keeps their numbers.)
#pragma once
#include <stdint.h>

namespace fpp {

// re-test of a group's queue after its first miss: batch corners of at most this many nodes
#ifndef FPP_REFILTER_MAX
#define FPP_REFILTER_MAX 16
#endif
constexpr uint32_t REFILTER_MAX = FPP_REFILTER_MAX;

__device__ __forceinline__ uint64_t fpp_uniform64(uint64_t x) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(x >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
}

// Per-lane select by a wave-uniform lane mask: lane i gets `set` when bit i of m is set, else
// `clr`.  IB: one v_cndmask reading the mask as its condition register pair (inverse ballot)
// instead of the 64-bit shift, and and compare of the C++ form.  Only the one-wave kernels use it:
// in the 1024-thread kernels the compiler holds some of these masks in VGPRs, which the inverse
// ballot cannot read ("illegal VGPR to SGPR copy").
template <bool IB>
__device__ __forceinline__ uint32_t fpp_lane_sel(uint64_t m, uint32_t set, uint32_t clr) {
    if constexpr (IB)
        return __builtin_amdgcn_inverse_ballot_w64(m) ? set : clr;
    else
        return ((m >> __lane_id()) & 1ull) ? set : clr;
}

#ifdef FP_PIPE_STATS
#define FPP_ASM_CNT_CHECK "s_add_u32 %[nchk], %[nchk], 1\n\t"
#else
#define FPP_ASM_CNT_CHECK ""
#endif

// Exec-masked serial loop for ONE group g: exact first fit of the
// containers queued on group g, in lane (= FFD) order.  gfx950 issues one instruction of a
// wave every ~3.5 cycles and a scalar branch costs ~10-15 (tools/ubench/isa.hip), so the
// loop is cut to straight-line code with one branch per container:
//   * the placement updates node l's record with three VALU ops under exec = {l} -- no
//     readlane / writelane round trip; a miss leaves exec empty and the ops do nothing;
//   * exec = lowest bit of the feasibility mask is s_ff1 / s_lshl / s_and (a miss gives 0);
//   * the assignment goes to lane t as v_mov under exec = {t}: gbg | l, which is FP_NONE
//     (0xFFFFFFFF) on a miss (l = -1).  The caller derives `placed` and the next candidate
//     group of the misses from asg once per group (vector ops off the chain).
// touched |= the nodes placed on (for the deferred mask / used-bit bookkeeping).
// STOP: leave the loop after the first miss, with q = the containers not yet checked (the
// caller re-filters them against the group's current state); else run q to the end.  The two
// bodies differ in one line (qx = miss ? 0 : q) and in the register the loop test reads.
#define FPP_GX_BODY(SEL, TEST)                                                              \
    "s_cmp_eq_u64 %[q], 0\n\t"                                                             \
    "s_cbranch_scc1 .Lfgx_end%=\n\t"                                                       \
    "s_mov_b64 %[esv], exec\n"                                                             \
    ".Lfgx_loop%=:\n\t"                                                                    \
    "s_ff1_i32_b64 %[t], %[q]\n\t"                                                         \
    "v_readlane_b32 %[kc], %[cpu], %[t]\n\t"                                               \
    "v_readlane_b32 %[km], %[mem], %[t]\n\t"                                               \
    "v_readlane_b32 %[kr], %[req], %[t]\n\t"                                               \
    "v_readlane_b32 %[kx], %[conf], %[t]\n\t"                                              \
    "s_bitset0_b64 %[q], %[t]\n\t"                                                         \
    FPP_ASM_CNT_CHECK                                                                      \
    "v_cmp_ge_u32_e64 %[m1], %[rcf], %[kc]\n\t"                                            \
    "v_cmp_ge_u32_e64 %[m2], %[rmf], %[km]\n\t"                                            \
    "v_and_b32_e32 %[t0], %[kr], %[rlab]\n\t"                                              \
    "v_and_or_b32 %[t0], %[rcu], %[kx], %[t0]\n\t"                                         \
    "v_cmp_eq_u32_e64 %[m3], 0, %[t0]\n\t"                                                 \
    "s_and_b64 %[m1], %[m1], %[m2]\n\t"                                                    \
    "s_and_b64 %[m1], %[m1], %[m3]\n\t"                                                    \
    SEL                                                                                    \
    "s_ff1_i32_b64 %[l], %[m1]\n\t"                                                        \
    "s_lshl_b64 %[m2], 1, %[l]\n\t"                                                        \
    "s_and_b64 exec, %[m2], %[m1]\n\t"        /* {l}, or {} on a miss */                   \
    "v_subrev_u32_e32 %[rcf], %[kc], %[rcf]\n\t"                                           \
    "v_subrev_u32_e32 %[rmf], %[km], %[rmf]\n\t"                                           \
    "v_or_b32_e32 %[rcu], %[kx], %[rcu]\n\t"                                               \
    "s_or_b64 %[touched], %[touched], exec\n\t"                                            \
    "s_or_b32 %[nv], %[gbg], %[l]\n\t"         /* FP_NONE on a miss */                     \
    "s_lshl_b64 exec, 1, %[t]\n\t"                                                         \
    "v_mov_b32_e32 %[asg], %[nv]\n\t"                                                      \
    "s_mov_b64 exec, %[esv]\n\t"                                                           \
    "s_cmp_lg_u64 " TEST ", 0\n\t"                                                         \
    "s_cbranch_scc1 .Lfgx_loop%=\n"                                                        \
    ".Lfgx_end%=:"
#define FPP_GX_OPERANDS                                                                                         \
    : [q] "+s"(q), [touched] "+s"(touched), [asg] "+v"(asg), [rcf] "+v"(rcf), [rmf] "+v"(rmf), [rcu] "+v"(rcu), \
      [nchk] "+s"(nchk), [t] "=&s"(t), [kc] "=&s"(kc), [km] "=&s"(km), [kr] "=&s"(kr), [kx] "=&s"(kx),          \
      [l] "=&s"(l), [nv] "=&s"(nv), [m1] "=&s"(m1), [m2] "=&s"(m2), [m3] "=&s"(m3), [esv] "=&s"(esv),           \
      [qx] "=&s"(qx), [t0] "=&v"(t0)                                                                            \
    : [rlab] "v"(rlab), [cpu] "v"(cpu), [mem] "v"(mem), [req] "v"(req), [conf] "v"(conf), [gbg] "s"(gbg)       \
    : "scc", "memory"
template <bool STOP>
__device__ __forceinline__ void fpp_asm_group_x(uint64_t &q, uint64_t &touched, uint32_t &asg, uint32_t &rcf,
                                                uint32_t &rmf, uint32_t &rcu, uint32_t rlab, uint32_t cpu,
                                                uint32_t mem, uint32_t req, uint32_t conf, uint32_t gbg,
                                                uint32_t &nchk) {
    uint32_t t, kc, km, kr, kx, l, nv;
    uint64_t m1, m2, m3, esv, qx;
    uint32_t t0;
    if constexpr (STOP)
        asm volatile(FPP_GX_BODY("s_cselect_b64 %[qx], %[q], 0\n\t", "%[qx]") FPP_GX_OPERANDS);
    else
        asm volatile(FPP_GX_BODY("", "%[q]") FPP_GX_OPERANDS);
    (void)qx;
    // the asm's scalar outputs are wave-uniform, which divergence analysis cannot see: say so,
    // so that they can feed the next call's "+s" operands inside the caller's loop
    q = fpp_uniform64(q);
    touched = fpp_uniform64(touched);
    nchk = (uint32_t)__builtin_amdgcn_readfirstlane((int)nchk);
}
#undef FPP_GX_BODY
#undef FPP_GX_OPERANDS

// The serial loop over queue q with the re-test after each first miss: see fpp_group_x.
// gbg = the group's first node index.
__device__ __forceinline__ void fpp_refilter_loop(uint64_t q, uint64_t &touched, uint32_t &asg, uint32_t &rcf,
                                                  uint32_t &rmf, uint32_t &rcu, uint32_t rlab, uint32_t cpu,
                                                  uint32_t mem, uint32_t req, uint32_t conf, uint32_t gbg,
                                                  uint32_t &nchk, uint32_t qc, uint32_t qm) {
    // Stop at the first miss and re-test the rest of the queue, vector-parallel, against the
    // group's current state: a miss usually means the group just filled up for the batch's
    // sizes, so the containers behind it fail too (failed checks: 33 k of 71 k per config-4
    // scenario, 1.2 M of 1.96 M in config 3; almost none are visible at the queue's start).
    // The test is exact: the nodes of the batch corner (every node that could take the batch's
    // smallest demands) are broadcast and each queued lane tests its own container; one that
    // fits none of them now never will (monotone).  A large corner, or a re-test that drops
    // nothing, finishes the queue in the plain loop.
    fpp_asm_group_x<true>(q, touched, asg, rcf, rmf, rcu, rlab, cpu, mem, req, conf, gbg, nchk);
    while (q) {
        uint64_t e = (__builtin_amdgcn_ballot_w64(rcf >= qc) & __builtin_amdgcn_ballot_w64(rmf >= qm));
        uint64_t fit = 0;
        if (__builtin_popcountll(e) <= REFILTER_MAX) {
            bool ok = false;
            while (e) {
                const uint32_t l = (uint32_t)__builtin_ctzll(e);
                e &= e - 1;
                const uint32_t ncf = __builtin_amdgcn_readlane(rcf, l), nmf = __builtin_amdgcn_readlane(rmf, l);
                const uint32_t nlb = __builtin_amdgcn_readlane(rlab, l), ncu = __builtin_amdgcn_readlane(rcu, l);
                ok |= (ncf >= cpu) & (nmf >= mem) & (((req & nlb) | (conf & ncu)) == 0u);
            }
            fit = q & __builtin_amdgcn_ballot_w64(ok);
        } else {
            fit = q;
        }
        if (fit == q) {  // nothing to drop: the rest of the queue in the plain loop
            fpp_asm_group_x<false>(q, touched, asg, rcf, rmf, rcu, rlab, cpu, mem, req, conf, gbg, nchk);
            break;
        }
        q = fit;  // the dropped lanes keep asg = FP_NONE: misses of this group
        fpp_asm_group_x<true>(q, touched, asg, rcf, rmf, rcu, rlab, cpu, mem, req, conf, gbg, nchk);
    }
}

// The serial group loop (fpp_groups): the exec-masked loop with its re-test plus the per-group
// vector epilogue -- placed bits of the hits, next candidate group of the misses.
template <uint32_t g, uint32_t G, bool IB = false>
__device__ __forceinline__ void fpp_group_x(uint64_t q, uint64_t &placed, uint64_t &touched, uint32_t &asg,
                                            uint32_t &nxt, uint32_t &rcf, uint32_t &rmf, uint32_t &rcu,
                                            uint32_t rlab, uint32_t cpu, uint32_t mem, uint32_t req, uint32_t conf,
                                            uint32_t cand, uint32_t cand_hi, uint32_t gb64, uint32_t &nchk,
                                            uint32_t &nhit, uint32_t qc, uint32_t qm) {
    const uint64_t q0 = q;
    fpp_refilter_loop(q, touched, asg, rcf, rmf, rcu, rlab, cpu, mem, req, conf, gb64 + g * 64u, nchk, qc, qm);
    q = q0;
    uint64_t hit;
    if constexpr (IB) {  // one-wave kernels: q is a wave-uniform SGPR mask
        hit = q & __builtin_amdgcn_ballot_w64(asg != 0xFFFFFFFFu);
    } else {
        const bool inq = (q >> __lane_id()) & 1ull;
        hit = __builtin_amdgcn_ballot_w64(inq && asg != 0xFFFFFFFFu);
    }
#ifdef FP_PIPE_STATS
    nhit += (uint32_t)__builtin_popcountll(hit);
#else
    (void)nhit;
#endif
    placed |= hit;
    {  // the misses move on to their next candidate group (a select: no divergent branch)
        const uint64_t above = (((uint64_t)cand_hi << 32) | cand) & ~((2ull << g) - 1ull);
        const uint32_t nx = above ? (uint32_t)__builtin_ctzll(above) : G;
        if constexpr (IB) nxt = fpp_lane_sel<true>(q & ~hit, nx, nxt);
        else nxt = (((q >> __lane_id()) & 1ull) && asg == 0xFFFFFFFFu) ? nx : nxt;
    }
}

}  // namespace fpp
