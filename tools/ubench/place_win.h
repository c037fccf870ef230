// Windowed first fit over one 64-node group (k_ffd_pipe's group-major loop, one group).
//
// fpp_asm_group (fp_pipe_asm.h) re-evaluates the group's vector records for every queued
// container: v_cmp into scalar masks, then readlanes / writelanes for the placement -- about
// four VALU <-> SALU round trips (~50 cycles each on gfx950) per container on the FFD chain.
// Here the queue is taken FP_WIN containers at a time:
//   1. every container of the window gets its feasibility mask over the 64 nodes from the
//      records at the window's start (independent VALU work, the round trips overlap);
//   2. the window is resolved in order on the scalar unit (one asm block per container,
//      fpw_resolve).  A node no container of the window has been placed on still has its
//      window-start record, so its mask bit is exact; a node placed on in the window is
//      re-checked on its current record (capacity and conflicts -- labels never change).
//      Monotonicity (SPEC.md 2.3): a node infeasible at the window start stays infeasible, so
//      the first surviving bit is the sequential first fit;
//   3. the record of the node placed on last lives in SGPRs (a fill-phase queue lands on one
//      node many times in a row) and goes back to the vector records when another node is
//      placed on and at the window's end.
// Bit for bit the sequential first fit of fpp_asm_group (tools/ubench/place.hip checks both
// on the same queues; the GPU parity tests check the pipeline against the oracle).
#pragma once
#include <stdint.h>

namespace fpp {

// v_writelane_b32 (no clang builtin for it in this toolchain; the LLVM intrinsic by name)
extern "C" __device__ int fp_writelane(int val, int lane_sel, int old) __asm("llvm.amdgcn.writelane.i32");

#ifndef FP_WIN
#define FP_WIN 8
#endif

#ifdef FP_PIPE_STATS
#define FPW_CNT_CHECK "s_add_u32 %[nchk], %[nchk], 1\n\t"
#define FPW_CNT_HIT "s_add_u32 %[nhit], %[nhit], 1\n\t"
#else
#define FPW_CNT_CHECK ""
#define FPW_CNT_HIT ""
#endif

// Resolve container t (lane t of the queue; t >= 64: empty window slot) against its
// window-start mask m; (kc, km, kx) = its cpu, memory and conflict bits.  State: tw = nodes
// placed on in this window; (cn, ccf, cmf, ccu) = the SGPR copy of node cn's current record
// (always a real node: the window starts with node 0 cached).  A hit writes asg[t] and sets
// placed bit t; a miss writes nxt[t] = the container's next candidate group above g (G: none).
// Straight-line for the common cases (land on the cached node, or on the first untouched
// candidate); the general loop over touched candidates is the rare slow path.
template <uint32_t g, uint32_t G>
__device__ __forceinline__ void fpw_resolve(uint32_t t, uint64_t m, uint32_t kc, uint32_t km, uint32_t kx,
                                            uint64_t &tw, uint32_t &cn, uint32_t &ccf, uint32_t &cmf, uint32_t &ccu,
                                            uint64_t &placed, uint32_t &asg, uint32_t &nxt, uint32_t &rcf,
                                            uint32_t &rmf, uint32_t &rcu, uint32_t cand, uint32_t cand_hi,
                                            uint32_t gbg, uint32_t &nchk, uint32_t &nhit) {
    constexpr uint32_t nmask = g < 32 ? ~((2u << g) - 1u) : 0u;  // candidate groups above g
    constexpr uint32_t nmask_hi = g < 32 ? 0xFFFFFFFFu : ~((2u << (g & 31)) - 1u);
    uint32_t fc, xu, xo, best, tmp, xcf, xmf, xcu, m0sv;
    uint64_t u, o;
    asm volatile(
        "s_cmp_gt_u32 %[t], 63\n\t"
        "s_cbranch_scc1 .Lfw_end%=\n\t"
        FPW_CNT_CHECK
        // fc: the cached node is a candidate and still fits
        "s_bitcmp1_b64 %[m], %[cn]\n\t"
        "s_cselect_b32 %[fc], 1, 0\n\t"
        "s_cmp_ge_u32 %[ccf], %[kc]\n\t"
        "s_cselect_b32 %[fc], %[fc], 0\n\t"
        "s_cmp_ge_u32 %[cmf], %[km]\n\t"
        "s_cselect_b32 %[fc], %[fc], 0\n\t"
        "s_and_b32 %[tmp], %[ccu], %[kx]\n\t"
        "s_cselect_b32 %[fc], 0, %[fc]\n\t"
        // xu: first untouched candidate (exact); xo: first touched, uncached candidate
        "s_andn2_b64 %[u], %[m], %[tw]\n\t"
        "s_ff1_i32_b64 %[xu], %[u]\n\t"
        "s_and_b64 %[o], %[m], %[tw]\n\t"
        "s_bitset0_b64 %[o], %[cn]\n\t"
        "s_ff1_i32_b64 %[xo], %[o]\n\t"
        "s_cmp_eq_u32 %[fc], 0\n\t"
        "s_cselect_b32 %[best], -1, %[cn]\n\t"
        "s_min_u32 %[best], %[best], %[xu]\n\t"    // -1 (none) is the largest unsigned
        "s_cmp_lt_u32 %[xo], %[best]\n\t"
        "s_cbranch_scc1 .Lfw_slow%=\n"
        ".Lfw_pick%=:\n\t"
        "s_cmp_eq_u32 %[best], %[cn]\n\t"
        "s_cbranch_scc1 .Lfw_place%=\n\t"
        "s_cmp_eq_u32 %[best], -1\n\t"
        "s_cbranch_scc1 .Lfw_miss%=\n\t"
        // node best becomes the cached node: write the old one back, load best's record
        "s_mov_b32 %[m0sv], m0\n\t"
        "s_mov_b32 m0, %[cn]\n\t"
        "v_writelane_b32 %[rcf], %[ccf], m0\n\t"
        "v_writelane_b32 %[rmf], %[cmf], m0\n\t"
        "v_writelane_b32 %[rcu], %[ccu], m0\n\t"
        "s_mov_b32 m0, %[m0sv]\n\t"
        "s_nop 0\n\t"                                // v_writelane -> v_readlane of the same VGPR
        "v_readlane_b32 %[ccf], %[rcf], %[best]\n\t"
        "v_readlane_b32 %[cmf], %[rmf], %[best]\n\t"
        "v_readlane_b32 %[ccu], %[rcu], %[best]\n\t"
        "s_mov_b32 %[cn], %[best]\n"
        ".Lfw_place%=:\n\t"
        FPW_CNT_HIT
        "s_sub_u32 %[ccf], %[ccf], %[kc]\n\t"
        "s_sub_u32 %[cmf], %[cmf], %[km]\n\t"
        "s_or_b32 %[ccu], %[ccu], %[kx]\n\t"
        "s_bitset1_b64 %[tw], %[cn]\n\t"
        "s_bitset1_b64 %[placed], %[t]\n\t"
        "s_or_b32 %[tmp], %[gbg], %[cn]\n\t"
        "s_mov_b32 %[m0sv], m0\n\t"
        "s_mov_b32 m0, %[t]\n\t"
        "v_writelane_b32 %[asg], %[tmp], m0\n\t"
        "s_mov_b32 m0, %[m0sv]\n\t"
        "s_branch .Lfw_end%=\n"
        ".Lfw_slow%=:\n\t"
        // a node placed on earlier in the window (not the cached one) comes first: check the
        // touched, uncached candidates below best one by one on their (current) vector records
        "v_readlane_b32 %[xcf], %[rcf], %[xo]\n\t"
        "v_readlane_b32 %[xmf], %[rmf], %[xo]\n\t"
        "v_readlane_b32 %[xcu], %[rcu], %[xo]\n\t"
        "s_bitset0_b64 %[o], %[xo]\n\t"
        "s_cmp_ge_u32 %[xcf], %[kc]\n\t"
        "s_cselect_b32 %[tmp], 1, 0\n\t"
        "s_cmp_ge_u32 %[xmf], %[km]\n\t"
        "s_cselect_b32 %[tmp], %[tmp], 0\n\t"
        "s_and_b32 %[xcu], %[xcu], %[kx]\n\t"
        "s_cselect_b32 %[tmp], 0, %[tmp]\n\t"
        "s_cmp_eq_u32 %[tmp], 0\n\t"
        "s_cselect_b32 %[best], %[best], %[xo]\n\t"
        "s_cbranch_scc0 .Lfw_pick%=\n\t"           // xo fits: it is the first fit
        "s_ff1_i32_b64 %[xo], %[o]\n\t"
        "s_cmp_lt_u32 %[xo], %[best]\n\t"
        "s_cbranch_scc1 .Lfw_slow%=\n\t"
        "s_branch .Lfw_pick%=\n"
        ".Lfw_miss%=:\n\t"
        // no node of g: the container's next candidate group (none: G)
        "v_readlane_b32 %[xcf], %[cand], %[t]\n\t"
        "v_readlane_b32 %[xmf], %[candhi], %[t]\n\t"
        "s_and_b32 %[xcf], %[xcf], %[nmask]\n\t"
        "s_and_b32 %[xmf], %[xmf], %[nmaskhi]\n\t"
        "s_ff1_i32_b32 %[xcu], %[xmf]\n\t"
        "s_add_u32 %[xcu], %[xcu], 32\n\t"
        "s_cmp_eq_u32 %[xmf], 0\n\t"
        "s_cselect_b32 %[xcu], %[gnone], %[xcu]\n\t"
        "s_ff1_i32_b32 %[tmp], %[xcf]\n\t"
        "s_cmp_eq_u32 %[xcf], 0\n\t"
        "s_cselect_b32 %[tmp], %[xcu], %[tmp]\n\t"
        "s_mov_b32 %[m0sv], m0\n\t"
        "s_mov_b32 m0, %[t]\n\t"
        "v_writelane_b32 %[nxt], %[tmp], m0\n\t"
        "s_mov_b32 m0, %[m0sv]\n"
        ".Lfw_end%=:"
        : [tw] "+s"(tw), [cn] "+s"(cn), [ccf] "+s"(ccf), [cmf] "+s"(cmf), [ccu] "+s"(ccu), [placed] "+s"(placed),
          [asg] "+v"(asg), [nxt] "+v"(nxt), [rcf] "+v"(rcf), [rmf] "+v"(rmf), [rcu] "+v"(rcu), [nchk] "+s"(nchk),
          [nhit] "+s"(nhit), [fc] "=&s"(fc), [xu] "=&s"(xu), [xo] "=&s"(xo), [best] "=&s"(best), [tmp] "=&s"(tmp),
          [xcf] "=&s"(xcf), [xmf] "=&s"(xmf), [xcu] "=&s"(xcu), [m0sv] "=&s"(m0sv), [u] "=&s"(u), [o] "=&s"(o)
        : [t] "s"(t), [m] "s"(m), [kc] "s"(kc), [km] "s"(km), [kx] "s"(kx), [cand] "v"(cand),
          [candhi] "v"(cand_hi), [gbg] "s"(gbg), [nmask] "i"(nmask), [nmaskhi] "i"(nmask_hi), [gnone] "i"(G)
        : "scc", "memory");
}

template <uint32_t g, uint32_t G>
__device__ __forceinline__ void fpw_group(uint64_t q, uint64_t &placed, uint64_t &touched, uint32_t &asg,
                                          uint32_t &nxt, uint32_t &rcf, uint32_t &rmf, uint32_t &rcu, uint32_t rlab,
                                          uint32_t cpu, uint32_t mem, uint32_t req, uint32_t conf, uint32_t cand,
                                          uint32_t cand_hi, uint32_t gb64, uint32_t &nchk, uint32_t &nhit) {
    const uint32_t gbg = gb64 + g * 64u;  // gb64 is a multiple of 64: node index = gbg | lane
    while (q) {
        uint64_t M[FP_WIN];
        uint32_t T[FP_WIN], KC[FP_WIN], KM[FP_WIN], KX[FP_WIN];
#pragma unroll
        for (int j = 0; j < FP_WIN; ++j) {
            T[j] = q ? (uint32_t)__builtin_ctzll(q) : 64u;
            q &= q - 1;
            const uint32_t t = T[j] & 63u;
            KC[j] = __builtin_amdgcn_readlane(cpu, t);
            KM[j] = __builtin_amdgcn_readlane(mem, t);
            KX[j] = __builtin_amdgcn_readlane(conf, t);
            const uint32_t c_req = __builtin_amdgcn_readlane(req, t);
            M[j] = __builtin_amdgcn_ballot_w64(rcf >= KC[j]) & __builtin_amdgcn_ballot_w64(rmf >= KM[j]) &
                   __builtin_amdgcn_ballot_w64(((rlab & c_req) | (rcu & KX[j])) == 0u);
        }
        uint64_t tw = 0;
        uint32_t cn = 0;
        uint32_t ccf = __builtin_amdgcn_readlane(rcf, 0), cmf = __builtin_amdgcn_readlane(rmf, 0),
                 ccu = __builtin_amdgcn_readlane(rcu, 0);
#pragma unroll
        for (int j = 0; j < FP_WIN; ++j)
            fpw_resolve<g, G>(T[j], M[j], KC[j], KM[j], KX[j], tw, cn, ccf, cmf, ccu, placed, asg, nxt, rcf, rmf, rcu,
                              cand, cand_hi, gbg, nchk, nhit);
        rcf = (uint32_t)fp_writelane((int)ccf, (int)cn, (int)rcf);
        rmf = (uint32_t)fp_writelane((int)cmf, (int)cn, (int)rmf);
        rcu = (uint32_t)fp_writelane((int)ccu, (int)cn, (int)rcu);
        touched |= tw;
    }
}

}  // namespace fpp
