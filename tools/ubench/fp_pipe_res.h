// Windowed exact first fit of one 64-node group with a SCALAR resolve (k_ffd_pipe's group loop).
//
// The serial loop (fpp_group_x, fp_pipe_asm.h) pays one wave-wide VALU -> SALU -> EXEC -> VALU
// round trip per queued container (~172 cycles).  Here the work is split in two:
//
//   1. Snapshot masks (vector, off the chain).  The group's live nodes -- those that can take the
//      batch's smallest demands, so every node a queued container may ever use -- are taken in
//      node order, at most 32 per chunk, and copied into lanes 0..K-1 of three table VGPRs
//      (slot k = the k-th live node).  Node-major over the slots, every queued container (one per
//      lane) tests the slot's record and shifts the result into its 32-bit slot mask: bit k =
//      "fits slot k at the chunk's start".
//   2. Scalar resolve (the chain).  Containers are taken in lane (= FFD) order.  A container's
//      first fit is the lowest slot k of its mask whose CURRENT record still fits it: a slot that
//      did not fit at the chunk's start never will (capacity only shrinks, conflict bits only
//      accumulate: SPEC.md 2.3 monotonicity), and a slot that did is re-tested on its current
//      record -- three v_readlane of the table, the three tests on the SALU, three v_writelane for
//      the placement.  No wave-wide compare, ballot or EXEC switch sits on the chain.
//
// Chunks: a group with more than 32 live nodes is resolved 32 live nodes at a time, in node order,
// each chunk taking the containers the previous one did not place, in order -- a pipeline over
// node ranges, which is the sequential first fit.
//
// A container with cpu = mem = conflict = 0 changes no record; the caller keeps such containers
// out of the queue (the all-zero ones) or sends the queue to the serial loop (label-only ones).
#pragma once
#include <stdint.h>

namespace fpp {

#ifndef FP_RES_MAX
#define FP_RES_MAX 32  // live nodes per chunk (32-bit slot masks; lane 63 is the sentinel)
#endif

// v_writelane_b32 by intrinsic name (no clang builtin in this toolchain)
extern "C" __device__ int fp_res_writelane(int val, int lane_sel, int old) __asm("llvm.amdgcn.writelane.i32");

// Resolve the queue q (lanes, FFD order) against the table (lanes 0..K-1 of tcf/tmf/tcu).
// vm: per-lane slot mask; out: per-lane slot placed on (unchanged on a miss).
// Lane 63 of the table is a sentinel, (0, 0, all conflict bits): an empty mask selects slot -1,
// whose readlane reads lane 63 (the low six bits of the select), where every container with a
// nonzero cpu, mem or conflict fails -- and the fail path ends the container with its mask
// empty.  A container with cpu = mem = conflict = 0 "lands" on the sentinel, which changes no
// record, and records slot -1 = 0xFFFFFFFF: a miss, as its empty mask says.
__device__ __forceinline__ void fpp_res_chain(uint64_t q, uint32_t vm, uint32_t cpu, uint32_t mem, uint32_t conf,
                                              uint32_t &tcf, uint32_t &tmf, uint32_t &tcu, uint32_t &out) {
    uint32_t t, m, c, mm, x, k, a, b, u, tt, m0sv;
    asm volatile(
        "s_mov_b32 %[m0sv], m0\n\t"
        "s_cmp_eq_u64 %[q], 0\n\t"
        "s_cbranch_scc1 .Lres_end%=\n"
        ".Lres_loop%=:\n\t"
        "s_ff1_i32_b64 %[t], %[q]\n\t"
        "v_readlane_b32 %[m], %[vm], %[t]\n\t"
        "v_readlane_b32 %[c], %[cpu], %[t]\n\t"
        "v_readlane_b32 %[mm], %[mem], %[t]\n\t"
        "v_readlane_b32 %[x], %[conf], %[t]\n\t"
        "s_bitset0_b64 %[q], %[t]\n"
        ".Lres_try%=:\n\t"
        "s_ff1_i32_b32 %[k], %[m]\n\t"
        "v_readlane_b32 %[a], %[tcf], %[k]\n\t"
        "v_readlane_b32 %[b], %[tmf], %[k]\n\t"
        "v_readlane_b32 %[u], %[tcu], %[k]\n\t"
        "s_and_b32 %[tt], %[u], %[x]\n\t"
        "s_cbranch_scc1 .Lres_fail%=\n\t"
        "s_sub_u32 %[a], %[a], %[c]\n\t"
        "s_cbranch_scc1 .Lres_fail%=\n\t"
        "s_sub_u32 %[b], %[b], %[mm]\n\t"
        "s_cbranch_scc1 .Lres_fail%=\n\t"
        "s_or_b32 %[u], %[u], %[x]\n\t"
        "s_mov_b32 m0, %[k]\n\t"
        "v_writelane_b32 %[tcf], %[a], m0\n\t"
        "v_writelane_b32 %[tmf], %[b], m0\n\t"
        "v_writelane_b32 %[tcu], %[u], m0\n\t"
        "s_mov_b32 m0, %[t]\n\t"
        "v_writelane_b32 %[out], %[k], m0\n\t"
        "s_cmp_lg_u64 %[q], 0\n\t"
        "s_cbranch_scc1 .Lres_loop%=\n\t"
        "s_branch .Lres_end%=\n"
        ".Lres_fail%=:\n\t"
        "s_bitset0_b32 %[m], %[k]\n\t"
        "s_cmp_lg_u32 %[m], 0\n\t"
        "s_cbranch_scc1 .Lres_try%=\n\t"
        "s_cmp_lg_u64 %[q], 0\n\t"
        "s_cbranch_scc1 .Lres_loop%=\n"
        ".Lres_end%=:\n\t"
        "s_mov_b32 m0, %[m0sv]"
        : [q] "+s"(q), [tcf] "+v"(tcf), [tmf] "+v"(tmf), [tcu] "+v"(tcu), [out] "+v"(out), [t] "=&s"(t),
          [m] "=&s"(m), [c] "=&s"(c), [mm] "=&s"(mm), [x] "=&s"(x), [k] "=&s"(k), [a] "=&s"(a), [b] "=&s"(b),
          [u] "=&s"(u), [tt] "=&s"(tt), [m0sv] "=&s"(m0sv)
        : [vm] "v"(vm), [cpu] "v"(cpu), [mem] "v"(mem), [conf] "v"(conf)
        : "scc", "memory");
}

// One group's queue q.  Records rcf/rmf/rcu/rlab (lane = node; rlab = ~labels), containers
// cpu/mem/req/conf (lane = queue position), batch corner (qc, qm).  Placed containers get
// asg = gbg | node lane; touched |= nodes placed on.  Returns the queued lanes left unplaced.
// PERM: the table is compacted by one ds_permute per record (live lane l pushes to lane slot(l)),
// else by K v_writelane per record (microbenchmark A/B).
template <bool PERM = true>
__device__ __forceinline__ uint64_t fpp_res_group(uint64_t q, uint64_t &touched, uint32_t &asg, uint32_t &rcf,
                                                  uint32_t &rmf, uint32_t &rcu, uint32_t rlab, uint32_t cpu,
                                                  uint32_t mem, uint32_t req, uint32_t conf, uint32_t gbg,
                                                  uint32_t qc, uint32_t qm) {
    const uint32_t lane = __lane_id();
    uint64_t live = __builtin_amdgcn_ballot_w64((rcf >= qc) & (rmf >= qm));
    while (live && q) {
        // the chunk: the lowest FP_RES_MAX live nodes
        uint64_t ch = live;
        if (__builtin_popcountll(ch) > FP_RES_MAX) {
            uint64_t e = ch;
#pragma unroll 1
            for (int i = 0; i < FP_RES_MAX; ++i) e &= e - 1;
            ch &= ~e;
        }
        live &= ~ch;
        const uint32_t K = (uint32_t)__builtin_popcountll(ch);
        // slot of a live lane = live lanes below it
        const uint32_t my = __builtin_amdgcn_mbcnt_hi((uint32_t)(ch >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ch, 0u));
        const bool in = (ch >> lane) & 1ull;
        uint32_t tcf, tmf, tcu, tln, vm = 0;
        if (PERM) {
            // live lane l -> lane slot(l); the others park on lane 62 (K <= 32: never a slot)
            const int dst = (int)((in ? my : 62u) << 2);
            tcf = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)rcf);
            tmf = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)rmf);
            tcu = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)rcu);
            const uint32_t tnl = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)rlab);
            tln = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)lane);
            // slot masks, node-major from the highest slot down (bit k = slot k)
#pragma unroll 1
            for (uint32_t k = K; k-- > 0;) {
                const uint32_t cf = __builtin_amdgcn_readlane(tcf, k), mf = __builtin_amdgcn_readlane(tmf, k);
                const uint32_t cu = __builtin_amdgcn_readlane(tcu, k), nl = __builtin_amdgcn_readlane(tnl, k);
                const bool fit = (cpu <= cf) & (mem <= mf) & (((req & nl) | (conf & cu)) == 0u);
                vm = (vm << 1) | (fit ? 1u : 0u);
            }
        } else {
            tcf = 0; tmf = 0; tcu = 0; tln = 0;
            uint64_t e = ch;
            for (uint32_t k = K; k-- > 0;) {
                const uint32_t l = 63u - (uint32_t)__builtin_clzll(e);
                e &= ~(1ull << l);
                const uint32_t cf = __builtin_amdgcn_readlane(rcf, l), mf = __builtin_amdgcn_readlane(rmf, l);
                const uint32_t cu = __builtin_amdgcn_readlane(rcu, l), nl = __builtin_amdgcn_readlane(rlab, l);
                const bool fit = (cpu <= cf) & (mem <= mf) & (((req & nl) | (conf & cu)) == 0u);
                vm = (vm << 1) | (fit ? 1u : 0u);
                tcf = (uint32_t)fp_res_writelane((int)cf, (int)k, (int)tcf);
                tmf = (uint32_t)fp_res_writelane((int)mf, (int)k, (int)tmf);
                tcu = (uint32_t)fp_res_writelane((int)cu, (int)k, (int)tcu);
                tln = (uint32_t)fp_res_writelane((int)l, (int)k, (int)tln);
            }
        }
        // lane 63: the sentinel (fpp_res_chain)
        if (lane == 63) { tcf = 0u; tmf = 0u; tcu = 0xFFFFFFFFu; }
        uint32_t slot = 0xFFFFFFFFu;
        fpp_res_chain(q, vm, cpu, mem, conf, tcf, tmf, tcu, slot);
        // write the chunk's records back: live lane l holds slot popcount(ch below l)
        const uint32_t ncf = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(my << 2), (int)tcf);
        const uint32_t nmf = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(my << 2), (int)tmf);
        const uint32_t ncu = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(my << 2), (int)tcu);
        touched |= __builtin_amdgcn_ballot_w64(in && (ncf != rcf || nmf != rmf || ncu != rcu));
        if (in) { rcf = ncf; rmf = nmf; rcu = ncu; }
        // placed containers: slot -> node lane
        const bool hit = ((q >> lane) & 1ull) && slot != 0xFFFFFFFFu;
        const uint32_t nl = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((slot & 63u) << 2), (int)tln);
        if (hit) asg = gbg | nl;
        q &= ~__builtin_amdgcn_ballot_w64(hit);
    }
    return q;
}

// Drop-in for fpp_group_x in the group-major loop: the resolve, then the per-group epilogue
// (placed bits of the hits, next candidate group of the misses).
template <uint32_t g, uint32_t G>
__device__ __forceinline__ void fpp_group_res(uint64_t q, uint64_t &placed, uint64_t &touched, uint32_t &asg,
                                              uint32_t &nxt, uint32_t &rcf, uint32_t &rmf, uint32_t &rcu,
                                              uint32_t rlab, uint32_t cpu, uint32_t mem, uint32_t req, uint32_t conf,
                                              uint32_t cand, uint32_t cand_hi, uint32_t gb64, uint32_t &nhit,
                                              uint32_t qc, uint32_t qm) {
    const uint64_t left = fpp_res_group<true>(q, touched, asg, rcf, rmf, rcu, rlab, cpu, mem, req, conf,
                                              gb64 + g * 64u, qc, qm);
    const uint64_t hit = q & ~left;
#ifdef FP_PIPE_STATS
    nhit += (uint32_t)__builtin_popcountll(hit);
#else
    (void)nhit;
#endif
    placed |= hit;
    const uint32_t lane = __lane_id();
    if ((left >> lane) & 1ull) {
        const uint64_t above = (((uint64_t)cand_hi << 32) | cand) & ~((2ull << g) - 1ull);
        nxt = above ? (uint32_t)__builtin_ctzll(above) : G;
    }
}

}  // namespace fpp
