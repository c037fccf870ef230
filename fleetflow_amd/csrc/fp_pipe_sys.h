// Systolic exact first fit of one 64-node group (k_ffd_pipe's group loop for long queues).
//
// The serial loop (fpp_group_x, fp_pipe_asm.h) checks one queued container per iteration
// against all 64 nodes: ~172 cycles of a VALU -> SALU -> EXEC -> VALU dependency chain per
// container, so a group that fills with ~480 containers keeps its stage busy for ~35 us and
// the config-3 front advances one group at a time.
//
// Here the NODES travel instead: the group's live nodes (those that can take the batch's
// smallest demands) are compacted into positions 0..L-1 and rotated one lane per step
// (DPP wave_ror:1), while the queued containers sit still, compacted into lanes 0..Q-1 in
// FFD order.  At step tau lane t holds position tau - t, so
//   * container t tests positions 0, 1, 2, ... at steps t, t+1, t+2, ... (first fit order);
//   * position p meets containers 0, 1, 2, ... at steps p, p+1, ... (FFD order),
// and every (container, node) test sees exactly the placements of the earlier containers
// on that node: the sequential first fit, bit for bit.  A step is ~20 wave instructions for
// up to 64 tests, so a queue of Q containers that mostly fits costs ~Q + (first-fit
// position) steps instead of Q serial checks.
//
// Containers still pending after `max_steps` finish in the serial loop with the node state
// of that moment.  That is exact too: a pending container t has failed positions <= tau - t,
// which stay infeasible (capacity only shrinks, SPEC.md 2.3), and every earlier pending
// container is checked before it.
#pragma once
#include <stdint.h>

#include "fp_pipe_asm.h"

namespace fpp {

#ifdef FP_PIPE_STATS
// systolic-call diagnostics (FP_PIPE_STATS_FINE builds, tools/sys_stats.py): [0] calls [1] queued Q
// [2] live L [3] steps [4] placed [5] live nodes that fit at least one queued container (2-D +
// labels/conflicts, batch-start state) [6] largest placement position + 1, summed over calls.  A
// loop over the queue and seven atomics per call: they doubled config 3's plain diagnostics time
__device__ unsigned long long g_sys_stats[8];
#endif

__device__ __forceinline__ uint32_t sys_push(uint32_t dst_lane, uint32_t v) {  // ds_permute_b32
    return (uint32_t)__builtin_amdgcn_ds_permute((int)(dst_lane << 2), (int)v);
}
__device__ __forceinline__ uint32_t sys_pull(uint32_t src_lane, uint32_t v) {  // ds_bpermute_b32
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)v);
}
// OR over the wave of a 32-bit value (DPP row shifts + row broadcasts, then lane 63)
__device__ __forceinline__ uint32_t sys_wave_or(uint32_t x) {
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);   // row_shr:1
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);   // row_shr:2
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);   // row_shr:4
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);   // row_shr:8
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// (Measured and removed in round 4, numbers in DESIGN.md 4.3: narrowing the live set to the
// queue's (cpu, mem) staircase, 65.2 vs 64.3 ms on config 3; ending the step loop at its first
// miss, 66.8 vs 64 ms; re-testing the serial finish after each miss, no difference.)

// One group's queue q (lanes = containers in FFD order; cpu/mem/req/conf per lane) against
// the group's records (lane = node: rcf, rmf, rcu, rlab = ~labels).  qc/qm: the batch's
// smallest cpu / mem demands (a superset bound: nodes below them are never live).
// Returns in asg the node (gbg | l) of every placed queued lane and FP_NONE for the others
// of q (left for the caller: misses, or `left` = still pending for the serial finish);
// touched |= the nodes placed on.
// The step loop.
// Phase A (tau < L): the window of started containers grows by one lane per step,
// win = lanes 0..tau.  Phase B (tau >= L): it slides, win = lanes tau-L+1..tau, and
// container tau - L, which has tested every live position, leaves `pend` (a miss).
// Per step: exec = win & pend, three v_cmpx narrow it to the containers that fit the
// position in their lane (EXEC = EXEC & test on gfx950), the placement is three VALU
// ops under that exec, then the node records rotate one lane (DPP wave_ror:1).
// The loop ends when pend is empty, or (phase B) after max_steps steps; on exit
// tau = the rotations applied.  Wait states: a VALU write of a rotated register, and
// v_cmpx's EXEC write, are >= 5 instructions ahead of the DPP reading it.
// Assumes every lane of the wave is active (k_ffd_pipe's group loop).
__device__ __forceinline__ void fpp_sys_steps(uint32_t &xc, uint32_t &xm, uint32_t &xu, uint32_t &xl, uint32_t kc,
                                              uint32_t km, uint32_t kr, uint32_t kx, uint32_t &apos, uint64_t &pend,
                                              uint32_t &tau, uint32_t L, uint32_t max_steps) {
    uint64_t win = 0, esv;
    uint32_t u = 0, t0;
    asm volatile(
        "s_mov_b64 %[esv], exec\n"
        ".LsysA%=:\n\t"
        "s_lshl_b64 %[win], %[win], 1\n\t"
        "s_bitset1_b64 %[win], 0\n\t"
        "s_and_b64 exec, %[win], %[pend]\n\t"
        "v_cmpx_ge_u32_e32 vcc, %[xc], %[kc]\n\t"
        "v_cmpx_ge_u32_e32 vcc, %[xm], %[km]\n\t"
        "v_and_b32_e32 %[t0], %[xl], %[kr]\n\t"
        "v_and_or_b32 %[t0], %[xu], %[kx], %[t0]\n\t"
        "v_cmpx_eq_u32_e32 vcc, 0, %[t0]\n\t"
        "v_sub_u32_e32 %[xc], %[xc], %[kc]\n\t"
        "v_sub_u32_e32 %[xm], %[xm], %[km]\n\t"
        "v_or_b32_e32 %[xu], %[xu], %[kx]\n\t"
        "v_mov_b32_e32 %[apos], %[tau]\n\t"
        "s_andn2_b64 %[pend], %[pend], exec\n\t"
        "s_cbranch_scc0 .LsysEnd%=\n\t"
        "s_mov_b64 exec, %[esv]\n\t"
        "s_add_u32 %[tau], %[tau], 1\n\t"
        "v_mov_b32_dpp %[xl], %[xl] wave_ror:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %[xc], %[xc] wave_ror:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %[xm], %[xm] wave_ror:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %[xu], %[xu] wave_ror:1 row_mask:0xf bank_mask:0xf\n\t"
        "s_cmp_lt_u32 %[tau], %[L]\n\t"
        "s_cbranch_scc1 .LsysA%=\n"
        ".LsysB%=:\n\t"
        "s_cmp_ge_u32 %[tau], %[cap]\n\t"
        "s_cbranch_scc1 .LsysEnd%=\n\t"
        "s_lshl_b64 %[win], %[win], 1\n\t"
        "s_bitset0_b64 %[pend], %[u]\n\t"
        "s_add_u32 %[u], %[u], 1\n\t"
        "s_and_b64 exec, %[win], %[pend]\n\t"
        "v_cmpx_ge_u32_e32 vcc, %[xc], %[kc]\n\t"
        "v_cmpx_ge_u32_e32 vcc, %[xm], %[km]\n\t"
        "v_and_b32_e32 %[t0], %[xl], %[kr]\n\t"
        "v_and_or_b32 %[t0], %[xu], %[kx], %[t0]\n\t"
        "v_cmpx_eq_u32_e32 vcc, 0, %[t0]\n\t"
        "v_sub_u32_e32 %[xc], %[xc], %[kc]\n\t"
        "v_sub_u32_e32 %[xm], %[xm], %[km]\n\t"
        "v_or_b32_e32 %[xu], %[xu], %[kx]\n\t"
        "v_mov_b32_e32 %[apos], %[tau]\n\t"
        "s_add_u32 %[tau], %[tau], 1\n\t"
        "s_andn2_b64 %[pend], %[pend], exec\n\t"
        "s_mov_b64 exec, %[esv]\n\t"
        "v_mov_b32_dpp %[xl], %[xl] wave_ror:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %[xc], %[xc] wave_ror:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %[xm], %[xm] wave_ror:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %[xu], %[xu] wave_ror:1 row_mask:0xf bank_mask:0xf\n\t"
        "s_cbranch_scc1 .LsysB%=\n"
        ".LsysEnd%=:\n\t"
        "s_mov_b64 exec, %[esv]"
        : [xc] "+v"(xc), [xm] "+v"(xm), [xu] "+v"(xu), [xl] "+v"(xl), [apos] "+v"(apos), [pend] "+s"(pend),
          [tau] "+s"(tau), [win] "+s"(win), [u] "+s"(u), [esv] "=&s"(esv), [t0] "=&v"(t0)
        : [kc] "v"(kc), [km] "v"(km), [kr] "v"(kr), [kx] "v"(kx), [L] "s"(L), [cap] "s"(max_steps)
        : "scc", "vcc", "memory");
    pend = fpp_uniform64(pend);
    tau = (uint32_t)__builtin_amdgcn_readfirstlane((int)tau);
}

struct SysOut {
    uint64_t left;  // queued lanes not resolved within max_steps (serial finish)
};

__device__ __forceinline__ SysOut fpp_sys_group(uint64_t q, uint64_t &touched, uint32_t &asg, uint32_t &rcf,
                                                uint32_t &rmf, uint32_t &rcu, uint32_t rlab, uint32_t cpu,
                                                uint32_t mem, uint32_t req, uint32_t conf, uint32_t gbg, uint32_t qc,
                                                uint32_t qm, uint32_t max_steps) {
    const uint32_t lane = __lane_id();
    const uint64_t below = (1ull << lane) - 1ull;
    SysOut out{0};
    // live nodes: the batch corner (a node outside it fits no container of the batch, now or
    // later) -> positions 0..L-1, in node order
    const uint64_t lm = (__builtin_amdgcn_ballot_w64(rcf >= qc) & __builtin_amdgcn_ballot_w64(rmf >= qm));
    const uint32_t L = (uint32_t)__builtin_popcountll(lm);
    if (L == 0) {  // nothing can fit: every queued container misses the group
        if ((q >> lane) & 1ull) asg = 0xFFFFFFFFu;
        return out;
    }
    // (A per-call prefilter -- label union, conflict intersection and the largest free cpu /
    // mem over the live nodes, four wave reductions -- cost more than the misses it dropped:
    // config 3 65.2 -> 68.7 ms.  Misses end at the step cap and in the serial finish instead.)
    const bool inq = (q >> lane) & 1ull;
    const uint32_t Q = (uint32_t)__builtin_popcountll(q);
    // containers -> lanes 0..Q-1 (rank among the queued), the others after them
    const uint32_t rq = inq ? (uint32_t)__builtin_popcountll(q & below) : Q + (uint32_t)__builtin_popcountll(~q & below);
    const uint32_t kc = sys_push(rq, cpu), km = sys_push(rq, mem), kr = sys_push(rq, req), kx = sys_push(rq, conf);
    const bool live = (lm >> lane) & 1ull;
    const uint32_t pos = live ? (uint32_t)__builtin_popcountll(lm & below) : L + (uint32_t)__builtin_popcountll(~lm & below);
    // position p starts at lane (64 - p) & 63: after tau rotations lane t holds position tau - t
    const uint32_t at0 = (64u - pos) & 63u;
    uint32_t xc = sys_push(at0, rcf), xm = sys_push(at0, rmf), xu = sys_push(at0, rcu), xl = sys_push(at0, rlab);
    const uint32_t pmap = sys_push(pos, lane);  // lane p: the node lane of position p
    if (((64u - lane) & 63u) >= L) {             // filler positions fit nothing
        xc = 0u; xm = 0u; xu = 0xFFFFFFFFu; xl = 0xFFFFFFFFu;
    }
    uint64_t pend = Q >= 64 ? ~0ull : ((1ull << Q) - 1ull);  // compacted containers still open
    uint32_t tau = 0;                                         // steps taken = rotations applied
    uint32_t apos = 0xFFFFFFFFu;                              // step of the placement (compacted lane)
    fpp_sys_steps(xc, xm, xu, xl, kc, km, kr, kx, apos, pend, tau, L, max_steps);
#if defined(FP_PIPE_STATS) && defined(FP_PIPE_STATS_FINE)
    {
        // live nodes some queued container fits at the batch-start state (before the steps: the
        // records below are still the node lanes' own)
        bool useful = false;
        uint64_t qq = q;
        while (qq) {
            const uint32_t t = (uint32_t)__builtin_ctzll(qq);
            qq &= qq - 1;
            const uint32_t c_c = __builtin_amdgcn_readlane(cpu, t), c_m = __builtin_amdgcn_readlane(mem, t);
            const uint32_t c_r = __builtin_amdgcn_readlane(req, t), c_x = __builtin_amdgcn_readlane(conf, t);
            useful |= (rcf >= c_c) & (rmf >= c_m) & (((rlab & c_r) | (rcu & c_x)) == 0u);
        }
        const uint32_t nu = (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(useful && live));
        const uint32_t maxp = apos != 0xFFFFFFFFu ? ((apos - lane) & 63u) + 1u : 0u;
        uint32_t mp = maxp;
        for (uint32_t o = 32; o; o >>= 1) mp = max(mp, (uint32_t)__shfl_xor((int)mp, (int)o));
        if (lane == 0) {
            atomicAdd(&g_sys_stats[0], 1ull);
            atomicAdd(&g_sys_stats[1], (unsigned long long)Q);
            atomicAdd(&g_sys_stats[2], (unsigned long long)L);
            atomicAdd(&g_sys_stats[3], (unsigned long long)tau);
            atomicAdd(&g_sys_stats[5], (unsigned long long)nu);
            atomicAdd(&g_sys_stats[6], (unsigned long long)mp);
        }
        const uint32_t npl = (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(apos != 0xFFFFFFFFu));
        if (lane == 0) atomicAdd(&g_sys_stats[4], (unsigned long long)npl);
    }
#endif
    // records back to node lanes: after tau rotations position p is at lane (tau - p) & 63
    const uint32_t src = (tau - pos) & 63u;
    const uint32_t ncf = sys_pull(src, xc), nmf = sys_pull(src, xm), ncu = sys_pull(src, xu);
    if (live) { rcf = ncf; rmf = nmf; rcu = ncu; }
    // placements: position -> node lane, then back to the container's own lane
    if (apos != 0xFFFFFFFFu) apos = (apos - lane) & 63u;  // step -> position tested at that step
    const uint32_t nl = sys_pull(apos & 63u, pmap);
    const uint32_t cnode = apos != 0xFFFFFFFFu ? gbg + nl : 0xFFFFFFFFu;
    const uint32_t back = sys_pull(rq, cnode);
    const uint64_t pend_here = (uint64_t)sys_pull(rq, (uint32_t)((pend >> lane) & 1ull));  // pend bit of my rank
    if (inq) asg = back;
    out.left = __builtin_amdgcn_ballot_w64(inq && pend_here != 0);
    // nodes placed on: OR of the one-hot node bits of the placed containers
    const uint32_t bl = apos != 0xFFFFFFFFu && nl < 32 ? 1u << nl : 0u;
    const uint32_t bh = apos != 0xFFFFFFFFu && nl >= 32 ? 1u << (nl - 32) : 0u;
    touched |= ((uint64_t)sys_wave_or(bh) << 32) | sys_wave_or(bl);
    return out;
}

}  // namespace fpp

#include "fp_pipe_sysv.h"
#include "fp_pipe_sysd.h"

namespace fpp {

// Drop-in for fpp_group_x (same arguments): the systolic loop, the serial finish of what it
// left open, and the same per-group vector epilogue (placed bits of the hits, next candidate
// group of the misses).
template <uint32_t g, uint32_t G>
__device__ __forceinline__ void fpp_group_sys(uint64_t q, uint64_t &placed, uint64_t &touched, uint32_t &asg,
                                              uint32_t &nxt, uint32_t &rcf, uint32_t &rmf, uint32_t &rcu,
                                              uint32_t rlab, uint32_t cpu, uint32_t mem, uint32_t req, uint32_t conf,
                                              uint32_t cand, uint32_t cand_hi, uint32_t gb64, uint32_t &nchk,
                                              uint32_t &nhit, uint32_t qc, uint32_t qm, uint32_t extra) {
    const uint32_t gbg = gb64 + g * 64u;
    // `extra`: steps the systolic phase runs past the queue length before the serial loop
    // takes the containers still open (PipeArgs::sys_extra)
    // extra bit 15: the VALU-only step loop (fp_pipe_sysv.h, FP_OPT_SYSTOLIC_VALU)
    // extra bit 14: the DPP-folded step loop (fp_pipe_sysd.h, FP_OPT_SYSTOLIC_VALU = 2)
    const uint32_t cap = (uint32_t)__builtin_popcountll(q) + (extra & 0x3FFFu);
    const SysOut so = (extra & 0x8000u)
                          ? fpp_sysv_group(q, touched, asg, rcf, rmf, rcu, rlab, cpu, mem, req, conf, gbg, qc, qm, cap)
                      : (extra & 0x4000u)
                          // one-group stages take their used nodes from the final records (k_ffd_pipe)
                          ? fpp_sysd_group<(G > 1)>(q, touched, asg, rcf, rmf, rcu, rlab, cpu, mem, req, conf, gbg, qc,
                                                    qm, cap)
                          : fpp_sys_group(q, touched, asg, rcf, rmf, rcu, rlab, cpu, mem, req, conf, gbg, qc, qm, cap);
    uint64_t left = fpp_uniform64(so.left);
    touched = fpp_uniform64(touched);
    if (left) fpp_asm_group_x<false>(left, touched, asg, rcf, rmf, rcu, rlab, cpu, mem, req, conf, gbg, nchk);
    const uint32_t lane = __lane_id();
    const bool inq = (q >> lane) & 1ull;
    const uint64_t hit = __builtin_amdgcn_ballot_w64(inq && asg != 0xFFFFFFFFu);
    if (G == 1 && (extra & 0xC000u) == 0x4000u) {
        // the DPP-folded fill of a one-group stage leaves `touched` alone and k_ffd_pipe counts the
        // nodes whose records changed; a label-only container (cpu = mem = conf = 0, req != 0)
        // changes none, so its node is marked here (n_nodes_used undercounted)
        uint64_t lo = __builtin_amdgcn_ballot_w64(inq && asg != 0xFFFFFFFFu && (cpu | mem | conf) == 0u);
        while (lo) {
            const uint32_t l = (uint32_t)__builtin_ctzll(lo);
            lo &= lo - 1;
            touched |= 1ull << ((__builtin_amdgcn_readlane(asg, l) - gbg) & 63u);
        }
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
        nxt = (inq && asg == 0xFFFFFFFFu) ? nx : nxt;
    }
}

}  // namespace fpp
