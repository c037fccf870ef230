// Hand-scheduled candidate loop of k_ffd_pipe (one batch, one stage): exact first fit,
// container by container in FFD order.  Same algorithm and state as the C++ loop in
// fp_pipe.hip, written as one inline-asm block so that
//   * a group's four records are read through ONE s_set_gpr_idx window and written back
//     through one (the records sit in fixed VGPR tuples, v[88:127], pinned by operand
//     constraints -- the only way to name an indexed base register in inline asm);
//   * label and conflict become one test: ((~lab & req) | (cu & conf)) == 0;
//   * the check loop has one scalar exit test per candidate and a single SCC branch on
//     the match;
//   * the bucket-mask update is one ds_mskor_b64 with no per-lane select of the old value.
// gfx950 (GFX9 encoding): one SGPR per VALU op, lane selects come from SALU results or
// M0, and M0 is reloaded after every s_set_gpr_idx window (the window overwrites it);
// M0 is restored on exit (the compiler treats it as reserved).  Written for 2..10-group
// stages (the wide geometry): records v[88:127], scratch v[76:87], so the wave stays
// within 128 VGPRs (four workgroups of four waves per CU).
#pragma once
#include <stdint.h>

// re-test of a group's queue after its first miss (fpp_group_x), with a batch corner of at
// most FP_REFILTER_MAX nodes; -DFP_REFILTER=0 for A/B runs
#ifndef FP_REFILTER
#define FP_REFILTER 1
#endif
#ifndef FP_REFILTER_MAX
#define FP_REFILTER_MAX 16
#endif

namespace fpp {

__device__ __forceinline__ uint64_t fpp_uniform64(uint64_t x) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(x >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
}

typedef uint32_t rec10 __attribute__((ext_vector_type(10)));

#ifdef FP_PIPE_STATS
#define FPP_ASM_CNT_CHECK "s_add_u32 %[nchk], %[nchk], 1\n\t"
#define FPP_ASM_CNT_HIT "s_add_u32 %[nhit], %[nhit], 1\n\t"
#else
#define FPP_ASM_CNT_CHECK ""
#define FPP_ASM_CNT_HIT ""
#endif

// todo: containers (lanes) with candidate groups, cleared as they are processed
// placed / asg / used: placed-lane mask, per-lane assignment, per-lane used-group bits
// rcf rmf rcu rlab: the stage's records (cpu_free, mem_free, conflict_used, ~labels)
// lsel: ~0 on lanes 0-31 (cpu thresholds), 0 on lanes 32-63 (mem thresholds)
// maddr: LDS byte address of this lane's mask word in group 0 (group stride 512 B)
__device__ __forceinline__ void fpp_asm_batch(uint64_t &todo, uint64_t &placed, uint32_t &asg, uint32_t &used,
                                              rec10 &rcf, rec10 &rmf, rec10 &rcu, rec10 &rlab, uint32_t cpu,
                                              uint32_t mem, uint32_t req, uint32_t conf, uint32_t cand,
                                              uint32_t my_t, uint32_t lsel, uint32_t maddr, uint32_t gb64,
                                              uint32_t &nchk, uint32_t &nhit) {
    uint32_t ti, cc, ccpu, cmem, creq, cconf, g, l, oc, om, m0sv;
    uint64_t tbit, m, m2;
    asm volatile(
        "s_mov_b32 %[m0sv], m0\n\t"
        "v_mov_b32 v82, 1\n\t"
        "v_mov_b32 v83, 0\n\t"
        "v_mov_b32 v84, 0\n\t"
        "v_mov_b32 v85, 0\n\t"
        "s_cmp_eq_u64 %[todo], 0\n\t"
        "s_cbranch_scc1 .Lfpp_end%=\n"
        ".Lfpp_cont%=:\n\t"
        "s_ff1_i32_b64 %[ti], %[todo]\n\t"
        "s_lshl_b64 %[tbit], 1, %[ti]\n\t"
        "s_andn2_b64 %[todo], %[todo], %[tbit]\n\t"
        "v_readlane_b32 %[cc], %[cand], %[ti]\n\t"
        "v_readlane_b32 %[ccpu], %[cpu], %[ti]\n\t"
        "v_readlane_b32 %[cmem], %[mem], %[ti]\n\t"
        "v_readlane_b32 %[creq], %[req], %[ti]\n\t"
        "v_readlane_b32 %[cconf], %[conf], %[ti]\n"
        ".Lfpp_check%=:\n\t"
        "s_ff1_i32_b32 %[g], %[cc]\n\t"
        "s_set_gpr_idx_on %[g], gpr_idx(SRC0)\n\t"
        "v_mov_b32 v76, v88\n\t"
        "v_mov_b32 v77, v98\n\t"
        "v_mov_b32 v78, v108\n\t"
        "v_mov_b32 v79, v118\n\t"
        "s_set_gpr_idx_off\n\t"
        FPP_ASM_CNT_CHECK
        "s_bitset0_b32 %[cc], %[g]\n\t"
        "v_cmp_ge_u32_e64 %[m], v76, %[ccpu]\n\t"
        "v_cmp_ge_u32_e64 %[m2], v77, %[cmem]\n\t"
        "v_and_b32_e32 v79, %[creq], v79\n\t"
        "v_and_or_b32 v79, v78, %[cconf], v79\n\t"
        "s_and_b64 %[m], %[m], %[m2]\n\t"
        "v_cmp_eq_u32_e64 %[m2], 0, v79\n\t"
        "s_and_b64 %[m], %[m], %[m2]\n\t"
        "s_cbranch_scc1 .Lfpp_hit%=\n\t"
        "s_cmp_lg_u32 %[cc], 0\n\t"
        "s_cbranch_scc1 .Lfpp_check%=\n\t"
        "s_branch .Lfpp_next%=\n"
        ".Lfpp_hit%=:\n\t"
        FPP_ASM_CNT_HIT
        "s_ff1_i32_b64 %[l], %[m]\n\t"
        "v_readlane_b32 %[oc], v76, %[l]\n\t"
        "v_readlane_b32 %[om], v77, %[l]\n\t"
        "v_readlane_b32 %[creq], v78, %[l]\n\t"
        "v_readlane_b32 %[cc], %[used], %[l]\n\t"
        "s_mov_b32 m0, %[l]\n\t"
        "s_sub_u32 %[ccpu], %[oc], %[ccpu]\n\t"    // new cpu_free
        "s_sub_u32 %[cmem], %[om], %[cmem]\n\t"    // new mem_free
        "s_or_b32 %[creq], %[creq], %[cconf]\n\t"  // new conflict_used
        "s_bitset1_b32 %[cc], %[g]\n\t"            // node used
        "v_writelane_b32 v76, %[ccpu], m0\n\t"
        "v_writelane_b32 v77, %[cmem], m0\n\t"
        "v_writelane_b32 v78, %[creq], m0\n\t"
        "v_writelane_b32 %[used], %[cc], m0\n\t"
        "s_set_gpr_idx_on %[g], gpr_idx(DST)\n\t"
        "v_mov_b32 v88, v76\n\t"
        "v_mov_b32 v98, v77\n\t"
        "v_mov_b32 v108, v78\n\t"
        "s_set_gpr_idx_off\n\t"
        // bucket masks (lanes 0-31 cpu, 32-63 mem): clear bit l where T <= old && T > new
        "v_mov_b32 v86, %[om]\n\t"
        "v_bfi_b32 v86, %[lsel], %[oc], v86\n\t"
        "v_mov_b32 v87, %[cmem]\n\t"
        "v_bfi_b32 v87, %[lsel], %[ccpu], v87\n\t"
        "v_cmp_le_u32_e64 %[m], %[myt], v86\n\t"
        "v_cmp_gt_u32_e64 %[m2], %[myt], v87\n\t"
        "s_and_b64 %[m], %[m], %[m2]\n\t"
        "v_lshlrev_b64 v[80:81], %[l], v[82:83]\n\t"
        "v_cndmask_b32_e64 v80, 0, v80, %[m]\n\t"
        "v_cndmask_b32_e64 v81, 0, v81, %[m]\n\t"
        "v_lshl_add_u32 v86, %[g], 9, %[maddr]\n\t"
        "ds_mskor_b64 v86, v[80:81], v[84:85]\n\t"
        // assignment of lane ti: gb64 + g * 64 + l
        "s_lshl_b32 %[oc], %[g], 6\n\t"
        "s_add_u32 %[oc], %[oc], %[gb64]\n\t"
        "s_or_b32 %[oc], %[oc], %[l]\n\t"
        "s_mov_b32 m0, %[ti]\n\t"
        "v_writelane_b32 %[asg], %[oc], m0\n\t"
        "s_or_b64 %[placed], %[placed], %[tbit]\n"
        ".Lfpp_next%=:\n\t"
        "s_cmp_lg_u64 %[todo], 0\n\t"
        "s_cbranch_scc1 .Lfpp_cont%=\n"
        ".Lfpp_end%=:\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_mov_b32 m0, %[m0sv]"
        : [todo] "+s"(todo), [placed] "+s"(placed), [asg] "+v"(asg), [used] "+v"(used),
          [nchk] "+s"(nchk), [nhit] "+s"(nhit), [rcf] "+{v[88:97]}"(rcf), [rmf] "+{v[98:107]}"(rmf),
          [rcu] "+{v[108:117]}"(rcu), [rlab] "+{v[118:127]}"(rlab), [ti] "=&s"(ti), [cc] "=&s"(cc),
          [ccpu] "=&s"(ccpu), [cmem] "=&s"(cmem), [creq] "=&s"(creq), [cconf] "=&s"(cconf), [g] "=&s"(g),
          [l] "=&s"(l), [oc] "=&s"(oc), [om] "=&s"(om), [tbit] "=&s"(tbit), [m] "=&s"(m), [m2] "=&s"(m2),
          [m0sv] "=&s"(m0sv)
        : [cand] "v"(cand), [cpu] "v"(cpu), [mem] "v"(mem), [req] "v"(req), [conf] "v"(conf), [myt] "v"(my_t),
          [lsel] "v"(lsel), [maddr] "v"(maddr), [gb64] "s"(gb64)
        : "scc", "memory", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85",
          "v86", "v87");
}

// Group-major candidate loop for ONE group g (the default build): exact first fit of the
// containers queued on group g, in lane (= FFD) order.  Same checks as fpp_asm_batch, but
// the group's four records are plain "+v" operands -- the group index is a compile-time
// constant of the caller, so there is no s_set_gpr_idx window and no indexed copy: a check
// is 4 readlanes, 3 compares, 2 SALU ANDs and a branch.  A miss moves the container to its
// next candidate group (nxt lane ti = first cand bit above g, or G for none); a hit updates
// lane l of the records with v_writelane, records the assignment and sets bit l of
// `touched`.  The bucket masks and the used-node bits are brought up to date once per
// group and batch by the caller, from `touched` (off the per-placement chain).
// Every per-group constant is an immediate (the group index is a template parameter), so a
// wide stage keeps no per-group scalars live:
//   q       lanes queued on g (consumed)        gb64   gbase * 64 (SGPR); + g * 64 immediate
//   G       groups per stage: "no further candidate"
template <uint32_t g, uint32_t G>
__device__ __forceinline__ void fpp_asm_group(uint64_t q, uint64_t &placed, uint64_t &touched, uint32_t &asg,
                                              uint32_t &nxt, uint32_t &rcf, uint32_t &rmf, uint32_t &rcu,
                                              uint32_t rlab, uint32_t cpu, uint32_t mem, uint32_t req, uint32_t conf,
                                              uint32_t cand, uint32_t cand_hi, uint32_t gb64, uint32_t &nchk,
                                              uint32_t &nhit, uint32_t, uint32_t) {
    constexpr uint32_t nmask = g < 32 ? ~((2u << g) - 1u) : 0u;        // candidate groups above g
    constexpr uint32_t nmask_hi = g < 32 ? 0xFFFFFFFFu : ~((2u << (g & 31)) - 1u);
    constexpr uint32_t goff = g * 64u;
    uint32_t ti, ccpu, cmem, creq, cconf, l, oc, om, ocu, ous, m0sv, t0;
    uint64_t tbit, m, m2;
    asm volatile(
        "s_mov_b32 %[m0sv], m0\n\t"
        "s_cmp_eq_u64 %[q], 0\n\t"
        "s_cbranch_scc1 .Lfpg_end%=\n"
        ".Lfpg_cont%=:\n\t"
        "s_ff1_i32_b64 %[ti], %[q]\n\t"
        "s_lshl_b64 %[tbit], 1, %[ti]\n\t"
        "s_andn2_b64 %[q], %[q], %[tbit]\n\t"
        "v_readlane_b32 %[ccpu], %[cpu], %[ti]\n\t"
        "v_readlane_b32 %[cmem], %[mem], %[ti]\n\t"
        "v_readlane_b32 %[creq], %[req], %[ti]\n\t"
        "v_readlane_b32 %[cconf], %[conf], %[ti]\n\t"
        FPP_ASM_CNT_CHECK
        "v_cmp_ge_u32_e64 %[m], %[rcf], %[ccpu]\n\t"
        "v_cmp_ge_u32_e64 %[m2], %[rmf], %[cmem]\n\t"
        "v_and_b32_e32 %[t0], %[creq], %[rlab]\n\t"
        "v_and_or_b32 %[t0], %[rcu], %[cconf], %[t0]\n\t"
        "s_and_b64 %[m], %[m], %[m2]\n\t"
        "v_cmp_eq_u32_e64 %[m2], 0, %[t0]\n\t"
        "s_and_b64 %[m], %[m], %[m2]\n\t"
        "s_cbranch_scc1 .Lfpg_hit%=\n\t"
        // miss: the container's next candidate group (none: G); candidate groups are a
        // 64-bit set in (cand, cand_hi)
        "v_readlane_b32 %[oc], %[cand], %[ti]\n\t"
        "v_readlane_b32 %[ocu], %[candhi], %[ti]\n\t"
        "s_and_b32 %[oc], %[oc], %[nmask]\n\t"
        "s_and_b32 %[ocu], %[ocu], %[nmaskhi]\n\t"
        "s_ff1_i32_b32 %[ous], %[ocu]\n\t"
        "s_add_u32 %[ous], %[ous], 32\n\t"
        "s_cmp_eq_u32 %[ocu], 0\n\t"
        "s_cselect_b32 %[ous], %[gnone], %[ous]\n\t"
        "s_ff1_i32_b32 %[om], %[oc]\n\t"
        "s_cmp_eq_u32 %[oc], 0\n\t"
        "s_cselect_b32 %[om], %[ous], %[om]\n\t"
        "s_mov_b32 m0, %[ti]\n\t"
        "v_writelane_b32 %[nxt], %[om], m0\n\t"
        "s_cmp_lg_u64 %[q], 0\n\t"
        "s_cbranch_scc1 .Lfpg_cont%=\n\t"
        "s_branch .Lfpg_end%=\n"
        ".Lfpg_hit%=:\n\t"
        FPP_ASM_CNT_HIT
        "s_ff1_i32_b64 %[l], %[m]\n\t"
        "v_readlane_b32 %[oc], %[rcf], %[l]\n\t"
        "v_readlane_b32 %[om], %[rmf], %[l]\n\t"
        "v_readlane_b32 %[ocu], %[rcu], %[l]\n\t"
        "s_mov_b32 m0, %[l]\n\t"
        "s_sub_u32 %[ccpu], %[oc], %[ccpu]\n\t"    // new cpu_free
        "s_sub_u32 %[cmem], %[om], %[cmem]\n\t"    // new mem_free
        "s_or_b32 %[ocu], %[ocu], %[cconf]\n\t"    // new conflict_used
        "v_writelane_b32 %[rcf], %[ccpu], m0\n\t"
        "v_writelane_b32 %[rmf], %[cmem], m0\n\t"
        "v_writelane_b32 %[rcu], %[ocu], m0\n\t"
        "s_lshl_b64 %[m2], 1, %[l]\n\t"
        "s_or_b64 %[touched], %[touched], %[m2]\n\t"
        // assignment of lane ti: (gbase + g) * 64 + l
        "s_add_u32 %[oc], %[gb64], %[goff]\n\t"
        "s_or_b32 %[oc], %[oc], %[l]\n\t"
        "s_mov_b32 m0, %[ti]\n\t"
        "v_writelane_b32 %[asg], %[oc], m0\n\t"
        "s_or_b64 %[placed], %[placed], %[tbit]\n\t"
        "s_cmp_lg_u64 %[q], 0\n\t"
        "s_cbranch_scc1 .Lfpg_cont%=\n"
        ".Lfpg_end%=:\n\t"
        "s_mov_b32 m0, %[m0sv]"
        : [q] "+s"(q), [placed] "+s"(placed), [touched] "+s"(touched), [asg] "+v"(asg), [nxt] "+v"(nxt),
          [rcf] "+v"(rcf), [rmf] "+v"(rmf), [rcu] "+v"(rcu), [nchk] "+s"(nchk), [nhit] "+s"(nhit),
          [ti] "=&s"(ti), [ccpu] "=&s"(ccpu), [cmem] "=&s"(cmem), [creq] "=&s"(creq), [cconf] "=&s"(cconf),
          [l] "=&s"(l), [oc] "=&s"(oc), [om] "=&s"(om), [ocu] "=&s"(ocu), [ous] "=&s"(ous), [m0sv] "=&s"(m0sv),
          [tbit] "=&s"(tbit), [m] "=&s"(m), [m2] "=&s"(m2), [t0] "=&v"(t0)
        : [rlab] "v"(rlab), [cpu] "v"(cpu), [mem] "v"(mem), [req] "v"(req), [conf] "v"(conf), [cand] "v"(cand),
          [candhi] "v"(cand_hi), [gb64] "s"(gb64), [nmask] "i"(nmask), [nmaskhi] "i"(nmask_hi), [gnone] "i"(G),
          [goff] "i"(goff)
        : "scc", "memory");
}

// Exec-masked serial loop for ONE group g (the default build): exact first fit of the
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

// The serial loop over queue q with the re-test after each first miss (FP_REFILTER): see
// fpp_group_x.  gbg = the group's first node index.
__device__ __forceinline__ void fpp_refilter_loop(uint64_t q, uint64_t &touched, uint32_t &asg, uint32_t &rcf,
                                                  uint32_t &rmf, uint32_t &rcu, uint32_t rlab, uint32_t cpu,
                                                  uint32_t mem, uint32_t req, uint32_t conf, uint32_t gbg,
                                                  uint32_t &nchk, uint32_t qc, uint32_t qm) {
#if FP_REFILTER
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
        uint64_t e = __builtin_amdgcn_ballot_w64((rcf >= qc) & (rmf >= qm));
        uint64_t fit = 0;
        if (__builtin_popcountll(e) <= FP_REFILTER_MAX) {
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
#else
    (void)qc; (void)qm;
    fpp_asm_group_x<false>(q, touched, asg, rcf, rmf, rcu, rlab, cpu, mem, req, conf, gbg, nchk);
#endif
}

// Drop-in for fpp_asm_group (same arguments): the exec-masked loop plus the per-group
// vector epilogue -- placed bits of the hits, next candidate group of the misses.
template <uint32_t g, uint32_t G>
__device__ __forceinline__ void fpp_group_x(uint64_t q, uint64_t &placed, uint64_t &touched, uint32_t &asg,
                                            uint32_t &nxt, uint32_t &rcf, uint32_t &rmf, uint32_t &rcu,
                                            uint32_t rlab, uint32_t cpu, uint32_t mem, uint32_t req, uint32_t conf,
                                            uint32_t cand, uint32_t cand_hi, uint32_t gb64, uint32_t &nchk,
                                            uint32_t &nhit, uint32_t qc, uint32_t qm) {
    const uint64_t q0 = q;
    fpp_refilter_loop(q, touched, asg, rcf, rmf, rcu, rlab, cpu, mem, req, conf, gb64 + g * 64u, nchk, qc, qm);
    q = q0;
    const uint32_t lane = __lane_id();
    const bool inq = (q >> lane) & 1ull;
    const uint64_t hit = __builtin_amdgcn_ballot_w64(inq && asg != 0xFFFFFFFFu);
#ifdef FP_PIPE_STATS
    nhit += (uint32_t)__builtin_popcountll(hit);
#else
    (void)nhit;
#endif
    placed |= hit;
    if (inq && asg == 0xFFFFFFFFu) {
        const uint64_t above = (((uint64_t)cand_hi << 32) | cand) & ~((2ull << g) - 1ull);
        nxt = above ? (uint32_t)__builtin_ctzll(above) : G;
    }
}

}  // namespace fpp
