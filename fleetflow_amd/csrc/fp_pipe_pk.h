// Packed-capacity exact first fit (k_ffd_pipe's range-specialised check).
//
// When every cpu and every mem value of a batch (containers' demands and nodes' free capacity)
// is a multiple of 2^sc_c resp. 2^sc_m and below 2^(15 + sc_c) resp. 2^(15 + sc_m), the pair
// fits one 32-bit word with a clear guard bit above each 15-bit field:
//     w = (cpu >> sc_c) << 16 | (mem >> sc_m)              bits 15 and 31 clear
// and for a node record w_n and a container demand w_k
//     d = w_n - w_k        (one 32-bit subtraction)
//     fits in cpu and mem  <=>  (d & 0x80008000) == 0, and then d is the node's new record.
// (mem_n < mem_k borrows into bit 15; otherwise cpu_n < cpu_k sets bit 31, and no borrow crosses
// into the upper field.)  The shifts are exact because every value of the batch is a multiple of
// them, and capacity only ever loses demands, so records stay multiples.  With the label and
// conflict terms, the whole exact check is
//     z = (d & G) | (req & ~labels) | (conf & conflict_used)      fits <=> z == 0
// one VALU compare instead of three compares and two SALU ANDs, and one VALU placement op
// instead of two.  The u32 path (fp_pipe_asm.h, fp_pipe_sysd.h) stays for full-range inputs.
#pragma once
#include <stdint.h>

#include "fp_pipe_sys.h"  // SysOut, sys_push / sys_pull / sys_wave_or (and fp_pipe_asm.h)

namespace fpp {

constexpr uint32_t PK_GUARD = 0x80008000u;  // the two guard bits
constexpr uint32_t PK_FIELD_MAX = 0x7FFFu;   // largest packed field

__device__ __forceinline__ uint32_t pk_pack(uint32_t cpu, uint32_t mem, uint32_t sc_c, uint32_t sc_m) {
    return ((cpu >> sc_c) << 16) | (mem >> sc_m);
}
__device__ __forceinline__ uint32_t pk_cpu(uint32_t w, uint32_t sc_c) { return (w >> 16) << sc_c; }
__device__ __forceinline__ uint32_t pk_mem(uint32_t w, uint32_t sc_m) { return (w & 0xFFFFu) << sc_m; }
// w_n can take w_k in cpu and mem
__device__ __forceinline__ bool pk_fits(uint32_t wn, uint32_t wk) { return ((wn - wk) & PK_GUARD) == 0u; }

#ifdef FP_PIPE_STATS
#define FPP_PK_CNT_CHECK "s_add_u32 %[nchk], %[nchk], 1\n\t"
#else
#define FPP_PK_CNT_CHECK ""
#endif

// fpp_asm_group_x (fp_pipe_asm.h) on packed records: per container 3 readlanes (kw, req, conf),
// d = rw - kw, z = (d & G) | (kr & rlab) | (kx & rcu), ONE v_cmp, then the exec-masked placement
// rw = d, rcu |= kx (22 instructions per container against 26).  SCC for STOP's select comes from
// the s_and that sets exec (= hit).
#define FPP_GXP_BODY(SEL, TEST)                                                             \
    "s_cmp_eq_u64 %[q], 0\n\t"                                                             \
    "s_cbranch_scc1 .Lfgxp_end%=\n\t"                                                      \
    "s_mov_b64 %[esv], exec\n"                                                             \
    ".Lfgxp_loop%=:\n\t"                                                                   \
    "s_ff1_i32_b64 %[t], %[q]\n\t"                                                         \
    "v_readlane_b32 %[kw], %[cw], %[t]\n\t"                                                \
    "v_readlane_b32 %[kr], %[req], %[t]\n\t"                                               \
    "v_readlane_b32 %[kx], %[conf], %[t]\n\t"                                              \
    "s_bitset0_b64 %[q], %[t]\n\t"                                                         \
    FPP_PK_CNT_CHECK                                                                       \
    "v_subrev_u32_e32 %[d], %[kw], %[rw]\n\t"                                              \
    "v_and_b32_e32 %[t0], %[kr], %[rlab]\n\t"                                              \
    "v_and_or_b32 %[t0], %[rcu], %[kx], %[t0]\n\t"                                         \
    "v_and_or_b32 %[t0], %[d], %[gm], %[t0]\n\t"                                           \
    "v_cmp_eq_u32_e64 %[m1], 0, %[t0]\n\t"                                                 \
    "s_ff1_i32_b64 %[l], %[m1]\n\t"                                                        \
    "s_lshl_b64 %[m2], 1, %[l]\n\t"                                                        \
    "s_and_b64 exec, %[m2], %[m1]\n\t"        /* {l}, or {} on a miss; SCC = hit */        \
    SEL                                                                                    \
    "v_mov_b32_e32 %[rw], %[d]\n\t"                                                        \
    "v_or_b32_e32 %[rcu], %[kx], %[rcu]\n\t"                                               \
    "s_or_b64 %[touched], %[touched], exec\n\t"                                            \
    "s_or_b32 %[nv], %[gbg], %[l]\n\t"         /* FP_NONE on a miss */                     \
    "s_lshl_b64 exec, 1, %[t]\n\t"                                                         \
    "v_mov_b32_e32 %[asg], %[nv]\n\t"                                                      \
    "s_mov_b64 exec, %[esv]\n\t"                                                           \
    "s_cmp_lg_u64 " TEST ", 0\n\t"                                                         \
    "s_cbranch_scc1 .Lfgxp_loop%=\n"                                                       \
    ".Lfgxp_end%=:"
#define FPP_GXP_OPERANDS                                                                                       \
    : [q] "+s"(q), [touched] "+s"(touched), [asg] "+v"(asg), [rw] "+v"(rw), [rcu] "+v"(rcu), [nchk] "+s"(nchk), \
      [t] "=&s"(t), [kw] "=&s"(kw), [kr] "=&s"(kr), [kx] "=&s"(kx), [l] "=&s"(l), [nv] "=&s"(nv),              \
      [m1] "=&s"(m1), [m2] "=&s"(m2), [esv] "=&s"(esv), [qx] "=&s"(qx), [t0] "=&v"(t0), [d] "=&v"(d)         \
    : [rlab] "v"(rlab), [cw] "v"(cw), [req] "v"(req), [conf] "v"(conf), [gbg] "s"(gbg), [gm] "s"(gm)          \
    : "scc", "memory"
template <bool STOP>
__device__ __forceinline__ void fpp_asm_group_xp(uint64_t &q, uint64_t &touched, uint32_t &asg, uint32_t &rw,
                                                 uint32_t &rcu, uint32_t rlab, uint32_t cw, uint32_t req,
                                                 uint32_t conf, uint32_t gbg, uint32_t &nchk) {
    uint32_t t, kw, kr, kx, l, nv, t0, d;
    uint64_t m1, m2, esv, qx;
    const uint32_t gm = PK_GUARD;
    if constexpr (STOP)
        asm volatile(FPP_GXP_BODY("s_cselect_b64 %[qx], %[q], 0\n\t", "%[qx]") FPP_GXP_OPERANDS);
    else
        asm volatile(FPP_GXP_BODY("", "%[q]") FPP_GXP_OPERANDS);
    (void)qx;
    q = fpp_uniform64(q);
    touched = fpp_uniform64(touched);
    nchk = (uint32_t)__builtin_amdgcn_readfirstlane((int)nchk);
}
#undef FPP_GXP_BODY
#undef FPP_GXP_OPERANDS

// fpp_refilter_loop on packed records (qw = the batch corner, packed)
__device__ __forceinline__ void fpp_refilter_loop_p(uint64_t q, uint64_t &touched, uint32_t &asg, uint32_t &rw,
                                                    uint32_t &rcu, uint32_t rlab, uint32_t cw, uint32_t req,
                                                    uint32_t conf, uint32_t gbg, uint32_t &nchk, uint32_t qw) {
    fpp_asm_group_xp<true>(q, touched, asg, rw, rcu, rlab, cw, req, conf, gbg, nchk);
    while (q) {
        uint64_t e = __builtin_amdgcn_ballot_w64(pk_fits(rw, qw));
        uint64_t fit = 0;
        if (__builtin_popcountll(e) <= REFILTER_MAX) {
            bool ok = false;
            while (e) {
                const uint32_t l = (uint32_t)__builtin_ctzll(e);
                e &= e - 1;
                const uint32_t nw = __builtin_amdgcn_readlane(rw, l);
                const uint32_t nlb = __builtin_amdgcn_readlane(rlab, l), ncu = __builtin_amdgcn_readlane(rcu, l);
                ok |= ((((nw - cw) & PK_GUARD) | (req & nlb) | (conf & ncu)) == 0u);
            }
            fit = q & __builtin_amdgcn_ballot_w64(ok);
        } else {
            fit = q;
        }
        if (fit == q) {
            fpp_asm_group_xp<false>(q, touched, asg, rw, rcu, rlab, cw, req, conf, gbg, nchk);
            break;
        }
        q = fit;
        fpp_asm_group_xp<true>(q, touched, asg, rw, rcu, rlab, cw, req, conf, gbg, nchk);
    }
}

// fpp_group_x on packed records (same epilogue)
template <uint32_t g, uint32_t G, bool IB = false>
__device__ __forceinline__ void fpp_group_xp(uint64_t q, uint64_t &placed, uint64_t &touched, uint32_t &asg,
                                             uint32_t &nxt, uint32_t &rw, uint32_t &rcu, uint32_t rlab, uint32_t cw,
                                             uint32_t req, uint32_t conf, uint32_t cand, uint32_t cand_hi,
                                             uint32_t gb64, uint32_t &nchk, uint32_t &nhit, uint32_t qw) {
    const uint64_t q0 = q;
    fpp_refilter_loop_p(q, touched, asg, rw, rcu, rlab, cw, req, conf, gb64 + g * 64u, nchk, qw);
    q = q0;
    uint64_t hit;
    if constexpr (IB) {
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
    {
        const uint64_t above = (((uint64_t)cand_hi << 32) | cand) & ~((2ull << g) - 1ull);
        const uint32_t nx = above ? (uint32_t)__builtin_ctzll(above) : G;
        if constexpr (IB) nxt = fpp_lane_sel<true>(q & ~hit, nx, nxt);
        else nxt = (((q >> __lane_id()) & 1ull) && asg == 0xFFFFFFFFu) ? nx : nxt;
    }
}

// ---- the DPP-folded systolic fill on packed records (fp_pipe_sysd.h's layout) ----
// Node records xw (packed capacity), xu (conflicts used), xl (~labels) rotate one lane per step,
// folded into the DPP operand of the first instruction that reads them; container t (lane t,
// FFD order) tests position tau - t at step tau.  Per lane a state word st: ~0 before the
// container starts, 0 while it runs, the counter value c of its placement step afterwards
// (c = PK_C0 + tau - lane, never 0), so it joins the test as one more OR term:
//   st   = (lane == tau) ? 0 : st           lane tau starts (SGPR lane mask m, shifted per step)
//   z    = (rot(xl) & kr) | (rot(xu) & kx) | st | (d & G),  d = rot(xw) - kw
//   fits : z == 0;  xw = fits ? d : rot(xw);  xu = fits ? rot(xu) | kx : rot(xu);  st = fits ? c : st
// 14 VALU instructions and one SALU per step (fp_pipe_sysd.h: 18 VALU).  A container that has
// passed every live position keeps rotating through the fillers (which reject every container
// that is not all-zero; all-zero ones never enter) and then the live positions again, where it
// cannot fit either: capacity only shrinks.
constexpr uint32_t PK_C0 = 0x40000000u;
#define FPP_SP_DPP " wave_ror:1 row_mask:0xf bank_mask:0xf\n\t"
#define FPP_SP_STEP                                                   \
    "v_cndmask_b32_e64 %[st], %[st], 0, %[m]\n\t"                    \
    "s_lshl_b64 %[m], %[m], 1\n\t"                                   \
    "v_and_b32_dpp %[ta], %[xl], %[kr]" FPP_SP_DPP                   \
    "v_and_b32_dpp %[tb], %[xu], %[kx]" FPP_SP_DPP                   \
    "v_sub_u32_dpp %[d], %[xw], %[kw]" FPP_SP_DPP                    \
    "v_or3_b32 %[t], %[ta], %[tb], %[st]\n\t"                        \
    "v_or_b32_dpp %[tu], %[xu], %[kx]" FPP_SP_DPP                    \
    "v_and_or_b32 %[t], %[d], %[gm], %[t]\n\t"                       \
    "v_mov_b32_dpp %[xl], %[xl]" FPP_SP_DPP                          \
    "v_cmp_eq_u32_e32 vcc, 0, %[t]\n\t"                              \
    "v_cndmask_b32_dpp %[xw], %[xw], %[d], vcc" FPP_SP_DPP           \
    "v_cndmask_b32_dpp %[xu], %[xu], %[tu], vcc" FPP_SP_DPP          \
    "v_cndmask_b32_e32 %[st], %[st], %[c], vcc\n\t"                  \
    "v_add_u32_e32 %[c], 1, %[c]\n\t"

// steps per exit check (one ballot + branches): 16.  Config 3's kernel 50.4-50.8 (8) -> 47.2-47.8 ms
// (16), 47.4-47.7 (24), 49.7-49.8 (32), 58.0 (4); config 2 0.70 -> 0.66 ms (profiles/r07f_*, r07g_*):
// a check costs more than the steps a longer block wastes at the end of a queue
#ifndef FPP_SP_UNROLL
#define FPP_SP_UNROLL 16
#endif

// Runs steps (in blocks of FPP_SP_UNROLL) until every container has started and none is still
// running, or `cap` steps; returns the steps taken (= rotations applied).
__device__ __forceinline__ uint32_t fpp_sysp_steps(uint32_t &xw, uint32_t &xu, uint32_t &xl, uint32_t kw,
                                                   uint32_t kr, uint32_t kx, uint32_t &st, uint32_t &c, uint32_t L,
                                                   uint32_t Q, uint32_t cap) {
    uint32_t tau = 0;
    uint64_t m = 1;  // lane tau's bit
    const uint32_t gm = PK_GUARD;
    while (true) {
        uint32_t ta, tb, t, d, tu;
        asm volatile(
            FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP
#if FPP_SP_UNROLL >= 8
            FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP
#endif
#if FPP_SP_UNROLL >= 16
            FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP
#endif
#if FPP_SP_UNROLL >= 24
            FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP
#endif
#if FPP_SP_UNROLL >= 32
            FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP FPP_SP_STEP
#endif
            "s_nop 1"
            : [xw] "+v"(xw), [xu] "+v"(xu), [xl] "+v"(xl), [st] "+v"(st), [c] "+v"(c), [m] "+s"(m),
              [ta] "=&v"(ta), [tb] "=&v"(tb), [t] "=&v"(t), [d] "=&v"(d), [tu] "=&v"(tu)
            : [kw] "v"(kw), [kr] "v"(kr), [kx] "v"(kx), [gm] "s"(gm)
            : "vcc", "scc");
        m = fpp_uniform64(m);
        tau += FPP_SP_UNROLL;
        if (tau >= cap) break;
        // running: started, not placed, and the next position still live
        if (tau >= Q && !__builtin_amdgcn_ballot_w64(st == 0u && c - PK_C0 < L && __lane_id() < Q)) break;
    }
    return tau;
}

// fpp_sysd_group on packed records (same contract; qw = the batch corner, packed).  TOUCHED as
// there: one-group stages leave `touched` to the caller.
template <bool TOUCHED = true>
__device__ __forceinline__ SysOut fpp_sysp_group(uint64_t q, uint64_t &touched, uint32_t &asg, uint32_t &rw,
                                                 uint32_t &rcu, uint32_t rlab, uint32_t cw, uint32_t req,
                                                 uint32_t conf, uint32_t gbg, uint32_t qw, uint32_t max_steps) {
    const uint32_t lane = __lane_id();
    SysOut out{0};
    const uint64_t lm = __builtin_amdgcn_ballot_w64(pk_fits(rw, qw));
    const uint32_t L = (uint32_t)__builtin_popcountll(lm);
    if (L == 0) {
        if ((q >> lane) & 1ull) asg = 0xFFFFFFFFu;
        return out;
    }
    const bool inq = (q >> lane) & 1ull;
    const uint32_t Q = (uint32_t)__builtin_popcountll(q);
    const bool qpre = (q & (q + 1ull)) == 0ull, lfull = lm == ~0ull;
    const uint32_t qa = __builtin_amdgcn_mbcnt_hi((uint32_t)(q >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)q, 0u));
    const uint32_t rq = qpre ? lane : inq ? qa : Q + lane - qa;
    uint32_t kw = cw, kr = req, kx = conf;
    if (!qpre) { kw = sys_push(rq, cw); kr = sys_push(rq, req); kx = sys_push(rq, conf); }
    // lanes without a queued container: a demand no record can take (a 0x8000 field always borrows)
    kw = lane < Q ? kw : PK_GUARD;
    const bool live = (lm >> lane) & 1ull;
    const uint32_t la = __builtin_amdgcn_mbcnt_hi((uint32_t)(lm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)lm, 0u));
    const uint32_t pos = live ? la : L + lane - la;
    // position p starts at lane (63 - p) & 63: one rotation behind the first step
    const uint32_t at0 = (63u - pos) & 63u;
    uint32_t xw = sys_push(at0, rw), xu = sys_push(at0, rcu), xl = sys_push(at0, rlab);
    const uint32_t pmap = lfull ? lane : sys_push(pos, lane);
    const bool filler = ((63u - lane) & 63u) >= L;  // filler positions fit nothing
    xw = filler ? 0u : xw;
    xu = filler ? 0xFFFFFFFFu : xu;
    xl = filler ? 0xFFFFFFFFu : xl;
    uint32_t st = 0xFFFFFFFFu;  // not started (lanes >= Q start too, with a demand that never fits)
    uint32_t c = PK_C0 - lane;
    const uint32_t cap = max_steps < Q + L ? max_steps : Q + L;
    const uint32_t tau = fpp_sysp_steps(xw, xu, xl, kw, kr, kx, st, c, L, Q, cap);
    // after tau steps position p is at lane (tau - 1 - p) & 63
    const uint32_t src = (tau - 1u - pos) & 63u;
    const uint32_t nw = sys_pull(src, xw), ncu = sys_pull(src, xu);
    rw = live ? nw : rw;
    rcu = live ? ncu : rcu;
    const bool pl = st != 0u && st != 0xFFFFFFFFu;  // placed: st = c of that step
    const uint32_t apos = pl ? st - PK_C0 : 0xFFFFFFFFu;               // the position it took
    const uint32_t nl = lfull ? (apos & 63u) : sys_pull(apos & 63u, pmap);
    const uint32_t cnode = pl ? gbg + nl : 0xFFFFFFFFu;
    const uint32_t back = qpre ? cnode : sys_pull(rq, cnode);
    // still open: running with live positions ahead, or never started (cap reached first)
    const uint32_t open = ((st == 0u && c - PK_C0 < L) || st == 0xFFFFFFFFu) ? 1u : 0u;
    const uint32_t open_here = qpre ? open : sys_pull(rq, open);
    asg = inq ? back : asg;
    out.left = __builtin_amdgcn_ballot_w64(inq && open_here != 0);
    if (TOUCHED) {
        const uint32_t bl = pl && nl < 32 ? 1u << nl : 0u;
        const uint32_t bh = pl && nl >= 32 ? 1u << (nl - 32) : 0u;
        touched |= ((uint64_t)sys_wave_or(bh) << 32) | sys_wave_or(bl);
    }
    return out;
}

// fpp_group_sys (fp_pipe_sys.h) on packed records: the packed systolic fill, the packed serial
// finish of what it left open, the same epilogue.  One-group stages (TOUCHED = false) mark the nodes
// of label-only placements here (k_ffd_pipe counts the others from changed records).
template <uint32_t g, uint32_t G>
__device__ __forceinline__ void fpp_group_sysp(uint64_t q, uint64_t &placed, uint64_t &touched, uint32_t &asg,
                                               uint32_t &nxt, uint32_t &rw, uint32_t &rcu, uint32_t rlab, uint32_t cw,
                                               uint32_t req, uint32_t conf, uint32_t cand, uint32_t cand_hi,
                                               uint32_t gb64, uint32_t &nchk, uint32_t &nhit, uint32_t qw,
                                               uint32_t extra) {
    const uint32_t gbg = gb64 + g * 64u;
    const uint32_t cap = (uint32_t)__builtin_popcountll(q) + (extra & 0x3FFFu);
    const SysOut so = fpp_sysp_group<(G > 1)>(q, touched, asg, rw, rcu, rlab, cw, req, conf, gbg, qw, cap);
    uint64_t left = fpp_uniform64(so.left);
    touched = fpp_uniform64(touched);
    if (left) fpp_asm_group_xp<false>(left, touched, asg, rw, rcu, rlab, cw, req, conf, gbg, nchk);
    const uint32_t lane = __lane_id();
    const bool inq = (q >> lane) & 1ull;
    const uint64_t hit = __builtin_amdgcn_ballot_w64(inq && asg != 0xFFFFFFFFu);
    if (G == 1) {
        uint64_t lo = __builtin_amdgcn_ballot_w64(inq && asg != 0xFFFFFFFFu && (cw | conf) == 0u);
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
    {
        const uint64_t above = (((uint64_t)cand_hi << 32) | cand) & ~((2ull << g) - 1ull);
        const uint32_t nx = above ? (uint32_t)__builtin_ctzll(above) : G;
        nxt = (inq && asg == 0xFFFFFFFFu) ? nx : nxt;
    }
}

#undef FPP_SP_STEP
#undef FPP_SP_DPP

}  // namespace fpp
