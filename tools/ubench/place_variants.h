// Scheduling variants of the exec-masked group loop (fpp_asm_group_x) for tools/ubench/place.hip.
// V = 1: baseline (fpp_asm_group_x order); 2: assignment by v_writelane (m0) instead of an
// exec-masked v_mov; 3: software pipelined (the next container's fetch between the compares and
// the mask ANDs), pairs per iteration, exec-masked assignment; 4: as 3 with v_writelane.
#pragma once
#include <stdint.h>

namespace fppv {

#define PV_FETCH(T, KC, KM, KR, KX)                                  \
    "s_ff1_i32_b64 %[" T "], %[q]\n\t"                               \
    "s_bitset0_b64 %[q], %[" T "]\n\t"                               \
    "v_readlane_b32 %[" KC "], %[cpu], %[" T "]\n\t"                 \
    "v_readlane_b32 %[" KM "], %[mem], %[" T "]\n\t"                 \
    "v_readlane_b32 %[" KR "], %[req], %[" T "]\n\t"                 \
    "v_readlane_b32 %[" KX "], %[conf], %[" T "]\n\t"
#define PV_CMP(KC, KM, KR, KX)                                       \
    "v_cmp_ge_u32_e64 %[m1], %[rcf], %[" KC "]\n\t"                  \
    "v_cmp_ge_u32_e64 %[m2], %[rmf], %[" KM "]\n\t"                  \
    "v_and_b32_e32 %[t0], %[" KR "], %[rlab]\n\t"                    \
    "v_and_or_b32 %[t0], %[rcu], %[" KX "], %[t0]\n\t"               \
    "v_cmp_eq_u32_e64 %[m3], 0, %[t0]\n\t"
#define PV_SEL                                                       \
    "s_and_b64 %[m1], %[m1], %[m2]\n\t"                              \
    "s_and_b64 %[m1], %[m1], %[m3]\n\t"                              \
    "s_ff1_i32_b64 %[l], %[m1]\n\t"                                  \
    "s_lshl_b64 %[m2], 1, %[l]\n\t"                                  \
    "s_and_b64 exec, %[m2], %[m1]\n\t"
#define PV_UPD(KC, KM, KX)                                           \
    "v_subrev_u32_e32 %[rcf], %[" KC "], %[rcf]\n\t"                 \
    "v_subrev_u32_e32 %[rmf], %[" KM "], %[rmf]\n\t"                 \
    "v_or_b32_e32 %[rcu], %[" KX "], %[rcu]\n\t"                     \
    "s_or_b64 %[touched], %[touched], exec\n\t"
#define PV_ASGX(T)                                                   \
    "s_or_b32 %[nv], %[gbg], %[l]\n\t"                               \
    "s_lshl_b64 exec, 1, %[" T "]\n\t"                               \
    "v_mov_b32_e32 %[asg], %[nv]\n\t"                                \
    "s_mov_b64 exec, %[esv]\n\t"
#define PV_ASGW(T)                                                   \
    "s_mov_b64 exec, %[esv]\n\t"                                     \
    "s_or_b32 %[nv], %[gbg], %[l]\n\t"                               \
    "s_mov_b32 m0, %[" T "]\n\t"                                     \
    "v_writelane_b32 %[asg], %[nv], m0\n\t"

#define PV_OPS                                                                                                   \
    : [q] "+s"(q), [touched] "+s"(touched), [asg] "+v"(asg), [rcf] "+v"(rcf), [rmf] "+v"(rmf), [rcu] "+v"(rcu), \
      [ta] "=&s"(ta), [tb] "=&s"(tb), [ac] "=&s"(ac), [am] "=&s"(am), [ar] "=&s"(ar), [ax] "=&s"(ax),          \
      [bc] "=&s"(bc), [bm] "=&s"(bm), [br] "=&s"(br), [bx] "=&s"(bx), [l] "=&s"(l), [nv] "=&s"(nv),             \
      [cnt] "=&s"(cnt), [m0sv] "=&s"(m0sv), [m1] "=&s"(m1), [m2] "=&s"(m2), [m3] "=&s"(m3), [esv] "=&s"(esv),   \
      [t0] "=&v"(t0)                                                                                             \
    : [rlab] "v"(rlab), [cpu] "v"(cpu), [mem] "v"(mem), [req] "v"(req), [conf] "v"(conf), [gbg] "s"(gbg)       \
    : "scc", "memory"

template <int V>
__device__ __forceinline__ void group_v(uint64_t q, uint64_t &touched, uint32_t &asg, uint32_t &rcf, uint32_t &rmf,
                                        uint32_t &rcu, uint32_t rlab, uint32_t cpu, uint32_t mem, uint32_t req,
                                        uint32_t conf, uint32_t gbg) {
    uint32_t ta, tb, ac, am, ar, ax, bc, bm, br, bx, l, nv, cnt, m0sv;
    uint64_t m1, m2, m3, esv;
    uint32_t t0;
    if constexpr (V == 1) {
        asm volatile(
            "s_cmp_eq_u64 %[q], 0\n\t"
            "s_cbranch_scc1 .Lpv_end%=\n\t"
            "s_mov_b32 %[m0sv], m0\n\t"
            "s_mov_b64 %[esv], exec\n"
            ".Lpv_loop%=:\n\t"
            PV_FETCH("ta", "ac", "am", "ar", "ax")
            PV_CMP("ac", "am", "ar", "ax")
            PV_SEL
            PV_UPD("ac", "am", "ax")
            PV_ASGX("ta")
            "s_cmp_lg_u64 %[q], 0\n\t"
            "s_cbranch_scc1 .Lpv_loop%=\n\t"
            "s_mov_b32 m0, %[m0sv]\n"
            ".Lpv_end%=:"
            PV_OPS);
    } else if constexpr (V == 2) {
        asm volatile(
            "s_cmp_eq_u64 %[q], 0\n\t"
            "s_cbranch_scc1 .Lpv_end%=\n\t"
            "s_mov_b32 %[m0sv], m0\n\t"
            "s_mov_b64 %[esv], exec\n"
            ".Lpv_loop%=:\n\t"
            PV_FETCH("ta", "ac", "am", "ar", "ax")
            PV_CMP("ac", "am", "ar", "ax")
            PV_SEL
            PV_UPD("ac", "am", "ax")
            PV_ASGW("ta")
            "s_cmp_lg_u64 %[q], 0\n\t"
            "s_cbranch_scc1 .Lpv_loop%=\n\t"
            "s_mov_b32 m0, %[m0sv]\n"
            ".Lpv_end%=:"
            PV_OPS);
    } else if constexpr (V == 3 || V == 4) {
#define PV_ASG(T) (V == 3 ? PV_ASGX(T) : PV_ASGW(T))
        // count-based: pairs, then an odd tail; the fetch of a container past the end reads lane 63
        // (harmless: it is never checked)
        if constexpr (V == 3) {
            asm volatile(
                "s_cmp_eq_u64 %[q], 0\n\t"
                "s_cbranch_scc1 .Lpv_end%=\n\t"
                "s_mov_b32 %[m0sv], m0\n\t"
                "s_mov_b64 %[esv], exec\n\t"
                "s_bcnt1_i32_b64 %[cnt], %[q]\n\t"
                PV_FETCH("ta", "ac", "am", "ar", "ax")
                "s_lshr_b32 %[cnt], %[cnt], 1\n\t"
                "s_cmp_eq_u32 %[cnt], 0\n\t"
                "s_cbranch_scc1 .Lpv_tail%=\n"
                ".Lpv_loop%=:\n\t"
                PV_CMP("ac", "am", "ar", "ax")
                PV_FETCH("tb", "bc", "bm", "br", "bx")
                PV_SEL
                PV_UPD("ac", "am", "ax")
                PV_ASGX("ta")
                PV_CMP("bc", "bm", "br", "bx")
                PV_FETCH("ta", "ac", "am", "ar", "ax")
                PV_SEL
                PV_UPD("bc", "bm", "bx")
                PV_ASGX("tb")
                "s_sub_u32 %[cnt], %[cnt], 1\n\t"
                "s_cmp_lg_u32 %[cnt], 0\n\t"
                "s_cbranch_scc1 .Lpv_loop%=\n"
                ".Lpv_tail%=:\n\t"
                "s_cmp_lt_i32 %[ta], 0\n\t"
                "s_cbranch_scc1 .Lpv_done%=\n\t"
                PV_CMP("ac", "am", "ar", "ax")
                PV_SEL
                PV_UPD("ac", "am", "ax")
                PV_ASGX("ta")
                ".Lpv_done%=:\n\t"
                "s_mov_b32 m0, %[m0sv]\n"
                ".Lpv_end%=:"
                PV_OPS);
        } else {
            asm volatile(
                "s_cmp_eq_u64 %[q], 0\n\t"
                "s_cbranch_scc1 .Lpv_end%=\n\t"
                "s_mov_b32 %[m0sv], m0\n\t"
                "s_mov_b64 %[esv], exec\n\t"
                "s_bcnt1_i32_b64 %[cnt], %[q]\n\t"
                PV_FETCH("ta", "ac", "am", "ar", "ax")
                "s_lshr_b32 %[cnt], %[cnt], 1\n\t"
                "s_cmp_eq_u32 %[cnt], 0\n\t"
                "s_cbranch_scc1 .Lpv_tail%=\n"
                ".Lpv_loop%=:\n\t"
                PV_CMP("ac", "am", "ar", "ax")
                PV_FETCH("tb", "bc", "bm", "br", "bx")
                PV_SEL
                PV_UPD("ac", "am", "ax")
                PV_ASGW("ta")
                PV_CMP("bc", "bm", "br", "bx")
                PV_FETCH("ta", "ac", "am", "ar", "ax")
                PV_SEL
                PV_UPD("bc", "bm", "bx")
                PV_ASGW("tb")
                "s_sub_u32 %[cnt], %[cnt], 1\n\t"
                "s_cmp_lg_u32 %[cnt], 0\n\t"
                "s_cbranch_scc1 .Lpv_loop%=\n"
                ".Lpv_tail%=:\n\t"
                "s_cmp_lt_i32 %[ta], 0\n\t"
                "s_cbranch_scc1 .Lpv_done%=\n\t"
                PV_CMP("ac", "am", "ar", "ax")
                PV_SEL
                PV_UPD("ac", "am", "ax")
                PV_ASGW("ta")
                ".Lpv_done%=:\n\t"
                "s_mov_b32 m0, %[m0sv]\n"
                ".Lpv_end%=:"
                PV_OPS);
        }
#undef PV_ASG
    }
}

// same epilogue as fpp_group_x (placed bits, next candidate group of the misses)
template <int V, uint32_t g, uint32_t G>
__device__ __forceinline__ void group_vx(uint64_t q, uint64_t &placed, uint64_t &touched, uint32_t &asg,
                                         uint32_t &nxt, uint32_t &rcf, uint32_t &rmf, uint32_t &rcu, uint32_t rlab,
                                         uint32_t cpu, uint32_t mem, uint32_t req, uint32_t conf, uint32_t cand,
                                         uint32_t cand_hi, uint32_t gb64) {
    group_v<V>(q, touched, asg, rcf, rmf, rcu, rlab, cpu, mem, req, conf, gb64 + g * 64u);
    const uint32_t lane = __lane_id();
    const bool inq = (q >> lane) & 1ull;
    const uint64_t hit = __builtin_amdgcn_ballot_w64(inq && asg != 0xFFFFFFFFu);
    placed |= hit;
    if (inq && asg == 0xFFFFFFFFu) {
        const uint64_t above = (((uint64_t)cand_hi << 32) | cand) & ~((2ull << g) - 1ull);
        nxt = above ? (uint32_t)__builtin_ctzll(above) : G;
    }
}

}  // namespace fppv

namespace fppv {

// ---- node-major fill (first fit = node-major greedy; see fp_pipe.hip) ----
__device__ __forceinline__ uint32_t dpp_add_scan(uint32_t x) {  // inclusive, 64 lanes
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false); // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false); // row_bcast:31
    return x;
}
__device__ __forceinline__ uint32_t dpp_or_scan(uint32_t x) {
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
    return x;
}

template <uint32_t g, uint32_t G>
__device__ __forceinline__ void group_node_major(uint64_t q, uint64_t &placed, uint64_t &touched, uint32_t &asg,
                                                 uint32_t &nxt, uint32_t &rcf, uint32_t &rmf, uint32_t &rcu,
                                                 uint32_t rlab, uint32_t cpu, uint32_t mem, uint32_t req,
                                                 uint32_t conf, uint32_t cand, uint32_t cand_hi, uint32_t gb64) {
    const uint32_t lane = __lane_id();
    const uint32_t gbg = gb64 + g * 64u;
    const bool inq0 = (q >> lane) & 1ull;
    uint32_t qc = inq0 ? cpu : 0xFFFFFFFFu, qm = inq0 ? mem : 0xFFFFFFFFu;
    for (int o = 32; o; o >>= 1) {
        qc = min(qc, (uint32_t)__shfl_xor((int)qc, o));
        qm = min(qm, (uint32_t)__shfl_xor((int)qm, o));
    }
    qc = __builtin_amdgcn_readfirstlane(qc);
    qm = __builtin_amdgcn_readfirstlane(qm);
    uint64_t e = __builtin_amdgcn_ballot_w64(rcf >= qc && rmf >= qm);
    uint64_t Q = q;
    while (Q && e) {
        const uint32_t n = (uint32_t)__builtin_ctzll(e);
        e &= e - 1;
        uint32_t ncf = __builtin_amdgcn_readlane(rcf, n), nmf = __builtin_amdgcn_readlane(rmf, n);
        uint32_t ncu = __builtin_amdgcn_readlane(rcu, n);
        const uint32_t nlab = __builtin_amdgcn_readlane(rlab, n);
        bool took = false;
        while (true) {
            const bool el = ((Q >> lane) & 1ull) && cpu <= ncf && mem <= nmf && ((req & nlab) | (conf & ncu)) == 0u;
            const uint64_t E = __builtin_amdgcn_ballot_w64(el);
            if (!E) break;
            const uint32_t pc = dpp_add_scan(el ? cpu : 0u), pm = dpp_add_scan(el ? mem : 0u);
            const uint32_t px = dpp_or_scan(el ? conf : 0u);
            const uint32_t sx = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)px, 0x138, 0xF, 0xF, true);  // wave_shr:1
            const bool ok = el && pc <= ncf && pm <= nmf && (conf & sx) == 0u;
            const uint64_t F = E & ~__builtin_amdgcn_ballot_w64(ok);
            const uint64_t below = F ? ((1ull << __builtin_ctzll(F)) - 1ull) : ~0ull;
            const uint64_t T = E & below;
            const uint32_t last = 63u - (uint32_t)__builtin_clzll(T);
            ncf -= __builtin_amdgcn_readlane(pc, last);
            nmf -= __builtin_amdgcn_readlane(pm, last);
            ncu |= __builtin_amdgcn_readlane(px, last);
            if ((T >> lane) & 1ull) asg = gbg | n;
            Q &= ~T;
            took = true;
            if (!F) break;
        }
        if (took) {
            if (lane == n) { rcf = ncf; rmf = nmf; rcu = ncu; }
            touched |= 1ull << n;
        }
    }
    const bool inq = (Q >> lane) & 1ull;
    placed |= q & ~Q;
    if (inq0) {
        if (inq) {
            asg = 0xFFFFFFFFu;
            const uint64_t above = (((uint64_t)cand_hi << 32) | cand) & ~((2ull << g) - 1ull);
            nxt = above ? (uint32_t)__builtin_ctzll(above) : G;
        }
    }
}

}  // namespace fppv
