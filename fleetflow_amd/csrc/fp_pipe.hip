// fp_pipe.hip -- stage 3 FFD as an intra-workgroup tile pipeline (SPEC.md 2.3).
//
// A scenario's N nodes are cut into tiles of G groups of 64 nodes; one wave (a
// pipeline stage) owns a tile, W stages form a workgroup (a segment) and B
// segments cover the scenario.  A stage keeps its tile's node records (cpu_free,
// mem_free, conflict_used, labels) in VGPRs, so it checks a whole 64-node group
// with a wavefront ballot (lowest set lane = first fit inside the group).
// Containers stream through the stages in FFD order: stage 0 reads the sorted
// container list from HBM, places what fits its tile and forwards the rest, in
// order, to the next stage -- through an LDS ring inside a workgroup, through an
// unbounded global ring between segments; what the last stage cannot place is
// NOFIT.
//
// Exactness: a container lands in the first tile holding a feasible node, and a
// tile's state only depends on the containers that reached it, in FFD order --
// so the pipeline computes exactly the sequential first fit.
//
// Pruning (exact): per 64-node group g and threshold bucket k, two 64-bit masks
// B_cpu[g][k] = {l : sched && cpu_free >= Tc[k]} and B_mem[g][k] = {l : sched &&
// mem_free >= Tm[k]}.  A container in buckets (kc, km) (Tc[kc] <= cpu,
// Tm[km] <= mem) can only fit nodes in B_cpu[g][kc] & B_mem[g][km].  Free
// capacity only shrinks (SPEC.md 2.3 monotonicity), so masks are maintained by
// clearing bits on placement and a stale mask is always a superset: only
// candidate groups get the exact check.
#include "fp_internal.h"
// The candidate loop is group-major (below): every register access uses a compile-time
// group index.  (Round 1's container-major loops and the A/B variants of rounds 2-3 are in git
// history; DESIGN.md 7 keeps their numbers.)
#include "fp_pipe_asm.h"
#include "fp_pipe_sys.h"
#include "fp_pipe_pk.h"
#include "fp_pipe_tus.h"
#include <stdlib.h>
#include <string.h>
#include <mutex>
#include <type_traits>
#include <utility>

#ifdef FP_PIPE_STATS
// diagnostics build only: per stage w: [0] visits [1] cand checks [2] hits [3] batches
// [4] input-spin iterations [5] output-spin iterations, then s_memtime cycles in
// [8] input [9] prescan [10] candidate loop [11] results+forward [12] output wait
// [13] whole loop
__device__ unsigned long long g_pipe_stats[16 * 16];
#define STAT_ADD(w, i, v) atomicAdd(&g_pipe_stats[(w) * 16 + (i)], (unsigned long long)(v))
#define STAT_CLK() __builtin_amdgcn_s_memtime()
#define STAT_ON 1
// per group-queue timers ([6] check loop, [7] mask upkeep cycles, [14] queues, [15] touched nodes)
// and the global-link forwarding timer: they doubled config 3's diagnostics time, so only with
// FP_PIPE_STATS_FINE
// (tools/build_variant.sh _statsfine -DFP_PIPE_STATS -DFP_PIPE_STATS_FINE)
#ifdef FP_PIPE_STATS_FINE
#define STAT_GCLK() __builtin_amdgcn_s_memtime()
#define STAT_FINE 1
#else
#define STAT_GCLK() 0ull
#define STAT_FINE 0
#endif
// per-batch timeline of scenario 0, global stages 0-15 (k_ffd_pipe: the record's fields)
constexpr int TL_B = 2048;
__device__ unsigned long long g_pipe_tl[16 * TL_B * 8];
// per global stage of scenario 0 (s_memrealtime, 100 MHz, device-wide): [0] start [1] first
// input [2] loop end [3] busy cycles (prescan + candidate loop, s_memtime) [4] batches
// [5] output-wait cycles [6] input-spin iterations [7] placements
constexpr int SPAN_MAX = 4096;
__device__ unsigned long long g_stage_span[SPAN_MAX * 8];
#else
#define STAT_ADD(w, i, v) ((void)0)
#define STAT_CLK() 0ull
#define STAT_GCLK() 0ull
#define STAT_ON 0
#define STAT_FINE 0
#endif

// Wave priority of the FFD stages (s_setprio, MI355X_MICROARCH.md "Two waves per SIMD" items 2 and 4),
// PipeArgs::prio: 0 off; 1 raised to FP_PRIO_LEVEL while a wave runs its group loop (exact checks and
// fills: the placement chain); 2 raised for a batch's whole work, lowered while the wave polls its
// input.  r05a A/B (profiles/r05a_prio_ab.jsonl, FFD ms): 512 config-4 scenarios 6.96-7.00 -> 6.20-6.30
// (mode 1) / 6.61-6.68 (mode 2); config 3 64.8-65.0 -> 63.6-63.8 / 64.6-65.0; 4096 scenarios
// 15.06-15.08 -> 15.16-15.19 / 15.03: mode 1 except for the throughput kernel (wide12_big)
#ifndef FP_PRIO_LEVEL
#define FP_PRIO_LEVEL 2
#endif

namespace fpp {

constexpr int K = 32;               // threshold buckets per dimension
static_assert(K == FP_BUCKETS, "fp_place.hip and the pipeline agree on the bucket count");
constexpr uint32_t END = 0x80000000u;
// s_idx bit 31: the container never enters the pipeline (segment 0 writes assign FP_NONE and the
// reason code its s_req word carries: CYCLE, or NOFIT from the stage-2 screen, k_node_summary)
constexpr uint32_t CYC = 0x80000000u;
// Deadlock guard: a wait longer than this (s_memrealtime runs at 100 MHz) aborts the
// launch with FP_EDEVICE.  Downstream stages legitimately wait for most of a long
// launch, so the bound is wall-clock time, not an iteration count.
constexpr uint64_t SPIN_TICKS = 100ull * 1000 * 1000 * 60;  // 60 s (FP_OPT_SPIN_TICKS overrides: tests)
constexpr uint32_t MAX_G = 16;      // groups per stage (4 record VGPRs per group)
constexpr int SPIN_MAX = 12;         // longest back-off sleep of an idle stage (x 64 cycles)
constexpr int NF = 5;               // ring fields: cpu, mem, req, conf, idx
constexpr uint32_t IDX_POS_MASK = (1u << 21) - 1;  // position bits of a packed s_idx word

struct PipeArgs {
    uint32_t C, N, scen_base, W, G, R;
    uint32_t B;       // segments (workgroups) per scenario
    uint32_t S;       // scenarios of the launch
    uint32_t lag;     // ticket lag between consecutive segments of a scenario (see the kernel)
    uint32_t slots;   // slots per global link: a ring when `bounded`, else every container fits
    uint32_t bounded; // 1: links are rings with back-pressure (every segment co-resident, lag 0)
    uint32_t flush;   // idle flushes of partial output slots: bit 0 LDS rings, bit 1 global links (bounded)
    uint32_t kpack;   // 1: s_idx carries the bucket indices (bits 21-25 cpu, 26-30 mem; C <= 2^21)
    uint32_t publish; // full slots per head publish on a global link (1 when bounded: see the kernel)
    uint32_t pub_mask; // the unbounded-only kernel publishes when (head & pub_mask) == 0 (a power of two
                       // <= publish, minus 1): no loop-carried counter
    uint32_t sys;     // systolic group fill: queues of >= (sys & 0xFFFF) containers, (sys >> 16) extra
                      // steps before the serial finish (0: serial loop only)
    uint32_t *ticket; // workgroup ticket -> (scenario, segment) in launch order
    uint32_t *gabort; // launch-wide abort word (bounded spins)
    uint32_t *ghead;  // [S][B-1] link control, 256 B apart: [0] head, [32] consumer tail
    uint32_t *gdata;  // [S][B-1][slots][2][64] link slots: row 0 = count, row 1 = FFD positions
    uint32_t *part;   // [S][B][2] per-segment (n_used, n_rej)
    const uint32_t *s_cpu, *s_mem, *s_req, *s_conf, *s_idx;  // FFD-sorted SoA [S][C]; idx bit31 = skip
    uint32_t *cf, *mf;
    const uint32_t *lab;
    uint32_t *cu;
    const uint8_t *sched;
    uint32_t *assign;
    uint8_t *reason;
    uint64_t *cost;
    uint32_t *err;
    uint64_t spin_ticks;    // deadlock guard, s_memrealtime ticks (100 MHz)
    const uint32_t *thr;    // [2K] device: ascending thresholds, cpu then mem, thr[0] = thr[K] = 0
    uint32_t prio;          // wave priority mode (FP_PRIO_LEVEL comment)
    // packed-capacity pair (fp_pipe_pk.h): the batch's OR of every cpu value [0] and mem value [1]
    // (containers and schedulable nodes; k_scen_sort / k_make_keys / k_node_summary), and the mode:
    // 0 = the u32 kernel alone; 1 / 2 = the u32 / packed kernel of a pair launched back to back,
    // each running the batch only when the values do not / do pack (the other one returns)
    uint32_t *rng;  // [3]: [2] = the kernel that ran (1 u32, 2 packed; fp_ctx_place_path)
    uint32_t pk_mode;
};

// Control words (heads, tails, counts, abort flags) are read by every lane at one address: the
// loads below return them wave-uniform (readfirstlane), so that the loop exits they decide are
// uniform too.  Divergence analysis cannot see that a same-address load is uniform; a loop exit it
// believes divergent keeps every loop-carried counter of the kernel in VGPRs (and spills them).
__device__ __forceinline__ uint32_t lds_acq(uint32_t *p) {
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void lds_rel(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Cross-workgroup links follow MI355X_MICROARCH.md "Valid forms", table row 1:
// every payload dword is stored sc1 (relaxed agent-scope store), the storing wave
// drains with s_waitcnt vmcnt(0), then ONE lane stores the head with an agent-scope
// atomic store; the consumer polls the head with sc1 loads and reads every payload
// dword with sc1 loads, so no acquire fence is needed.
__device__ __forceinline__ uint32_t g_ld(const uint32_t *p) {
    return __hip_atomic_load(const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t g_ld_u(const uint32_t *p) {  // a control word: wave-uniform
    return __builtin_amdgcn_readfirstlane(g_ld(p));
}
__device__ __forceinline__ void g_st(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Spin on an LDS word until pred holds; bounded, with a workgroup abort flag.
template <class Pred>
__device__ __forceinline__ bool spin(uint32_t *word, Pred pred, uint32_t *abort_flag, uint32_t *err,
                                     uint64_t ticks, uint32_t &iters) {
    uint32_t n = 0;
    uint64_t t0 = 0;
    while (true) {
        const uint32_t v = lds_acq(word);
        if (pred(v)) { iters += n; return true; }
        if (lds_acq(abort_flag)) return false;
        if ((++n & 1023u) == 0) {
            const uint64_t now = __builtin_amdgcn_s_memrealtime();
            if (!t0) {
                t0 = now;
            } else if (now - t0 > ticks) {
                lds_rel(abort_flag, 1u);
                if ((threadIdx.x & 63) == 0) atomicMax(err, (uint32_t)(-FP_EDEVICE));
                return false;
            }
        }
        // back off: a spinning wave still takes issue slots from its CU's busy waves
        if (n < 8) __builtin_amdgcn_s_sleep(1);
        else if (n < 32) __builtin_amdgcn_s_sleep(4);
        else __builtin_amdgcn_s_sleep(SPIN_MAX);
    }
}


// bucket index: largest k with T[k] <= v (T ascending, T[0] = 0; lane base + k holds
// T[k]).  Binary search through ds_bpermute: no scalar registers held across the
// main loop (hoisted per-threshold readlanes spill SGPRs).
__device__ __forceinline__ uint32_t bucket_of(uint32_t v, uint32_t my_t, int base) {
    uint32_t k = 0;
#pragma unroll
    for (uint32_t step = K / 2; step; step >>= 1) {
        const uint32_t t = (uint32_t)__shfl((int)my_t, (int)(base + k + step));
        k += t <= v ? step : 0u;
    }
    return k;
}

// number of set bits of a wave mask below this lane (v_mbcnt: no per-lane below-mask kept live)
__device__ __forceinline__ uint32_t fpp_rank(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// min over the wave's 64 lanes, broadcast (DPP row shifts + row broadcasts into lane 63;
// lanes without a DPP source read UINT32_MAX, the identity of min)
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x111, 0xF, 0xF, false));  // row_shr:1
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x112, 0xF, 0xF, false));  // row_shr:2
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x114, 0xF, 0xF, false));  // row_shr:4
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x118, 0xF, 0xF, false));  // row_shr:8
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x142, 0xA, 0xF, false));  // row_bcast:15
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x143, 0xC, 0xF, false));  // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}


constexpr size_t LCTL = 64;  // u32 per global link control block: [0] head, [LCTL / 2] tail

// Bounded global link: wait (wave-uniform) until the producer may write every slot below
// `need`, i.e. need - tail <= slots.  `seen` caches the consumer's tail so the common case
// reads no memory.  Same abort and deadlock guard as the consumer's head poll.
__device__ __forceinline__ bool gring_wait(uint32_t *tail, uint32_t need, uint32_t slots, uint32_t &seen,
                                           const PipeArgs &a, uint32_t *abort_flag, uint32_t lane,
                                           uint32_t &iters) {
    if (need - seen <= slots) return true;
    uint32_t n = 0;
    uint64_t t0 = 0;
    while (true) {
        seen = g_ld_u(tail);
        if (need - seen <= slots) { iters += n; return true; }
        if (g_ld_u(a.gabort) || lds_acq(abort_flag)) return false;
        if ((++n & 255u) == 0) {
            const uint64_t now = __builtin_amdgcn_s_memrealtime();
            if (!t0) {
                t0 = now;
            } else if (now - t0 > a.spin_ticks) {
                g_st(a.gabort, 1u);
                lds_rel(abort_flag, 1u);
                if (lane == 0) atomicMax(a.err, (uint32_t)(-FP_EDEVICE));
                return false;
            }
        }
        if (n < 8) __builtin_amdgcn_s_sleep(2);
        else __builtin_amdgcn_s_sleep(SPIN_MAX);
    }
}

// Node records (cpu_free, mem_free, conflict_used, labels) of a wave's tile live
// in that wave's VGPRs: G compile-time groups, 4 registers each.  The prescan
// reads them with static indices; the candidate loop reads and updates group g
// (wave-uniform) through s_set_gpr_idx-indexed moves.  LDS then holds only the
// masks and the rings, so two workgroups fit on one CU.
// LDS layout (bytes; every region 16-aligned):
//   M   : W*G*K*2 u64           B_cpu / B_mem interleaved per (g, k)
//   CTL : (W-1)*8 u32 + 8 u32   per link [0]=head [1]=tail [2..2+R)=slot counts; then
//                               CNT [0]=n_used [1]=n_rej [2]=abort
//   D   : (W-1)*R*NF*64 u32     ring slots, field-major
// a tile's records of one kind, one register per group (a plain array, register-promoted
// with static indices)
template <uint32_t G>
using RecT = uint32_t[G];

// the group-major loop over a stage's groups, g a compile-time constant in every call.
// After a group's queue: the used-node bits and (UPD) the bucket masks catch up with the
// nodes the queue placed on (`touched`), once per group and batch instead of per placement.
// Bucket lane k (lanes 0-31 cpu thresholds, 32-63 mem) clears node l's bit when the node's
// free capacity is now below the threshold.
//
// Queue prefilter: group g's records do not change before its queue is processed, so a
// queued container that fits no node of g NOW never will (monotone) and leaves for its
// next candidate group without a serial check.  The test is vector-parallel over the
// queue: the nodes that could take the batch's smallest demands (the batch corner, qc/qm)
// are broadcast one at a time and every lane tests its own container.  It pays while the
// corner holds few nodes (the filled-up frontier group); above PF_MAX_* nodes the queue
// goes to the serial loop unfiltered.
// Corner-node limit of the prefilter, by stage width (r03m A/B, profiles/r03m_ab*.jsonl): narrow
// (<= 4-group) stages 4 -- config 3 65.3 -> 64.1 ms (16: 65.3, 32: 70.8); wide stages off -- config
// 4 17.54 -> 17.28 ms (4: 17.48, 32: 17.96).
#ifndef FPP_PF_MAX_WIDE  // without the mask upkeep too: 4 / 16 corner nodes in the wide stages, config 4
#define FPP_PF_MAX_WIDE 0  // 11.98-12.01 against 11.20-11.31 ms (profiles/r08y_prefilter_wide_ab.jsonl)
#endif
#ifndef FPP_PF_MAX_NARROW
#define FPP_PF_MAX_NARROW 4
#endif
constexpr uint32_t PF_MAX_NARROW = FPP_PF_MAX_NARROW, PF_MAX_WIDE = FPP_PF_MAX_WIDE;
// lane selects by inverse ballot in the one-wave kernels' group bookkeeping (fpp_lane_sel)
#ifndef FPP_IB
#define FPP_IB 1
#endif
#ifndef FPP_IB1024  // ... and in the 1024-thread kernels of more than SYS_MAX_G groups: on since the mask
#define FPP_IB1024 1  // upkeep went (512 / 1024 scenarios 4.91-4.97 / 6.15-6.20 vs 4.96-5.01 / 6.19-6.31 ms,
#endif                // profiles/r08z_ib1024_ab.jsonl; with the upkeep round 5 measured 6.43 / 7.79 vs 6.21 / 7.58)
// the systolic group fill (fp_pipe_sys.h) is compiled for stages of at most this many groups
constexpr uint32_t SYS_MAX_G = 4;
// ... and the packed one (fp_pipe_pk.h) for stages of at most this many (its records take one VGPR
// fewer per group)
// Bucket-mask upkeep (UPD in fpp_groups): clearing a touched node's bucket bits after each group's
// queue keeps the masks tight, but with the packed records a check costs less than the upkeep: off,
// the masks stay as the stage built them (a stale mask is a superset, so the plans are the same --
// identical digests), and config 4's FFD went 12.16 -> 11.18 ms, 2048 / 1024 / 512 scenarios 8.79 ->
// 7.92, 6.91 -> 6.23, 5.63 -> 4.98 ms (profiles/r08vw_mask_upkeep_ab.jsonl).  Round 2 measured the
// opposite for its u32 20-group stages (57 vs 66 ms).  1 turns it back on.
#ifndef FPP_MASK_UPKEEP
#define FPP_MASK_UPKEEP 0
#endif
#ifndef FPP_PK_SYS_MAX_G
#define FPP_PK_SYS_MAX_G 4
#endif
constexpr uint32_t PK_SYS_MAX_G = FPP_PK_SYS_MAX_G;
// The serial loop over one group's queue is the exec-masked loop (fp_pipe_asm.h fpp_group_x:
// 172 vs 264 cycles per container for round 2's readlane / writelane loop).
template <uint32_t G, bool UPD, bool IB, bool PK, uint32_t... gs, class Rec>
__device__ __forceinline__ void fpp_groups(std::integer_sequence<uint32_t, gs...>, uint32_t &nxt, uint64_t &placed,
                                           uint32_t &asg, uint32_t &used, uint32_t &used_hi, Rec &rcf, Rec &rmf,
                                           Rec &rcu, const Rec &rlab, uint32_t cpu, uint32_t mem, uint32_t req,
                                           uint32_t conf, uint32_t cand, uint32_t cand_hi, uint32_t my_t, uint32_t lane,
                                           uint64_t *Mw, uint32_t mlane, uint32_t gb64, uint32_t qc, uint32_t qm, uint32_t &nchk,
                                           uint32_t &nhit, uint32_t sys, unsigned long long (&gst)[4], uint32_t cw,
                                           uint32_t qw, uint32_t sc_c, uint32_t sc_m) {
    // PK (fp_pipe_pk.h): rcf[g] holds the packed (cpu, mem) record and rmf is unused; cw / qw are the
    // container's and the batch corner's packed demands, sc_c / sc_m the batch's shifts
    constexpr uint32_t pf_max = G <= SYS_MAX_G ? PF_MAX_NARROW : PF_MAX_WIDE;
    (
        [&] {
            uint64_t q = __builtin_amdgcn_ballot_w64(nxt == gs);
            if (pf_max > 0 && q) {
                uint64_t e;
                if constexpr (PK) e = __builtin_amdgcn_ballot_w64(pk_fits(rcf[gs], qw));
                else e = (__builtin_amdgcn_ballot_w64(rcf[gs] >= qc) & __builtin_amdgcn_ballot_w64(rmf[gs] >= qm));
                if (__builtin_popcountll(e) <= pf_max) {
                    bool ok = false;
                    while (e) {
                        const uint32_t l = (uint32_t)__builtin_ctzll(e);
                        e &= e - 1;
                        const uint32_t nlb = __builtin_amdgcn_readlane(rlab[gs], l);
                        const uint32_t ncu = __builtin_amdgcn_readlane(rcu[gs], l);
                        if constexpr (PK) {
                            const uint32_t nw = __builtin_amdgcn_readlane(rcf[gs], l);
                            ok |= ((((nw - cw) & PK_GUARD) | (req & nlb) | (conf & ncu)) == 0u);
                        } else {
                            const uint32_t ncf = __builtin_amdgcn_readlane(rcf[gs], l);
                            const uint32_t nmf = __builtin_amdgcn_readlane(rmf[gs], l);
                            ok |= (ncf >= cpu) & (nmf >= mem) & (((req & nlb) | (conf & ncu)) == 0u);
                        }
                    }
                    const uint64_t fit = q & __builtin_amdgcn_ballot_w64(ok);
                    if (q != fit) {  // the others move on: next candidate group above g, or none
                        const uint64_t above = (((uint64_t)cand_hi << 32) | cand) & ~((2ull << gs) - 1ull);
                        const uint32_t nx = above ? (uint32_t)__builtin_ctzll(above) : G;
                        nxt = ((q & ~fit) >> lane) & 1ull ? nx : nxt;
                    }
                    q = fit;
                }
            }
            if (q) {
                uint64_t touched = 0;
                const unsigned long long gc0 = STAT_GCLK();
                // long queues (a filling group): the systolic loop, else the serial one
                // (compiled for the narrow stages only: the wide kernels stay within their VGPR budget)
                if constexpr (PK) {
                    if (G <= PK_SYS_MAX_G && sys && (uint32_t)__builtin_popcountll(q) >= (sys & 0xFFFFu))
                        fpp_group_sysp<gs, G>(q, placed, touched, asg, nxt, rcf[gs], rcu[gs], rlab[gs], cw, req, conf,
                                              cand, cand_hi, gb64, nchk, nhit, qw, sys >> 16);
                    else
                        fpp_group_xp<gs, G, IB>(q, placed, touched, asg, nxt, rcf[gs], rcu[gs], rlab[gs], cw, req, conf,
                                                cand, cand_hi, gb64, nchk, nhit, qw);
                } else {
                    if (G <= SYS_MAX_G && sys && (uint32_t)__builtin_popcountll(q) >= (sys & 0xFFFFu))
                        fpp_group_sys<gs, G>(q, placed, touched, asg, nxt, rcf[gs], rmf[gs], rcu[gs], rlab[gs], cpu, mem,
                                             req, conf, cand, cand_hi, gb64, nchk, nhit, qc, qm, sys >> 16);
                    else
                        fpp_group_x<gs, G, IB>(q, placed, touched, asg, nxt, rcf[gs], rmf[gs], rcu[gs], rlab[gs], cpu, mem,
                                               req, conf, cand, cand_hi, gb64, nchk, nhit, qc, qm);
                }
                const unsigned long long gc1 = STAT_GCLK();
                if (STAT_FINE) { gst[0] += gc1 - gc0; gst[2] += 1; gst[3] += (uint32_t)__builtin_popcountll(touched); }
                if (touched) {
                    // a touched node's new free capacity (unpacked in the packed kernels)
                    auto node_cm = [&](uint32_t l, uint32_t &nc, uint32_t &nm) {
                        if constexpr (PK) {
                            const uint32_t nw = __builtin_amdgcn_readlane(rcf[gs], l);
                            nc = pk_cpu(nw, sc_c);
                            nm = pk_mem(nw, sc_m);
                        } else {
                            nc = __builtin_amdgcn_readlane(rcf[gs], l);
                            nm = __builtin_amdgcn_readlane(rmf[gs], l);
                        }
                    };
                    if constexpr (IB) {
                        // one-wave kernels: lane selects read the masks directly (fpp_lane_sel).
                        // Bucket lane k clears node l's bit when the node's new free capacity is
                        // below T[k] (cpu for lanes 0-31, mem for 32-63): per touched node, two
                        // compares give the lanes to clear as a wave mask, and one select per half
                        // sets bit l there.
                        if (gs < 32) used = fpp_lane_sel<true>(touched, used | (1u << gs), used);
                        else used_hi = fpp_lane_sel<true>(touched, used_hi | (1u << (gs & 31)), used_hi);
                        if (UPD) {
                            uint32_t clr_lo = 0, clr_hi = 0;
                            uint64_t tt = touched;
                            while (tt) {
                                const uint32_t l = (uint32_t)__builtin_ctzll(tt);
                                tt &= tt - 1;
                                uint32_t nc, nm;
                                node_cm(l, nc, nm);
                                const uint64_t below = (__builtin_amdgcn_ballot_w64(my_t > nc) & 0xFFFFFFFFull) |
                                                       (__builtin_amdgcn_ballot_w64(my_t > nm) & ~0xFFFFFFFFull);
                                if (l < 32) clr_lo = fpp_lane_sel<true>(below, clr_lo | (1u << l), clr_lo);
                                else clr_hi = fpp_lane_sel<true>(below, clr_hi | (1u << (l & 31)), clr_hi);
                            }
                            const uint64_t clr = ((uint64_t)clr_hi << 32) | clr_lo;
                            // the group's mask word of this bucket lane at an immediate offset from one
                            // per-lane LDS address (a per-group address was hoisted and spilled)
                            if (__builtin_amdgcn_ballot_w64(clr != 0))
                                asm volatile("ds_and_b64 %0, %1 offset:%2" ::"v"(mlane), "v"(~clr),
                                             "i"(gs * K * 2 * 8) : "memory");
                        }
                    } else {
                        const bool me = (touched >> lane) & 1ull;
                        if (gs < 32) used |= me ? (1u << gs) : 0u;
                        else used_hi |= me ? (1u << (gs & 31)) : 0u;
                        if (UPD) {
                            uint64_t clr = 0, tt = touched;
                            while (tt) {
                                const uint32_t l = (uint32_t)__builtin_ctzll(tt);
                                tt &= tt - 1;
                                uint32_t nc, nm;
                                node_cm(l, nc, nm);
                                // a bit at or below the node's new free capacity stays; every bit above
                                // it goes (clearing a bit that was already clear is harmless, so the
                                // capacity before the queue is not needed)
                                clr |= (my_t > (lane < 32 ? nc : nm)) ? (1ull << l) : 0ull;
                            }
                            if (__builtin_amdgcn_ballot_w64(clr != 0))
                                atomicAnd((unsigned long long *)&Mw[(size_t)gs * K * 2 + (lane & (K - 1)) * 2 + (lane >> 5)],
                                          ~clr);
                        }
                    }
                }
                if (STAT_FINE) gst[1] += STAT_GCLK() - gc1;
            }
        }(),
        ...);
}

// BLK: 1024 for multi-stage segments (W <= 16 waves, <= 128 VGPRs each); 64 for the one-wave
// segments of the wide geometry, whose 13..40 groups of records take 4 VGPRs per group, compiled
// for WIDE_WAVES waves per SIMD (3: at most 168 VGPRs, 12 segments in flight per CU).
// One-wave segments of 12 groups (many-scenario batches) are compiled for WIDE12_WAVES waves per
// SIMD: 5 fits them in 96 VGPRs (32 B of scratch) and 20 segments per CU -- config-4 FFD 20.9 ->
// 18.7 ms against the 1024-thread kernel's 107 VGPRs and four waves (6 waves: 80 VGPRs, 100 B of
// scratch, 19.2 ms).
constexpr uint32_t WIDE_WAVES = 3, WIDE12_WAVES = 5;
// Batches of at least WIDE12_BIG_S scenarios use a second 12-group instantiation compiled for six
// waves per SIMD (80 VGPRs, 84 B of scratch, 6144 resident segments): config 4 at 4096 scenarios
// FFD 14.93-14.95 vs 15.20-15.23 ms; at 2048 it loses (10.21-10.35 vs 9.87-9.90), the spills costing
// more than the extra slots buy (profiles/r04x_waves_ab.jsonl).  The 8-group segments of batches of up to
// 1024 scenarios stay at five waves (k_ffd_pipe<8, 1024>, 82 VGPRs): six or seven waves ran 1024
// scenarios 8.69 / 9.18 vs 8.46-8.54 ms (profiles/r04ab_small8_waves_ab.jsonl)
#ifndef FPP_BIG_WAVES
#define FPP_BIG_WAVES 6
#endif
#ifndef FPP_BIG_S
#define FPP_BIG_S 4096
#endif
[[maybe_unused]] constexpr uint32_t WIDE12_BIG_WAVES = FPP_BIG_WAVES, WIDE12_BIG_S = FPP_BIG_S;
// Batch prescan: a group with an empty batch corner skips its bucket-mask loads in the wide stages
// (config-4 FFD 17.38 -> 15.72 ms: a batch that passes a segment mostly has every corner empty);
// the narrow stages keep the branch-free form (config 3: 64.3 vs 65.3 ms with the skip; r03z A/B,
// profiles/r03z_prescan_ab.jsonl).  A batch without candidates skips the group loop (config-4
// FFD 15.62 -> 15.06 ms, config 3 64.3 -> 63.6 ms; r03aa/r03ab).  Measured slower and removed in
// round 4: per-group capacity bounds in place of the corner ballots (15.73 vs 15.08
// ms, r03af), req / conf of link input loaded after the prescan (15.45 vs 15.08 ms, r03ac).
template <uint32_t G, uint32_t BLK, uint32_t WV = 0, bool PK = false>
__global__ __launch_bounds__(BLK, BLK == 64 ? (WV ? WV : G == 12 ? WIDE12_WAVES : WIDE_WAVES) : 1) void
k_ffd_pipe(const PipeArgs a_arg) {
    // the arguments are read through the kernarg segment (memory), not promoted to SGPRs for the
    // whole kernel: held in SGPRs they spilled into VGPR lanes (wide kernel: 781 v_readlane vs 296,
    // config-4 FFD 16.7 vs 15.2 ms; narrow kernel by value: config 3 65.9 vs 65.0 ms, r04o A/B)
#if defined(__HIP_DEVICE_COMPILE__)
    const PipeArgs &a = *(const PipeArgs *)__builtin_amdgcn_kernarg_segment_ptr();
#else
    const PipeArgs &a = a_arg;  // the host pass only type-checks the body
#endif
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // one-wave segments (BLK == 64) are a compile-time W = 1: the LDS-ring paths between stages
    // of a segment drop out of those kernels
#ifndef FPP_W1
#define FPP_W1 1
#endif
    constexpr bool one_wave = BLK == 64 && FPP_W1;
    const uint32_t W = one_wave ? 1u : a.W, R = a.R, B = a.B, prio = a.prio;
    const uint32_t w = one_wave ? 0u : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t C = a.C, N = a.N;
    // the FFD position inside an s_idx word (above it: CYCLE bit 31, packed buckets)
    const uint32_t pmask = a.kpack ? IDX_POS_MASK : ~CYC;
    // per-lane group bit sets (schedulable / candidate groups): 64-bit above 32 groups
    using GM = typename std::conditional<(G > 32), uint64_t, uint32_t>::type;

    uint64_t *M = reinterpret_cast<uint64_t *>(smem);
    uint32_t *CTL = reinterpret_cast<uint32_t *>(M + (size_t)W * G * K * 2);
    uint32_t *CNT = CTL + (W - 1) * 8;
    uint32_t *D = CNT + 8;

    // the packed pair: this kernel runs the batch only if its values pack (PK) / do not (!PK)
    uint32_t sc_c = 0, sc_m = 0;
    if (PK || a.pk_mode) {
        const uint32_t orc = __builtin_amdgcn_readfirstlane(a.rng[0]), orm = __builtin_amdgcn_readfirstlane(a.rng[1]);
        sc_c = orc ? (uint32_t)__builtin_ctz(orc) : 0u;
        sc_m = orm ? (uint32_t)__builtin_ctz(orm) : 0u;
        const bool packs = (orc >> sc_c) <= PK_FIELD_MAX && (orm >> sc_m) <= PK_FIELD_MAX;
        if (packs != PK) return;  // uniform: the other kernel of the pair takes the batch
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && a.rng) a.rng[2] = PK ? 2u : 1u;  // fp_ctx_place_path
    for (uint32_t i = threadIdx.x; i < (W - 1) * 8 + 8; i += blockDim.x) CTL[i] = 0;
    __syncthreads();
    // Ticket order = start order.  Ticket t is round r = t / B, segment b = t % B, and
    // scenario s = r - b * lag: segment b of scenario s starts `lag` rounds after segment
    // b - 1 of it.  Segment b only ever waits on segment b - 1, which took an earlier
    // ticket, is running or done, and never waits on b (global links hold every
    // container) -- so the chain progresses whatever the residency or dispatch order.
    // lag = 0 runs a scenario's segments side by side (one scenario: the pipeline is all
    // the parallelism there is); with many scenarios a lag of about the resident
    // segment count starts a segment when its input is (nearly) complete, so it is busy
    // for its whole lifetime instead of waiting on its upstream half the time.
    // Tickets naming no scenario (the ramp at either end) are skipped; a workgroup
    // that finds none left exits.
    if (threadIdx.x == 0) {
        const uint32_t total = (a.S + (B - 1) * a.lag) * B;
        uint32_t t;
        while (true) {
            t = atomicAdd(a.ticket, 1u);
            if (t >= total) { t = 0xFFFFFFFFu; break; }
            const uint32_t r = t / B, bb = t % B;
            if (r >= bb * a.lag && r - bb * a.lag < a.S) break;
        }
        CNT[4] = t;
    }
    __syncthreads();
    const uint32_t tk = __builtin_amdgcn_readfirstlane(CNT[4]);
    if (tk == 0xFFFFFFFFu) return;  // uniform: every wave of the workgroup leaves
    const uint32_t b = tk % B, s = tk / B - b * a.lag;
    const size_t cb = (size_t)s * C, nb = (size_t)s * N;

    // ---- stage the tile into LDS and build the bucket masks ----
    // lane k < 32 holds Tc[k], lane 32 + k holds Tm[k] (K == 32: one wave covers both)
    static_assert(K == 32, "mask/threshold lane layout assumes K == 32");
    const uint32_t my_t = a.thr[lane];
    const uint32_t gbase = (b * W + w) * G;             // first (global) group of this tile
    uint64_t *Mw = M + (size_t)w * G * K * 2;           // the tile's masks
    // LDS byte address of this bucket lane's mask word of group 0 (one-wave kernels' mask upkeep)
    const uint32_t mlane = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint64_t *)(Mw + (lane & (K - 1)) * 2 + (lane >> 5));
    // The tile's node records.  Unschedulable (and padding) nodes are stored so that every
    // container with a nonzero field fails the exact check on them: cpu = mem = 0, all
    // conflict bits used, all (inverted) label bits missing.  The all-zero container, which
    // would pass, never reaches the check (placed on the tile's first schedulable node).
    // rlab holds ~labels: label and conflict tests become one ((~lab & req) | (cu & conf)) == 0.
    RecT<G> rcf, rmf, rcu, rlab;
    GM schedbits = 0;                                   // bit g: node (g, lane) schedulable
    uint32_t usedbits = 0, used_hi = 0;                 // bit g (g - 32 in used_hi): node (g, lane) used
    {
        // branch-free loads from one base address per array (group g at an immediate
        // offset, padding lanes clamped to node 0): divergent per-group branches here kept
        // 64-bit addresses of every group live at once and set the kernel's VGPR count
        const uint32_t n0 = gbase * 64 + lane;
        const uint32_t *cf0 = a.cf + nb + n0, *mf0 = a.mf + nb + n0, *cu0 = a.cu + nb + n0, *lb0 = a.lab + nb + n0;
        const uint8_t *sc0 = a.sched + nb + n0;
#pragma unroll
        for (uint32_t g = 0; g < G; ++g) {
            const bool in = n0 + g * 64 < N;
            const int o = in ? (int)(g * 64) : -(int)n0;  // padding lanes read node 0 of the scenario
            const bool sc = in && sc0[o] != 0;
            const uint32_t x = cf0[o], y = mf0[o], z = cu0[o], l = lb0[o];
            if constexpr (PK) {
                rcf[g] = sc ? pk_pack(x, y, sc_c, sc_m) : 0u;  // rmf unused
            } else {
                rcf[g] = sc ? x : 0u;
                rmf[g] = sc ? y : 0u;
            }
            rcu[g] = sc ? z : 0xFFFFFFFFu;
            rlab[g] = sc ? ~l : 0xFFFFFFFFu;
            schedbits |= sc ? (GM(1) << g) : GM(0);
        }
    }
    uint32_t zs_g = G, zs_l = 0;  // the tile's first schedulable node (all-zero containers)
#pragma unroll
    for (uint32_t g = 0; g < G; ++g) {
        const uint64_t sm = __builtin_amdgcn_ballot_w64(((schedbits >> g) & 1u) != 0);
        if (zs_g == G && sm) {
            zs_g = g;
            zs_l = (uint32_t)__builtin_ctzll(sm);
        }
    }
    // bucket-major (a rolled loop): two thresholds live in scalars at a time -- hoisting all
    // 64 of them out of an unrolled loop spilled scalars into VGPR lanes
#pragma unroll 1
    for (uint32_t k = 0; k < (uint32_t)K; ++k) {
        const uint32_t tc = __builtin_amdgcn_readlane(my_t, k), tm = __builtin_amdgcn_readlane(my_t, K + k);
#pragma unroll
        for (uint32_t g = 0; g < G; ++g) {  // every lane takes part in each ballot
            const bool sc = (schedbits >> g) & 1u;
            const uint32_t ncf = PK ? pk_cpu(rcf[g], sc_c) : rcf[g], nmf = PK ? pk_mem(rcf[g], sc_m) : rmf[g];
            const uint64_t bc = __builtin_amdgcn_ballot_w64(sc & (ncf >= tc));
            const uint64_t bm = __builtin_amdgcn_ballot_w64(sc & (nmf >= tm));
            if (lane == k) {
                Mw[((size_t)g * K + k) * 2] = bc;
                Mw[((size_t)g * K + k) * 2 + 1] = bm;
            }
        }
    }
    __syncthreads();

    const bool has_out = w + 1 < W;
    const bool g_in = w == 0 && b > 0;                  // input from segment b-1
    const bool g_out = w + 1 == W && b + 1 < B;         // output to segment b+1
    // a global link slot: [0] = count (or END), [64..127] = the containers' FFD positions;
    // the consumer re-reads their fields from the sorted SoA (4 B per forwarded container
    // instead of 20: links sized for every container stay 5x smaller)
    const size_t LSLOT = 2 * 64;                        // u32 per global slot
    uint32_t *gin_head = a.ghead + ((size_t)s * (B - 1) + (b - 1)) * LCTL;
    uint32_t *gin_data = a.gdata + ((size_t)s * (B - 1) + (b - 1)) * a.slots * LSLOT;
    uint32_t *gout_head = a.ghead + ((size_t)s * (B - 1) + b) * LCTL;
    uint32_t *gout_data = a.gdata + ((size_t)s * (B - 1) + b) * a.slots * LSLOT;
    // bounded links: the consumer publishes how many slots it has finished with (tail, a
    // separate 128-B line); the producer writes slot h only while h - tail < slots.  Slot
    // index = sequence number mod slots (identity when unbounded: slots >= every slot).
    // the six-wave many-scenario kernel only ever runs unbounded links (lag = S phases; the launch
    // takes the five-wave one when a bounded ring is forced): slot index = sequence number, and the
    // ring waits, tail publishes and idle flushes of the global links compile out
    constexpr bool unbounded_only = BLK == 64 && WV != 0;
    const uint32_t gslots = a.slots, gbounded = unbounded_only ? 0u : a.bounded;
    const uint32_t gflush = unbounded_only ? (a.flush & 1u) : a.flush;
#define GSLOT(i) (unbounded_only ? (uint32_t)(i) : (uint32_t)(i) % gslots)
    uint32_t otail_seen = 0;                            // last tail read from the consumer
    uint32_t *octl = CTL + w * 8;
    uint32_t *ictl = CTL + (w - 1) * 8;
    uint32_t *odata = D + (size_t)w * R * NF * 64;
    uint32_t *idata = D + (size_t)(w - 1) * R * NF * 64;
    uint32_t *abort_flag = &CNT[2];
    uint32_t ohead = 0, ofill = 0, itail = 0, k0 = 0;
    uint32_t ihead_seen = 0;  // last head read from the upstream link
    // full slots written but not yet published (global link): the head store and the wait for
    // the slot stores before it (s_waitcnt vmcnt(0)) are paid once per a.publish slots; the end
    // of the stream publishes the rest
    uint32_t opend = 0;
    uint32_t n_used = 0, n_rej = 0;
    uint32_t st_spin_in = 0, st_spin_out = 0, st_visits = 0, st_checks = 0, st_hits = 0, st_batches = 0;
    unsigned long long ck_in = 0, ck_pre = 0, ck_cand = 0, ck_fwd = 0, ck_wait = 0, ck_gx = 0, ck_gu = 0;
    uint32_t st_queues = 0, st_touched = 0;
    const unsigned long long ck_t0 = STAT_CLK();
    unsigned long long ck_a, ck_b;
#ifdef FP_PIPE_STATS
    const unsigned long long sp_start = __builtin_amdgcn_s_memrealtime();
    unsigned long long sp_first = 0;
#endif
    bool alive = true;
    while (alive) {
        if (prio == 2u) __builtin_amdgcn_s_setprio(0);  // polls / spins at the lowest priority
        ck_a = STAT_CLK();
#ifdef FP_PIPE_STATS
        const unsigned long long tl_top = ck_a;  // timeline: the previous batch's end
        unsigned long long tl_avail = ck_a;      // timeline: this batch's input available
#endif
        uint32_t cpu = 0, mem = 0, req = 0, conf = 0, idx = 0;
        bool valid = false;
        if (g_in) {
            // poll the upstream segment's head (sc1), bounded; then sc1 payload loads
            uint32_t n_sp = 0;
            uint64_t t0 = 0;
            bool got = itail < ihead_seen;  // a head seen earlier already covers this slot: no poll
            while (!got) {
                ihead_seen = g_ld_u(gin_head);
                if (ihead_seen > itail) { got = true; break; }
                if (g_ld_u(a.gabort) || lds_acq(abort_flag)) break;
                if ((++n_sp & 255u) == 0) {
                    const uint64_t now = __builtin_amdgcn_s_memrealtime();
                    if (!t0) {
                        t0 = now;
                    } else if (now - t0 > a.spin_ticks) {
                        g_st(a.gabort, 1u);
                        lds_rel(abort_flag, 1u);
                        if (lane == 0) atomicMax(a.err, (uint32_t)(-FP_EDEVICE));
                        break;
                    }
                }
                if (n_sp < 8) __builtin_amdgcn_s_sleep(2);
                else __builtin_amdgcn_s_sleep(SPIN_MAX);
            }
            st_spin_in += n_sp;
            if (!got) break;
#ifdef FP_PIPE_STATS
            tl_avail = STAT_CLK();
#endif
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only
            // slots before itail are finished with: their loads returned last iteration
            // (the container fields they addressed were consumed), so the producer may
            // reuse them.  Published every 4 slots (the ring keeps that much slack).
            // With idle flushes the producer reads it as "the consumer is on my last slot":
            // published every slot then.
            if (((gflush & 2u) || (gbounded && (itail & 3u) == 0)) && lane == 0) g_st(gin_head + LCTL / 2, itail);
            const uint32_t *sd = gin_data + (size_t)GSLOT(itail) * LSLOT;
            // the count is wave-uniform: say so, or the loop exit below reads as divergent and every
            // loop-carried counter of the kernel is kept (and spilled) in VGPRs
            const uint32_t n = g_ld_u(sd);
            const uint32_t pos = g_ld(sd + 64 + lane);  // with the count: one round trip
            if (n & END) break;
            valid = lane < n;
            if (valid) {
                idx = pos;  // the packed s_idx word (position | buckets)
                const uint32_t p = pos & pmask;
                cpu = a.s_cpu[cb + p];
                mem = a.s_mem[cb + p];
                req = a.s_req[cb + p];
                conf = a.s_conf[cb + p];
            }
            itail++;
        } else if (w == 0) {
            if (k0 >= C) break;
            const uint32_t i = k0 + lane;
            valid = i < C;
            if (valid) {
                cpu = a.s_cpu[cb + i];
                mem = a.s_mem[cb + i];
                req = a.s_req[cb + i];
                conf = a.s_conf[cb + i];
                idx = a.s_idx[cb + i];
            }
            const bool cyc = valid && (idx & CYC);
            if (cyc) {  // CYCLE member, or screened out by stage 2 (NOFIT): s_req holds the reason
                const uint32_t j = idx & pmask;
                a.assign[cb + j] = FP_NONE;
                a.reason[cb + j] = (uint8_t)req;
            }
            n_rej += (uint32_t)__popcll(__ballot(cyc));
            valid = valid && !cyc;
            k0 += 64;
        } else {
            const uint32_t want = itail;
            if (!spin(&ictl[0], [want](uint32_t h) { return h != want; }, abort_flag, a.err, a.spin_ticks, st_spin_in)) break;
#ifdef FP_PIPE_STATS
            tl_avail = STAT_CLK();
#endif
            const uint32_t slot = itail % R;
            const uint32_t n = __builtin_amdgcn_readfirstlane(ictl[2 + slot]);
            if (n & END) break;
            const uint32_t *sd = idata + (size_t)slot * NF * 64;
            valid = lane < n;
            if (valid) {
                cpu = sd[lane];
                mem = sd[64 + lane];
                req = sd[128 + lane];
                conf = sd[192 + lane];
                idx = sd[256 + lane];
            }
            itail++;
            lds_rel(&ictl[1], itail);
        }
        // idle flush (global link): the consumer's tail, loaded now and used after the
        // candidate loop, so its round trip overlaps this batch's work
        uint32_t tail_async = 0;
        const bool tail_issued = (gflush & 2u) && g_out && ofill != 0;
        if (tail_issued) tail_async = g_ld(gout_head + LCTL / 2);
        // bucket indices: packed into s_idx by k_gather_sorted (one binary search per container
        // instead of one per container and stage), else searched here
        uint32_t kc, km;
        if (a.kpack) {
            kc = (idx >> 21) & (uint32_t)(K - 1);
            km = (idx >> 26) & (uint32_t)(K - 1);
        } else {
            kc = bucket_of(cpu, my_t, 0);
            km = bucket_of(mem, my_t, K);
        }
        if (prio == 2u) __builtin_amdgcn_s_setprio(FP_PRIO_LEVEL);  // the batch's work
        ck_b = STAT_CLK(); ck_in += ck_b - ck_a; ck_a = ck_b;
#ifdef FP_PIPE_STATS
        if (!sp_first) sp_first = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef FP_PIPE_STATS
        const unsigned long long ck_t0_batch = ck_b;
#endif

        // Lane-parallel candidate groups, a superset of the feasible groups (masks
        // only lose bits).  Two filters are ANDed:
        //  * per-container bucket masks B_cpu[g][kc] & B_mem[g][km];
        //  * an exact 2-D "corner" mask of the batch:
        //    E[g] = {l : cpu_free >= min cpu && mem_free >= min mem} (unschedulable
        //    records are zero, so they drop out unless a demand is zero).
        //    FFD order makes a batch's cpu range narrow, so the corner is tight in
        //    cpu.  One corner per 64-container batch ran the config-4 bench 12% faster
        //    than one per 8 containers (1.64 vs 1.96 checks per container, but an 8x
        //    cheaper prescan on every stage a container visits).
        // the valid lanes are a prefix holding the batch in FFD order (cpu non-increasing), so the
        // smallest cpu is the last valid lane's
        const uint64_t vm = __builtin_amdgcn_ballot_w64(valid);
        const uint32_t qc = vm ? __builtin_amdgcn_readlane(cpu, 63 - __builtin_clzll(vm)) : 0xFFFFFFFFu;
        const uint32_t qm = wave_min(valid ? mem : 0xFFFFFFFFu);
        // packed demands (this batch's values are multiples of the shifts: exact)
        const uint32_t cw = PK ? pk_pack(cpu, mem, sc_c, sc_m) : 0u;
        const uint32_t qw = PK ? pk_pack(qc, qm, sc_c, sc_m) : 0u;
        // every mask load is issued before the first use (no per-group LDS round trip)
        const uint32_t oc = kc * 2, om = km * 2 + 1;
        constexpr bool prescan_skip = G > SYS_MAX_G;
        GM cand = 0;
#pragma unroll
        for (uint32_t g = 0; g < G; ++g) {
            const uint64_t e = PK ? __builtin_amdgcn_ballot_w64(pk_fits(rcf[g], qw))
                                  : (__builtin_amdgcn_ballot_w64(rcf[g] >= qc) & __builtin_amdgcn_ballot_w64(rmf[g] >= qm));
            const uint64_t *mg = Mw + (size_t)g * K * 2;
            if (prescan_skip) {
                // a group whose corner is empty fits no container of the batch: no mask loads
                // (most wide-stage batches pass through with every corner empty)
                if (e) cand |= (mg[oc] & mg[om] & e) ? GM(1) << g : GM(0);
            } else {
                cand |= (mg[oc] & mg[om] & e) ? GM(1) << g : GM(0);
            }
        }
        cand = valid ? cand : GM(0);
        const bool zero = valid && (cpu | mem | req | conf) == 0u;
        uint64_t todo = __builtin_amdgcn_ballot_w64(cand != 0 && !zero);
        uint64_t placed = 0;
        uint32_t my_assign = FP_NONE;
        if (STAT_ON) {
            st_batches++;
            st_visits += (uint32_t)__popcll(__ballot(valid));
        }
        ck_b = STAT_CLK(); ck_pre += ck_b - ck_a; ck_a = ck_b;
#ifdef FP_PIPE_STATS
        const unsigned long long tl_pre = ck_b;
        const uint32_t tl_checks0 = st_checks, tl_hits0 = st_hits, tl_todo = (uint32_t)__popcll(todo);
#endif
        // Exact first fit, GROUP-major.  Container t's checks must see every earlier
        // container's placement in the group being checked, and nothing else matters to
        // it: placements in other groups touch other nodes.  So instead of walking the
        // containers in order, each checking its candidate groups, the groups are walked
        // in order (a compile-time loop) and each group takes the containers that reach
        // it in container order: group g's queue is every todo lane whose next candidate
        // group is g.  A container that finds no feasible node in g moves on to its next
        // candidate group, which is > g and so still to come.  Every container sees group
        // g after exactly the earlier containers that reached g -- the sequential first
        // fit, bit for bit -- and every record access has a static register index (no
        // s_set_gpr_idx windows, no indexed copies).
        {
            uint32_t nxt = ((todo >> lane) & 1ull) ? (cand ? (uint32_t)__builtin_ctzll((uint64_t)cand) : G) : G;
            // the hand-scheduled loop of fp_pipe_asm.h, one asm block per (static) group;
            // one-group stages leave their bucket masks at the tile's start state (still
            // exact: a stale mask is a superset): config 3 (1 x 1M x 100k) ran 127 -> 104 ms
            // without the update, while config 4's 20-group stages need it (57 vs 66 ms)
            uint32_t nchk = 0, nhit = 0;
            unsigned long long gst[4] = {0, 0, 0, 0};  // diagnostics: check-loop / bookkeeping cycles, queues, touched
            if (prio == 1u && todo) __builtin_amdgcn_s_setprio(FP_PRIO_LEVEL);
            if (todo)
                fpp_groups<G, (G > 1) && FPP_MASK_UPKEEP, (BLK == 64 || (FPP_IB1024 && G > SYS_MAX_G)) && FPP_IB, PK>(std::make_integer_sequence<uint32_t, G>{}, nxt, placed, my_assign, usedbits,
                                       used_hi, rcf, rmf, rcu, rlab, cpu, mem, req, conf, (uint32_t)cand,
                                       (uint32_t)((uint64_t)cand >> 32), my_t, lane, Mw, mlane,
                                       __builtin_amdgcn_readfirstlane(gbase * 64u), qc, qm, nchk, nhit, a.sys, gst,
                                       cw, qw, sc_c, sc_m);
            if (prio == 1u && todo) __builtin_amdgcn_s_setprio(0);
            if (STAT_ON) { st_checks += nchk; st_hits += nhit; }
            if (STAT_FINE) { ck_gx += gst[0]; ck_gu += gst[1]; st_queues += (uint32_t)gst[2]; st_touched += (uint32_t)gst[3]; }
        }
        if (zs_g < G) {
            // all-zero containers change no record: each takes the first schedulable node
            const uint64_t zm = __builtin_amdgcn_ballot_w64(zero);
            if (zm) {
                placed |= zm;
                my_assign = zero ? (gbase + zs_g) * 64 + zs_l : my_assign;
                if (zs_g < 32) usedbits |= lane == zs_l ? (1u << zs_g) : 0u;
                else used_hi |= lane == zs_l ? (1u << (zs_g & 31)) : 0u;
            }
        }
        ck_b = STAT_CLK(); ck_cand += ck_b - ck_a; ck_a = ck_b;
#ifdef FP_PIPE_STATS
        const unsigned long long tl_cand = ck_b;
        const uint32_t tl_idx = st_batches - 1;
#endif
        // a placed container's reason is OK by definition: k_unsort derives it from the assignment, so
        // the pipeline stores only the node (reasons are written for the unplaced: CYCLE / screened
        // NOFIT in segment 0, NOFIT at the last stage)
        if ((placed >> lane) & 1ull) a.assign[cb + (idx & pmask)] = my_assign;
#ifdef FP_PIPE_STATS
        if (s == 0 && lane == 0 && tl_idx < (uint32_t)TL_B && b * W + w < 16) {
            // global stage b * W + w; per batch (s_memtime): [0] loop top (= the previous batch's end)
            // [1] input available [2] input read [3] prescan end [4] group loop end, then [5] checks
            // [6] hits [7] todo | valid << 32
            unsigned long long *tl = &g_pipe_tl[((size_t)(b * W + w) * TL_B + tl_idx) * 8];
            tl[0] = tl_top; tl[1] = tl_avail; tl[2] = ck_t0_batch; tl[3] = tl_pre; tl[4] = tl_cand;
            tl[5] = st_checks - tl_checks0; tl[6] = st_hits - tl_hits0;
            tl[7] = tl_todo | ((unsigned long long)__popcll(vm) << 32);
        }
#endif
        const bool fwd = valid && !((placed >> lane) & 1ull);
        // Idle flush: a partial output slot normally waits until 64 containers fill it.  While
        // the consumer is idle (it has taken every published slot) that wait is pure latency
        // on the FFD chain -- the first containers a filling stage rejects are exactly what the
        // next stage needs to start its own fill -- so the partial slot is published at once.
        if (g_out) {
            // append to the open global slot; publish each full slot (never blocks)
            const uint64_t fm = __builtin_amdgcn_ballot_w64(fwd);
            const uint32_t f = (uint32_t)__popcll(fm);
            if (f) {
                const uint32_t pos = ofill + fpp_rank(fm);
                // slots ohead and ohead + 1 must be free (wave-uniform; bounded links only)
                if (gbounded &&
                    !gring_wait(gout_head + LCTL / 2, ohead + 2, gslots, otail_seen, a, abort_flag, lane, st_spin_out)) {
                    alive = false;
                    break;
                }
                if (fwd) {
                    uint32_t *sd = gout_data + (size_t)GSLOT(ohead + (pos >= 64 ? 1 : 0)) * LSLOT;
                    g_st(sd + 64 + (pos & 63u), idx);
                }
                if (ofill + f >= 64) {
                    if (lane == 0) g_st(gout_data + (size_t)GSLOT(ohead) * LSLOT, 64u);
                    ohead++;
                    if (unbounded_only ? (ohead & a.pub_mask) == 0 : ++opend >= a.publish) {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        if (lane == 0) g_st(gout_head, ohead);
                        opend = 0;
                    }
                    ofill = ofill + f - 64;
                } else {
                    ofill += f;
                }
            }
            // the consumer publishes slot j's index when it takes slot j (tail lags by one)
            if (tail_issued && ofill && __builtin_amdgcn_readfirstlane(tail_async) + 1u >= ohead) {
                if (lane == 0) g_st(gout_data + (size_t)GSLOT(ohead) * LSLOT, ofill);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                ohead++;
                if (lane == 0) g_st(gout_head, ohead);
                ofill = 0;
                opend = 0;
            }
            if (STAT_FINE) { ck_b = STAT_GCLK(); ck_fwd += ck_b - ck_a; }
            continue;
        }
        if (!has_out) {
            if (fwd) {
                a.assign[cb + (idx & pmask)] = FP_NONE;
                a.reason[cb + (idx & pmask)] = FP_REASON_NOFIT;
            }
            n_rej += (uint32_t)__popcll(__ballot(fwd));
            continue;
        }
        const uint64_t fm = __ballot(fwd);
        const uint32_t f = (uint32_t)__popcll(fm);
        if (f) {
            const uint32_t pos = ofill + fpp_rank(fm);
            uint32_t *od = odata + (size_t)(ohead % R) * NF * 64;
            if (fwd && pos < 64) {
                od[pos] = cpu; od[64 + pos] = mem; od[128 + pos] = req; od[192 + pos] = conf; od[256 + pos] = idx;
            }
            if (ofill + f >= 64) {
                octl[2 + ohead % R] = 64;
                ohead++;
                lds_rel(&octl[0], ohead);
                const uint32_t h = ohead;
                ck_b = STAT_CLK(); ck_fwd += ck_b - ck_a; ck_a = ck_b;
                if (!spin(&octl[1], [h, R](uint32_t tl) { return h - tl < R; }, abort_flag, a.err, a.spin_ticks, st_spin_out)) {
                    alive = false;
                    break;
                }
                ck_b = STAT_CLK(); ck_wait += ck_b - ck_a; ck_a = ck_b;
                od = odata + (size_t)(ohead % R) * NF * 64;
                if (fwd && pos >= 64) {
                    const uint32_t p = pos - 64;
                    od[p] = cpu; od[64 + p] = mem; od[128 + p] = req; od[192 + p] = conf; od[256 + p] = idx;
                }
                ofill = ofill + f - 64;
            } else {
                ofill += f;
            }
        }
        // idle flush (see the global link above): the consumer has taken every published slot
        if ((gflush & 1u) && ofill && lds_acq(&octl[1]) == ohead) {
            octl[2 + ohead % R] = ofill;
            ohead++;
            lds_rel(&octl[0], ohead);
            const uint32_t h = ohead;
            if (!spin(&octl[1], [h, R](uint32_t tl) { return h - tl < R; }, abort_flag, a.err, a.spin_ticks, st_spin_out)) {
                alive = false;
                break;
            }
            ofill = 0;
        }
    }

#ifdef FP_PIPE_STATS
    if (s == 0 && lane == 0 && b * W + w < (uint32_t)SPAN_MAX) {
        unsigned long long *sp = &g_stage_span[(size_t)(b * W + w) * 8];
        sp[0] = sp_start; sp[1] = sp_first; sp[2] = __builtin_amdgcn_s_memrealtime();
        sp[3] = ck_pre + ck_cand; sp[4] = st_batches; sp[5] = ck_wait; sp[6] = st_spin_in; sp[7] = st_hits;
    }
#endif
    // ---- flush + end of stream ----
    if (g_out && !lds_acq(abort_flag) &&
        (!gbounded || gring_wait(gout_head + LCTL / 2, ohead + 2, gslots, otail_seen, a, abort_flag, lane, st_spin_out))) {
        if (ofill) {
            if (lane == 0) g_st(gout_data + (size_t)GSLOT(ohead) * LSLOT, ofill);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            ohead++;
            if (lane == 0) g_st(gout_head, ohead);
        }
        if (lane == 0) g_st(gout_data + (size_t)GSLOT(ohead) * LSLOT, END);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ohead++;
        if (lane == 0) g_st(gout_head, ohead);
    }
    if (has_out && !lds_acq(abort_flag)) {
        bool ok = true;
        if (ofill) {
            octl[2 + ohead % R] = ofill;
            ohead++;
            lds_rel(&octl[0], ohead);
            const uint32_t h = ohead;
            ok = spin(&octl[1], [h, R](uint32_t tl) { return h - tl < R; }, abort_flag, a.err, a.spin_ticks, st_spin_out);
        }
        if (ok) {
            octl[2 + ohead % R] = END;
            ohead++;
            lds_rel(&octl[0], ohead);
        }
    }
    if (G == 1) {
        // one-group stages: the systolic fill does not track the nodes it placed on; a placement of a
        // container with nonzero cpu, mem or conf changes its node's record (capacity only shrinks,
        // and a conflict bit must be new to fit); all-zero containers set usedbits above and
        // label-only ones (only req nonzero) are marked by fpp_group_sys
        const uint32_t n = gbase * 64 + lane;
        if (n < N && (schedbits & 1u) &&
            ((PK ? (a.cf[nb + n] != pk_cpu(rcf[0], sc_c) || a.mf[nb + n] != pk_mem(rcf[0], sc_m))
                 : (a.cf[nb + n] != rcf[0] || a.mf[nb + n] != rmf[0])) ||
             a.cu[nb + n] != rcu[0]))
            usedbits |= 1u;
    }
    {  // nodes of this stage that received a container
        uint32_t u = (uint32_t)__popc(usedbits) + (uint32_t)__popc(used_hi);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) u += (uint32_t)__shfl_xor((int)u, o);
        n_used = u;
    }
    if (lane == 0) {
        // stats slot: global stage b * W + w when the scenario has at most 16, else w
        const uint32_t st_slot = (B * W <= 16u) ? b * W + w : w;
        (void)st_slot;
        atomicAdd(&CNT[0], n_used);
        atomicAdd(&CNT[1], n_rej);
        STAT_ADD(st_slot, 0, st_visits); STAT_ADD(st_slot, 1, st_checks); STAT_ADD(st_slot, 2, st_hits);
        STAT_ADD(st_slot, 3, st_batches); STAT_ADD(st_slot, 4, st_spin_in); STAT_ADD(st_slot, 5, st_spin_out);
        STAT_ADD(st_slot, 8, ck_in); STAT_ADD(st_slot, 9, ck_pre); STAT_ADD(st_slot, 10, ck_cand); STAT_ADD(st_slot, 11, ck_fwd);
        STAT_ADD(st_slot, 12, ck_wait); STAT_ADD(st_slot, 13, STAT_CLK() - ck_t0);
        STAT_ADD(st_slot, 6, ck_gx); STAT_ADD(st_slot, 7, ck_gu); STAT_ADD(st_slot, 14, st_queues);
        STAT_ADD(st_slot, 15, st_touched);
    }
    (void)ck_t0; (void)ck_in; (void)ck_pre; (void)ck_cand; (void)ck_fwd; (void)ck_wait; (void)ck_gx; (void)ck_gu;
    (void)st_queues; (void)st_touched;
    (void)st_spin_in; (void)st_spin_out; (void)st_visits; (void)st_checks; (void)st_hits; (void)st_batches;
#undef GSLOT
    // write the tile's node state back (registers -> HBM)
#pragma unroll
    for (uint32_t g = 0; g < G; ++g) {
        const uint32_t n = (gbase + g) * 64 + lane;
        if (n < N && ((schedbits >> g) & 1u)) {  // unschedulable records were never loaded
            a.cf[nb + n] = PK ? pk_cpu(rcf[g], sc_c) : rcf[g];
            a.mf[nb + n] = PK ? pk_mem(rcf[g], sc_m) : rmf[g];
            a.cu[nb + n] = rcu[g];
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        a.part[((size_t)s * B + b) * 2] = CNT[0];
        a.part[((size_t)s * B + b) * 2 + 1] = CNT[1];
    }
}

// cost[s] from the per-segment partial counts (SPEC.md 2.4)
__global__ void k_cost_reduce(uint32_t S, uint32_t B, uint32_t scen_base, const uint32_t *__restrict__ part,
                              uint64_t *__restrict__ cost) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    uint32_t used = 0, rej = 0;
    for (uint32_t b = 0; b < B; ++b) {
        used += part[((size_t)s * B + b) * 2];
        rej += part[((size_t)s * B + b) * 2 + 1];
    }
    cost[s] = fpd::pack_cost(rej, used, scen_base + s);
}

// Sorted SoA for the pipeline.  cpu and mem come back out of the sorted radix keys
// (key = [scenario] << kbits | (cmax - c) << mbits | (mmax - m), coalesced; the scenario
// field, if any, is masked off; c/m are the values, or their dense ranks decoded through
// the value tables cval/mval), so only req, conf and level are gathered at random;
// without keys (all-zero or all-equal demands) everything is.
// The buckets of both demands (one binary search over the thresholds, in LDS) ride in the
// position word when positions fit 21 bits (PipeArgs::kpack).
// ---- stage 2 on the pristine node table, as an exact early NOFIT screen ----
// Per scenario, the feasibility sweep (SPEC.md 2.3) against one summary record that dominates
// every schedulable node: the union of their labels and the intersection of their used
// conflict bits.  A container whose required labels are outside the union, or whose conflict
// bits every node has already used, has no feasible node now (feasible count 0, fp_feasibility)
// and none later (capacity and free conflicts only shrink, SPEC.md 2.3 monotonicity): it is
// NOFIT without entering the pipeline, exactly as the sequential first fit would reject it at
// the last node.  In the synthetic configs 3 and 4 that is every container requiring one of the
// 19 label bits no node carries (~18 %): each of them used to walk every segment.
// RANGE: the same pass also ORs the schedulable nodes' free cpu / mem into rng[0] / rng[1] (the
// packed-capacity decision, fp_pipe_pk.h; one atomic per block and word).  !SUMM: that alone.
template <bool SUMM, bool RANGE>
__global__ __launch_bounds__(256) void k_node_summary(uint32_t N, const uint32_t *__restrict__ cf,
                                                      const uint32_t *__restrict__ mf, const uint32_t *__restrict__ lab,
                                                      const uint32_t *__restrict__ cu,
                                                      const uint8_t *__restrict__ sched, uint32_t *__restrict__ summ,
                                                      uint32_t *__restrict__ rng) {
    const size_t nb = (size_t)blockIdx.x * N;
    uint32_t u = 0, a = 0xFFFFFFFFu, oc = 0, om = 0;
    // NS_U nodes per thread in flight (one block per scenario: a single load triple per thread at
    // a time left the pass latency-bound, 0.23 ms for config 4's 4096 x 5k nodes)
    constexpr uint32_t NS_U = 4;
    for (uint32_t n0 = threadIdx.x; n0 < N; n0 += NS_U * blockDim.x) {
        uint32_t l[NS_U], c[NS_U], x[NS_U], y[NS_U];
        uint8_t sc[NS_U];
#pragma unroll
        for (uint32_t k = 0; k < NS_U; ++k) {
            const uint32_t n = n0 + k * blockDim.x;
            sc[k] = n < N ? sched[nb + n] : 0;
            if (SUMM) {
                l[k] = n < N ? lab[nb + n] : 0u;
                c[k] = n < N ? cu[nb + n] : 0xFFFFFFFFu;
            }
            if (RANGE) {
                x[k] = n < N ? cf[nb + n] : 0u;
                y[k] = n < N ? mf[nb + n] : 0u;
            }
        }
#pragma unroll
        for (uint32_t k = 0; k < NS_U; ++k) {
            if (sc[k]) {
                if (SUMM) {
                    u |= l[k];
                    a &= c[k];
                }
                if (RANGE) {
                    oc |= x[k];
                    om |= y[k];
                }
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        u |= (uint32_t)__shfl_xor((int)u, o);
        a &= (uint32_t)__shfl_xor((int)a, o);
        oc |= (uint32_t)__shfl_xor((int)oc, o);
        om |= (uint32_t)__shfl_xor((int)om, o);
    }
    __shared__ uint32_t red[4][4];
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[0][w] = u; red[1][w] = a; red[2][w] = oc; red[3][w] = om; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint32_t q = 1; q < blockDim.x / 64; ++q) { u |= red[0][q]; a &= red[1][q]; oc |= red[2][q]; om |= red[3][q]; }
        if (SUMM) {
            summ[(size_t)blockIdx.x * 4] = u;
            summ[(size_t)blockIdx.x * 4 + 1] = a;
        }
        if (RANGE) {
            fp_or_new_bits(&rng[0], oc);
            fp_or_new_bits(&rng[1], om);
        }
    }
}

__device__ __forceinline__ bool screened(const uint32_t *sm, uint32_t req, uint32_t conf) {
    return ((req & ~sm[0]) | (conf & sm[1])) != 0u;
}

// bucket thresholds for k_gather_sorted: thr [0, K) cpu, [K, 2K) mem (device), kpack as PipeArgs
template <class KeyT>
__global__ void k_gather_sorted(const uint32_t *__restrict__ thr, uint32_t kpack, uint32_t S, uint32_t C,
                                const uint32_t *__restrict__ order,
                                const KeyT *__restrict__ skeys, uint32_t mbits, uint64_t cmax, uint64_t mmax,
                                const uint32_t *__restrict__ cval, const uint32_t *__restrict__ mval,
                                const uint32_t *__restrict__ cpu, const uint32_t *__restrict__ mem,
                                const uint32_t *__restrict__ req, const uint32_t *__restrict__ conf,
                                const uint32_t *__restrict__ level, const uint32_t *__restrict__ summ,
                                uint32_t *__restrict__ s_cpu, uint32_t *__restrict__ s_mem,
                                uint32_t *__restrict__ s_req, uint32_t *__restrict__ s_conf,
                                uint32_t *__restrict__ s_idx) {
    // S * C < 2^32 (fp_dev_place_batch_impl checks): 32-bit index arithmetic, and four
    // independent elements per thread in flight (the req/conf gathers are dependent loads)
    const uint32_t total = S * C;
    // one tile of 4 x blockDim contiguous elements per block; blocks b and b + 8 share an XCD, so
    // the XCD-contiguous tile order below keeps each XCD's running blocks inside ~5 config-4
    // scenarios at a time (their random req/conf/level lines fit its 4 MB L2)
    const uint32_t lb = (gridDim.x & 7u) ? blockIdx.x : (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    const uint32_t stride = blockDim.x;
    __shared__ uint32_t T[2 * K];
    if (threadIdx.x < 2 * K) T[threadIdx.x] = thr[threadIdx.x];
    __syncthreads();
    // largest k with T[k] <= v (T ascending, T[0] = 0)
    auto bucket = [](const uint32_t *t, uint32_t v) {
        uint32_t k = 0;
#pragma unroll
        for (uint32_t step = K / 2; step; step >>= 1) k += t[k + step] <= v ? step : 0u;
        return k;
    };
    {
        const size_t i0 = (size_t)lb * 4 * blockDim.x + threadIdx.x;
        uint32_t j[4], src[4], r[4], f[4], cy[4], cv[4], mv[4], pos[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const size_t i = i0 + (size_t)u * stride;
            if (i < total) j[u] = __builtin_nontemporal_load(&order[i]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const size_t i = i0 + (size_t)u * stride;
            if (i < total) {
                pos[u] = (uint32_t)i % C;                        // sorted position in the scenario
                src[u] = (uint32_t)i - pos[u] + j[u];            // i < total < 2^32
                if (skeys) {
                    const uint64_t k = __builtin_nontemporal_load(&skeys[i]);
                    cv[u] = (uint32_t)(cmax - (mbits >= 64 ? 0ull : ((k >> mbits) & cmax)));
                    mv[u] = (uint32_t)(mmax - (k & mmax));
                }
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const size_t i = i0 + (size_t)u * stride;
            if (i < total) {
                r[u] = req[src[u]];
                f[u] = conf[src[u]];
                cy[u] = (level && level[src[u]] == FP_NONE) ? CYC : 0u;
                if (cy[u]) {
                    r[u] = FP_REASON_CYCLE;
                } else if (summ && screened(summ + (size_t)((uint32_t)i / C) * 4, r[u], f[u])) {
                    cy[u] = CYC;
                    r[u] = FP_REASON_NOFIT;
                }
                if (skeys) {
                    if (cval) cv[u] = cval[cv[u]];
                    if (mval) mv[u] = mval[mv[u]];
                } else {
                    cv[u] = cpu[src[u]];
                    mv[u] = mem[src[u]];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const size_t i = i0 + (size_t)u * stride;
            if (i < total) {
                // streaming traffic bypasses L2 retention so the random req/conf lines stay
                __builtin_nontemporal_store(cv[u], &s_cpu[i]);
                __builtin_nontemporal_store(mv[u], &s_mem[i]);
                __builtin_nontemporal_store(r[u], &s_req[i]);
                __builtin_nontemporal_store(f[u], &s_conf[i]);
                // the pipeline carries the SORTED position: its assign/reason stores land
                // next to each other (k_unsort restores container order, coalesced)
                const uint32_t kb = kpack ? (bucket(T, cv[u]) << 21) | (bucket(T + K, mv[u]) << 26) : 0u;
                __builtin_nontemporal_store(pos[u] | kb | cy[u], &s_idx[i]);
            }
        }
    }
}

// The rest of the sorted SoA after k_scen_sort (fp_place.hip) wrote order, cpu, mem and the
// position word: req and conf gathered at random (same XCD-contiguous tiles as
// k_gather_sorted, so an XCD's random lines stay in its L2) and the CYCLE bit from level.
// (Interleaving req/conf in round 3's k_digits pass for one 8-byte read per container: gather
// 2.18 -> 1.68 ms, but k_digits 0.39 -> 1.05 ms.)
__global__ void k_gather_payload(uint32_t S, uint32_t C, const uint32_t *__restrict__ order,
                                 const uint32_t *__restrict__ req, const uint32_t *__restrict__ conf,
                                 const uint32_t *__restrict__ level, const uint32_t *__restrict__ summ,
                                 uint32_t *__restrict__ s_req, uint32_t *__restrict__ s_conf,
                                 uint32_t *__restrict__ s_idx) {
    const uint32_t total = S * C;
    const uint32_t lb = (gridDim.x & 7u) ? blockIdx.x : (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    const uint32_t i0 = lb * 4 * blockDim.x + threadIdx.x;
    uint32_t src[4], r[4], f[4], cy[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint32_t i = i0 + u * blockDim.x;
        if (i < total) src[u] = i - i % C + __builtin_nontemporal_load(&order[i]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint32_t i = i0 + u * blockDim.x;
        if (i < total) {
            r[u] = req[src[u]];
            f[u] = conf[src[u]];
            cy[u] = (level && level[src[u]] == FP_NONE) ? CYC : 0u;
            if (cy[u]) {
                r[u] = FP_REASON_CYCLE;
            } else if (summ && screened(summ + (size_t)(i / C) * 4, r[u], f[u])) {
                cy[u] = CYC;
                r[u] = FP_REASON_NOFIT;
            }
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint32_t i = i0 + u * blockDim.x;
        if (i < total) {
            __builtin_nontemporal_store(r[u], &s_req[i]);
            __builtin_nontemporal_store(f[u], &s_conf[i]);
            if (cy[u]) s_idx[i] |= CYC;
        }
    }
}

// The same payload as k_gather_payload with every HBM access coalesced: one workgroup per
// scenario.  Each thread owns the sorted positions t + 1024 j; per half of them (25 per thread:
// registers) it keeps their container indices, then streams the scenario's (req, conf) pairs
// through LDS in chunks of PL_CHUNK and picks its positions' values out of the chunk that holds
// them (level the same way first, for the CYCLE bits).  k_gather_payload's two random 4-B reads
// per container ran at the L2 request rate (2.2 ms for 4096 x 50k).  C <= PL_MAX_C.
constexpr uint32_t PL_THREADS = 1024, PL_H = 25, PL_MAX_C = PL_THREADS * PL_H * 2;
constexpr uint32_t PL_CHUNK = 18 * 1024;  // (req, conf) pairs: 144 KB of LDS
__global__ __launch_bounds__(1024) void k_payload_lds(uint32_t C, const uint32_t *__restrict__ order,
                                                      const uint32_t *__restrict__ req,
                                                      const uint32_t *__restrict__ conf,
                                                      const uint32_t *__restrict__ level,
                                                      const uint32_t *__restrict__ summ,
                                                      uint32_t *__restrict__ s_req, uint32_t *__restrict__ s_conf,
                                                      uint32_t *__restrict__ s_idx) {
    extern __shared__ uint2 pl_lds2[];
    uint32_t *pl_lds = reinterpret_cast<uint32_t *>(pl_lds2);
    const uint32_t t = threadIdx.x;
    const size_t cb = (size_t)blockIdx.x * C;
    const uint32_t sm0 = summ ? summ[(size_t)blockIdx.x * 4] : 0xFFFFFFFFu;
    const uint32_t sm1 = summ ? summ[(size_t)blockIdx.x * 4 + 1] : 0u;
    for (uint32_t h = 0; h < 2; ++h) {
        const uint32_t pbase = h * PL_THREADS * PL_H + t;
        if (h * PL_THREADS * PL_H >= C) break;  // uniform: every thread meets the same barriers
        uint32_t o[PL_H];
#pragma unroll
        for (uint32_t j = 0; j < PL_H; ++j) {
            const uint32_t p = pbase + PL_THREADS * j;
            o[j] = p < C ? __builtin_nontemporal_load(&order[cb + p]) : 0xFFFFFFFFu;
        }
        uint32_t vr[PL_H], vf[PL_H];
        uint32_t cy = 0;
        if (level) {
            for (uint32_t a0 = 0; a0 < C; a0 += 2 * PL_CHUNK) {
                const uint32_t n = C - a0 < 2 * PL_CHUNK ? C - a0 : 2 * PL_CHUNK;
                __syncthreads();
#pragma unroll 4
                for (uint32_t i = t; i < n; i += PL_THREADS) pl_lds[i] = __builtin_nontemporal_load(&level[cb + a0 + i]);
                __syncthreads();
#pragma unroll
                for (uint32_t j = 0; j < PL_H; ++j) {
                    const uint32_t d = o[j] - a0;
                    if (d < n) cy |= (uint32_t)(pl_lds[d] == FP_NONE) << j;
                }
            }
        }
        for (uint32_t a0 = 0; a0 < C; a0 += PL_CHUNK) {
            const uint32_t n = C - a0 < PL_CHUNK ? C - a0 : PL_CHUNK;
            __syncthreads();
#pragma unroll 4
            for (uint32_t i = t; i < n; i += PL_THREADS)
                pl_lds2[i] = make_uint2(__builtin_nontemporal_load(&req[cb + a0 + i]), __builtin_nontemporal_load(&conf[cb + a0 + i]));
            __syncthreads();
#pragma unroll
            for (uint32_t j = 0; j < PL_H; ++j) {
                const uint32_t d = o[j] - a0;
                if (d < n) { const uint2 x = pl_lds2[d]; vr[j] = x.x; vf[j] = x.y; }
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < PL_H; ++j) {
            const uint32_t p = pbase + PL_THREADS * j;
            if (p < C) {
                uint32_t r = vr[j];
                const bool c = (cy >> j) & 1u, x = ((r & ~sm0) | (vf[j] & sm1)) != 0u;
                if (c) r = FP_REASON_CYCLE;
                else if (summ && x) r = FP_REASON_NOFIT;
                __builtin_nontemporal_store(r, &s_req[cb + p]);
                __builtin_nontemporal_store(vf[j], &s_conf[cb + p]);
                if (c || (summ && x)) s_idx[cb + p] |= CYC;
            }
        }
    }
}

// assign/reason from FFD (sorted) order back to container order, per scenario and per
// range of container indices held in LDS: every read and write is coalesced.  The
// pipeline's stores hit the sorted arrays at positions that advance together, so its
// partial lines merge in L2 instead of costing a 64-byte write each (round 1 wrote the
// container-order arrays directly: 2.2 GB of WRITE_SIZE per 512-scenario launch for
// 0.13 GB of outputs).
// LDS holds a range of container indices per workgroup: 3 B per container (u16 node index,
// u8 reason) when every node index fits 16 bits (N < 65535: one workgroup covers a config-4
// scenario), 5 B otherwise.
constexpr uint32_t UNSORT_SPAN16 = 50 * 1024;  // 150 KB of LDS
constexpr uint32_t UNSORT_SPAN32 = 30 * 1024;  // 150 KB of LDS
template <bool NARROW>
__global__ __launch_bounds__(1024) void k_unsort(uint32_t C, uint32_t H, uint32_t span,
                                                 const uint32_t *__restrict__ order,
                                                 const uint32_t *__restrict__ asg_s, const uint8_t *__restrict__ rsn_s,
                                                 uint32_t *__restrict__ assign, uint8_t *__restrict__ reason) {
    using A = typename std::conditional<NARROW, uint16_t, uint32_t>::type;
    extern __shared__ __attribute__((aligned(16))) unsigned char ulds[];
    A *la = reinterpret_cast<A *>(ulds);
    uint8_t *lr = ulds + (size_t)span * sizeof(A);
    const uint32_t s = blockIdx.x / H, h = blockIdx.x % H;
    const uint32_t lo = h * span, hi = min(C, lo + span);
    const size_t cb = (size_t)s * C;
    constexpr uint32_t U = 8;  // loads in flight per thread
    for (uint32_t p0 = threadIdx.x; p0 < C; p0 += blockDim.x * U) {
        uint32_t j[U], av[U];
        uint8_t rv[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t p = p0 + u * blockDim.x;
            j[u] = p < C ? __builtin_nontemporal_load(&order[cb + p]) : 0xFFFFFFFFu;
            av[u] = p < C ? __builtin_nontemporal_load(&asg_s[cb + p]) : 0u;
            rv[u] = p < C ? __builtin_nontemporal_load(&rsn_s[cb + p]) : 0;
        }
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            if (j[u] >= lo && j[u] < hi) {
                la[j[u] - lo] = (A)av[u];  // FP_NONE -> 0xFFFF when narrow
                // placed: OK (the pipeline writes no reason for a placed container)
                lr[j[u] - lo] = av[u] != FP_NONE ? (uint8_t)FP_REASON_OK : rv[u];
            }
        }
    }
    __syncthreads();
    for (uint32_t j = lo + threadIdx.x; j < hi; j += blockDim.x) {
        const A v = la[j - lo];
        __builtin_nontemporal_store(NARROW && v == (A)0xFFFF ? FP_NONE : (uint32_t)v, &assign[cb + j]);
        reason[cb + j] = lr[j - lo];
    }
}

size_t lds_bytes(uint32_t W, uint32_t G, uint32_t R) {
    return (size_t)W * G * K * 16 + ((size_t)(W - 1) * 8 + 8) * 4 + (size_t)(W - 1) * R * NF * 64 * 4;
}

// G is a template parameter (records are register arrays); one instantiation per G
template <uint32_t G, uint32_t BLK = 1024, uint32_t WV = 0, bool PK = false>
static int launch_g(hipStream_t st, unsigned grid, unsigned block, size_t lds, const PipeArgs &a) {
    if (block > BLK) return FP_EINVAL;
    FP_HIP(hipFuncSetAttribute((const void *)k_ffd_pipe<G, BLK, WV, PK>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds));
    k_ffd_pipe<G, BLK, WV, PK><<<grid, block, lds, st>>>(a);
    return FP_OK;
}

typedef int (*launch_fn)(hipStream_t, unsigned, unsigned, size_t, const PipeArgs &);
#ifndef FPP_KERNEL_TU  // (fp_pipe_tu.hip compiles one kernel of fp_pipe_tus.h, below)
// The kernels of fp_pipe_tus.h: with FPP_SPLIT each lives in its own translation unit (fp_pipe_tu.hip,
// the Makefile's FFD_TUS: each under its own LLVM machine scheduler) and is reached through its
// launcher; without (the one-TU diagnostics build) they are instantiated here.
struct TuKernel {
    uint32_t G, BLK, WV, PK;
    launch_fn launch;
    const void *(*kernel)();
};
static_assert(WIDE12_BIG_WAVES == 6, "fp_pipe_tus.h names the six-wave 4096-scenario kernel");
#ifdef FPP_SPLIT
}  // namespace fpp
#define FPP_TU_DECL(name, G, BLK, WV, PK)                                                    \
    int fpp_tu_launch_##name(hipStream_t, unsigned, unsigned, size_t, const void *);         \
    const void *fpp_tu_kernel_##name();
FPP_TUS(FPP_TU_DECL)
#undef FPP_TU_DECL
namespace fpp {
#define FPP_TU_ENTRY(name, G, BLK, WV, PK)                                                                     \
    {G, BLK, WV, PK,                                                                                           \
     [](hipStream_t st, unsigned gr, unsigned bl, size_t l, const PipeArgs &a) {                                \
         return ::fpp_tu_launch_##name(st, gr, bl, l, &a);                                                    \
     },                                                                                                        \
     ::fpp_tu_kernel_##name},
#else
#define FPP_TU_ENTRY(name, G, BLK, WV, PK) \
    {G, BLK, WV, PK, launch_g<G, BLK, WV, (bool)PK>, [] { return (const void *)k_ffd_pipe<G, BLK, WV, (bool)PK>; }},
#endif
static const TuKernel kTu[] = {FPP_TUS(FPP_TU_ENTRY)};
#undef FPP_TU_ENTRY
// (G, BLK, WV) has a u32 kernel in kTu: the tables below leave it out
constexpr bool in_tu(uint32_t G, uint32_t BLK, uint32_t WV) {
#define FPP_TU_IS(name, g, blk, wv, pk) || ((g) == G && (blk) == BLK && (wv) == WV && !(pk))
    return false FPP_TUS(FPP_TU_IS);
#undef FPP_TU_IS
}
static const TuKernel *tu_find(uint32_t G, uint32_t BLK, uint32_t WV, bool PK) {
    for (const TuKernel &k : kTu)
        if (k.G == G && k.BLK == BLK && k.WV == WV && (k.PK != 0) == PK) return &k;
    return nullptr;
}
template <uint32_t G, uint32_t BLK = 1024, uint32_t WV = 0>
static constexpr launch_fn main_launch() {
    if constexpr (in_tu(G, BLK, WV)) return nullptr;
    else return launch_g<G, BLK, WV>;
}
template <uint32_t G, uint32_t BLK = 1024, uint32_t WV = 0>
static inline const void *main_kernel() {
    if constexpr (in_tu(G, BLK, WV)) return nullptr;
    else return (const void *)k_ffd_pipe<G, BLK, WV>;
}
// the u32 kernels not in kTu, by G: 1024-thread (multi-stage) and one-wave (wide) segments
static const launch_fn kLaunch[MAX_G + 1] = {
    nullptr,           main_launch<1>(),  main_launch<2>(),  main_launch<3>(),  main_launch<4>(),
    main_launch<5>(),  main_launch<6>(),  main_launch<7>(),  main_launch<8>(),  main_launch<9>(),
    main_launch<10>(), main_launch<11>(), main_launch<12>(), main_launch<13>(), main_launch<14>(),
    main_launch<15>(), main_launch<16>()};
static const void *const kKernel[MAX_G + 1] = {
    nullptr,           main_kernel<1>(),  main_kernel<2>(),  main_kernel<3>(),  main_kernel<4>(),
    main_kernel<5>(),  main_kernel<6>(),  main_kernel<7>(),  main_kernel<8>(),  main_kernel<9>(),
    main_kernel<10>(), main_kernel<11>(), main_kernel<12>(), main_kernel<13>(), main_kernel<14>(),
    main_kernel<15>(), main_kernel<16>()};
// one-wave segments (W = 1) of 13..40 groups: G rounded up to a multiple of 4 (the padding
// groups hold unschedulable records, which no container fits)
constexpr uint32_t MAX_G_WIDE = 40;
static const launch_fn kLaunchWide[MAX_G_WIDE / 4 + 1] = {
    nullptr, nullptr, nullptr, main_launch<12, 64>(), main_launch<16, 64>(), main_launch<20, 64>(),
    main_launch<24, 64>(), main_launch<28, 64>(), main_launch<32, 64>(), main_launch<36, 64>(), main_launch<40, 64>()};
static const void *const kKernelWide[MAX_G_WIDE / 4 + 1] = {
    nullptr, nullptr, nullptr, main_kernel<12, 64>(), main_kernel<16, 64>(), main_kernel<20, 64>(),
    main_kernel<24, 64>(), main_kernel<28, 64>(), main_kernel<32, 64>(), main_kernel<36, 64>(), main_kernel<40, 64>()};
static inline bool wide_g(uint32_t W, uint32_t G) { return W == 1 && G >= 12; }
// the six-wave 12-group instantiation (WIDE12_BIG_S)
static inline bool wide12_big(uint32_t S, uint32_t W, uint32_t G) { return W == 1 && G == 12 && S >= WIDE12_BIG_S; }
// The kernel of a geometry (PK: the packed one, if compiled; else null).  big: the six-wave
// 12-group kernel (fp_pipe_launch takes it only with unbounded links).
static void pipe_kernel(uint32_t G, uint32_t W, bool big, bool PK, launch_fn *l, const void **k) {
    const bool wide = wide_g(W, G);
    const uint32_t BLK = wide ? 64u : 1024u, WV = big ? WIDE12_BIG_WAVES : 0u;
    *l = nullptr;
    *k = nullptr;
    if (const TuKernel *t = tu_find(G, BLK, WV, PK)) {
        *l = t->launch;
        *k = t->kernel();
        return;
    }
    if (PK || big) return;
    if (wide) {
        if (G % 4 == 0 && G / 4 < sizeof(kLaunchWide) / sizeof(kLaunchWide[0])) {
            *l = kLaunchWide[G / 4];
            *k = kKernelWide[G / 4];
        }
    } else if (G < sizeof(kLaunch) / sizeof(kLaunch[0])) {
        *l = kLaunch[G];
        *k = kKernel[G];
    }
}
#endif  // !FPP_KERNEL_TU

}  // namespace fpp

#ifdef FPP_KERNEL_TU
// this translation unit's one kernel and its launcher (fp_pipe_tu.hip renames the namespace)
#define FPP_TU_CAT2(a, b) a##b
#define FPP_TU_CAT(a, b) FPP_TU_CAT2(a, b)
int FPP_TU_CAT(fpp_tu_launch_, FPP_TU_NAME)(hipStream_t st, unsigned grid, unsigned block, size_t lds, const void *args) {
    return fpp::launch_g<FPP_TU_G, FPP_TU_BLK, FPP_TU_WV, (bool)FPP_TU_PK>(st, grid, block, lds,
                                                                          *static_cast<const fpp::PipeArgs *>(args));
}
const void *FPP_TU_CAT(fpp_tu_kernel_, FPP_TU_NAME)() {
    return (const void *)fpp::k_ffd_pipe<FPP_TU_G, FPP_TU_BLK, FPP_TU_WV, (bool)FPP_TU_PK>;
}
#endif

#ifndef FPP_KERNEL_TU

using namespace fpp;

// Pipeline geometry for N nodes: W waves (stages) of G groups per workgroup
// (segment) and B segments per scenario.  One segment holds at most
// MAX_SEG_GROUPS groups: 4 stages x 10 groups (20 KB of masks + rings).  Measured
// on the config-4 bench (512 x 50k x 5k): 2 segments of 4 stages ran 16.0 ms, one
// segment of 8 stages 17.1 ms, 4 x 2 16.7 ms, 8 x 1 17.1 ms -- the unbounded
// global link decouples the halves better than a 2-4 slot LDS ring, and more
// than ~4 segments adds link latency to the FFD chain.
constexpr uint32_t MAX_SEG_GROUPS = 40;
constexpr size_t LDS_HALF_CU = 80 * 1024;
// S x groups at or below which stages hold one group.  Config 3 (1 x 1M x 100k, 1563
// groups): 160 ms with one-group stages vs 181 ms with 10-group stages (hand-scheduled loop).
constexpr uint64_t kNarrowWaves = 4096;

bool fp_pipe_plan(const fp_ctx *c, uint32_t S, uint32_t N, uint32_t *G_out, uint32_t *W_out, uint32_t *B_out,
                  size_t *lds_out) {
    const uint32_t NG = (N + 63) / 64;
    const size_t cap = 160 * 1024;
    if (NG == 0) {
        *G_out = 1; *W_out = 1; *B_out = 1; *lds_out = lds_bytes(1, 1, 2);
        return true;
    }
    // FP_OPT_PIPE_W / FP_OPT_PIPE_SEG: force the stage count / groups per segment (tuning
    // experiments and tests)
    const int forced_w = (int)fp_opt(c, FP_OPT_PIPE_W, 0);
    const int forced_seg = (int)fp_opt(c, FP_OPT_PIPE_SEG, 0);
    // Few scenarios leave the GPU idle: one group (64 nodes) per stage then shortens the
    // chain -- config 2 (1 x 10k x 1k): 2.39 ms vs 3.02 ms with 10-group stages; config 3
    // (1 x 1M x 100k): 160 ms vs 181 ms.  Many scenarios get one-wave segments of up to 40
    // groups (W = 1): the stages of a segment were busy one at a time anyway (the
    // placement frontier moves through them), so one wave does the same work in about the
    // same time while a scenario needs fewer registers than with 4-stage segments.
    const bool narrow = (uint64_t)S * NG <= kNarrowWaves;
    // one-wave segments hold at most 12 groups (96 VGPRs at five waves per SIMD, 20
    // segments in flight per CU; WIDE12_WAVES).  With lagged segment tickets (the kernel) a segment runs
    // on complete input, so more, smaller segments keep more waves busy: config 4 (79
    // groups) 7 segments of 12 groups 28.3 ms, 10 of 8 groups 28.2, 4 of 20 groups 30.3,
    // 3 of 24-28 groups 30.2.  (Without the lag, when a segment waited on its upstream
    // half its life, 4 segments of 20 groups were best: 56.7 ms vs 64.1 for 5 of 16.)
    // Round 4 (sweeps of config 4's per-GPU loads, profiles/r04p_*, r04q_*, r04ad_*): the strong-scaled
    // ranks of the 8-GPU run hold 512-1024 scenarios, where a scenario's own chain sets the time and
    // more stages per segment pay: up to 512 scenarios 2 segments of 4 stages x 10 groups (6.87 ms
    // FFD vs 7.30 for one-wave 8-group segments, 7.51 for 12), up to 1024 5 segments of 2 stages x
    // 8 groups (8.19 vs 8.46 and 8.73), above that one-wave 12-group segments (2048: 9.91 vs 10.19
    // with 8 groups; 4096: 15.2 vs 18.9 with 16).
    const bool mid4 = !narrow && S <= 512, mid2 = !narrow && !mid4 && S <= 1024;
    const uint32_t seg_groups = forced_seg > 0 && forced_seg <= (int)MAX_SEG_GROUPS ? (uint32_t)forced_seg
                                : narrow ? 4u : (forced_w > 1 || mid4) ? MAX_SEG_GROUPS : mid2 ? 16u : 12u;
    const uint32_t B = (NG + seg_groups - 1) / seg_groups;
    const uint32_t per_seg = (NG + B - 1) / B;
    const uint32_t first_w = forced_w > 0 ? (uint32_t)forced_w : narrow ? 4u : mid4 ? 4u : mid2 ? 2u : 1u;
    // a forced stage count is tried first; sizes it cannot serve fall back to the list
    for (uint32_t W : {first_w, 4u, 8u, 2u, 1u, 12u, 16u}) {
        if (W > per_seg && W > 1) continue;
        uint32_t G = (per_seg + W - 1) / W;
        if (wide_g(W, G)) {
            G = (G + 3) / 4 * 4;
            if (G > MAX_G_WIDE) continue;
        } else if (G > MAX_G) {
            continue;
        }
        const uint32_t Wn = (per_seg + G - 1) / G;  // drop empty tail stages
        const size_t lds = lds_bytes(Wn, G, 2);
        if (lds > cap) continue;
        *G_out = G; *W_out = Wn; *B_out = B; *lds_out = lds;
        return true;
    }
    return false;
}

// Launch geometry and link sizing for one fp_pipe_launch.
struct PipeGeom {
    uint32_t G, W, B, R;
    size_t lds;
    uint32_t lag;       // segment ticket lag (kernel comment)
    uint32_t slots;     // slots per global link
    uint32_t bounded;   // links are rings with back-pressure
    uint32_t resident;  // workgroups of this kernel resident on the device at once (0: unknown)
    uint32_t sys;       // systolic group fill for queues of >= sys containers (0: off)
    uint32_t sys_extra; // systolic steps past the queue length before the serial finish
    uint32_t prio;      // wave priority mode (PipeArgs::prio)
};

// Per-device gate of bounded launches (fp_pipe_launch): the event the last bounded launch on the
// device recorded on its stream, and the lock that orders the wait / launch / record of each.
struct BoundedGate {
    std::mutex m;
    hipEvent_t ev = nullptr;
};
constexpr int kMaxGateDevices = 64;
static BoundedGate g_bounded_gate[kMaxGateDevices];

// Global link ring size when every segment of the launch is co-resident: 256 slots x 64
// containers in flight per link (128 KB).  FP_OPT_LINK_SLOTS overrides (>= 8; tests force
// small rings to exercise back-pressure).
constexpr uint32_t LINK_RING_SLOTS = 256;

static bool pipe_geom(fp_ctx *c, uint32_t S, uint32_t C, uint32_t N, PipeGeom *g) {
    if (!fp_pipe_plan(c, S, N, &g->G, &g->W, &g->B, &g->lds)) return false;
    const uint32_t G = g->G, W = g->W, B = g->B;
    // deepest ring (2..4 slots) that keeps two workgroups per CU (else one)
    uint32_t R = 2;
    for (uint32_t r = 4; r > 2; --r)
        if (lds_bytes(W, G, r) <= LDS_HALF_CU) { R = r; break; }
    // FP_OPT_PIPE_R: force the ring depth, 2..6 (a link's control block holds 6 slot counts)
    {
        const int64_t fr = fp_opt(c, FP_OPT_PIPE_R, 0);
        if (fr >= 2 && fr <= 6 && lds_bytes(W, G, (uint32_t)fr) <= 160 * 1024) R = (uint32_t)fr;
    }
    g->R = R;
    g->lds = lds_bytes(W, G, R);
    // resident segments on this device (0 if unknown)
    // (the kernel fp_pipe_launch will run: the six-wave one only with unbounded links)
    // (and of its packed twin when there is one: the smaller of the two, either may run the batch)
    auto resident_of = [&](bool big) -> uint64_t {
        int dev_cu = 0;
        (void)hipDeviceGetAttribute(&dev_cu, hipDeviceAttributeMultiprocessorCount, c->device);
        uint64_t res = 0;
        for (const bool pk : {false, true}) {
            launch_fn l;
            const void *fn;
            pipe_kernel(G, W, big, pk, &l, &fn);
            int occ = 0;
            if (!fn) continue;
            if (dev_cu <= 0 || hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, (int)(W * 64), g->lds) != hipSuccess ||
                occ <= 0)
                return 0;
            const uint64_t r = (uint64_t)occ * (uint64_t)dev_cu;
            res = res && res < r ? res : r;
        }
        return res;
    };
    uint64_t slots_total = resident_of(wide12_big(S, W, G));
    g->resident = (uint32_t)(slots_total < 0xFFFFFFFFull ? slots_total : 0xFFFFFFFFull);
    const bool fits = B > 1 && slots_total && (uint64_t)S * B <= slots_total;
    // segment lag (kernel comment).  Measured FFD kernel ms (7 segments of 12 groups, 4096
    // resident slots):
    //   S=4096: lag 600 29.0, 1170 27.5, 2340 26.9, 3000 26.5, 4096 26.3
    //   S=2048: lag 0 31.2, 256 19.2, 512 16.7, 1024 15.3, 2048 14.6
    //   S=1024: lag 0 18.6, 256 12.2, 512 11.4, 1024 11.3
    //   S=512 (fits at once): lag 0 10.8, 128 10.3, 512 10.6; S<=256 within 2%.
    // A segment that never waits on its upstream beats overlap between a scenario's
    // segments once the batch holds more segments than the GPU: lag = S runs the segments
    // index by index (phase b starts as phase b-1's tickets drain).  Batches that fit at
    // once keep lag 0 so all segments run concurrently.  FP_OPT_PIPE_LAG overrides.
    g->lag = (uint32_t)fp_opt(c, FP_OPT_PIPE_LAG, (B > 1 && S > 1 && slots_total && !fits) ? S : 0u);
    // Global links.  With lag 0 a producer blocked on a full bounded ring waits for its
    // consumer, the next segment of the same scenario, which took a later ticket.  The
    // lowest unfinished ticket's scenario always has every remaining segment resident when
    // this launch holds at least B slots, so its chain drains and back-pressure cannot
    // deadlock.  Rings are therefore used only when the whole batch fits (S * B slots) and a
    // scenario's chain fits twice over (2 * B), a margin for other work sharing the device
    // (fleetplace.h); otherwise a consumer may start only after its producer finished (lag =
    // S phases, more segments than slots), so the link holds every container:
    // (C + 63) / 64 + 2 slots.
    const uint32_t full = (C + 63) / 64 + 2;
    uint32_t ring = LINK_RING_SLOTS;
    {
        const int64_t v = fp_opt(c, FP_OPT_LINK_SLOTS, 0);
        if (v >= 8 && v < (int64_t)full) ring = (uint32_t)v;
    }
    const bool margin = 2ull * B <= slots_total;
    g->bounded = (uint32_t)fp_opt(c, FP_OPT_LINK_BOUNDED, (fits && margin && g->lag == 0 && ring < full) ? 1 : 0);
    if (B <= 1) g->bounded = 0;
    g->slots = g->bounded ? (ring < full ? ring : full) : full;
    if (g->bounded && wide12_big(S, W, G)) {
        // a bounded ring runs the five-wave 12-group kernel (fp_pipe_launch), which holds fewer
        // segments: report (FP_GEOM_RESIDENT) and size against that one.  The automatic
        // choice never bounds such a batch (S * B exceeds either kernel's slots), only a forced one
        const uint64_t r5 = resident_of(false);
        g->resident = (uint32_t)(r5 < 0xFFFFFFFFull ? r5 : 0xFFFFFFFFull);
    }
    // systolic group fill (fp_pipe_sys.h): queues of at least this many containers (compiled for
    // stages of at most SYS_MAX_G groups)
    // Default: queues of >= 32 containers in the narrow stages (configs 2 / 3 / 5: one scenario,
    // one-group stages); config 3's k_ffd_pipe 72.1 -> 65.2 ms, config 2 0.81 -> 0.75 ms, every
    // threshold from 1 to 48 within 1 % (tools/sys_sweep.py, profiles/r03c_sys_sweep.jsonl)
    g->sys = G <= (SYS_MAX_G > PK_SYS_MAX_G ? SYS_MAX_G : PK_SYS_MAX_G) ? (uint32_t)fp_opt(c, FP_OPT_SYSTOLIC, 32) : 0u;
    if (g->sys > 64) g->sys = 64;
    g->sys_extra = (uint32_t)fp_opt(c, FP_OPT_SYSTOLIC_EXTRA, 16);
    if (g->sys_extra > 128) g->sys_extra = 128;
    {  // step loop: 0 exec-masked (fp_pipe_sys.h), 1 VALU-only (fp_pipe_sysv.h), 2 DPP-folded (fp_pipe_sysd.h,
       // the default: 109-123 vs 134-153 cycles per container in tools/ubench/systolic.hip, r05e)
        const int64_t sv = fp_opt(c, FP_OPT_SYSTOLIC_VALU, 2);
        if (sv == 1) g->sys_extra |= 0x8000u;
        else if (sv == 2) g->sys_extra |= 0x4000u;
    }
    {
        const int64_t pv = fp_opt(c, FP_OPT_PIPE_PRIO, wide12_big(S, W, G) ? 0 : 1);
        g->prio = pv >= 0 && pv <= 2 ? (uint32_t)pv : 0u;
    }
    return true;
}

// Workspace bytes fp_pipe_launch takes (0 if the geometry does not fit).
size_t fp_pipe_ws_bytes(fp_ctx *c, uint32_t S, uint32_t C, uint32_t N) {
    PipeGeom g;
    if (!pipe_geom(c, S, C, N, &g)) return 0;
    const size_t SC = (size_t)S * C, nlinks = (size_t)S * (g.B - 1);
    return 5 * SC * 4 + SC * 5 + 256 + nlinks * LCTL * 4 + (size_t)S * g.B * 8 + 8 + nlinks * g.slots * 2 * 64 * 4 +
           (size_t)S * 16 + 11 * 256;
}

uint32_t fp_pipe_kpack(const fp_ctx *c, uint32_t C) {
    return C <= (IDX_POS_MASK + 1u) && fp_opt(c, FP_OPT_KPACK, 1) != 0;
}

int fp_pipe_soa_take(fp_ctx *c, size_t SC, fp_pipe_soa *soa) {
    soa->s_cpu = (uint32_t *)fp_ws_take(c, SC * 4);
    soa->s_mem = (uint32_t *)fp_ws_take(c, SC * 4);
    soa->s_req = (uint32_t *)fp_ws_take(c, SC * 4);
    soa->s_conf = (uint32_t *)fp_ws_take(c, SC * 4);
    soa->s_idx = (uint32_t *)fp_ws_take(c, SC * 4);
    return (soa->s_cpu && soa->s_mem && soa->s_req && soa->s_conf && soa->s_idx) ? FP_OK : FP_ENOMEM;
}

int fp_pipe_launch(fp_ctx *c, uint32_t S, uint32_t C, uint32_t N, uint32_t scen_base, const uint32_t *order,
                   const void *skeys, uint32_t key_bytes, uint32_t mbits, uint64_t cmax, uint64_t mmax,
                   const uint32_t *cval, const uint32_t *mval, const fp_batch *b, const uint32_t *thr,
                   const fp_pipe_soa *ready, uint32_t *rng) {
    PipeGeom geo;
    if (!pipe_geom(c, S, C, N, &geo)) return FP_EOVERFLOW;
    const uint32_t G = geo.G, W = geo.W, B = geo.B, R = geo.R, slots = geo.slots;
    const size_t lds = geo.lds;
    if (C >= 0x80000000u) return FP_EOVERFLOW;
    if ((uint64_t)S * B > 0xFFFFFFFFull) return FP_EOVERFLOW;
    hipStream_t st = c->stream;
    const size_t SC = (size_t)S * C;
    const size_t nlinks = (size_t)S * (B - 1);
    fp_pipe_soa soa;
    if (ready) soa = *ready;
    else if (int rc0 = fp_pipe_soa_take(c, SC, &soa)) return rc0;
    uint32_t *s_cpu = soa.s_cpu, *s_mem = soa.s_mem, *s_req = soa.s_req, *s_conf = soa.s_conf, *s_idx = soa.s_idx;
    uint32_t *ctl = (uint32_t *)fp_ws_take(c, 256 + nlinks * LCTL * 4);  // ticket, abort | link control
    uint32_t *part = (uint32_t *)fp_ws_take(c, (size_t)S * B * 8 + 8);
    uint32_t *gdata = nlinks ? (uint32_t *)fp_ws_take(c, nlinks * slots * 2 * 64 * 4) : nullptr;
    uint32_t *asg_s = (uint32_t *)fp_ws_take(c, SC * 4);  // plan in FFD order (k_unsort input)
    uint8_t *rsn_s = (uint8_t *)fp_ws_take(c, SC);
    if (!ctl || !part || (nlinks && !gdata) || !asg_s || !rsn_s) return FP_ENOMEM;
    FP_HIP(hipMemsetAsync(ctl, 0, 256 + nlinks * LCTL * 4, st));
    // buckets ride in s_idx when positions fit 21 bits (FP_OPT_KPACK = 0: search per stage)
    const uint32_t kpack = fp_pipe_kpack(c, C);
    // stage-2 screen (k_node_summary): per-scenario label union / conflict intersection of the
    // schedulable nodes; FP_OPT_SCREEN = 0 sends every container through the pipeline
    uint32_t *summ = nullptr;
    if (N && fp_opt(c, FP_OPT_SCREEN, 1)) {
        summ = (uint32_t *)fp_ws_take(c, (size_t)S * 16);
        if (!summ) return FP_ENOMEM;
    }
    // the packed pair (fp_pipe_pk.h): the batch's node values join the containers' OR (rng, from the sort)
    launch_fn u32fn = nullptr, pkfn = nullptr;
    const bool big = wide12_big(S, W, G) && !geo.bounded;  // (idle flushes of global links need bounded)
    {
        const void *k_;
        pipe_kernel(G, W, big, false, &u32fn, &k_);
        if (rng && fp_opt(c, FP_OPT_PACKED, 1) != 0) pipe_kernel(G, W, big, true, &pkfn, &k_);
        if (!u32fn) return FP_EOVERFLOW;
    }
    if (N && (summ || pkfn)) {
        if (summ && pkfn) k_node_summary<true, true><<<S, 256, 0, st>>>(N, b->cpu_free, b->mem_free, b->labels, b->conflict_used, b->schedulable, summ, rng);
        else if (summ) k_node_summary<true, false><<<S, 256, 0, st>>>(N, b->cpu_free, b->mem_free, b->labels, b->conflict_used, b->schedulable, summ, rng);
        else k_node_summary<false, true><<<S, 256, 0, st>>>(N, b->cpu_free, b->mem_free, b->labels, b->conflict_used, b->schedulable, summ, rng);
        FP_HIP(hipGetLastError());
    }
    const int64_t pl_mode = fp_opt(c, FP_OPT_PAYLOAD_LDS, 1);
    if (ready && C && C <= PL_MAX_C && pl_mode != 0) {
        // k_scen_sort wrote order, cpu, mem and the position words; req / conf / CYCLE bits
        // through LDS, one workgroup per scenario
        const size_t pl = (size_t)PL_CHUNK * 8;
        // (a one-sweep variant writing each position in the chunk pass that holds its container
        // -- partial lines per pass -- ran 3.6 ms slower per config-4 step, in a sweep whose inputs
        // were not yet synchronised with the generator: r03k_payload_ab.jsonl; dropped)
        FP_HIP(hipFuncSetAttribute((const void *)k_payload_lds, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl));
        k_payload_lds<<<S, PL_THREADS, pl, st>>>(C, order, b->req_labels, b->conflict, b->level, summ, s_req, s_conf,
                                                 s_idx);
        FP_HIP(hipGetLastError());
    } else if (ready) {  // the same with random gathers
        size_t g = (SC + 1023) / 1024;
        if (g >= 64) g = (g + 7) & ~(size_t)7;
        k_gather_payload<<<(unsigned)g, 256, 0, st>>>(S, C, order, b->req_labels, b->conflict, b->level, summ,
                                                      s_req, s_conf, s_idx);
        FP_HIP(hipGetLastError());
    } else {
        size_t g = (SC + 1023) / 1024;  // one tile of 1024 elements per block
        if (g >= 64) g = (g + 7) & ~(size_t)7;  // a multiple of 8: XCD-contiguous mapping
        if (key_bytes == 4)
            k_gather_sorted<uint32_t><<<(unsigned)g, 256, 0, st>>>(
                thr, kpack, S, C, order, (const uint32_t *)skeys, mbits, cmax, mmax, cval, mval, b->cpu_m, b->mem_mib, b->req_labels,
                b->conflict, b->level, summ, s_cpu, s_mem, s_req, s_conf, s_idx);
        else
            k_gather_sorted<uint64_t><<<(unsigned)g, 256, 0, st>>>(
                thr, kpack, S, C, order, (const uint64_t *)skeys, mbits, cmax, mmax, cval, mval, b->cpu_m, b->mem_mib, b->req_labels,
                b->conflict, b->level, summ, s_cpu, s_mem, s_req, s_conf, s_idx);
        FP_HIP(hipGetLastError());
    }
    PipeArgs a;
    a.C = C; a.N = N; a.scen_base = scen_base; a.W = W; a.G = G; a.R = R;
    a.B = B; a.slots = slots; a.bounded = geo.bounded; a.ticket = ctl; a.gabort = ctl + 32; a.ghead = ctl + 64;
    a.gdata = gdata;
    a.S = S;
    a.lag = geo.lag;
    a.kpack = kpack;
    // idle flushes: LDS rings always (producer and consumer share the workgroup); global links
    // only when bounded -- their consumer runs beside the producer and back-pressure bounds
    // the extra partial slots (an unbounded link is sized for full slots only).
    // FP_OPT_PIPE_FLUSH = mask of the two (0 disables).
    a.flush = (geo.bounded ? 3u : 1u) & (uint32_t)fp_opt(c, FP_OPT_PIPE_FLUSH, 3);
    a.part = part;
    a.s_cpu = s_cpu; a.s_mem = s_mem; a.s_req = s_req; a.s_conf = s_conf; a.s_idx = s_idx;
    a.cf = b->cpu_free; a.mf = b->mem_free; a.lab = b->labels; a.cu = b->conflict_used; a.sched = b->schedulable;
    a.assign = asg_s; a.reason = rsn_s; a.cost = b->cost; a.err = c->d_err;
    a.spin_ticks = (uint64_t)fp_opt(c, FP_OPT_SPIN_TICKS, (int64_t)SPIN_TICKS);
    a.sys = geo.sys ? (geo.sys | (geo.sys_extra << 16)) : 0u;
    // Head publishes on a link that holds every container (lag = S: the consumer runs a phase
    // later) are batched: FP_OPT_LINK_PUBLISH full slots per head store and vmcnt(0) drain.  A
    // bounded ring publishes every slot: its producer may wait on the consumer's tail, which
    // moves only on published slots.
    // Default: 32 slots at 4096 scenarios and more, 8 below -- at 2048 / 1024 scenarios the
    // consumer phase starts sooner (7.70-7.74 / 6.01-6.03 against 7.91-7.92 / 6.11-6.24 ms), at 4096
    // 8 is +0.3 % (profiles/r09h_link_publish_sweep.jsonl).
    {
        const int64_t pv = fp_opt(c, FP_OPT_LINK_PUBLISH, S >= 4096 ? 32 : 8);
        a.publish = geo.bounded ? 1u : (uint32_t)(pv < 1 ? 1 : pv > 1024 ? 1024 : pv);
        uint32_t p2 = 1;
        while (p2 * 2 <= a.publish) p2 *= 2;
        a.pub_mask = p2 - 1;
    }
    // bucket thresholds (device; fp_place.hip k_thresholds chooses them -- any ascending choice
    // with T0 = 0 is exact, it only decides how tight the candidate masks are)
    a.thr = thr;
    a.prio = geo.prio;
    const bool wide = wide_g(W, G);
    if (G < 1 || (wide ? (G > MAX_G_WIDE || G % 4) : G > MAX_G)) return FP_EOVERFLOW;
    // A bounded launch's producers wait on consumers of the same launch, so it needs its segments
    // co-resident (pipe_geom: the batch fits the device, a scenario's chain twice over).  Another
    // context's bounded launch on the same device could hold the slots it needs; bounded launches
    // of this process are therefore serialised per device (BoundedGate): each waits, on its own
    // stream, for the previous one to finish.  Unbounded launches never wait on a consumer and
    // finish whatever else runs, so they only delay a bounded one, never block it.
    std::unique_lock<std::mutex> gate_lock;
    BoundedGate *gate = nullptr;
    if (geo.bounded) {
        if (c->device < 0 || c->device >= kMaxGateDevices) return FP_EINVAL;
        gate = &g_bounded_gate[c->device];
        gate_lock = std::unique_lock<std::mutex>(gate->m);
        if (!gate->ev) FP_HIP(hipEventCreateWithFlags(&gate->ev, hipEventDisableTiming));
        else FP_HIP(hipStreamWaitEvent(st, gate->ev, 0));
    }
    hipEvent_t ev;
    fp_prof_begin(c, FP_K_PLACE, &ev);
    // the six-wave kernel is compiled for unbounded links only (see the kernel; `big` above)
    int rc;
    a.rng = rng;
    if (pkfn) {
        // the pair, back to back: the u32 kernel returns at once when the batch packs, the packed
        // one when it does not (each reads the batch's OR words first)
        a.pk_mode = 1;
        rc = u32fn(st, (unsigned)(S * B), W * 64, lds, a);
        if (!rc) {
            FP_HIP(hipGetLastError());
            a.pk_mode = 2;
            rc = pkfn(st, (unsigned)(S * B), W * 64, lds, a);
        }
    } else {
        a.pk_mode = 0;
        rc = u32fn(st, (unsigned)(S * B), W * 64, lds, a);
    }
    if (rc) return rc;
    FP_HIP(hipGetLastError());
    fp_prof_end(c, FP_K_PLACE, ev);
    if (gate) {
        FP_HIP(hipEventRecord(gate->ev, st));
        gate_lock.unlock();
    }
    {
        const bool narrow16 = N < 0xFFFFu;  // node indices and FP_NONE (-> 0xFFFF) fit 16 bits
        const uint32_t span = narrow16 ? UNSORT_SPAN16 : UNSORT_SPAN32;
        const uint32_t H = (C + span - 1) / span;
        const size_t ul = (size_t)span * (narrow16 ? 3 : 5);
        const void *fn = narrow16 ? (const void *)k_unsort<true> : (const void *)k_unsort<false>;
        FP_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ul));
        if (narrow16)
            k_unsort<true><<<(unsigned)(S * H), 1024, ul, st>>>(C, H, span, order, asg_s, rsn_s, b->assign, b->reason);
        else
            k_unsort<false><<<(unsigned)(S * H), 1024, ul, st>>>(C, H, span, order, asg_s, rsn_s, b->assign, b->reason);
        FP_HIP(hipGetLastError());
    }
    if (b->cost) {
        k_cost_reduce<<<(S + 255) / 256, 256, 0, st>>>(S, B, scen_base, part, b->cost);
        FP_HIP(hipGetLastError());
    }
    return FP_OK;
}

// The pipeline fp_dev_place_batch runs for S x C x N on this ctx (fleetplace.h FP_GEOM_*).
int fp_place_geometry_impl(fp_ctx *c, uint32_t S, uint32_t C, uint32_t N, uint32_t *out) {
    PipeGeom g;
    if (!pipe_geom(c, S, C, N, &g)) return FP_EOVERFLOW;
    const uint32_t v[FP_GEOM_COUNT] = {g.G, g.W, g.B, g.R, g.lag, g.slots, g.bounded, g.resident, g.sys};
    memcpy(out, v, sizeof(v));
    return FP_OK;
}

#ifdef FP_PIPE_STATS
extern "C" int fp_debug_pipe_timeline(unsigned long long *out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pipe_tl), sizeof(unsigned long long) * 16 * TL_B * 8) != hipSuccess)
        return FP_EDEVICE;
    return FP_OK;
}
extern "C" int fp_debug_stage_span(unsigned long long *out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stage_span), sizeof(unsigned long long) * SPAN_MAX * 8) != hipSuccess)
        return FP_EDEVICE;
    return FP_OK;
}
// s_memtime ticks per s_memrealtime tick (100 MHz) over a ~2 ms spin: the shader clock
__global__ void k_debug_clock(unsigned long long *out) {
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = r0;
    while (r1 - r0 < 200000) r1 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = c1 - c0; out[1] = r1 - r0; }
}
extern "C" int fp_debug_clock_ghz(fp_ctx *c, double *ghz) {
    unsigned long long *d = nullptr, h[2] = {0, 0};
    if (hipMalloc(&d, 16) != hipSuccess) return FP_ENOMEM;
    k_debug_clock<<<1, 64, 0, c->stream>>>(d);
    const bool ok = hipMemcpyAsync(h, d, 16, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
                    hipStreamSynchronize(c->stream) == hipSuccess;
    (void)hipFree(d);
    if (!ok || !h[1]) return FP_EDEVICE;
    *ghz = (double)h[0] / (double)h[1] * 0.1;
    return FP_OK;
}
#ifdef FP_PIPE_STATS
extern "C" int fp_debug_sys_stats(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sys_stats), sizeof(unsigned long long) * 8) != hipSuccess)
        return FP_EDEVICE;
    if (reset) {
        static const unsigned long long zero[8] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_sys_stats), zero, sizeof(zero)) != hipSuccess) return FP_EDEVICE;
    }
    return FP_OK;
}
#endif

extern "C" int fp_debug_pipe_stats(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pipe_stats), sizeof(unsigned long long) * 16 * 16) != hipSuccess)
        return FP_EDEVICE;
    if (reset) {
        static unsigned long long zero[16 * 16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_pipe_stats), zero, sizeof(zero)) != hipSuccess) return FP_EDEVICE;
    }
    return FP_OK;
}
#endif
#endif  // !FPP_KERNEL_TU
