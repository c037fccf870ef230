// Micro-benchmark: one group's exact first fit, serial exec-masked loop (fpp_group_x,
// fp_pipe_asm.h) vs the systolic loop (fp_pipe_sys.h) with and without the serial finish.
// Every variant must produce the serial loop's assignment and records (mismatches column).
// One wave per SIMD (NW waves on one CU, each on its own copy of the same queue).
//   pattern 0: fill phase, 64 x (64000 m, 256 GiB) nodes, containers 4000 m / 1 GiB
//   pattern 1: mixed node types, 4000 m containers with descending memory, ports, labels
//   pattern 2: config-3-like labels (4 one-hot dimensions), ports + anti-affinity
//   pattern 3: a partly filled group (random free capacity), descending demands, 25% labels
//   pattern 4: a full group: almost nothing fits (the pass-through case)
// Variants 7-9 run the packed-capacity check (fp_pipe_pk.h) when the pattern's values pack
// (every value a multiple of 2^sc and below 2^(15 + sc)); "n/a" otherwise.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../fleetflow_amd/csrc systolic.hip -o systolic
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "fp_pipe_asm.h"
#include "fp_pipe_sys.h"
#include "fp_pipe_sysv.h"
#include "fp_pipe_sysd.h"
#include "fp_pipe_pk.h"

using namespace fpp;

__device__ __forceinline__ uint32_t hsh(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

__device__ void setup(int pattern, uint32_t r, uint32_t lane, uint32_t &rcf, uint32_t &rmf, uint32_t &rcu,
                      uint32_t &rlab, uint32_t &cpu, uint32_t &mem, uint32_t &req, uint32_t &conf) {
    rlab = 0; rcu = 0; req = 0; conf = 0;
    const uint32_t ty = hsh(lane * 7 + 1 + r * 131) % 5;
    if (pattern == 0) {
        rcf = 64000; rmf = 262144; cpu = 4000; mem = 1024;
    } else if (pattern == 1) {
        rcf = 4000u << ty; rmf = ty == 4 ? 262144u : 8192u << ty;
        rlab = ~(1u << (hsh(lane * 7 + 2) % 3));
        cpu = 4000; mem = 16384 - lane * 64;
        conf = hsh(lane * 7 + 3) % 10 == 0 ? 1u << (hsh(lane * 7 + 4) % 16) : 0u;
        req = hsh(lane * 7 + 5) % 5 == 0 ? 1u << (hsh(lane * 7 + 6) % 3) : 0u;
    } else if (pattern == 2) {
        rcf = 4000u << ty; rmf = ty == 4 ? 262144u : 8192u << ty;
        rlab = ~((1u << (hsh(lane * 9 + 2) % 3)) | (1u << (3 + hsh(lane * 9 + 3) % 4)) |
                 (1u << (7 + hsh(lane * 9 + 4) % 4)) | (1u << (11 + hsh(lane * 9 + 5) % 2)));
        cpu = 4000; mem = 16384 - lane * 64;
        conf = (hsh(lane * 5 + 1) % 10 == 0 ? 1u << (hsh(lane * 5 + 2) % 16) : 0u) |
               (hsh(lane * 5 + 3) % 5 == 0 ? 1u << (16 + hsh(lane * 5 + 4) % 16) : 0u);
        req = hsh(lane * 5 + 6) % 10 < 3 ? 1u << (hsh(lane * 5 + 7) % 13) : 0u;
    } else if (pattern == 3) {
        rcf = hsh(lane * 11 + r) % 16000; rmf = hsh(lane * 13 + r) % 65536;
        rlab = ~((1u << (hsh(lane * 9 + 2) % 3)) | (1u << (3 + hsh(lane * 9 + 3) % 4)));
        cpu = 3000 - lane * 30; mem = 8192 - lane * 100;
        conf = hsh(lane * 5 + 3 + r) % 5 == 0 ? 1u << (16 + hsh(lane * 5 + 4) % 16) : 0u;
        req = hsh(lane * 5 + 6 + r) % 4 == 0 ? 1u << (hsh(lane * 5 + 7) % 7) : 0u;
    } else {
        rcf = 1000 + (hsh(lane + r) % 500); rmf = 4096; cpu = 2000 - lane; mem = 1024;
    }
}

template <int V>
__global__ void k_sys(uint64_t *out, uint32_t *res, int pattern, uint32_t reps, uint32_t extra) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t tot = 0, nplaced = 0;
    uint32_t asg = 0, rcf = 0, rmf = 0, rcu = 0, nxt = 0;
    for (uint32_t r = 0; r < reps; ++r) {
        uint32_t rlab, cpu, mem, req, conf;
        setup(pattern, r & 7, lane, rcf, rmf, rcu, rlab, cpu, mem, req, conf);
        // the batch corner of the queue
        uint32_t qc = cpu, qm = mem;
        for (int o = 32; o; o >>= 1) {
            qc = min(qc, (uint32_t)__shfl_xor((int)qc, o));
            qm = min(qm, (uint32_t)__shfl_xor((int)qm, o));
        }
        qc = __builtin_amdgcn_readfirstlane(qc);
        qm = __builtin_amdgcn_readfirstlane(qm);
        uint64_t placed = 0, touched = 0;
        uint32_t nchk = 0, nhit = 0;
        asg = 0xFFFFFFFFu;
        nxt = 0;
        const uint64_t q = ~0ull;
        __builtin_amdgcn_sched_barrier(0);
        // packed form (V >= 7): shifts from the OR of every cpu / mem value of the pattern
        uint32_t rw = 0, cw = 0, qw = 0, sc_c = 0, sc_m = 0;
        bool pk_ok = true;
        if constexpr (V >= 7) {
            const uint32_t oc = sys_wave_or(rcf | cpu), om = sys_wave_or(rmf | mem);
            sc_c = oc ? (uint32_t)__builtin_ctz(oc) : 0u;
            sc_m = om ? (uint32_t)__builtin_ctz(om) : 0u;
            pk_ok = (oc >> sc_c) <= PK_FIELD_MAX && (om >> sc_m) <= PK_FIELD_MAX;
            rw = pk_pack(rcf, rmf, sc_c, sc_m);
            cw = pk_pack(cpu, mem, sc_c, sc_m);
            qw = pk_pack(qc, qm, sc_c, sc_m);
            if (!pk_ok && lane == 0) out[63] = 1;  // not packable: reported n/a
        }
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        if constexpr (V >= 7) {
            if (V == 7) {
                fpp_group_xp<0, 1>(q, placed, touched, asg, nxt, rw, rcu, rlab, cw, req, conf, 1u, 0u, 0u, nchk, nhit, qw);
            } else {
                const uint32_t cap = V == 8 ? 1000u : (uint32_t)__builtin_popcountll(q) + extra;
                SysOut so = fpp_sysp_group(q, touched, asg, rw, rcu, rlab, cw, req, conf, 0u, qw, cap);
                uint64_t left = __builtin_amdgcn_readfirstlane((uint32_t)so.left) |
                                ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(so.left >> 32)) << 32);
                if (left) fpp_asm_group_xp<false>(left, touched, asg, rw, rcu, rlab, cw, req, conf, 0u, nchk);
                placed = __builtin_amdgcn_ballot_w64(asg != 0xFFFFFFFFu);
            }
        } else if constexpr (V == 0) {
            fpp_group_x<0, 1>(q, placed, touched, asg, nxt, rcf, rmf, rcu, rlab, cpu, mem, req, conf, 1u, 0u, 0u, nchk,
                              nhit, qc, qm);
        } else {
            const uint32_t cap = (V == 1 || V == 3 || V == 5) ? 1000u : (uint32_t)__builtin_popcountll(q) + extra;
            SysOut so = V >= 5   ? fpp_sysd_group(q, touched, asg, rcf, rmf, rcu, rlab, cpu, mem, req, conf, 0u, qc, qm, cap)
                        : V >= 3 ? fpp_sysv_group(q, touched, asg, rcf, rmf, rcu, rlab, cpu, mem, req, conf, 0u, qc, qm, cap)
                                 : fpp_sys_group(q, touched, asg, rcf, rmf, rcu, rlab, cpu, mem, req, conf, 0u, qc, qm, cap);
            uint64_t left = __builtin_amdgcn_readfirstlane((uint32_t)so.left) |
                            ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(so.left >> 32)) << 32);
            if (left) fpp_asm_group_x<false>(left, touched, asg, rcf, rmf, rcu, rlab, cpu, mem, req, conf, 0u, nchk);
            placed = __builtin_amdgcn_ballot_w64(asg != 0xFFFFFFFFu);
        }
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (V >= 7) {  // records back to real units for the comparison with the serial loop
            rcf = pk_cpu(rw, sc_c);
            rmf = pk_mem(rw, sc_m);
        }
        tot += t1 - t0;
        nplaced += __builtin_popcountll(placed);
        if (r == reps - 1 && threadIdx.x < 64) {
            res[lane] = asg; res[64 + lane] = rcf; res[128 + lane] = rmf; res[192 + lane] = rcu;
            res[256 + lane] = (uint32_t)(touched >> lane) & 1u;
        }
    }
    if (lane == 0) {
        out[(threadIdx.x >> 6) * 2] = tot;
        out[(threadIdx.x >> 6) * 2 + 1] = nplaced;
    }
}

int main() {
    uint64_t *d;
    uint32_t *dr;
    hipMalloc(&d, 64 * 8);
    hipMalloc(&dr, 5 * 64 * 4);
    const uint32_t reps = 64;
    const char *names[10] = {"serial exec-masked (fpp_group_x)", "systolic, full", "systolic, Q+extra + serial",
                            "VALU systolic, full", "VALU systolic, Q+extra + serial", "DPP-folded systolic, full",
                            "DPP-folded, Q+extra + serial", "packed serial (fpp_group_xp)", "packed systolic, full",
                            "packed systolic, Q+extra + serial"};
    for (int pattern : {0, 1, 2, 3, 4}) {
        uint32_t ref[320], got[320];
        for (int v = 0; v <= 9; ++v) {
            for (uint32_t extra : {0u, 8u, 16u}) {
                if ((v < 2 || v == 3 || v == 5 || v == 7 || v == 8) && extra) continue;
                for (int nw : {1, 4}) {
                    uint64_t h[64] = {0};
                    for (int it = 0; it < 2; ++it) {
                        hipMemset(d, 0, 64 * 8);
                        if (v == 0) k_sys<0><<<1, nw * 64>>>(d, dr, pattern, reps, extra);
                        else if (v == 1) k_sys<1><<<1, nw * 64>>>(d, dr, pattern, reps, extra);
                        else if (v == 2) k_sys<2><<<1, nw * 64>>>(d, dr, pattern, reps, extra);
                        else if (v == 3) k_sys<3><<<1, nw * 64>>>(d, dr, pattern, reps, extra);
                        else if (v == 4) k_sys<4><<<1, nw * 64>>>(d, dr, pattern, reps, extra);
                        else if (v == 5) k_sys<5><<<1, nw * 64>>>(d, dr, pattern, reps, extra);
                        else if (v == 6) k_sys<6><<<1, nw * 64>>>(d, dr, pattern, reps, extra);
                        else if (v == 7) k_sys<7><<<1, nw * 64>>>(d, dr, pattern, reps, extra);
                        else if (v == 8) k_sys<8><<<1, nw * 64>>>(d, dr, pattern, reps, extra);
                        else k_sys<9><<<1, nw * 64>>>(d, dr, pattern, reps, extra);
                        if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
                        hipMemcpy(h, d, 64 * 8, hipMemcpyDeviceToHost);
                    }
                    hipMemcpy(v == 0 ? ref : got, dr, sizeof(ref), hipMemcpyDeviceToHost);
                    int bad = 0;
                    if (v) for (int i = 0; i < 320; ++i) bad += ref[i] != got[i];
                    if (h[63]) {
                        printf("pattern %d %-34s extra %2u waves %d: n/a (values do not pack)\n", pattern, names[v],
                               extra, nw);
                        continue;
                    }
                    printf("pattern %d %-34s extra %2u waves %d: %7.1f cycles per container (%llu placed of %u) "
                           "mismatches %d\n", pattern, names[v], extra, nw, (double)h[0] / (64.0 * reps),
                           (unsigned long long)h[1], 64 * reps, bad);
                }
            }
        }
    }
    return 0;
}
