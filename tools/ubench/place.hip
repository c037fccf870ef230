// Micro-benchmark: cycles per container of the FFD group loop on one 64-node group and a
// 64-container queue, serial loop (fpp_asm_group, fp_pipe_asm.h) vs the windowed loop
// and its scheduling variants (place_variants.h); all must produce identical plans and records.
//   pattern 0: fill phase, 64 x (64000 m, 256 GiB) nodes, containers 4000 m / 1 GiB
//   pattern 1: mixed node types (SPEC 3.2 sizes), containers 4000 m with descending memory,
//              10% port conflicts, 20% label requirements
// One workgroup of NW waves on one CU (every wave runs the same queue).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../fleetflow_amd/csrc place.hip -o place
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "fp_pipe_asm.h"
#include "place_variants.h"

using namespace fpp;

__device__ __forceinline__ uint32_t hsh(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

template <int V>
__global__ void k_place(uint64_t *out, uint32_t *res, int pattern, uint32_t reps) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t tot = 0, nplaced = 0;
    uint32_t asg = 0xFFFFFFFFu, rcf = 0, rmf = 0, rcu = 0, nxt = 0;
    for (uint32_t r = 0; r < reps; ++r) {
        uint32_t rlab = 0, cpu, mem, req = 0, conf = 0;
        if (pattern == 0) {
            rcf = 64000; rmf = 262144; rcu = 0;
            cpu = 4000; mem = 1024;
        } else if (pattern == 2) {
            // config-3-like (SPEC 3.2): mixed node types with one tier/region/class/arch label each,
            // containers 4000 m with descending memory, 30% one label of 13, 10% port, 20% anti-affinity
            const uint32_t ty = hsh(lane * 7 + 1) % 5;
            rcf = 4000u << ty; rmf = ty == 4 ? 262144u : 8192u << ty; rcu = 0;
            rlab = ~((1u << (hsh(lane * 9 + 2) % 3)) | (1u << (3 + hsh(lane * 9 + 3) % 4)) |
                     (1u << (7 + hsh(lane * 9 + 4) % 4)) | (1u << (11 + hsh(lane * 9 + 5) % 2)));
            cpu = 4000; mem = 16384 - lane * 64;
            conf = (hsh(lane * 5 + 1) % 10 == 0 ? 1u << (hsh(lane * 5 + 2) % 16) : 0u) |
                   (hsh(lane * 5 + 3) % 5 == 0 ? 1u << (16 + hsh(lane * 5 + 4) % 16) : 0u);
            req = hsh(lane * 5 + 6) % 10 < 3 ? 1u << (hsh(lane * 5 + 7) % 13) : 0u;
        } else {
            const uint32_t ty = hsh(lane * 7 + 1) % 5;
            rcf = 4000u << ty; rmf = ty == 4 ? 262144u : 8192u << ty; rcu = 0;
            rlab = ~(1u << (hsh(lane * 7 + 2) % 3));                 // ~labels: one tier bit
            cpu = 4000; mem = 16384 - lane * 64;
            conf = hsh(lane * 7 + 3) % 10 == 0 ? 1u << (hsh(lane * 7 + 4) % 16) : 0u;
            req = hsh(lane * 7 + 5) % 5 == 0 ? 1u << (hsh(lane * 7 + 6) % 3) : 0u;
        }
        const uint32_t cand = 1, cand_hi = 0;
        uint64_t placed = 0, touched = 0;
        uint32_t nchk = 0, nhit = 0;
        asg = 0xFFFFFFFFu; nxt = 0;
        const uint64_t q = ~0ull;
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        if constexpr (V == 0)
            fpp_asm_group<0, 1>(q, placed, touched, asg, nxt, rcf, rmf, rcu, rlab, cpu, mem, req, conf, cand, cand_hi,
                                0u, nchk, nhit);
        else if constexpr (V == 5)
            fppv::group_node_major<0, 1>(q, placed, touched, asg, nxt, rcf, rmf, rcu, rlab, cpu, mem, req, conf, cand,
                                         cand_hi, 0u);
        else
            fppv::group_vx<V, 0, 1>(q, placed, touched, asg, nxt, rcf, rmf, rcu, rlab, cpu, mem, req, conf, cand,
                                    cand_hi, 0u);
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
        tot += t1 - t0;
        nplaced += __builtin_popcountll(placed);
        (void)touched;
    }
    if (lane == 0) {
        out[(threadIdx.x >> 6) * 2] = tot;
        out[(threadIdx.x >> 6) * 2 + 1] = nplaced;
    }
    if (threadIdx.x < 64) {
        res[lane] = asg; res[64 + lane] = rcf; res[128 + lane] = rmf; res[192 + lane] = rcu; res[256 + lane] = nxt;
    }
}

int main() {
    uint64_t *d;
    uint32_t *dr;
    hipMalloc(&d, 64 * 8);
    hipMalloc(&dr, 5 * 64 * 4);
    const uint32_t reps = 200;
    const char *names[] = {"round-2 serial", "execmask (V1)", "writelane asg (V2)", "pipelined pairs (V3)",
                           "pipelined pairs + writelane (V4)", "node-major scans (V5)"};
    for (int pattern : {0, 1, 2}) {
        uint32_t ref[320], got[320];
        for (int v = 0; v <= 5; ++v) {
            for (int nw : {1, 4}) {
                uint64_t h[64] = {0};
                for (int it = 0; it < 2; ++it) {
                    hipMemset(d, 0, 64 * 8);
                    switch (v) {
                        case 0: k_place<0><<<1, nw * 64>>>(d, dr, pattern, reps); break;
                        case 1: k_place<1><<<1, nw * 64>>>(d, dr, pattern, reps); break;
                        case 2: k_place<2><<<1, nw * 64>>>(d, dr, pattern, reps); break;
                        case 3: k_place<3><<<1, nw * 64>>>(d, dr, pattern, reps); break;
                        case 4: k_place<4><<<1, nw * 64>>>(d, dr, pattern, reps); break;
                        default: k_place<5><<<1, nw * 64>>>(d, dr, pattern, reps); break;
                    }
                    hipDeviceSynchronize();
                    hipMemcpy(h, d, 64 * 8, hipMemcpyDeviceToHost);
                }
                hipMemcpy(v == 0 ? ref : got, dr, sizeof(ref), hipMemcpyDeviceToHost);
                int bad = 0;
                if (v) for (int i = 0; i < 320; ++i) bad += ref[i] != got[i];
                printf("pattern %d %-34s waves %d: %7.1f cycles per container (%llu placed of %u) mismatches %d\n",
                       pattern, names[v], nw, (double)h[0] / (64.0 * reps), (unsigned long long)h[1], 64 * reps, bad);
            }
        }
    }
    return 0;
}
