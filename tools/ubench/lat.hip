// Micro-benchmark: single-wave latencies of the instruction patterns on the FFD
// critical path (one wave alone on its SIMD).  Prints cycles per iteration.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 1000
typedef uint32_t v32u __attribute__((ext_vector_type(32)));

__global__ void k_lat(uint64_t *out, const uint32_t *in, uint32_t seed) {
    __shared__ uint64_t lds[1024];
    const uint32_t lane = threadIdx.x;
    for (int i = lane; i < 1024; i += 64) lds[i] = 0x0123456789abcdefull * (i + 1);
    __syncthreads();
    uint32_t x = in[lane], y = in[lane + 64];
    uint64_t t0, t1;
    int slot = 0;
    // (0) dependent VALU chain
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) { x = x * 3u + y; __builtin_amdgcn_sched_barrier(0); }
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[slot] = t1 - t0;
    slot++;
    // (1) ballot -> scalar branch chain (compare, ballot, test, branch)
    uint32_t acc = 0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        uint64_t m = __builtin_amdgcn_ballot_w64(x > (uint32_t)i * seed);
        if (m) acc += (uint32_t)__builtin_ctzll(m); else acc ^= 1;
        x += acc;
        __builtin_amdgcn_sched_barrier(0);
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[slot] = t1 - t0;
    slot++;
    // (2) readlane -> scalar -> readlane chain
    uint32_t s = 0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) { s = __builtin_amdgcn_readlane(x + s, s & 63); __builtin_amdgcn_sched_barrier(0); }
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[slot] = t1 - t0;
    x += s;
    slot++;
    // (3) uniform LDS read -> wait -> use as address (pointer chase)
    uint32_t p = seed & 1023;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) { p = (uint32_t)(lds[p] >> 7) & 1023u; __builtin_amdgcn_sched_barrier(0); }
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[slot] = t1 - t0;
    x += p;
    slot++;
    // (4) dynamic register index read (s_set_gpr_idx) chained through the index
    v32u v;
#pragma unroll
    for (int k = 0; k < 32; ++k) v[k] = in[k * 64 + lane];
    uint32_t j = seed & 31;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        uint32_t r = v[j];
        j = __builtin_amdgcn_readfirstlane(r) & 31u;
        __builtin_amdgcn_sched_barrier(0);
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[slot] = t1 - t0;
    x += j;
    slot++;
    // (5) dynamic register write + read
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        uint32_t r = v[j];
        v[j] = lane == (j & 63) ? r + 1 : r;
        j = (j * 7u + 3u) & 31u;
        __builtin_amdgcn_sched_barrier(0);
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[slot] = t1 - t0;
    slot++;
    // (6) ds_and_b64 no-return (throughput of the mask update)
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        __hip_atomic_fetch_and(&lds[(lane + i) & 1023], ~(1ull << (i & 63)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __builtin_amdgcn_sched_barrier(0);
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[slot] = t1 - t0;
    slot++;
    // (8) all-lane ds_and_b64 then a dependent ds_read_b64 (latency of the pair)
    {
        uint64_t acc8 = 0;
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < ITERS; ++i) {
            __hip_atomic_fetch_and(&lds[(lane + (uint32_t)acc8) & 1023], ~(1ull << (i & 63)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            acc8 += lds[(lane * 3 + i) & 1023] & 1;
            __builtin_amdgcn_sched_barrier(0);
        }
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[slot] = t1 - t0;
        x += (uint32_t)acc8;
        slot++;
    }
    // (9) all-lane ds_write_b64 then dependent ds_read_b64
    {
        uint64_t acc9 = 0;
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < ITERS; ++i) {
            lds[(lane + (uint32_t)acc9) & 1023] = acc9 + i;
            acc9 += lds[(lane * 3 + i) & 1023] & 1;
            __builtin_amdgcn_sched_barrier(0);
        }
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[slot] = t1 - t0;
        x += (uint32_t)acc9;
        slot++;
    }
    // (10) lane-varying ds_read_b64 -> compare -> ballot -> branch chain
    {
        uint32_t p10 = 0;
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < ITERS; ++i) {
            uint64_t r = lds[(lane + p10 * 64) & 1023];
            uint64_t m = __builtin_amdgcn_ballot_w64((uint32_t)r > (uint32_t)(i * seed));
            p10 = m ? (uint32_t)__builtin_ctzll(m) & 15 : p10 + 1;
            __builtin_amdgcn_sched_barrier(0);
        }
        t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[slot] = t1 - t0;
        x += p10;
        slot++;
    }
    // (7) empty loop
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) { asm volatile("" ::: "memory"); __builtin_amdgcn_sched_barrier(0); }
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[slot] = t1 - t0;
    slot++;
    uint32_t sum = x;
#pragma unroll
    for (int k = 0; k < 32; ++k) sum += v[k];
    if (lane == 0) out[15] = sum;
}

int main() {
    uint64_t *d_out; uint32_t *d_in;
    hipMalloc(&d_out, 16 * 8); hipMalloc(&d_in, 64 * 64 * 4);
    uint32_t h_in[64 * 64];
    for (int i = 0; i < 64 * 64; ++i) h_in[i] = (i * 2654435761u) >> 3;
    hipMemcpy(d_in, h_in, sizeof(h_in), hipMemcpyHostToDevice);
    const char *names[] = {"dep VALU mul-add", "ballot->branch", "readlane chain", "LDS uniform chase",
                           "gpr_idx read chain", "gpr_idx write+read", "ds_and_b64 nortn", "atomic+dep read", "write+dep read", "lds->ballot->branch", "empty loop"};
    for (int rep = 0; rep < 3; ++rep) {
        k_lat<<<1, 64>>>(d_out, d_in, 12345);
        hipDeviceSynchronize();
        uint64_t h[16];
        hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost);
        if (rep == 2)
            for (int i = 0; i < 11; ++i) printf("%-22s %7.1f cycles/iter\n", names[i], (double)h[i] / ITERS);
    }
    return 0;
}
