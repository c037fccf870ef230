// Micro-benchmark: issue cost of single instructions / short idioms for one wave (cycles per
// repetition of a 32x-unrolled inline-asm body, s_memtime).  Calibrates the FFD chain model.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 isa.hip -o isa
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define R4(x) x x x x
#define R32(x) R4(R4(x)) R4(x) R4(x)

#define BENCH(idx, body, ...)                                                   \
    {                                                                           \
        const uint64_t t0 = __builtin_amdgcn_s_memtime();                      \
        for (int i = 0; i < 16; ++i) asm volatile(R32(body) __VA_ARGS__);      \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();                      \
        if (threadIdx.x == 0) out[idx] = t1 - t0;                              \
    }

__global__ void k_isa(uint64_t *out, uint32_t seed) {
    uint32_t s0 = seed, s1 = seed * 3u, s2 = 5;
    uint64_t d0 = seed;
    uint32_t v0 = threadIdx.x, v1 = threadIdx.x * 7u;
    // 0: dependent s_add_u32 chain
    BENCH(0, "s_add_u32 %0, %0, %1\n\t", : "+s"(s0) : "s"(s1) : "scc");
    // 1: independent s_add_u32 (alternating two destinations)
    BENCH(1, "s_add_u32 %0, %2, 1\n\ts_add_u32 %1, %2, 2\n\t", : "=&s"(s0), "=&s"(s1) : "s"(s2) : "scc");
    // 2: dependent s_ff1_i32_b64 + s_lshl
    BENCH(2, "s_ff1_i32_b64 %0, %1\n\ts_lshl_b64 %1, %1, 1\n\t", : "=&s"(s0), "+s"(d0) : : "scc");
    // 3: s_cmp + s_cselect chain
    BENCH(3, "s_cmp_ge_u32 %0, %1\n\ts_cselect_b32 %0, %1, %0\n\t", : "+s"(s0) : "s"(s1) : "scc");
    // 4: s_bitcmp1_b64 + s_cselect
    BENCH(4, "s_bitcmp1_b64 %1, %0\n\ts_cselect_b32 %0, 3, 5\n\t", : "+s"(s0) : "s"(d0) : "scc");
    // 5: v_readlane -> dependent s_add (round trip)
    BENCH(5, "v_readlane_b32 %0, %1, 3\n\ts_add_u32 %0, %0, 1\n\tv_mov_b32 %1, %0\n\t", : "+s"(s0), "+v"(v0) : : "scc");
    // 6: independent v_add_u32 (VALU issue rate)
    BENCH(6, "v_add_u32 %0, %0, 1\n\tv_add_u32 %1, %1, 1\n\t", : "+v"(v0), "+v"(v1));
    // 7: dependent v_add_u32 chain
    BENCH(7, "v_add_u32 %0, %0, %1\n\t", : "+v"(v0) : "v"(v1));
    // 8: v_cmp_e64 -> s_and (VALU -> SALU round trip)
    BENCH(8, "v_cmp_ge_u32_e64 %1, %2, %0\n\ts_and_b64 %1, %1, %1\n\ts_ff1_i32_b64 %0, %1\n\t", : "+s"(s0), "=&s"(d0) : "v"(v1) : "scc");
    // 9: taken short forward branch
    BENCH(9, "s_branch 0\n\t", : :);
    // 10: s_cbranch_scc1 not taken
    BENCH(10, "s_cmp_eq_u32 %0, 12345\n\ts_cbranch_scc1 0\n\t", : : "s"(s2) : "scc");
    // 11: v_writelane (SGPR value, m0 lane) independent
    BENCH(11, "v_writelane_b32 %0, %1, 5\n\t", : "+v"(v0) : "s"(s1));
    // 12: v_readlane independent
    BENCH(12, "v_readlane_b32 %0, %1, 5\n\t", : "=s"(s0) : "v"(v1));
    // 13: s_nop 0
    BENCH(13, "s_nop 0\n\t", : :);
    // 14: v_cmp_e64 independent (mask into SGPR pair)
    BENCH(14, "v_cmp_ge_u32_e64 %0, %1, %2\n\t", : "=s"(d0) : "v"(v0), "v"(v1));
    uint64_t e0;
    // 15: s_mov exec (all) + v_add
    BENCH(15, "s_mov_b64 exec, %1\n\tv_add_u32 %0, %0, 1\n\t", : "+v"(v0) : "s"(~0ull));
    // 16: v_cmpx chain (exec &= test) then restore
    BENCH(16, "v_cmpx_le_u32_e32 %1, %0\n\ts_mov_b64 exec, %2\n\t", : "+v"(v0) : "s"(s2), "s"(~0ull) : "vcc");
    // 17: v_cmpx -> s_ff1 exec -> s_lshl -> s_and exec -> v_add -> restore
    BENCH(17, "v_cmpx_le_u32_e32 %2, %0\n\ts_ff1_i32_b64 %1, exec\n\ts_lshl_b64 %4, 1, %1\n\ts_and_b64 exec, exec, %4\n\tv_add_u32 %0, %0, 1\n\ts_mov_b64 exec, %3\n\t",
          : "+v"(v0), "=&s"(s0) : "s"(s2), "s"(~0ull), "s"(d0) : "vcc", "scc");
    // 18: v_readlane -> v_cmp_e64 reading it (VALU SGPR write -> VALU read)
    BENCH(18, "v_readlane_b32 %1, %0, 3\n\tv_cmp_ge_u32_e64 %2, %0, %1\n\tv_add_u32 %0, %0, 1\n\t", : "+v"(v0), "=&s"(s0), "=&s"(e0));
    // 19: v_cmp_e64 -> s_and -> s_ff1 -> s_lshl -> s_and exec -> v_add -> s_mov exec (the execmask chain)
    BENCH(19, "v_cmp_ge_u32_e64 %4, %0, %2\n\ts_and_b64 %4, %4, %4\n\ts_ff1_i32_b64 %1, %4\n\ts_lshl_b64 %4, 1, %1\n\ts_and_b64 exec, exec, %4\n\tv_add_u32 %0, %0, 1\n\ts_mov_b64 exec, %3\n\t",
          : "+v"(v0), "=&s"(s0), "+s"(s2) : "s"(~0ull), "s"(d0) : "vcc", "scc");
    if (threadIdx.x == 0) out[31] = s0 + s1 + d0 + v0 + v1 + e0;
}

int main() {
    uint64_t *d;
    hipMalloc(&d, 32 * 8);
    const char *names[] = {"s_add dep", "s_add x2 indep", "s_ff1_b64+s_lshl_b64 dep", "s_cmp+s_cselect dep",
                           "s_bitcmp1_b64+s_cselect", "v_readlane->s_add->v_mov", "v_add x2 indep", "v_add dep",
                           "v_cmp_e64->s_and->s_ff1", "s_branch taken", "s_cmp+s_cbranch not taken", "v_writelane",
                           "v_readlane", "s_nop 0", "v_cmp_e64", "s_mov exec+v_add", "v_cmpx+s_mov exec",
                           "cmpx->ff1 exec->lshl->and exec->v_add->restore", "v_readlane->v_cmp(sgpr)->v_add",
                           "v_cmp->s_and->ff1->lshl->and exec->v_add->restore"};
    for (int nw : {1, 4}) {
        uint64_t h[32];
        for (int it = 0; it < 3; ++it) {
            k_isa<<<1, 64 * nw>>>(d, 12345);
            hipDeviceSynchronize();
        }
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        printf("waves %d\n", nw);
        for (int i = 0; i < 20; ++i) printf("  %-28s %6.2f cycles per body\n", names[i], (double)h[i] / (16.0 * 32.0));
    }
    return 0;
}
