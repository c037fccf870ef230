// Micro-benchmark: one wave's cost of the scalar idioms a windowed FFD resolver would put on the
// placement chain (cycles per body, s_memtime, 32x-unrolled inline asm, one wave alone on its SIMD
// and four waves on one CU).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 lat_salu.hip -o lat_salu
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define R4(x) x x x x
#define R32(x) R4(R4(x)) R4(x) R4(x)

#define BENCH(idx, pro, body, epi, ...)                                        \
    {                                                                           \
        const uint64_t t0 = __builtin_amdgcn_s_memtime();                      \
        for (int i = 0; i < 16; ++i) asm volatile(pro R32(body) epi __VA_ARGS__); \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();                      \
        if (threadIdx.x == 0) out[idx] = t1 - t0;                              \
    }

// SGPR table s[80:87] = (i + 3) & 7, m0 saved in %[sv]
#define TBL_PRO                                                                     \
    "s_mov_b32 %[sv], m0\n\ts_mov_b32 s80, 3\n\ts_mov_b32 s81, 4\n\ts_mov_b32 s82, 5\n\t" \
    "s_mov_b32 s83, 6\n\ts_mov_b32 s84, 7\n\ts_mov_b32 s85, 0\n\ts_mov_b32 s86, 1\n\ts_mov_b32 s87, 2\n\t"
#define TBL_EPI "s_mov_b32 m0, %[sv]\n\t"
#define TBL_CLOB "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "scc", "memory"

__global__ void k_lat(uint64_t *out, uint32_t seed) {
    uint32_t s0 = seed & 7, s1 = seed * 3u, s2 = 5, sv = 0, s3 = 0, s4 = 0, s5 = 0;
    uint64_t d0 = seed, d1 = 0;
    uint32_t v0 = threadIdx.x & 63, v1 = (threadIdx.x * 7u + 1) & 63;
    // 0: dependent s_add_u32 chain
    BENCH(0, "", "s_add_u32 %0, %0, %1\n\t", "", : "+s"(s0) : "s"(s1) : "scc");
    s0 &= 7;
    // 1: dependent s_movrels chain: m0 = x; x = s[80 + m0]
    BENCH(1, TBL_PRO, "s_mov_b32 m0, %[x]\n\ts_movrels_b32 %[x], s80\n\t", TBL_EPI,
          : [x] "+s"(s0), [sv] "+s"(sv) : : TBL_CLOB);
    s0 &= 7;
    // 2: s_ff1 into m0 then s_movrels (index from a mask)
    BENCH(2, TBL_PRO, "s_ff1_i32_b32 m0, %[x]\n\ts_movrels_b32 %[x], s80\n\ts_or_b32 %[x], %[x], 0x100\n\t", TBL_EPI,
          : [x] "+s"(s0), [sv] "+s"(sv) : : TBL_CLOB);
    s0 &= 7;
    // 3: s_movreld write then s_movrels read of the same slot (read-after-write through m0)
    BENCH(3, TBL_PRO, "s_mov_b32 m0, %[x]\n\ts_movreld_b32 s80, %[x]\n\ts_movrels_b32 %[x], s80\n\ts_and_b32 %[x], %[x], 7\n\t", TBL_EPI,
          : [x] "+s"(s0), [sv] "+s"(sv) : : TBL_CLOB);
    s0 &= 7;
    // 4: dependent v_readlane with an SGPR lane select (lane values are lane ids)
    BENCH(4, "", "v_readlane_b32 %0, %1, %0\n\t", "", : "+s"(s0) : "v"(v1));
    // 5: v_readlane -> s_add (SGPR select from the previous s_add)
    BENCH(5, "", "v_readlane_b32 %0, %1, %0\n\ts_and_b32 %0, %0, 63\n\t", "", : "+s"(s0) : "v"(v1) : "scc");
    // 6: four independent readlanes (constant lanes): issue rate
    BENCH(6, "", "v_readlane_b32 %0, %4, 1\n\tv_readlane_b32 %1, %4, 2\n\tv_readlane_b32 %2, %4, 3\n\tv_readlane_b32 %3, %4, 4\n\t", "",
          : "=&s"(s3), "=&s"(s4), "=&s"(s5), "=&s"(s2) : "v"(v1));
    // 7: cmp + not-taken cbranch, dependent s_sub between
    BENCH(7, "", "s_sub_u32 %0, %0, 1\n\ts_cbranch_scc1 0\n\t", "", : "+s"(s1) : : "scc");
    // 8: three not-taken cbranches on independent tests
    BENCH(8, "", "s_and_b32 %1, %0, 0\n\ts_cbranch_scc1 0\n\ts_cmp_gt_u32 %0, -1\n\ts_cbranch_scc1 0\n\ts_cmp_eq_u32 %0, 12345\n\ts_cbranch_scc1 0\n\t", "",
          : "+s"(s2), "=&s"(s3) : : "scc");
    s0 &= 7;
    // 9: the resolver fast path: node = ff1(mask) -> m0, 3 table reads, 3 capacity tests with
    //    not-taken branches, 3 table writes, mask bit clear (the table stays within 0..7)
    BENCH(9, TBL_PRO,
          "s_ff1_i32_b32 m0, %[m]\n\t"
          "s_movrels_b32 %[a], s80\n\t"
          "s_movrels_b32 %[b], s81\n\t"
          "s_movrels_b32 %[c], s82\n\t"
          "s_and_b32 %[t], %[c], 0x100\n\t"
          "s_cbranch_scc1 0\n\t"
          "s_sub_u32 %[a], %[a], 0\n\t"
          "s_cbranch_scc1 0\n\t"
          "s_sub_u32 %[b], %[b], 0\n\t"
          "s_cbranch_scc1 0\n\t"
          "s_movreld_b32 s80, %[a]\n\t"
          "s_movreld_b32 s81, %[b]\n\t"
          "s_or_b32 %[c], %[c], 0\n\t"
          "s_movreld_b32 s82, %[c]\n\t"
          "s_or_b32 %[m], %[m], %[a]\n\t",
          TBL_EPI,
          : [m] "+s"(s2), [a] "=&s"(s3), [b] "=&s"(s4), [c] "=&s"(s5), [t] "=&s"(s1), [sv] "+s"(sv) : : TBL_CLOB);
    // 10: v_cmp_e64 into an SGPR pair -> s_and_b64 -> s_ff1 (VALU -> SALU round trip)
    BENCH(10, "", "v_cmp_ge_u32_e64 %1, %2, %0\n\ts_and_b64 %1, %1, %1\n\ts_ff1_i32_b64 %0, %1\n\t", "",
          : "+s"(s0), "=&s"(d0) : "v"(v1) : "scc");
    // 11: s_bitcmp1_b64 + s_cselect (touched-node test)
    BENCH(11, "", "s_bitcmp1_b64 %1, %0\n\ts_cselect_b32 %0, 3, 5\n\t", "", : "+s"(s0) : "s"(d1) : "scc");
    // 12: s_lshl_b64 + s_or_b64 (bit set through a computed mask) dependent
    BENCH(12, "", "s_lshl_b64 %1, 1, %0\n\ts_or_b64 %2, %2, %1\n\ts_ff1_i32_b64 %0, %2\n\t", "",
          : "+s"(s0), "=&s"(d0), "+s"(d1) : : "scc");
    // 13: v_writelane with an SGPR lane select (m0) independent
    BENCH(13, "s_mov_b32 %[sv], m0\n\ts_mov_b32 m0, 5\n\t", "v_writelane_b32 %[v], %[x], m0\n\t", "s_mov_b32 m0, %[sv]\n\t",
          : [v] "+v"(v0), [sv] "+s"(sv) : [x] "s"(s1));
    if (threadIdx.x == 0) out[31] = s0 + s1 + s2 + s3 + s4 + s5 + d0 + d1 + v0 + v1 + sv;
}

int main() {
    uint64_t *d;
    hipMalloc(&d, 32 * 8);
    const char *names[] = {"s_add dep", "s_movrels chain (m0=x; x=tbl[m0])", "s_ff1->m0->s_movrels->s_or",
                           "movreld+movrels same slot", "v_readlane(sel=prev) chain", "v_readlane->s_and chain",
                           "4x v_readlane indep", "s_sub+cbranch not taken dep", "3x test+cbranch not taken",
                           "resolver fast path (15 SALU, 3 br)", "v_cmp_e64->s_and->s_ff1", "s_bitcmp1+s_cselect",
                           "s_lshl_b64+s_or_b64+s_ff1 dep", "v_writelane (m0 lane)"};
    for (int nw : {1, 4}) {
        uint64_t h[32];
        for (int it = 0; it < 3; ++it) {
            k_lat<<<1, 64 * nw>>>(d, 12345);
            if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
        }
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        printf("waves %d\n", nw);
        for (int i = 0; i < 14; ++i) printf("  %-38s %7.2f cycles per body\n", names[i], (double)h[i] / (16.0 * 32.0));
    }
    return 0;
}
