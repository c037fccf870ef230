// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths k_ffd_pipe
// uses (MI355X_MICROARCH.md: only 16-B/lane streaming reads and writes are calibrated there).
// Each kernel moves a known number of bytes through HBM once (arrays >> 256 MB Infinity Cache,
// distinct buffers per kernel, every line touched exactly once):
//   r4   4-B/lane coalesced reads            (segment 0's SoA input, one u32 field per array)
//   r16  16-B/lane coalesced reads           (the guide's calibrated case)
//   g4   4-B/lane sparse gathers, increasing  (a link consumer re-reading forwarded containers:
//        positions)                            every 4th u32, so every 64-B half line is touched)
//   w4   4-B/lane coalesced writes           (assign in FFD order, link positions)
//   w1   1-B/lane coalesced writes           (reason in FFD order)
//   w16  16-B/lane coalesced writes
// Run one kernel per process (argv[1]) under `rocprofv3 --pmc FETCH_SIZE` and again under
// `--pmc WRITE_SIZE`; tools/fetchcal.sh collects the counter per kernel and divides by the
// printed byte count.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 fetchcal.hip -o fetchcal
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

constexpr size_t BYTES = 1ull << 30;  // 1 GiB per access stream (4x the Infinity Cache)

__global__ void r4(const uint32_t *__restrict__ a, size_t n, uint32_t *out) {
    uint32_t s = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 0x9E3779B9u) out[0] = s;
}
__global__ void r16(const uint4 *__restrict__ a, size_t n, uint32_t *out) {
    uint32_t s = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        s += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (s == 0x9E3779B9u) out[0] = s;
}
// lane l of wave w reads u32 index 4 * (w * 64 + l): one dword per 16 B, so every 64-B half of
// every 128-B line is touched once
__global__ void g4(const uint32_t *__restrict__ a, size_t n, uint32_t *out) {
    uint32_t s = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; 4 * i < n; i += (size_t)gridDim.x * blockDim.x)
        s += a[4 * i];
    if (s == 0x9E3779B9u) out[0] = s;
}
__global__ void w4(uint32_t *__restrict__ a, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = (uint32_t)i;
}
__global__ void w1(uint8_t *__restrict__ a, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = (uint8_t)i;
}
__global__ void w16(uint4 *__restrict__ a, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

int main(int argc, char **argv) {
    const char *k = argc > 1 ? argv[1] : "r4";
    void *buf = nullptr;
    uint32_t *out = nullptr;
    if (hipMalloc(&buf, BYTES) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    if (hipMemset(buf, 1, BYTES) != hipSuccess) return 1;
    // evict the buffer from the Infinity Cache: stream another 1 GiB through it first
    void *flush = nullptr;
    if (hipMalloc(&flush, BYTES) != hipSuccess || hipMemset(flush, 2, BYTES) != hipSuccess) return 1;
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    const unsigned grid = 256 * 8, block = 256;
    size_t bytes = BYTES;
    if (!strcmp(k, "r4")) r4<<<grid, block>>>((const uint32_t *)buf, BYTES / 4, out);
    else if (!strcmp(k, "r16")) r16<<<grid, block>>>((const uint4 *)buf, BYTES / 16, out);
    else if (!strcmp(k, "g4")) { g4<<<grid, block>>>((const uint32_t *)buf, BYTES / 4, out); bytes = BYTES; }
    else if (!strcmp(k, "w4")) w4<<<grid, block>>>((uint32_t *)buf, BYTES / 4);
    else if (!strcmp(k, "w1")) w1<<<grid, block>>>((uint8_t *)buf, BYTES);
    else if (!strcmp(k, "w16")) w16<<<grid, block>>>((uint4 *)buf, BYTES / 16);
    else return 2;
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    // bytes whose lines the kernel touches (g4 touches every 64-B half line: all of them)
    printf("{\"kernel\": \"%s\", \"bytes\": %zu}\n", k, bytes);
    return 0;
}
