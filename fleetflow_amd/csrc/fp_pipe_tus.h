// The k_ffd_pipe instantiations compiled in translation units of their own (fp_pipe_tu.hip, one
// object per entry, each under the LLVM machine scheduler the Makefile's FFD_TUS gives it).
// X(name, G, BLK, WV, PK):
//   big / bigp  the 4096-scenario kernel (one-wave 12-group segments, six waves per SIMD), u32 / packed
//   w12 / w12p  one-wave 12-group segments at five waves per SIMD (2048-scenario loads, bounded rings)
//   m8  / m8p   2-stage segments of 8 groups (1024-scenario loads)
//   m10 / m10p  4-stage segments of 10 groups (512-scenario loads)
//   n1  / n1p   one-group stages (configs 2, 3, 5: few scenarios)
// fp_pipe.hip (FPP_SPLIT) launches these through fpp_tu_launch_<name>; every other geometry is
// instantiated in fp_pipe.hip itself (u32 only).  tests/test_rust_binding.py checks that this list
// and the Makefile's FFD_TUS name the same kernels.
#pragma once

#define FPP_TUS(X)            \
    X(big, 12, 64, 6, 0)      \
    X(bigp, 12, 64, 6, 1)     \
    X(w12, 12, 64, 0, 0)      \
    X(w12p, 12, 64, 0, 1)     \
    X(m8, 8, 1024, 0, 0)      \
    X(m8p, 8, 1024, 0, 1)     \
    X(m10, 10, 1024, 0, 0)    \
    X(m10p, 10, 1024, 0, 1)   \
    X(n1, 1, 1024, 0, 0)      \
    X(n1p, 1, 1024, 0, 1)
