// The 4096-scenario FFD kernel alone (k_ffd_pipe<12, 64, WIDE12_BIG_WAVES>), so that the Makefile
// can compile it under its own LLVM scheduling strategy; fp_pipe.hip (built with FPP_SPLIT_BIG)
// launches it through fpp::launch_wide12_big.  Everything else of fp_pipe.hip is excluded here.
// Its namespace is renamed so that the non-template kernels and helpers it also compiles do not
// collide with fp_pipe.hip's at link time.
#define FPP_BIG_TU 1
#define fpp fpp_big
#include "fp_pipe.hip"
