// One k_ffd_pipe instantiation of fp_pipe_tus.h in a translation unit of its own, so that the
// Makefile can compile it under its own LLVM machine scheduler (FFD_TUS: -DFPP_TU_NAME, _G, _BLK,
// _WV, _PK).  fp_pipe.hip (built with FPP_SPLIT) launches it through fpp_tu_launch_<name>.  The
// namespace is renamed per unit, so that the non-template kernels and helpers it also compiles do
// not collide at link time.
#define FPP_KERNEL_TU 1
#define FPP_NS_CAT2(a, b) a##b
#define FPP_NS_CAT(a, b) FPP_NS_CAT2(a, b)
#define fpp FPP_NS_CAT(fpp_tu_, FPP_TU_NAME)
#include "fp_pipe.hip"
