// WGRAD instances of the specialised implicit-GEMM core with bf16 MFMA operands (cv_gemm.hpp,
// MT = MMA_BF16); the shape checks live in cv_gemm_wgrad.hip, which forwards here.
#include "cv_gemm.hpp"

namespace cv {

int gemm_fast_wgrad_bf16(const Args& a, int BM, int BN, dim3 grid, hipStream_t st) {
  return fast::dispatch_tiles<OP_WGRAD, fast::MMA_BF16>(a, a.b.xf, BM, BN, grid, st);
}

}  // namespace cv
