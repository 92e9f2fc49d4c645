// SCATTER instances of the specialised implicit-GEMM core with bf16 MFMA operands (cv_gemm.hpp,
// MT = MMA_BF16); the shape checks live in cv_gemm_scatter.hip, which forwards here.
#include "cv_gemm.hpp"

namespace cv {

int gemm_fast_scatter_bf16(const Args& a, int BM, int BN, dim3 grid, hipStream_t st) {
  return fast::dispatch_tiles<OP_SCATTER, fast::MMA_BF16>(a, 0, BM, BN, grid, st);
}

}  // namespace cv
