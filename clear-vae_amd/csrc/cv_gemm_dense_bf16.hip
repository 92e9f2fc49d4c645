// DENSE instances of the specialised implicit-GEMM core with bf16 MFMA operands (cv_gemm.hpp,
// MT = MMA_BF16); the shape checks and the B-layout choice live in cv_gemm_dense.hip.
#include "cv_gemm.hpp"

namespace cv {

int gemm_fast_dense_bf16(const Args& a, int xb, int BM, int BN, dim3 grid, hipStream_t st) {
  return fast::dispatch_tiles<OP_DENSE, fast::MMA_BF16>(a, xb, BM, BN, grid, st);
}

}  // namespace cv
