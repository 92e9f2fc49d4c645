// DENSE instances of the specialised implicit-GEMM core (cv_gemm.hpp); one translation
// unit per op so the instances compile in parallel.
#include "cv_gemm.hpp"

namespace cv {

int gemm_fast_dense(const Args& a, int BM, int BN, dim3 grid, hipStream_t st) {
  if ((a.lda & 3) || (a.K & 3) || (a.a_pix > 1 && (a.a_ch & 3))) return -1;
  int xb;
  if (a.wlayout == 1) {
    if ((a.ldb & 3) || (a.N & 3)) return -1;
    xb = fast::DB_NCONT;
  } else if (a.a_pix <= 1) {
    if (a.ldb & 3) return -1;
    xb = fast::DB_KCONT;
  } else {
    xb = fast::DB_KPERM;
  }
  // 32-bit element offsets in the kernel
  if ((long)a.M * a.lda >= (1L << 31) || (long)(a.wlayout ? a.K : a.N) * a.ldb >= (1L << 31)) return -1;
  if (a.mma == CV_MMA_BF16) return gemm_fast_dense_bf16(a, xb, BM, BN, grid, st);
  return fast::dispatch_tiles<OP_DENSE, fast::MMA_F32>(a, xb, BM, BN, grid, st);
}

}  // namespace cv

#ifdef CV_STAMPS
CV_STAMPS_SETTER(cv_debug_set_stamps_dense)
#endif
