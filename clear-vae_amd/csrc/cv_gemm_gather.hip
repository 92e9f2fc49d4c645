// GATHER instances of the specialised implicit-GEMM core (cv_gemm.hpp); one translation
// unit per op so the instances compile in parallel.
#include "cv_gemm.hpp"

namespace cv {

int gemm_fast_gather(const Args& a, int BM, int BN, dim3 grid, hipStream_t st) {
  if ((a.g.cb % BK) || a.a.nchw || (a.g.cs & 3) || a.g.kh * a.g.kw > 32) return -1;
  // 32-bit element offsets in the kernel
  if ((long)a.g.n * a.g.hb * a.g.wb * a.g.cb >= (1L << 31) || (long)a.g.n * a.g.hs * a.g.ws * a.g.cs >= (1L << 31))
    return -1;
  if (a.mma == CV_MMA_BF16) return gemm_fast_gather_bf16(a, BM, BN, grid, st);
  return fast::dispatch_tiles<OP_GATHER, fast::MMA_F32>(a, 0, BM, BN, grid, st);
}

}  // namespace cv

#ifdef CV_STAMPS
CV_STAMPS_SETTER(cv_debug_set_stamps_gather)
#endif
