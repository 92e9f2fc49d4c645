// Shared definitions of the implicit-GEMM kernels (cv_igemm.hip: generic kernel + host launch;
// cv_gemm.hpp / cv_gemm_*.hip: the specialised MFMA core).
#pragma once
#include "cv_common.hpp"

namespace cv {

constexpr int BK = 32;
#ifndef CV_DEPTH
#define CV_DEPTH 2  // register-ring depth (tiles staged ahead + 1); 3 measured slower (occupancy)
#endif
constexpr int NT = 256;

enum { OP_GATHER = 0, OP_SCATTER = 1, OP_WGRAD = 2, OP_DENSE = 3 };

#ifdef CV_STAMPS
// Instrumented builds only (make stamps): per-block timeline [hw_id][8] u64 =
// {realtime entry, prologue done, main loop done, exit, memtime entry, memtime exit, HW_ID, XCC_ID}
static __device__ unsigned long long* g_stamps;  // one per translation unit
#define CV_STAMPS_SETTER(fn)                                                          \
  extern "C" int fn(void* buf) {                                                      \
    return hipMemcpyToSymbol(HIP_SYMBOL(cv::g_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : 1; \
  }
#define CV_STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memrealtime()
#else
#define CV_STAMP(v)
#endif


struct Args {
  int op;
  Geo g;
  cv_operand a;        // GATHER: big-grid input; SCATTER: small-grid input; WGRAD: small-grid; DENSE: A
  cv_operand b;        // WGRAD: big-grid operand
  const float* w;      // GATHER: packed [tap][cb][cs]; SCATTER: packed [tap][cs][cb]; DENSE: Linear weight
  int wlayout;         // DENSE: 0 -> W[col*ldb + k], 1 -> W[k*ldb + col]
  int ldb;
  const float* bias;
  float* gbias;        // WGRAD: bias gradient via an extra all-ones B column
  float* part;         // WGRAD split-K: partial tiles [split][M][N(+1)] (else fp32 atomics)
  float* out;
  int accumulate;      // atomicAdd into out (split-K)
  cv_epilogue ep;
  int M, N, K;         // GEMM sizes (SCATTER: per class sizes computed in-kernel; N excludes bias col)
  int kchunk;          // K elements per split (multiple of BK)
  int lda, a_pix, a_ch;      // DENSE: A row stride; NCHW-flatten permutation of A columns (a_pix=1: none)
  int ldo, o_pix, o_ch;      // DENSE: out row stride; permutation of output columns
  int ca_n, cb_n, ce_n;      // feature counts of a / b / epilogue BN constants (0 = unused)
  int mma;                   // CV_MMA_FP32 / CV_MMA_BF16 operand precision of the specialised core
  int tiles_x, tiles_y, tiles_z;  // two-tile launch of the specialised core (gemm_kernel2): the tile grid
  // in-launch split-K of an under-filled long-K GATHER (specialised one-tile core only): gridDim.z slices of
  // kchunk; each slice leaves its fragment slab in fix_part, the last of a tile's slices (fix_cnt ticket)
  // sums the slabs in slice order and runs the epilogue.  Null: no split.
  float* fix_part;
  unsigned* fix_cnt;
  // XCD-grouped tile order (specialised core, GATHER / SCATTER without a K split; WGRAD: M-tile-fastest order):
  // hardware workgroup id t runs on XCD t % 8, and every XCD gets a contiguous range of logical tiles enumerated
  // minor-first over the tiles that read the same operand (SCATTER: the s^2 parity classes and N tiles of one
  // small-grid tile; GATHER: the N tiles of one M tile; WGRAD: the M tiles of one (N tile, K split)), so each
  // operand tile is fetched into one XCD's L2 once
  int xcd;
  // two-tile SCATTER launch whose parity classes differ in K (stride 2, odd kernel: 1 / 2 / 2 / 4 taps): the
  // slot -> tile permutation that balances the workgroups' K work (gemm_kernel2).  cls_order: the classes by
  // taps, heaviest first; 0 classes: identity order
  int bal_ncls;
  int cls_order[4];
  // pixel-major tiles (specialised core, cv_gemm_tile.inc): GATHER / SCATTER rows, WGRAD K index ordered
  // pixel-major (r = pixel * n + image) instead of image-major, so a tile of BM | n rows (a K tile of BK | n) sits
  // at ONE pixel; the conv's padding taps (or pixels) are then the same for the whole tile and its K loop skips them
  int pm;
  // fast divisors (filled by finalize_divs at launch)
  FDiv f_cb, f_cs, f_kw, f_ws, f_hws, f_ach, f_opix, f_sdiv, f_s, f_n;
};

// ------------------------------------------------------------------ operand transform helpers
struct XfA {
  const BnFwdC* f;
  const BnBwdC* bw;
};

__device__ __forceinline__ float xf_apply(const cv_operand& o, const XfA& c, int ch, float x, float y) {
  if (o.xf == CV_XF_BNRELU) return bn_relu(x, c.f[ch]);
  if (o.xf == CV_XF_BNBWD) return bn_bwd(x, y, c.bw[ch]);
  return x;
}

__device__ __forceinline__ float4 xf_apply4(const cv_operand& o, const XfA& c, int ch0, float4 v, float4 yy) {
  if (o.xf == CV_XF_NONE) return v;
  v.x = xf_apply(o, c, ch0 + 0, v.x, yy.x);
  v.y = xf_apply(o, c, ch0 + 1, v.y, yy.y);
  v.z = xf_apply(o, c, ch0 + 2, v.z, yy.z);
  v.w = xf_apply(o, c, ch0 + 3, v.w, yy.w);
  return v;
}

// BN constants of an operand into LDS (block-cooperative replica fold; scratch: 4*NT doubles)
__device__ __forceinline__ void fill_consts(const cv_operand& o, int nfeat, float* lds, double* scratch, XfA& c) {
  c.f = reinterpret_cast<const BnFwdC*>(lds);
  c.bw = reinterpret_cast<const BnBwdC*>(lds);
  if (o.xf == CV_XF_BNRELU) {
    BnFwdC* d = reinterpret_cast<BnFwdC*>(lds);
    bn_fold<NT>(o.bn, false, scratch, [&](int f, double s, double q, double, double) {
      if (f < nfeat) d[f] = bn_fwd_const_s(o.bn, f, s, q);
    });
  } else if (o.xf == CV_XF_BNBWD) {
    BnBwdC* d = reinterpret_cast<BnBwdC*>(lds);
    bn_fold<NT>(o.bn, true, scratch, [&](int f, double s, double q, double gs, double gq) {
      if (f < nfeat) d[f] = bn_bwd_const_s(o.bn, f, s, q, gs, gq);
    });
  }
}

__host__ __device__ inline int xf_floats(int xf, int nfeat) {
  if (xf == CV_XF_BNRELU) return 4 * nfeat;
  if (xf == CV_XF_BNBWD) return 5 * nfeat;
  return 0;
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 z4() { return make_float4(0.f, 0.f, 0.f, 0.f); }


// specialised core (cv_gemm.hpp), one translation unit per op; returns -1 when the call is not one it serves
int gemm_fast_gather(const Args& a, int BM, int BN, dim3 grid, hipStream_t st);
int gemm_fast_scatter(const Args& a, int BM, int BN, dim3 grid, hipStream_t st);
int gemm_fast_wgrad(const Args& a, int BM, int BN, dim3 grid, hipStream_t st);
int gemm_fast_dense(const Args& a, int BM, int BN, dim3 grid, hipStream_t st);
// bf16-operand instances (cv_gemm_*_bf16.hip), called by the above when a.mma == CV_MMA_BF16
int gemm_fast_gather_bf16(const Args& a, int BM, int BN, dim3 grid, hipStream_t st);
int gemm_fast_scatter_bf16(const Args& a, int BM, int BN, dim3 grid, hipStream_t st);
int gemm_fast_wgrad_bf16(const Args& a, int BM, int BN, dim3 grid, hipStream_t st);
int gemm_fast_dense_bf16(const Args& a, int xb, int BM, int BN, dim3 grid, hipStream_t st);
// occupancy query: while non-null, a gemm_fast_* call that would launch stores the chosen kernel's
// resident workgroups per CU here instead (and launches nothing)
extern thread_local int* g_fast_occ_query;

}  // namespace cv
