// Image-edge convolutions on gfx950: the layers with <= 4 channels on the big-grid side, i.e. the
// first Conv2d on the image (code/src/models/vae.py:15-16 / :113-114) and the last ConvTranspose2d
// back to it (vae.py:43 / :153), in all three directions.
//
// As implicit GEMMs these have K (gather), N (scatter) or N (wgrad) of 9..48: every MFMA tile would be
// mostly padding and the per-element im2col address arithmetic of the generic kernels dominates.
// Here a workgroup owns one image band: it stages the band's input rows ONCE in LDS with the fused
// BatchNorm transform applied (zero halo = the conv's zero padding, which the reference applies to
// the transformed activation), the weights next to them, and then every output element is a short
// dot product over LDS words that are either broadcast (weights, wave-uniform taps) or bank-spread
// (activation rows at a padded pitch).  Global traffic is the activation tensors once each.
//
//   edge_gather : out[small px][32] = sum_{tap, c<CB} T(big[gather(px, tap)][c]) * Wg[tap][c][32]
//                 (Conv2d forward on the image; ConvTranspose2d-to-image backward-data)
//   edge_scatter: out[big px][CB]  = sum_{tap in parity class, ch<32} T(small[..][ch]) * Ws[tap][ch][CB]
//                 (ConvTranspose2d-to-image forward), one wave per stride-parity class
//   edge_wgrad  : part[blk][o][tap*CB + c] = sum_{px in blk} T(small[px][o]) * T(big[gather(px,tap)][c])
//                 (both layers' weight gradients, + the conv bias column); the split partials are
//                 summed by cv_igemm.hip's wgrad_reduce_kernel
#include <stdlib.h>
#include "cv_common.hpp"

namespace cv {

int wgrad_reduce_launch(const float* part, int split, int M, int N, int ntot, int cb, int kk, float* gw,
                        float* gbias, hipStream_t st);

namespace edge {

#ifdef CV_STAMPS
// instrumented builds only (make stamps): per-workgroup phase timeline [wg][8] u64 (s_memrealtime, 100 MHz),
// the same layout as cv_direct.hip's: {entry, weights + constants, staged, MFMA done, stores issued, exit, HW_ID,
// XCC_ID}
static __device__ unsigned long long* g_estamps;
#define CV_ESTAMP(v) const unsigned long long v = __builtin_amdgcn_s_memrealtime()
#define CV_ESTAMP_WRITE()                                                                                 \
  if (threadIdx.x == 0 && g_estamps) {                                                                    \
    const unsigned long long st5 = __builtin_amdgcn_s_memrealtime();                                      \
    unsigned long long* o = g_estamps + (size_t)(blockIdx.x + gridDim.x * blockIdx.y) * 8;                \
    o[0] = st0; o[1] = st1; o[2] = st2; o[3] = st3; o[4] = st4; o[5] = st5;                               \
    o[6] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));                                        \
    o[7] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11));                                       \
  }
#else
#define CV_ESTAMP(v)
#define CV_ESTAMP_WRITE()
#endif

constexpr int ET = 256;
__device__ __forceinline__ f32x4 lds4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
constexpr int CS = 32;   // small-grid channels served
constexpr int SP = 36;   // LDS pitch (floats) of a 32-channel pixel: 16 lanes of b128 reads cover all 64 banks

struct EArgs {
  Geo g;
  cv_operand big;    // <= 4-channel image-side operand
  cv_operand small;  // 32-channel operand (scatter input / wgrad)
  const float* w;
  const float* bias;
  float* out;        // gather/scatter output; wgrad partials [blk][32][ncol]
  cv_epilogue ep;
  int rows;          // gather / wgrad: small rows per band; scatter: big rows per band
  int ipb;           // wgrad: images per workgroup; scatter: small rows staged per band (max)
  int ncol;          // wgrad: columns (KK*KK*CB, + 1 for the bias)
};

// constants of a fused operand transform into LDS (kf for BNRELU, kb for BNBWD), features < C;
// finalised producer constants are copied when their ticket says they exist
__device__ __forceinline__ void xf_consts(const cv_operand& o, BnFwdC* kf, BnBwdC* kb, double* scratch) {
  const cv_bn& b = o.bn;
  if (o.xf == CV_XF_BNRELU) {
    if (b.train && b.cfwd && b.ticket && b.ticket[0] != 0u) {
      for (int f = threadIdx.x; f < b.C; f += ET) {
        BnFwdC k;
        k.sc = b.cfwd[f];
        k.mu = b.cfwd[b.C + f];
        k.be = b.cfwd[2 * b.C + f];
        k.istd = b.cfwd[3 * b.C + f];
        kf[f] = k;
      }
      __syncthreads();
    } else {
      bn_fold<ET>(b, false, scratch, [&](int f, double s, double q, double, double) { kf[f] = bn_fwd_const_s(b, f, s, q); });
    }
  } else if (o.xf == CV_XF_BNBWD) {
    if (b.train && b.cbwd && b.ticket && b.ticket[1] != 0u) {
      for (int f = threadIdx.x; f < b.C; f += ET) {
        BnBwdC k;
        k.sc = b.cbwd[f];
        k.c1 = b.cbwd[b.C + f];
        k.mu = b.cbwd[2 * b.C + f];
        k.istd = b.cbwd[3 * b.C + f];
        k.c2 = b.cbwd[4 * b.C + f];
        kb[f] = k;
      }
      __syncthreads();
    } else {
      bn_fold<ET>(b, true, scratch, [&](int f, double s, double q, double gs, double gq) {
        kb[f] = bn_bwd_const_s(b, f, s, q, gs, gq);
      });
    }
  }
}

__device__ __forceinline__ float xf_apply(int xf, float x, float y, int c, const BnFwdC* kf, const BnBwdC* kb) {
  if (xf == CV_XF_BNRELU) return bn_relu(x, kf[c]);
  if (xf == CV_XF_BNBWD) return bn_bwd(x, y, kb[c]);
  return x;
}

constexpr int BU = 16;  // elements of x (and y) per thread per batch of stage_big (VAE64 gather band: 14)
// one batch of stage_big's loads from element `base` (zero outside the image; ok = inside)
template <int CB, bool Y = true>
__device__ __forceinline__ void big_load(const Geo& g, const cv_operand& o, int n, int yb0, int xb0, int NR, int NC,
                                         int base, float (&v)[BU], float* yv) {
  const int tot = NR * NC * CB;
  const FDiv fnc = FDiv::make(NC);
#pragma unroll
  for (int q = 0; q < BU; ++q) {
    const int i = base + q * ET;
    const int c = i % CB, rc = i / CB;
    const int rr = fnc.div(rc), cc = rc - rr * NC;
    const int yb = yb0 + rr, xb = xb0 + cc;
    v[q] = 0.f;
    if (Y) yv[q] = 0.f;
    if (i < tot && (unsigned)yb < (unsigned)g.hb && (unsigned)xb < (unsigned)g.wb) {
      const size_t off = o.nchw ? ((size_t)(n * CB + c) * g.hb + yb) * g.wb + xb
                                : ((size_t)(n * g.hb + yb) * g.wb + xb) * CB + c;
      v[q] = o.x[off];
      if (Y && o.xf == CV_XF_BNBWD) yv[q] = o.y[off];
    }
  }
}
// Stage rows [yb0, yb0+NR) x cols [xb0, xb0+NC) x CB of image n of the big-grid operand, transformed,
// zero outside the image (the conv's zero padding of the transformed tensor), as dst[(rr*NC + cc)*CB + c].
// PRE: the first batch was requested earlier (big_load at base = threadIdx.x into pv / py).
template <int CB, bool PRE = false>
__device__ __forceinline__ void stage_big(const Geo& g, const cv_operand& o, int n, int yb0, int xb0, int NR, int NC,
                                          const BnFwdC* kf, const BnBwdC* kb, float* dst, const float* pv = nullptr,
                                          const float* py = nullptr) {
  const int tot = NR * NC * CB;
  const FDiv fnc = FDiv::make(NC);
  for (int base = threadIdx.x; base < tot; base += ET * BU) {
    float v[BU], yv[BU];
    if (PRE && base == (int)threadIdx.x) {
#pragma unroll
      for (int q = 0; q < BU; ++q) {
        v[q] = pv[q];
        yv[q] = py ? py[q] : 0.f;
      }
    } else {
      big_load<CB>(g, o, n, yb0, xb0, NR, NC, base, v, yv);
    }
#pragma unroll
    for (int q = 0; q < BU; ++q) {
      const int i = base + q * ET;
      const int c = i % CB, rc = i / CB;
      const int rr = fnc.div(rc), cc = rc - rr * NC;
      const bool ok = (unsigned)(yb0 + rr) < (unsigned)g.hb && (unsigned)(xb0 + cc) < (unsigned)g.wb;
      if (i < tot) dst[i] = ok ? xf_apply(o.xf, v[q], yv[q], c, kf, kb) : 0.f;
    }
  }
}

// Stage small-grid pixels [p0, p0+np) of image n (32 channels, NHWC) transformed, as dst[px*PITCH + ch].
// Thread t always handles the channel quad 4 (t & 7) (ET is a multiple of 8), so its transform constants
// are read from LDS once, into registers (reading them per element cost 2-way-conflicted LDS reads per
// value); up to U float4 of x (and y) per thread are requested before the first transform.
constexpr int SU = 8;  // float4 of x (and y) per thread per batch of stage_small
// The first batch (base = threadIdx.x) of stage_small's loads, issued before the transform constants exist
// (stage_small<PITCH, true> then starts from these registers): the kernel's prologue round trips overlap.
// (Y: also the pre-BN tensor of a BN-backward operand)
template <bool Y>
__device__ __forceinline__ void small_prefetch(const Geo& g, const cv_operand& o, int n, int p0, int np, float4 (&v)[SU],
                                               float4* yv) {
  const int tot4 = np * (CS / 4);
  const float4* x4 = reinterpret_cast<const float4*>(o.x + ((size_t)n * g.hs * g.ws + p0) * CS);
  const float4* y4 = reinterpret_cast<const float4*>(o.y ? o.y + ((size_t)n * g.hs * g.ws + p0) * CS : nullptr);
#pragma unroll
  for (int q = 0; q < SU; ++q) {
    const int i = threadIdx.x + q * ET;
    v[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (Y) yv[q] = v[q];
    if (i < tot4) {
      v[q] = x4[i];
      if (Y) yv[q] = y4[i];
    }
  }
}
template <int PITCH, bool PRE = false>
__device__ __forceinline__ void stage_small(const Geo& g, const cv_operand& o, int n, int p0, int np,
                                            const BnFwdC* kf, const BnBwdC* kb, float* dst,
                                            const float4* pv = nullptr, const float4* py = nullptr) {
  constexpr int U = SU;
  const int tot4 = np * (CS / 4);
  const int c0 = (threadIdx.x & 7) * 4;
  BnFwdC f[4];
  BnBwdC b[4];
  if (o.xf == CV_XF_BNRELU) {
#pragma unroll
    for (int k = 0; k < 4; ++k) f[k] = kf[c0 + k];
  } else if (o.xf == CV_XF_BNBWD) {
#pragma unroll
    for (int k = 0; k < 4; ++k) b[k] = kb[c0 + k];
  }
  const float4* x4 = reinterpret_cast<const float4*>(o.x + ((size_t)n * g.hs * g.ws + p0) * CS);
  const float4* y4 = reinterpret_cast<const float4*>(o.y ? o.y + ((size_t)n * g.hs * g.ws + p0) * CS : nullptr);
  for (int base = threadIdx.x; base < tot4; base += ET * U) {
    float4 v[U], yv[U];
    if (PRE && base == (int)threadIdx.x) {
#pragma unroll
      for (int q = 0; q < U; ++q) {
        v[q] = pv[q];
        yv[q] = py ? py[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    } else {
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const int i = base + q * ET;
        v[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        yv[q] = v[q];
        if (i < tot4) {
          v[q] = x4[i];
          if (o.xf == CV_XF_BNBWD) yv[q] = y4[i];
        }
      }
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int i = base + q * ET;
      if (i < tot4) {
        const int px = i >> 3;
        float4 r = v[q];
        if (o.xf == CV_XF_BNRELU) {
          r.x = bn_relu(r.x, f[0]);
          r.y = bn_relu(r.y, f[1]);
          r.z = bn_relu(r.z, f[2]);
          r.w = bn_relu(r.w, f[3]);
        } else if (o.xf == CV_XF_BNBWD) {
          r.x = bn_bwd(r.x, yv[q].x, b[0]);
          r.y = bn_bwd(r.y, yv[q].y, b[1]);
          r.z = bn_bwd(r.z, yv[q].z, b[2]);
          r.w = bn_bwd(r.w, yv[q].w, b[3]);
        }
        *reinterpret_cast<float4*>(dst + px * PITCH + c0) = r;
      }
    }
  }
}

// Sum NC per-thread (s1, s2) channel statistics over the workgroup and add them (fp64) to one replica.
template <int NC>
__device__ __forceinline__ void stats_out(const float* s1, const float* s2, double* stat_out, int C, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const float a = wave_sum(s1[j]), b = wave_sum(s2[j]);
    if (lane == 0) {
      red[w * 2 * NC + j] = a;
      red[w * 2 * NC + NC + j] = b;
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * NC) {
    const int j = threadIdx.x;
    double v = 0.0;
#pragma unroll
    for (int q = 0; q < ET / 64; ++q) v += (double)red[q * 2 * NC + j];
    const int ch = j < NC ? j : j - NC;
    if (ch < C) {
      const int repl = (blockIdx.y * gridDim.x + blockIdx.x) % CV_STAT_REPL(C);
      atomic_add_f64(stat_out + (size_t)repl * 2 * C + (j < NC ? 0 : C) + ch, v);
    }
  }
}

// ---------------------------------------------------------------- gather (32 outputs per pixel)
// The band's <= 256 pixels x 32 outputs x K = KK*KK*CB taps is a small dense GEMM: v_mfma_f32_16x16x4_f32
// with the weights (B, <= 48 x 32) held as fragments in registers for the whole kernel and the
// im2col operand (A) read straight out of the staged band: wave w owns pixels [64w, 64w+64) as four
// 16-row tiles, lane l reads pixel 16i + (l&15) at tap-channel k = 4s + (l>>4).
constexpr int GP = 36;  // LDS pitch (floats) of the gather's output tile
template <int CB, int KK>
__global__ __launch_bounds__(ET, 3) void edge_gather_kernel(const EArgs P) {
  constexpr int NK = KK * KK * CB;
  constexpr int KS = (NK + 3) / 4;  // k-steps
  __shared__ BnFwdC kf[4];
  __shared__ BnBwdC kb[4];
  __shared__ BnFwdC ke[CS];
  __shared__ float red[ET / 64][2][CS];
  extern __shared__ __attribute__((aligned(16))) float sIn[];
  const Geo& g = P.g;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = blockIdx.y;
  const int r0 = blockIdx.x * P.rows;
  const int R = min(P.rows, g.hs - r0);
  const int NC = (g.ws - 1) * g.s + KK;
  const int NR = (R - 1) * g.s + KK;
  // B fragments: W[k = 4s + (l>>4)][n = 16j + (l&15)], packed gather layout [tap][cb][cs] = [k][32]
  float bw[KS][2];
  const int kq = lane >> 4, nl = lane & 15;
#pragma unroll
  for (int st = 0; st < KS; ++st) {
    const int k = 4 * st + kq;
#pragma unroll
    for (int j = 0; j < 2; ++j) bw[st][j] = (k < NK) ? P.w[k * CS + 16 * j + nl] : 0.f;
  }
  // this lane's tap-channel offsets inside a receptive field, per k-step
  int koff[KS];
#pragma unroll
  for (int st = 0; st < KS; ++st) {
    const int k = 4 * st + kq;
    const int tap = k / CB, c = k - tap * CB, kh = tap / KK, kw = tap - kh * KK;
    koff[st] = (k < NK) ? (kh * NC + kw) * CB + c : 0;
  }
  // the band's first batch is requested before the constants (x-only operands: the register budget keeps
  // 3 workgroups per CU; a BN-backward operand stages after them)
  float bv[BU];
  const bool pre = P.big.xf != CV_XF_BNBWD;
  if (pre) big_load<CB, false>(g, P.big, n, r0 * g.s - g.p, -g.p, NR, NC, t, bv, nullptr);
  double* scratch = reinterpret_cast<double*>(sIn);  // (fold scratch: the staging area, unused yet)
  xf_consts(P.big, kf, kb, scratch);
  const int mode = P.ep.stat_mode;
  if (mode == CV_STAT_BWD) {
    cv_operand eo;
    eo.xf = CV_XF_BNRELU;
    eo.bn = P.ep.ebn;
    __syncthreads();
    xf_consts(eo, ke, nullptr, scratch);
  }
  __syncthreads();
  if (pre) stage_big<CB, true>(g, P.big, n, r0 * g.s - g.p, -g.p, NR, NC, kf, kb, sIn, bv, nullptr);
  else stage_big<CB>(g, P.big, n, r0 * g.s - g.p, -g.p, NR, NC, kf, kb, sIn);
  __syncthreads();
  const int npx = R * g.ws;
  int abase[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int px = 64 * w + 16 * i + nl;
    const int rl = px / g.ws, xs = px - rl * g.ws;
    abase[i] = (px < npx) ? ((rl * g.s) * NC + xs * g.s) * CB : 0;
  }
  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (64 * w < npx) {
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      float a[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = sIn[abase[i] + koff[st]];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], bw[st][j], acc[i][j], 0, 0, 0);
    }
  }
  // epilogue through LDS: the fragments (lane: rows 4*(l>>4) + r of each 16-row tile, column 16j + (l&15))
  // are parked in a [px][GP] tile, then every thread streams 16-byte chunks of the band's output (one
  // contiguous NHWC range) with the bias, the ReLU mask / statistics of the epilogue, and 16-byte loads of
  // the epilogue's pre-BN tensor.  A chunk's 4 channels are c0 = 4 (t & 7) + 0..3 for every chunk a
  // thread takes (ET is a multiple of 8), so each thread accumulates the statistics of 4 fixed channels.
  __syncthreads();  // (every wave is done with the staged band)
  float* sT = sIn;
  if (64 * w < npx) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int px = 64 * w + 16 * i + 4 * kq + r;
        if (px >= npx) continue;
#pragma unroll
        for (int j = 0; j < 2; ++j) sT[px * GP + 16 * j + nl] = acc[i][j][r];  // (GP = 36: 4 rows -> 64 banks)
      }
  }
  __syncthreads();
  const int c0 = 4 * (t & 7);
  f32x4 b4 = f32x4{0.f, 0.f, 0.f, 0.f};
  if (P.bias) b4 = f32x4{P.bias[c0], P.bias[c0 + 1], P.bias[c0 + 2], P.bias[c0 + 3]};
  BnFwdC kc[4];
  if (mode == CV_STAT_BWD) {
#pragma unroll
    for (int k = 0; k < 4; ++k) kc[k] = ke[c0 + k];
  }
  f32x4 s1 = f32x4{0.f, 0.f, 0.f, 0.f}, s2 = s1;
  const size_t pimg = ((size_t)n * g.hs + r0) * g.ws;
  const int nq = npx * (CS / 4);
  constexpr int UQ = 4;
  for (int q0 = t; q0 < nq; q0 += ET * UQ) {
    f32x4 y4[UQ];
    if (mode == CV_STAT_BWD) {
#pragma unroll
      for (int u = 0; u < UQ; ++u) {
        const int q = q0 + u * ET;
        y4[u] = q < nq ? *reinterpret_cast<const f32x4*>(P.ep.ey + (pimg + (q >> 3)) * CS + c0) : s1;
      }
    }
#pragma unroll
    for (int u = 0; u < UQ; ++u) {
      const int q = q0 + u * ET;
      if (q >= nq) continue;
      const int px = q >> 3;
      f32x4 v = lds4(sT + px * GP + c0) + b4;
      if (mode == CV_STAT_BWD) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (P.ep.erelu && bn_out(y4[u][k], kc[k]) <= 0.f) v[k] = 0.f;
          s1[k] += v[k];
          s2[k] += v[k] * ((y4[u][k] - kc[k].mu) * kc[k].istd);
        }
      } else if (mode == CV_STAT_FWD) {
        s1 += v;
        s2 += v * v;
      }
      *reinterpret_cast<f32x4*>(P.out + (pimg + px) * CS + c0) = v;
    }
  }
  if (mode != CV_STAT_NONE) {
    // lanes l, l^8, l^16, ..., l^56 hold the same 4 channels: fold them, then the waves in wave order
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int m = 8; m < 64; m <<= 1) {
        s1[k] += __shfl_xor(s1[k], m, 64);
        s2[k] += __shfl_xor(s2[k], m, 64);
      }
    }
    __syncthreads();  // (red aliases nothing, but the tile reads above must be complete before reuse below)
    if (lane < 8) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        red[w][0][c0 + k] = s1[k];
        red[w][1][c0 + k] = s2[k];
      }
    }
    __syncthreads();
    if (t < 2 * CS) {
      const int q = t / CS, col = t - q * CS;
      double v = 0.0;
#pragma unroll
      for (int ww = 0; ww < ET / 64; ++ww) v += (double)red[ww][q][col];
      const int repl = (blockIdx.y * gridDim.x + blockIdx.x) % CV_STAT_REPL(CS);
      atomic_add_f64(P.ep.stat_out + (size_t)repl * 2 * CS + q * CS + col, v);
    }
  }
}

// ---------------------------------------------------------------- scatter (CB outputs per pixel)
// ConvTranspose2d to the image (stride 2) as a gather GEMM over 2x2 output blocks.  Block (by, bx) holds
// the four big pixels (2 by - p + cy, 2 bx - p + cx), cy, cx in {0, 1} — one of each stride-parity class
// — and every one of them is fed by the same 2x2 small neighbourhood (by - 1 + dy, bx - 1 + dx) through
// tap (kh, kw) = (cy + 2 - 2 dy, cx + 2 - 2 dx) (yb = 2 ys - p + kh; taps >= KK have zero weight).  So
// the layer is one dense contraction on v_mfma_f32_16x16x4_f32: M = blocks, K = 4 neighbours x 32
// channels, N = 4 classes x CB output channels (12 of 16 columns for CB = 3), the weights held as B
// fragments in registers for the whole kernel and the A fragments read from the band's small rows
// staged in LDS (BN + ReLU applied once there).  Blocks partition the big pixels, so every output is
// written once, with its bias, into an LDS tile of the band's big rows, which leave in 16-byte stores
// (one contiguous NHWC range) together with the statistics epilogue.
// (Round 2 ran this layer as per-class VALU dot products — 4x the FMAs' own instruction count issued,
// ~54 us on the VAE64 layer; a col2im variant through LDS read-modify-writes measured 70 us.)
// The decoder output (cv_output_loss: the output BatchNorm2d + Sigmoid, vae.py:44-45 / :154-155, the reconstruction
// term and its backward seed, losses.py:41-47) fused behind the ConvT-to-image forward (OUT = true): every
// workgroup publishes its band's BN sums, waits until all have (the host launches this form only when the whole
// grid is resident at once; the wait is bounded, a timeout sets g_eo_sync[3] and proceeds), folds the output
// BN's constants and turns its band — still in LDS — into x_hat, the reconstruction sum and dv, with the
// arithmetic of output_loss_kernel.  The last workgroup out resets the counters.
// One-channel image (CB = 1: MNIST's decoder output): only 4 of the 16 MFMA columns would carry a class, so the
// contraction runs on v_mfma_f32_4x4x1f32 instead, A (the 4 classes' weights, from lanes 0..3) broadcast to the 16
// blocks and B = one staged small-grid value per lane: lane l accumulates all four classes of image block l of a
// 64-block tile (4x fewer MFMA cycles per block than the 16-column tile).  The weights stay in LDS, [class][q*32 + ch]
// at pitch WKP4, behind the output tile, followed by one zero pixel that out-of-image neighbours read.
constexpr int WKP4 = 4 * CS + 4;
__host__ __device__ constexpr int m4_off(int ipb, int ws, int rb, int wb) {
  const int e = ipb * ws * SP + 2 * rb * wb;  // staged rows + the output tile (CB = 1)
  const int lo = 4 * ET * (int)(sizeof(double) / sizeof(float));  // (clear of the BN fold scratch: 4 ET doubles)
  return ((e > lo ? e : lo) + 3) & ~3;
}
constexpr int M4_EXTRA = 4 * WKP4 + SP;  // floats

struct OArgs {
  cv_bn bn;               // the output BatchNorm2d (this launch's statistics epilogue fills its sums)
  const float* x;         // [n][CB][hb][wb] the input batch (NCHW)
  float* xhat;            // NCHW
  double* rec_out;        // [CV_REC_REPL] += sum (xhat - x)^2 / n
  float* dv;              // NHWC backward seed (nullptr: forward only)
  double* gstat;          // [REPL][2][CB] backward sums
  const float* rec_scale;
};
__device__ unsigned g_eo_sync[4];  // [0] arrivals, [1] finishes, [3] timeout flag

template <int CB, int KK, bool OUT, bool M4 = CB == 1>
__global__ __launch_bounds__(ET, OUT ? 4 : 1) void edge_scatter_kernel(const EArgs P, const OArgs O) {
  constexpr int NCOL = 4 * CB;  // GEMM columns: class (2 cy + cx) * CB + output channel
  static_assert(NCOL <= 16 && KK <= 4, "one 16-column tile; taps cy + 2 - 2 dy < 4");
  __shared__ BnFwdC kf[CS];
  __shared__ BnBwdC kb[CS];
  __shared__ float sb[4];
  __shared__ float red[(ET / 64) * 2 * 4];
  extern __shared__ __attribute__((aligned(16))) float sIn[];
  const Geo& g = P.g;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, kq = lane >> 4, nl = lane & 15;
  const int n = blockIdx.y;
  const int nby = (g.hb - 1 + g.p) / 2 + 1, nbx = (g.wb - 1 + g.p) / 2 + 1;  // block rows / columns
  const int bb0 = blockIdx.x * P.rows;
  CV_ESTAMP(st0);
  const int RBb = min(P.rows, nby - bb0);
  // small rows [ys_lo, ys_hi] feed block rows [bb0, bb0 + RBb); big rows [yb0, yb1) are the band's output
  const int ys_lo = max(bb0 - 1, 0), ys_hi = min(bb0 + RBb - 1, g.hs - 1);
  const int nrs = ys_hi - ys_lo + 1;
  const int yb0 = max(2 * bb0 - g.p, 0), yb1 = min(2 * (bb0 + RBb) - g.p, g.hb);
  float* sOut = sIn + (size_t)P.ipb * g.ws * SP;  // [yb1 - yb0][wb][CB]
  // B fragments: neighbour q = 2 dy + dx, k-step s: lane (kq, nl) holds W[tap(q, class nl / CB)][ch 8 kq + s][nl % CB].
  // The block matrix W'[col][q * 32 + ch] is built once per workgroup in LDS from the packed scatter layout
  // [tap][cs][cb] (coalesced reads of the KK*KK*32*CB weights), pitch WKP: the 16 lanes of a b128 read hit
  // 16 disjoint 4-bank groups
  constexpr int WKP = 4 * CS + 4;
  static_assert(!M4 || CB == 1, "the 4x4x1 form serves one output channel");
  float* sW4 = sIn + m4_off(P.ipb, g.ws, P.rows, g.wb);  // (M4) [4][WKP4], then the zero pixel
  float* sZ = sW4 + 4 * WKP4;
  // the block-matrix weights: all 8 per thread in flight
  float* sWb = M4 ? sW4 : sIn + 4 * ET * 2;  // [16][WKP] behind the fold scratch, inside the (not yet used) staging area
  if constexpr (M4) {
    constexpr int NW4 = 4 * 4 * CS / ET;
    static_assert(NW4 * ET == 4 * 4 * CS, "class weights: whole rounds of ET");
    float wv[NW4];
#pragma unroll
    for (int r = 0; r < NW4; ++r) {
      const int i = t + r * ET;
      const int c2 = i / (4 * CS), k = i - c2 * (4 * CS), q = k / CS, ch = k - q * CS;
      const int kh = (c2 >> 1) + 2 - 2 * (q >> 1), kw = (c2 & 1) + 2 - 2 * (q & 1);
      wv[r] = (kh < KK && kw < KK) ? P.w[(kh * KK + kw) * CS + ch] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < NW4; ++r) {
      const int i = t + r * ET;
      const int c2 = i / (4 * CS), k = i - c2 * (4 * CS);
      sW4[c2 * WKP4 + k] = wv[r];
    }
    if (t < SP) sZ[t] = 0.f;
  } else {
    constexpr int NWB = 16 * 4 * CS / ET;
    static_assert(NWB * ET == 16 * 4 * CS, "block matrix: whole rounds of ET");
    float wv[NWB];
#pragma unroll
    for (int r = 0; r < NWB; ++r) {
      const int i = t + r * ET;
      const int col = i / (4 * CS), k = i - col * (4 * CS), q = k / CS, ch = k - q * CS;
      const int c2 = col / CB, c3 = col - c2 * CB;
      const int kh = (c2 >> 1) + 2 - 2 * (q >> 1), kw = (c2 & 1) + 2 - 2 * (q & 1);
      wv[r] = (col < NCOL && kh < KK && kw < KK) ? P.w[((kh * KK + kw) * CS + ch) * CB + c3] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < NWB; ++r) {
      const int i = t + r * ET;
      const int col = i / (4 * CS), k = i - col * (4 * CS);
      sWb[col * WKP + k] = wv[r];
    }
  }
  const int cls = nl / CB, cb = nl - cls * CB, cy = cls >> 1, cx = cls & 1;
  if (t < CB) sb[t] = P.bias ? P.bias[t] : 0.f;
  xf_consts(P.small, kf, kb, reinterpret_cast<double*>(sIn));  // (fold scratch: the staging area, unused yet)
  __syncthreads();
  CV_ESTAMP(st1);
  float bw[4][8];
  if constexpr (!M4) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 w0 = lds4(sWb + nl * WKP + q * CS + 8 * kq), w1 = lds4(sWb + nl * WKP + q * CS + 8 * kq + 4);
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        bw[q][st] = w0[st];
        bw[q][st + 4] = w1[st];
      }
    }
    __syncthreads();  // (the staging below overwrites the block matrix)
  }
  if (nrs > 0) {
    stage_small<SP>(g, P.small, n, ys_lo * g.ws, nrs * g.ws, kf, kb, sIn);
  }
  __syncthreads();
  CV_ESTAMP(st2);
  const float bias = nl < NCOL ? sb[cb] : 0.f;
  const int nblk = RBb * nbx, ntile = (nblk + 15) / 16;
  const FDiv fnbx = FDiv::make(nbx);
  if constexpr (M4) {
    const float b0 = sb[0];
    const float* wp = sW4 + (lane & 3) * WKP4;  // (lanes 0..3 are the broadcast A block)
    for (int tile = w; tile < (nblk + 63) / 64; tile += 4) {
      const int blk = 64 * tile + lane;
      const int br = fnbx.div(blk), bx = blk - br * nbx, by = bb0 + br;
      const float* ap[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ys = by - 1 + (q >> 1), xs = bx - 1 + (q & 1);
        const bool ok = blk < nblk && ys >= ys_lo && ys <= ys_hi && (unsigned)xs < (unsigned)g.ws;
        ap[q] = ok ? sIn + ((ys - ys_lo) * g.ws + xs) * SP : sZ;
      }
      // one accumulator per neighbour (independent chains), summed in neighbour order
      f32x4 accq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) accq[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c4 = 0; c4 < CS / 4; ++c4) {
        f32x4 a[4], b[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          a[q] = lds4(wp + q * CS + 4 * c4);
          b[q] = lds4(ap[q] + 4 * c4);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int q = 0; q < 4; ++q) accq[q] = __builtin_amdgcn_mfma_f32_4x4x1f32(a[q][k], b[q][k], accq[q], 4, 0, 0);
      }
      const f32x4 acc = (accq[0] + accq[1]) + (accq[2] + accq[3]);
      // acc[i]: class i = (cy, cx) of block blk
      if (blk < nblk) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int yb = 2 * by - g.p + (i >> 1), xb = 2 * bx - g.p + (i & 1);
          if (yb >= yb0 && yb < yb1 && (unsigned)xb < (unsigned)g.wb) sOut[(yb - yb0) * g.wb + xb] = acc[i] + b0;
        }
      }
    }
  } else
  for (int tile = w; tile < ntile; tile += 4) {
    // A: this lane's block (row nl of the tile), channels 8 kq .. 8 kq + 7 of each neighbour
    const int blk = 16 * tile + nl;
    const int br = fnbx.div(blk), bx = blk - br * nbx, by = bb0 + br;
    // one accumulator per neighbour: four independent MFMA chains (a single chain of 32 dependent MFMAs
    // leaves the matrix pipe waiting on its own results), summed in neighbour order
    // (all four neighbours' fragments read first, then the chains interleaved neighbour-innermost: 32 MFMAs of
    // which no two consecutive depend on each other — chained one neighbour at a time, every MFMA waited for
    // the previous one's result)
    f32x4 accq[4], a0[4], a1[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      accq[q] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int ys = by - 1 + (q >> 1), xs = bx - 1 + (q & 1);
      const bool ok = blk < nblk && ys >= ys_lo && ys <= ys_hi && (unsigned)xs < (unsigned)g.ws;
      const float* ap = sIn + (ok ? ((ys - ys_lo) * g.ws + xs) * SP + 8 * kq : 0);  // (SP = 36: conflict-free)
      a0[q] = lds4(ap);
      a1[q] = lds4(ap + 4);
      if (!ok) a0[q] = a1[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int st = 0; st < 8; ++st)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        accq[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(st < 4 ? a0[q][st] : a1[q][st - 4], bw[q][st], accq[q], 0, 0, 0);
    const f32x4 acc = (accq[0] + accq[1]) + (accq[2] + accq[3]);
    // acc[r]: block 16 tile + 4 kq + r, column nl = (class, cb)
    if (nl < NCOL) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b2 = 16 * tile + 4 * kq + r;
        if (b2 >= nblk) continue;
        const int r2 = fnbx.div(b2), x2 = b2 - r2 * nbx;
        const int yb = 2 * (bb0 + r2) - g.p + cy, xb = 2 * x2 - g.p + cx;
        if (yb >= yb0 && yb < yb1 && (unsigned)xb < (unsigned)g.wb)
          sOut[((yb - yb0) * g.wb + xb) * CB + cb] = acc[r] + bias;
      }
    }
  }
  __syncthreads();
  CV_ESTAMP(st3);
  // the band's output rows are one contiguous range: 16-byte stores (+ the statistics epilogue)
  const int mode = P.ep.stat_mode;
  float s1[CB], s2[CB];
#pragma unroll
  for (int j = 0; j < CB; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  const int tot = (yb1 - yb0) * g.wb * CB;
  // (P.out == nullptr: the statistics only, no output tensor — cv_conv_forward with out = NULL)
  float* dst = P.out ? P.out + (size_t)(n * g.hb + yb0) * g.wb * CB : nullptr;
  const int tot4 = tot >> 2;
  for (int i = t; i < tot4; i += ET) {
    const f32x4 v = lds4(sOut + 4 * i);
    if (dst) *reinterpret_cast<f32x4*>(dst + 4 * i) = v;
    if (mode == CV_STAT_FWD) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int j = (4 * i + k) % CB;
#pragma unroll
        for (int c = 0; c < CB; ++c)
          if (c == j) { s1[c] += v[k]; s2[c] += v[k] * v[k]; }
      }
    }
  }
  for (int i = 4 * tot4 + t; i < tot; i += ET) {
    const float v = sOut[i];
    if (dst) dst[i] = v;
    if (mode == CV_STAT_FWD) {
      const int j = i % CB;
#pragma unroll
      for (int c = 0; c < CB; ++c)
        if (c == j) { s1[c] += v; s2[c] += v * v; }
    }
  }
  CV_ESTAMP(st4);
  if (mode == CV_STAT_FWD) stats_out<CB>(s1, s2, P.ep.stat_out, CB, red);
  if constexpr (!OUT) {
    CV_ESTAMP_WRITE();
  }
  if constexpr (OUT) {
    __shared__ BnFwdC ko[4];
    __shared__ double ored[ET / 64][1 + 2 * 4];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned nblk = gridDim.x * gridDim.y;
    if (t == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __hip_atomic_fetch_add(g_eo_sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int it = 0;
      while (__hip_atomic_load(g_eo_sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < nblk) {
        __builtin_amdgcn_s_sleep(8);
        if (++it > (1 << 20)) {
          __hip_atomic_store(g_eo_sync + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    if (t < CB) {  // the output BN's constants from the replica sums (every workgroup's are in)
      double a = 0.0, q = 0.0;
      const int R = CV_STAT_REPL(CB);
      for (int r = 0; r < R; ++r) {
        a += __hip_atomic_load(O.bn.stat + (size_t)r * 2 * CB + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        q += __hip_atomic_load(O.bn.stat + (size_t)r * 2 * CB + CB + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      ko[t] = bn_fwd_const_s(O.bn, t, a, q);
    }
    __syncthreads();
    const float scale = (O.rec_scale ? O.rec_scale[0] : 1.0f) * 2.0f / (float)g.n;
    float rec = 0.f, o1[CB], o2[CB];
#pragma unroll
    for (int j = 0; j < CB; ++j) { o1[j] = 0.f; o2[j] = 0.f; }
    const size_t band0 = (size_t)(n * g.hb + yb0) * g.wb * CB;
    for (int i = t; i < tot; i += ET) {
      const int c = i % CB, pix = i / CB, yy = yb0 + pix / g.wb, xx = pix - (pix / g.wb) * g.wb;
      const size_t nchw = ((size_t)(n * CB + c) * g.hb + yy) * g.wb + xx;
      const float yv = sOut[i];
      BnFwdC kk;
#pragma unroll
      for (int j = 0; j < CB; ++j)
        if (j == c) kk = ko[j];
      const float v = bn_out(yv, kk);
      const float xh = 1.0f / (1.0f + expf(-v));
      const float diff = xh - O.x[nchw];
      O.xhat[nchw] = xh;
      rec = fmaf(diff, diff, rec);
      if (O.dv) {
        const float dd = scale * diff * xh * (1.0f - xh);
        O.dv[band0 + i] = dd;
#pragma unroll
        for (int j = 0; j < CB; ++j)
          if (j == c) {
            o1[j] += dd;
            o2[j] += dd * ((yv - kk.mu) * kk.istd);
          }
      }
    }
    double vals[1 + 2 * CB];
    vals[0] = (double)rec;
#pragma unroll
    for (int j = 0; j < CB; ++j) { vals[1 + j] = (double)o1[j]; vals[1 + CB + j] = (double)o2[j]; }
#pragma unroll
    for (int q = 0; q < 1 + 2 * CB; ++q) {
      const double v = wave_sum(vals[q]);
      if (lane == 0) ored[w][q] = v;
    }
    __syncthreads();
    if (t == 0) {
      const unsigned blk = blockIdx.y * gridDim.x + blockIdx.x;
      double r = 0.0;
#pragma unroll
      for (int ww = 0; ww < ET / 64; ++ww) r += ored[ww][0];
      atomic_add_f64(O.rec_out + blk % CV_REC_REPL, r / (double)g.n);
      if (O.dv) {
        const int repl = blk % CV_STAT_REPL(CB);
#pragma unroll
        for (int j = 0; j < CB; ++j) {
          double a = 0.0, bq = 0.0;
#pragma unroll
          for (int ww = 0; ww < ET / 64; ++ww) {
            a += ored[ww][1 + j];
            bq += ored[ww][1 + CB + j];
          }
          atomic_add_f64(O.gstat + (size_t)repl * 2 * CB + j, a);
          atomic_add_f64(O.gstat + (size_t)repl * 2 * CB + CB + j, bq);
        }
      }
      if (__hip_atomic_fetch_add(g_eo_sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nblk - 1) {
        __hip_atomic_store(g_eo_sync + 0, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(g_eo_sync + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// ---------------------------------------------------------------- weight gradient (split partials)
// dW[o][col] = sum_px A[o][px] B[px][col] on v_mfma_f32_16x16x4_f32: M = 32 small channels (2 tiles),
// N = ncol <= 64 columns (tap*CB + c, then the conv bias column of ones), K = the workgroup's pixels,
// each wave taking every 4th group of 4 pixels of a band.  A = the staged small band (pitch WP: the
// four lane groups' pixel rows land on disjoint banks), B = the staged big band through the lane's
// column offsets.  The waves' 32 x ncol partials are folded in LDS in wave order.
constexpr int WP = 48;
template <int CB, int KK, int NT>
__global__ __launch_bounds__(ET, 3) void edge_wgrad_kernel(const EArgs P) {
  constexpr int NK = KK * KK * CB;
  __shared__ BnFwdC kfs[CS];
  __shared__ BnBwdC kbs[CS];
  __shared__ BnFwdC kfb[4];
  __shared__ BnBwdC kbb[4];
  __shared__ double scratch[4 * ET];
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const Geo& g = P.g;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int kq = lane >> 4, nl = lane & 15;
  const int ncol = P.ncol;
  const int R = P.rows;
  const int NC = (g.ws - 1) * g.s + KK;
  // the big band's first batch (x-only operands, e.g. the input image) is requested before the constants
  const int nbk = (g.hs + R - 1) / R;
  const int n0 = blockIdx.x / nbk, r00 = (blockIdx.x - n0 * nbk) * R;
  const int NR0 = (min(R, g.hs - r00) - 1) * g.s + KK;
  float bv[BU];
  const bool pre = P.big.xf != CV_XF_BNBWD;
  if (pre) big_load<CB, false>(g, P.big, n0, r00 * g.s - g.p, -g.p, NR0, NC, t, bv, nullptr);
  xf_consts(P.small, kfs, kbs, scratch);
  xf_consts(P.big, kfb, kbb, scratch);
  __syncthreads();
  float* sA = lds;                          // [R*ws][WP]
  float* sB = lds + (size_t)R * g.ws * WP;  // [NR][NC][CB] (+1 zero word)
  // this lane's columns: offset in a receptive field, or -1 (bias: ones), -2 (padding: zeros)
  int coff[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = 16 * j + nl;
    if (col < NK) {
      const int tap = col / CB, c = col - tap * CB, kh = tap / KK, kw = tap - kh * KK;
      coff[j] = (kh * NC + kw) * CB + c;
    } else {
      coff[j] = (col < ncol) ? -1 : -2;
    }
  }
  f32x4 acc[2][NT];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const FDiv fws = FDiv::make(g.ws);
  const int nb = (g.hs + R - 1) / R;
  {
    const int n = blockIdx.x / nb;
    {
      const int r0 = (blockIdx.x - n * nb) * R;
      const int Rb = min(R, g.hs - r0);
      const int NR = (Rb - 1) * g.s + KK;
      stage_small<WP>(g, P.small, n, r0 * g.ws, Rb * g.ws, kfs, kbs, sA);
      if (pre) stage_big<CB, true>(g, P.big, n, r0 * g.s - g.p, -g.p, NR, NC, kfb, kbb, sB, bv, nullptr);
      else stage_big<CB>(g, P.big, n, r0 * g.s - g.p, -g.p, NR, NC, kfb, kbb, sB);
      __syncthreads();
      const int npx = Rb * g.ws;
      for (int p0 = 4 * w; p0 < npx; p0 += 16) {
        const int px = p0 + kq;
        const bool ok = px < npx;
        const int rl = fws.div(px), xs = px - rl * g.ws;
        const int bb = ((rl * g.s) * NC + xs * g.s) * CB;
        float a[2], b[NT];
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = ok ? sA[px * WP + 16 * i + nl] : 0.f;
#pragma unroll
        for (int j = 0; j < NT; ++j) b[j] = coff[j] >= 0 ? (ok ? sB[bb + coff[j]] : 0.f) : (coff[j] == -1 && ok ? 1.f : 0.f);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
      }
      __syncthreads();
    }
  }
  // fold the waves' tiles in wave order: red[w][o][col], o = 16i + 4(l>>4) + r, col = 16j + (l&15)
  float* red = lds;
  const int NP = 16 * NT;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[((size_t)w * CS + 16 * i + 4 * kq + r) * NP + 16 * j + nl] = acc[i][j][r];
  __syncthreads();
  float* part = P.out + (size_t)blockIdx.x * CS * ncol;
  for (int e = t; e < CS * ncol; e += ET) {
    const int o = e / ncol, col = e - o * ncol;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < ET / 64; ++ww) v += red[((size_t)ww * CS + o) * NP + col];
    part[e] = v;
  }
}

// ---------------------------------------------------------------- ConvTranspose2d-to-image backward, both halves
// The backward-data gather (big -> small, with the STAT_BWD epilogue of the small side's BatchNorm) and the
// weight gradient (small x big) of the last ConvTranspose2d (vae.py:43 / :153) read the same band of the
// image-side gradient (BN backward applied) and the same small-grid rows, whose BatchNorm (forward constants)
// is both the epilogue's mask layer and the weight gradient's input transform.  One launch stages the big band
// and the small rows once and runs both contractions; the staging, the MFMA order and the epilogue are those of
// edge_gather_kernel and edge_wgrad_kernel, so the outputs are bit-identical to the two separate launches.
// P: the gather's arguments (big = gout, out = gin, ep), Q: the weight gradient's (small = X, out = partials).
template <int CB, int KK, int NT>
__global__ __launch_bounds__(ET, 2) void edge_bwd_kernel(const EArgs P, const EArgs Q) {
  constexpr int NK = KK * KK * CB;
  constexpr int KS = (NK + 3) / 4;
  __shared__ BnFwdC kfs[CS];  // the small side's forward constants (weight-gradient transform, epilogue mask)
  __shared__ BnBwdC kbs[CS];
  __shared__ BnFwdC kfb[4];
  __shared__ BnBwdC kbb[4];   // the big side's backward constants
  __shared__ float red[ET / 64][2][CS];
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const Geo& g = P.g;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int kq = lane >> 4, nl = lane & 15;
  const int n = blockIdx.y;
  const int r0 = blockIdx.x * P.rows;
  const int R = min(P.rows, g.hs - r0);
  const int NC = (g.ws - 1) * g.s + KK;
  const int NR = (R - 1) * g.s + KK;
  // gather B fragments (packed gather weights [tap][cb][cs]) and tap-channel offsets
  float bw[KS][2];
#pragma unroll
  for (int st = 0; st < KS; ++st) {
    const int k = 4 * st + kq;
#pragma unroll
    for (int j = 0; j < 2; ++j) bw[st][j] = (k < NK) ? P.w[k * CS + 16 * j + nl] : 0.f;
  }
  int koff[KS];
#pragma unroll
  for (int st = 0; st < KS; ++st) {
    const int k = 4 * st + kq;
    const int tap = k / CB, c = k - tap * CB, kh = tap / KK, kw = tap - kh * KK;
    koff[st] = (k < NK) ? (kh * NC + kw) * CB + c : 0;
  }
  // weight-gradient columns: offset in a receptive field, or -1 (bias: ones), -2 (padding: zeros)
  const int ncol = Q.ncol;
  int coff[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = 16 * j + nl;
    if (col < NK) {
      const int tap = col / CB, c = col - tap * CB, kh = tap / KK, kw = tap - kh * KK;
      coff[j] = (kh * NC + kw) * CB + c;
    } else {
      coff[j] = (col < ncol) ? -1 : -2;
    }
  }
  double* scratch = reinterpret_cast<double*>(lds);  // (fold scratch: the staging area, unused yet)
  xf_consts(Q.small, kfs, kbs, scratch);
  xf_consts(P.big, kfb, kbb, scratch);
  __syncthreads();
  float* sA = lds;                          // [R*ws][WP] small rows, transformed
  float* sB = lds + (size_t)P.rows * g.ws * WP;  // [NR][NC][CB] big band, transformed
  stage_small<WP>(g, Q.small, n, r0 * g.ws, R * g.ws, kfs, kbs, sA);
  stage_big<CB>(g, P.big, n, r0 * g.s - g.p, -g.p, NR, NC, kfb, kbb, sB);
  __syncthreads();
  const int npx = R * g.ws;
  // ---- gather: out[px][32] = sum_k big[gather(px, k)] W[k][32]  (edge_gather_kernel's contraction)
  int abase[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int px = 64 * w + 16 * i + nl;
    const int rl = px / g.ws, xs = px - rl * g.ws;
    abase[i] = (px < npx) ? ((rl * g.s) * NC + xs * g.s) * CB : 0;
  }
  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (64 * w < npx) {
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      float a[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = sB[abase[i] + koff[st]];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], bw[st][j], acc[i][j], 0, 0, 0);
    }
  }
  // ---- weight gradient: dW[o][col] = sum_px small[px][o] big[gather(px, col)]  (edge_wgrad_kernel's)
  f32x4 wacc[2][NT];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) wacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    const FDiv fws = FDiv::make(g.ws);
    for (int p0 = 4 * w; p0 < npx; p0 += 16) {
      const int px = p0 + kq;
      const bool ok = px < npx;
      const int rl = fws.div(px), xs = px - rl * g.ws;
      const int bb = ((rl * g.s) * NC + xs * g.s) * CB;
      float a[2], b[NT];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = ok ? sA[px * WP + 16 * i + nl] : 0.f;
#pragma unroll
      for (int j = 0; j < NT; ++j) b[j] = coff[j] >= 0 ? (ok ? sB[bb + coff[j]] : 0.f) : (coff[j] == -1 && ok ? 1.f : 0.f);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) wacc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], wacc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();  // (every wave is done with the staged operands)
  // ---- gather epilogue through an LDS tile (edge_gather_kernel's)
  float* sT = lds;
  if (64 * w < npx) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int px = 64 * w + 16 * i + 4 * kq + r;
        if (px >= npx) continue;
#pragma unroll
        for (int j = 0; j < 2; ++j) sT[px * GP + 16 * j + nl] = acc[i][j][r];
      }
  }
  __syncthreads();
  const int mode = P.ep.stat_mode;
  const int c0 = 4 * (t & 7);
  BnFwdC kc[4];
  if (mode == CV_STAT_BWD) {
#pragma unroll
    for (int k = 0; k < 4; ++k) kc[k] = kfs[c0 + k];
  }
  f32x4 s1 = f32x4{0.f, 0.f, 0.f, 0.f}, s2 = s1;
  const size_t pimg = ((size_t)n * g.hs + r0) * g.ws;
  const int nq = npx * (CS / 4);
  constexpr int UQ = 4;
  for (int q0 = t; q0 < nq; q0 += ET * UQ) {
    f32x4 y4[UQ];
    if (mode == CV_STAT_BWD) {
#pragma unroll
      for (int u = 0; u < UQ; ++u) {
        const int q = q0 + u * ET;
        y4[u] = q < nq ? *reinterpret_cast<const f32x4*>(P.ep.ey + (pimg + (q >> 3)) * CS + c0) : s1;
      }
    }
#pragma unroll
    for (int u = 0; u < UQ; ++u) {
      const int q = q0 + u * ET;
      if (q >= nq) continue;
      const int px = q >> 3;
      f32x4 v = lds4(sT + px * GP + c0);
      if (mode == CV_STAT_BWD) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (P.ep.erelu && bn_out(y4[u][k], kc[k]) <= 0.f) v[k] = 0.f;
          s1[k] += v[k];
          s2[k] += v[k] * ((y4[u][k] - kc[k].mu) * kc[k].istd);
        }
      }
      *reinterpret_cast<f32x4*>(P.out + (pimg + px) * CS + c0) = v;
    }
  }
  if (mode == CV_STAT_BWD) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int m = 8; m < 64; m <<= 1) {
        s1[k] += __shfl_xor(s1[k], m, 64);
        s2[k] += __shfl_xor(s2[k], m, 64);
      }
    }
    if (lane < 8) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        red[w][0][c0 + k] = s1[k];
        red[w][1][c0 + k] = s2[k];
      }
    }
  }
  __syncthreads();  // (the tile reads are complete: the fold area below reuses it; red is published)
  if (mode == CV_STAT_BWD && t < 2 * CS) {
    const int q = t / CS, col = t - q * CS;
    double v = 0.0;
#pragma unroll
    for (int ww = 0; ww < ET / 64; ++ww) v += (double)red[ww][q][col];
    const int repl = (blockIdx.y * gridDim.x + blockIdx.x) % CV_STAT_REPL(CS);
    atomic_add_f64(P.ep.stat_out + (size_t)repl * 2 * CS + q * CS + col, v);
  }
  // ---- weight-gradient partials: the waves' tiles folded in wave order (edge_wgrad_kernel's)
  float* wred = lds;
  const int NP = 16 * NT;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) wred[((size_t)w * CS + 16 * i + 4 * kq + r) * NP + 16 * j + nl] = wacc[i][j][r];
  __syncthreads();
  float* part = Q.out + (size_t)(blockIdx.y * gridDim.x + blockIdx.x) * CS * ncol;
  for (int e = t; e < CS * ncol; e += ET) {
    const int o = e / ncol, col = e - o * ncol;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < ET / 64; ++ww) v += wred[((size_t)ww * CS + o) * NP + col];
    part[e] = v;
  }
}

// ---------------------------------------------------------------- host side
// small-grid rows per band of the gather / weight-gradient / fused backward launches: one row per thread
// (ET / ws), at most the image; CV_EDGE_ROWS=<rows> overrides (A/B knob), clamped to ET / ws: the gather and
// fused-backward kernels compute ET pixels per band (one per thread), so a taller band would leave its
// last pixels unwritten in the LDS output tile that the epilogue streams out
int edge_rows_for(int ws, int hs, int ovr) {
  const int cap = ws >= ET ? 1 : ET / ws;
  int r = cap;
  if (ovr > 0) r = ovr < cap ? ovr : cap;
  return r > hs ? hs : r;
}
static int edge_rows(const Geo& g) {
  static int ovr = -2;
  if (ovr == -2) {
    const char* e = getenv("CV_EDGE_ROWS");
    ovr = e ? atoi(e) : -1;
  }
  return edge_rows_for(g.ws, g.hs, ovr);
}

static bool ep_ok(const cv_epilogue* ep, int C) {
  if (!ep || ep->stat_mode == CV_STAT_NONE) return true;
  if (!ep->stat_out || ep->stat_div > 1) return false;
  if (ep->stat_mode == CV_STAT_BWD) return ep->ey != nullptr && ep->ebn.C == C;
  return true;
}

static int set_lds(const void* kern, size_t bytes) {
  if (bytes <= 64 * 1024) return 0;
  if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess) {
    (void)hipGetLastError();
    return 1;
  }
  return 0;
}

static int launch(const void* kern, dim3 grid, size_t lds, const EArgs& a, hipStream_t st, const char* what) {
  if (set_lds(kern, lds)) {
    set_error("%s: LDS carve-out of %zu bytes refused", what, lds);
    return 1;
  }
  EArgs arg = a;
  void* params[] = {&arg};
  note_launch(kern);
  if (hipLaunchKernel(kern, grid, dim3(ET), params, lds, st) != hipSuccess) {
    (void)hipGetLastError();
    set_error("%s: launch failed", what);
    return 2;
  }
  return 0;
}

#define CV_EDGE_PICK(K, ...)                                 \
  do {                                                                 \
    if (cb == 1 && kk == 3) kern = (const void*)K<1, 3 __VA_ARGS__>;   \
    else if (cb == 1 && kk == 4) kern = (const void*)K<1, 4 __VA_ARGS__>; \
    else if (cb == 2 && kk == 3) kern = (const void*)K<2, 3 __VA_ARGS__>; \
    else if (cb == 2 && kk == 4) kern = (const void*)K<2, 4 __VA_ARGS__>; \
    else if (cb == 3 && kk == 3) kern = (const void*)K<3, 3 __VA_ARGS__>; \
    else if (cb == 3 && kk == 4) kern = (const void*)K<3, 4 __VA_ARGS__>; \
    else if (cb == 4 && kk == 3) kern = (const void*)K<4, 3 __VA_ARGS__>; \
    else if (cb == 4 && kk == 4) kern = (const void*)K<4, 4 __VA_ARGS__>; \
  } while (0)

static bool geo_ok(const Geo& g) {
  return g.cs == CS && g.ws <= ET && g.cb >= 1 && g.cb <= 4 && g.kh == g.kw && (g.kh == 3 || g.kh == 4) && g.s >= 1 && g.s <= 2 &&
         (long)g.n * g.hb * g.wb * g.cb < (1L << 31) && (long)g.n * g.hs * g.ws * CS < (1L << 31);
}

}  // namespace edge

#ifdef CV_STAMPS
extern "C" int cv_debug_set_stamps_edge(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(cv::edge::g_estamps), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}
#endif

using namespace edge;

int edge_gather(const Geo& g, const cv_operand* in, const float* wg, const float* bias, float* out,
                const cv_epilogue* ep, hipStream_t st) {
  if (!geo_ok(g) || !ep_ok(ep, CS)) return -1;
  if (in->xf != CV_XF_NONE && (in->nchw || in->bn.C != g.cb)) return -1;
  if (in->xf == CV_XF_BNBWD && !in->y) return -1;
  EArgs a;
  memset(&a, 0, sizeof(a));
  a.g = g;
  a.big = *in;
  a.w = wg;
  a.bias = bias;
  a.out = out;
  if (ep) a.ep = *ep;
  else a.ep.stat_mode = CV_STAT_NONE;
  a.rows = edge_rows(g);
  const int kk = g.kh, cb = g.cb;
  size_t lds = (size_t)((a.rows - 1) * g.s + kk) * ((g.ws - 1) * g.s + kk) * cb * sizeof(float);
  const size_t tile = (size_t)a.rows * g.ws * GP * sizeof(float);  // the epilogue's output tile
  if (tile > lds) lds = tile;
  if (lds < 4 * ET * sizeof(double)) lds = 4 * ET * sizeof(double);  // (BN fold scratch)
  if (lds > 96 * 1024) return -1;
  const void* kern = nullptr;
  CV_EDGE_PICK(edge_gather_kernel);
  return launch(kern, dim3(cdiv(g.hs, a.rows), g.n), lds, a, st, "edge_gather");
}

static int edge_scatter_impl(const Geo& g, const cv_operand* in, const float* ws, const float* bias, float* out,
                             const cv_epilogue* ep, const OArgs* o, hipStream_t st);

int edge_scatter(const Geo& g, const cv_operand* in, const float* ws, const float* bias, float* out,
                 const cv_epilogue* ep, hipStream_t st) {
  return edge_scatter_impl(g, in, ws, bias, out, ep, nullptr, st);
}

// the ConvT-to-image forward with the decoder output fused (OArgs); -1 when not applicable (then the caller runs
// edge_scatter and cv_output_loss)
int edge_scatter_out(const Geo& g, const cv_operand* in, const float* ws, const float* bias, float* out,
                     const cv_epilogue* ep, const cv_bn* obn, const float* x, float* xhat, double* rec_out, float* dv,
                     double* gstat, const float* rec_scale, hipStream_t st) {
  if (!ep || ep->stat_mode != CV_STAT_FWD || !obn || !obn->train || obn->C != g.cb || obn->stat != ep->stat_out ||
      !x || !xhat || !rec_out || (dv && !gstat))
    return -1;
  OArgs o;
  o.bn = *obn;
  o.x = x;
  o.xhat = xhat;
  o.rec_out = rec_out;
  o.dv = dv;
  o.gstat = gstat;
  o.rec_scale = rec_scale;
  return edge_scatter_impl(g, in, ws, bias, out, ep, &o, st);
}

static int edge_scatter_impl(const Geo& g, const cv_operand* in, const float* ws, const float* bias, float* out,
                             const cv_epilogue* ep, const OArgs* o, hipStream_t st) {
  // (the statistics epilogue of this layer is the forward one: the decoder's output BatchNorm)
  if (!geo_ok(g) || g.s != 2 || (g.hb & 1) || (g.wb & 1) || !ep_ok(ep, g.cb)) return -1;
  if (ep && ep->stat_mode == CV_STAT_BWD) return -1;
  if (in->nchw || (in->xf != CV_XF_NONE && in->bn.C != CS) || (in->xf == CV_XF_BNBWD && !in->y)) return -1;
  EArgs a;
  memset(&a, 0, sizeof(a));
  a.g = g;
  a.small = *in;
  a.w = ws;
  a.bias = bias;
  a.out = out;
  if (ep) a.ep = *ep;
  else a.ep.stat_mode = CV_STAT_NONE;
  const int kk = g.kh, cb = g.cb;
  // bands of block rows (2 big rows each): as many as fit ~36 KB of staged small rows (VAE64: 7 block rows
  // = 8 small rows, 3-4 workgroups per CU; MNIST: a whole image), shortened while the grid has fewer than
  // 512 workgroups (down to 2).  CV_EDGE_SCATTER_RB=<rows> overrides (A/B knob).
  const int nby = (g.hb - 1 + g.p) / 2 + 1;
  if (kk > 4 || 4 * cb > 16 || g.p < 0 || g.p > 2) return -1;
  int rb = (36 * 1024) / (g.ws * SP * (int)sizeof(float)) - 1;
  if (rb > nby) rb = nby;
  if (rb < 1) rb = 1;
  while (rb > 2 && (long)g.n * cdiv(nby, rb) < 512) {
    const int r2 = (rb + 1) / 2;
    if (r2 >= rb) break;
    rb = r2;
  }
  rb = cdiv(nby, cdiv(nby, rb));  // even bands
  {
    static int ovr = -2;
    if (ovr == -2) {
      const char* e = getenv("CV_EDGE_SCATTER_RB");
      ovr = e ? atoi(e) : -1;
    }
    if (ovr > 0) rb = ovr < nby ? ovr : nby;
  }
  a.rows = rb;
  a.ipb = rb + 1;  // (scatter: small rows staged per band, sizes the LDS carve-up)
  size_t lds = ((size_t)a.ipb * g.ws * SP + (size_t)2 * rb * g.wb * cb) * sizeof(float);
  const size_t pre = 4 * ET * sizeof(double) + 16 * (4 * CS + 4) * sizeof(float);  // fold scratch + block matrix
  if (lds < pre) lds = pre;
  if (cb == 1) lds = ((size_t)m4_off(a.ipb, g.ws, rb, g.wb) + M4_EXTRA) * sizeof(float);  // (>= pre)
  if (lds > 96 * 1024) return -1;
  const void* kern = nullptr;
  const dim3 grid(cdiv(nby, rb), g.n);
  OArgs oa;
  memset(&oa, 0, sizeof(oa));
  if (o) {
    CV_EDGE_PICK(edge_scatter_kernel, , true);
    // every workgroup resident at once (half the device's slots: margin for other streams' kernels)
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = -1;
      (void)hipGetLastError();
    }
    int occ = 0;
    if (!kern || set_lds(kern, lds) || cus <= 0 ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, ET, lds) != hipSuccess) {
      (void)hipGetLastError();
      return -1;
    }
    if ((long)grid.x * grid.y > (long)occ * cus / 2) return -1;
    oa = *o;
  } else {
    CV_EDGE_PICK(edge_scatter_kernel, , false);
  }
  {
    static int m4 = -1;  // CV_EDGE_M4=0: the one-channel image on the 16-column tile (A/B)
    if (m4 < 0) {
      const char* e = getenv("CV_EDGE_M4");
      m4 = e ? atoi(e) != 0 : 1;
    }
    if (!m4 && cb == 1)
      kern = o ? (kk == 3 ? (const void*)edge_scatter_kernel<1, 3, true, false> : (const void*)edge_scatter_kernel<1, 4, true, false>)
               : (kk == 3 ? (const void*)edge_scatter_kernel<1, 3, false, false> : (const void*)edge_scatter_kernel<1, 4, false, false>);
  }
  if (set_lds(kern, lds)) {
    set_error("edge_scatter: LDS carve-out of %zu bytes refused", lds);
    return 1;
  }
  EArgs arg = a;
  void* params[] = {&arg, &oa};
  note_launch(kern);
  if (hipLaunchKernel(kern, grid, dim3(ET), params, lds, st) != hipSuccess) {
    (void)hipGetLastError();
    set_error("edge_scatter: launch failed");
    return 2;
  }
  return 0;
}



// workgroups of the weight-gradient split, one per (image, band) (also sizes its workspace)
static int edge_wgrad_blocks(const Geo& g) { return g.n * cdiv(g.hs, edge_rows(g)); }

size_t edge_wgrad_ws_bytes(const Geo& g, bool bias) {
  if (!geo_ok(g)) return 0;
  const int ncol = g.kh * g.kw * g.cb + (bias ? 1 : 0);
  return (size_t)edge_wgrad_blocks(g) * CS * ncol * sizeof(float);
}

int edge_wgrad(const Geo& g, const cv_operand* small, const cv_operand* big, float* gw, float* gbias, float* work,
               size_t work_bytes, hipStream_t st) {
  if (!geo_ok(g) || !work) return -1;
  if (small->nchw || (small->xf != CV_XF_NONE && small->bn.C != CS) || (small->xf == CV_XF_BNBWD && !small->y))
    return -1;
  if ((big->xf != CV_XF_NONE && (big->nchw || big->bn.C != g.cb)) || (big->xf == CV_XF_BNBWD && !big->y)) return -1;
  EArgs a;
  memset(&a, 0, sizeof(a));
  a.g = g;
  a.small = *small;
  a.big = *big;
  const int nk = g.kh * g.kw * g.cb;
  a.ncol = nk + (gbias ? 1 : 0);
  const int nblk = edge_wgrad_blocks(g);
  a.ipb = 1;
  if (work_bytes < (size_t)nblk * CS * a.ncol * sizeof(float)) return -1;
  a.out = work;
  a.rows = edge_rows(g);
  const int kk = g.kh, cb = g.cb;
  const int NR = (a.rows - 1) * g.s + kk, NC = (g.ws - 1) * g.s + kk;
  if (a.ncol > 64) return -1;
  const int NT = (a.ncol + 15) / 16;
  size_t lds = ((size_t)a.rows * g.ws * WP + (size_t)NR * NC * cb) * sizeof(float);
  const size_t lred = (size_t)(ET / 64) * CS * 16 * NT * sizeof(float);
  if (lred > lds) lds = lred;
  if (lds > 96 * 1024) return -1;
  const void* kern = nullptr;
  if (NT == 1) CV_EDGE_PICK(edge_wgrad_kernel, , 1);
  else if (NT == 2) CV_EDGE_PICK(edge_wgrad_kernel, , 2);
  else if (NT == 3) CV_EDGE_PICK(edge_wgrad_kernel, , 3);
  else CV_EDGE_PICK(edge_wgrad_kernel, , 4);
  if (launch(kern, dim3(nblk), lds, a, st, "edge_wgrad")) return 1;
  return wgrad_reduce_launch(work, nblk, CS, nk, a.ncol, g.cb, g.kh * g.kw, gw, gbias, st);
}

// Both halves of the ConvTranspose2d-to-image backward in one launch (edge_bwd_kernel), when the geometry is
// the edge kernels' and the epilogue's BatchNorm is the weight gradient's input transform; -1 otherwise (the
// caller runs edge_gather / edge_wgrad or the generic kernels)
int edge_bwd(const Geo& g, const cv_operand* gout, const float* wg, float* gin, const cv_epilogue* ep,
             const cv_operand* x, float* gw, float* work, size_t work_bytes, hipStream_t st) {
  if (!geo_ok(g) || !work || !ep || ep->stat_mode != CV_STAT_BWD || !ep_ok(ep, CS)) return -1;
  if (gout->xf != CV_XF_BNBWD || gout->nchw || gout->bn.C != g.cb || !gout->y) return -1;
  if (x->xf != CV_XF_BNRELU || x->nchw || x->bn.C != CS) return -1;
  const cv_bn &eb = ep->ebn, &xb = x->bn;  // the same layer on both sides
  if (eb.stat != xb.stat || eb.cfwd != xb.cfwd || eb.ticket != xb.ticket || eb.gamma != xb.gamma || !eb.train ||
      !xb.train)
    return -1;
  EArgs a, b;
  memset(&a, 0, sizeof(a));
  a.g = g;
  a.big = *gout;
  a.w = wg;
  a.out = gin;
  a.ep = *ep;
  a.rows = edge_rows(g);
  b = a;
  b.small = *x;
  const int nk = g.kh * g.kw * g.cb;
  b.ncol = nk;
  const int nblk = edge_wgrad_blocks(g);
  if (work_bytes < (size_t)nblk * CS * b.ncol * sizeof(float)) return -1;
  b.out = work;
  const int kk = g.kh, cb = g.cb;
  const int NR = (a.rows - 1) * g.s + kk, NC = (g.ws - 1) * g.s + kk;
  const int NT = (b.ncol + 15) / 16;
  size_t lds = ((size_t)a.rows * g.ws * WP + (size_t)NR * NC * cb) * sizeof(float);
  const size_t tile = (size_t)a.rows * g.ws * GP * sizeof(float);
  const size_t lred = (size_t)(ET / 64) * CS * 16 * NT * sizeof(float);
  if (tile > lds) lds = tile;
  if (lred > lds) lds = lred;
  if (lds < 4 * ET * sizeof(double)) lds = 4 * ET * sizeof(double);
  if (lds > 96 * 1024 || b.ncol > 64) return -1;
  const void* kern = nullptr;
  if (NT == 1) CV_EDGE_PICK(edge_bwd_kernel, , 1);
  else if (NT == 2) CV_EDGE_PICK(edge_bwd_kernel, , 2);
  else if (NT == 3) CV_EDGE_PICK(edge_bwd_kernel, , 3);
  else CV_EDGE_PICK(edge_bwd_kernel, , 4);
  if (!kern) return -1;
  if (set_lds(kern, lds)) {
    set_error("edge_bwd: LDS carve-out of %zu bytes refused", lds);
    return 1;
  }
  void* params[] = {&a, &b};
  note_launch(kern);
  if (hipLaunchKernel(kern, dim3(cdiv(g.hs, a.rows), g.n), dim3(ET), params, lds, st) != hipSuccess) {
    (void)hipGetLastError();
    set_error("edge_bwd: launch failed");
    return 2;
  }
  return wgrad_reduce_launch(work, nblk, CS, nk, b.ncol, g.cb, g.kh * g.kw, gw, nullptr, st);
}

}  // namespace cv
