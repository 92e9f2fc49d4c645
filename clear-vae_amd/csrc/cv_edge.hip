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
#include "cv_common.hpp"

namespace cv {

int wgrad_reduce_launch(const float* part, int split, int M, int N, int ntot, int cb, int kk, float* gw,
                        float* gbias, hipStream_t st);

namespace edge {

constexpr int ET = 256;
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
  int ipb;           // wgrad: images per workgroup
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

// Stage rows [yb0, yb0+NR) x cols [xb0, xb0+NC) x CB of image n of the big-grid operand, transformed,
// zero outside the image, as dst[(rr*NC + cc)*CB + c].  8 loads in flight per thread.
template <int CB>
__device__ __forceinline__ void stage_big(const Geo& g, const cv_operand& o, int n, int yb0, int xb0, int NR, int NC,
                                          const BnFwdC* kf, const BnBwdC* kb, float* dst) {
  constexpr int U = 8;
  const int tot = NR * NC * CB;
  const FDiv fnc = FDiv::make(NC);
  for (int base = threadIdx.x; base < tot; base += ET * U) {
    float v[U], yv[U];
    bool ok[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int i = base + q * ET;
      const int c = i % CB, rc = i / CB;
      const int rr = fnc.div(rc), cc = rc - rr * NC;
      const int yb = yb0 + rr, xb = xb0 + cc;
      ok[q] = i < tot && (unsigned)yb < (unsigned)g.hb && (unsigned)xb < (unsigned)g.wb;
      v[q] = 0.f;
      yv[q] = 0.f;
      if (ok[q]) {
        const size_t off = o.nchw ? ((size_t)(n * CB + c) * g.hb + yb) * g.wb + xb
                                  : ((size_t)(n * g.hb + yb) * g.wb + xb) * CB + c;
        v[q] = o.x[off];
        if (o.xf == CV_XF_BNBWD) yv[q] = o.y[off];
      }
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int i = base + q * ET;
      if (i < tot) dst[i] = ok[q] ? xf_apply(o.xf, v[q], yv[q], i % CB, kf, kb) : 0.f;
    }
  }
}

// Stage small-grid pixels [p0, p0+np) of image n (32 channels, NHWC) transformed, as dst[px*PITCH + ch].
template <int PITCH>
__device__ __forceinline__ void stage_small(const Geo& g, const cv_operand& o, int n, int p0, int np,
                                            const BnFwdC* kf, const BnBwdC* kb, float* dst) {
  constexpr int U = 4;
  const int tot4 = np * (CS / 4);
  const float4* x4 = reinterpret_cast<const float4*>(o.x + ((size_t)n * g.hs * g.ws + p0) * CS);
  const float4* y4 = reinterpret_cast<const float4*>(o.y ? o.y + ((size_t)n * g.hs * g.ws + p0) * CS : nullptr);
  for (int base = threadIdx.x; base < tot4; base += ET * U) {
    float4 v[U], yv[U];
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
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int i = base + q * ET;
      if (i < tot4) {
        const int px = i >> 3, c0 = (i & 7) * 4;
        float4 r;
        r.x = xf_apply(o.xf, v[q].x, yv[q].x, c0, kf, kb);
        r.y = xf_apply(o.xf, v[q].y, yv[q].y, c0 + 1, kf, kb);
        r.z = xf_apply(o.xf, v[q].z, yv[q].z, c0 + 2, kf, kb);
        r.w = xf_apply(o.xf, v[q].w, yv[q].w, c0 + 3, kf, kb);
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
template <int CB, int KK>
__global__ __launch_bounds__(ET) void edge_gather_kernel(const EArgs P) {
  constexpr int NK = KK * KK * CB;
  constexpr int KS = (NK + 3) / 4;  // k-steps
  __shared__ BnFwdC kf[4];
  __shared__ BnBwdC kb[4];
  __shared__ BnFwdC ke[CS];
  __shared__ double scratch[4 * ET];
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
  xf_consts(P.big, kf, kb, scratch);
  const int mode = P.ep.stat_mode;
  if (mode == CV_STAT_BWD) {
    cv_operand eo;
    eo.xf = CV_XF_BNRELU;
    eo.bn = P.ep.ebn;
    xf_consts(eo, ke, nullptr, scratch);
  }
  __syncthreads();
  stage_big<CB>(g, P.big, n, r0 * g.s - g.p, -g.p, NR, NC, kf, kb, sIn);
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
  // epilogue: lane holds rows 4*(l>>4) + r of each 16-row tile, column 16j + (l&15)
  float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f};
  float bj[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) bj[j] = P.bias ? P.bias[16 * j + nl] : 0.f;
  BnFwdC kej[2];
  if (mode == CV_STAT_BWD) {
    kej[0] = ke[nl];
    kej[1] = ke[16 + nl];
  }
  const size_t pimg = ((size_t)n * g.hs + r0) * g.ws;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int px = 64 * w + 16 * i + 4 * kq + r;
      if (px >= npx) continue;
      const size_t o = (pimg + px) * CS;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = 16 * j + nl;
        float v = acc[i][j][r] + bj[j];
        if (mode == CV_STAT_BWD) {
          const float y = P.ep.ey[o + col];
          if (P.ep.erelu && bn_out(y, kej[j]) <= 0.f) v = 0.f;
          s1[j] += v;
          s2[j] += v * ((y - kej[j].mu) * kej[j].istd);
        } else if (mode == CV_STAT_FWD) {
          s1[j] += v;
          s2[j] += v * v;
        }
        P.out[o + col] = v;
      }
    }
  if (mode != CV_STAT_NONE) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {  // fold the four row groups (lanes l, l^16, l^32, l^48 share a column)
      s1[j] += __shfl_xor(s1[j], 16, 64);
      s1[j] += __shfl_xor(s1[j], 32, 64);
      s2[j] += __shfl_xor(s2[j], 16, 64);
      s2[j] += __shfl_xor(s2[j], 32, 64);
    }
    if (lane < 16) {
      red[w][0][lane] = s1[0];
      red[w][0][16 + lane] = s1[1];
      red[w][1][lane] = s2[0];
      red[w][1][16 + lane] = s2[1];
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
// stride 2, even output extents, bands of an even number of big rows: wave w owns parity class
// (w >> 1, w & 1), so its taps (and their weight words) are wave-uniform
template <int CB, int KK>
__global__ __launch_bounds__(ET) void edge_scatter_kernel(const EArgs P) {
  constexpr int NK = KK * KK;
  __shared__ float4 sW[NK * CB * 8];  // [tap][cb][32]
  __shared__ float sbias[4];
  __shared__ BnFwdC kf[CS];
  __shared__ BnBwdC kb[CS];
  __shared__ BnFwdC ke[4];
  __shared__ double scratch[4 * ET];
  __shared__ float red[(ET / 64) * 2 * 4];
  extern __shared__ __attribute__((aligned(16))) float sIn[];
  const Geo& g = P.g;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = blockIdx.y;
  const int B0 = blockIdx.x * P.rows;
  const int RB = min(P.rows, g.hb - B0);
  // small rows feeding big rows [B0, B0+RB)
  const int num = B0 + g.p - (KK - 1);
  const int ys_lo = num <= 0 ? 0 : (num + 1) / 2;
  const int ys_hi = min(g.hs - 1, (B0 + RB - 1 + g.p) / 2);
  const int nrs = ys_hi - ys_lo + 1;
  // weights: packed scatter layout [tap][cs][cb] -> [tap][cb][cs]
  for (int i = t; i < NK * CB * CS; i += ET) {
    const int tap = i / (CB * CS), r = i - tap * CB * CS, cb = r / CS, cs = r - cb * CS;
    reinterpret_cast<float*>(sW)[i] = P.w[(tap * CS + cs) * CB + cb];
  }
  if (t < CB) sbias[t] = P.bias ? P.bias[t] : 0.f;
  xf_consts(P.small, kf, kb, scratch);
  const int mode = P.ep.stat_mode;
  if (mode == CV_STAT_BWD) {
    cv_operand eo;
    eo.xf = CV_XF_BNRELU;
    eo.bn = P.ep.ebn;
    xf_consts(eo, ke, nullptr, scratch);
  }
  __syncthreads();
  float* sOut = sIn + (size_t)(P.rows / 2 + (KK + 1) / 2 + 1) * g.ws * SP;  // [RB][wb][CB]
  if (nrs > 0) stage_small<SP>(g, P.small, n, ys_lo * g.ws, nrs * g.ws, kf, kb, sIn);
  __syncthreads();
  float s1[CB], s2[CB];
#pragma unroll
  for (int j = 0; j < CB; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  const int ry = w >> 1, rx = w & 1;
  const int ky0 = (ry + g.p) & 1, kx0 = (rx + g.p) & 1;  // B0 even: the class's first tap row / column
  const int cy = (RB - ry + 1) / 2, cx = (g.wb - rx + 1) / 2;
  const int ncls = cy * cx;
  constexpr int TH = (KK + 1) / 2;  // taps per class and direction
  constexpr int PPL = 4;            // class pixels per lane: each weight word read feeds 4 pixels
  for (int q0 = 0; q0 < ncls; q0 += 64 * PPL) {
    int yb[PPL], xb[PPL];
    bool live[PPL];
    float acc[PPL][CB];
#pragma unroll
    for (int u = 0; u < PPL; ++u) {
      const int q = q0 + 64 * u + lane;
      live[u] = q < ncls;
      const int iy = q / cx, ix = q - iy * cx;
      yb[u] = B0 + ry + 2 * iy;
      xb[u] = rx + 2 * ix;
#pragma unroll
      for (int j = 0; j < CB; ++j) acc[u][j] = sbias[j];
    }
#pragma unroll 1
    for (int jy = 0; jy < TH; ++jy) {
      const int kh = ky0 + 2 * jy;
      if (kh >= KK) continue;
#pragma unroll 1
      for (int jx = 0; jx < TH; ++jx) {
        const int kw = kx0 + 2 * jx;
        if (kw >= KK) continue;
        const float4* src[PPL];
        bool ok[PPL];
#pragma unroll
        for (int u = 0; u < PPL; ++u) {
          const int ys = (yb[u] + g.p - kh) >> 1, xs = (xb[u] + g.p - kw) >> 1;
          ok[u] = live[u] && ys >= 0 && ys < g.hs && xs >= 0 && xs < g.ws;
          src[u] = reinterpret_cast<const float4*>(sIn + (ok[u] ? ((ys - ys_lo) * g.ws + xs) * SP : 0));
        }
        const float4* wr = sW + (kh * KK + kw) * CB * 8;
#pragma unroll 2
        for (int c4 = 0; c4 < 8; ++c4) {
          float4 x4[PPL];
#pragma unroll
          for (int u = 0; u < PPL; ++u) x4[u] = ok[u] ? src[u][c4] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int j = 0; j < CB; ++j) {
            const float4 w4 = wr[j * 8 + c4];
#pragma unroll
            for (int u = 0; u < PPL; ++u) {
              acc[u][j] = fmaf(x4[u].x, w4.x, acc[u][j]);
              acc[u][j] = fmaf(x4[u].y, w4.y, acc[u][j]);
              acc[u][j] = fmaf(x4[u].z, w4.z, acc[u][j]);
              acc[u][j] = fmaf(x4[u].w, w4.w, acc[u][j]);
            }
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < PPL; ++u) {
      if (!live[u]) continue;
      const size_t po = ((size_t)(n * g.hb + yb[u]) * g.wb + xb[u]) * CB;
      const int lo = ((yb[u] - B0) * g.wb + xb[u]) * CB;
#pragma unroll
      for (int j = 0; j < CB; ++j) {
        float v = acc[u][j];
        if (mode == CV_STAT_BWD) {
          const float yv = P.ep.ey[po + j];
          if (P.ep.erelu && bn_out(yv, ke[j]) <= 0.f) v = 0.f;
          s1[j] += v;
          s2[j] += v * ((yv - ke[j].mu) * ke[j].istd);
        } else if (mode == CV_STAT_FWD) {
          s1[j] += v;
          s2[j] += v * v;
        }
        sOut[lo + j] = v;
      }
    }
  }
  // the band's output rows are one contiguous range: stored after every weight load (no global
  // store before them lets the compiler keep the wave-uniform weights on the scalar path)
  __syncthreads();
  {
    const int tot = RB * g.wb * CB;
    float* dst = P.out + (size_t)(n * g.hb + B0) * g.wb * CB;
    for (int i = t; i < tot; i += ET) dst[i] = sOut[i];
  }
  if (mode != CV_STAT_NONE) stats_out<CB>(s1, s2, P.ep.stat_out, CB, red);
}

// ---------------------------------------------------------------- weight gradient (split partials)
// dW[o][col] = sum_px A[o][px] B[px][col] on v_mfma_f32_16x16x4_f32: M = 32 small channels (2 tiles),
// N = ncol <= 64 columns (tap*CB + c, then the conv bias column of ones), K = the workgroup's pixels,
// each wave taking every 4th group of 4 pixels of a band.  A = the staged small band (pitch WP: the
// four lane groups' pixel rows land on disjoint banks), B = the staged big band through the lane's
// column offsets.  The waves' 32 x ncol partials are folded in LDS in wave order.
constexpr int WP = 48;
template <int CB, int KK, int NT>
__global__ __launch_bounds__(ET) void edge_wgrad_kernel(const EArgs P) {
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
  xf_consts(P.small, kfs, kbs, scratch);
  xf_consts(P.big, kfb, kbb, scratch);
  __syncthreads();
  const int R = P.rows;
  const int NC = (g.ws - 1) * g.s + KK;
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
      stage_big<CB>(g, P.big, n, r0 * g.s - g.p, -g.p, NR, NC, kfb, kbb, sB);
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

// ---------------------------------------------------------------- host side
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
  a.rows = g.ws >= ET ? 1 : ET / g.ws;
  if (a.rows > g.hs) a.rows = g.hs;
  const int kk = g.kh, cb = g.cb;
  const size_t lds = (size_t)((a.rows - 1) * g.s + kk) * ((g.ws - 1) * g.s + kk) * cb * sizeof(float);
  if (lds > 96 * 1024) return -1;
  const void* kern = nullptr;
  CV_EDGE_PICK(edge_gather_kernel);
  return launch(kern, dim3(cdiv(g.hs, a.rows), g.n), lds, a, st, "edge_gather");
}

int edge_scatter(const Geo& g, const cv_operand* in, const float* ws, const float* bias, float* out,
                 const cv_epilogue* ep, hipStream_t st) {
  if (!geo_ok(g) || g.s != 2 || (g.hb & 1) || (g.wb & 1) || !ep_ok(ep, g.cb)) return -1;
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
  // bands of an even number of big rows, ~1024 output pixels each
  int rb = (4 * ET) / g.wb;
  rb &= ~1;
  if (rb < 2) rb = 2;
  if (rb > g.hb) rb = g.hb;
  a.rows = rb;
  const int kk = g.kh, cb = g.cb;
  const int nrs = rb / 2 + (kk + 1) / 2 + 1;
  const size_t lds = ((size_t)nrs * g.ws * SP + (size_t)rb * g.wb * cb) * sizeof(float);
  if (lds > 96 * 1024) return -1;
  const void* kern = nullptr;
  CV_EDGE_PICK(edge_scatter_kernel);
  return launch(kern, dim3(cdiv(g.hb, rb), g.n), lds, a, st, "edge_scatter");
}

static int edge_rows(const Geo& g) {
  const int r = g.ws >= ET ? 1 : ET / g.ws;
  return r > g.hs ? g.hs : r;
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

}  // namespace cv
