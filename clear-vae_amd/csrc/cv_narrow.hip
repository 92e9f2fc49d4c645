// Direct (VALU) kernels for the convolutions with <= 4 channels on one side: the image-facing ends
// of the CLEAR-VAE encoder and decoder (code/src/models/vae.py:15-16 / :113-114 first Conv2d on the
// 1- or 3-channel image, :43 / :153 last ConvTranspose2d back to the image).
//
// As implicit GEMMs these have N (or K) of 1..48 — a 16x16 MFMA tile would be >90 % padding and the
// launch is pure per-workgroup latency — so they run as grid-stride loops of one output pixel per
// thread, weights broadcast from LDS, fused BatchNorm transforms and the same epilogue contract as
// cv_igemm.hip (bias, STAT_FWD / STAT_BWD statistics into replicated fp64 buffers).  These layers are
// HBM-bound: the algorithmic traffic is the activation tensor on the wide side.
//
//   narrow_gather : out[small px][cs] = sum_{tap, c<cb} T(big[gather(px, tap)][c]) * Wg[tap][c][cs]
//                   (Conv2d forward on the image, ConvTranspose2d-to-image backward-data), cs == 32
//   narrow_scatter: out[big px][cb] = sum_{tap in parity class, c<cs} T(small[..][c]) * Ws[tap][c][cb]
//                   (ConvTranspose2d-to-image forward, Conv2d-on-image backward-data), cb <= 4
#include "cv_common.hpp"

namespace cv {

constexpr int NNT = 256;

struct NArgs {
  Geo g;
  cv_operand a;
  const float* w;
  const float* bias;
  float* out;
  cv_epilogue ep;
  long M;  // output pixels
};

// ---------------------------------------------------------------- statistics epilogue (shared)
// per-thread (s1, s2) for NC channels -> block reduction -> fp64 atomics into one replica
template <int NC>
__device__ __forceinline__ void stats_flush(const float* s1, const float* s2, double* stat_out, int C, float* red) {
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
    for (int q = 0; q < NNT / 64; ++q) v += (double)red[q * 2 * NC + j];
    const int ch = j < NC ? j : j - NC;
    if (ch < C) {
      const int repl = blockIdx.x % CV_STAT_REPL(C);
      atomic_add_f64(stat_out + (size_t)repl * 2 * C + (j < NC ? 0 : C) + ch, v);
    }
  }
}

// ---------------------------------------------------------------- narrow gather (cs = 32 outputs)
template <int CS>
__global__ __launch_bounds__(NNT) void narrow_gather_kernel(const NArgs P) {
  constexpr int KMAX = 64;
  __shared__ float4 Ws[KMAX * CS / 4];
  __shared__ float bs[CS];
  __shared__ BnFwdC kf[4];
  __shared__ BnBwdC kb[4];
  __shared__ BnFwdC ke[CS];
  __shared__ double scratch[4 * NNT];
  __shared__ float red[(NNT / 64) * 2 * CS];
  const int t = threadIdx.x;
  const Geo& g = P.g;
  const int K = g.kh * g.kw * g.cb;
  for (int i = t; i < K * CS / 4; i += NNT) Ws[i] = reinterpret_cast<const float4*>(P.w)[i];
  for (int i = t; i < CS; i += NNT) bs[i] = P.bias ? P.bias[i] : 0.f;
  if (P.a.xf == CV_XF_BNRELU)
    bn_fold<NNT>(P.a.bn, false, scratch, [&](int f, double s, double q, double, double) {
      if (f < 4) kf[f] = bn_fwd_const_s(P.a.bn, f, s, q);
    });
  else if (P.a.xf == CV_XF_BNBWD)
    bn_fold<NNT>(P.a.bn, true, scratch, [&](int f, double s, double q, double gs, double gq) {
      if (f < 4) kb[f] = bn_bwd_const_s(P.a.bn, f, s, q, gs, gq);
    });
  const int mode = P.ep.stat_mode;
  if (mode == CV_STAT_BWD)
    bn_fold<NNT>(P.ep.ebn, false, scratch, [&](int f, double s, double q, double, double) {
      if (f < CS) ke[f] = bn_fwd_const_s(P.ep.ebn, f, s, q);
    });
  __syncthreads();

  float s1[CS], s2[CS];
#pragma unroll
  for (int j = 0; j < CS; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  const int hw = g.hs * g.ws;
  for (long p = (long)blockIdx.x * NNT + t; p < P.M; p += (long)gridDim.x * NNT) {
    const int n = (int)(p / hw);
    const int rem = (int)(p - (long)n * hw);
    const int ys = rem / g.ws, xs = rem - ys * g.ws;
    const int y0 = ys * g.s - g.p, x0 = xs * g.s - g.p;
    float acc[CS];
#pragma unroll
    for (int j = 0; j < CS; ++j) acc[j] = bs[j];
    for (int kh = 0; kh < g.kh; ++kh) {
      const int yb = y0 + kh;
      if ((unsigned)yb >= (unsigned)g.hb) continue;
      for (int kw = 0; kw < g.kw; ++kw) {
        const int xb = x0 + kw;
        if ((unsigned)xb >= (unsigned)g.wb) continue;
        for (int c = 0; c < g.cb; ++c) {
          const size_t off = P.a.nchw ? ((size_t)(n * g.cb + c) * g.hb + yb) * g.wb + xb
                                      : ((size_t)(n * g.hb + yb) * g.wb + xb) * g.cb + c;
          float v = P.a.x[off];
          if (P.a.xf == CV_XF_BNRELU) v = bn_relu(v, kf[c]);
          else if (P.a.xf == CV_XF_BNBWD) v = bn_bwd(v, P.a.y[off], kb[c]);
          const float4* wr = Ws + ((kh * g.kw + kw) * g.cb + c) * (CS / 4);
#pragma unroll
          for (int j = 0; j < CS / 4; ++j) {
            const float4 w4 = wr[j];
            acc[4 * j + 0] = fmaf(v, w4.x, acc[4 * j + 0]);
            acc[4 * j + 1] = fmaf(v, w4.y, acc[4 * j + 1]);
            acc[4 * j + 2] = fmaf(v, w4.z, acc[4 * j + 2]);
            acc[4 * j + 3] = fmaf(v, w4.w, acc[4 * j + 3]);
          }
        }
      }
    }
    float4* o4 = reinterpret_cast<float4*>(P.out + (size_t)p * CS);
    if (mode == CV_STAT_BWD) {
      const float4* y4 = reinterpret_cast<const float4*>(P.ep.ey + (size_t)p * CS);
#pragma unroll
      for (int j = 0; j < CS / 4; ++j) {
        const float4 yv = y4[j];
        const float yy[4] = {yv.x, yv.y, yv.z, yv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int ch = 4 * j + e;
          float v = acc[ch];
          if (P.ep.erelu && bn_out(yy[e], ke[ch]) <= 0.f) v = 0.f;
          acc[ch] = v;
          s1[ch] += v;
          s2[ch] += v * ((yy[e] - ke[ch].mu) * ke[ch].istd);
        }
      }
    } else if (mode == CV_STAT_FWD) {
#pragma unroll
      for (int j = 0; j < CS; ++j) {
        s1[j] += acc[j];
        s2[j] += acc[j] * acc[j];
      }
    }
#pragma unroll
    for (int j = 0; j < CS / 4; ++j) o4[j] = make_float4(acc[4 * j], acc[4 * j + 1], acc[4 * j + 2], acc[4 * j + 3]);
  }
  if (mode != CV_STAT_NONE) stats_flush<CS>(s1, s2, P.ep.stat_out, CS, red);
}

// ---------------------------------------------------------------- narrow scatter (cb <= 4 outputs)
template <int CB>
__global__ __launch_bounds__(NNT) void narrow_scatter_kernel(const NArgs P) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const Geo& g = P.g;
  const int taps = g.kh * g.kw;
  // LDS: Ws[tap][cs][CB] | BnFwdC/BnBwdC[cs] | scratch (4*NNT doubles) | red
  float* Wl = sm;
  float* kc = Wl + ((taps * g.cs * CB + 3) & ~3);
  double* scratch = reinterpret_cast<double*>(kc + 8 * g.cs);
  float* red = reinterpret_cast<float*>(scratch + 4 * NNT);
  __shared__ float bs[4];
  __shared__ BnFwdC ke[4];
  const int t = threadIdx.x;
  for (int i = t; i < taps * g.cs * CB; i += NNT) Wl[i] = P.w[i];
  if (t < CB) bs[t] = P.bias ? P.bias[t] : 0.f;
  BnFwdC* kf = reinterpret_cast<BnFwdC*>(kc);
  BnBwdC* kb = reinterpret_cast<BnBwdC*>(kc);
  if (P.a.xf == CV_XF_BNRELU)
    bn_fold<NNT>(P.a.bn, false, scratch, [&](int f, double s, double q, double, double) {
      kf[f] = bn_fwd_const_s(P.a.bn, f, s, q);
    });
  else if (P.a.xf == CV_XF_BNBWD)
    bn_fold<NNT>(P.a.bn, true, scratch, [&](int f, double s, double q, double gs, double gq) {
      kb[f] = bn_bwd_const_s(P.a.bn, f, s, q, gs, gq);
    });
  const int mode = P.ep.stat_mode;
  if (mode == CV_STAT_BWD)
    bn_fold<NNT>(P.ep.ebn, false, scratch, [&](int f, double s, double q, double, double) {
      if (f < 4) ke[f] = bn_fwd_const_s(P.ep.ebn, f, s, q);
    });
  __syncthreads();

  float s1[CB], s2[CB];
#pragma unroll
  for (int j = 0; j < CB; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  const int hw = g.hb * g.wb;
  const int cs4 = g.cs / 4;
  for (long p = (long)blockIdx.x * NNT + t; p < P.M; p += (long)gridDim.x * NNT) {
    const int n = (int)(p / hw);
    const int rem = (int)(p - (long)n * hw);
    const int yb = rem / g.wb, xb = rem - yb * g.wb;
    float acc[CB];
#pragma unroll
    for (int j = 0; j < CB; ++j) acc[j] = bs[j];
    for (int kh = 0; kh < g.kh; ++kh) {
      const int ty = yb + g.p - kh;
      if (ty < 0) break;  // ty decreases with kh
      const int ys = ty / g.s;
      if (ys * g.s != ty || ys >= g.hs) continue;
      for (int kw = 0; kw < g.kw; ++kw) {
        const int tx = xb + g.p - kw;
        if (tx < 0) break;
        const int xs = tx / g.s;
        if (xs * g.s != tx || xs >= g.ws) continue;
        const size_t base = ((size_t)(n * g.hs + ys) * g.ws + xs) * g.cs;
        const float* wt = Wl + (size_t)(kh * g.kw + kw) * g.cs * CB;
        for (int c4 = 0; c4 < cs4; ++c4) {
          float4 v = *reinterpret_cast<const float4*>(P.a.x + base + 4 * c4);
          float vv[4] = {v.x, v.y, v.z, v.w};
          if (P.a.xf == CV_XF_BNRELU) {
#pragma unroll
            for (int e = 0; e < 4; ++e) vv[e] = bn_relu(vv[e], kf[4 * c4 + e]);
          } else if (P.a.xf == CV_XF_BNBWD) {
            const float4 y = *reinterpret_cast<const float4*>(P.a.y + base + 4 * c4);
            const float yy[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) vv[e] = bn_bwd(vv[e], yy[e], kb[4 * c4 + e]);
          }
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int j = 0; j < CB; ++j) acc[j] = fmaf(vv[e], wt[(4 * c4 + e) * CB + j], acc[j]);
        }
      }
    }
    float* o = P.out + (size_t)p * CB;
    if (mode == CV_STAT_BWD) {
#pragma unroll
      for (int j = 0; j < CB; ++j) {
        const float yv = P.ep.ey[(size_t)p * CB + j];
        float v = acc[j];
        if (P.ep.erelu && bn_out(yv, ke[j]) <= 0.f) v = 0.f;
        acc[j] = v;
        s1[j] += v;
        s2[j] += v * ((yv - ke[j].mu) * ke[j].istd);
      }
    } else if (mode == CV_STAT_FWD) {
#pragma unroll
      for (int j = 0; j < CB; ++j) {
        s1[j] += acc[j];
        s2[j] += acc[j] * acc[j];
      }
    }
#pragma unroll
    for (int j = 0; j < CB; ++j) o[j] = acc[j];
  }
  if (mode != CV_STAT_NONE) stats_flush<CB>(s1, s2, P.ep.stat_out, CB, red);
}

// ---------------------------------------------------------------- host side
static int check_ep(const cv_epilogue* ep, int C, const char* what) {
  if (!ep || ep->stat_mode == CV_STAT_NONE) return 0;
  CV_REQUIRE(ep->stat_out != nullptr, "%s: epilogue stats output missing", what);
  CV_REQUIRE(ep->stat_div <= 1, "%s: stat_div must be 1 for a conv", what);
  if (ep->stat_mode == CV_STAT_BWD)
    CV_REQUIRE(ep->ey != nullptr && ep->ebn.C == C, "%s: STAT_BWD needs the BN input of width %d", what, C);
  return 0;
}

static int grid_for(long M) {
  long b = (M + NNT - 1) / NNT;
  if (b > 2048) b = 2048;
  return (int)(b < 1 ? 1 : b);
}

int narrow_gather(const Geo& g, const cv_operand* in, const float* wg, const float* bias, float* out,
                  const cv_epilogue* ep, hipStream_t st) {
  if (g.cb > 4 || g.cs != 32 || g.kh * g.kw * g.cb > 64) return -1;
  if (in->xf != CV_XF_NONE) CV_REQUIRE(in->bn.C == g.cb, "narrow_gather: BN width %d != %d", in->bn.C, g.cb);
  if (check_ep(ep, g.cs, "narrow_gather")) return 1;
  NArgs a;
  memset(&a, 0, sizeof(a));
  a.g = g;
  a.a = *in;
  a.w = wg;
  a.bias = bias;
  a.out = out;
  if (ep) a.ep = *ep;
  else a.ep.stat_mode = CV_STAT_NONE;
  a.M = (long)g.n * g.hs * g.ws;
  hipLaunchKernelGGL(narrow_gather_kernel<32>, dim3(grid_for(a.M)), dim3(NNT), 0, st, a);
  CV_LAUNCH_CHECK("narrow_gather");
  return 0;
}

int narrow_scatter(const Geo& g, const cv_operand* in, const float* ws, const float* bias, float* out,
                   const cv_epilogue* ep, hipStream_t st) {
  if (g.cb > 4 || (g.cs & 3) || g.cs > 256 || g.kh * g.kw > 16) return -1;
  if (in->xf != CV_XF_NONE) CV_REQUIRE(in->bn.C == g.cs, "narrow_scatter: BN width %d != %d", in->bn.C, g.cs);
  CV_REQUIRE(!in->nchw, "narrow_scatter: NHWC input required");
  if (check_ep(ep, g.cb, "narrow_scatter")) return 1;
  NArgs a;
  memset(&a, 0, sizeof(a));
  a.g = g;
  a.a = *in;
  a.w = ws;
  a.bias = bias;
  a.out = out;
  if (ep) a.ep = *ep;
  else a.ep.stat_mode = CV_STAT_NONE;
  a.M = (long)g.n * g.hb * g.wb;
  const size_t lds = (size_t)((g.kh * g.kw * g.cs * 4 + 3) & ~3) * 4 + 8 * g.cs * 4 + 4 * NNT * 8 + (NNT / 64) * 8 * 4;
  CV_REQUIRE(lds <= 64 * 1024, "narrow_scatter: LDS %zu", lds);
  const dim3 grid(grid_for(a.M)), blk(NNT);
  switch (g.cb) {
    case 1: hipLaunchKernelGGL(narrow_scatter_kernel<1>, grid, blk, lds, st, a); break;
    case 2: hipLaunchKernelGGL(narrow_scatter_kernel<2>, grid, blk, lds, st, a); break;
    case 3: hipLaunchKernelGGL(narrow_scatter_kernel<3>, grid, blk, lds, st, a); break;
    default: hipLaunchKernelGGL(narrow_scatter_kernel<4>, grid, blk, lds, st, a); break;
  }
  CV_LAUNCH_CHECK("narrow_scatter");
  return 0;
}

}  // namespace cv
