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
// thread = (output pixel, channel quad): 8 lanes share a pixel (same input loads, coalesced by the
// memory pipeline) and each owns a float4 of output channels, so a wave stores 1 KiB contiguously.
// The KK x KK x CB receptive field is loaded in one unrolled burst before any arithmetic, so a
// thread waits for one memory latency per pixel, not one per tap.
template <int CS, int KK, int CB>
__global__ __launch_bounds__(NNT) void narrow_gather_kernel(const NArgs P) {
  constexpr int K = KK * KK * CB;
  constexpr int NQ = CS / 4;          // lanes per pixel
  constexpr int PPB = NNT / NQ;       // pixels per block iteration
  __shared__ float4 Ws[K * NQ];
  __shared__ float4 bs[NQ];
  __shared__ BnFwdC kf[4];
  __shared__ BnBwdC kb[4];
  __shared__ BnFwdC ke[CS];
  __shared__ double scratch[4 * NNT];
  __shared__ float red[(NNT / 64) * 2 * CS];
  const int t = threadIdx.x;
  const Geo& g = P.g;
  for (int i = t; i < K * NQ; i += NNT) Ws[i] = reinterpret_cast<const float4*>(P.w)[i];
  for (int i = t; i < NQ; i += NNT)
    bs[i] = P.bias ? make_float4(P.bias[4 * i], P.bias[4 * i + 1], P.bias[4 * i + 2], P.bias[4 * i + 3])
                   : make_float4(0.f, 0.f, 0.f, 0.f);
  const int xf = P.a.xf;
  if (xf == CV_XF_BNRELU)
    bn_fold<NNT>(P.a.bn, false, scratch, [&](int f, double s, double q, double, double) {
      if (f < 4) kf[f] = bn_fwd_const_s(P.a.bn, f, s, q);
    });
  else if (xf == CV_XF_BNBWD)
    bn_fold<NNT>(P.a.bn, true, scratch, [&](int f, double s, double q, double gs, double gq) {
      if (f < 4) kb[f] = bn_bwd_const_s(P.a.bn, f, s, q, gs, gq);
    });
  const int mode = P.ep.stat_mode;
  if (mode == CV_STAT_BWD)
    bn_fold<NNT>(P.ep.ebn, false, scratch, [&](int f, double s, double q, double, double) {
      if (f < CS) ke[f] = bn_fwd_const_s(P.ep.ebn, f, s, q);
    });
  __syncthreads();

  const int q = t % NQ, pl = t / NQ;
  float4 wq[K];  // this lane's channel quad of every tap's weights (K <= 16)
#pragma unroll
  for (int i = 0; i < K; ++i) wq[i] = Ws[i * NQ + q];
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  const int hw = g.hs * g.ws;
  for (long p = (long)blockIdx.x * PPB + pl; p < P.M; p += (long)gridDim.x * PPB) {
    const int n = (int)(p / hw);
    const int rem = (int)(p - (long)n * hw);
    const int ys = rem / g.ws, xs = rem - ys * g.ws;
    const int y0 = ys * g.s - g.p, x0 = xs * g.s - g.p;
    float v[K], yv[K];
    unsigned long long okm = 0;  // receptive-field validity (zero padding stays 0 after the transform)
#pragma unroll
    for (int kh = 0; kh < KK; ++kh)
#pragma unroll
      for (int kw = 0; kw < KK; ++kw)
#pragma unroll
        for (int c = 0; c < CB; ++c) {
          const int i = (kh * KK + kw) * CB + c;
          const int yb = y0 + kh, xb = x0 + kw;
          v[i] = 0.f;
          yv[i] = 0.f;
          if ((unsigned)yb < (unsigned)g.hb && (unsigned)xb < (unsigned)g.wb) {
            const size_t off = P.a.nchw ? ((size_t)(n * CB + c) * g.hb + yb) * g.wb + xb
                                        : ((size_t)(n * g.hb + yb) * g.wb + xb) * CB + c;
            v[i] = P.a.x[off];
            if (xf == CV_XF_BNBWD) yv[i] = P.a.y[off];
            okm |= 1ull << i;
          }
        }
    float4 acc = bs[q];
#pragma unroll
    for (int i = 0; i < K; ++i) {
      const int c = i % CB;
      float a = v[i];
      const bool ok = (okm >> i) & 1ull;
      if (xf == CV_XF_BNRELU) a = ok ? bn_relu(a, kf[c]) : 0.f;
      else if (xf == CV_XF_BNBWD) a = ok ? bn_bwd(a, yv[i], kb[c]) : 0.f;
      const float4 w4 = wq[i];
      acc.x = fmaf(a, w4.x, acc.x);
      acc.y = fmaf(a, w4.y, acc.y);
      acc.z = fmaf(a, w4.z, acc.z);
      acc.w = fmaf(a, w4.w, acc.w);
    }
    float vv[4] = {acc.x, acc.y, acc.z, acc.w};
    const size_t o = (size_t)p * CS + 4 * q;
    if (mode == CV_STAT_BWD) {
      const float4 ey = *reinterpret_cast<const float4*>(P.ep.ey + o);
      const float yy[4] = {ey.x, ey.y, ey.z, ey.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const BnFwdC k = ke[4 * q + e];
        if (P.ep.erelu && bn_out(yy[e], k) <= 0.f) vv[e] = 0.f;
        s1[e] += vv[e];
        s2[e] += vv[e] * ((yy[e] - k.mu) * k.istd);
      }
    } else if (mode == CV_STAT_FWD) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s1[e] += vv[e];
        s2[e] += vv[e] * vv[e];
      }
    }
    *reinterpret_cast<float4*>(P.out + o) = make_float4(vv[0], vv[1], vv[2], vv[3]);
  }
  if (mode != CV_STAT_NONE) {
    // lanes l, l^NQ, l^2NQ, ... own the same channel quad: butterfly over the pixel lanes
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int o = NQ; o < 64; o <<= 1) {
        s1[e] += __shfl_xor(s1[e], o, 64);
        s2[e] += __shfl_xor(s2[e], o, 64);
      }
    const int lane = t & 63, w = t >> 6;
    if (lane < NQ) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        red[w * 2 * CS + 4 * lane + e] = s1[e];
        red[w * 2 * CS + CS + 4 * lane + e] = s2[e];
      }
    }
    __syncthreads();
    if (t < 2 * CS) {
      double acc2 = 0.0;
#pragma unroll
      for (int w2 = 0; w2 < NNT / 64; ++w2) acc2 += (double)red[w2 * 2 * CS + t];
      const int repl = blockIdx.x % CV_STAT_REPL(CS);
      atomic_add_f64(P.ep.stat_out + (size_t)repl * 2 * CS + t, acc2);
    }
  }
}

// ---------------------------------------------------------------- narrow scatter (cb <= 4 outputs)
// 4 lanes per big-grid output pixel, each owning 8 of the CS = 32 input channels; the pixels of a
// block belong to one stride-parity class (blockIdx.y), so every lane walks the same NT2 x NT2 taps.
// All of a lane's tap loads are issued before any arithmetic; partial sums meet by two shuffles.
template <int CB, int NT2>
__global__ __launch_bounds__(NNT) void narrow_scatter_kernel(const NArgs P) {
  constexpr int CS = 32, LPP = 4, CPL = CS / LPP;  // channels per lane (2 float4)
  constexpr int TP = NT2 * NT2;                      // taps of a class
  __shared__ float Wl[16 * CS * CB];
  __shared__ BnFwdC kf[CS];
  __shared__ BnBwdC kb[CS];
  __shared__ double scratch[4 * NNT];
  __shared__ float red[(NNT / 64) * 2 * 4];
  __shared__ float bs[4];
  __shared__ BnFwdC ke[4];
  const Geo& g = P.g;
  const int t = threadIdx.x;
  for (int i = t; i < g.kh * g.kw * CS * CB; i += NNT) Wl[i] = P.w[i];
  if (t < CB) bs[t] = P.bias ? P.bias[t] : 0.f;
  const int xf = P.a.xf;
  if (xf == CV_XF_BNRELU)
    bn_fold<NNT>(P.a.bn, false, scratch, [&](int f, double s, double q, double, double) {
      kf[f] = bn_fwd_const_s(P.a.bn, f, s, q);
    });
  else if (xf == CV_XF_BNBWD)
    bn_fold<NNT>(P.a.bn, true, scratch, [&](int f, double s, double q, double gs, double gq) {
      kb[f] = bn_bwd_const_s(P.a.bn, f, s, q, gs, gq);
    });
  const int mode = P.ep.stat_mode;
  if (mode == CV_STAT_BWD)
    bn_fold<NNT>(P.ep.ebn, false, scratch, [&](int f, double s, double q, double, double) {
      if (f < 4) ke[f] = bn_fwd_const_s(P.ep.ebn, f, s, q);
    });
  __syncthreads();

  const int s = g.s, cls = blockIdx.y;
  const int ry = cls / s, rx = cls % s;
  const int yb0 = (((ry - g.p) % s) + s) % s, xb0 = (((rx - g.p) % s) + s) % s;
  const int cy = (g.hb > yb0) ? (g.hb - yb0 + s - 1) / s : 0;
  const int cx = (g.wb > xb0) ? (g.wb - xb0 + s - 1) / s : 0;
  const int nty = (g.kh > ry) ? (g.kh - ry + s - 1) / s : 0;
  const int ntx = (g.kw > rx) ? (g.kw - rx + s - 1) / s : 0;
  const long Mc = (long)g.n * cy * cx;
  const int sub = t % LPP, c0 = sub * CPL;
  // this lane's 8 channels: BatchNorm constants and the class's tap weights live in registers
  float k_sc[CPL], k_mu[CPL], k_be[CPL], k_c1[CPL], k_c2[CPL];
#pragma unroll
  for (int e = 0; e < CPL; ++e) {
    k_sc[e] = 1.f; k_mu[e] = 0.f; k_be[e] = 0.f; k_c1[e] = 0.f; k_c2[e] = 0.f;
    if (xf == CV_XF_BNRELU) {
      const BnFwdC k = kf[c0 + e];
      k_sc[e] = k.sc; k_mu[e] = k.mu; k_be[e] = k.be;
    } else if (xf == CV_XF_BNBWD) {
      const BnBwdC k = kb[c0 + e];
      k_sc[e] = k.sc; k_mu[e] = k.mu; k_be[e] = k.istd; k_c1[e] = k.c1; k_c2[e] = k.c2;
    }
  }
  float wr[TP][CPL][CB];
#pragma unroll
  for (int jy = 0; jy < NT2; ++jy)
#pragma unroll
    for (int jx = 0; jx < NT2; ++jx) {
      const int kh = ry + s * jy, kw = rx + s * jx;
      const bool tap_ok = jy < nty && jx < ntx;
#pragma unroll
      for (int e = 0; e < CPL; ++e)
#pragma unroll
        for (int j = 0; j < CB; ++j)
          wr[jy * NT2 + jx][e][j] = tap_ok ? Wl[((kh * g.kw + kw) * CS + c0 + e) * CB + j] : 0.f;
    }
  const FDiv f_cycx = FDiv::make(cy * cx), f_cx = FDiv::make(cx);
  float s1[CB], s2[CB];
#pragma unroll
  for (int j = 0; j < CB; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  const long rstride = (long)gridDim.x * (NNT / LPP);
  // every lane runs the same trip count (the shuffles below need whole waves)
  const long trips = (Mc + rstride - 1) / rstride;
  for (long it = 0; it < trips; ++it) {
    const long r = it * rstride + (long)blockIdx.x * (NNT / LPP) + t / LPP;
    const bool live = r < Mc;
    const int rr = live ? (int)r : 0;
    const int n = f_cycx.div(rr);
    const int rem = rr - n * cy * cx;
    const int ty = f_cx.div(rem), tx = rem - ty * cx;
    const int yb = yb0 + s * ty, xb = xb0 + s * tx;
    float4 xv[TP][2], yv4[TP][2];
    bool ok[TP];
#pragma unroll
    for (int jy = 0; jy < NT2; ++jy)
#pragma unroll
      for (int jx = 0; jx < NT2; ++jx) {
        const int tp = jy * NT2 + jx;
        const int kh = ry + s * jy, kw = rx + s * jx;
        const int py = yb + g.p - kh, px = xb + g.p - kw;
        const int ys = py >> 1, xs = px >> 1;  // s == 2 (host-checked); exact within the class
        ok[tp] = live && jy < nty && jx < ntx && py >= 0 && px >= 0 && ys < g.hs && xs < g.ws;
        xv[tp][0] = xv[tp][1] = make_float4(0.f, 0.f, 0.f, 0.f);
        yv4[tp][0] = yv4[tp][1] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ok[tp]) {
          const float* src = P.a.x + ((size_t)(n * g.hs + ys) * g.ws + xs) * CS + c0;
          xv[tp][0] = *reinterpret_cast<const float4*>(src);
          xv[tp][1] = *reinterpret_cast<const float4*>(src + 4);
          if (xf == CV_XF_BNBWD) {
            const float* ysrc = P.a.y + ((size_t)(n * g.hs + ys) * g.ws + xs) * CS + c0;
            yv4[tp][0] = *reinterpret_cast<const float4*>(ysrc);
            yv4[tp][1] = *reinterpret_cast<const float4*>(ysrc + 4);
          }
        }
      }
    float acc[CB];
#pragma unroll
    for (int j = 0; j < CB; ++j) acc[j] = 0.f;
#pragma unroll
    for (int jy = 0; jy < NT2; ++jy)
#pragma unroll
      for (int jx = 0; jx < NT2; ++jx) {
        const int tp = jy * NT2 + jx;
        if (!ok[tp]) continue;
        const float xs8[8] = {xv[tp][0].x, xv[tp][0].y, xv[tp][0].z, xv[tp][0].w,
                              xv[tp][1].x, xv[tp][1].y, xv[tp][1].z, xv[tp][1].w};
        const float ys8[8] = {yv4[tp][0].x, yv4[tp][0].y, yv4[tp][0].z, yv4[tp][0].w,
                              yv4[tp][1].x, yv4[tp][1].y, yv4[tp][1].z, yv4[tp][1].w};
#pragma unroll
        for (int e = 0; e < CPL; ++e) {
          float a = xs8[e];
          if (xf == CV_XF_BNRELU) a = fmaxf(fmaf(a - k_mu[e], k_sc[e], k_be[e]), 0.f);
          else if (xf == CV_XF_BNBWD) a = k_sc[e] * (a - k_c1[e] - (ys8[e] - k_mu[e]) * k_be[e] * k_c2[e]);
#pragma unroll
          for (int j = 0; j < CB; ++j) acc[j] = fmaf(a, wr[tp][e][j], acc[j]);
        }
      }
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      acc[j] += __shfl_xor(acc[j], 1, 64);
      acc[j] += __shfl_xor(acc[j], 2, 64);
    }
    if (live && sub == 0) {
      const size_t po = ((size_t)(n * g.hb + yb) * g.wb + xb) * CB;
#pragma unroll
      for (int j = 0; j < CB; ++j) {
        float v = acc[j] + bs[j];
        if (mode == CV_STAT_BWD) {
          const float yv = P.ep.ey[po + j];
          if (P.ep.erelu && bn_out(yv, ke[j]) <= 0.f) v = 0.f;
          s1[j] += v;
          s2[j] += v * ((yv - ke[j].mu) * ke[j].istd);
        } else if (mode == CV_STAT_FWD) {
          s1[j] += v;
          s2[j] += v * v;
        }
        P.out[po + j] = v;
      }
    }
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
  if (g.cs != 32 || g.kh != g.kw || (g.kh != 3 && g.kh != 4) || (g.cb != 1 && g.cb != 3)) return -1;
  if (g.cb != 1) return -1;  // K = 27 / 48 (3-channel images) is a real contraction: MFMA igemm
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
  long blocks = (a.M + 31) / 32;  // 32 pixels per block iteration
  if (blocks > 1024) blocks = 1024;
  const dim3 grid((int)blocks), blk(NNT);
  note_launch(g.kh == 3 ? (const void*)narrow_gather_kernel<32, 3, 1> : (const void*)narrow_gather_kernel<32, 4, 1>);
  if (g.kh == 3) hipLaunchKernelGGL((narrow_gather_kernel<32, 3, 1>), grid, blk, 0, st, a);
  else hipLaunchKernelGGL((narrow_gather_kernel<32, 4, 1>), grid, blk, 0, st, a);
  CV_LAUNCH_CHECK("narrow_gather");
  return 0;
}

int narrow_scatter(const Geo& g, const cv_operand* in, const float* ws, const float* bias, float* out,
                   const cv_epilogue* ep, hipStream_t st) {
  if (g.cb > 4 || g.cs != 32 || g.s != 2 || g.kh != g.kw || (g.kh != 3 && g.kh != 4)) return -1;
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
  const long rows = (long)g.n * cdiv(g.hb, g.s) * cdiv(g.wb, g.s);  // largest class
  long bx = (rows + 63) / 64;  // 64 pixels per block iteration
  if (bx > 512) bx = 512;       // bounds the fp64 atomics per statistics address
  const dim3 grid((int)bx, g.s * g.s), blk(NNT);
#define CV_NS(CBV) do { note_launch((const void*)narrow_scatter_kernel<CBV, 2>); hipLaunchKernelGGL((narrow_scatter_kernel<CBV, 2>), grid, blk, 0, st, a); } while (0)
  switch (g.cb) {
    case 1: CV_NS(1); break;
    case 2: CV_NS(2); break;
    case 3: CV_NS(3); break;
    default: CV_NS(4); break;
  }
#undef CV_NS
  CV_LAUNCH_CHECK("narrow_scatter");
  return 0;
}

}  // namespace cv
