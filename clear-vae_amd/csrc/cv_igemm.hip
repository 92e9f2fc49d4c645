// Implicit-GEMM convolution / linear kernels on fp32 MFMA (v_mfma_f32_16x16x4_f32) for gfx950.
//
// One templated main loop serves every dense contraction of the CLEAR-VAE step:
//   GATHER  : out[small pixel][cs]  = sum_{tap,cb} T(big[pixel*s-p+tap][cb]) * w(cs,cb,tap)
//             (Conv2d forward, ConvTranspose2d backward-data, the 4 latent heads as a whole-image conv)
//   SCATTER : out[big pixel][cb]    = sum_{tap,cs} T(small[(pixel+p-tap)/s][cs]) * w(cs,cb,tap)
//             (Conv2d backward-data, ConvTranspose2d forward, the heads' backward-data), decomposed
//             into stride^2 parity classes so every class is a dense GEMM with no masked taps
//   WGRAD   : dw(cs,cb,tap)        += sum_{small pixel} T(small[pixel][cs]) * T(big[gather][cb])
//             (grad_weight of every conv / convT / head), split-K over pixels, fp32 atomics
//   DENSE   : out[row][col]         = sum_k T(A[row][perm(k)]) * W(k,col)   (decoder Linear)
// T() is the fused BatchNorm(+ReLU) forward or backward transform (cv_common.hpp); BN batch
// statistics of the produced tensor are reduced in the epilogue (fp64 atomics, 8 replicas).
//
// Reference arithmetic replaced: nn.Conv2d / nn.ConvTranspose2d / nn.Linear / nn.BatchNorm2d / ReLU
// of code/src/models/vae.py:15-46 (VAE) and :113-156 (VAE64), forward and autograd backward.
//
// Tile: BM x BN x 16, 256 threads = 4 waves laid out WM x WN; each wave owns (BM/WM) x (BN/WN)
// as 16x16 MFMA tiles. Operands are staged global -> registers -> LDS (k-major, padded so the
// ds_read_b32 operand fetches are bank-conflict free), the next tile's global loads are issued
// before the current tile's MFMAs (register double buffering).
#include "cv_common.hpp"

namespace cv {

constexpr int BK = 16;
constexpr int NT = 256;

enum { OP_GATHER = 0, OP_SCATTER = 1, OP_WGRAD = 2, OP_DENSE = 3 };

// generic geometry shared by the conv problems (small grid S, big grid B, yb = ys*s - p + kh)
struct Geo {
  int n, hs, ws, cs, hb, wb, cb, kh, kw, s, p;
};

// Per-problem arguments (passed by value as the kernel argument).
struct Args {
  int op;
  Geo g;
  cv_operand a;        // GATHER: big-grid input; SCATTER: small-grid input; WGRAD: small-grid; DENSE: A
  cv_operand b;        // WGRAD: big-grid operand
  const float* w;      // weights (GATHER/SCATTER/DENSE)
  int wlayout;         // DENSE: 0 -> W[col*ldb + k], 1 -> W[k*ldb + col]
  int ldb;
  const float* bias;
  float* gbias;        // WGRAD: bias gradient via an extra all-ones B column
  float* out;
  int accumulate;      // atomicAdd into out (split-K)
  cv_epilogue ep;
  int M, N, K;         // GEMM sizes (SCATTER: per class sizes computed in-kernel)
  int ksplit;          // number of K splits (grid.z for GATHER/WGRAD/DENSE)
  int kchunk;          // K elements per split (multiple of BK)
  // DENSE
  int lda, a_pix, a_ch;      // A row stride; NCHW-flatten permutation of A columns (a_pix=1: none)
  int ldo, o_pix, o_ch;      // out row stride; permutation of output columns
  // constants sizes (LDS)
  int ca_n, cb_n, ce_n;      // feature counts of a / b / epilogue BN constants (0 = unused)
};

// ------------------------------------------------------------------ operand transform helpers
struct XfA {
  // LDS views of constants
  const BnFwdC* f;
  const BnBwdC* bw;
};

__device__ __forceinline__ float xf_apply(const cv_operand& o, const XfA& c, int ch, float x, float y) {
  if (o.xf == CV_XF_BNRELU) return bn_relu(x, c.f[ch]);
  if (o.xf == CV_XF_BNBWD) return bn_bwd(x, y, c.bw[ch]);
  return x;
}

__device__ __forceinline__ void fill_consts(const cv_operand& o, int nfeat, float* lds, XfA& c) {
  c.f = reinterpret_cast<const BnFwdC*>(lds);
  c.bw = reinterpret_cast<const BnBwdC*>(lds);
  if (o.xf == CV_XF_BNRELU) {
    BnFwdC* d = reinterpret_cast<BnFwdC*>(lds);
    for (int i = threadIdx.x; i < nfeat; i += NT) d[i] = bn_fwd_const(o.bn, i);
  } else if (o.xf == CV_XF_BNBWD) {
    BnBwdC* d = reinterpret_cast<BnBwdC*>(lds);
    for (int i = threadIdx.x; i < nfeat; i += NT) d[i] = bn_bwd_const(o.bn, i);
  }
}

__host__ __device__ inline int xf_floats(int xf, int nfeat) {
  if (xf == CV_XF_BNRELU) return 4 * nfeat;
  if (xf == CV_XF_BNBWD) return 5 * nfeat;
  return 0;
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// ------------------------------------------------------------------ the kernel
template <int BM, int BN>
__global__ __launch_bounds__(NT) void igemm_kernel(const Args P) {
  constexpr int WN = (BN >= 32) ? 2 : 1;
  constexpr int WM = 4 / WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  static_assert(FM >= 1 && FN >= 1, "tile too small");
  constexpr int LDA = BM + 16;
  constexpr int LDB = BN + ((BN % 32) == 0 ? 16 : 0);
  constexpr int AR = BM * BK / NT;  // A floats per thread
  constexpr int BR = BN * BK / NT;  // B floats per thread (may be < 1 -> handled as 1 with guard)
  constexpr int BRR = BR > 0 ? BR : 1;

  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* As = smem;
  float* Bs = As + BK * LDA;
  float* red = Bs + BK * LDB;          // epilogue reduction scratch: 2 * WM * BN floats
  float* cst = red + 2 * WM * BN;      // BN constants
  float* cstA = cst;
  float* cstB = cstA + xf_floats(P.a.xf, P.ca_n);
  float* cstE = cstB + xf_floats(P.b.xf, P.cb_n);

  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int wm = wid / WN, wn = wid % WN;

  // ---------------- block -> (m0, n0, k-range, class)
  int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  int M = P.M, N = P.N, K = P.K;
  int kbeg = 0, kend = K;
  // SCATTER class data
  int ry = 0, rx = 0, yb0 = 0, xb0 = 0, cy = 1, cx = 1, nty = 1, ntx = 1;
  if (P.op == OP_SCATTER) {
    const int s = P.g.s;
    const int cls = blockIdx.z;
    ry = cls / s;
    rx = cls % s;
    // big rows with (yb + p) % s == ry
    yb0 = (((ry - P.g.p) % s) + s) % s;
    xb0 = (((rx - P.g.p) % s) + s) % s;
    cy = (P.g.hb > yb0) ? (P.g.hb - yb0 + s - 1) / s : 0;
    cx = (P.g.wb > xb0) ? (P.g.wb - xb0 + s - 1) / s : 0;
    nty = (P.g.kh > ry) ? (P.g.kh - ry + s - 1) / s : 0;
    ntx = (P.g.kw > rx) ? (P.g.kw - rx + s - 1) / s : 0;
    M = P.g.n * cy * cx;
    K = nty * ntx * P.g.cs;
    kend = K;
    if (m0 >= M) return;
  } else {
    const int z = blockIdx.z;
    kbeg = z * P.kchunk;
    kend = min(K, kbeg + P.kchunk);
    if (kbeg >= kend) return;
  }

  // ---------------- prologue: BN constants into LDS
  XfA ca, cb, ce;
  fill_consts(P.a, P.ca_n, cstA, ca);
  fill_consts(P.b, P.cb_n, cstB, cb);
  ce.f = nullptr;
  ce.bw = nullptr;
  if (P.ep.stat_mode == CV_STAT_BWD) {
    BnFwdC* d = reinterpret_cast<BnFwdC*>(cstE);
    for (int i = t; i < P.ce_n; i += NT) d[i] = bn_fwd_const(P.ep.ebn, i);
  }
  __syncthreads();

  // ---------------- per-thread A-row decode (row-oriented problems)
  constexpr int RA = (BM >= 64) ? BM / 64 : 1;
  int r_n[RA], r_y[RA], r_x[RA];
  bool r_ok[RA];
  const int quad = (t >> 4) & 3;
  if (P.op == OP_GATHER || P.op == OP_SCATTER || P.op == OP_DENSE) {
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const int r = m0 + (t & 15) + 16 * (t >> 6) + 64 * i;
      r_ok[i] = (r < M) && (BM >= 64 || (t >> 6) < BM / 16);
      const int rr = r_ok[i] ? r : 0;
      if (P.op == OP_GATHER) {
        const int hw = P.g.hs * P.g.ws;
        r_n[i] = rr / hw;
        const int rem = rr - r_n[i] * hw;
        r_y[i] = rem / P.g.ws;
        r_x[i] = rem - r_y[i] * P.g.ws;
      } else if (P.op == OP_SCATTER) {
        const int hw = cy * cx;
        r_n[i] = rr / hw;
        const int rem = rr - r_n[i] * hw;
        const int ty = rem / cx, tx = rem - ty * cx;
        r_y[i] = yb0 + P.g.s * ty;  // big-grid coordinates
        r_x[i] = xb0 + P.g.s * tx;
      } else {
        r_n[i] = rr;
        r_y[i] = 0;
        r_x[i] = 0;
      }
    }
  }

  float ra[AR], rb[BRR];

  // ---------------- operand fetchers
  auto fetchA = [&](int k0) {
    if (P.op == OP_GATHER) {
      const Geo& g = P.g;
      const int kq = k0 + 4 * quad;
      const bool vec = (g.cb % 4) == 0 && !P.a.nchw;
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        if (vec) {
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          if (r_ok[i] && kq < kend) {
            const int tap = kq / g.cb, c0 = kq - tap * g.cb;
            const int kh = tap / g.kw, kw = tap - kh * g.kw;
            const int yb = r_y[i] * g.s - g.p + kh, xb = r_x[i] * g.s - g.p + kw;
            if (yb >= 0 && yb < g.hb && xb >= 0 && xb < g.wb) {
              const size_t off = ((size_t)(r_n[i] * g.hb + yb) * g.wb + xb) * g.cb + c0;
              v = ld4(P.a.x + off);
              if (P.a.xf != CV_XF_NONE) {
                float4 yy = make_float4(0.f, 0.f, 0.f, 0.f);
                if (P.a.xf == CV_XF_BNBWD) yy = ld4(P.a.y + off);
                v.x = xf_apply(P.a, ca, c0 + 0, v.x, yy.x);
                v.y = xf_apply(P.a, ca, c0 + 1, v.y, yy.y);
                v.z = xf_apply(P.a, ca, c0 + 2, v.z, yy.z);
                v.w = xf_apply(P.a, ca, c0 + 3, v.w, yy.w);
              }
            }
          }
          ra[4 * i + 0] = v.x; ra[4 * i + 1] = v.y; ra[4 * i + 2] = v.z; ra[4 * i + 3] = v.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float v = 0.f;
            const int k = kq + j;
            if (r_ok[i] && k < kend) {
              const int tap = k / g.cb, c = k - tap * g.cb;
              const int kh = tap / g.kw, kw = tap - kh * g.kw;
              const int yb = r_y[i] * g.s - g.p + kh, xb = r_x[i] * g.s - g.p + kw;
              if (yb >= 0 && yb < g.hb && xb >= 0 && xb < g.wb) {
                const size_t off = P.a.nchw ? ((size_t)(r_n[i] * g.cb + c) * g.hb + yb) * g.wb + xb
                                            : ((size_t)(r_n[i] * g.hb + yb) * g.wb + xb) * g.cb + c;
                const float yv = (P.a.xf == CV_XF_BNBWD) ? P.a.y[off] : 0.f;
                v = xf_apply(P.a, ca, c, P.a.x[off], yv);
              }
            }
            ra[4 * i + j] = v;
          }
        }
      }
    } else if (P.op == OP_SCATTER) {
      const Geo& g = P.g;
      const int kq = k0 + 4 * quad;
      const bool vec = (g.cs % 4) == 0;
#pragma unroll
      for (int i = 0; i < RA; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (!vec || j == 0) {
            const int k = kq + j;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (r_ok[i] && k < kend) {
              const int tap = k / g.cs, c = k - tap * g.cs;
              const int jy = tap / ntx, jx = tap - jy * ntx;
              const int kh = ry + g.s * jy, kw = rx + g.s * jx;
              const int ys = (r_y[i] + g.p - kh) / g.s, xs = (r_x[i] + g.p - kw) / g.s;
              if (ys >= 0 && ys < g.hs && xs >= 0 && xs < g.ws &&
                  (r_y[i] + g.p - kh) >= 0 && (r_x[i] + g.p - kw) >= 0) {
                const size_t off = ((size_t)(r_n[i] * g.hs + ys) * g.ws + xs) * g.cs + c;
                if (vec) {
                  v = ld4(P.a.x + off);
                  if (P.a.xf != CV_XF_NONE) {
                    float4 yy = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (P.a.xf == CV_XF_BNBWD) yy = ld4(P.a.y + off);
                    v.x = xf_apply(P.a, ca, c + 0, v.x, yy.x);
                    v.y = xf_apply(P.a, ca, c + 1, v.y, yy.y);
                    v.z = xf_apply(P.a, ca, c + 2, v.z, yy.z);
                    v.w = xf_apply(P.a, ca, c + 3, v.w, yy.w);
                  }
                } else {
                  const float yv = (P.a.xf == CV_XF_BNBWD) ? P.a.y[off] : 0.f;
                  v.x = xf_apply(P.a, ca, c, P.a.x[off], yv);
                }
              }
            }
            if (vec) {
              ra[4 * i + 0] = v.x; ra[4 * i + 1] = v.y; ra[4 * i + 2] = v.z; ra[4 * i + 3] = v.w;
            } else {
              ra[4 * i + j] = v.x;
            }
          }
        }
      }
    } else if (P.op == OP_DENSE) {
      const int kq = k0 + 4 * quad;
#pragma unroll
      for (int i = 0; i < RA; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = kq + j;
          float v = 0.f;
          if (r_ok[i] && k < kend) {
            const int col = (P.a_pix > 1) ? (k % P.a_pix) * P.a_ch + k / P.a_pix : k;
            const size_t off = (size_t)r_n[i] * P.lda + col;
            const float yv = (P.a.xf == CV_XF_BNBWD) ? P.a.y[off] : 0.f;
            // constants are per logical feature k (BN1d) or per channel k / a_pix (BN2d)
            v = xf_apply(P.a, ca, (P.ca_n == K) ? k : k / P.a_pix, P.a.x[off], yv);
          }
          ra[4 * i + j] = v;
        }
      }
    } else {  // OP_WGRAD: A(m = cs, k = small pixel) = T(small[pix][cs]); As[k][m]
      const Geo& g = P.g;
      constexpr int MQ = BM / 4;                 // float4 per pixel row of the tile
      constexpr int PER = (MQ * BK) / NT;        // float4 per thread (>=1 when BM>=64)
      constexpr int PERR = PER > 0 ? PER : 1;
#pragma unroll
      for (int e = 0; e < PERR; ++e) {
        const int idx = t + NT * e;
        const int mq = idx % MQ, kk = idx / MQ;
        const int pix = k0 + kk;
        const int c0 = m0 + 4 * mq;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (kk < BK && pix < kend) {
          const size_t off = (size_t)pix * g.cs + c0;
          if ((g.cs % 4) == 0 && c0 + 3 < g.cs) {
            v = ld4(P.a.x + off);
            float4 yy = make_float4(0.f, 0.f, 0.f, 0.f);
            if (P.a.xf == CV_XF_BNBWD) yy = ld4(P.a.y + off);
            if (P.a.xf != CV_XF_NONE) {
              v.x = xf_apply(P.a, ca, c0 + 0, v.x, yy.x);
              v.y = xf_apply(P.a, ca, c0 + 1, v.y, yy.y);
              v.z = xf_apply(P.a, ca, c0 + 2, v.z, yy.z);
              v.w = xf_apply(P.a, ca, c0 + 3, v.w, yy.w);
            }
          } else {
            float tmp[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              tmp[j] = 0.f;
              if (c0 + j < g.cs) {
                const float yv = (P.a.xf == CV_XF_BNBWD) ? P.a.y[off + j] : 0.f;
                tmp[j] = xf_apply(P.a, ca, c0 + j, P.a.x[off + j], yv);
              }
            }
            v = make_float4(tmp[0], tmp[1], tmp[2], tmp[3]);
          }
        }
        ra[4 * e + 0] = v.x; ra[4 * e + 1] = v.y; ra[4 * e + 2] = v.z; ra[4 * e + 3] = v.w;
      }
    }
  };

  auto storeA = [&]() {
    if (P.op == OP_WGRAD) {
      constexpr int MQ = BM / 4;
      constexpr int PER = (MQ * BK) / NT;
      constexpr int PERR = PER > 0 ? PER : 1;
#pragma unroll
      for (int e = 0; e < PERR; ++e) {
        const int idx = t + NT * e;
        const int mq = idx % MQ, kk = idx / MQ;
        if (kk < BK) {
#pragma unroll
          for (int j = 0; j < 4; ++j) As[kk * LDA + 4 * mq + j] = ra[4 * e + j];
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        const int m = (t & 15) + 16 * (t >> 6) + 64 * i;
        if (m < BM) {
#pragma unroll
          for (int j = 0; j < 4; ++j) As[(4 * quad + j) * LDA + m] = ra[4 * i + j];
        }
      }
    }
  };

  auto fetchB = [&](int k0) {
#pragma unroll
    for (int e = 0; e < BRR; ++e) {
      const int idx = t + NT * e;
      const int nn = idx % BN, kk = idx / BN;
      const int col = n0 + nn, k = k0 + kk;
      float v = 0.f;
      if (kk < BK && col < N && k < kend) {
        if (P.op == OP_GATHER) {
          const Geo& g = P.g;
          const int tap = k / g.cb, c = k - tap * g.cb;
          // w(cs=col, cb=c, tap)
          v = P.w[((size_t)col * g.cb + c) * (g.kh * g.kw) + tap];
        } else if (P.op == OP_SCATTER) {
          const Geo& g = P.g;
          const int tap = k / g.cs, c = k - tap * g.cs;
          const int jy = tap / ntx, jx = tap - jy * ntx;
          const int kh = ry + g.s * jy, kw = rx + g.s * jx;
          v = P.w[(((size_t)c * g.cb + col) * g.kh + kh) * g.kw + kw];
        } else if (P.op == OP_DENSE) {
          v = P.wlayout ? P.w[(size_t)k * P.ldb + col] : P.w[(size_t)col * P.ldb + k];
        } else if (P.gbias && col == N - 1) {  // WGRAD bias column
          v = 1.0f;
        } else {  // WGRAD: B(k = small pixel, col = (tap, cb)) = T(big[gather(pix, tap)][cb])
          const Geo& g = P.g;
          const int tap = col / g.cb, c = col - tap * g.cb;
          const int kh = tap / g.kw, kw = tap - kh * g.kw;
          const int hw = g.hs * g.ws;
          const int nimg = k / hw, rem = k - nimg * hw;
          const int ys = rem / g.ws, xs = rem - ys * g.ws;
          const int yb = ys * g.s - g.p + kh, xb = xs * g.s - g.p + kw;
          if (yb >= 0 && yb < g.hb && xb >= 0 && xb < g.wb) {
            const size_t off = P.b.nchw ? ((size_t)(nimg * g.cb + c) * g.hb + yb) * g.wb + xb
                                        : ((size_t)(nimg * g.hb + yb) * g.wb + xb) * g.cb + c;
            const float yv = (P.b.xf == CV_XF_BNBWD) ? P.b.y[off] : 0.f;
            v = xf_apply(P.b, cb, c, P.b.x[off], yv);
          }
        }
      }
      rb[e] = v;
    }
  };

  auto storeB = [&]() {
#pragma unroll
    for (int e = 0; e < BRR; ++e) {
      const int idx = t + NT * e;
      const int nn = idx % BN, kk = idx / BN;
      if (kk < BK) Bs[kk * LDB + nn] = rb[e];
    }
  };

  // ---------------- main loop
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  fetchA(kbeg);
  fetchB(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    __syncthreads();
    storeA();
    storeB();
    __syncthreads();
    if (k0 + BK < kend) {
      fetchA(k0 + BK);
      fetchB(k0 + BK);
    }
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      const int kr = kk + (lane >> 4);
      float av[FM], bv[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) av[i] = As[kr * LDA + wm * TM + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < FN; ++j) bv[j] = Bs[kr * LDB + wn * TN + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
  }

  // ---------------- epilogue
  const bool stats = P.ep.stat_mode != CV_STAT_NONE;
  const int repl = blockIdx.x % CV_STAT_REPL;
  float s1[FN], s2[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) { s1[j] = 0.f; s2[j] = 0.f; }

#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = n0 + wn * TN + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * TM + i * 16 + (lane >> 4) * 4 + r;
        float v = acc[i][j][r];
        if (row >= M || col >= N) continue;
        if (P.op == OP_WGRAD) {
          if (P.gbias && col == N - 1) {
            atomicAdd(P.gbias + row, v);
            continue;
          }
          // row = cs, col = (tap, cb) -> w layout [cs][cb][kh][kw]
          const Geo& g = P.g;
          const int tap = col / g.cb, c = col - tap * g.cb;
          atomicAdd(P.out + ((size_t)row * g.cb + c) * (g.kh * g.kw) + tap, v);
          continue;
        }
        size_t off;
        if (P.op == OP_GATHER) {
          off = (size_t)row * P.g.cs + col;
        } else if (P.op == OP_SCATTER) {
          const int hw = cy * cx;
          const int nimg = row / hw, rem = row - nimg * hw;
          const int ty = rem / cx, tx = rem - ty * cx;
          const int yb = yb0 + P.g.s * ty, xb = xb0 + P.g.s * tx;
          off = ((size_t)(nimg * P.g.hb + yb) * P.g.wb + xb) * P.g.cb + col;
        } else {
          const int oc = (P.o_pix > 1) ? (col % P.o_pix) * P.o_ch + col / P.o_pix : col;
          off = (size_t)row * P.ldo + oc;
        }
        if (P.bias && (!P.accumulate || blockIdx.z == 0)) v += P.bias[col];
        if (P.accumulate) {
          atomicAdd(P.out + off, v);
          continue;
        }
        if (P.ep.stat_mode == CV_STAT_BWD) {
          const int f = col / P.ep.stat_div;
          const float yv = P.ep.ey[off];
          const BnFwdC k = reinterpret_cast<const BnFwdC*>(cstE)[f];
          if (P.ep.erelu && bn_out(yv, k) <= 0.f) v = 0.f;
          P.out[off] = v;
          s1[j] += v;
          s2[j] += v * ((yv - k.mu) * k.istd);
        } else {
          P.out[off] = v;
          if (stats) {
            s1[j] += v;
            s2[j] += v * v;
          }
        }
      }
    }
  }

  if (stats && !P.accumulate && P.op != OP_WGRAD) {
    // reduce per column: lanes with equal (lane & 15), then the WM waves sharing wn
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      s1[j] += __shfl_xor(s1[j], 16, 64);
      s1[j] += __shfl_xor(s1[j], 32, 64);
      s2[j] += __shfl_xor(s2[j], 16, 64);
      s2[j] += __shfl_xor(s2[j], 32, 64);
    }
    __syncthreads();  // red may alias nothing, but As/Bs are free now
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int c = wn * TN + j * 16 + lane;
        red[(wm)*BN + c] = s1[j];
        red[WM * BN + wm * BN + c] = s2[j];
      }
    }
    __syncthreads();
    if (t < BN) {
      const int col = n0 + t;
      if (col < N) {
        double a = 0.0, b = 0.0;
#pragma unroll
        for (int w = 0; w < WM; ++w) {
          a += (double)red[w * BN + t];
          b += (double)red[WM * BN + w * BN + t];
        }
        const int f = col / P.ep.stat_div;
        const int C = (P.ep.stat_mode == CV_STAT_BWD) ? P.ce_n : P.ep.ebn.C;
        double* so = P.ep.stat_out + (size_t)repl * 2 * C;
        atomic_add_f64(so + f, a);
        atomic_add_f64(so + C + f, b);
      }
    }
  }
}

// ------------------------------------------------------------------ host-side launch
static size_t lds_bytes(const Args& a, int BM_, int BN_) {
  const int WN = (BN_ >= 32) ? 2 : 1, WM = 4 / WN;
  const int LDA = BM_ + 16, LDB = BN_ + ((BN_ % 32) == 0 ? 16 : 0);
  size_t f = (size_t)BK * LDA + (size_t)BK * LDB + 2 * WM * BN_;
  f += xf_floats(a.a.xf, a.ca_n) + xf_floats(a.b.xf, a.cb_n);
  if (a.ep.stat_mode == CV_STAT_BWD) f += 4 * (size_t)a.ce_n;
  return f * sizeof(float);
}

template <int BM, int BN>
static int launch_t(const Args& a, dim3 grid, hipStream_t st) {
  const size_t lds = lds_bytes(a, BM, BN);
  CV_REQUIRE(lds <= 160 * 1024, "igemm: LDS request %zu bytes exceeds 160 KiB", lds);
  if (lds > 64 * 1024) {
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute((const void*)igemm_kernel<BM, BN>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          160 * 1024);
      attr_set = true;
    }
  }
  hipLaunchKernelGGL((igemm_kernel<BM, BN>), grid, dim3(NT), lds, st, a);
  CV_LAUNCH_CHECK("igemm");
  return 0;
}

static int launch(Args& a, int BM_, int BN_, int gz, hipStream_t st) {
  // grid.x covers M (for SCATTER the largest class), grid.y covers N
  const int gx = cdiv(a.M, BM_), gy = cdiv(a.N, BN_);
  dim3 grid(gx, gy, gz);
  CV_REQUIRE(gx > 0 && gy > 0 && gz > 0, "igemm: empty grid");
  CV_REQUIRE(gx < (1 << 30) && gy < 65536 && gz < 65536, "igemm: grid too large");
  if (BM_ == 128 && BN_ == 64) return launch_t<128, 64>(a, grid, st);
  if (BM_ == 128 && BN_ == 32) return launch_t<128, 32>(a, grid, st);
  if (BM_ == 64 && BN_ == 64) return launch_t<64, 64>(a, grid, st);
  if (BM_ == 64 && BN_ == 32) return launch_t<64, 32>(a, grid, st);
  if (BM_ == 64 && BN_ == 16) return launch_t<64, 16>(a, grid, st);
  if (BM_ == 128 && BN_ == 16) return launch_t<128, 16>(a, grid, st);
  cv::set_error("igemm: unsupported tile %dx%d", BM_, BN_);
  return 1;
}

static int pick_bn(int N) {
  if (N <= 16) return 16;
  if (N <= 32) return 32;
  return 64;
}

// number of K splits: aim for ~1024 workgroups but keep >= 256 K elements per split
static int pick_split(long tiles, long K, int requested) {
  if (requested > 0) return requested;
  long want = (1024 + tiles - 1) / tiles;
  long maxs = K / 256;
  if (maxs < 1) maxs = 1;
  if (want > maxs) want = maxs;
  if (want < 1) want = 1;
  if (want > 512) want = 512;
  return (int)want;
}

static void init_args(Args& a) {
  memset(&a, 0, sizeof(a));
  a.a.xf = CV_XF_NONE;
  a.b.xf = CV_XF_NONE;
  a.ep.stat_mode = CV_STAT_NONE;
  a.ep.stat_div = 1;
  a.a_pix = 1;
  a.o_pix = 1;
  a.ksplit = 1;
}

static int check_operand(const cv_operand* o, const char* what) {
  CV_REQUIRE(o != nullptr && o->x != nullptr, "%s: null operand", what);
  CV_REQUIRE(o->xf >= CV_XF_NONE && o->xf <= CV_XF_BNBWD, "%s: bad transform %d", what, o->xf);
  if (o->xf != CV_XF_NONE) {
    CV_REQUIRE(o->bn.C > 0 && o->bn.count > 0, "%s: BN constants missing", what);
    if (o->bn.train) CV_REQUIRE(o->bn.stat != nullptr, "%s: BN batch stats missing", what);
    else CV_REQUIRE(o->bn.running_mean && o->bn.running_var, "%s: BN running stats missing", what);
  }
  if (o->xf == CV_XF_BNBWD) {
    CV_REQUIRE(o->y != nullptr, "%s: BN backward needs the pre-BN tensor", what);
    if (o->bn.train) CV_REQUIRE(o->bn.gstat != nullptr, "%s: BN backward sums missing", what);
  }
  return 0;
}

static int apply_epilogue(Args& a, const cv_epilogue* ep, int ncols, const char* what) {
  if (!ep || ep->stat_mode == CV_STAT_NONE) return 0;
  a.ep = *ep;
  if (a.ep.stat_div <= 0) a.ep.stat_div = 1;
  CV_REQUIRE(ep->stat_out != nullptr, "%s: epilogue stats output missing", what);
  CV_REQUIRE(!a.accumulate, "%s: epilogue statistics need a non-split output", what);
  const int nf = (ncols + a.ep.stat_div - 1) / a.ep.stat_div;
  if (ep->stat_mode == CV_STAT_BWD) {
    CV_REQUIRE(ep->ey != nullptr && ep->ebn.C > 0, "%s: STAT_BWD needs the BN input", what);
    CV_REQUIRE(ep->ebn.C == nf, "%s: STAT_BWD feature count %d != %d", what, ep->ebn.C, nf);
    a.ce_n = ep->ebn.C;
  } else {
    a.ep.ebn.C = nf;
  }
  return 0;
}

static Geo geo_of(const cv_conv* g) {
  Geo o;
  o.n = g->n;
  o.kh = g->kh;
  o.kw = g->kw;
  o.s = g->stride;
  o.p = g->pad;
  if (!g->transposed) {  // small = output, big = input
    o.hs = g->h_out; o.ws = g->w_out; o.cs = g->c_out;
    o.hb = g->h_in;  o.wb = g->w_in;  o.cb = g->c_in;
  } else {               // small = input, big = output
    o.hs = g->h_in;  o.ws = g->w_in;  o.cs = g->c_in;
    o.hb = g->h_out; o.wb = g->w_out; o.cb = g->c_out;
  }
  return o;
}

static int check_conv(const cv_conv* g) {
  CV_REQUIRE(g && g->n > 0 && g->c_in > 0 && g->c_out > 0 && g->kh > 0 && g->kw > 0 && g->stride > 0 &&
                 g->pad >= 0,
             "conv: bad geometry");
  const cv_conv& c = *g;
  if (!c.transposed) {
    const int ho = (c.h_in + 2 * c.pad - c.kh) / c.stride + 1, wo = (c.w_in + 2 * c.pad - c.kw) / c.stride + 1;
    CV_REQUIRE(ho == c.h_out && wo == c.w_out, "conv: output %dx%d != expected %dx%d", c.h_out, c.w_out, ho, wo);
  } else {
    const int ho = (c.h_in - 1) * c.stride - 2 * c.pad + c.kh;  // + output_padding in [0, stride)
    const int wo = (c.w_in - 1) * c.stride - 2 * c.pad + c.kw;
    CV_REQUIRE(c.h_out >= ho && c.h_out < ho + c.stride && c.w_out >= wo && c.w_out < wo + c.stride,
               "convT: output %dx%d inconsistent with input %dx%d", c.h_out, c.w_out, c.h_in, c.w_in);
  }
  return 0;
}

// GATHER with small = rows.  `in` is the big-grid tensor.
static int run_gather(const Geo& g, const cv_operand* in, const float* w, const float* bias, float* out,
                      int accumulate, const cv_epilogue* ep, hipStream_t st, const char* what) {
  Args a;
  init_args(a);
  a.op = OP_GATHER;
  a.g = g;
  a.a = *in;
  a.ca_n = (in->xf != CV_XF_NONE) ? g.cb : 0;
  if (in->xf != CV_XF_NONE) CV_REQUIRE(in->bn.C == g.cb, "%s: BN width %d != channels %d", what, in->bn.C, g.cb);
  a.w = w;
  a.bias = bias;
  a.out = out;
  a.M = g.n * g.hs * g.ws;
  a.N = g.cs;
  a.K = g.kh * g.kw * g.cb;
  a.accumulate = accumulate;
  if (apply_epilogue(a, ep, a.N, what)) return 1;
  const int BM_ = (a.M >= 64 * 512) ? 128 : 64;
  const int BN_ = pick_bn(a.N);
  long tiles = (long)cdiv(a.M, BM_) * cdiv(a.N, BN_);
  int split = 1;
  if (accumulate) split = pick_split(tiles, a.K, 0);
  a.kchunk = ((cdiv(a.K, split) + BK - 1) / BK) * BK;
  split = cdiv(a.K, a.kchunk);
  a.ksplit = split;
  return launch(a, BM_, BN_, split, st);
}

// SCATTER with big = rows. `in` is the small-grid tensor.
static int run_scatter(const Geo& g, const cv_operand* in, const float* w, const float* bias, float* out,
                       const cv_epilogue* ep, hipStream_t st, const char* what) {
  Args a;
  init_args(a);
  a.op = OP_SCATTER;
  a.g = g;
  a.a = *in;
  a.ca_n = (in->xf != CV_XF_NONE) ? g.cs : 0;
  if (in->xf != CV_XF_NONE) CV_REQUIRE(in->bn.C == g.cs, "%s: BN width %d != channels %d", what, in->bn.C, g.cs);
  a.w = w;
  a.bias = bias;
  a.out = out;
  // largest class: ceil(hb/s) x ceil(wb/s)
  a.M = g.n * cdiv(g.hb, g.s) * cdiv(g.wb, g.s);
  a.N = g.cb;
  a.K = cdiv(g.kh, g.s) * cdiv(g.kw, g.s) * g.cs;
  if (apply_epilogue(a, ep, a.N, what)) return 1;
  // every big pixel must be written exactly once: classes with no taps write bias only -> the
  // kernel handles K == 0 by skipping the main loop.
  const int BM_ = (a.M >= 64 * 512) ? 128 : 64;
  const int BN_ = pick_bn(a.N);
  return launch(a, BM_, BN_, g.s * g.s, st);
}

static int run_wgrad(const Geo& g, const cv_operand* small, const cv_operand* big, float* gw, float* gbias,
                     int split_k, hipStream_t st) {
  Args a;
  init_args(a);
  a.op = OP_WGRAD;
  a.g = g;
  a.a = *small;
  a.b = *big;
  a.ca_n = (small->xf != CV_XF_NONE) ? g.cs : 0;
  a.cb_n = (big->xf != CV_XF_NONE) ? g.cb : 0;
  if (small->xf != CV_XF_NONE) CV_REQUIRE(small->bn.C == g.cs, "wgrad: small-grid BN width mismatch");
  if (big->xf != CV_XF_NONE) CV_REQUIRE(big->bn.C == g.cb, "wgrad: big-grid BN width mismatch");
  a.out = gw;
  a.gbias = gbias;
  a.M = g.cs;
  a.N = g.kh * g.kw * g.cb + (gbias ? 1 : 0);
  a.K = g.n * g.hs * g.ws;
  a.accumulate = 1;
  const int BM_ = (a.M >= 128) ? 128 : 64;
  const int BN_ = pick_bn(a.N);
  long tiles = (long)cdiv(a.M, BM_) * cdiv(a.N, BN_);
  int split = pick_split(tiles, a.K, split_k);
  a.kchunk = ((cdiv(a.K, split) + BK - 1) / BK) * BK;
  split = cdiv(a.K, a.kchunk);
  a.ksplit = split;
  return launch(a, BM_, BN_, split, st);
}

}  // namespace cv

using namespace cv;

extern "C" int cv_conv_forward(const cv_conv* g, const cv_operand* in, const float* weight, const float* bias,
                               float* out, const cv_epilogue* ep, cv_stream_t stream) {
  clear_error();
  if (check_conv(g) || check_operand(in, "conv_forward")) return 1;
  CV_REQUIRE(weight && out, "conv_forward: null weight/out");
  const Geo geo = geo_of(g);
  if (!g->transposed) return run_gather(geo, in, weight, bias, out, 0, ep, S(stream), "conv_forward");
  return run_scatter(geo, in, weight, bias, out, ep, S(stream), "convT_forward");
}

extern "C" int cv_conv_backward_data(const cv_conv* g, const cv_operand* gout, const float* weight, float* gin,
                                     const cv_epilogue* ep, cv_stream_t stream) {
  clear_error();
  if (check_conv(g) || check_operand(gout, "conv_backward_data")) return 1;
  CV_REQUIRE(weight && gin, "conv_backward_data: null weight/gin");
  const Geo geo = geo_of(g);
  if (!g->transposed) return run_scatter(geo, gout, weight, nullptr, gin, ep, S(stream), "conv_backward_data");
  return run_gather(geo, gout, weight, nullptr, gin, 0, ep, S(stream), "convT_backward_data");
}

extern "C" int cv_conv_backward_weight(const cv_conv* g, const cv_operand* in, const cv_operand* gout,
                                       float* gweight, float* gbias, int split_k, cv_stream_t stream) {
  clear_error();
  if (check_conv(g) || check_operand(in, "conv_backward_weight") || check_operand(gout, "conv_backward_weight"))
    return 1;
  CV_REQUIRE(gweight, "conv_backward_weight: null gweight");
  const Geo geo = geo_of(g);
  // conv: small = dY, big = X ; convT: small = X, big = dY
  CV_REQUIRE(!g->transposed || !gbias, "convT bias gradient is not a WGRAD column (use a reduction)");
  if (!g->transposed) return run_wgrad(geo, gout, in, gweight, gbias, split_k, S(stream));
  return run_wgrad(geo, in, gout, gweight, nullptr, split_k, S(stream));
}

// ---------------------------------------------------------------- linear layers
extern "C" int cv_linear_forward(const cv_linear* g, const cv_operand* in, const float* weight, const float* bias,
                                 float* out, int accumulate, const cv_epilogue* ep, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(g && g->n > 0 && g->in_features > 0 && g->out_features > 0, "linear_forward: bad geometry");
  if (check_operand(in, "linear_forward")) return 1;
  CV_REQUIRE(weight && out, "linear_forward: null weight/out");
  const int ip = g->in_pix > 0 ? g->in_pix : 1, op = g->out_pix > 0 ? g->out_pix : 1;
  CV_REQUIRE(ip == 1 || ip * g->in_ch == g->in_features, "linear_forward: in_pix*in_ch != in_features");
  CV_REQUIRE(op == 1 || op * g->out_ch == g->out_features, "linear_forward: out_pix*out_ch != out_features");
  Args a;
  init_args(a);
  a.op = OP_DENSE;
  a.a = *in;
  a.ca_n = 0;
  if (in->xf != CV_XF_NONE) {
    a.ca_n = in->bn.C;
    CV_REQUIRE(in->bn.C == g->in_features || (ip > 1 && in->bn.C == g->in_ch), "linear_forward: BN width mismatch");
  }
  a.w = weight;
  a.wlayout = 0;
  a.ldb = g->in_features;
  a.bias = bias;
  a.out = out;
  a.accumulate = accumulate;
  a.M = g->n;
  a.N = g->out_features;
  a.K = g->in_features;
  a.lda = g->in_features;
  a.a_pix = ip;
  a.a_ch = g->in_ch;
  a.ldo = g->out_features;
  a.o_pix = op;
  a.o_ch = g->out_ch;
  if (apply_epilogue(a, ep, a.N, "linear_forward")) return 1;
  const int BM_ = 64, BN_ = pick_bn(a.N);
  long tiles = (long)cdiv(a.M, BM_) * cdiv(a.N, BN_);
  int split = accumulate ? pick_split(tiles, a.K, 0) : 1;
  a.kchunk = ((cdiv(a.K, split) + BK - 1) / BK) * BK;
  split = cdiv(a.K, a.kchunk);
  return launch(a, BM_, BN_, split, S(stream));
}

extern "C" int cv_linear_backward_data(const cv_linear* g, const cv_operand* gout, const float* weight, float* gin,
                                       int accumulate, const cv_epilogue* ep, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(g && g->n > 0 && g->in_features > 0 && g->out_features > 0, "linear_backward_data: bad geometry");
  if (check_operand(gout, "linear_backward_data")) return 1;
  CV_REQUIRE(weight && gin, "linear_backward_data: null weight/gin");
  const int ip = g->in_pix > 0 ? g->in_pix : 1, op = g->out_pix > 0 ? g->out_pix : 1;
  // gin[n][perm_in(k)] = sum_o T(gout[n][perm_out(o)]) * W[o][k]
  Args a;
  init_args(a);
  a.op = OP_DENSE;
  a.a = *gout;
  a.ca_n = 0;
  if (gout->xf != CV_XF_NONE) {
    a.ca_n = gout->bn.C;
    CV_REQUIRE(gout->bn.C == g->out_features, "linear_backward_data: BN width must equal out_features");
  }
  a.w = weight;
  a.wlayout = 1;
  a.ldb = g->in_features;
  a.out = gin;
  a.accumulate = accumulate;
  a.M = g->n;
  a.N = g->in_features;
  a.K = g->out_features;
  a.lda = g->out_features;
  a.a_pix = op;
  a.a_ch = g->out_ch;
  a.ldo = g->in_features;
  a.o_pix = ip;
  a.o_ch = g->in_ch;
  if (apply_epilogue(a, ep, a.N, "linear_backward_data")) return 1;
  const int BM_ = 64, BN_ = pick_bn(a.N);
  long tiles = (long)cdiv(a.M, BM_) * cdiv(a.N, BN_);
  int split = accumulate ? pick_split(tiles, a.K, 0) : 1;
  a.kchunk = ((cdiv(a.K, split) + BK - 1) / BK) * BK;
  split = cdiv(a.K, a.kchunk);
  return launch(a, BM_, BN_, split, S(stream));
}

extern "C" int cv_linear_backward_weight(const cv_linear* g, const cv_operand* gout, const cv_operand* in,
                                         float* gweight, float* gbias, int split_k, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(g && g->n > 0, "linear_backward_weight: bad geometry");
  if (check_operand(gout, "linear_backward_weight") || check_operand(in, "linear_backward_weight")) return 1;
  const int ip = g->in_pix > 0 ? g->in_pix : 1;
  CV_REQUIRE(g->out_pix <= 1, "linear_backward_weight: permuted outputs unsupported (use cv_declinear_*)");
  CV_REQUIRE(gout->xf == CV_XF_NONE, "linear_backward_weight: transform on gout unsupported");
  // Expressed as a WGRAD over a 1x1 "small grid" (rows = batch) and an in_pix "big grid":
  //   dW[o][c][pix] = sum_n gout[n][o] * T(in[n][pix][c])   (== Linear weight [o][c*pix + p])
  Geo geo;
  geo.n = g->n;
  geo.hs = 1; geo.ws = 1; geo.cs = g->out_features;
  if (ip > 1) {
    int side = 1;
    while (side * side < ip) ++side;
    CV_REQUIRE(side * side == ip, "linear_backward_weight: in_pix must be a square image");
    geo.hb = side; geo.wb = side; geo.cb = g->in_ch; geo.kh = side; geo.kw = side;
  } else {
    geo.hb = 1; geo.wb = 1; geo.cb = g->in_features; geo.kh = 1; geo.kw = 1;
  }
  geo.s = 1;
  geo.p = 0;
  return run_wgrad(geo, gout, in, gweight, gbias, split_k, S(stream));
}
