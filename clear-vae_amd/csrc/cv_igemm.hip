// Implicit-GEMM convolution / linear kernels on fp32 MFMA (v_mfma_f32_16x16x4_f32) for gfx950.
//
// One templated main loop serves every dense contraction of the CLEAR-VAE step:
//   GATHER  : out[small pixel][cs]  = sum_{tap,cb} T(big[pixel*s-p+tap][cb]) * w(cs,cb,tap)
//             (Conv2d forward, ConvTranspose2d backward-data)
//   SCATTER : out[big pixel][cb]    = sum_{tap,cs} T(small[(pixel+p-tap)/s][cs]) * w(cs,cb,tap)
//             (Conv2d backward-data, ConvTranspose2d forward), decomposed into stride^2 parity classes
//             so every class is a dense GEMM with no masked taps
//   WGRAD   : dw(cs,cb,tap)        += sum_{small pixel} T(small[pixel][cs]) * T(big[gather][cb])
//             (grad_weight of every conv / convT / linear), split-K over pixels, fp32 atomics
//   DENSE   : out[row][col]         = sum_k T(A[row][perm(k)]) * W(k,col)   (Linear layers)
// T() is the fused BatchNorm(+ReLU) forward or backward transform (cv_common.hpp); BN batch
// statistics of the produced tensor are reduced in the epilogue (fp64 atomics, 8 replicas).
//
// Reference arithmetic replaced: nn.Conv2d / nn.ConvTranspose2d / nn.Linear / nn.BatchNorm2d / ReLU
// of code/src/models/vae.py:15-46 (VAE) and :113-156 (VAE64), forward and autograd backward.
//
// Tile: BM x BN x 32, 256 threads = 4 waves laid out WM x WN; each wave owns (BM/WM) x (BN/WN)
// as 16x16 MFMA tiles.  Operands go global -> registers -> LDS (k-major, padded so the ds_read_b32
// fragment reads are bank-conflict free); LDS is double-buffered, so a K tile costs one barrier,
// and the next tile's global loads are in flight during the current tile's MFMAs.  Conv weights
// are pre-packed once per step (cv_pack_conv_weights) into GEMM-native [K][N] rows, so the B
// operand is a coalesced float4 stream with no index arithmetic; activation gathers are float4
// along channels with all integer division hoisted to once per row (rows) or once per K tile.
#include "cv_igemm.hpp"

namespace cv {

// ------------------------------------------------------------------ the kernel
// Operand staging: global -> registers (raw values, a validity mask) -> [after the MFMAs of the
// current tile] BatchNorm transform -> LDS.  Deferring the transform to the store keeps the next
// tile's loads in flight across the current tile's MFMAs (a transform at load time would wait for
// them immediately).
//
// LDS images:
//   row-oriented A (GATHER/SCATTER/DENSE): [BK/4 quads][BM rows][4 k] -- the ds_write_b128 of a
//     (row, quad) staging float4 is contiguous, and the 64 lanes of an MFMA A-fragment read
//     (16 rows x 4 k) are 64 consecutive floats (bank-conflict free);
//   WGRAD A: [BK][BM + 16] k-major (staged as float4 along M);
//   B: [BK][BN (+16)] k-major.
template <int OP, int BM, int BN>
__global__ __launch_bounds__(NT) void igemm_kernel(const Args P) {
  constexpr int WN = (BN >= 32) ? 2 : 1;
  constexpr int WM = 4 / WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  static_assert(FM >= 1 && FN >= 1, "tile too small");
  constexpr bool ROWS = OP != OP_WGRAD;
  constexpr int LDA = ROWS ? BM : BM + 16;
  constexpr int LDB = BN + ((BN % 32) == 0 ? 16 : 0);
  constexpr int RA = BM / 32;                               // A rows per thread (row-oriented)
  constexpr int AW = (BM * BK / 4 + NT - 1) / NT;           // WGRAD A float4 per thread
  constexpr int BW = (BN * BK / 4 + NT - 1) / NT;           // B float4 per thread
  constexpr int RAW = ROWS ? RA : AW;
  constexpr int ABUF = BK * LDA + (ROWS ? 0 : 0), BBUF = BK * LDB;

  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* As = smem;                     // [2][ABUF]
  float* Bs = As + 2 * ABUF;            // [2][BBUF]
  float* red = Bs + 2 * BBUF;           // epilogue reduction scratch: 2 * WM * BN floats
  float* cstA = red + 2 * WM * BN;      // BN constants
  // DENSE with a BatchNorm1d over the K features (decoder Linear backward): constants only for this
  // block's K chunk, indexed k - kbeg (folding all K features per block was 65k fp64 loads each)
  const bool bn1d = (OP == OP_DENSE) && P.ca_n == P.K && P.a.xf != CV_XF_NONE;
  float* cstB = cstA + xf_floats(P.a.xf, bn1d ? P.kchunk : P.ca_n);
  float* cstE = cstB + xf_floats(P.b.xf, P.cb_n);

  CV_STAMP(st0);
#ifdef CV_STAMPS
  const unsigned long long mt0 = __builtin_amdgcn_s_memtime();
#endif
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const Geo& g = P.g;

  // ---------------- block -> (m0, n0, k-range, class)
  // WGRAD: XCD-aware order.  Hardware workgroup b runs on XCD b % 8; the bijection below hands each
  // XCD a contiguous range of logical ids enumerated N-tile fastest, then M-tile, then split, so the
  // blocks that read one split's K range (the same dY / X rows) share one XCD's L2 (PMC: 4.9x less
  // memory-side fetch on conv3's weight gradient).  The row-oriented ops keep the hardware order:
  // their parity classes / M tiles differ in cost and round-robin spreads them over all XCDs.
  const int gx = gridDim.x, gy = gridDim.y;
  const int nwg = gx * gy * gridDim.z;
  const int hw_id = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (OP == OP_WGRAD) {
    const int xcd = hw_id & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (hw_id >> 3);
    by = lid % gy;
    bx = (lid / gy) % gx;
    bz = lid / (gx * gy);
  }
  const int m0 = bx * BM, n0 = by * BN;
  int M = P.M, K = P.K;
  const int N = P.N + ((OP == OP_WGRAD && P.gbias) ? 1 : 0);
  int kbeg = 0, kend = K;
  int ry = 0, rx = 0, yb0 = 0, xb0 = 0, cy = 1, cx = 1, ntx = 1;
  FDiv f_cx = FDiv::make(1), f_cycx = FDiv::make(1), f_ntx = FDiv::make(1);
  if (OP == OP_SCATTER) {
    const int s = g.s, cls = bz;
    ry = cls / s;
    rx = cls % s;
    yb0 = (((ry - g.p) % s) + s) % s;  // big rows with (yb + p) % s == ry
    xb0 = (((rx - g.p) % s) + s) % s;
    cy = (g.hb > yb0) ? (g.hb - yb0 + s - 1) / s : 0;
    cx = (g.wb > xb0) ? (g.wb - xb0 + s - 1) / s : 0;
    const int nty = (g.kh > ry) ? (g.kh - ry + s - 1) / s : 0;
    ntx = (g.kw > rx) ? (g.kw - rx + s - 1) / s : 0;
    M = g.n * cy * cx;
    K = nty * ntx * g.cs;
    kend = K;
    if (m0 >= M) return;
    f_cx = FDiv::make(cx);
    f_cycx = FDiv::make(cy * cx);
    f_ntx = FDiv::make(ntx);
  } else {
    kbeg = bz * P.kchunk;
    kend = min(K, kbeg + P.kchunk);
    if (kbeg >= kend) return;
  }

  // ---------------- prologue: BN constants into LDS (the A buffers serve as the fold's scratch)
  double* fold_scratch = reinterpret_cast<double*>(As);
  static_assert(2 * BK * (ROWS ? BM : BM + 16) * sizeof(float) >= 4 * NT * sizeof(double), "fold scratch");
  XfA ca, cb;
  if (bn1d) {
    ca.f = reinterpret_cast<const BnFwdC*>(cstA);
    ca.bw = reinterpret_cast<const BnBwdC*>(cstA);
    for (int idx = t; idx < kend - kbeg; idx += NT) {
      int f = kbeg + idx;
      if (P.a_pix > 1) {
        const int pix = f / P.a_ch, c = f - pix * P.a_ch;
        f = c * P.a_pix + pix;
      }
      if (P.a.xf == CV_XF_BNRELU) reinterpret_cast<BnFwdC*>(cstA)[idx] = bn_fwd_const(P.a.bn, f);
      else reinterpret_cast<BnBwdC*>(cstA)[idx] = bn_bwd_const(P.a.bn, f);
    }
  } else {
    fill_consts(P.a, P.ca_n, cstA, fold_scratch, ca);
  }
  fill_consts(P.b, P.cb_n, cstB, fold_scratch, cb);
  if (P.ep.stat_mode == CV_STAT_BWD) {
    BnFwdC* d = reinterpret_cast<BnFwdC*>(cstE);
    bn_fold<NT>(P.ep.ebn, false, fold_scratch, [&](int f, double s, double q, double, double) {
      if (f < P.ce_n) d[f] = bn_fwd_const_s(P.ep.ebn, f, s, q);
    });
  }

  // ---------------- per-thread A-row decode (row-oriented): rows (t&15)+16*(t>>7)+32*i, quad (t>>4)&7
  const int quad = (t >> 4) & 7;
  int r_n[RA], r_y[RA], r_x[RA];
  bool r_ok[RA];
  if (ROWS) {
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const int r = m0 + (t & 15) + 16 * (t >> 7) + 32 * i;
      r_ok[i] = r < M;
      const int rr = r_ok[i] ? r : 0;
      if (OP == OP_GATHER) {
        const int hw = g.hs * g.ws;
        r_n[i] = P.f_hws.div(rr);
        const int rem = rr - r_n[i] * hw;
        const int ys = P.f_ws.div(rem), xs = rem - ys * g.ws;
        r_y[i] = ys * g.s - g.p;  // big-grid origin of the receptive field
        r_x[i] = xs * g.s - g.p;
      } else if (OP == OP_SCATTER) {
        const int hw = cy * cx;
        r_n[i] = f_cycx.div(rr);
        const int rem = rr - r_n[i] * hw;
        const int ty = f_cx.div(rem), tx = rem - ty * cx;
        r_y[i] = yb0 + g.s * ty + g.p;  // (yb + p); ys = (r_y - kh) / s
        r_x[i] = xb0 + g.s * tx + g.p;
      } else {
        r_n[i] = rr;
        r_y[i] = 0;
        r_x[i] = 0;
      }
    }
  }
  __syncthreads();

  // launch-uniform choice between the vectorised (deferred-transform) and scalar operand paths
  const bool a_vec = (OP == OP_GATHER) ? ((g.cb & 3) == 0 && !P.a.nchw)
                   : (OP == OP_SCATTER) ? ((g.cs & 3) == 0)
                   : (OP == OP_DENSE) ? ((P.lda & 3) == 0 && (P.K & 3) == 0 && (P.a_pix == 1 || (P.a_ch & 3) == 0))
                   : ((g.cs & 3) == 0);
  const bool b_vec = (OP == OP_WGRAD) && (g.cb & 3) == 0 && !P.b.nchw;
  const bool a_bwd = P.a.xf == CV_XF_BNBWD, b_bwd = P.b.xf == CV_XF_BNBWD;

  // one register stage of a K tile (raw operand values, BN-backward partners, validity masks)
  struct Stage {
    float4 ra[RAW], rya[RAW];
    float4 rb[BW], ryb[BW];
    unsigned amask, bmask;
  };

  // DENSE: the K loop runs in the storage order of A (k' = pix*a_ch + c for an NCHW-flattened
  // input); lf() is the PyTorch feature index of k' (weight column / BN1d feature)
  auto lf = [&](int kk) -> int {
    if (P.a_pix <= 1) return kk;
    const int pix = P.f_ach.div(kk), c = kk - pix * P.a_ch;
    return c * P.a_pix + pix;
  };

  // ---------------- A: fetch raw values into registers
  auto fetchA = [&](Stage& S, int k0) {
    S.amask = 0;
    if (ROWS) {
      const int kq = k0 + 4 * quad;
      if (a_vec) {
        if (OP == OP_GATHER) {
          const int tap = P.f_cb.div(kq), c0 = kq - tap * g.cb;
          const int kh = P.f_kw.div(tap), kw = tap - kh * g.kw;
#pragma unroll
          for (int i = 0; i < RA; ++i) {
            const int yb = r_y[i] + kh, xb = r_x[i] + kw;
            S.ra[i] = z4();
            S.rya[i] = z4();
            if (r_ok[i] && kq < kend && (unsigned)yb < (unsigned)g.hb && (unsigned)xb < (unsigned)g.wb) {
              const size_t off = ((size_t)(r_n[i] * g.hb + yb) * g.wb + xb) * g.cb + c0;
              S.ra[i] = ld4(P.a.x + off);
              if (a_bwd) S.rya[i] = ld4(P.a.y + off);
              S.amask |= 1u << i;
            }
          }
        } else if (OP == OP_SCATTER) {
          const int tap = P.f_cs.div(kq), c0 = kq - tap * g.cs;
          const int jy = f_ntx.div(tap), jx = tap - jy * ntx;
          const int kh = ry + g.s * jy, kw = rx + g.s * jx;
#pragma unroll
          for (int i = 0; i < RA; ++i) {
            const int py = r_y[i] - kh, px = r_x[i] - kw;  // divisible by s by construction
            S.ra[i] = z4();
            S.rya[i] = z4();
            if (r_ok[i] && kq < kend && py >= 0 && px >= 0) {
              const int ys = P.f_s.div(py), xs = P.f_s.div(px);
              if (ys < g.hs && xs < g.ws) {
                const size_t off = ((size_t)(r_n[i] * g.hs + ys) * g.ws + xs) * g.cs + c0;
                S.ra[i] = ld4(P.a.x + off);
                if (a_bwd) S.rya[i] = ld4(P.a.y + off);
                S.amask |= 1u << i;
              }
            }
          }
        } else {  // DENSE, storage-order k'
#pragma unroll
          for (int i = 0; i < RA; ++i) {
            S.ra[i] = z4();
            S.rya[i] = z4();
            if (r_ok[i] && kq < kend) {
              const size_t off = (size_t)r_n[i] * P.lda + kq;
              S.ra[i] = ld4(P.a.x + off);
              if (a_bwd) S.rya[i] = ld4(P.a.y + off);
              S.amask |= 1u << i;
            }
          }
        }
      } else {  // scalar path (transform applied here)
#pragma unroll
        for (int i = 0; i < RA; ++i) {
          float tmp[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            tmp[j] = 0.f;
            const int k = kq + j;
            if (!r_ok[i] || k >= kend) continue;
            size_t off;
            int ch;
            bool ok = true;
            if (OP == OP_GATHER) {
              const int tap = P.f_cb.div(k), c = k - tap * g.cb;
              const int kh = P.f_kw.div(tap), kw = tap - kh * g.kw;
              const int yb = r_y[i] + kh, xb = r_x[i] + kw;
              ok = (unsigned)yb < (unsigned)g.hb && (unsigned)xb < (unsigned)g.wb;
              off = P.a.nchw ? ((size_t)(r_n[i] * g.cb + c) * g.hb + yb) * g.wb + xb
                             : ((size_t)(r_n[i] * g.hb + yb) * g.wb + xb) * g.cb + c;
              ch = c;
            } else if (OP == OP_SCATTER) {
              const int tap = P.f_cs.div(k), c = k - tap * g.cs;
              const int jy = f_ntx.div(tap), jx = tap - jy * ntx;
              const int py = r_y[i] - (ry + g.s * jy), px = r_x[i] - (rx + g.s * jx);
              ok = py >= 0 && px >= 0 && P.f_s.div(py) < g.hs && P.f_s.div(px) < g.ws;
              off = ((size_t)(r_n[i] * g.hs + (ok ? P.f_s.div(py) : 0)) * g.ws + (ok ? P.f_s.div(px) : 0)) * g.cs + c;
              ch = c;
            } else {
              off = (size_t)r_n[i] * P.lda + k;
              const int f = lf(k);
              ch = bn1d ? k - kbeg : (P.a_pix > 1 ? P.f_ach.mod(k) : f);
            }
            if (ok) {
              const float yv = a_bwd ? P.a.y[off] : 0.f;
              tmp[j] = xf_apply(P.a, ca, ch, P.a.x[off], yv);
            }
          }
          S.ra[i] = make_float4(tmp[0], tmp[1], tmp[2], tmp[3]);
        }
      }
    } else {  // WGRAD A(m = cs, k = small pixel): float4 along cs
      constexpr int MQ = BM / 4;
#pragma unroll
      for (int e = 0; e < AW; ++e) {
        const int idx = t + NT * e;
        const int mq = idx % MQ, kk = idx / MQ;
        const int pix = k0 + kk, c0 = m0 + 4 * mq;
        S.ra[e] = z4();
        S.rya[e] = z4();
        if (kk < BK && pix < kend) {
          const size_t off = (size_t)pix * g.cs + c0;
          if (a_vec) {
            if (c0 < g.cs) {
              S.ra[e] = ld4(P.a.x + off);
              if (a_bwd) S.rya[e] = ld4(P.a.y + off);
              S.amask |= 1u << e;
            }
          } else {
            float tmp[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              tmp[j] = 0.f;
              if (c0 + j < g.cs) {
                const float yv = a_bwd ? P.a.y[off + j] : 0.f;
                tmp[j] = xf_apply(P.a, ca, c0 + j, P.a.x[off + j], yv);
              }
            }
            S.ra[e] = make_float4(tmp[0], tmp[1], tmp[2], tmp[3]);
          }
        }
      }
    }
  };

  // ---------------- A: transform (vector paths) + store to LDS
  auto storeA = [&](Stage& S, float* Ab, int k0) {
    if (ROWS) {
      const int kq = k0 + 4 * quad;
      int ch0 = 0;
      if (a_vec && P.a.xf != CV_XF_NONE) {
        if (OP == OP_GATHER) ch0 = P.f_cb.mod(kq);
        else if (OP == OP_SCATTER) ch0 = P.f_cs.mod(kq);
        else ch0 = (P.a_pix > 1) ? P.f_ach.mod(kq) : kq;
      }
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        float4 v = S.ra[i];
        if (a_vec && P.a.xf != CV_XF_NONE) {
          if (S.amask & (1u << i)) {
            if (bn1d) {  // BN1d: constants of this block's K chunk, in k order
              v = xf_apply4(P.a, ca, kq - kbeg, v, S.rya[i]);
            } else {
              v = xf_apply4(P.a, ca, ch0, v, S.rya[i]);
            }
          }
        }
        const int m = (t & 15) + 16 * (t >> 7) + 32 * i;
        *reinterpret_cast<float4*>(Ab + (quad * BM + m) * 4) = v;
      }
    } else {
      constexpr int MQ = BM / 4;
#pragma unroll
      for (int e = 0; e < AW; ++e) {
        const int idx = t + NT * e;
        const int mq = idx % MQ, kk = idx / MQ;
        float4 v = S.ra[e];
        if (a_vec && P.a.xf != CV_XF_NONE && (S.amask & (1u << e))) v = xf_apply4(P.a, ca, m0 + 4 * mq, v, S.rya[e]);
        if (kk < BK) *reinterpret_cast<float4*>(Ab + kk * LDA + 4 * mq) = v;
      }
    }
  };

  // ---------------- B: one float4 of a K row (4 consecutive columns) per slot
  constexpr int NQ = BN / 4;
  auto fetchB = [&](Stage& S, int k0) {
    S.bmask = 0;
#pragma unroll
    for (int e = 0; e < BW; ++e) {
      const int idx = t + NT * e;
      const int nq = idx % NQ, kk = idx / NQ;
      const int col = n0 + 4 * nq, k = k0 + kk;
      float4 v = z4();
      S.ryb[e] = z4();
      if (kk < BK && k < kend && col < N) {
        if (OP == OP_GATHER) {  // packed [K = tap*cb][cs]
          if (col + 3 < N && (g.cs & 3) == 0) {
            v = ld4(P.w + (size_t)k * g.cs + col);
          } else {
            float tmp[4] = {0.f, 0.f, 0.f, 0.f};
            for (int j = 0; j < 4 && col + j < N; ++j) tmp[j] = P.w[(size_t)k * g.cs + col + j];
            v = make_float4(tmp[0], tmp[1], tmp[2], tmp[3]);
          }
        } else if (OP == OP_SCATTER) {  // packed [tap][cs][cb]; class taps
          const int tap = P.f_cs.div(k), c = k - tap * g.cs;
          const int jy = f_ntx.div(tap), jx = tap - jy * ntx;
          const int kh = ry + g.s * jy, kw = rx + g.s * jx;
          const size_t rowo = ((size_t)(kh * g.kw + kw) * g.cs + c) * g.cb;
          if (col + 3 < N && (g.cb & 3) == 0) {
            v = ld4(P.w + rowo + col);
          } else {
            float tmp[4] = {0.f, 0.f, 0.f, 0.f};
            for (int j = 0; j < 4 && col + j < N; ++j) tmp[j] = P.w[rowo + col + j];
            v = make_float4(tmp[0], tmp[1], tmp[2], tmp[3]);
          }
        } else if (OP == OP_DENSE) {
          const int kl = lf(k);
          float tmp[4] = {0.f, 0.f, 0.f, 0.f};
          if (P.wlayout) {
            if (col + 3 < N && (P.ldb & 3) == 0) {
              v = ld4(P.w + (size_t)kl * P.ldb + col);
              tmp[0] = v.x; tmp[1] = v.y; tmp[2] = v.z; tmp[3] = v.w;
            } else {
              for (int j = 0; j < 4 && col + j < N; ++j) tmp[j] = P.w[(size_t)kl * P.ldb + col + j];
            }
          } else {
            for (int j = 0; j < 4 && col + j < N; ++j) tmp[j] = P.w[(size_t)(col + j) * P.ldb + kl];
          }
          v = make_float4(tmp[0], tmp[1], tmp[2], tmp[3]);
        } else {  // WGRAD: B(k = small pixel, col = (tap, cb)) = T(big[gather(pix, tap)][cb])
          const int hw = g.hs * g.ws;
          const int nimg = P.f_hws.div(k), rem = k - nimg * hw;
          const int ys = P.f_ws.div(rem), xs = rem - ys * g.ws;
          const int nreal = P.N;
          if (col >= nreal) {  // bias column (nreal % 4 == 0 when gbias is used)
            v = make_float4(col == nreal ? 1.f : 0.f, 0.f, 0.f, 0.f);
          } else if (b_vec) {
            const int tap = P.f_cb.div(col), c0 = col - tap * g.cb;
            const int kh = P.f_kw.div(tap), kw = tap - kh * g.kw;
            const int yb = ys * g.s - g.p + kh, xb = xs * g.s - g.p + kw;
            if ((unsigned)yb < (unsigned)g.hb && (unsigned)xb < (unsigned)g.wb) {
              const size_t off = ((size_t)(nimg * g.hb + yb) * g.wb + xb) * g.cb + c0;
              v = ld4(P.b.x + off);
              if (b_bwd) S.ryb[e] = ld4(P.b.y + off);
              S.bmask |= 1u << e;
            }
          } else {
            float tmp[4] = {0.f, 0.f, 0.f, 0.f};
            for (int j = 0; j < 4 && col + j < nreal; ++j) {
              const int cc = col + j;
              const int tap = P.f_cb.div(cc), c = cc - tap * g.cb;
              const int kh = P.f_kw.div(tap), kw = tap - kh * g.kw;
              const int yb = ys * g.s - g.p + kh, xb = xs * g.s - g.p + kw;
              if ((unsigned)yb < (unsigned)g.hb && (unsigned)xb < (unsigned)g.wb) {
                const size_t off = P.b.nchw ? ((size_t)(nimg * g.cb + c) * g.hb + yb) * g.wb + xb
                                            : ((size_t)(nimg * g.hb + yb) * g.wb + xb) * g.cb + c;
                const float yv = b_bwd ? P.b.y[off] : 0.f;
                tmp[j] = xf_apply(P.b, cb, c, P.b.x[off], yv);
              }
            }
            if (P.gbias && col + 3 >= nreal) {
              for (int j = 0; j < 4; ++j)
                if (col + j == nreal) tmp[j] = 1.f;
            }
            v = make_float4(tmp[0], tmp[1], tmp[2], tmp[3]);
          }
        }
      }
      S.rb[e] = v;
    }
  };

  auto storeB = [&](Stage& S, float* Bb) {
#pragma unroll
    for (int e = 0; e < BW; ++e) {
      const int idx = t + NT * e;
      const int nq = idx % NQ, kk = idx / NQ;
      float4 v = S.rb[e];
      if (OP == OP_WGRAD && b_vec && P.b.xf != CV_XF_NONE && (S.bmask & (1u << e))) {
        const int col = n0 + 4 * nq;
        v = xf_apply4(P.b, cb, P.f_cb.mod(col), v, S.ryb[e]);
      }
      if (kk < BK) *reinterpret_cast<float4*>(Bb + kk * LDB + 4 * nq) = v;
    }
  };

  // ---------------- main loop (double-buffered LDS, one barrier per K tile)
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // CV_DEPTH-deep register ring: tile t is staged in slot t % D; at step t the loads of tile t+D-1
  // are issued, tile t is multiplied from LDS, then tile t+1 (loaded D-2 steps earlier) is
  // transformed and stored to the other LDS buffer -- so D-1 tiles of loads are in flight across
  // every MFMA phase.
  constexpr int D = CV_DEPTH;
  Stage stg[D];
  const int nt = (kend - kbeg + BK - 1) / BK;
#pragma unroll
  for (int d = 0; d < D - 1; ++d) {
    if (d < nt) {
      fetchA(stg[d], kbeg + d * BK);
      fetchB(stg[d], kbeg + d * BK);
    }
  }
  storeA(stg[0], As, kbeg);
  storeB(stg[0], Bs);
  __syncthreads();
  CV_STAMP(st1);
  for (int tb = 0; tb < nt; tb += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int tt = tb + d;
      if (tt >= nt) break;
      if (tt + D - 1 < nt) {
        fetchA(stg[(d + D - 1) % D], kbeg + (tt + D - 1) * BK);
        fetchB(stg[(d + D - 1) % D], kbeg + (tt + D - 1) * BK);
      }
      const float* Ab = As + (tt & 1) * ABUF;
      const float* Bb = Bs + (tt & 1) * BBUF;
#pragma unroll
      for (int kk = 0; kk < BK; kk += 4) {
        const int kr = kk + (lane >> 4);
        float av[FM], bv[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int m = wm * TM + i * 16 + (lane & 15);
          av[i] = ROWS ? Ab[((kk >> 2) * BM + m) * 4 + (lane >> 4)] : Ab[kr * LDA + m];
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) bv[j] = Bb[kr * LDB + wn * TN + j * 16 + (lane & 15)];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
      if (tt + 1 < nt) {
        storeA(stg[(d + 1) % D], As + ((tt + 1) & 1) * ABUF, kbeg + (tt + 1) * BK);
        storeB(stg[(d + 1) % D], Bs + ((tt + 1) & 1) * BBUF);
      }
      __syncthreads();
    }
  }

  CV_STAMP(st2);
  // ---------------- epilogue
  const bool stats = P.ep.stat_mode != CV_STAT_NONE;
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
        if (OP == OP_WGRAD) {
          if (P.part) {  // plain store of this split's partial tile; wgrad_reduce_kernel sums them
            P.part[((size_t)bz * M + row) * N + col] = v;
            continue;
          }
          const int tap = P.f_cb.div(col), c = col - tap * g.cb;  // w layout [cs][cb][kh][kw]
          float* dst = (col >= P.N) ? P.gbias + row : P.out + ((size_t)row * g.cb + c) * (g.kh * g.kw) + tap;
          if (gridDim.z == 1) *dst += v;  // single writer
          else atomicAdd(dst, v);
          continue;
        }
        size_t off;
        if (OP == OP_GATHER) {
          off = (size_t)row * g.cs + col;
        } else if (OP == OP_SCATTER) {
          const int hw = cy * cx;
          const int nimg = f_cycx.div(row), rem = row - nimg * hw;
          const int ty = f_cx.div(rem), tx = rem - ty * cx;
          const int yb = yb0 + g.s * ty, xb = xb0 + g.s * tx;
          off = ((size_t)(nimg * g.hb + yb) * g.wb + xb) * g.cb + col;
        } else {
          const int oc = (P.o_pix > 1) ? P.f_opix.mod(col) * P.o_ch + P.f_opix.div(col) : col;
          off = (size_t)row * P.ldo + oc;
        }
        if (P.bias && (!P.accumulate || bz == 0)) v += P.bias[col];
        if (P.accumulate) {
          atomicAdd(P.out + off, v);
          continue;
        }
        if (P.ep.stat_mode == CV_STAT_BWD) {
          const int f = P.f_sdiv.div(col);
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

  if (OP != OP_WGRAD && stats && !P.accumulate) {
    // reduce per column: lanes with equal (lane & 15), then the WM waves sharing wn
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      s1[j] += __shfl_xor(s1[j], 16, 64);
      s1[j] += __shfl_xor(s1[j], 32, 64);
      s2[j] += __shfl_xor(s2[j], 16, 64);
      s2[j] += __shfl_xor(s2[j], 32, 64);
    }
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int c = wn * TN + j * 16 + lane;
        red[wm * BN + c] = s1[j];
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
        const int f = P.f_sdiv.div(col);
        const int C = (P.ep.stat_mode == CV_STAT_BWD) ? P.ce_n : P.ep.ebn.C;
        const int repl = hw_id % CV_STAT_REPL(C);
        double* so = P.ep.stat_out + (size_t)repl * 2 * C;
        atomic_add_f64(so + f, a);
        atomic_add_f64(so + C + f, b);
      }
    }
  }
#ifdef CV_STAMPS
  if (t == 0 && g_stamps) {
    const unsigned long long st3 = __builtin_amdgcn_s_memrealtime(), mt1 = __builtin_amdgcn_s_memtime();
    unsigned long long* o = g_stamps + (size_t)hw_id * 8;
    o[0] = st0; o[1] = st1; o[2] = st2; o[3] = st3; o[4] = mt0; o[5] = mt1;
    o[6] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
    o[7] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11));
  }
#endif
}

// ------------------------------------------------------------------ weight packing
// Wg[tap][cb][cs] (GATHER) and Ws[tap][cs][cb] (SCATTER) from w(cs, cb, tap) = W[cs][cb][kh][kw]
constexpr int MAX_PACK = 16;
struct PackArgs {
  const float* src[MAX_PACK];
  float* dg[MAX_PACK];
  float* ds[MAX_PACK];
  int cs[MAX_PACK], cb[MAX_PACK], kk[MAX_PACK];
  int n;
  // the step's zeroed buffers (cv_pack_conv_weights_zero): the blockIdx.y == n slice clears them
  uint32_t* zp[8];
  long zstart[9];  // prefix sums of 4-byte words (zvec: of 16-byte units)
  int zn;
  int zvec;        // every zeroed buffer 16-byte aligned and sized: 16-byte stores
  // copies done by the same slice (cv_pack_conv_weights_zero_copy: the step's input batch), 16-byte units
  uint4* cd[4];
  const uint4* csrc[4];
  long cstart[5];
  int cn;
  // flat 1-D grid: workgroups [wg0[l], wg0[l + 1]) pack layer l, the workgroups from wg0[n] on zero / copy
  int wg0[MAX_PACK + 1];
  // Adam fused in (cv_adam_pack_step; ad == 0: off): the packing workgroups update their tile's parameters (p, m,
  // v at the arena offset of src) before packing the new values; the slice workgroups update the arena ranges no
  // item covers (plain); the last workgroup to finish advances the step counters
  int ad;
  float* ap;
  const float* ag;
  float* am;
  float* av;
  const float* hyper;
  int64_t* step;
  const float* gscale;
  int64_t* aux;
  long plain0[2 * MAX_PACK + 2];
  long plainn[2 * MAX_PACK + 2];
  int nplain;
  int hold;  // 1: the last workgroup leaves step[0] / aux as they are (a first part of a split update)
};

// Adam constants of the step (the arithmetic of adam_kernel, cv_mi.hip); computed by thread 0 into sh[8]
__device__ __forceinline__ void adam_consts(const PackArgs& a, float* sh) {
  if (threadIdx.x == 0) {
    const long t_step = a.step[0] + 1;
    const double b1 = a.hyper[1], b2 = a.hyper[2];
    const double bc1 = 1.0 - pow(b1, (double)t_step);
    const double bc2 = 1.0 - pow(b2, (double)t_step);
    sh[0] = (float)(-(double)a.hyper[0] / bc1);
    sh[1] = (float)sqrt(bc2);
    sh[2] = (float)(1.0 - b1);
    sh[3] = (float)(1.0 - b2);
    sh[4] = a.hyper[2];
    sh[5] = a.hyper[3];
    sh[6] = a.hyper[4];
    sh[7] = a.gscale ? a.gscale[0] : 1.0f;
  }
}
// torch.optim.Adam on one element (adam_kernel's upd): returns the new parameter, updates mm / vv
__device__ __forceinline__ float adam_upd(const float* c, float g, float pp, float& mm, float& vv) {
  g *= c[7];
  if (c[6] != 0.f) g = g + c[6] * pp;
  mm = mm + c[2] * (g - mm);
  vv = vv * c[4] + c[3] * g * g;
  const float den = sqrtf(vv) / c[1] + c[5];
  return pp + c[0] * (mm / den);
}
// the step counters: every workgroup of an Adam launch arrives once; the last advances step[0] (and aux)
__device__ __forceinline__ void adam_arrive(const PackArgs& a, int* flag) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long prev = atomicAdd((unsigned long long*)(a.step + 1), 1ull);
    *flag = prev == (unsigned long long)(gridDim.x - 1);
  }
  __syncthreads();
  if (*flag && threadIdx.x == 0) {
    if (!a.hold) {
      a.step[0] += 1;
      if (a.aux) a.aux[0] += 1;
    }
    a.step[1] = 0;
  }
}
// the slice workgroups of an Adam launch: the arena ranges no packed item covers
__device__ __forceinline__ void adam_plain_slice(const PackArgs& a, const float* c, const long b, const long nb) {
  long tot = 0;
  for (int r = 0; r < a.nplain; ++r) tot += a.plainn[r];
  for (long i = b * 256 + threadIdx.x; i < tot; i += nb * 256) {
    int r = 0;
    long o = i;
    while (r + 1 < a.nplain && o >= a.plainn[r]) o -= a.plainn[r++];
    const long e = a.plain0[r] + o;
    float mm = a.am[e], vv = a.av[e];
    const float np = adam_upd(c, a.ag[e], a.ap[e], mm, vv);
    a.am[e] = mm;
    a.av[e] = vv;
    a.ap[e] = np;
  }
}
// the layer of flat workgroup v (wg0 prefix sums; v >= wg0[n]: the zero / copy slice, returns n)
__device__ __forceinline__ int pack_layer_of(const PackArgs& a, int v) {
  int l = 0;
  while (l < a.n && v >= a.wg0[l + 1]) ++l;
  return l;
}

// the zero / copy slice: workgroup b of nb zeroes the listed buffers and does the listed copies (grid-stride)
__device__ __forceinline__ void pack_zero_slice(const PackArgs& a, const long b, const long nb) {
  const long total = a.zstart[a.zn];
  for (long i = b * 256 + threadIdx.x; i < total; i += nb * 256) {
    int b = 0;
    while (b + 1 < a.zn && i >= a.zstart[b + 1]) ++b;
    if (a.zvec) reinterpret_cast<uint4*>(a.zp[b])[i - a.zstart[b]] = make_uint4(0u, 0u, 0u, 0u);
    else a.zp[b][i - a.zstart[b]] = 0u;
  }
  const long ctot = a.cstart[a.cn];
  for (long i = b * 256 + threadIdx.x; i < ctot; i += nb * 256) {
    int b = 0;
    while (b + 1 < a.cn && i >= a.cstart[b + 1]) ++b;
    a.cd[b][i - a.cstart[b]] = a.csrc[b][i - a.cstart[b]];
  }
}
// small layers: one destination element per thread, each destination walked in its own order
__global__ __launch_bounds__(256) void pack_small_kernel(const PackArgs a) {
  __shared__ float ac[8];
  __shared__ int flag;
  const int v = blockIdx.x, l = pack_layer_of(a, v);
  if (a.ad) {
    adam_consts(a, ac);
    __syncthreads();
  }
  if (l == a.n) {
    if (a.ad) {
      adam_plain_slice(a, ac, v - a.wg0[l], (long)gridDim.x - a.wg0[l]);
      adam_arrive(a, &flag);
    } else {
      pack_zero_slice(a, v - a.wg0[l], (long)gridDim.x - a.wg0[l]);
    }
    return;
  }
  const int cs = a.cs[l], cbn = a.cb[l], kk = a.kk[l];
  const int total = cs * cbn * kk;
  const float* __restrict__ src = a.src[l];
  const FDiv f_cs = FDiv::make(cs), f_cb = FDiv::make(cbn);
  const int b = v - a.wg0[l], nb = a.wg0[l + 1] - a.wg0[l];
  if (a.ad) {  // one source element per thread: Adam, then its two packed positions
    const long o0 = src - a.ap;
    const FDiv f_kk = FDiv::make(kk);
    for (int e = b * 256 + threadIdx.x; e < total; e += nb * 256) {
      const long o = o0 + e;
      float mm = a.am[o], vv = a.av[o];
      const float np = adam_upd(ac, a.ag[o], a.ap[o], mm, vv);
      a.am[o] = mm;
      a.av[o] = vv;
      a.ap[o] = np;
      const int q = f_kk.div(e), tap = e - q * kk, c_s = f_cb.div(q), c_b = q - c_s * cbn;
      if (a.dg[l]) a.dg[l][(tap * cbn + c_b) * cs + c_s] = np;
      if (a.ds[l]) a.ds[l][(tap * cs + c_s) * cbn + c_b] = np;
    }
    adam_arrive(a, &flag);
    return;
  }
  for (int j = b * 256 + threadIdx.x; j < total; j += nb * 256) {
    if (a.dg[l]) {  // [tap][cb][cs]
      const int q = f_cs.div(j), c_s = j - q * cs, tap = f_cb.div(q), c_b = q - tap * cbn;
      a.dg[l][j] = src[(c_s * cbn + c_b) * kk + tap];
    }
    if (a.ds[l]) {  // [tap][cs][cb]
      const int q = f_cb.div(j), c_b = j - q * cbn, tap = f_cs.div(q), c_s = q - tap * cs;
      a.ds[l][j] = src[(c_s * cbn + c_b) * kk + tap];
    }
  }
}

// LDS-tiled transpose: a workgroup stages a 16 (cs) x 32 (cb) x taps block of W[cs][cb][tap] with
// coalesced loads (each cs row of the block is 32*taps contiguous floats), then writes both copies
// from LDS in their own orders: Wg[tap][cb][cs] in runs of 16 cs, Ws[tap][cs][cb] in runs of 32 cb.
constexpr int PK_CS = 16, PK_CB = 32, PK_MAXK = 16;
__global__ __launch_bounds__(256) void pack_kernel(const PackArgs a) {
  __shared__ float tile[PK_CS * PK_CB * (PK_MAXK + 1)];
  __shared__ float ac[8];
  __shared__ int flag;
  const int v = blockIdx.x, l = pack_layer_of(a, v);
  if (a.ad) {
    adam_consts(a, ac);
    __syncthreads();
  }
  if (l == a.n) {
    if (a.ad) {
      adam_plain_slice(a, ac, v - a.wg0[l], (long)gridDim.x - a.wg0[l]);
      adam_arrive(a, &flag);
    } else {
      pack_zero_slice(a, v - a.wg0[l], (long)gridDim.x - a.wg0[l]);
    }
    return;
  }
  const long ao0 = a.ad ? a.src[l] - a.ap : 0;  // (the item's arena offset: Adam's g / m / v at the same place)
  const int cs = a.cs[l], cbn = a.cb[l], kk = a.kk[l];
  const int tcb = (cbn + PK_CB - 1) / PK_CB;
  const int ntile = ((cs + PK_CS - 1) / PK_CS) * tcb;
  const float* __restrict__ src = a.src[l];
  const int pitch = kk + 1;  // odd: the column walks below hit distinct banks
  const int tb = v - a.wg0[l], tnb = a.wg0[l + 1] - a.wg0[l];
  for (int tile_id = tb; tile_id < ntile; tile_id += tnb) {
    const int cs0 = (tile_id / tcb) * PK_CS, cb0 = (tile_id % tcb) * PK_CB;
    const int ncs = min(PK_CS, cs - cs0), ncb = min(PK_CB, cbn - cb0);
    const int run = ncb * kk;  // contiguous floats per cs row of the block
    const FDiv f_run = FDiv::make(run), f_kk = FDiv::make(kk), f_cs = FDiv::make(ncs), f_cb = FDiv::make(ncb);
    // PU loads per thread in flight (one round trip per PU * 256 elements; a load -> LDS store per
    // iteration walked the 8K-element block in 32 dependent round trips)
    constexpr int PU = 8;
    const int tot = ncs * run;
    for (int e0 = threadIdx.x; e0 < tot; e0 += 256 * PU) {
      float v[PU];
      if (a.ad) {  // Adam on the tile's elements (every load of the batch first), the new values packed below
        float g[PU], m[PU], w[PU];
#pragma unroll
        for (int u = 0; u < PU; ++u) {
          const int e = e0 + u * 256;
          const int i = f_run.div(e), r = e - i * run;
          const long o = ao0 + (e < tot ? ((long)(cs0 + i) * cbn + cb0) * kk + r : 0);
          v[u] = a.ap[o];
          g[u] = a.ag[o];
          m[u] = a.am[o];
          w[u] = a.av[o];
        }
#pragma unroll
        for (int u = 0; u < PU; ++u) {
          const int e = e0 + u * 256;
          const int i = f_run.div(e), r = e - i * run;
          const long o = ao0 + ((long)(cs0 + i) * cbn + cb0) * kk + r;
          if (e < tot) {
            v[u] = adam_upd(ac, g[u], v[u], m[u], w[u]);
            a.am[o] = m[u];
            a.av[o] = w[u];
            a.ap[o] = v[u];
          }
        }
      } else {
#pragma unroll
        for (int u = 0; u < PU; ++u) {
          const int e = e0 + u * 256;
          const int i = f_run.div(e), r = e - i * run;
          v[u] = e < tot ? src[((size_t)(cs0 + i) * cbn + cb0) * kk + r] : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        const int e = e0 + u * 256;
        const int i = f_run.div(e), r = e - i * run;  // r = (cb - cb0)*kk + tap
        const int j = f_kk.div(r), tap = r - j * kk;
        if (e < tot) tile[(i * PK_CB + j) * pitch + tap] = v[u];
      }
    }
    __syncthreads();
    if (a.dg[l])  // [tap][cb][cs]: runs of ncs
      for (int e = threadIdx.x; e < kk * ncb * ncs; e += 256) {
        const int q = f_cs.div(e), i = e - q * ncs, tap = f_cb.div(q), j = q - tap * ncb;
        a.dg[l][((size_t)tap * cbn + cb0 + j) * cs + cs0 + i] = tile[(i * PK_CB + j) * pitch + tap];
      }
    if (a.ds[l])  // [tap][cs][cb]: runs of ncb
      for (int e = threadIdx.x; e < kk * ncs * ncb; e += 256) {
        const int q = f_cb.div(e), j = e - q * ncb, tap = f_cs.div(q), i = q - tap * ncs;
        a.ds[l][((size_t)tap * cs + cs0 + i) * cbn + cb0 + j] = tile[(i * PK_CB + j) * pitch + tap];
      }
    __syncthreads();
  }
  if (a.ad) adam_arrive(a, &flag);
}

// ------------------------------------------------------------------ split-K reduction of WGRAD
// gw[row][c][tap] += sum_s part[s][row][tap*cb + c]; gbias[row] += sum_s part[s][row][N].
// Block = 64 consecutive partial-tile elements x 4 split groups; blockIdx.y takes a slice of the
// splits (fp32 atomics combine the slices when gridDim.y > 1), so every thread sums <= ~8 slabs.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int split, int zper,
                                                           int M, int N, int ntot, int cb, int kk, float* gw,
                                                           float* gbias) {
  __shared__ float red[4][64];
  const int t = threadIdx.x, ol = t & 63, zg = t >> 6;
  const long o = (long)blockIdx.x * 64 + ol;  // element of the [M][ntot] partial tile
  const long total = (long)M * ntot;
  const size_t sstride = (size_t)M * ntot;
  const int z0 = blockIdx.y * zper, z1 = min(split, z0 + zper);
  float acc = 0.f;
  if (o < total) {
    const float* p = part + o;
    int z = z0 + zg;
    for (; z + 12 < z1; z += 16) {
      const float a0 = p[(size_t)z * sstride], a1 = p[(size_t)(z + 4) * sstride];
      const float a2 = p[(size_t)(z + 8) * sstride], a3 = p[(size_t)(z + 12) * sstride];
      acc += (a0 + a1) + (a2 + a3);
    }
    for (; z < z1; z += 4) acc += p[(size_t)z * sstride];
  }
  red[zg][ol] = acc;
  __syncthreads();
  if (t < 64 && o < total) {
    const float v = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
    const int row = (int)(o / ntot), col = (int)(o - (long)row * ntot);
    float* dst;
    if (col < N) {
      const int tap = col / cb, c = col - tap * cb;
      dst = gw + ((size_t)row * cb + c) * kk + tap;
    } else {
      if (!gbias) return;
      dst = gbias + row;
    }
    if (gridDim.y == 1) *dst += v;
    else atomicAdd(dst, v);
  }
}

// ------------------------------------------------------------------ host-side launch
static size_t lds_bytes(const Args& a, int BM_, int BN_) {
  const int WN = (BN_ >= 32) ? 2 : 1, WM = 4 / WN;
  const int LDA = (a.op == OP_WGRAD) ? BM_ + 16 : BM_, LDB = BN_ + ((BN_ % 32) == 0 ? 16 : 0);
  size_t f = 2 * ((size_t)BK * LDA + (size_t)BK * LDB) + 2 * WM * BN_;
  const bool bn1d = a.op == OP_DENSE && a.ca_n == a.K && a.a.xf != CV_XF_NONE;
  f += xf_floats(a.a.xf, bn1d ? a.kchunk : a.ca_n) + xf_floats(a.b.xf, a.cb_n);
  if (a.ep.stat_mode == CV_STAT_BWD) f += 4 * (size_t)a.ce_n;
  return f * sizeof(float);
}

template <int OP, int BM, int BN>
static int launch_t(const Args& a, dim3 grid, hipStream_t st) {
  const size_t lds = lds_bytes(a, BM, BN);
  CV_REQUIRE(lds <= 160 * 1024, "igemm: LDS request %zu bytes exceeds 160 KiB", lds);
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)igemm_kernel<OP, BM, BN>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      cv::set_error("igemm: LDS carve-out of %zu bytes refused: %s", lds, hipGetErrorString(e));
      return 1;
    }
  }
  note_launch((const void*)igemm_kernel<OP, BM, BN>);
  hipLaunchKernelGGL((igemm_kernel<OP, BM, BN>), grid, dim3(NT), lds, st, a);
  CV_LAUNCH_CHECK("igemm");
  return 0;
}

template <int OP>
static int launch_op(const Args& a, int BM_, int BN_, dim3 grid, hipStream_t st) {
  if (BM_ == 128 && BN_ == 64) return launch_t<OP, 128, 64>(a, grid, st);
  if (BM_ == 128 && BN_ == 32) return launch_t<OP, 128, 32>(a, grid, st);
  if (BM_ == 128 && BN_ == 16) return launch_t<OP, 128, 16>(a, grid, st);
  if (BM_ == 64 && BN_ == 64) return launch_t<OP, 64, 64>(a, grid, st);
  if (BM_ == 64 && BN_ == 32) return launch_t<OP, 64, 32>(a, grid, st);
  if (BM_ == 64 && BN_ == 16) return launch_t<OP, 64, 16>(a, grid, st);
  cv::set_error("igemm: unsupported tile %dx%d", BM_, BN_);
  return 1;
}

static void finalize_divs(Args& a) {
  a.f_cb = FDiv::make(a.g.cb);
  a.f_cs = FDiv::make(a.g.cs);
  a.f_kw = FDiv::make(a.g.kw);
  a.f_ws = FDiv::make(a.g.ws);
  a.f_hws = FDiv::make((uint32_t)a.g.hs * a.g.ws);
  a.f_ach = FDiv::make(a.a_ch);
  a.f_opix = FDiv::make(a.o_pix);
  a.f_sdiv = FDiv::make(a.ep.stat_div);
  a.f_s = FDiv::make(a.g.s);
  a.f_n = FDiv::make(a.g.n);
}

// 1: route every call to the generic kernel (kernel-variant comparisons in tests only)
static int g_force_generic = 0;

thread_local int* g_fast_occ_query = nullptr;

// resident workgroups per CU of the specialised-core kernel a launch with this tile would pick
// (0 when the generic kernel would serve it)
static int fast_occupancy(const Args& a0, int BM_, int BN_) {
  if (g_force_generic) return 0;
  Args a = a0;
  finalize_divs(a);
  int occ = 0;
  g_fast_occ_query = &occ;
  const dim3 grid(1, 1, 1);
  int r = -1;
  switch (a.op) {
    case OP_GATHER: r = gemm_fast_gather(a, BM_, BN_, grid, nullptr); break;
    case OP_SCATTER: r = gemm_fast_scatter(a, BM_, BN_, grid, nullptr); break;
    case OP_WGRAD: r = gemm_fast_wgrad(a, BM_, BN_, grid, nullptr); break;
    default: r = gemm_fast_dense(a, BM_, BN_, grid, nullptr); break;
  }
  g_fast_occ_query = nullptr;
  return r >= 0 ? occ : 0;
}

static int device_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

static int launch(Args& a, int BM_, int BN_, int gz, hipStream_t st) {
  finalize_divs(a);
  const int Ntot = a.N + ((a.op == OP_WGRAD && a.gbias) ? 1 : 0);
  const int gx = cdiv(a.M, BM_), gy = cdiv(Ntot, BN_);
  dim3 grid(gx, gy, gz);
  CV_REQUIRE(gx > 0 && gy > 0 && gz > 0, "igemm: empty grid");
  CV_REQUIRE(gx < (1 << 30) && gy < 65536 && gz < 65536, "igemm: grid too large");
  if (!g_force_generic) {  // the specialised core serves every vectorisable call
    int r = -1;
    switch (a.op) {
      case OP_GATHER: r = gemm_fast_gather(a, BM_, BN_, grid, st); break;
      case OP_SCATTER: r = gemm_fast_scatter(a, BM_, BN_, grid, st); break;
      case OP_WGRAD: r = gemm_fast_wgrad(a, BM_, BN_, grid, st); break;
      default: r = gemm_fast_dense(a, BM_, BN_, grid, st); break;
    }
    if (r >= 0) return r;
  }
  switch (a.op) {
    case OP_GATHER: return launch_op<OP_GATHER>(a, BM_, BN_, grid, st);
    case OP_SCATTER: return launch_op<OP_SCATTER>(a, BM_, BN_, grid, st);
    case OP_WGRAD: return launch_op<OP_WGRAD>(a, BM_, BN_, grid, st);
    default: return launch_op<OP_DENSE>(a, BM_, BN_, grid, st);
  }
}

// Row-oriented tile: prefer 64-wide N tiles, shrink N (keeping BM=64) until there are >= 512
// workgroups (measured against 256/384/768/1024-workgroup targets on both bench configs: best or
// within noise).  BM=128 lost everywhere once the BM=64 narrow variants hold 3 workgroups per CU
// (VAE64 conv1 bwd-data 170 -> 112 us, convT4 fwd 92 -> 79 us).
static void pick_tile(long M, int N, int& BM_, int& BN_) {
  // A/B overrides: CV_BM128_MIN (rows from which BM=128 is used), CV_MIN_BLOCKS (N-shrink target)
  static long bm128_min = -1, min_blocks = -1;
  if (bm128_min < 0) {
    const char* e = getenv("CV_BM128_MIN");
    bm128_min = e ? atol(e) : (1L << 40);
    const char* f = getenv("CV_MIN_BLOCKS");
    min_blocks = f ? atol(f) : 512;
  }
  BN_ = (N <= 16) ? 16 : (N <= 32) ? 32 : 64;
  BM_ = (M >= bm128_min) ? 128 : 64;
  while (BN_ > 16 && (long)cdiv(M, BM_) * cdiv(N, BN_) < min_blocks) BN_ >>= 1;
}

// number of K splits: aim for ~1024 workgroups but keep >= 4 K tiles per split
static int pick_split(long tiles, long K, int requested) {
  if (requested > 0) return requested;
  long want = (1024 + tiles - 1) / tiles;
  long maxs = K / (4 * BK);
  if (maxs < 1) maxs = 1;
  if (want > maxs) want = maxs;
  if (want < 1) want = 1;
  if (want > 1024) want = 1024;
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
    CV_REQUIRE(!ep->ebn.ticket || ep->ebn.C == nf, "%s: STAT_FWD layer width %d != %d", what, ep->ebn.C, nf);
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
  CV_REQUIRE(g->mma == CV_MMA_FP32 || g->mma == CV_MMA_BF16, "conv: bad mma precision %d", g->mma);
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

// Per-device workspace of the in-launch split-K (cv_set_gemm_workspace): fragment slabs + per-tile tickets.
// Borrowed from the caller (the library never allocates); GATHER launches on one stream use it one at a time.
constexpr int FIX_MAX_DEV = 16;
constexpr size_t FIX_CNT_WORDS = 4096;  // tickets (zeroed by the caller at registration; self-resetting)
static void* g_fix_work[FIX_MAX_DEV];
static size_t g_fix_bytes[FIX_MAX_DEV];

static bool fix_workspace(float*& part, unsigned*& cnt, size_t& part_bytes) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= FIX_MAX_DEV) {
    (void)hipGetLastError();
    return false;
  }
  if (!g_fix_work[dev] || g_fix_bytes[dev] <= FIX_CNT_WORDS * 4) return false;
  cnt = static_cast<unsigned*>(g_fix_work[dev]);
  part = reinterpret_cast<float*>(static_cast<char*>(g_fix_work[dev]) + FIX_CNT_WORDS * 4);
  part_bytes = g_fix_bytes[dev] - FIX_CNT_WORDS * 4;
  return true;
}

// K slices of an under-filled long-K GATHER: the launch's tiles use less than half of the chip's CUs and
// each would walk >= 16 K tiles alone (VAE64's deep layers at small batches: conv5 forward at 32-256
// images/GPU is 16-128 tiles of K = 4096).  Powers of two while tiles x slices <= 2 x CUs and every slice
// keeps >= 8 K tiles.  CV_SPLITK=0: off (A/B).
static int gather_split(long tiles, int ktiles) {
  static int mode = -1;
  if (mode < 0) {
    const char* e = getenv("CV_SPLITK");
    mode = e ? atoi(e) : 1;
  }
  if (mode == 0 || g_force_generic || ktiles < 16) return 1;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    (void)hipGetLastError();
  }
  if (2 * tiles > cus) return 1;
  int s = 1;
  while (tiles * s * 2 <= 2L * cus && ktiles / (s * 2) >= 8 && s < 16) s *= 2;
  return s;
}

// Pixel-major tiles (Args::pm, cv_gemm_tile.inc) when they pay: the conv's (small pixel, tap) pairs that land in
// the padding — zero products the image-major tiles issue anyway — are >= 10 % of all pairs (VAE64's conv5 / convT1:
// 2x2 <-> 4x4, 28 of 64; conv4 / convT2: 60 of 256; MNIST's conv3 / convT1: 44 of 144), the tile divides the batch
// (rows_tile: BM rows of GATHER / SCATTER, BK K elements of WGRAD) and <= 16 taps / small pixels fit the tile's
// 4-bit lists.  CV_PM=0: off (A/B).
static int g_pm_mode = -1;     // (cv_debug_pm)
static int g_pm_launches = 0;  // calls that took pixel-major tiles (cv_debug_pm_count)
static bool pm_pays(const Geo& g, int rows_tile) {
  if (g_pm_mode < 0) {
    const char* e = getenv("CV_PM");
    g_pm_mode = e ? atoi(e) : 1;
  }
  if (!g_pm_mode || g_force_generic || rows_tile <= 0 || g.n % rows_tile || g.kh * g.kw > 16) return false;
  long valid = 0;
  for (int ys = 0; ys < g.hs; ++ys)
    for (int xs = 0; xs < g.ws; ++xs)
      for (int kh = 0; kh < g.kh; ++kh)
        for (int kw = 0; kw < g.kw; ++kw)
          valid += ((unsigned)(ys * g.s - g.p + kh) < (unsigned)g.hb && (unsigned)(xs * g.s - g.p + kw) < (unsigned)g.wb);
  const bool on = 10 * valid <= 9L * g.hs * g.ws * g.kh * g.kw;
  g_pm_launches += on ? 1 : 0;
  return on;
}

// the other packing of the current call's weights (cv_conv_*_kpack: the k-contiguous B image of the direct
// kernels, [tap][co][ci]), else null
static thread_local const float* g_wk = nullptr;

// GATHER with small = rows.  `in` is the big-grid tensor; w is packed [tap][cb][cs].
// CV_FUSED_OUT=1: the ConvT-to-image forward and the decoder output in one launch with a grid-wide wait for the
// output BN's sums (edge_scatter_out); measured slower (MNIST 0.582 -> 0.616 ms/step: the fused launch needs a
// 4-workgroups-per-CU register budget to be co-resident and ran 57.6 us against 16 + 9.7 us).  Its bounded
// grid-wide wait proceeds on a timeout (g_eo_sync[3]) with partial BN sums that no host code reads back, so the
// form exists only in a diagnostic build (-DCV_GRID_WAIT_AB=1) for A/B runs, never in the shipped library
static int fused_out_enabled() {
#if defined(CV_GRID_WAIT_AB) && CV_GRID_WAIT_AB
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("CV_FUSED_OUT");
    on = (e && atoi(e) != 0) ? 1 : 0;
  }
  return on;
#else
  return 0;
#endif
}

static int run_gather(const Geo& g, const cv_operand* in, const float* w, const float* bias, float* out,
                      const cv_epilogue* ep, hipStream_t st, const char* what, int mma) {
  if (!g_force_generic) {
    const int er = edge_gather(g, in, w, bias, out, ep, st);
    if (er >= 0) return er;
    const int dr = direct_gather(g, in, g_wk, bias, out, ep, st, mma);
    if (dr >= 0) return dr;
  }
  const int nr = narrow_gather(g, in, w, bias, out, ep, st);
  if (nr >= 0) return nr;
  Args a;
  init_args(a);
  a.op = OP_GATHER;
  a.mma = mma;
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
  if (apply_epilogue(a, ep, a.N, what)) return 1;
  int BM_, BN_;
  pick_tile(a.M, a.N, BM_, BN_);
  a.kchunk = ((a.K + BK - 1) / BK) * BK;
  // long K (>= 32 K tiles): wide 64-column tiles split along K fill the chip with 4x fewer passes over the
  // A operand than the narrow tiles pick_tile shrinks to for parallelism (C5's conv5 forward: 64 tiles x 4
  // slices of 32 K tiles instead of 256 tiles of 128)
  if (a.K % BK == 0 && a.K / BK >= 32 && a.N >= 64 && BN_ < 64) {
    const long t64 = (long)cdiv(a.M, 64) * cdiv(a.N, 64);
    if (t64 * gather_split(t64, a.K / BK) >= (long)cdiv(a.M, BM_) * cdiv(a.N, BN_)) {
      BM_ = 64;
      BN_ = 64;
    }
  }
  a.pm = (g.cb % BK == 0 && pm_pays(g, BM_)) ? 1 : 0;
  const long tiles = (long)cdiv(a.M, BM_) * cdiv(a.N, BN_);
  const int split = (a.K % BK == 0) ? gather_split(tiles, a.K / BK) : 1;
  float* part = nullptr;
  unsigned* cnt = nullptr;
  size_t pbytes = 0;
  if (split > 1 && tiles <= (long)FIX_CNT_WORDS && fix_workspace(part, cnt, pbytes) &&
      (size_t)tiles * split * BM_ * BN_ * sizeof(float) <= pbytes) {
    Args s = a;
    s.kchunk = cdiv(a.K / BK, split) * BK;
    s.fix_part = part;
    s.fix_cnt = cnt;
    finalize_divs(s);
    const dim3 grid(cdiv(s.M, BM_), cdiv(s.N, BN_), cdiv(a.K, s.kchunk));
    const int r = gemm_fast_gather(s, BM_, BN_, grid, st);  // (the generic kernel has no slab combine)
    if (r >= 0) return r;
  }
  return launch(a, BM_, BN_, 1, st);
}

// SCATTER with big = rows. `in` is the small-grid tensor; w is packed [tap][cs][cb].
static int run_scatter(const Geo& g, const cv_operand* in, const float* w, const float* bias, float* out,
                       const cv_epilogue* ep, hipStream_t st, const char* what, int mma) {
  if (!g_force_generic) {
    const int er = edge_scatter(g, in, w, bias, out, ep, st);
    if (er >= 0) return er;
    CV_REQUIRE(out, "%s: statistics-only output (out = NULL) is served by the image-side edge scatter only", what);
    const int dr = direct_scatter(g, in, g_wk, bias, out, ep, st, mma);
    if (dr >= 0) return dr;
  }
  CV_REQUIRE(out, "%s: statistics-only output (out = NULL) is served by the image-side edge scatter only", what);
  const int nr = narrow_scatter(g, in, w, bias, out, ep, st);
  if (nr >= 0) return nr;
  Args a;
  init_args(a);
  a.op = OP_SCATTER;
  a.mma = mma;
  a.g = g;
  a.a = *in;
  a.ca_n = (in->xf != CV_XF_NONE) ? g.cs : 0;
  if (in->xf != CV_XF_NONE) CV_REQUIRE(in->bn.C == g.cs, "%s: BN width %d != channels %d", what, in->bn.C, g.cs);
  a.w = w;
  a.bias = bias;
  a.out = out;
  a.M = g.n * cdiv(g.hb, g.s) * cdiv(g.wb, g.s);  // largest class
  a.N = g.cb;
  a.K = cdiv(g.kh, g.s) * cdiv(g.kw, g.s) * g.cs;
  if (apply_epilogue(a, ep, a.N, what)) return 1;
  int BM_, BN_;
  pick_tile((long)a.M * g.s * g.s, a.N, BM_, BN_);
  a.pm = (g.cs % BK == 0 && pm_pays(g, BM_)) ? 1 : 0;
  // in-launch split-K as in run_gather, for kernels whose stride-parity classes all have the same taps
  // (kh, kw multiples of the stride: every class has K = a.K) and even class extents
  const int ss = g.s * g.s;
  if (g.kh % g.s == 0 && g.kw % g.s == 0 && g.hb % g.s == 0 && g.wb % g.s == 0 && a.K % BK == 0 && a.K / BK >= 32) {
    if (a.N >= 64 && BN_ < 64) {
      const long t64 = (long)cdiv(a.M, 64) * cdiv(a.N, 64) * ss;
      if (t64 * gather_split(t64, a.K / BK) >= (long)cdiv(a.M, BM_) * cdiv(a.N, BN_) * ss) {
        BM_ = 64;
        BN_ = 64;
      }
    }
    const long tiles = (long)cdiv(a.M, BM_) * cdiv(a.N, BN_) * ss;
    const int split = gather_split(tiles, a.K / BK);
    float* part = nullptr;
    unsigned* cnt = nullptr;
    size_t pbytes = 0;
    if (split > 1 && tiles <= (long)FIX_CNT_WORDS && fix_workspace(part, cnt, pbytes) &&
        (size_t)tiles * split * BM_ * BN_ * sizeof(float) <= pbytes) {
      Args s = a;
      s.kchunk = cdiv(a.K / BK, split) * BK;
      s.fix_part = part;
      s.fix_cnt = cnt;
      finalize_divs(s);
      const dim3 grid(cdiv(s.M, BM_), cdiv(s.N, BN_), ss * cdiv(a.K, s.kchunk));
      const int r = gemm_fast_scatter(s, BM_, BN_, grid, st);
      if (r >= 0) return r;
    }
  }
  return launch(a, BM_, BN_, g.s * g.s, st);
}

struct WPlan {
  int BM, BN, split, kchunk;
};

// Split-K plan of a WGRAD problem (independent of whether a bias column is present, so the
// workspace query and the launch agree): ~1024 workgroups, >= 8 K tiles per split (>= 4 when the
// problem would otherwise not fill the 256 CUs).  128-row tiles when M allows, unless their grid would hold
// <= 2 workgroups per CU (few K tiles: MNIST's conv3-sized gradients, VAE64's conv5): then 64-row tiles, twice
// the workgroups (MNIST decoder convT1 gradient 37.2 -> 35.0 us, VAE64 conv5 pair 200.6 -> 195.3 us; applied
// everywhere they cost VAE64's 1024-workgroup gradients ~7 us each).
// cap_ovr >= 0 replaces the dual-capture row cap (the workspace query takes the max over both choices).
// tgt_ovr > 0 replaces the workgroup target (pixel-major launches: wgrad_pm_target).
static WPlan wgrad_plan(int M, int N, long K, int split_k, int cap_ovr = -1, long tgt_ovr = 0) {
  WPlan w;
  const int Ntot = N + 1;
  w.BN = (Ntot <= 16) ? 16 : (Ntot <= 32) ? 32 : 64;
  const long ktiles = (K + BK - 1) / BK;
  static long target = -1;  // A/B override: CV_WGRAD_TARGET (workgroups the split aims for)
  static int bm_ovr = -2;   // A/B override: CV_WGRAD_BM = 64 / 128 (row tile whenever M allows)
  if (target < 0) {
    const char* e = getenv("CV_WGRAD_TARGET");
    target = e ? atol(e) : 1024;
    if (target < 1) target = 1024;
    e = getenv("CV_WGRAD_BM");
    bm_ovr = e ? atoi(e) : -1;
  }
  auto split_for = [&](int bm) -> long {
    if (split_k > 0) return split_k > 4096 ? 4096 : split_k;
    const long tiles = (long)cdiv(M, bm) * cdiv(Ntot, w.BN);
    const long tg = tgt_ovr > 0 ? tgt_ovr : target;
    long split = (tg + tiles - 1) / tiles;
    long maxs = ktiles / 8;
    if (tiles * maxs < 256) maxs = ktiles / 4;
    if (maxs < 1) maxs = 1;
    if (split > maxs) split = maxs;
    if (split < 1) split = 1;
    return split > 4096 ? 4096 : split;
  };
  w.BM = (M >= 128) ? 128 : 64;
  // (inside a dual launch the weight gradient takes 64-row tiles: the 128-row tile's ~260 registers would hold the
  // whole grid to one workgroup per CU)
  const int cap = split_k > 0 ? 0 : cap_ovr >= 0 ? cap_ovr : dual_wgrad_bm_cap();
  if (cap && w.BM > cap) w.BM = cap;
  if (w.BM == 128) {
    if (bm_ovr == 64) {
      w.BM = 64;
    } else if (bm_ovr != 128 && split_k <= 0) {
      const long wgs = (long)cdiv(M, 128) * cdiv(Ntot, w.BN) * split_for(128);
      if (wgs <= 512) w.BM = 64;  // (2 x the 256 CUs; a constant, so the workspace query needs no device)
    }
  }
  const long split = split_for(w.BM);
  w.kchunk = (int)(((K + split - 1) / split + BK - 1) / BK) * BK;
  w.split = (int)((K + w.kchunk - 1) / w.kchunk);
  return w;
}

// Queried outside any capture, so it must cover both row tiles a launch may take: the plain plan and the one capped
// at 64 rows inside a dual grid (today the capped split never exceeds the uncapped one, but nothing forces that).
// Workgroups a pixel-major WGRAD launch aims for.  Its tiles walk only the pixels their tap reads inside the image, so
// they are shorter than the plain plan assumes; where 64-row tiles alone give >= 256 workgroups (VAE64's conv5 and
// convT1 gradients: 512 tiles) the launch takes no K split at all — every tile writes its gradient block once, no
// split-K partials for cv_step_reduce (C3's conv5 pair 189.9 -> 160.3 us in-step); below that (conv4 / convT2: 128
// tiles) the plain target's split stays (256 there measured the pair 168 -> 187 us).  CV_PM_WTARGET: a fixed target
// (A/B).
long dual_wgrad_slots();  // (cv_dual.hip)

static long wgrad_pm_target(long tiles64 = 0) {
  static long v = -1;
  if (v < 0) {
    const char* e = getenv("CV_PM_WTARGET");
    v = e ? atol(e) : 0;
    if (v < 0) v = 0;
  }
  if (v > 0) return v;
  // (a target of 256 against >= 256 64-row tiles: the 128-row split is then 1, so wgrad_plan takes 64-row tiles
  // at split 1 — a target of tiles64 itself would not, wgrad_plan's tile count includes the bias column)
  return tiles64 >= 256 ? 256 : 0;
}

static size_t wgrad_ws_bytes(int M, int N, long K, int split_k) {
  size_t b = 0;
  const long t64 = (long)cdiv(M, 64) * cdiv(N + 1, (N + 1 <= 16) ? 16 : (N + 1 <= 32) ? 32 : 64);
  for (int cap : {0, 64})
    for (long tg : {0L, wgrad_pm_target(t64)}) {
      const WPlan w = wgrad_plan(M, N, K, split_k, cap, tg);
      size_t need = w.split > 1 ? (size_t)w.split * M * (N + 1) * sizeof(float) : 0;
      // (the self-reducing form's fragment slabs: whole BM x BN tiles per split, bias column included)
      const size_t slab = w.split > 1 ? (size_t)w.split * cdiv(M, w.BM) * w.BM * cdiv(N + 1, w.BN) * w.BN * sizeof(float)
                                      : 0;
      if (slab > need) need = slab;
      if (need > b) b = need;
    }
  return b;
}

// Deferred weight gradients (cv_*_backward_weight_deferred): while a sink is set, the split-K partial
// tiles are left in the caller's workspace and their layout is recorded instead of launching the reduction;
// cv_step_reduce later sums every deferred gradient of the step in one launch.
static thread_local cv_wgrad_defer* g_defer_sink = nullptr;
static int g_wgrad_self = -1;  // self-reducing deferred split-K (opt-in: CV_WGRAD_SELF, cv_debug_wgrad_self)

static int launch_wgrad_reduce(const float* part, int split, int M, int N, int ntot, int cb, int kk, float* gw,
                               float* gbias, hipStream_t st) {
  if (g_defer_sink) {
    cv_wgrad_defer& d = *g_defer_sink;
    d.part = part;
    d.split = split;
    d.M = M;
    d.N = N;
    d.ntot = ntot;
    d.cb = cb;
    d.kk = kk;
    d.gweight = gw;
    d.gbias = gbias;
    return 0;
  }
  const int gx = cdiv((long)M * ntot, 64);
  int gy = cdiv(split, 32);  // <= 32 slabs per block (8 per thread)
  const int zper = cdiv(split, gy);
  gy = cdiv(split, zper);
  note_launch((const void*)wgrad_reduce_kernel);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(gx, gy), dim3(256), 0, st, part, split, zper, M, N, ntot, cb, kk, gw,
                     gbias);
  CV_LAUNCH_CHECK("wgrad_reduce");
  return 0;
}

int wgrad_reduce_launch(const float* part, int split, int M, int N, int ntot, int cb, int kk, float* gw,
                        float* gbias, hipStream_t st) {
  return launch_wgrad_reduce(part, split, M, N, ntot, cb, kk, gw, gbias, st);
}

static int run_wgrad(const Geo& g, const cv_operand* small, const cv_operand* big, float* gw, float* gbias,
                     int split_k, float* work, size_t work_bytes, hipStream_t st, int mma) {
  if (split_k <= 0 && !g_force_generic) {
    const int er = edge_wgrad(g, small, big, gw, gbias, work, work_bytes, st);
    if (er >= 0) return er;
  }
  Args a;
  init_args(a);
  a.op = OP_WGRAD;
  a.mma = mma;
  a.g = g;
  a.a = *small;
  a.b = *big;
  a.ca_n = (small->xf != CV_XF_NONE) ? g.cs : 0;
  a.cb_n = (big->xf != CV_XF_NONE) ? g.cb : 0;
  if (small->xf != CV_XF_NONE) CV_REQUIRE(small->bn.C == g.cs, "wgrad: small-grid BN width mismatch");
  if (big->xf != CV_XF_NONE) CV_REQUIRE(big->bn.C == g.cb, "wgrad: big-grid BN width mismatch");
  CV_REQUIRE(!small->nchw, "wgrad: the small-grid operand must be NHWC");
  a.out = gw;
  a.gbias = gbias;
  a.M = g.cs;
  a.N = g.kh * g.kw * g.cb;
  CV_REQUIRE(!gbias || (a.N % 4) == 0, "wgrad: bias column needs taps*channels % 4 == 0");
  a.K = g.n * g.hs * g.ws;
  // bf16 contractions aim their K split at fewer workgroups (CV_WGRAD_TARGET_BF16, default 512; the fp32 default
  // stays 1024): with the weight gradients beside the backward-data on a side stream, C5's bf16 shard 1.090 -> 1.078
  // ms (same box, two rounds), its fp32 twin and CelebA neutral-to-slower at 512
  static long bf16_tg = -1;
  if (bf16_tg < 0) {
    const char* e = getenv("CV_WGRAD_TARGET_BF16");
    bf16_tg = e ? atol(e) : 512;
    if (bf16_tg < 0) bf16_tg = 0;
  }
  WPlan w = wgrad_plan(a.M, a.N, a.K, split_k, -1, mma == CV_MMA_BF16 ? bf16_tg : 0);
  const int Ntot = a.N + (gbias ? 1 : 0);
  // pixel-major K (a K tile = 32 images at one small pixel; an N tile = one tap): the tile skips the pixels at which
  // its tap reads padding (the split is then re-cut per tile over the pixels it visits)
  a.pm = (!gbias && g.cb % w.BN == 0 && g.hs * g.ws <= 16 && pm_pays(g, BK)) ? 1 : 0;
  if (a.pm && split_k <= 0) {
    const long tg = wgrad_pm_target((long)cdiv(a.M, 64) * cdiv(Ntot, w.BN));
    if (tg > 0) w = wgrad_plan(a.M, a.N, a.K, split_k, -1, tg);
  }
  if (split_k <= 0) {  // inside a served dual grid: at most the slots its first resident round leaves (A/B knob)
    const long free = dual_wgrad_slots();
    const long tiles = (long)cdiv(a.M, w.BM) * cdiv(Ntot, w.BN);
    if (free > 0 && tiles * w.split > free && free >= tiles) w = wgrad_plan(a.M, a.N, a.K, split_k, -1, (free / tiles) * tiles);
  }
  if (split_k <= 0 && w.split > 1) {
    // one round of resident workgroups: a second, partial round costs a whole extra workgroup time
    // (prologue + K loop + epilogue) while fewer, longer splits only lengthen the K loop
    const long tiles = (long)cdiv(a.M, w.BM) * cdiv(Ntot, w.BN);
    a.kchunk = w.kchunk;
    a.gbias = gbias;
    const int occ = fast_occupancy(a, w.BM, w.BN);
    const long slots = (long)device_cus() * occ;
    if (occ > 0 && tiles * w.split > slots && tiles <= slots) {
      const long s2 = slots / tiles;
      w.kchunk = (int)(((a.K + s2 - 1) / s2 + BK - 1) / BK) * BK;
      w.split = (int)((a.K + w.kchunk - 1) / w.kchunk);
    }
  }
  a.kchunk = w.kchunk;
  {
    static int log = -1;
    if (log < 0) log = getenv("CV_WGRAD_LOG") ? 1 : 0;
    if (log)
      fprintf(stderr, "wgrad M=%d N=%d K=%d pm=%d BM=%d BN=%d split=%d kchunk=%d\n", a.M, a.N, a.K, a.pm, w.BM, w.BN,
              w.split, w.kchunk);
  }
  static int atomic_splits = -1;  // A/B knob CV_WGRAD_ATOMIC=1: split-K tiles added with fp32 atomics, no partials
  if (atomic_splits < 0) {
    const char* e = getenv("CV_WGRAD_ATOMIC");
    atomic_splits = (e && atoi(e) != 0) ? 1 : 0;
  }
  if (atomic_splits) work = nullptr;
  // Self-reducing split (deferred gradients, opt-in CV_WGRAD_SELF=1 / cv_debug_wgrad_self): every K slice parks its
  // fragments as a slab in `work` and takes its tile's ticket (the device's in-launch split-K tickets,
  // cv_set_gemm_workspace); the slice that draws the last ticket sums the slabs in slice order and adds the tile into
  // gweight / gbias itself, so no partials are left for cv_step_reduce to read back (VAE64 bs = 256: ~240 MB per
  // step).  Measured slower (round 6, same box, two rounds): MNIST 0.4748 -> 0.6097 ms, CelebA 2.093 -> 2.269 ms,
  // PACS 0.894 -> 0.962 ms, C5 bf16 1.213 -> 1.412 ms — the last slice of every tile sums 8-16 slabs alone, a serial
  // tail per tile, where cv_step_reduce streams all partials at ~4.6 TB/s in one wide launch.
  if (g_wgrad_self < 0) {
    const char* e = getenv("CV_WGRAD_SELF");
    g_wgrad_self = e ? (atoi(e) != 0) : 0;
  }
  if (w.split > 1 && work && g_wgrad_self && g_defer_sink) {
    const long tiles = (long)cdiv(a.M, w.BM) * cdiv(Ntot, w.BN);
    const size_t slab = (size_t)w.split * tiles * w.BM * w.BN * sizeof(float);
    float* fpart = nullptr;
    unsigned* cnt = nullptr;
    size_t pbytes = 0;
    if (tiles <= (long)FIX_CNT_WORDS && work_bytes >= slab && fix_workspace(fpart, cnt, pbytes)) {
      a.fix_part = work;
      a.fix_cnt = cnt;
      if (launch(a, w.BM, w.BN, w.split, st)) return 1;
      return 0;  // (the defer record stays split 0: nothing left to reduce)
    }
  }
  if (w.split > 1 && work) {
    const size_t need = (size_t)w.split * a.M * Ntot * sizeof(float);
    CV_REQUIRE(work_bytes >= need, "wgrad: workspace %zu bytes < %zu needed", work_bytes, need);
    a.part = work;
  }
  if (launch(a, w.BM, w.BN, w.split, st)) return 1;
  if (a.part) return launch_wgrad_reduce(work, w.split, a.M, a.N, Ntot, g.cb, g.kh * g.kw, gw, gbias, st);
  return 0;
}

}  // namespace cv

using namespace cv;

extern "C" size_t cv_gemm_workspace_bytes(void) {
  // 512 slices of one 64 x 64 fp32 tile each + the ticket words
  return FIX_CNT_WORDS * 4 + (size_t)512 * 64 * 64 * sizeof(float);
}

extern "C" int cv_set_gemm_workspace(void* work, size_t bytes) {
  clear_error();
  int dev = 0;
  CV_REQUIRE(hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < FIX_MAX_DEV, "set_gemm_workspace: no device");
  CV_REQUIRE(!work || bytes > FIX_CNT_WORDS * 4, "set_gemm_workspace: %zu bytes is too small", bytes);
  CV_REQUIRE(!work || (reinterpret_cast<uintptr_t>(work) & 15) == 0, "set_gemm_workspace: pointer not 16-byte aligned");
  g_fix_work[dev] = work;
  g_fix_bytes[dev] = work ? bytes : 0;
  return 0;
}

extern "C" int cv_debug_wgrad_self(int on) {
  const int prev = g_wgrad_self;
  if (on >= 0) g_wgrad_self = on ? 1 : 0;
  return prev;
}

extern "C" int cv_debug_pm(int on) {
  const int prev = g_pm_mode;
  if (on >= 0) g_pm_mode = on ? 1 : 0;
  return prev;
}

extern "C" int cv_debug_pm_count(int reset) {
  const int n = g_pm_launches;
  if (reset) g_pm_launches = 0;
  return n;
}

extern "C" int cv_debug_force_generic_gemm(int on) {
  const int prev = g_force_generic;
  g_force_generic = on ? 1 : 0;
  return prev;
}

#ifdef CV_STAMPS
CV_STAMPS_SETTER(cv_debug_set_stamps)
#endif

static int pack_launch(const cv_conv_pack* items, int n, void* const* zptrs, const size_t* zbytes, int zcount,
                       cv_stream_t stream, void* const* cdst = nullptr, const void* const* csrc = nullptr,
                       const size_t* cbytes = nullptr, int ccount = 0, const PackArgs* adam = nullptr) {
  CV_REQUIRE((items || n == 0) && n >= 0 && n <= MAX_PACK && (n > 0 || zcount > 0 || ccount > 0),
             "pack_conv_weights: 0..%d items (0 only with buffers to zero or copy)", MAX_PACK);
  CV_REQUIRE(zcount >= 0 && zcount <= 8 && (!zcount || (zptrs && zbytes)), "pack_conv_weights: 0..8 zeroed buffers");
  CV_REQUIRE(ccount >= 0 && ccount <= 4 && (!ccount || (cdst && csrc && cbytes)), "pack_conv_weights: 0..4 copies");
  PackArgs a;
  memset(&a, 0, sizeof(a));
  if (adam) {  // (the Adam block: fields from ad on)
    a.ad = 1;
    a.ap = adam->ap; a.ag = adam->ag; a.am = adam->am; a.av = adam->av;
    a.hyper = adam->hyper; a.step = adam->step; a.gscale = adam->gscale; a.aux = adam->aux;
    a.hold = adam->hold;
    a.nplain = adam->nplain;
    for (int i = 0; i < adam->nplain; ++i) { a.plain0[i] = adam->plain0[i]; a.plainn[i] = adam->plainn[i]; }
  }
  a.cn = ccount;
  for (int i = 0; i < ccount; ++i) {
    CV_REQUIRE(cdst[i] && csrc[i] && cbytes[i] % 16 == 0 && (((uintptr_t)cdst[i] | (uintptr_t)csrc[i]) & 15) == 0,
               "pack_conv_weights: copy %d not 16-byte aligned and sized", i);
    a.cd[i] = (uint4*)cdst[i];
    a.csrc[i] = (const uint4*)csrc[i];
    a.cstart[i + 1] = a.cstart[i] + (long)(cbytes[i] / 16);
  }
  a.zn = zcount;
  a.zvec = 1;
  for (int i = 0; i < zcount; ++i) {
    CV_REQUIRE(zptrs[i] && zbytes[i] % 4 == 0 && ((uintptr_t)zptrs[i] & 3) == 0,
               "pack_conv_weights: zero buffer %d not 4-byte granular", i);
    a.zp[i] = (uint32_t*)zptrs[i];
    a.zvec = a.zvec && zbytes[i] % 16 == 0 && ((uintptr_t)zptrs[i] & 15) == 0;
  }
  for (int i = 0; i < zcount; ++i) a.zstart[i + 1] = a.zstart[i] + (long)(zbytes[i] / (a.zvec ? 16 : 4));
  long mx = 0;
  for (int i = 0; i < n; ++i) {
    const cv_conv_pack& p = items[i];
    CV_REQUIRE(p.src && (p.gather || p.scatter) && p.cs > 0 && p.cb > 0 && p.kh > 0 && p.kw > 0,
               "pack_conv_weights: item %d incomplete", i);
    a.src[i] = p.src;
    a.dg[i] = p.gather;
    a.ds[i] = p.scatter;
    a.cs[i] = p.cs;
    a.cb[i] = p.cb;
    a.kk[i] = p.kh * p.kw;
    const long tot = (long)p.cs * p.cb * p.kh * p.kw;
    CV_REQUIRE(tot < (1L << 31), "pack_conv_weights: item %d too large", i);
    mx = tot > mx ? tot : mx;
  }
  a.n = n;
  bool tiled = mx >= 256 * 1024;  // big layers: the LDS-tiled transpose; small ones: more parallelism
  for (int i = 0; i < n; ++i)
    if (a.kk[i] > PK_MAXK) tiled = false;
  // One flat grid: each layer gets exactly the workgroups it has work for (its tiles, or its elements / 256, capped
  // at 1024), then the zero / copy slice (~4 16-byte units per thread).  (The 2-D grid of round 5 gave every layer the
  // widest layer's row of workgroups: on VAE64 ~10k of its 11k workgroups found no tile and only took dispatch slots
  // and their LDS.)
  a.wg0[0] = 0;
  for (int i = 0; i < n; ++i) {
    long t = tiled ? (long)cdiv(a.cs[i], PK_CS) * cdiv(a.cb[i], PK_CB)
                   : ((long)a.cs[i] * a.cb[i] * a.kk[i] + 255) / 256;
    if (t > 1024) t = 1024;
    a.wg0[i + 1] = a.wg0[i] + (int)t;
  }
  long zg = 0;
  if (zcount || ccount) {
    zg = (a.zstart[zcount] + a.cstart[ccount] + 1023) / 1024;
    if (zg < 1) zg = 1;
    if (zg > 1024) zg = 1024;
  }
  if (a.ad) {  // (Adam: the slice updates the plain ranges, ~4 elements per thread)
    long tot = 0;
    for (int r = 0; r < a.nplain; ++r) tot += a.plainn[r];
    zg = (tot + 1023) / 1024;
    if (zg < 1) zg = 1;
    if (zg > 1024) zg = 1024;
  }
  const dim3 grid((unsigned)(a.wg0[n] + zg));
  if (tiled) hipLaunchKernelGGL(pack_kernel, grid, dim3(256), 0, S(stream), a);
  else hipLaunchKernelGGL(pack_small_kernel, grid, dim3(256), 0, S(stream), a);
  CV_LAUNCH_CHECK("pack_conv_weights");
  return 0;
}

extern "C" int cv_pack_conv_weights(const cv_conv_pack* items, int n, cv_stream_t stream) {
  clear_error();
  return pack_launch(items, n, nullptr, nullptr, 0, stream);
}

extern "C" int cv_pack_conv_weights_zero(const cv_conv_pack* items, int n, void* const* zero_ptrs,
                                         const size_t* zero_bytes, int zero_count, cv_stream_t stream) {
  clear_error();
  return pack_launch(items, n, zero_ptrs, zero_bytes, zero_count, stream);
}

static int adam_pack_part(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t numel,
                          const float* hyper, int64_t* step, const float* grad_scale, int64_t* aux_counter,
                          const cv_conv_pack* items, int n, int advance, cv_stream_t stream);

extern "C" int cv_adam_pack_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                                 int64_t numel, const float* hyper, int64_t* step, const float* grad_scale,
                                 int64_t* aux_counter, const cv_conv_pack* items, int n, cv_stream_t stream) {
  return adam_pack_part(params, grads, exp_avg, exp_avg_sq, numel, hyper, step, grad_scale, aux_counter, items, n, 1,
                        stream);
}

extern "C" int cv_adam_pack_step_part(float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                                      int64_t numel, const float* hyper, int64_t* step, const float* grad_scale,
                                      int64_t* aux_counter, const cv_conv_pack* items, int n, int advance,
                                      cv_stream_t stream) {
  return adam_pack_part(params, grads, exp_avg, exp_avg_sq, numel, hyper, step, grad_scale, aux_counter, items, n,
                        advance, stream);
}

static int adam_pack_part(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t numel,
                          const float* hyper, int64_t* step, const float* grad_scale, int64_t* aux_counter,
                          const cv_conv_pack* items, int n, int advance, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(params && grads && exp_avg && exp_avg_sq && hyper && step && numel > 0 && items && n > 0 &&
                 n <= MAX_PACK, "adam_pack_step: bad args");
  // the items' parameter ranges inside the arena, sorted: the plain ranges are the gaps
  long lo[MAX_PACK], hi[MAX_PACK];
  int ord[MAX_PACK];
  for (int i = 0; i < n; ++i) {
    const cv_conv_pack& it = items[i];
    const long o = it.src - params, len = (long)it.cs * it.cb * it.kh * it.kw;
    CV_REQUIRE(it.src >= params && o + len <= numel, "adam_pack_step: item %d outside the parameter arena", i);
    lo[i] = o;
    hi[i] = o + len;
    ord[i] = i;
  }
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j)
      if (lo[ord[j]] < lo[ord[i]]) { const int q = ord[i]; ord[i] = ord[j]; ord[j] = q; }
  PackArgs ad;
  memset(&ad, 0, sizeof(ad));
  ad.ap = params; ad.ag = grads; ad.am = exp_avg; ad.av = exp_avg_sq;
  ad.hyper = hyper; ad.step = step; ad.gscale = grad_scale; ad.aux = aux_counter;
  ad.hold = advance ? 0 : 1;
  long cur = 0;
  for (int k = 0; k < n; ++k) {
    const int i = ord[k];
    CV_REQUIRE(lo[i] >= cur, "adam_pack_step: items %d overlap", i);
    if (lo[i] > cur) { ad.plain0[ad.nplain] = cur; ad.plainn[ad.nplain] = lo[i] - cur; ++ad.nplain; }
    cur = hi[i];
  }
  if (numel > cur) { ad.plain0[ad.nplain] = cur; ad.plainn[ad.nplain] = numel - cur; ++ad.nplain; }
  if (!ad.nplain) { ad.plain0[0] = 0; ad.plainn[0] = 0; ad.nplain = 1; }
  return pack_launch(items, n, nullptr, nullptr, 0, stream, nullptr, nullptr, nullptr, 0, &ad);
}

extern "C" int cv_pack_conv_weights_zero_copy(const cv_conv_pack* items, int n, void* const* zero_ptrs,
                                              const size_t* zero_bytes, int zero_count, void* const* copy_dst,
                                              const void* const* copy_src, const size_t* copy_bytes, int copy_count,
                                              cv_stream_t stream) {
  clear_error();
  return pack_launch(items, n, zero_ptrs, zero_bytes, zero_count, stream, copy_dst, copy_src, copy_bytes, copy_count);
}

extern "C" int cv_conv_forward(const cv_conv* g, const cv_operand* in, const float* wpacked, const float* bias,
                               float* out, const cv_epilogue* ep, cv_stream_t stream) {
  clear_error();
  if (check_conv(g) || check_operand(in, "conv_forward")) return 1;
  CV_REQUIRE(wpacked, "conv_forward: null weight");
  // out == NULL: statistics only (the image-side ConvTranspose2d whose output is read by nothing but its BatchNorm's
  // batch statistics: CLEAR-MIM's estimator forwards); served by the edge scatter alone
  CV_REQUIRE(out || (ep && ep->stat_mode == CV_STAT_FWD && g->transposed), "conv_forward: null out needs a "
             "ConvTranspose2d with the forward statistics epilogue");
  const Geo geo = geo_of(g);
  if (!g->transposed) return run_gather(geo, in, wpacked, bias, out, ep, S(stream), "conv_forward", g->mma);
  return run_scatter(geo, in, wpacked, bias, out, ep, S(stream), "convT_forward", g->mma);
}

extern "C" int cv_conv_backward_data(const cv_conv* g, const cv_operand* gout, const float* wpacked, float* gin,
                                     const cv_epilogue* ep, cv_stream_t stream) {
  clear_error();
  if (check_conv(g) || check_operand(gout, "conv_backward_data")) return 1;
  CV_REQUIRE(wpacked && gin, "conv_backward_data: null weight/gin");
  const Geo geo = geo_of(g);
  if (!g->transposed)
    return run_scatter(geo, gout, wpacked, nullptr, gin, ep, S(stream), "conv_backward_data", g->mma);
  return run_gather(geo, gout, wpacked, nullptr, gin, ep, S(stream), "convT_backward_data", g->mma);
}

extern "C" int cv_conv_forward_kpack(const cv_conv* g, const cv_operand* in, const float* wpacked,
                                     const float* wkpack, const float* bias, float* out, const cv_epilogue* ep,
                                     cv_stream_t stream) {
  g_wk = wkpack;
  const int r = cv_conv_forward(g, in, wpacked, bias, out, ep, stream);
  g_wk = nullptr;
  return r;
}

extern "C" int cv_conv_backward_data_kpack(const cv_conv* g, const cv_operand* gout, const float* wpacked,
                                           const float* wkpack, float* gin, const cv_epilogue* ep,
                                           cv_stream_t stream) {
  g_wk = wkpack;
  const int r = cv_conv_backward_data(g, gout, wpacked, gin, ep, stream);
  g_wk = nullptr;
  return r;
}

extern "C" size_t cv_conv_wgrad_workspace_bytes(const cv_conv* g, int split_k) {
  if (!g) return 0;
  const Geo geo = geo_of(g);
  const size_t gen = wgrad_ws_bytes(geo.cs, geo.kh * geo.kw * geo.cb, (long)geo.n * geo.hs * geo.ws, split_k);
  const size_t edge = split_k > 0 ? 0 : edge_wgrad_ws_bytes(geo, true);
  return gen > edge ? gen : edge;
}

extern "C" int cv_conv_backward_weight(const cv_conv* g, const cv_operand* in, const cv_operand* gout,
                                       float* gweight, float* gbias, int split_k, float* work, size_t work_bytes,
                                       cv_stream_t stream) {
  clear_error();
  if (check_conv(g) || check_operand(in, "conv_backward_weight") || check_operand(gout, "conv_backward_weight"))
    return 1;
  CV_REQUIRE(gweight, "conv_backward_weight: null gweight");
  const Geo geo = geo_of(g);
  CV_REQUIRE(!g->transposed || !gbias, "convT bias gradient is not a WGRAD column (use a reduction)");
  // conv: small = dY, big = X ; convT: small = X, big = dY
  if (!g->transposed) return run_wgrad(geo, gout, in, gweight, gbias, split_k, work, work_bytes, S(stream), g->mma);
  return run_wgrad(geo, in, gout, gweight, nullptr, split_k, work, work_bytes, S(stream), g->mma);
}

extern "C" int cv_conv_backward_weight_deferred(const cv_conv* g, const cv_operand* in, const cv_operand* gout,
                                                float* gweight, float* gbias, float* work, size_t work_bytes,
                                                cv_wgrad_defer* defer, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(defer && work, "conv_backward_weight_deferred: needs a defer record and a workspace");
  memset(defer, 0, sizeof(*defer));  // split 0: the launch wrote gweight / gbias directly
  g_defer_sink = defer;
  const int r = cv_conv_backward_weight(g, in, gout, gweight, gbias, 0, work, work_bytes, stream);
  g_defer_sink = nullptr;
  return r;
}

extern "C" int cv_output_loss(const cv_bn* bn, const float* y, const float* x, int n, int c, int hw, float* xhat,
                              double* rec_out, float* dv_out, double* gstat_out, const float* rec_scale,
                              cv_stream_t stream);

extern "C" int cv_convt_output_loss(const cv_conv* g, const cv_operand* in, const float* wpacked, const float* bias,
                                    float* y, const cv_epilogue* ep, const cv_bn* bn, const float* x, float* xhat,
                                    double* rec_out, float* dv_out, double* gstat_out, const float* rec_scale,
                                    cv_stream_t stream) {
  clear_error();
  if (check_conv(g) || check_operand(in, "convT_output_loss")) return 1;
  CV_REQUIRE(wpacked && y && bn && x && xhat && rec_out, "convT_output_loss: null args");
  if (g->transposed && !g_force_generic && fused_out_enabled()) {
    const int r = edge_scatter_out(geo_of(g), in, wpacked, bias, y, ep, bn, x, xhat, rec_out, dv_out, gstat_out,
                                   rec_scale, S(stream));
    if (r >= 0) return r;
  }
  const int r = cv_conv_forward(g, in, wpacked, bias, y, ep, stream);
  if (r) return r;
  return cv_output_loss(bn, y, x, g->n, g->c_out, g->h_out * g->w_out, xhat, rec_out, dv_out, gstat_out, rec_scale,
                        stream);
}

extern "C" int cv_conv_backward_deferred(const cv_conv* g, const cv_operand* gout, const float* wpacked, float* gin,
                                         const cv_epilogue* ep, const cv_operand* in, float* gweight, float* gbias,
                                         float* work, size_t work_bytes, cv_wgrad_defer* defer, cv_stream_t stream) {
  clear_error();
  if (check_conv(g) || check_operand(gout, "conv_backward") || check_operand(in, "conv_backward")) return 1;
  CV_REQUIRE(wpacked && gin && gweight && defer && work, "conv_backward: null weight / gin / gweight / defer / work");
  if (g->transposed && !gbias && !g_force_generic) {  // the image-side ConvTranspose2d: one launch for both halves
    memset(defer, 0, sizeof(*defer));
    g_defer_sink = defer;
    const int r = edge_bwd(geo_of(g), gout, wpacked, gin, ep, in, gweight, work, work_bytes, S(stream));
    g_defer_sink = nullptr;
    if (r >= 0) return r;
  }
  const int r = cv_conv_backward_data(g, gout, wpacked, gin, ep, stream);
  if (r) return r;
  return cv_conv_backward_weight_deferred(g, in, gout, gweight, gbias, work, work_bytes, defer, stream);
}

extern "C" int cv_conv_backward_deferred_kpack(const cv_conv* g, const cv_operand* gout, const float* wpacked,
                                               const float* wkpack, float* gin, const cv_epilogue* ep,
                                               const cv_operand* in, float* gweight, float* gbias, float* work,
                                               size_t work_bytes, cv_wgrad_defer* defer, cv_stream_t stream) {
  // the layer's backward-data and weight-gradient launches as one dual grid where the pair is served
  // (cv_dual.hip); the image-side layer's fused edge launch and every other path launch as they are planned
  dual_begin();
  g_wk = wkpack;
  const int r = cv_conv_backward_deferred(g, gout, wpacked, gin, ep, in, gweight, gbias, work, work_bytes, defer,
                                          stream);
  g_wk = nullptr;
  const int r2 = dual_end(S(stream), r == 0);
  return r ? r : r2;
}

// cv_conv_backward_deferred_kpack with the weight-gradient launch on a second stream (`side`) where the pair is not
// one dual grid: the layer's weight gradient needs only what the previous layers' launches have written (its input
// activation and this layer's output gradient), like its backward-data, so it runs beside that and the next
// layers' backward-data instead of between them.  `side` first waits for the work issued on `stream` before this
// call (an event; in a capture the side stream joins the graph there), then takes the weight-gradient launch; the
// caller joins `side` back before anything reads the deferred partials (cv_step_reduce).  A served dual grid, the
// image-side layer's fused launch and the self-reducing form (whose ticket words are the stream's in-launch split-K
// workspace) stay on `stream`.
static hipEvent_t g_side_fork[FIX_MAX_DEV];

extern "C" int cv_conv_backward_deferred_kpack_side(const cv_conv* g, const cv_operand* gout, const float* wpacked,
                                                    const float* wkpack, float* gin, const cv_epilogue* ep,
                                                    const cv_operand* in, float* gweight, float* gbias, float* work,
                                                    size_t work_bytes, cv_wgrad_defer* defer, cv_stream_t side,
                                                    cv_stream_t stream) {
  if (g_wgrad_self < 0) {
    const char* e = getenv("CV_WGRAD_SELF");
    g_wgrad_self = e ? (atoi(e) != 0) : 0;
  }
  // (the image-side layers — <= 4 channels on one side — take the edge kernels' fused launch: on `stream`)
  if (!side || side == stream || !g || (g->c_in <= 4 || g->c_out <= 4) || g_wgrad_self || g_force_generic)
    return cv_conv_backward_deferred_kpack(g, gout, wpacked, wkpack, gin, ep, in, gweight, gbias, work, work_bytes,
                                           defer, stream);
  clear_error();
  if (check_conv(g) || check_operand(gout, "conv_backward") || check_operand(in, "conv_backward")) return 1;
  CV_REQUIRE(wpacked && gin && gweight && defer && work, "conv_backward: null weight / gin / gweight / defer / work");
  int dev = 0;
  CV_REQUIRE(hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < FIX_MAX_DEV, "conv_backward_side: no device");
  if (!g_side_fork[dev] && hipEventCreateWithFlags(&g_side_fork[dev], hipEventDisableTiming) != hipSuccess) {
    (void)hipGetLastError();
    g_side_fork[dev] = nullptr;
    set_error("conv_backward_side: event creation failed");
    return 2;
  }
  if (hipEventRecord(g_side_fork[dev], S(stream)) != hipSuccess ||
      hipStreamWaitEvent(S(side), g_side_fork[dev], 0) != hipSuccess) {
    (void)hipGetLastError();
    set_error("conv_backward_side: fork of the side stream failed");
    return 2;
  }
  dual_begin();
  dual_side(true);
  g_wk = wkpack;
  int r = cv_conv_backward_data(g, gout, wpacked, gin, ep, stream);
  // (the weight gradient's own stream is `side`: a launch path the dual capture does not take — the generic core,
  // the edge kernels — issues there directly; a captured one is issued by dual_end, on `stream` inside a served dual
  // grid, else on `side`)
  if (r == 0) r = cv_conv_backward_weight_deferred(g, in, gout, gweight, gbias, work, work_bytes, defer, side);
  g_wk = nullptr;
  dual_side(false);
  const int r2 = dual_end(S(stream), r == 0, S(side));
  return r ? r : r2;
}

// ---------------------------------------------------------------- linear layers
static int linear_launch(Args& a, int accumulate, hipStream_t st) {
  int BM_, BN_;
  pick_tile(a.M, a.N, BM_, BN_);
  long tiles = (long)cdiv(a.M, BM_) * cdiv(a.N, BN_);
  int split = accumulate ? pick_split(tiles, a.K, 0) : 1;
  a.kchunk = ((cdiv(a.K, split) + BK - 1) / BK) * BK;
  split = cdiv(a.K, a.kchunk);
  return launch(a, BM_, BN_, split, st);
}

extern "C" int cv_linear_forward(const cv_linear* g, const cv_operand* in, const float* weight, const float* bias,
                                 float* out, int accumulate, const cv_epilogue* ep, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(g && g->n > 0 && g->in_features > 0 && g->out_features > 0, "linear_forward: bad geometry");
  CV_REQUIRE(g->mma == CV_MMA_FP32 || g->mma == CV_MMA_BF16, "linear_forward: bad mma precision %d", g->mma);
  if (check_operand(in, "linear_forward")) return 1;
  CV_REQUIRE(weight && out, "linear_forward: null weight/out");
  const int ip = g->in_pix > 0 ? g->in_pix : 1, op = g->out_pix > 0 ? g->out_pix : 1;
  CV_REQUIRE(ip == 1 || ip * g->in_ch == g->in_features, "linear_forward: in_pix*in_ch != in_features");
  CV_REQUIRE(op == 1 || op * g->out_ch == g->out_features, "linear_forward: out_pix*out_ch != out_features");
  Args a;
  init_args(a);
  a.op = OP_DENSE;
  a.mma = g->mma;
  a.a = *in;
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
  return linear_launch(a, accumulate, S(stream));
}

extern "C" int cv_linear_backward_data(const cv_linear* g, const cv_operand* gout, const float* weight, float* gin,
                                       int accumulate, const cv_epilogue* ep, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(g && g->n > 0 && g->in_features > 0 && g->out_features > 0, "linear_backward_data: bad geometry");
  CV_REQUIRE(g->mma == CV_MMA_FP32 || g->mma == CV_MMA_BF16, "linear_backward_data: bad mma precision %d", g->mma);
  if (check_operand(gout, "linear_backward_data")) return 1;
  CV_REQUIRE(weight && gin, "linear_backward_data: null weight/gin");
  const int ip = g->in_pix > 0 ? g->in_pix : 1, op = g->out_pix > 0 ? g->out_pix : 1;
  // gin[n][perm_in(k)] = sum_o T(gout[n][perm_out(o)]) * W[o][k]
  Args a;
  init_args(a);
  a.op = OP_DENSE;
  a.mma = g->mma;
  a.a = *gout;
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
  return linear_launch(a, accumulate, S(stream));
}

extern "C" size_t cv_linear_wgrad_workspace_bytes(const cv_linear* g, int split_k) {
  if (!g) return 0;
  return wgrad_ws_bytes(g->out_features, g->in_features, g->n, split_k);
}

extern "C" int cv_linear_backward_weight(const cv_linear* g, const cv_operand* gout, const cv_operand* in,
                                         float* gweight, float* gbias, int split_k, float* work, size_t work_bytes,
                                         cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(g && g->n > 0, "linear_backward_weight: bad geometry");
  CV_REQUIRE(g->mma == CV_MMA_FP32 || g->mma == CV_MMA_BF16, "linear_backward_weight: bad mma precision %d", g->mma);
  if (check_operand(gout, "linear_backward_weight") || check_operand(in, "linear_backward_weight")) return 1;
  const int ip = g->in_pix > 0 ? g->in_pix : 1;
  CV_REQUIRE(g->out_pix <= 1, "linear_backward_weight: permuted outputs unsupported (use cv_declinear_*)");
  CV_REQUIRE(gout->xf == CV_XF_NONE, "linear_backward_weight: transform on gout unsupported");
  // a WGRAD over a 1x1 "small grid" (rows = batch) and an in_pix "big grid":
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
  return run_wgrad(geo, gout, in, gweight, gbias, split_k, work, work_bytes, S(stream), g->mma);
}

extern "C" int cv_linear_backward_weight_deferred(const cv_linear* g, const cv_operand* gout, const cv_operand* in,
                                                  float* gweight, float* gbias, float* work, size_t work_bytes,
                                                  cv_wgrad_defer* defer, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(defer && work, "linear_backward_weight_deferred: needs a defer record and a workspace");
  memset(defer, 0, sizeof(*defer));
  g_defer_sink = defer;
  const int r = cv_linear_backward_weight(g, gout, in, gweight, gbias, 0, work, work_bytes, stream);
  g_defer_sink = nullptr;
  return r;
}
