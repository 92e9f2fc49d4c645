// BatchNorm bookkeeping, decoder output (BN + Sigmoid + reconstruction loss) and the decoder
// Linear -> BatchNorm1d backward for gfx950.
//
// Reference arithmetic replaced:
//   nn.BatchNorm2d/1d running statistics (momentum 0.1, unbiased running var)   vae.py:17-44
//   decoder tail BatchNorm2d(C) + Sigmoid                                       vae.py:44-45, 154-155
//   vae_loss reconstruction term: mean_n sum_{chw} (xhat - x)^2                 losses.py:36-47
//   decoder Linear(z, 2048) -> BatchNorm1d(2048) -> ReLU backward               vae.py:33-35
#include "cv_common.hpp"
#include "cv_ntxent.hpp"

namespace cv {

// ---------------------------------------------------------------- running statistics
constexpr int MAX_BN = 16;
struct RunArgs {
  cv_bn bn[MAX_BN];
  int64_t* nbt[MAX_BN];
  int nl;
  float momentum;
};

// blockIdx.y = layer.  Narrow layers (C < 256): one block, replica folds spread over the block (bn_fold);
// wide layers: blockIdx.x takes channels [256 x, 256 x + 256), one channel per thread (the BN1d layer's
// 2048 features were 8 sequential replica folds per thread in one block)
__global__ __launch_bounds__(256) void bn_running_kernel(const RunArgs a) {
  __shared__ double scratch[4 * 256];
  const int l = blockIdx.y;
  if (l >= a.nl) return;
  const cv_bn& b = a.bn[l];
  float* rm = const_cast<float*>(b.running_mean);
  float* rv = const_cast<float*>(b.running_var);
  const float m = a.momentum;
  auto update = [&](int c, double s, double q, double, double) {
    const double n = (double)b.count;
    const double mean = s / n;
    double var = q / n - mean * mean;
    if (var < 0.0) var = 0.0;
    const double unbiased = (b.count > 1) ? var * n / (n - 1.0) : var;
    rm[c] = m * (float)mean + (1.0f - m) * rm[c];
    rv[c] = m * (float)unbiased + (1.0f - m) * rv[c];
  };
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.nbt[l]) a.nbt[l][0] += 1;
  if (b.C >= 256) {  // (the same per-channel fold as bn_fold's one-channel-per-thread path)
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c < b.C) {
      double s = 0.0, q = 0.0;
      bn_sums(b.stat, b.C, c, s, q);
      update(c, s, q, 0.0, 0.0);
    }
    return;
  }
  if (blockIdx.x != 0) return;
  bn_fold<256>(b, false, scratch, update);
}

struct GradArgs {
  cv_bn bn[MAX_BN];
  float* dg[MAX_BN];
  float* db[MAX_BN];
  int nl;
};
__global__ __launch_bounds__(256) void bn_grads_kernel(const GradArgs a) {
  __shared__ double scratch[4 * 256];
  const int l = blockIdx.y;
  if (l >= a.nl) return;
  cv_bn b = a.bn[l];
  b.stat = b.gstat;  // fold the backward sums
  float* dg = a.dg[l];
  float* db = a.db[l];
  bn_fold<256>(b, false, scratch, [&](int c, double s, double q, double, double) {
    if (db) db[c] = (float)s;
    if (dg) dg[c] = (float)q;
  });
}

__global__ void bn_stats_kernel(const cv_bn b, float* mean, float* invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= b.C) return;
  float m, is;
  bn_mean_istd(b, c, m, is);
  mean[c] = m;
  invstd[c] = is;
}

// ---------------------------------------------------------------- decoder output
// xhat (NCHW) = sigmoid((y - mu)*sc + beta), y NHWC.  One thread per output element in NCHW order.
constexpr int OUT_MAXC = 4;

__global__ __launch_bounds__(256) void output_fwd_kernel(const cv_bn b, const float* __restrict__ y, int n, int c,
                                                         int hw, float* __restrict__ xhat) {
  __shared__ BnFwdC k[OUT_MAXC];
  __shared__ double scratch[4 * 256];
  bn_fold<256>(b, false, scratch, [&](int f, double s, double q, double, double) { k[f] = bn_fwd_const_s(b, f, s, q); });
  const long total = (long)n * c * hw;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int p = (int)(i % hw);
    const long nc = i / hw;
    const int ch = (int)(nc % c);
    const long img = nc / c;
    const float v = bn_out(y[(img * hw + p) * c + ch], k[ch]);
    xhat[i] = 1.0f / (1.0f + expf(-v));
  }
}

// Fused output + reconstruction loss + backward seed.  Elements are visited in NHWC order so the
// dv store (NHWC) is coalesced; x / xhat are NCHW.
// grid-stride over element batches of OL_U per thread: all loads of a batch are issued first
constexpr int OL_U = 4;
struct OutLossArgs {
  cv_bn b;
  const float* y;
  const float* x;
  int n, c, hw;
  FDiv fc, fhw;
  float* xhat;
  double* rec_out;
  float* dv;
  double* gstat;
  const float* rec_scale;
};
// workgroup bx of gx (a grid of its own, or its share of an auxiliary-role grid)
__device__ __forceinline__ void output_loss_body(const OutLossArgs& A, const int bx, const int gx) {
  const cv_bn& b = A.b;
  const float* __restrict__ y = A.y;
  const float* __restrict__ x = A.x;
  const int n = A.n, c = A.c, hw = A.hw;
  const FDiv fc = A.fc, fhw = A.fhw;
  float* __restrict__ xhat = A.xhat;
  double* rec_out = A.rec_out;
  float* __restrict__ dv = A.dv;
  double* gstat = A.gstat;
  const float* rec_scale = A.rec_scale;
  __shared__ BnFwdC k[OUT_MAXC];
  __shared__ double red[4][1 + 2 * OUT_MAXC];
  __shared__ double scratch[4 * 256];
  const int total = n * c * hw;
  const int base0 = bx * 256 * OL_U;
  float yv[OL_U], xv[OL_U];
  int nchw[OL_U], chs[OL_U];
  auto load = [&](int base) {
#pragma unroll
    for (int u = 0; u < OL_U; ++u) {
      const int i = base + u * 256 + threadIdx.x;
      yv[u] = 0.f;
      xv[u] = 0.f;
      nchw[u] = -1;
      chs[u] = 0;
      if (i < total) {
        const int pix = fc.div(i);  // img*hw + p
        const int ch = i - pix * c;
        const int img = fhw.div(pix);
        const int p = pix - img * hw;
        nchw[u] = (img * c + ch) * hw + p;
        chs[u] = ch;
        yv[u] = y[i];
        xv[u] = x[nchw[u]];
      }
    }
  };
  load(base0);  // (the first batch is requested before the BN fold: its latency overlaps the replica reads)
  bn_fold<256>(b, false, scratch, [&](int f, double s, double q, double, double) { k[f] = bn_fwd_const_s(b, f, s, q); });
  const float scale = (rec_scale ? rec_scale[0] : 1.0f) * 2.0f / (float)n;
  float rec = 0.f;
  float s1[OUT_MAXC], s2[OUT_MAXC];
#pragma unroll
  for (int j = 0; j < OUT_MAXC; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  for (int base = base0; base < total; base += gx * 256 * OL_U) {
    if (base != base0) load(base);
#pragma unroll
    for (int u = 0; u < OL_U; ++u) {
      if (nchw[u] < 0) continue;
      const int ch = chs[u];
      const BnFwdC kk = k[ch];
      const float v = bn_out(yv[u], kk);
      const float xh = 1.0f / (1.0f + expf(-v));
      const float diff = xh - xv[u];
      xhat[nchw[u]] = xh;
      rec = fmaf(diff, diff, rec);
      if (dv) {
        const float d = scale * diff * xh * (1.0f - xh);
        dv[base + u * 256 + threadIdx.x] = d;
#pragma unroll
        for (int j = 0; j < OUT_MAXC; ++j)
          if (j == ch) {
            s1[j] += d;
            s2[j] += d * ((yv[u] - kk.mu) * kk.istd);
          }
      }
    }
  }
  // block reduction (fp64 for the outputs)
  double vals[1 + 2 * OUT_MAXC];
  vals[0] = (double)rec;
#pragma unroll
  for (int j = 0; j < OUT_MAXC; ++j) { vals[1 + j] = (double)s1[j]; vals[1 + OUT_MAXC + j] = (double)s2[j]; }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 1 + 2 * OUT_MAXC; ++q) {
    double v = wave_sum(vals[q]);
    if (lane == 0) red[w][q] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double r = red[0][0] + red[1][0] + red[2][0] + red[3][0];
    atomic_add_f64(rec_out + bx % CV_REC_REPL, r / (double)n);
    if (dv) {
      const int repl = bx % CV_STAT_REPL(c);
      for (int j = 0; j < c; ++j) {
        const double a = red[0][1 + j] + red[1][1 + j] + red[2][1 + j] + red[3][1 + j];
        const double bb = red[0][1 + OUT_MAXC + j] + red[1][1 + OUT_MAXC + j] + red[2][1 + OUT_MAXC + j] +
                          red[3][1 + OUT_MAXC + j];
        atomic_add_f64(gstat + (size_t)repl * 2 * c + j, a);
        atomic_add_f64(gstat + (size_t)repl * 2 * c + c + j, bb);
      }
    }
  }
}

__global__ __launch_bounds__(256) void output_loss_kernel(const OutLossArgs A) { output_loss_body(A, blockIdx.x, gridDim.x); }

// The output loss with a queued NT-Xent gradient phase as extra workgroups of the same grid (cv_ntxent_aux; the
// fused step queues it before the last ConvTranspose2d, whose grid the image-side scatter fills): the roles
// alternate over the first 2 x min(nd, na) workgroups, as in cv_aux.hip.  Register-resident phase (d <= 8) only.
struct OlAuxMap {
  int nd, na, agx;
};
__global__ __launch_bounds__(256) void output_loss_aux_kernel(const OutLossArgs A, const NtArgs P, const OlAuxMap m) {
  const int v = blockIdx.x;
  const int k2 = m.nd < m.na ? m.nd : m.na;
  int role, idx;
  if (v < 2 * k2) {
    role = v & 1;
    idx = v >> 1;
  } else {
    role = m.nd > m.na ? 0 : 1;
    idx = k2 + (v - 2 * k2);
  }
  if (role == 0) output_loss_body(A, idx, m.nd);
  else ntxent_grad_reg_body<8, NTR_JM>(P, idx % m.agx, idx / m.agx);
}

__global__ __launch_bounds__(256) void output_bwd_kernel(const cv_bn b, const float* __restrict__ y,
                                                         const float* __restrict__ xhat,
                                                         const float* __restrict__ dxhat, int n, int c, int hw,
                                                         float* __restrict__ dv, double* gstat) {
  __shared__ float2 mi[OUT_MAXC];
  __shared__ double red[4][2 * OUT_MAXC];
  __shared__ double scratch[4 * 256];
  bn_fold<256>(b, false, scratch, [&](int f, double s, double q, double, double) {
    float m_, i_;
    bn_mean_istd_s(b, f, s, q, m_, i_);
    mi[f] = make_float2(m_, i_);
  });
  const long total = (long)n * c * hw;
  float s1[OUT_MAXC], s2[OUT_MAXC];
#pragma unroll
  for (int j = 0; j < OUT_MAXC; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int ch = (int)(i % c);
    const long pix = i / c;
    const long img = pix / hw;
    const int p = (int)(pix - img * hw);
    const long nchw = (img * c + ch) * hw + p;
    const float xh = xhat[nchw];
    const float d = dxhat[nchw] * xh * (1.0f - xh);
    dv[i] = d;
#pragma unroll
    for (int j = 0; j < OUT_MAXC; ++j)
      if (j == ch) {
        s1[j] += d;
        s2[j] += d * ((y[i] - mi[ch].x) * mi[ch].y);
      }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < OUT_MAXC; ++j) {
    double a = wave_sum((double)s1[j]), bb = wave_sum((double)s2[j]);
    if (lane == 0) { red[w][j] = a; red[w][OUT_MAXC + j] = bb; }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int repl = blockIdx.x % CV_STAT_REPL(c);
    for (int j = 0; j < c; ++j) {
      atomic_add_f64(gstat + (size_t)repl * 2 * c + j, red[0][j] + red[1][j] + red[2][j] + red[3][j]);
      atomic_add_f64(gstat + (size_t)repl * 2 * c + c + j,
                     red[0][OUT_MAXC + j] + red[1][OUT_MAXC + j] + red[2][OUT_MAXC + j] + red[3][OUT_MAXC + j]);
    }
  }
}

// BN1d(+ReLU) applied elementwise; the tensor is stored in the Unflatten/NHWC order.  Thread =
// one storage column (constants computed once), looping over a chunk of rows: coalesced rows.
constexpr int BA_ROWS = 32;
__global__ __launch_bounds__(256) void bn_apply_kernel(const cv_bn b, const float* __restrict__ x,
                                                       float* __restrict__ out, int rows, int F, int pix, int ch,
                                                       int relu) {
  const int col = blockIdx.x * 256 + threadIdx.x;  // storage position p*ch + c
  if (col >= F) return;
  const int f = (pix > 1) ? (col % ch) * pix + col / ch : col;  // PyTorch feature c*pix + p
  const BnFwdC k = bn_fwd_const(b, f);
  const int r0 = blockIdx.y * BA_ROWS;
  constexpr int U = 8;
  for (int rb = r0; rb < min(rows, r0 + BA_ROWS); rb += U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = (rb + u < rows) ? x[(size_t)(rb + u) * F + col] : 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (rb + u >= rows) break;
      const float o = bn_out(v[u], k);
      out[(size_t)(rb + u) * F + col] = relu ? fmaxf(o, 0.f) : o;
    }
  }
}

static int elem_grid(long total) {
  long g = (total + 255) / 256;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

// ---------------------------------------------------------------- decoder Linear -> BN1d backward
// (1) mask + BN1d backward sums: block = 64 features x 64 rows, fp64 atomics into 8 replicas;
// (2) dW[f][k] += sum_n BNbwd(dz)[n][f] * z[n][k]: block = 64 features x 64 rows staged in LDS.
constexpr int DL_F = 64;
constexpr int DL_R = 64;

// Both kernels walk the activation in its storage (Unflatten / NHWC) order so loads are coalesced;
// storage column col holds PyTorch feature f(col) = (col % ch) * pix + col / ch.
__device__ __forceinline__ int dl_feature(int col, int pix, int ch) {
  if (pix <= 1) return col;
  const int p = col / ch;
  return (col - p * ch) * pix + p;
}

constexpr int DL_RPT = DL_R / 4;  // rows per thread (4 row groups per block)

// The block's 64 storage columns map to features dl_feature(col) that are pix apart, so a per-thread
// replica fold would issue 2-4 uncoalesced fp64 loads per replica in every thread.  Instead the 4 row
// groups each fold every 4th replica of the 64 features and the partials meet in LDS (fixed order).
__device__ __forceinline__ void dl_fold(const cv_bn& b, bool bwd, int f, bool live, double (*part)[4][DL_F],
                                        BnFwdC* kf, BnBwdC* kb) {
  const int t = threadIdx.x, cl = t % DL_F, rg = t / DL_F;
  const int F = b.C, R = CV_STAT_REPL(F);
  double s = 0.0, q = 0.0, gs = 0.0, gq = 0.0;
  if (live && b.train)
    for (int r = rg; r < R; r += 4) {
      s += b.stat[(size_t)r * 2 * F + f];
      q += b.stat[(size_t)r * 2 * F + F + f];
      if (bwd) {
        gs += b.gstat[(size_t)r * 2 * F + f];
        gq += b.gstat[(size_t)r * 2 * F + F + f];
      }
    }
  part[0][rg][cl] = s;
  part[1][rg][cl] = q;
  part[2][rg][cl] = gs;
  part[3][rg][cl] = gq;
  __syncthreads();
  if (t < DL_F) {
    double S = 0.0, Q = 0.0, GS = 0.0, GQ = 0.0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      S += part[0][g][t];
      Q += part[1][g][t];
      GS += part[2][g][t];
      GQ += part[3][g][t];
    }
    if (live) {
      if (bwd) kb[t] = bn_bwd_const_s(b, f, S, Q, GS, GQ);
      else kf[t] = bn_fwd_const_s(b, f, S, Q);
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void declinear_mask_kernel(int n, int F, int pix, int ch, float* da,
                                                             const float* __restrict__ h, const cv_bn b,
                                                             double* gstat) {
  __shared__ float r1[4][DL_F], r2[4][DL_F];
  __shared__ int fidx[DL_F];
  __shared__ double part[4][4][DL_F];
  __shared__ BnFwdC kf[DL_F];
  const int t = threadIdx.x;
  const int c0 = blockIdx.x * DL_F, rbase = blockIdx.y * DL_R;
  const int cl = t % DL_F, rg = t / DL_F;
  const int col = c0 + cl;
  const int f = col < F ? dl_feature(col, pix, ch) : 0;
  float hv[DL_RPT], dv[DL_RPT];
#pragma unroll
  for (int i = 0; i < DL_RPT; ++i) {  // issue every load of the column slice first
    const int r = rbase + rg + 4 * i;
    hv[i] = 0.f;
    dv[i] = 0.f;
    if (col < F && r < n) {
      hv[i] = h[(size_t)r * F + col];
      dv[i] = da[(size_t)r * F + col];
    }
  }
  dl_fold(b, false, f, col < F, part, kf, nullptr);
  BnFwdC k;
  if (col < F) k = kf[cl];
  float s1 = 0.f, s2 = 0.f;
  if (col < F) {
#pragma unroll
    for (int i = 0; i < DL_RPT; ++i) {
      const int r = rbase + rg + 4 * i;
      if (r >= n) continue;
      float d = dv[i];
      if (bn_out(hv[i], k) <= 0.f) d = 0.f;
      da[(size_t)r * F + col] = d;
      s1 += d;
      s2 += d * ((hv[i] - k.mu) * k.istd);
    }
  }
  r1[rg][cl] = s1;
  r2[rg][cl] = s2;
  if (rg == 0) fidx[cl] = f;
  __syncthreads();
  if (t < DL_F && c0 + t < F) {
    const double a = (double)r1[0][t] + r1[1][t] + r1[2][t] + r1[3][t];
    const double q = (double)r2[0][t] + r2[1][t] + r2[2][t] + r2[3][t];
    const int repl = (blockIdx.y * gridDim.x + blockIdx.x) % CV_STAT_REPL(F);
    atomic_add_f64(gstat + (size_t)repl * 2 * F + fidx[t], a);
    atomic_add_f64(gstat + (size_t)repl * 2 * F + F + fidx[t], q);
  }
}

// dW[f][k] += sum_n BNbwd(dz)[n][f] * z[n][k].  One workgroup owns DW_F consecutive storage columns and
// reduces over ALL n rows itself (64-row chunks, the next chunk's loads in flight while the current one
// is contracted), so every weight-gradient element has one writer: no atomics, deterministic.  (The
// round-1 version split the rows over 8 workgroups and met in fp32 atomics on addresses `pix` features
// apart: 31 us at MNIST shape.)  thread t: column t % DW_F, row group / k group t / DW_F.
constexpr int DW_F = 16;
constexpr int DW_G = 256 / DW_F;          // 16 row groups (loads) / k groups (contraction)

// RPT rows per thread per chunk (chunk = DW_G * RPT rows): as many as the LDS images allow, so the whole
// batch arrives in one or two load rounds instead of one exposed latency per 64 rows
template <int KPT, int RPT>
__global__ __launch_bounds__(256) void declinear_wgrad_kernel(int n, int F, int K, int pix, int ch,
                                                              const float* __restrict__ dz,
                                                              const float* __restrict__ h, const cv_bn b,
                                                              const float* __restrict__ z, float* gw) {
  constexpr int DW_R = DW_G * RPT;
  __shared__ float sd[DW_R][DW_F + 1];
  __shared__ float sz[DW_R][DW_G * KPT + 1];
  __shared__ BnBwdC kbs[DW_F];
  const int t = threadIdx.x;
  const int c0 = blockIdx.x * DW_F;
  const int cl = t % DW_F, rg = t / DW_F;
  const int col = c0 + cl;
  const bool live = col < F;
  const int f = live ? dl_feature(col, pix, ch) : 0;
  constexpr int KW = DW_G * KPT;           // z columns staged per chunk (>= K)
  constexpr int ZPT = (DW_R * KW + 255) / 256;
  float dv[RPT], hv[RPT], zv[ZPT];
  auto fetch = [&](int r0) {
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int r = r0 + rg + DW_G * i;
      const bool ok = live && r < n;
      dv[i] = ok ? dz[(size_t)r * F + col] : 0.f;
      hv[i] = ok ? h[(size_t)r * F + col] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < ZPT; ++j) {
      const int e = t + 256 * j;
      const int rr = e / KW, kk = e - rr * KW;
      zv[j] = (e < DW_R * KW && r0 + rr < n && kk < K) ? z[(size_t)(r0 + rr) * K + kk] : 0.f;
    }
  };
  fetch(0);
  // BN1d backward constants of the block's columns (replica fold, one thread per column)
  if (t < DW_F) {
    double s = 0.0, q = 0.0, gs = 0.0, gq = 0.0;
    if (live) {
      bn_sums(b.stat, F, f, s, q);
      bn_sums(b.gstat, F, f, gs, gq);
      kbs[t] = bn_bwd_const_s(b, f, s, q, gs, gq);
    }
  }
  __syncthreads();
  BnBwdC kb;
  if (live) kb = kbs[cl];
  float acc[KPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) acc[j] = 0.f;
  for (int r0 = 0; r0 < n; r0 += DW_R) {
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int r = r0 + rg + DW_G * i;
      sd[rg + DW_G * i][cl] = (live && r < n) ? bn_bwd(dv[i], hv[i], kb) : 0.f;
    }
#pragma unroll
    for (int j = 0; j < ZPT; ++j) {
      const int e = t + 256 * j;
      if (e < DW_R * KW) sz[e / KW][e % KW] = zv[j];
    }
    __syncthreads();
    if (r0 + DW_R < n) fetch(r0 + DW_R);
    const int rmax = min(DW_R, n - r0);
    for (int rr = 0; rr < rmax; ++rr) {
      const float d = sd[rr][cl];
#pragma unroll
      for (int j = 0; j < KPT; ++j) acc[j] = fmaf(d, sz[rr][rg * KPT + j], acc[j]);
    }
    __syncthreads();
  }
  if (live) {
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
      const int kk = rg * KPT + j;
      if (kk < K) gw[(size_t)f * K + kk] += acc[j];
    }
  }
}

// ---------------------------------------------------------------- end-of-backward reduction (cv_step_reduce)
// One launch for everything between the last backward GEMM and the optimizer: the split-K partial tiles of
// every deferred weight gradient (summed in fixed split order: one writer per element, deterministic), the
// BatchNorm affine gradients from the backward sums, and the running statistics from the forward sums.
// Replaces one wgrad_reduce launch per weight gradient, cv_bn_param_grads (x2) and cv_bn_update_running.
constexpr int MAX_DEFER = 24;
constexpr int MAX_PLAIN = 32;
constexpr int SR_PLAIN = 1024;  // arena elements per Adam block of the plain ranges
struct StepRedArgs {
  cv_wgrad_defer d[MAX_DEFER];
  int blk0[MAX_DEFER + 1];  // prefix sums of the reduction blocks of each deferred gradient
  int nd;
  cv_bn bn[MAX_BN];
  float* dg[MAX_BN];
  float* db[MAX_BN];
  int64_t* nbt[MAX_BN];
  int nbn, grads, running;
  int bnblk0[MAX_BN + 1];  // prefix sums of the blocks of each BN layer (wide layers: 256 channels per block)
  float momentum;
  // fused Adam (cv_step_reduce_adam; ap == nullptr: off).  Every gradient this launch finalises is stepped
  // where it is produced; the rest of the arena lies in the plain ranges [plain0, plain0 + plainn), stepped
  // by the trailing blocks (pblk0: prefix sums of their blocks)
  float* ap;
  float* ag;
  float* am;
  float* av;
  const float* hyper;
  int64_t* step;
  int64_t* aux;
  long plain0[MAX_PLAIN];
  int plainn[MAX_PLAIN];
  int pblk0[MAX_PLAIN + 1];
  int nplain;
  int nprod;  // blocks that reduce the deferred segments (grid-stride over blk0[nd] segments)
};
#ifndef CV_SR_E
#define CV_SR_E 64
#endif
// partial-tile elements per block (256-byte row segments), each summed by SR_G thread groups over every SR_G-th
// split.  64 (4 groups): MNIST step 0.4972 -> 0.4942 ms (the reduction 20.5 -> 17.6 us in-step), CelebA 2.1216 ->
// 2.1179 ms against 128 (2 groups); 32 (8 groups) lost on CelebA (2.137 ms).  -DCV_SR_E= rebuilds (A/B).
constexpr int SR_E = CV_SR_E;
constexpr int SR_G = 256 / SR_E;   // split groups per element (each thread sums every SR_G-th split)

// torch.optim.Adam (foreach) on one element of the arena, constants from adam_consts
struct AdamC {
  float step_size, bc2s, omb1, omb2, b2, eps, wd;
};
__device__ __forceinline__ AdamC adam_consts(const float* hyper, int64_t step0) {
  const long t_step = step0 + 1;
  const double b1 = hyper[1], b2 = hyper[2];
  const double bc1 = 1.0 - pow(b1, (double)t_step);
  const double bc2 = 1.0 - pow(b2, (double)t_step);
  AdamC c;
  c.step_size = (float)(-(double)hyper[0] / bc1);
  c.bc2s = (float)sqrt(bc2);
  c.omb1 = (float)(1.0 - b1);
  c.omb2 = (float)(1.0 - b2);
  c.b2 = hyper[2];
  c.eps = hyper[3];
  c.wd = hyper[4];
  return c;
}
__device__ __forceinline__ void adam_elem(const StepRedArgs& a, const AdamC& c, long i, float g) {
  float pp = a.ap[i], mm = a.am[i], vv = a.av[i];
  if (c.wd != 0.f) g = g + c.wd * pp;
  mm = mm + c.omb1 * (g - mm);
  vv = vv * c.b2 + c.omb2 * g * g;
  const float den = sqrtf(vv) / c.bc2s + c.eps;
  a.ap[i] = pp + c.step_size * (mm / den);
  a.am[i] = mm;
  a.av[i] = vv;
}

__device__ __forceinline__ void defer_segment(const StepRedArgs& a, const AdamC& ac, bool adam, int b, int t,
                                              float (*red)[SR_E + 1]) {
  {
    int di = 0;
    while (di + 1 < a.nd && b >= a.blk0[di + 1]) ++di;
    const cv_wgrad_defer& d = a.d[di];
    const int ol = t % SR_E, zg = t / SR_E;
    const long o = (long)(b - a.blk0[di]) * SR_E + ol;
    const long total = (long)d.M * d.ntot;
    const size_t sstride = (size_t)total;
    // the destination of this thread's element (threads < SR_E) is resolved and its current value
    // requested first, so the read-modify-write costs no extra latency after the reduction
    float* dst = nullptr;
    float old = 0.f;
    if (t < SR_E && o < total) {
      const int row = (int)(o / d.ntot), col = (int)(o - (long)row * d.ntot);
      if (col < d.N) {
        const int tap = col / d.cb, c = col - tap * d.cb;
        dst = d.gweight + ((size_t)row * d.cb + c) * d.kk + tap;
      } else if (d.gbias) {
        dst = d.gbias + row;
      }
      if (dst) old = *dst;
    }
    float acc = 0.f;
    if (o < total) {
      const float* p = d.part + o;
      int z = zg;
      for (; z + 7 * SR_G < d.split; z += 8 * SR_G) {  // 8 independent loads in flight per thread
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = p[(size_t)(z + u * SR_G) * sstride];
        acc += ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
      }
      // the < 8 remaining slices: every load issued before the first add (the adds keep the serial order;
      // absent slices add an exact 0)
      float v[7];
#pragma unroll
      for (int u = 0; u < 7; ++u) {
        const int zz = z + u * SR_G;
        v[u] = (zz < d.split) ? p[(size_t)zz * sstride] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 7; ++u) acc += v[u];
    }
    red[zg][ol] = acc;
    __syncthreads();
    if (dst) {
      float v = 0.f;
#pragma unroll
      for (int g = 0; g < SR_G; ++g) v += red[g][t];  // fixed order: deterministic
      const float g = old + v;
      *dst = g;
      if (adam) adam_elem(a, ac, dst - a.ag, g);
    }
    __syncthreads();  // (red is reused by the block's next segment)
  }
}

__device__ __forceinline__ void step_reduce_body(const StepRedArgs& a, const AdamC& ac, bool adam, int b, int t,
                                                 float (*red)[SR_E + 1], double* scratch) {
  if (b < a.nprod) {  // deferred weight gradients: segments of 64 partial-tile elements, grid-stride
    for (int sgm = b; sgm < a.blk0[a.nd]; sgm += a.nprod) defer_segment(a, ac, adam, sgm, t, red);
    return;
  }
  const int lb = b - a.nprod;
  if (lb >= a.bnblk0[a.nbn]) {  // fused Adam over a plain range of the arena
    const int pb = lb - a.bnblk0[a.nbn];
    if (!adam || pb >= a.pblk0[a.nplain]) return;
    int r = 0;
    while (r + 1 < a.nplain && pb >= a.pblk0[r + 1]) ++r;
    const long i0 = a.plain0[r] + (long)(pb - a.pblk0[r]) * SR_PLAIN;
    const long i1 = min(a.plain0[r] + (long)a.plainn[r], i0 + SR_PLAIN);
    for (long i = i0 + t; i < i1; i += 256) adam_elem(a, ac, i, a.ag[i]);
    return;
  }
  int l = 0;
  while (l + 1 < a.nbn && lb >= a.bnblk0[l + 1]) ++l;
  const int chunk = lb - a.bnblk0[l];
  const cv_bn& bn = a.bn[l];
  if (bn.C >= 256) {  // wide layers (the BN1d's 2048 features): one channel per thread, 256 channels per block,
    // the same per-channel replica folds as bn_fold's one-channel-per-thread path
    const int c = chunk * 256 + t;
    if (a.running && t == 0 && chunk == 0 && a.nbt[l]) a.nbt[l][0] += 1;
    if (c >= bn.C) return;
    if (a.grads) {
      double s1 = 0.0, s2 = 0.0;
      if (bn.train) bn_sums(bn.gstat, bn.C, c, s1, s2);
      float* dg = a.dg[l];
      float* db = a.db[l];
      if (db) {
        db[c] = (float)s1;
        if (adam) adam_elem(a, ac, db + c - a.ag, (float)s1);
      }
      if (dg) {
        dg[c] = (float)s2;
        if (adam) adam_elem(a, ac, dg + c - a.ag, (float)s2);
      }
    }
    if (a.running) {
      double s1 = 0.0, q = 0.0;
      if (bn.train) bn_sums(bn.stat, bn.C, c, s1, q);
      const double n = (double)bn.count;
      const double mean = s1 / n;
      double var = q / n - mean * mean;
      if (var < 0.0) var = 0.0;
      const double unbiased = (bn.count > 1) ? var * n / (n - 1.0) : var;
      float* rm = const_cast<float*>(bn.running_mean);
      float* rv = const_cast<float*>(bn.running_var);
      rm[c] = a.momentum * (float)mean + (1.0f - a.momentum) * rm[c];
      rv[c] = a.momentum * (float)unbiased + (1.0f - a.momentum) * rv[c];
    }
    return;
  }
  if (a.grads) {  // dgamma = sum dz*xhat, dbeta = sum dz (the backward sums)
    cv_bn gb = bn;
    gb.stat = bn.gstat;
    float* dg = a.dg[l];
    float* db = a.db[l];
    bn_fold<256>(gb, false, scratch, [&](int c, double s1, double s2, double, double) {
      if (db) {
        db[c] = (float)s1;
        if (adam) adam_elem(a, ac, db + c - a.ag, (float)s1);
      }
      if (dg) {
        dg[c] = (float)s2;
        if (adam) adam_elem(a, ac, dg + c - a.ag, (float)s2);
      }
    });
  }
  if (a.running) {  // running statistics, momentum update with the unbiased batch variance
    if (t == 0 && a.nbt[l]) a.nbt[l][0] += 1;
    float* rm = const_cast<float*>(bn.running_mean);
    float* rv = const_cast<float*>(bn.running_var);
    const float m = a.momentum;
    bn_fold<256>(bn, false, scratch, [&](int c, double s1, double q, double, double) {
      const double n = (double)bn.count;
      const double mean = s1 / n;
      double var = q / n - mean * mean;
      if (var < 0.0) var = 0.0;
      const double unbiased = (bn.count > 1) ? var * n / (n - 1.0) : var;
      rm[c] = m * (float)mean + (1.0f - m) * rm[c];
      rv[c] = m * (float)unbiased + (1.0f - m) * rv[c];
    });
  }
}

__global__ __launch_bounds__(256) void step_reduce_kernel(const StepRedArgs a) {
  __shared__ float red[SR_G][SR_E + 1];
  __shared__ double scratch[4 * 256];
  __shared__ AdamC acs;
  __shared__ int last;
  const int b = blockIdx.x, t = threadIdx.x;
  const bool adam = a.ap != nullptr;
  if (adam) {
    if (t == 0) acs = adam_consts(a.hyper, a.step[0]);  // every block reads step[0] before its ticket
    __syncthreads();
  }
  const AdamC ac = adam ? acs : AdamC{};
  step_reduce_body(a, ac, adam, b, t, red, scratch);
  if (adam) {  // the last block to arrive advances the step (and annealer) counters: arrivals counted in two
    __syncthreads();  // levels (64 group words step[2..65], then step[1]) so blocks do not serialise on one word
    if (t == 0) {
      const unsigned nblk = gridDim.x, gsz = (nblk + 63) / 64, ngrp = (nblk + gsz - 1) / gsz, grp = b / gsz;
      const unsigned gcnt = (grp + 1 == ngrp) ? nblk - grp * gsz : gsz;
      unsigned long long* gw = reinterpret_cast<unsigned long long*>(a.step + 2 + grp);
      last = 0;
      if (atomicAdd(gw, 1ull) == gcnt - 1) {
        *gw = 0;
        last = atomicAdd((unsigned long long*)(a.step + 1), 1ull) == ngrp - 1;
      }
    }
    __syncthreads();
    if (last && t == 0) {
      a.step[0] += 1;
      a.step[1] = 0;
      if (a.aux) a.aux[0] += 1;
    }
  }
}

// ---------------------------------------------------------------- multi-buffer zero
struct ZeroArgs {
  uint32_t* p[8];
  long words[8];
  long start[9];  // prefix sums of words
  int count;
};

__global__ __launch_bounds__(256) void zero_many_kernel(const ZeroArgs z) {
  const long total = z.start[z.count];
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    int b = 0;
#pragma unroll
    for (int q = 1; q < 8; ++q)
      if (q < z.count && i >= z.start[q]) b = q;
    z.p[b][i - z.start[b]] = 0u;
  }
}

struct CopyArgs {
  uint32_t* dst[8];
  const uint32_t* src[8];
  long start[9];  // prefix sums of the 4-byte word counts
  int count;
};

__global__ __launch_bounds__(256) void copy_many_kernel(const CopyArgs c) {
  const long total = c.start[c.count];
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    int b = 0;
#pragma unroll
    for (int q = 1; q < 8; ++q)
      if (q < c.count && i >= c.start[q]) b = q;
    c.dst[b][i - c.start[b]] = c.src[b][i - c.start[b]];
  }
}

}  // namespace cv

using namespace cv;

// 16-byte form (every buffer 16-byte aligned and sized): a quarter of the instructions for the step's batch copy
__global__ __launch_bounds__(256) void copy_many4_kernel(const CopyArgs c) {
  const long total = c.start[c.count];  // (units of 16 bytes here)
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    int b = 0;
#pragma unroll
    for (int q = 1; q < 8; ++q)
      if (q < c.count && i >= c.start[q]) b = q;
    reinterpret_cast<uint4*>(c.dst[b])[i - c.start[b]] = reinterpret_cast<const uint4*>(c.src[b])[i - c.start[b]];
  }
}

extern "C" int cv_copy_many(void* const* dst, const void* const* src, const size_t* bytes, int count,
                            cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(dst && src && bytes && count > 0 && count <= 8, "copy_many: 1..8 buffers");
  CopyArgs c;
  memset(&c, 0, sizeof(c));
  c.count = count;
  for (int i = 0; i < count; ++i) {
    CV_REQUIRE(dst[i] && src[i] && bytes[i] % 4 == 0 && ((uintptr_t)dst[i] | (uintptr_t)src[i]) % 4 == 0,
               "copy_many: buffer %d not 4-byte granular", i);
    c.dst[i] = (uint32_t*)dst[i];
    c.src[i] = (const uint32_t*)src[i];
    c.start[i + 1] = c.start[i] + (long)(bytes[i] / 4);
  }
  bool v16 = true;
  for (int i = 0; i < count; ++i)
    v16 = v16 && bytes[i] % 16 == 0 && ((uintptr_t)dst[i] | (uintptr_t)src[i]) % 16 == 0;
  if (v16) {
    for (int i = 0; i <= count; ++i) c.start[i] /= 4;
    long g = (c.start[count] + 255) / 256;
    if (g > 2048) g = 2048;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(copy_many4_kernel, dim3((int)g), dim3(256), 0, S(stream), c);
    CV_LAUNCH_CHECK("copy_many");
    return 0;
  }
  long g = (c.start[count] + 255) / 256;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(copy_many_kernel, dim3((int)g), dim3(256), 0, S(stream), c);
  CV_LAUNCH_CHECK("copy_many");
  return 0;
}

extern "C" int cv_zero_many(void* const* ptrs, const size_t* bytes, int count, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(ptrs && bytes && count > 0 && count <= 8, "zero_many: 1..8 buffers");
  ZeroArgs z;
  memset(&z, 0, sizeof(z));
  z.count = count;
  for (int i = 0; i < count; ++i) {
    CV_REQUIRE(ptrs[i] && bytes[i] % 4 == 0 && (uintptr_t)ptrs[i] % 4 == 0, "zero_many: buffer %d not 4-byte granular", i);
    z.p[i] = (uint32_t*)ptrs[i];
    z.words[i] = (long)(bytes[i] / 4);
    z.start[i + 1] = z.start[i] + z.words[i];
  }
  long g = (z.start[count] + 255) / 256;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(zero_many_kernel, dim3((int)g), dim3(256), 0, S(stream), z);
  CV_LAUNCH_CHECK("zero_many");
  return 0;
}

extern "C" int cv_bn_update_running(const cv_bn* bn, int nlayers, float momentum, int64_t* const* nbt,
                                    cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(bn && nlayers > 0 && nlayers <= MAX_BN, "bn_update_running: 1..%d layers", MAX_BN);
  RunArgs a;
  memset(&a, 0, sizeof(a));
  int cmax = 0;
  for (int i = 0; i < nlayers; ++i) {
    CV_REQUIRE(bn[i].stat && bn[i].running_mean && bn[i].running_var && bn[i].C > 0 && bn[i].count > 0,
               "bn_update_running: layer %d incomplete", i);
    a.bn[i] = bn[i];
    a.nbt[i] = nbt ? nbt[i] : nullptr;
    cmax = bn[i].C > cmax ? bn[i].C : cmax;
  }
  a.nl = nlayers;
  a.momentum = momentum;
  hipLaunchKernelGGL(bn_running_kernel, dim3(cdiv(cmax, 256), nlayers), dim3(256), 0, S(stream), a);
  CV_LAUNCH_CHECK("bn_update_running");
  return 0;
}

// Several forwards' momentum updates of the same layers in one launch, in order (CLEAR-MIM's five estimator forwards,
// trainer.py:873-888: each `vae(X)` moves every BatchNorm's running statistics once): set s of layer l folds its own
// batch sums; the thread (block) that owns a channel applies the sets one after the other.
constexpr int MAX_SETS = 8;
struct RunSetArgs {
  cv_bn bn[MAX_BN];
  const double* stat[MAX_SETS][MAX_BN];
  int64_t* nbt[MAX_BN];
  int nl, nsets;
  float momentum;
};
__global__ __launch_bounds__(256) void bn_running_sets_kernel(const RunSetArgs a) {
  __shared__ double scratch[4 * 256];
  const int l = blockIdx.y;
  if (l >= a.nl) return;
  cv_bn b = a.bn[l];
  float* rm = const_cast<float*>(b.running_mean);
  float* rv = const_cast<float*>(b.running_var);
  const float m = a.momentum;
  auto update = [&](int c, double s, double q, double, double) {
    const double n = (double)b.count;
    const double mean = s / n;
    double var = q / n - mean * mean;
    if (var < 0.0) var = 0.0;
    const double unbiased = (b.count > 1) ? var * n / (n - 1.0) : var;
    rm[c] = m * (float)mean + (1.0f - m) * rm[c];
    rv[c] = m * (float)unbiased + (1.0f - m) * rv[c];
  };
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.nbt[l]) a.nbt[l][0] += a.nsets;
  if (b.C >= 256) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c < b.C)
      for (int st = 0; st < a.nsets; ++st) {
        double s = 0.0, q = 0.0;
        bn_sums(a.stat[st][l], b.C, c, s, q);
        update(c, s, q, 0.0, 0.0);
      }
    return;
  }
  if (blockIdx.x != 0) return;
  for (int st = 0; st < a.nsets; ++st) {
    b.stat = a.stat[st][l];
    bn_fold<256>(b, false, scratch, update);
    __syncthreads();
  }
}

extern "C" int cv_bn_update_running_sets(const cv_bn* bn, int nlayers, int nsets, float momentum,
                                         int64_t* const* nbt, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(bn && nlayers > 0 && nlayers <= MAX_BN && nsets > 0 && nsets <= MAX_SETS,
             "bn_update_running_sets: 1..%d layers x 1..%d sets", MAX_BN, MAX_SETS);
  RunSetArgs a;
  memset(&a, 0, sizeof(a));
  int cmax = 0;
  for (int i = 0; i < nlayers; ++i) {
    for (int st = 0; st < nsets; ++st) {
      const cv_bn& x = bn[st * nlayers + i];
      CV_REQUIRE(x.stat && x.running_mean && x.running_var && x.C > 0 && x.count > 0,
                 "bn_update_running_sets: layer %d of set %d incomplete", i, st);
      CV_REQUIRE(x.running_mean == bn[i].running_mean && x.running_var == bn[i].running_var && x.C == bn[i].C &&
                     x.count == bn[i].count,
                 "bn_update_running_sets: set %d's layer %d is another BatchNorm", st, i);
      a.stat[st][i] = x.stat;
    }
    a.bn[i] = bn[i];
    a.nbt[i] = nbt ? nbt[i] : nullptr;
    cmax = bn[i].C > cmax ? bn[i].C : cmax;
  }
  a.nl = nlayers;
  a.nsets = nsets;
  a.momentum = momentum;
  hipLaunchKernelGGL(bn_running_sets_kernel, dim3(cdiv(cmax, 256), nlayers), dim3(256), 0, S(stream), a);
  CV_LAUNCH_CHECK("bn_update_running_sets");
  return 0;
}

extern "C" int cv_bn_apply(const cv_bn* bn, const float* x, float* out, int rows, int features, int pix, int ch,
                           int relu, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(bn && x && out && rows > 0 && features > 0 && bn->C == features, "bn_apply: bad args");
  CV_REQUIRE(pix <= 1 || pix * ch == features, "bn_apply: pix*ch != features");
  hipLaunchKernelGGL(bn_apply_kernel, dim3(cdiv(features, 256), cdiv(rows, BA_ROWS)), dim3(256), 0, S(stream), *bn,
                     x, out, rows, features, pix, ch, relu);
  CV_LAUNCH_CHECK("bn_apply");
  return 0;
}

extern "C" int cv_bn_param_grads(const cv_bn* bn, int nlayers, float* const* dgamma, float* const* dbeta,
                                 cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(bn && nlayers > 0 && nlayers <= MAX_BN && dgamma && dbeta, "bn_param_grads: 1..%d layers", MAX_BN);
  GradArgs a;
  memset(&a, 0, sizeof(a));
  int cmax = 0;
  for (int i = 0; i < nlayers; ++i) {
    CV_REQUIRE(bn[i].gstat && bn[i].C > 0, "bn_param_grads: layer %d incomplete", i);
    a.bn[i] = bn[i];
    a.dg[i] = dgamma[i];
    a.db[i] = dbeta[i];
    cmax = bn[i].C > cmax ? bn[i].C : cmax;
  }
  a.nl = nlayers;
  hipLaunchKernelGGL(bn_grads_kernel, dim3(1, nlayers), dim3(256), 0, S(stream), a);
  CV_LAUNCH_CHECK("bn_param_grads");
  return 0;
}

extern "C" int cv_bn_batch_stats(const cv_bn* bn, float* mean, float* invstd, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(bn && mean && invstd && bn->C > 0, "bn_batch_stats: bad args");
  hipLaunchKernelGGL(bn_stats_kernel, dim3(cdiv(bn->C, 256)), dim3(256), 0, S(stream), *bn, mean, invstd);
  CV_LAUNCH_CHECK("bn_batch_stats");
  return 0;
}

extern "C" int cv_output_forward(const cv_bn* bn, const float* y, int n, int c, int hw, float* xhat,
                                 cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(bn && y && xhat && n > 0 && c > 0 && c <= OUT_MAXC && hw > 0, "output_forward: bad args (C<=%d)",
             OUT_MAXC);
  CV_REQUIRE(bn->C == c, "output_forward: BN width %d != %d", bn->C, c);
  hipLaunchKernelGGL(output_fwd_kernel, dim3(elem_grid((long)n * c * hw)), dim3(256), 0, S(stream), *bn, y, n, c, hw,
                     xhat);
  CV_LAUNCH_CHECK("output_forward");
  return 0;
}

extern "C" int cv_output_loss(const cv_bn* bn, const float* y, const float* x, int n, int c, int hw, float* xhat,
                              double* rec_out, float* dv_out, double* gstat_out, const float* rec_scale,
                              cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(bn && y && x && xhat && rec_out && n > 0 && c > 0 && c <= OUT_MAXC && hw > 0,
             "output_loss: bad args (C<=%d)", OUT_MAXC);
  CV_REQUIRE(bn->C == c, "output_loss: BN width %d != %d", bn->C, c);
  CV_REQUIRE(!dv_out || gstat_out, "output_loss: dv needs gstat_out");
  CV_REQUIRE((long)n * c * hw < (1L << 31), "output_loss: tensor too large");
  long g = ((long)n * c * hw + 256 * OL_U - 1) / (256 * OL_U);
  if (g > 512) g = 512;
  const OutLossArgs A{*bn, y, x, n, c, hw, FDiv::make(c), FDiv::make(hw), xhat, rec_out, dv_out, gstat_out, rec_scale};
  // a queued NT-Xent gradient phase rides in this grid where served (cv_ntxent_aux; else it stays queued for its
  // flush)
  if (g_aux.set && g_aux.stream == S(stream) && g_aux.phase == 1 && aux_enabled() && g_aux.a.d <= 8 &&
      !g_aux.a.with_combine &&
      ntxent_reg_ok(g_aux.a, g_aux.a.nbr)) {
    const NtArgs P = g_aux.a;
    const int agx = (P.n + P.rpb - 1) / P.rpb;
    const OlAuxMap m{(int)g, agx * P.nbr, agx};
    g_aux.set = 0;
    note_launch((const void*)output_loss_aux_kernel);
    hipLaunchKernelGGL(output_loss_aux_kernel, dim3((unsigned)(m.nd + m.na)), dim3(256), 0, S(stream), A, P, m);
    aux_count_merged();
    CV_LAUNCH_CHECK("output_loss + NT-Xent");
    return 0;
  }
  hipLaunchKernelGGL(output_loss_kernel, dim3((int)g), dim3(256), 0, S(stream), A);
  CV_LAUNCH_CHECK("output_loss");
  return 0;
}

extern "C" int cv_output_backward(const cv_bn* bn, const float* y, const float* xhat, const float* dxhat, int n,
                                  int c, int hw, float* dv_out, double* gstat_out, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(bn && y && xhat && dxhat && dv_out && gstat_out && n > 0 && c > 0 && c <= OUT_MAXC && hw > 0,
             "output_backward: bad args");
  hipLaunchKernelGGL(output_bwd_kernel, dim3(elem_grid((long)n * c * hw)), dim3(256), 0, S(stream), *bn, y, xhat,
                     dxhat, n, c, hw, dv_out, gstat_out);
  CV_LAUNCH_CHECK("output_backward");
  return 0;
}

extern "C" int cv_declinear_backward_weight(const cv_linear* g, float* da, const float* h, const cv_bn* bn,
                                            double* gstat_out, const float* zin, float* gweight, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(g && da && h && bn && (gstat_out || gweight), "declinear_backward_weight: null args");
  CV_REQUIRE(!gweight || zin, "declinear_backward_weight: the weight gradient needs z");
  CV_REQUIRE(g->in_features <= 128, "declinear_backward_weight: latent width %d > 128", g->in_features);
  CV_REQUIRE(bn->C == g->out_features && bn->train, "declinear_backward_weight: BN1d must be train-mode, C=out");
  const int pix = g->out_pix > 0 ? g->out_pix : 1;
  const int F = g->out_features, K = g->in_features;
  dim3 grid(cdiv(F, DL_F), cdiv(g->n, DL_R));
  if (gstat_out) {  // mask + BN1d backward sums
    hipLaunchKernelGGL(declinear_mask_kernel, grid, dim3(256), 0, S(stream), g->n, F, pix, g->out_ch, da, h, *bn,
                       gstat_out);
    CV_LAUNCH_CHECK("declinear_mask");
  }
  if (!gweight) return 0;
  cv_bn b2 = *bn;
  if (gstat_out) b2.gstat = gstat_out;  // (else: da already masked, bn->gstat complete)
  CV_REQUIRE(b2.gstat != nullptr, "declinear_backward_weight: BN1d backward sums missing");
  const dim3 wgrid(cdiv(F, DW_F));
#define CV_DW(KPT_, RPT_)                                                                                     \
  hipLaunchKernelGGL((declinear_wgrad_kernel<KPT_, RPT_>), wgrid, dim3(256), 0, S(stream), g->n, F, K, pix, g->out_ch, \
                     da, h, b2, zin, gweight)
  // (static LDS <= 40 KB: chunk rows x (DW_F + 16 KPT + 2) floats)
  if (K <= DW_G) CV_DW(1, 16);
  else if (K <= 2 * DW_G) CV_DW(2, 12);
  else if (K <= 4 * DW_G) CV_DW(4, 8);
  else CV_DW(8, 4);
#undef CV_DW
  CV_LAUNCH_CHECK("declinear_wgrad");
  return 0;
}

static int step_reduce_launch(const cv_wgrad_defer* defers, int ndefer, const cv_bn* bn, int nbn,
                              float* const* dgamma, float* const* dbeta, int running, float momentum,
                              int64_t* const* nbt, const float* adam_arena[4], int64_t numel, const float* hyper,
                              int64_t* step, int64_t* aux, cv_stream_t stream);

extern "C" int cv_step_reduce(const cv_wgrad_defer* defers, int ndefer, const cv_bn* bn, int nbn, float* const* dgamma,
                              float* const* dbeta, int running, float momentum, int64_t* const* nbt,
                              cv_stream_t stream) {
  clear_error();
  return step_reduce_launch(defers, ndefer, bn, nbn, dgamma, dbeta, running, momentum, nbt, nullptr, 0, nullptr,
                            nullptr, nullptr, stream);
}

extern "C" int cv_step_reduce_adam(const cv_wgrad_defer* defers, int ndefer, const cv_bn* bn, int nbn,
                                   float* const* dgamma, float* const* dbeta, int running, float momentum,
                                   int64_t* const* nbt, float* params, float* grads, float* exp_avg, float* exp_avg_sq,
                                   int64_t numel, const float* hyper, int64_t* step, int64_t* aux_counter,
                                   cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(params && grads && exp_avg && exp_avg_sq && hyper && step && numel > 0, "step_reduce_adam: bad arena");
  const float* arena[4] = {params, grads, exp_avg, exp_avg_sq};
  return step_reduce_launch(defers, ndefer, bn, nbn, dgamma, dbeta, running, momentum, nbt, arena, numel, hyper,
                            step, aux_counter, stream);
}

static int step_reduce_launch(const cv_wgrad_defer* defers, int ndefer, const cv_bn* bn, int nbn,
                              float* const* dgamma, float* const* dbeta, int running, float momentum,
                              int64_t* const* nbt, const float* adam_arena[4], int64_t numel, const float* hyper,
                              int64_t* step, int64_t* aux, cv_stream_t stream) {
  CV_REQUIRE(ndefer >= 0 && ndefer <= MAX_DEFER && nbn >= 0 && nbn <= MAX_BN, "step_reduce: <= %d gradients, <= %d BN layers",
             MAX_DEFER, MAX_BN);
  CV_REQUIRE(ndefer == 0 || defers, "step_reduce: null defer list");
  CV_REQUIRE(nbn == 0 || bn, "step_reduce: null BN list");
  StepRedArgs a;
  memset(&a, 0, sizeof(a));
  int nb = 0;
  for (int i = 0; i < ndefer; ++i) {
    const cv_wgrad_defer& d = defers[i];
    a.blk0[a.nd] = nb;
    if (d.split <= 0) continue;  // that weight gradient was written directly
    CV_REQUIRE(d.part && d.gweight && d.M > 0 && d.ntot > 0 && d.N <= d.ntot && d.cb > 0 && d.kk > 0,
               "step_reduce: deferred gradient %d incomplete", i);
    a.d[a.nd] = d;
    nb += cdiv((long)d.M * d.ntot, SR_E);
    ++a.nd;
  }
  a.blk0[a.nd] = nb;
  for (int i = 0; i < nbn; ++i) {
    CV_REQUIRE(bn[i].C > 0 && bn[i].count > 0, "step_reduce: BN layer %d incomplete", i);
    CV_REQUIRE(!dgamma || bn[i].gstat, "step_reduce: BN layer %d has no backward sums", i);
    CV_REQUIRE(!running || (bn[i].stat && bn[i].running_mean && bn[i].running_var),
               "step_reduce: BN layer %d has no forward sums / running buffers", i);
    a.bn[i] = bn[i];
    a.dg[i] = dgamma ? dgamma[i] : nullptr;
    a.db[i] = dbeta ? dbeta[i] : nullptr;
    a.nbt[i] = nbt ? nbt[i] : nullptr;
  }
  a.nbn = nbn;
  for (int i = 0; i < nbn; ++i) a.bnblk0[i + 1] = a.bnblk0[i] + (bn[i].C >= 256 ? cdiv(bn[i].C, 256) : 1);
  a.grads = (dgamma || dbeta) ? 1 : 0;
  a.running = running;
  a.momentum = momentum;
  // without Adam every segment has its own block (no arrival ticket); with it the segments are shared by at most
  // 2048 blocks so the ticket stays cheap
  a.nprod = adam_arena ? (nb < 2048 ? nb : 2048) : nb;
  int blocks = a.nprod + a.bnblk0[nbn];
  if (adam_arena) {
    // the gradient ranges this launch finalises (steps them itself); the complement is stepped by plain blocks
    const float* g0 = adam_arena[1];
    struct Iv { long lo, hi; };
    Iv iv[3 * MAX_DEFER + 2 * MAX_BN];
    int niv = 0;
    auto cover = [&](const float* p, long n) -> int {
      if (!p || n <= 0) return 0;
      const long lo = (long)(p - g0);
      CV_REQUIRE(lo >= 0 && lo + n <= numel, "step_reduce_adam: a reduced gradient lies outside the arena");
      iv[niv++] = {lo, lo + n};
      return 0;
    };
    for (int i = 0; i < a.nd; ++i) {
      const cv_wgrad_defer& d = a.d[i];
      if (cover(d.gweight, (long)d.M * d.cb * d.kk)) return 1;
      if (d.ntot > d.N && cover(d.gbias, d.M)) return 1;
    }
    for (int i = 0; i < nbn; ++i) {
      if (a.grads && cover(a.dg[i], a.bn[i].C)) return 1;
      if (a.grads && cover(a.db[i], a.bn[i].C)) return 1;
    }
    for (int i = 1; i < niv; ++i)  // insertion sort by start
      for (int j = i; j > 0 && iv[j].lo < iv[j - 1].lo; --j) {
        const Iv tmp = iv[j];
        iv[j] = iv[j - 1];
        iv[j - 1] = tmp;
      }
    long pos = 0;
    int pb = 0;
    auto plain = [&](long lo, long hi) -> int {
      while (lo < hi) {
        CV_REQUIRE(a.nplain < MAX_PLAIN, "step_reduce_adam: more than %d plain ranges", MAX_PLAIN);
        const long n = hi - lo < (1L << 30) ? hi - lo : (1L << 30);
        a.plain0[a.nplain] = lo;
        a.plainn[a.nplain] = (int)n;
        a.pblk0[a.nplain] = pb;
        pb += (int)((n + SR_PLAIN - 1) / SR_PLAIN);
        ++a.nplain;
        lo += n;
      }
      return 0;
    };
    for (int i = 0; i < niv; ++i) {
      CV_REQUIRE(iv[i].lo >= pos, "step_reduce_adam: overlapping reduced gradients");
      if (plain(pos, iv[i].lo)) return 1;
      pos = iv[i].hi;
    }
    if (plain(pos, numel)) return 1;
    a.pblk0[a.nplain] = pb;
    a.ap = const_cast<float*>(adam_arena[0]);
    a.ag = const_cast<float*>(adam_arena[1]);
    a.am = const_cast<float*>(adam_arena[2]);
    a.av = const_cast<float*>(adam_arena[3]);
    a.hyper = hyper;
    a.step = step;
    a.aux = aux;
    blocks += pb;
  }
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(step_reduce_kernel, dim3(blocks), dim3(256), 0, S(stream), a);
  CV_LAUNCH_CHECK("step_reduce");
  return 0;
}
