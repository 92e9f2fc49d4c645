// MI estimators (CLUB-S, L1OutUB) and Adam for gfx950.
//
// The estimator q(y|x) is two 2-layer MLPs (mi_estimator.py:111-122, 152-163). A row of the batch is
// evaluated by ONE wave with lanes as units (dx, h, dy <= 64); inputs are broadcast with
// v_readlane, so a row costs ~2(dx+h) broadcasts + FMAs and no LDS traffic.
//   prep  (1 workgroup): on-device randperm (Philox keys + bitonic sort in LDS) for CLUB-S, the
//         closed-form column sums for L1OutUB, and the deterministic MI value;
//   grad  (row-parallel): dL/dx, dL/dy through the MLP (and optional MLP parameter gradients),
//         optionally chained through z = mu + eps*std into d(heads) (vae.py:56-60);
//   learn (1 workgroup): learning_loss forward/backward (mi_estimator.py:129-131) with the MLP
//         gradient reduced in registers then LDS, followed by the Adam update of the estimator
//         (trainer.py:874-888).
// L1OutUB follows the reference's broadcasting exactly (mi_estimator.py:181-191):
//   negative[b,c] = all_probs[b,c] + log(N-1 + e^-20) - log(N-1), result = mean_{b,c}(pos_c - neg_{b,c})
// which reduces to mean_c pos_c - mean_{b,c} all_probs[b,c] - delta, computed in O(N d).
#include "cv_common.hpp"

namespace cv {

__device__ __forceinline__ float bcast(float v, int k) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}

struct RowF {
  float xv;      // lane k < dx : x_k
  float a1, a3;  // lane u < h  : pre-activations
  float mu, lv;  // lane k < dy
};

__device__ __forceinline__ void mlp_fwd_row(const cv_mlp& P, const float* xrow, int lane, RowF& o) {
  o.xv = (lane < P.dx) ? xrow[lane] : 0.f;
  float a1 = 0.f, a3 = 0.f;
  if (lane < P.h) { a1 = P.b1[lane]; a3 = P.b3[lane]; }
  for (int k = 0; k < P.dx; ++k) {
    const float xk = bcast(o.xv, k);
    if (lane < P.h) {
      a1 = fmaf(P.w1[lane * P.dx + k], xk, a1);
      a3 = fmaf(P.w3[lane * P.dx + k], xk, a3);
    }
  }
  o.a1 = a1;
  o.a3 = a3;
  const float h1 = fmaxf(a1, 0.f), h3 = fmaxf(a3, 0.f);
  float mu = 0.f, lp = 0.f;
  if (lane < P.dy) { mu = P.b2[lane]; lp = P.b4[lane]; }
  for (int u = 0; u < P.h; ++u) {
    const float hu = bcast(h1, u), gu = bcast(h3, u);
    if (lane < P.dy) {
      mu = fmaf(P.w2[lane * P.h + u], hu, mu);
      lp = fmaf(P.w4[lane * P.h + u], gu, lp);
    }
  }
  o.mu = mu;
  o.lv = tanhf(lp);
}

// backward of one row: given dmu, dlv (lane k < dy) returns dx (lane k < dx); fills da1/da3 (lane u < h)
__device__ __forceinline__ float mlp_bwd_row(const cv_mlp& P, const RowF& f, float dmu, float dlv, int lane,
                                             float& da1, float& da3, float& dlvp) {
  dlvp = dlv * (1.f - f.lv * f.lv);
  float dh1 = 0.f, dh3 = 0.f;
  for (int k = 0; k < P.dy; ++k) {
    const float gm = bcast(dmu, k), gl = bcast(dlvp, k);
    if (lane < P.h) {
      dh1 = fmaf(P.w2[k * P.h + lane], gm, dh1);
      dh3 = fmaf(P.w4[k * P.h + lane], gl, dh3);
    }
  }
  da1 = (f.a1 > 0.f) ? dh1 : 0.f;
  da3 = (f.a3 > 0.f) ? dh3 : 0.f;
  float dx = 0.f;
  for (int u = 0; u < P.h; ++u) {
    const float g1 = bcast(da1, u), g3 = bcast(da3, u);
    if (lane < P.dx) dx = fmaf(P.w1[u * P.dx + lane], g1, fmaf(P.w3[u * P.dx + lane], g3, dx));
  }
  return dx;
}

// ---------------------------------------------------------------- prep (1 workgroup of 1024)
constexpr int MI_MAXN = 4096;
struct MiWork {   // workspace layout (bytes): perm[n] int, invperm[n] int, sums 4*64 double
  int* perm;
  int* invperm;
  double* sums;   // Sy[64], Sy2[64], E[64], M[64]
};
static inline size_t mi_work_bytes(int n) { return (size_t)2 * n * sizeof(int) + 4 * 64 * sizeof(double) + 64; }
__host__ __device__ inline MiWork mi_work(void* base, int n) {
  MiWork w;
  char* p = (char*)base;
  w.sums = (double*)p;
  p += 4 * 64 * sizeof(double);
  w.perm = (int*)p;
  p += n * sizeof(int);
  w.invperm = (int*)p;
  return w;
}

struct MiArgs {
  int kind;
  cv_mlp P;
  const float* x; int ldx;
  const float* y; int ldy;
  int n;
  const int64_t* perm_in;
  uint64_t seed; uint64_t* offset;
  void* work;
  float* mi_out;
  // grad
  const float* gscale; float gmul;
  float* dx; float* dy; int gld; int accumulate;
  const float* heads; const float* z; float* dheads; int d;  // chain mode (fused step)
  cv_mlp_grad G;                                           // optional parameter grads (atomics)
};

__global__ __launch_bounds__(1024) void mi_prep_kernel(const MiArgs A) {
  __shared__ unsigned int keys[MI_MAXN];
  __shared__ unsigned short idxs[MI_MAXN];
  __shared__ double red[16][4];
  __shared__ double wsum[16][2][64];
  const int n = A.n, t = threadIdx.x, lane = t & 63, w = t >> 6;
  MiWork W = mi_work(A.work, n);
  const uint64_t off = A.offset ? A.offset[0] : 0;
  if (A.kind == CV_MI_CLUBSAMPLE) {
    if (A.perm_in) {
      for (int i = t; i < n; i += 1024) {
        const int p = (int)A.perm_in[i];
        W.perm[i] = p;
        W.invperm[p] = i;
      }
    } else {
      int np2 = 1;
      while (np2 < n) np2 <<= 1;
      for (int i = t; i < np2; i += 1024) {
        keys[i] = (i < n) ? philox(A.seed, off ^ 0x5bd1e995ull, (uint64_t)i).x : 0xFFFFFFFFu;
        idxs[i] = (unsigned short)i;
      }
      __syncthreads();
      for (int k = 2; k <= np2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
          for (int i = t; i < np2; i += 1024) {
            const int ixj = i ^ j;
            if (ixj > i) {
              const bool up = (i & k) == 0;
              const unsigned int ki = keys[i], kj = keys[ixj];
              const unsigned short ii = idxs[i], ij = idxs[ixj];
              const bool gt = (ki > kj) || (ki == kj && ii > ij);
              if (gt == up) {
                keys[i] = kj; keys[ixj] = ki;
                idxs[i] = ij; idxs[ixj] = ii;
              }
            }
          }
          __syncthreads();
        }
      }
      for (int i = t; i < n; i += 1024) {
        const int p = idxs[i];
        W.perm[i] = p;
        W.invperm[p] = i;
      }
    }
    __syncthreads();
  }
  if (A.kind == CV_MI_L1OUT) {
    // column sums of y (fp64)
    for (int k = t; k < A.P.dy; k += 1024) {
      double s = 0.0, q = 0.0;
      for (int r = 0; r < n; ++r) {
        const double v = A.y[(size_t)r * A.ldy + k];
        s += v;
        q += v * v;
      }
      W.sums[k] = s;
      W.sums[64 + k] = q;
    }
    __syncthreads();
  }
  // per-row pass: one wave per row
  double acc0 = 0.0, acc1 = 0.0;  // CLUB: sum(pos-neg); L1Out: sum pos, sum A_b
  double eacc = 0.0, macc = 0.0;  // L1Out: per-lane E_k, M_k partials
  for (int r = w; r < n; r += 16) {
    RowF f;
    mlp_fwd_row(A.P, A.x + (size_t)r * A.ldx, lane, f);
    float term = 0.f, term2 = 0.f;
    double dterm = 0.0;
    if (lane < A.P.dy) {
      const float yv = A.y[(size_t)r * A.ldy + lane];
      const float el = expf(f.lv);
      if (A.kind == CV_MI_CLUBSAMPLE) {
        const float yp = A.y[(size_t)W.perm[r] * A.ldy + lane];
        const float pos = -((f.mu - yv) * (f.mu - yv)) / el;
        const float neg = -((f.mu - yp) * (f.mu - yp)) / el;
        term = pos - neg;
      } else {
        const float df = f.mu - yv;
        term = -(df * df) / 2.0f / el - f.lv / 2.0f;
        const double Sy = W.sums[lane], Sy2 = W.sums[64 + lane], m = f.mu;
        dterm = -(Sy2 - 2.0 * m * Sy + (double)n * m * m) / (2.0 * (double)el) - (double)n * (double)f.lv / 2.0;
        eacc += 1.0 / (double)el;
        macc += m / (double)el;
      }
    }
    (void)term2;
    acc0 += wave_sum((double)term);
    acc1 += wave_sum(dterm);
  }
  if (lane == 0) { red[w][0] = acc0; red[w][1] = acc1; }
  if (A.kind == CV_MI_L1OUT) {
    wsum[w][0][lane] = eacc;
    wsum[w][1][lane] = macc;
  }
  __syncthreads();
  if (t == 0) {
    double a0 = 0.0, a1 = 0.0;
    for (int i = 0; i < 16; ++i) { a0 += red[i][0]; a1 += red[i][1]; }
    double mi;
    if (A.kind == CV_MI_CLUBSAMPLE) {
      mi = a0 / (double)n / 2.0;
    } else {
      const double nn = (double)n;
      const double delta = log((nn - 1.0) + exp(-20.0)) - log(nn - 1.0);
      mi = a0 / nn - a1 / (nn * nn) - delta;
    }
    if (A.mi_out) A.mi_out[0] = (float)mi;
    if (A.offset) A.offset[0] = off + 1;
  }
  if (A.kind == CV_MI_L1OUT && t < 64) {
    double e = 0.0, m = 0.0;
    for (int i = 0; i < 16; ++i) { e += wsum[i][0][t]; m += wsum[i][1][t]; }
    W.sums[128 + t] = e;
    W.sums[192 + t] = m;
  }
}

// ---------------------------------------------------------------- row-parallel gradient
constexpr int MG_ROWS = 4;
__global__ __launch_bounds__(256) void mi_grad_kernel(const MiArgs A) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = blockIdx.x * MG_ROWS + w;
  if (r >= A.n) return;
  const int n = A.n;
  MiWork W = mi_work(A.work, n);
  const float g = A.gmul * (A.gscale ? A.gscale[0] : 1.0f);
  RowF f;
  mlp_fwd_row(A.P, A.x + (size_t)r * A.ldx, lane, f);
  float dmu = 0.f, dlv = 0.f, dyv = 0.f;
  if (A.kind == CV_MI_CLUBSAMPLE) {
    const float c = g / (2.0f * (float)n);
    if (lane < A.P.dy) {
      const float yv = A.y[(size_t)r * A.ldy + lane];
      const float yp = A.y[(size_t)W.perm[r] * A.ldy + lane];
      const float el = expf(f.lv);
      const float d1 = f.mu - yv, d2 = f.mu - yp;
      dmu = c * (-2.f * d1 + 2.f * d2) / el;
      dlv = c * (d1 * d1 - d2 * d2) / el;
      dyv = c * 2.f * d1 / el;
    }
    // row r also appears as y[perm[q]] for q = invperm[r]
    RowF fq;
    const int q = W.invperm[r];
    mlp_fwd_row(A.P, A.x + (size_t)q * A.ldx, lane, fq);
    if (lane < A.P.dy) {
      const float yv = A.y[(size_t)r * A.ldy + lane];
      dyv += c * (-2.f) * (fq.mu - yv) / expf(fq.lv);
    }
  } else {
    const float nn = (float)n;
    if (lane < A.P.dy) {
      const float yv = A.y[(size_t)r * A.ldy + lane];
      const float el = expf(f.lv);
      const float df = f.mu - yv;
      const float Sy = (float)W.sums[lane], Sy2 = (float)W.sums[64 + lane];
      const float E = (float)W.sums[128 + lane], M = (float)W.sums[192 + lane];
      // positive part (1/N) and the all-pairs part (1/N^2)
      dmu = g * (-df / (nn * el) - (Sy - nn * f.mu) / (nn * nn * el));
      const double sq = (double)Sy2 - 2.0 * (double)f.mu * Sy + (double)nn * f.mu * f.mu;
      dlv = g * ((df * df / (2.f * el) - 0.5f) / nn - ((float)(sq / (2.0 * el)) - nn / 2.f) / (nn * nn));
      dyv = g * (df / el / nn + (yv * E - M) / (nn * nn));
    }
  }
  float da1, da3, dlvp;
  const float dxv = mlp_bwd_row(A.P, f, dmu, dlv, lane, da1, da3, dlvp);
  // outputs
  if (A.dheads) {
    // x = z_c, y = z_s ; chain through z = mu + eps*exp(lv/2): dmu += dz, dlv += dz*(z-mu)/2
    const int d = A.d;
    if (lane < d) {
      const size_t hr = (size_t)r * 4 * d, zr = (size_t)r * 2 * d;
      const float muc = A.heads[hr + lane], mus = A.heads[hr + 2 * d + lane];
      A.dheads[hr + lane] += dxv;
      A.dheads[hr + d + lane] += dxv * (A.z[zr + lane] - muc) * 0.5f;
      A.dheads[hr + 2 * d + lane] += dyv;
      A.dheads[hr + 3 * d + lane] += dyv * (A.z[zr + d + lane] - mus) * 0.5f;
    }
  } else {
    if (A.dx && lane < A.P.dx) {
      float* p = A.dx + (size_t)r * A.gld + lane;
      *p = A.accumulate ? *p + dxv : dxv;
    }
    if (A.dy && lane < A.P.dy) {
      float* p = A.dy + (size_t)r * A.gld + lane;
      *p = A.accumulate ? *p + dyv : dyv;
    }
  }
  if (A.G.w1) {
    // parameter gradients of this row (atomics; the autograd path only)
    const cv_mlp& P = A.P;
    const float h1 = fmaxf(f.a1, 0.f), h3 = fmaxf(f.a3, 0.f);
    for (int k = 0; k < P.dy; ++k) {
      const float gm = bcast(dmu, k), gl = bcast(dlvp, k);
      if (lane < P.h) {
        atomicAdd(A.G.w2 + k * P.h + lane, gm * h1);
        atomicAdd(A.G.w4 + k * P.h + lane, gl * h3);
      }
    }
    if (lane < P.dy) {
      atomicAdd(A.G.b2 + lane, dmu);
      atomicAdd(A.G.b4 + lane, dlvp);
    }
    for (int k = 0; k < P.dx; ++k) {
      const float xk = bcast(f.xv, k);
      if (lane < P.h) {
        atomicAdd(A.G.w1 + lane * P.dx + k, da1 * xk);
        atomicAdd(A.G.w3 + lane * P.dx + k, da3 * xk);
      }
    }
    if (lane < P.h) {
      atomicAdd(A.G.b1 + lane, da1);
      atomicAdd(A.G.b3 + lane, da3);
    }
  }
}

// ---------------------------------------------------------------- learning step (1 workgroup)
struct LearnArgs {
  cv_mlp P;
  const float* x; int ldx;
  const float* y; int ldy;
  int n;
  float* loss_out;
  cv_mlp_grad G;     // gradient outputs (overwritten)
  // Adam (optional): flat arena
  float* params; const float* grads; float* m; float* v; long numel;
  const float* hyper; int64_t* step;
};

constexpr int LN_T = 512;  // 8 waves

template <int DM>
__global__ __launch_bounds__(LN_T) void mi_learn_kernel(const LearnArgs A) {
  __shared__ float sw1[64 * 64], sw2[64 * 64], sw3[64 * 64], sw4[64 * 64];
  __shared__ float sb1[64], sb2[64], sb3[64], sb4[64];
  __shared__ double red[LN_T / 64];
  const cv_mlp& P = A.P;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = A.n;
  // per-lane register accumulators: lane u owns dW1[u][:], dW3[u][:] (dx) and dW2[:][u], dW4[:][u] (dy)
  float g1[DM], g3[DM], g2[DM], g4[DM];
#pragma unroll
  for (int k = 0; k < DM; ++k) { g1[k] = 0.f; g3[k] = 0.f; g2[k] = 0.f; g4[k] = 0.f; }
  float gb1 = 0.f, gb3 = 0.f, gb2 = 0.f, gb4 = 0.f;
  double lsum = 0.0;
  const float inv_n = 1.0f / (float)n;
  for (int r = w; r < n; r += LN_T / 64) {
    RowF f;
    mlp_fwd_row(P, A.x + (size_t)r * A.ldx, lane, f);
    float dmu = 0.f, dlv = 0.f, term = 0.f;
    if (lane < P.dy) {
      const float yv = A.y[(size_t)r * A.ldy + lane];
      const float el = expf(f.lv);
      const float df = f.mu - yv;
      term = -(df * df) / el - f.lv;  // loglikeli summand
      dmu = inv_n * 2.f * df / el;    // d(-mean loglik)/dmu
      dlv = inv_n * (1.f - df * df / el);
    }
    lsum += wave_sum((double)term);
    float da1, da3, dlvp;
    (void)mlp_bwd_row(P, f, dmu, dlv, lane, da1, da3, dlvp);
    const float h1 = fmaxf(f.a1, 0.f), h3 = fmaxf(f.a3, 0.f);
#pragma unroll
    for (int k = 0; k < DM; ++k) {
      if (k < P.dy) {
        g2[k] = fmaf(bcast(dmu, k), h1, g2[k]);
        g4[k] = fmaf(bcast(dlvp, k), h3, g4[k]);
      }
      if (k < P.dx) {
        const float xk = bcast(f.xv, k);
        g1[k] = fmaf(da1, xk, g1[k]);
        g3[k] = fmaf(da3, xk, g3[k]);
      }
    }
    gb1 += da1;
    gb3 += da3;
    gb2 += dmu;
    gb4 += dlvp;
  }
  // cross-wave reduction into LDS (waves in sequence: deterministic)
  for (int i = t; i < 64 * 64; i += LN_T) { sw1[i] = 0.f; sw2[i] = 0.f; sw3[i] = 0.f; sw4[i] = 0.f; }
  if (t < 64) { sb1[t] = 0.f; sb2[t] = 0.f; sb3[t] = 0.f; sb4[t] = 0.f; }
  if (lane == 0) red[w] = lsum;
  __syncthreads();
  for (int ww = 0; ww < LN_T / 64; ++ww) {
    if (w == ww && lane < P.h) {
#pragma unroll
      for (int k = 0; k < DM; ++k) {
        if (k < P.dx) {
          sw1[lane * P.dx + k] += g1[k];
          sw3[lane * P.dx + k] += g3[k];
        }
        if (k < P.dy) {
          sw2[k * P.h + lane] += g2[k];
          sw4[k * P.h + lane] += g4[k];
        }
      }
      sb1[lane] += gb1;
      sb3[lane] += gb3;
    }
    if (w == ww && lane < P.dy) {
      sb2[lane] += gb2;
      sb4[lane] += gb4;
    }
    __syncthreads();
  }
  if (t == 0 && A.loss_out) {
    double s = 0.0;
    for (int i = 0; i < LN_T / 64; ++i) s += red[i];
    A.loss_out[0] = (float)(-(s / (double)n));
  }
  // write gradients
  for (int i = t; i < P.h * P.dx; i += LN_T) { A.G.w1[i] = sw1[i]; A.G.w3[i] = sw3[i]; }
  for (int i = t; i < P.dy * P.h; i += LN_T) { A.G.w2[i] = sw2[i]; A.G.w4[i] = sw4[i]; }
  for (int i = t; i < P.h; i += LN_T) { A.G.b1[i] = sb1[i]; A.G.b3[i] = sb3[i]; }
  for (int i = t; i < P.dy; i += LN_T) { A.G.b2[i] = sb2[i]; A.G.b4[i] = sb4[i]; }
  if (!A.params) return;
  __syncthreads();
  __threadfence_block();
  // Adam over the estimator arena (grads just written by this workgroup; re-read through L1 is fine
  // because the same CU wrote them)
  const long t_step = A.step[0] + 1;
  const float lr = A.hyper[0], b1 = A.hyper[1], b2 = A.hyper[2], eps = A.hyper[3], wd = A.hyper[4];
  const double bc1 = 1.0 - pow((double)b1, (double)t_step);
  const double bc2 = 1.0 - pow((double)b2, (double)t_step);
  const float step_size = (float)(-(double)lr / bc1);
  const float bc2s = (float)sqrt(bc2);
  const float omb1 = (float)(1.0 - (double)b1), omb2 = (float)(1.0 - (double)b2);
  for (long i = t; i < A.numel; i += LN_T) {
    float g = A.grads[i];
    float p = A.params[i];
    if (wd != 0.f) g = g + wd * p;
    float m = A.m[i];
    m = m + omb1 * (g - m);
    float v = A.v[i] * b2;
    v = v + omb2 * g * g;
    A.m[i] = m;
    A.v[i] = v;
    const float den = sqrtf(v) / bc2s + eps;
    A.params[i] = p + step_size * (m / den);
  }
  __syncthreads();
  if (t == 0) A.step[0] = t_step;
}

// ---------------------------------------------------------------- Adam over a flat arena
// torch.optim.Adam (foreach) over a flat arena: grid-stride float4 (the arena is 16-byte aligned and
// padded to a multiple of 4), bias corrections computed once per block.  The step counters are
// advanced by adam_advance_kernel right after (a one-thread launch, so no block has to detect being
// the last one through a contended atomic).
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ gr,
                                                   float* __restrict__ m, float* __restrict__ v, long numel,
                                                   const float* hyper, const int64_t* step, const float* gscale) {
  __shared__ float cst[8];
  if (threadIdx.x == 0) {
    const long t_step = step[0] + 1;
    const double b1 = hyper[1], b2 = hyper[2];
    const double bc1 = 1.0 - pow(b1, (double)t_step);
    const double bc2 = 1.0 - pow(b2, (double)t_step);
    cst[0] = (float)(-(double)hyper[0] / bc1);
    cst[1] = (float)sqrt(bc2);
    cst[2] = (float)(1.0 - b1);
    cst[3] = (float)(1.0 - b2);
    cst[4] = hyper[2];
    cst[5] = hyper[3];
    cst[6] = hyper[4];
    cst[7] = gscale ? gscale[0] : 1.0f;
  }
  __syncthreads();
  const float step_size = cst[0], bc2s = cst[1], omb1 = cst[2], omb2 = cst[3], b2f = cst[4], eps = cst[5];
  const float wd = cst[6], gs = cst[7];
  const long n4 = numel >> 2;
  auto upd = [&](float g, float pp, float& mm, float& vv) -> float {
    g *= gs;
    if (wd != 0.f) g = g + wd * pp;
    mm = mm + omb1 * (g - mm);
    vv = vv * b2f + omb2 * g * g;
    const float den = sqrtf(vv) / bc2s + eps;
    return pp + step_size * (mm / den);
  };
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const float4 g4 = reinterpret_cast<const float4*>(gr)[i];
    float4 p4 = reinterpret_cast<float4*>(p)[i];
    float4 m4 = reinterpret_cast<float4*>(m)[i];
    float4 v4 = reinterpret_cast<float4*>(v)[i];
    p4.x = upd(g4.x, p4.x, m4.x, v4.x);
    p4.y = upd(g4.y, p4.y, m4.y, v4.y);
    p4.z = upd(g4.z, p4.z, m4.z, v4.z);
    p4.w = upd(g4.w, p4.w, m4.w, v4.w);
    reinterpret_cast<float4*>(m)[i] = m4;
    reinterpret_cast<float4*>(v)[i] = v4;
    reinterpret_cast<float4*>(p)[i] = p4;
  }
  for (long i = (n4 << 2) + (long)blockIdx.x * 256 + threadIdx.x; i < numel; i += (long)gridDim.x * 256) {
    float mm = m[i], vv = v[i];
    p[i] = upd(gr[i], p[i], mm, vv);
    m[i] = mm;
    v[i] = vv;
  }
}

__global__ void adam_advance_kernel(int64_t* step, int64_t* aux) {
  step[0] += 1;
  step[1] = 0;
  if (aux) aux[0] += 1;
}

}  // namespace cv

using namespace cv;

extern "C" size_t cv_mi_workspace_bytes(int n) { return mi_work_bytes(n); }

static int check_mlp(const cv_mlp* P) {
  CV_REQUIRE(P && P->w1 && P->b1 && P->w2 && P->b2 && P->w3 && P->b3 && P->w4 && P->b4, "mi: MLP weights missing");
  CV_REQUIRE(P->dx > 0 && P->dx <= 64 && P->h > 0 && P->h <= 64 && P->dy > 0 && P->dy <= 64,
             "mi: MLP widths must be in 1..64 (dx=%d h=%d dy=%d)", P->dx, P->h, P->dy);
  return 0;
}

extern "C" int cv_mi_forward(int kind, const cv_mlp* mlp, const float* x, int ldx, const float* y, int ldy, int n,
                             const int64_t* perm, uint64_t seed, uint64_t* offset, void* work, float* mi_out,
                             cv_stream_t stream) {
  clear_error();
  if (check_mlp(mlp)) return 1;
  CV_REQUIRE(kind == CV_MI_CLUBSAMPLE || kind == CV_MI_L1OUT, "mi: unknown estimator %d", kind);
  CV_REQUIRE(x && y && work && n > 1 && n <= MI_MAXN, "mi_forward: bad args (2 <= n <= %d)", MI_MAXN);
  CV_REQUIRE(kind != CV_MI_CLUBSAMPLE || perm || offset, "mi_forward: CLUBSample needs perm or an RNG offset");
  MiArgs a;
  memset(&a, 0, sizeof(a));
  a.kind = kind;
  a.P = *mlp;
  a.x = x; a.ldx = ldx; a.y = y; a.ldy = ldy; a.n = n;
  a.perm_in = perm; a.seed = seed; a.offset = perm ? nullptr : offset;
  a.work = work;
  a.mi_out = mi_out;
  hipLaunchKernelGGL(mi_prep_kernel, dim3(1), dim3(1024), 0, S(stream), a);
  CV_LAUNCH_CHECK("mi_forward");
  return 0;
}

extern "C" int cv_mi_backward(int kind, const cv_mlp* mlp, const float* x, int ldx, const float* y, int ldy, int n,
                              void* work, const float* gscale, float gmul, float* dx, float* dy, int gld,
                              int accumulate, const cv_mlp_grad* g, const float* heads, const float* z,
                              float* dheads, int d, cv_stream_t stream) {
  clear_error();
  if (check_mlp(mlp)) return 1;
  CV_REQUIRE(x && y && work && n > 1 && n <= MI_MAXN, "mi_backward: bad args");
  CV_REQUIRE(!dheads || (heads && z && d == mlp->dx && d == mlp->dy), "mi_backward: chain mode needs heads, z, d");
  MiArgs a;
  memset(&a, 0, sizeof(a));
  a.kind = kind;
  a.P = *mlp;
  a.x = x; a.ldx = ldx; a.y = y; a.ldy = ldy; a.n = n;
  a.work = work;
  a.gscale = gscale; a.gmul = gmul;
  a.dx = dx; a.dy = dy; a.gld = gld; a.accumulate = accumulate;
  a.heads = heads; a.z = z; a.dheads = dheads; a.d = d;
  if (g) a.G = *g;
  hipLaunchKernelGGL(mi_grad_kernel, dim3(cdiv(n, MG_ROWS)), dim3(256), 0, S(stream), a);
  CV_LAUNCH_CHECK("mi_backward");
  return 0;
}

extern "C" int cv_mi_learning_step(const cv_mlp* mlp, const float* x, int ldx, const float* y, int ldy, int n,
                                   float* loss_out, const cv_mlp_grad* g, float* params, const float* grads,
                                   float* exp_avg, float* exp_avg_sq, int64_t numel, const float* hyper,
                                   int64_t* step, cv_stream_t stream) {
  clear_error();
  if (check_mlp(mlp)) return 1;
  CV_REQUIRE(x && y && g && g->w1 && n > 0, "mi_learning_step: bad args");
  CV_REQUIRE(!params || (grads && exp_avg && exp_avg_sq && hyper && step && numel > 0),
             "mi_learning_step: Adam arena incomplete");
  LearnArgs a;
  memset(&a, 0, sizeof(a));
  a.P = *mlp;
  a.x = x; a.ldx = ldx; a.y = y; a.ldy = ldy; a.n = n;
  a.loss_out = loss_out;
  a.G = *g;
  a.params = params; a.grads = grads; a.m = exp_avg; a.v = exp_avg_sq; a.numel = numel;
  a.hyper = hyper; a.step = step;
  const int dm = mlp->dx > mlp->dy ? mlp->dx : mlp->dy;
  if (dm <= 8) hipLaunchKernelGGL(mi_learn_kernel<8>, dim3(1), dim3(LN_T), 0, S(stream), a);
  else if (dm <= 16) hipLaunchKernelGGL(mi_learn_kernel<16>, dim3(1), dim3(LN_T), 0, S(stream), a);
  else if (dm <= 32) hipLaunchKernelGGL(mi_learn_kernel<32>, dim3(1), dim3(LN_T), 0, S(stream), a);
  else hipLaunchKernelGGL(mi_learn_kernel<64>, dim3(1), dim3(LN_T), 0, S(stream), a);
  CV_LAUNCH_CHECK("mi_learning_step");
  return 0;
}

extern "C" int cv_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t numel,
                            const float* hyper, int64_t* step, const float* grad_scale, int64_t* aux_counter,
                            cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(params && grads && exp_avg && exp_avg_sq && hyper && step && numel > 0, "adam_step: bad args");
  CV_REQUIRE(((uintptr_t)params | (uintptr_t)grads | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16 == 0,
             "adam_step: buffers must be 16-byte aligned");
  long g = (numel / 4 + 255) / 256;
  if (g > 512) g = 512;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(adam_kernel, dim3(g), dim3(256), 0, S(stream), params, grads, exp_avg, exp_avg_sq, (long)numel,
                     hyper, step, grad_scale);
  CV_LAUNCH_CHECK("adam_step");
  hipLaunchKernelGGL(adam_advance_kernel, dim3(1), dim3(1), 0, S(stream), step, aux_counter);
  CV_LAUNCH_CHECK("adam_advance");
  return 0;
}
