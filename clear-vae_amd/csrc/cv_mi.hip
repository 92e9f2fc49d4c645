// MI estimators (CLUB-S, L1OutUB) and Adam for gfx950.
//
// The estimator q(y|x) is two 2-layer MLPs (mi_estimator.py:111-122, 152-163). A row of the batch is
// evaluated by ONE wave with lanes as units (dx, h, dy <= 64); inputs are broadcast with
// v_readlane, and the four weight matrices are staged once per workgroup in LDS with an odd row
// pitch, so both the row walks (forward) and the column walks (backward) are bank-conflict free.
//   perm  (1 workgroup): on-device randperm (Philox keys + bitonic sort in LDS) for CLUB-S, the
//         closed-form column sums for L1OutUB;
//   rows  (row-parallel): the per-row MI terms, reduced per workgroup into fixed slots; the last
//         workgroup to arrive (ticket) folds the slots in block order (deterministic) into mi;
//   grad  (row-parallel): dL/dx, dL/dy through the MLP (and optional MLP parameter gradients),
//         optionally chained through z = mu + eps*std into d(heads) (vae.py:56-60);
//   learn (row-parallel, then element-parallel): learning_loss forward/backward (mi_estimator.py:
//         129-131) with the MLP gradient reduced in registers, then across the waves of a
//         workgroup in LDS, into per-workgroup partials; a second launch sums the partials per
//         parameter in block order and applies the estimator's Adam update (trainer.py:874-888).
// L1OutUB follows the reference's broadcasting exactly (mi_estimator.py:181-191):
//   negative[b,c] = all_probs[b,c] + log(N-1 + e^-20) - log(N-1), result = mean_{b,c}(pos_c - neg_{b,c})
// which reduces to mean_c pos_c - mean_{b,c} all_probs[b,c] - delta, computed in O(N d).
#include "cv_common.hpp"

namespace cv {

__device__ __forceinline__ float bcast(float v, int k) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}

// ---------------------------------------------------------------- estimator weights in LDS
// w1/w3 [u][k] (Linear(dx,h) weight rows), w2/w4 [k][u] (Linear(h,dy) weight rows), row pitch DM+1
// (odd): lane-strided row walks and lane-contiguous column walks both hit distinct banks.  64 rows,
// so lanes beyond the layer width read (ignored) in-bounds words.
template <int DM>
struct MlpLds {
  static constexpr int PW = DM + 1;
  float w1[64 * PW], w3[64 * PW];
  float w2[64 * PW], w4[64 * PW];
  float b1[64], b3[64], b2[64], b4[64];
};

template <int DM>
__device__ __forceinline__ void stage_mlp(const cv_mlp& P, MlpLds<DM>& L) {
  constexpr int PW = MlpLds<DM>::PW;
  const int t = threadIdx.x, nt = blockDim.x;
  const int dx = P.dx, h = P.h, dy = P.dy;
  // SU elements of each matrix per thread in flight per round trip, the four matrices' loads issued
  // together (a load -> LDS store per element made the staging one dependent round trip per element)
  constexpr int SU = 4;
  const int n13 = h * dx, n24 = dy * h;
  const int nn = n13 > n24 ? n13 : n24;
  for (int i0 = t; i0 < nn; i0 += nt * SU) {
    float a1[SU], a3[SU], a2[SU], a4[SU];
#pragma unroll
    for (int q = 0; q < SU; ++q) {
      const int i = i0 + q * nt;
      a1[q] = i < n13 ? P.w1[i] : 0.f;
      a3[q] = i < n13 ? P.w3[i] : 0.f;
      a2[q] = i < n24 ? P.w2[i] : 0.f;
      a4[q] = i < n24 ? P.w4[i] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < SU; ++q) {
      const int i = i0 + q * nt;
      if (i < n13) {
        const int u = i / dx, k = i - u * dx;
        L.w1[u * PW + k] = a1[q];
        L.w3[u * PW + k] = a3[q];
      }
      if (i < n24) {
        const int k = i / h, u = i - k * h;
        L.w2[k * PW + u] = a2[q];
        L.w4[k * PW + u] = a4[q];
      }
    }
  }
  for (int i = t; i < 64; i += nt) {
    L.b1[i] = (i < h) ? P.b1[i] : 0.f;
    L.b3[i] = (i < h) ? P.b3[i] : 0.f;
    L.b2[i] = (i < dy) ? P.b2[i] : 0.f;
    L.b4[i] = (i < dy) ? P.b4[i] : 0.f;
  }
  __syncthreads();
}

struct RowF {
  float xv;      // lane k < dx : x_k
  float a1, a3;  // lane u < h  : pre-activations (0 beyond h)
  float mu, lv;  // lane k < dy (0 beyond dy)
};

// forward of one row (accumulation from the bias, k = 0..dx-1 then u = 0..h-1)
template <int DM>
__device__ __forceinline__ void mlp_fwd_row(const MlpLds<DM>& L, int dx, int h, int dy, const float* xrow, int lane,
                                            RowF& o) {
  constexpr int PW = MlpLds<DM>::PW;
  o.xv = (lane < dx) ? xrow[lane] : 0.f;
  float a1 = L.b1[lane], a3 = L.b3[lane];
  const float* r1 = L.w1 + lane * PW;
  const float* r3 = L.w3 + lane * PW;
#pragma unroll
  for (int k = 0; k < DM; ++k) {
    if (k < dx) {
      const float xk = bcast(o.xv, k);
      a1 = fmaf(r1[k], xk, a1);
      a3 = fmaf(r3[k], xk, a3);
    }
  }
  if (lane >= h) { a1 = 0.f; a3 = 0.f; }
  o.a1 = a1;
  o.a3 = a3;
  const float h1 = fmaxf(a1, 0.f), h3 = fmaxf(a3, 0.f);
  float mu = L.b2[lane], lp = L.b4[lane];
  const float* r2 = L.w2 + lane * PW;
  const float* r4 = L.w4 + lane * PW;
#pragma unroll
  for (int u = 0; u < DM; ++u) {
    if (u < h) {
      const float hu = bcast(h1, u), gu = bcast(h3, u);
      mu = fmaf(r2[u], hu, mu);
      lp = fmaf(r4[u], gu, lp);
    }
  }
  o.mu = (lane < dy) ? mu : 0.f;
  o.lv = (lane < dy) ? tanhf(lp) : 0.f;
}

// backward of one row: given dmu, dlv (lane k < dy, 0 beyond) returns dx (lane k < dx, 0 beyond);
// fills da1/da3 (lane u < h, 0 beyond) and dlvp = d(pre-tanh)
template <int DM>
__device__ __forceinline__ float mlp_bwd_row(const MlpLds<DM>& L, int dx, int h, int dy, const RowF& f, float dmu,
                                             float dlv, int lane, float& da1, float& da3, float& dlvp) {
  constexpr int PW = MlpLds<DM>::PW;
  dlvp = dlv * (1.f - f.lv * f.lv);
  float dh1 = 0.f, dh3 = 0.f;
#pragma unroll
  for (int k = 0; k < DM; ++k) {
    if (k < dy) {
      const float gm = bcast(dmu, k), gl = bcast(dlvp, k);
      dh1 = fmaf(L.w2[k * PW + lane], gm, dh1);
      dh3 = fmaf(L.w4[k * PW + lane], gl, dh3);
    }
  }
  da1 = (f.a1 > 0.f) ? dh1 : 0.f;
  da3 = (f.a3 > 0.f) ? dh3 : 0.f;
  float dxv = 0.f;
#pragma unroll
  for (int u = 0; u < DM; ++u) {
    if (u < h) {
      const float g1 = bcast(da1, u), g3 = bcast(da3, u);
      dxv = fmaf(L.w1[u * PW + lane], g1, fmaf(L.w3[u * PW + lane], g3, dxv));
    }
  }
  return (lane < dx) ? dxv : 0.f;
}

// ---------------------------------------------------------------- workspace
constexpr int MI_MAXN = 4096;      // largest batch of the one-workgroup device permutation (bitonic sort in LDS)
constexpr int MI_MAXBIG = 1 << 20;  // largest batch at all (above MI_MAXN: mi_perm_big_kernel)
#ifndef CV_MI_NB
#define CV_MI_NB 64  // (64 row workgroups for the learning step measured +0.2 % on C3 over 32)
#endif
constexpr int MI_NB = CV_MI_NB;            // max row workgroups whose partials are folded
constexpr int MI_FP = 2 + 128;             // per-workgroup forward partial: acc0, acc1, E[64], M[64]
constexpr int MI_GSZ = 4 * 64 * 64 + 256;  // per-workgroup learning-gradient partial (lane-major)
struct MiWork {
  double* sums;       // Sy[64], Sy2[64], E[64], M[64]
  double* fpart;      // [MI_NB][MI_FP]
  double* lpart;      // [MI_NB]
  unsigned* ticket;   // [0] rows arrivals, [1] learn-reduce arrivals (self-resetting)
  float* gpart;       // [MI_NB][MI_GSZ]
  int* perm;
  int* invperm;
};
static inline size_t mi_work_bytes(int n) {
  return 4 * 64 * 8 + MI_NB * MI_FP * 8 + MI_NB * 8 + 64 + (size_t)MI_NB * MI_GSZ * 4 + (size_t)2 * n * 4 + 64;
}
__host__ __device__ inline MiWork mi_work(void* base, int n) {
  MiWork w;
  char* p = (char*)base;
  w.sums = (double*)p;
  p += 4 * 64 * 8;
  w.fpart = (double*)p;
  p += MI_NB * MI_FP * 8;
  w.lpart = (double*)p;
  p += MI_NB * 8;
  w.ticket = (unsigned*)p;
  p += 64;
  w.gpart = (float*)p;
  p += (size_t)MI_NB * MI_GSZ * 4;
  w.perm = (int*)p;
  p += (size_t)n * 4;
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

// a 64-bit store that bypasses the (per-XCD, non-coherent) L2, for a cross-workgroup hand-off
__device__ __forceinline__ void st_agent(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// last-arriving workgroup detection: producers drained, thread 0 takes a ticket; the last one
// acquires before the barrier that publishes the verdict, then resets the ticket for the next call
__device__ __forceinline__ bool last_block(unsigned* ticket, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned nblk = gridDim.x * gridDim.y * gridDim.z;
    const unsigned prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = prev == nblk - 1;
    *flag = last ? 1 : 0;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  return *flag != 0;
}

// ---------------------------------------------------------------- device permutation above MI_MAXN
// CLUBSample's torch.randperm (mi_estimator.py:138) for batches the one-workgroup bitonic sort below cannot hold
// (the reference has no cap): a keyed bijection of [0, n) evaluated per element — a 4-round balanced Feistel
// network on 2h bits (2^2h >= n, h >= 1) with Philox round functions, restricted to [0, n) by cycle walking (at
// most 4 expected steps: 2^2h < 4n).  Grid-stride, any number of workgroups; perm[i] and invperm[perm[i]] = i.
__device__ __forceinline__ unsigned feistel(unsigned x, int h, uint64_t seed, uint64_t off) {
  const unsigned mask = (1u << h) - 1u;
  unsigned L = x >> h, R = x & mask;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const unsigned f = philox(seed, off ^ 0x9e3779b97f4a7c15ull, ((uint64_t)r << 32) | R).x & mask;
    const unsigned nl = R;
    R = L ^ f;
    L = nl;
  }
  return (L << h) | R;
}

__global__ __launch_bounds__(256) void mi_perm_big_kernel(const MiArgs A) {
  const int n = A.n;
  MiWork W = mi_work(A.work, n);
  const uint64_t off = A.offset ? A.offset[0] : 0;  // (read before mi_perm_kernel advances it)
  int h = 1;
  while ((1ll << (2 * h)) < (long long)n) ++h;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    unsigned x = (unsigned)i;
    do {
      x = feistel(x, h, A.seed, off);
    } while (x >= (unsigned)n);
    W.perm[i] = (int)x;
    W.invperm[x] = i;
  }
}

// ---------------------------------------------------------------- perm / column sums (1 x 1024)
__global__ __launch_bounds__(1024) void mi_perm_kernel(const MiArgs A) {
  __shared__ unsigned int keys[MI_MAXN];
  __shared__ unsigned short idxs[MI_MAXN];
  __shared__ double cs[16][2][64];
  const int n = A.n, t = threadIdx.x;
  MiWork W = mi_work(A.work, n);
  const uint64_t off = A.offset ? A.offset[0] : 0;
  if (A.kind == CV_MI_CLUBSAMPLE && !A.perm_in && n > MI_MAXN) {
    // (mi_perm_big_kernel, launched before this one, wrote the permutation)
  } else if (A.kind == CV_MI_CLUBSAMPLE) {
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
  } else {
    // column sums of y (fp64): lane = column, 16 row groups folded in group order
    const int k = t & 63, g = t >> 6;
    double s = 0.0, q = 0.0;
    if (k < A.P.dy)
      for (int r = g; r < n; r += 16) {
        const double v = A.y[(size_t)r * A.ldy + k];
        s += v;
        q += v * v;
      }
    cs[g][0][k] = s;
    cs[g][1][k] = q;
    __syncthreads();
    if (t < 64) {
      double a = 0.0, b = 0.0;
      for (int i = 0; i < 16; ++i) { a += cs[i][0][t]; b += cs[i][1][t]; }
      W.sums[t] = a;
      W.sums[64 + t] = b;
    }
  }
  __syncthreads();
  if (t == 0 && A.offset) A.offset[0] = off + 1;
}

// ---------------------------------------------------------------- per-row MI terms (row-parallel)
template <int DM>
__global__ __launch_bounds__(256) void mi_rows_kernel(const MiArgs A) {
  __shared__ MlpLds<DM> L;
  __shared__ double red[4][2];
  __shared__ double wsum[4][2][64];
  __shared__ int flag;
  stage_mlp<DM>(A.P, L);
  const int n = A.n, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int dx = A.P.dx, h = A.P.h, dy = A.P.dy;
  MiWork W = mi_work(A.work, n);
  double acc0 = 0.0, acc1 = 0.0;  // CLUB: sum(pos-neg); L1Out: sum pos, sum A_b
  double eacc = 0.0, macc = 0.0;  // L1Out: per-lane E_k, M_k partials
  for (int r = blockIdx.x * 4 + w; r < n; r += gridDim.x * 4) {
    RowF f;
    mlp_fwd_row<DM>(L, dx, h, dy, A.x + (size_t)r * A.ldx, lane, f);
    float term = 0.f;
    double dterm = 0.0;
    if (lane < dy) {
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
    acc0 += wave_sum((double)term);
    acc1 += wave_sum(dterm);
  }
  if (lane == 0) { red[w][0] = acc0; red[w][1] = acc1; }
  wsum[w][0][lane] = eacc;
  wsum[w][1][lane] = macc;
  __syncthreads();
  double* fp = W.fpart + (size_t)blockIdx.x * MI_FP;
  if (t < 64) {
    double e = 0.0, m = 0.0;
    for (int i = 0; i < 4; ++i) { e += wsum[i][0][t]; m += wsum[i][1][t]; }
    st_agent(fp + 2 + t, e);
    st_agent(fp + 66 + t, m);
  } else if (t == 64) {
    double a0 = 0.0, a1 = 0.0;
    for (int i = 0; i < 4; ++i) { a0 += red[i][0]; a1 += red[i][1]; }
    st_agent(fp, a0);
    st_agent(fp + 1, a1);
  }
  if (!last_block(W.ticket, &flag)) return;
  const int nb = gridDim.x;
  // the workgroup partials folded in block order, FB blocks' loads in flight per batch (one dependent
  // load per block made this last workgroup the launch's tail)
  constexpr int FB = 16;
  if (t < 64) {
    double e = 0.0, m = 0.0;
    int b = 0;
    for (; b + FB <= nb; b += FB) {
      double ev[FB], mv[FB];
#pragma unroll
      for (int q = 0; q < FB; ++q) {
        ev[q] = W.fpart[(b + q) * MI_FP + 2 + t];
        mv[q] = W.fpart[(b + q) * MI_FP + 66 + t];
      }
#pragma unroll
      for (int q = 0; q < FB; ++q) { e += ev[q]; m += mv[q]; }
    }
    for (; b < nb; ++b) { e += W.fpart[b * MI_FP + 2 + t]; m += W.fpart[b * MI_FP + 66 + t]; }
    W.sums[128 + t] = e;
    W.sums[192 + t] = m;
  } else if (t == 64) {
    double a0 = 0.0, a1 = 0.0;
    int b = 0;
    for (; b + FB <= nb; b += FB) {
      double v0[FB], v1[FB];
#pragma unroll
      for (int q = 0; q < FB; ++q) {
        v0[q] = W.fpart[(b + q) * MI_FP];
        v1[q] = W.fpart[(b + q) * MI_FP + 1];
      }
#pragma unroll
      for (int q = 0; q < FB; ++q) { a0 += v0[q]; a1 += v1[q]; }
    }
    for (; b < nb; ++b) { a0 += W.fpart[b * MI_FP]; a1 += W.fpart[b * MI_FP + 1]; }
    double mi;
    if (A.kind == CV_MI_CLUBSAMPLE) {
      mi = a0 / (double)n / 2.0;
    } else {
      const double nn = (double)n;
      const double delta = log((nn - 1.0) + exp(-20.0)) - log(nn - 1.0);
      mi = a0 / nn - a1 / (nn * nn) - delta;
    }
    if (A.mi_out) A.mi_out[0] = (float)mi;
  }
}

// ---------------------------------------------------------------- row-parallel gradient
constexpr int MG_ROWS = 4;
template <int DM>
__global__ __launch_bounds__(256) void mi_grad_kernel(const MiArgs A) {
  __shared__ MlpLds<DM> L;
  stage_mlp<DM>(A.P, L);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = A.n;
  const int dx = A.P.dx, h = A.P.h, dy = A.P.dy;
  MiWork W = mi_work(A.work, n);
  const float g = A.gmul * (A.gscale ? A.gscale[0] : 1.0f);
  for (int r = blockIdx.x * MG_ROWS + w; r < n; r += gridDim.x * MG_ROWS) {
    RowF f;
    mlp_fwd_row<DM>(L, dx, h, dy, A.x + (size_t)r * A.ldx, lane, f);
    float dmu = 0.f, dlv = 0.f, dyv = 0.f;
    if (A.kind == CV_MI_CLUBSAMPLE) {
      const float c = g / (2.0f * (float)n);
      if (lane < dy) {
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
      mlp_fwd_row<DM>(L, dx, h, dy, A.x + (size_t)q * A.ldx, lane, fq);
      if (lane < dy) {
        const float yv = A.y[(size_t)r * A.ldy + lane];
        dyv += c * (-2.f) * (fq.mu - yv) / expf(fq.lv);
      }
    } else {
      const float nn = (float)n;
      if (lane < dy) {
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
    const float dxv = mlp_bwd_row<DM>(L, dx, h, dy, f, dmu, dlv, lane, da1, da3, dlvp);
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
      if (A.dx && lane < dx) {
        float* p = A.dx + (size_t)r * A.gld + lane;
        *p = A.accumulate ? *p + dxv : dxv;
      }
      if (A.dy && lane < dy) {
        float* p = A.dy + (size_t)r * A.gld + lane;
        *p = A.accumulate ? *p + dyv : dyv;
      }
    }
    if (A.G.w1) {
      // parameter gradients of this row (atomics; the autograd path only)
      const float h1 = fmaxf(f.a1, 0.f), h3 = fmaxf(f.a3, 0.f);
      for (int k = 0; k < dy; ++k) {
        const float gm = bcast(dmu, k), gl = bcast(dlvp, k);
        if (lane < h) {
          atomicAdd(A.G.w2 + k * h + lane, gm * h1);
          atomicAdd(A.G.w4 + k * h + lane, gl * h3);
        }
      }
      if (lane < dy) {
        atomicAdd(A.G.b2 + lane, dmu);
        atomicAdd(A.G.b4 + lane, dlvp);
      }
      for (int k = 0; k < dx; ++k) {
        const float xk = bcast(f.xv, k);
        if (lane < h) {
          atomicAdd(A.G.w1 + lane * dx + k, da1 * xk);
          atomicAdd(A.G.w3 + lane * dx + k, da3 * xk);
        }
      }
      if (lane < h) {
        atomicAdd(A.G.b1 + lane, da1);
        atomicAdd(A.G.b3 + lane, da3);
      }
    }
  }
}

// ---------------------------------------------------------------- learning step
struct LearnArgs {
  cv_mlp P;
  const float* x; int ldx;
  const float* y; int ldy;
  int n;
  void* work;
  float* loss_out;
  // Adam (optional): flat arena
  float* params; const float* grads; float* m; float* v; long numel;
  const float* hyper; int64_t* step;
};

// per-workgroup partial, lane-major with pitch 64: [dW1: k*64+u][dW3][dW2: k*64+u][dW4] (DM*64 each),
// then db1[64] db3[64] db2[64] db4[64]
template <int DM>
__global__ __launch_bounds__(256) void mi_learn_rows_kernel(const LearnArgs A) {
  __shared__ MlpLds<DM> L;
  __shared__ float sg[4 * DM * 64 + 256];
  __shared__ double red[4];
  stage_mlp<DM>(A.P, L);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = A.n, dx = A.P.dx, h = A.P.h, dy = A.P.dy;
  // per-lane register accumulators: lane u owns dW1[u][:], dW3[u][:] (dx) and dW2[:][u], dW4[:][u] (dy)
  float g1[DM], g3[DM], g2[DM], g4[DM];
#pragma unroll
  for (int k = 0; k < DM; ++k) { g1[k] = 0.f; g3[k] = 0.f; g2[k] = 0.f; g4[k] = 0.f; }
  float gb1 = 0.f, gb3 = 0.f, gb2 = 0.f, gb4 = 0.f;
  double lsum = 0.0;
  const float inv_n = 1.0f / (float)n;
  for (int r = blockIdx.x * 4 + w; r < n; r += gridDim.x * 4) {
    RowF f;
    mlp_fwd_row<DM>(L, dx, h, dy, A.x + (size_t)r * A.ldx, lane, f);
    float dmu = 0.f, dlv = 0.f, term = 0.f;
    if (lane < dy) {
      const float yv = A.y[(size_t)r * A.ldy + lane];
      const float el = expf(f.lv);
      const float df = f.mu - yv;
      term = -(df * df) / el - f.lv;  // loglikeli summand
      dmu = inv_n * 2.f * df / el;    // d(-mean loglik)/dmu
      dlv = inv_n * (1.f - df * df / el);
    }
    lsum += wave_sum((double)term);
    float da1, da3, dlvp;
    (void)mlp_bwd_row<DM>(L, dx, h, dy, f, dmu, dlv, lane, da1, da3, dlvp);
    const float h1 = fmaxf(f.a1, 0.f), h3 = fmaxf(f.a3, 0.f);
#pragma unroll
    for (int k = 0; k < DM; ++k) {
      if (k < dy) {
        g2[k] = fmaf(bcast(dmu, k), h1, g2[k]);
        g4[k] = fmaf(bcast(dlvp, k), h3, g4[k]);
      }
      if (k < dx) {
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
  // cross-wave reduction in LDS, waves in sequence (deterministic), lane-major (conflict free)
  if (lane == 0) red[w] = lsum;
  for (int ww = 0; ww < 4; ++ww) {
    if (w == ww) {
      const bool first = ww == 0;
#pragma unroll
      for (int k = 0; k < DM; ++k) {
        float* s1 = sg + k * 64 + lane;
        float* s3 = sg + (DM + k) * 64 + lane;
        float* s2 = sg + (2 * DM + k) * 64 + lane;
        float* s4 = sg + (3 * DM + k) * 64 + lane;
        *s1 = first ? g1[k] : *s1 + g1[k];
        *s3 = first ? g3[k] : *s3 + g3[k];
        *s2 = first ? g2[k] : *s2 + g2[k];
        *s4 = first ? g4[k] : *s4 + g4[k];
      }
      float* sb = sg + 4 * DM * 64;
      sb[lane] = first ? gb1 : sb[lane] + gb1;
      sb[64 + lane] = first ? gb3 : sb[64 + lane] + gb3;
      sb[128 + lane] = first ? gb2 : sb[128 + lane] + gb2;
      sb[192 + lane] = first ? gb4 : sb[192 + lane] + gb4;
    }
    __syncthreads();
  }
  MiWork W = mi_work(A.work, n);
  float4* dst = reinterpret_cast<float4*>(W.gpart + (size_t)blockIdx.x * MI_GSZ);
  const float4* src = reinterpret_cast<const float4*>(sg);
  for (int i = t; i < (4 * DM * 64 + 256) / 4; i += 256) dst[i] = src[i];
  if (t == 0) W.lpart[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// parameter segments of the estimator: canonical element j of segment s is partial word
// poff + (trans ? (j % inner)*64 + j / inner : (j / inner)*64 + j % inner)  (inner == 0: poff + j)
struct LearnSegs {
  float* g[8];
  int len[8], inner[8], poff[8], trans[8];
};

// one thread per estimator parameter (or per arena word with Adam): fold the workgroup partials in
// block order, write the gradient and take the Adam step on it
__global__ __launch_bounds__(256) void mi_learn_reduce_kernel(const LearnArgs A, const LearnSegs S, int nb,
                                                              int total) {
  __shared__ int flag;
  __shared__ float cst[8];
  __shared__ long s_step;
  MiWork W = mi_work(A.work, A.n);
  const bool adam = A.params != nullptr;
  if (adam && threadIdx.x == 0) {
    const long t_step = A.step[0] + 1;
    const double b1 = A.hyper[1], b2 = A.hyper[2];
    const double bc1 = 1.0 - pow(b1, (double)t_step);
    const double bc2 = 1.0 - pow(b2, (double)t_step);
    cst[0] = (float)(-(double)A.hyper[0] / bc1);
    cst[1] = (float)sqrt(bc2);
    cst[2] = (float)(1.0 - b1);
    cst[3] = (float)(1.0 - b2);
    cst[4] = A.hyper[2];
    cst[5] = A.hyper[3];
    cst[6] = A.hyper[4];
    s_step = t_step;
  }
  __syncthreads();
  const long dom = adam ? A.numel : (long)total;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < dom; i += (long)gridDim.x * 256) {
    int s = -1, j = 0;
    if (adam) {
      const float* p = A.grads + i;
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (p >= S.g[q] && p < S.g[q] + S.len[q]) { s = q; j = (int)(p - S.g[q]); }
    } else {
      int rem = (int)i;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (s < 0 && rem < S.len[q]) { s = q; j = rem; }
        if (s < 0) rem -= S.len[q];
      }
    }
    float g;
    if (s >= 0) {
      int off;
      if (S.inner[s] == 0) {
        off = S.poff[s] + j;
      } else {
        const int a = j / S.inner[s], b = j - a * S.inner[s];
        off = S.poff[s] + (S.trans[s] ? b * 64 + a : a * 64 + b);
      }
      // block order kept (deterministic), 32 partials in flight per batch (8 per batch left the 64-block
      // fold 8 dependent round trips long)
      g = 0.f;
      int bl = 0;
      for (; bl + 32 <= nb; bl += 32) {
        float pv[32];
#pragma unroll
        for (int q = 0; q < 32; ++q) pv[q] = W.gpart[(size_t)(bl + q) * MI_GSZ + off];
#pragma unroll
        for (int q = 0; q < 32; ++q) g += pv[q];
      }
      for (; bl + 8 <= nb; bl += 8) {
        float pv[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) pv[q] = W.gpart[(size_t)(bl + q) * MI_GSZ + off];
#pragma unroll
        for (int q = 0; q < 8; ++q) g += pv[q];
      }
      for (; bl < nb; ++bl) g += W.gpart[(size_t)bl * MI_GSZ + off];
      S.g[s][j] = g;
    } else {
      g = A.grads[i];  // arena padding (not an estimator parameter)
    }
    if (!adam) continue;
    const float step_size = cst[0], bc2s = cst[1], omb1 = cst[2], omb2 = cst[3], b2f = cst[4], eps = cst[5];
    const float wd = cst[6];
    const float p = A.params[i];
    if (wd != 0.f) g = g + wd * p;
    float m = A.m[i];
    m = m + omb1 * (g - m);
    float v = A.v[i] * b2f;
    v = v + omb2 * g * g;
    A.m[i] = m;
    A.v[i] = v;
    const float den = sqrtf(v) / bc2s + eps;
    A.params[i] = p + step_size * (m / den);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && A.loss_out) {
    double s = 0.0;
    int b = 0;
    for (; b + 16 <= nb; b += 16) {  // (16 loads in flight, block order kept)
      double lv[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) lv[q] = W.lpart[b + q];
#pragma unroll
      for (int q = 0; q < 16; ++q) s += lv[q];
    }
    for (; b < nb; ++b) s += W.lpart[b];
    A.loss_out[0] = (float)(-(s / (double)A.n));
  }
  if (!adam) return;
  // every workgroup read the step counter before taking its ticket: the last one advances it
  if (last_block(W.ticket + 1, &flag) && threadIdx.x == 0) A.step[0] = s_step;
}

// ---------------------------------------------------------------- Adam over a flat arena
// torch.optim.Adam (foreach) over a flat arena: grid-stride float4 (the arena is 16-byte aligned and
// padded to a multiple of 4), bias corrections computed once per block.  The last workgroup to
// arrive (arrivals counted in step[1]) advances the step counters.
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ gr,
                                                   float* __restrict__ m, float* __restrict__ v, long numel,
                                                   const float* hyper, int64_t* step, const float* gscale,
                                                   int64_t* aux) {
  __shared__ float cst[8];
  __shared__ int flag;
  // the first float4 of every thread is requested before thread 0's constants (two fp64 pow) and the barrier
  const long n4 = numel >> 2, i0 = (long)blockIdx.x * 256 + threadIdx.x;
  float4 g0 = make_float4(0.f, 0.f, 0.f, 0.f), p0 = g0, m0 = g0, v0 = g0;
  if (i0 < n4) {
    g0 = reinterpret_cast<const float4*>(gr)[i0];
    p0 = reinterpret_cast<const float4*>(p)[i0];
    m0 = reinterpret_cast<const float4*>(m)[i0];
    v0 = reinterpret_cast<const float4*>(v)[i0];
  }
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
  auto upd = [&](float g, float pp, float& mm, float& vv) -> float {
    g *= gs;
    if (wd != 0.f) g = g + wd * pp;
    mm = mm + omb1 * (g - mm);
    vv = vv * b2f + omb2 * g * g;
    const float den = sqrtf(vv) / bc2s + eps;
    return pp + step_size * (mm / den);
  };
  for (long i = i0; i < n4; i += (long)gridDim.x * 256) {
    const bool first = i == i0;
    const float4 g4 = first ? g0 : reinterpret_cast<const float4*>(gr)[i];
    float4 p4 = first ? p0 : reinterpret_cast<float4*>(p)[i];
    float4 m4 = first ? m0 : reinterpret_cast<float4*>(m)[i];
    float4 v4 = first ? v0 : reinterpret_cast<float4*>(v)[i];
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
  // every workgroup read step[0] (thread 0, before the first barrier) before taking its ticket
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long prev = atomicAdd((unsigned long long*)(step + 1), 1ull);
    flag = prev == (unsigned long long)(gridDim.x - 1);
  }
  __syncthreads();
  if (flag && threadIdx.x == 0) {
    step[0] += 1;
    step[1] = 0;
    if (aux) aux[0] += 1;
  }
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

// width bucket of the MLP (the register / LDS images are sized for it)
static int mlp_dm(const cv_mlp* P) {
  int m = P->dx > P->h ? P->dx : P->h;
  m = m > P->dy ? m : P->dy;
  return m <= 8 ? 8 : m <= 16 ? 16 : m <= 32 ? 32 : 64;
}

#define CV_MI_DISPATCH(dm, KERNEL, grid, block, st, arg)                          \
  do {                                                                            \
    if ((dm) == 8) hipLaunchKernelGGL(KERNEL<8>, grid, block, 0, st, arg);        \
    else if ((dm) == 16) hipLaunchKernelGGL(KERNEL<16>, grid, block, 0, st, arg); \
    else if ((dm) == 32) hipLaunchKernelGGL(KERNEL<32>, grid, block, 0, st, arg); \
    else hipLaunchKernelGGL(KERNEL<64>, grid, block, 0, st, arg);                 \
  } while (0)

static int mi_row_blocks(int n) {
  const int b = cdiv(n, 4);
  return b < MI_NB ? b : MI_NB;
}

extern "C" int cv_mi_forward(int kind, const cv_mlp* mlp, const float* x, int ldx, const float* y, int ldy, int n,
                             const int64_t* perm, uint64_t seed, uint64_t* offset, void* work, float* mi_out,
                             cv_stream_t stream) {
  clear_error();
  if (check_mlp(mlp)) return 1;
  CV_REQUIRE(kind == CV_MI_CLUBSAMPLE || kind == CV_MI_L1OUT, "mi: unknown estimator %d", kind);
  CV_REQUIRE(x && y && work && n > 1 && n <= MI_MAXBIG, "mi_forward: bad args (2 <= n <= %d)", MI_MAXBIG);
  CV_REQUIRE(kind != CV_MI_CLUBSAMPLE || perm || offset, "mi_forward: CLUBSample needs perm or an RNG offset");
  MiArgs a;
  memset(&a, 0, sizeof(a));
  a.kind = kind;
  a.P = *mlp;
  a.x = x; a.ldx = ldx; a.y = y; a.ldy = ldy; a.n = n;
  a.perm_in = perm; a.seed = seed; a.offset = perm ? nullptr : offset;
  a.work = work;
  a.mi_out = mi_out;
  if (kind == CV_MI_CLUBSAMPLE && !perm && n > MI_MAXN) {
    hipLaunchKernelGGL(mi_perm_big_kernel, dim3(cdiv(n, 256) < 256 ? cdiv(n, 256) : 256), dim3(256), 0, S(stream), a);
    CV_LAUNCH_CHECK("mi_forward.perm_big");
  }
  hipLaunchKernelGGL(mi_perm_kernel, dim3(1), dim3(1024), 0, S(stream), a);
  CV_LAUNCH_CHECK("mi_forward.perm");
  CV_MI_DISPATCH(mlp_dm(mlp), mi_rows_kernel, dim3(mi_row_blocks(n)), dim3(256), S(stream), a);
  CV_LAUNCH_CHECK("mi_forward.rows");
  return 0;
}

extern "C" int cv_mi_backward(int kind, const cv_mlp* mlp, const float* x, int ldx, const float* y, int ldy, int n,
                              void* work, const float* gscale, float gmul, float* dx, float* dy, int gld,
                              int accumulate, const cv_mlp_grad* g, const float* heads, const float* z,
                              float* dheads, int d, cv_stream_t stream) {
  clear_error();
  if (check_mlp(mlp)) return 1;
  CV_REQUIRE(x && y && work && n > 1 && n <= MI_MAXBIG, "mi_backward: bad args");
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
  int blocks = cdiv(n, MG_ROWS);
  if (blocks > 128) blocks = 128;
  CV_MI_DISPATCH(mlp_dm(mlp), mi_grad_kernel, dim3(blocks), dim3(256), S(stream), a);
  CV_LAUNCH_CHECK("mi_backward");
  return 0;
}

extern "C" int cv_mi_learning_step(const cv_mlp* mlp, const float* x, int ldx, const float* y, int ldy, int n,
                                   void* work, float* loss_out, const cv_mlp_grad* g, float* params,
                                   const float* grads, float* exp_avg, float* exp_avg_sq, int64_t numel,
                                   const float* hyper, int64_t* step, cv_stream_t stream) {
  clear_error();
  if (check_mlp(mlp)) return 1;
  CV_REQUIRE(x && y && work && g && g->w1 && g->b1 && g->w2 && g->b2 && g->w3 && g->b3 && g->w4 && g->b4 && n > 0,
             "mi_learning_step: bad args");
  CV_REQUIRE(!params || (grads && exp_avg && exp_avg_sq && hyper && step && numel > 0),
             "mi_learning_step: Adam arena incomplete");
  const int dx = mlp->dx, h = mlp->h, dy = mlp->dy;
  float* const gp[8] = {g->w1, g->w3, g->w2, g->w4, g->b1, g->b3, g->b2, g->b4};
  const int ln[8] = {h * dx, h * dx, dy * h, dy * h, h, h, dy, dy};
  if (params)
    for (int s = 0; s < 8; ++s)
      CV_REQUIRE(gp[s] >= grads && gp[s] + ln[s] <= grads + numel,
                 "mi_learning_step: with Adam the gradients must live in the grads arena");
  LearnArgs a;
  memset(&a, 0, sizeof(a));
  a.P = *mlp;
  a.x = x; a.ldx = ldx; a.y = y; a.ldy = ldy; a.n = n;
  a.work = work;
  a.loss_out = loss_out;
  a.params = params; a.grads = grads; a.m = exp_avg; a.v = exp_avg_sq; a.numel = numel;
  a.hyper = hyper; a.step = step;
  const int dm = mlp_dm(mlp);
  const int nb = mi_row_blocks(n);
  CV_MI_DISPATCH(dm, mi_learn_rows_kernel, dim3(nb), dim3(256), S(stream), a);
  CV_LAUNCH_CHECK("mi_learning_step.rows");
  const int pd = dm * 64;
  const int in[8] = {dx, dx, h, h, 0, 0, 0, 0};
  const int po[8] = {0, pd, 2 * pd, 3 * pd, 4 * pd, 4 * pd + 64, 4 * pd + 128, 4 * pd + 192};
  const int tr[8] = {1, 1, 0, 0, 0, 0, 0, 0};
  LearnSegs sg;
  int total = 0;
  for (int s = 0; s < 8; ++s) {
    sg.g[s] = gp[s]; sg.len[s] = ln[s]; sg.inner[s] = in[s]; sg.poff[s] = po[s]; sg.trans[s] = tr[s];
    total += ln[s];
  }
  const long dom = params ? (long)numel : (long)total;
  int blocks = cdiv(dom, 256);
  if (blocks > 256) blocks = 256;
  hipLaunchKernelGGL(mi_learn_reduce_kernel, dim3(blocks), dim3(256), 0, S(stream), a, sg, nb, total);
  CV_LAUNCH_CHECK("mi_learning_step.reduce");
  return 0;
}

extern "C" int cv_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t numel,
                            const float* hyper, int64_t* step, const float* grad_scale, int64_t* aux_counter,
                            cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(params && grads && exp_avg && exp_avg_sq && hyper && step && numel > 0, "adam_step: bad args");
  CV_REQUIRE(((uintptr_t)params | (uintptr_t)grads | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16 == 0,
             "adam_step: buffers must be 16-byte aligned");
  // up to 2048 workgroups (CV_ADAM_WG): the update is HBM-bound (7 x 4 bytes per parameter) and each thread has one
  // float4 of each operand in flight per iteration, so the bytes in flight scale with the resident waves (round 5's
  // 512-workgroup cap held the VAE64 arena's 171 MB at ~3.8 TB/s)
  static long cap = -1;
  if (cap < 0) {
    const char* e = getenv("CV_ADAM_WG");
    cap = e ? atol(e) : 2048;
    if (cap < 1) cap = 2048;
  }
  long g = (numel / 4 + 255) / 256;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(adam_kernel, dim3(g), dim3(256), 0, S(stream), params, grads, exp_avg, exp_avg_sq, (long)numel,
                     hyper, step, grad_scale, aux_counter);
  CV_LAUNCH_CHECK("adam_step");
  return 0;
}
