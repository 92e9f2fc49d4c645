// Device side of the NT-Xent contrastive terms and the latent combine (cv_latent.hip: the design notes, the host
// side and the C-ABI), shared with the auxiliary-role launches (cv_aux.hip) that run an NT-Xent phase as extra
// workgroups of another kernel's grid.
#pragma once
#include "cv_common.hpp"

namespace cv {

// Fused step version: dheads = [dmu_c, dlv_c, dmu_s, dlv_s] from KL (weight w from the annealer) and
// the decoder gradient dz through z = mu + eps*exp(lv/2).  losses[1..2] = kl_c, kl_s; losses[7] = w.
struct CombineArgs {
  const float* heads;
  const float* z;
  const float* dz;
  int n, d;
  float beta, loc, scale;
  const int64_t* anneal_step;
  const double* rec_in;
  float* dheads;
  float* losses;
  int accumulate;  // 1: dheads += (the contrastive / MI terms are already in it)
};

// The element-wise part of the combine over the batches that start at `first` + threadIdx.x and advance by `step`
// (one workgroup: 0, NTH * 8; several: a contiguous chunk each), with the workgroup's fp64 KL sums in *kc / *ks;
// returns the annealer weight.
template <int NTH>
__device__ __forceinline__ float combine_sums(const CombineArgs& C, int first, int step, double* scratch, double* kc_out,
                                              double* ks_out) {
  const float* __restrict__ heads = C.heads;
  const float* __restrict__ z = C.z;
  const float* __restrict__ dz = C.dz;
  float* __restrict__ dheads = C.dheads;
  const int n = C.n, d = C.d;
  const double t = (double)C.anneal_step[0];
  const float beta = C.beta, loc = C.loc, scale = C.scale;
  // LogisticAnnealer.slope (trainer.py:32-34): beta / (1 + exp(-(t - loc)/scale)), in double
  const float w = (float)((double)beta / (1.0 + exp(-(t - (double)loc) / (double)scale)));
  const float inv_n = 1.0f / (float)n;
  double sc = 0.0, ss = 0.0;
  const int zd = 2 * d, total = n * zd;
  // one workgroup walks n x 2d elements: batches of U elements per thread have all their loads in
  // flight before the first use (one memory latency per batch instead of one per element: 64 serial
  // latencies per thread at VAE64 bs=256).  Each thread still visits e = t, t + NTH, ... in order, so
  // the fp64 KL sums are bit-identical to the element-at-a-time loop.
  constexpr int U = 8;
  for (int base = first + threadIdx.x; base < total; base += step) {
    float m[U], l[U], g[U], zz[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int e = base + q * NTH;
      const int ec = e < total ? e : 0;
      const int r = ec / zd, j = ec - r * zd;
      const int blk = (j < d) ? 0 : 2, k = (j < d) ? j : j - d;
      m[q] = heads[(size_t)r * 4 * d + blk * d + k];
      l[q] = heads[(size_t)r * 4 * d + (blk + 1) * d + k];
      g[q] = dz ? dz[ec] : 0.f;
      zz[q] = z[ec];
    }
    // (accumulate: every old d(heads) value of the batch is read before the first store — loads and stores through
    // one pointer stay in program order, so element-wise read-modify-writes cost one dependent round trip each)
    float om[U], ol[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int e = base + q * NTH;
      const int ec = e < total ? e : 0;
      const int r = ec / zd, j = ec - r * zd;
      const int blk = (j < d) ? 0 : 2, k = (j < d) ? j : j - d;
      om[q] = C.accumulate ? dheads[(size_t)r * 4 * d + blk * d + k] : 0.f;
      ol[q] = C.accumulate ? dheads[(size_t)r * 4 * d + (blk + 1) * d + k] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int e = base + q * NTH;
      if (e >= total) break;
      const int r = e / zd, j = e - r * zd;
      const int blk = (j < d) ? 0 : 2, k = (j < d) ? j : j - d;
      const float el = expf(l[q]);
      const double term = (double)(1.0f + l[q] - m[q] * m[q] - el);
      if (j < d) sc += term; else ss += term;
      const float vm = w * m[q] * inv_n + g[q];
      const float vl = w * (-0.5f * inv_n) * (1.0f - el) + g[q] * (zz[q] - m[q]) * 0.5f;
      dheads[(size_t)r * 4 * d + blk * d + k] = C.accumulate ? om[q] + vm : vm;
      dheads[(size_t)r * 4 * d + (blk + 1) * d + k] = C.accumulate ? ol[q] + vl : vl;
    }
  }
  *kc_out = block_sum<NTH>(sc, scratch);
  *ks_out = block_sum<NTH>(ss, scratch);
  return w;
}

template <int NTH>
__device__ __forceinline__ void combine_body(const CombineArgs& C, double* scratch) {
  double kc, ks;
  const float w = combine_sums<NTH>(C, 0, NTH * 8, scratch, &kc, &ks);
  const int n = C.n;
  if (threadIdx.x == 0) {
    if (C.rec_in) {
      double r = 0.0;
      for (int q = 0; q < CV_REC_REPL; ++q) r += C.rec_in[q];
      C.losses[0] = (float)r;
    }
    C.losses[1] = (float)(-0.5 * kc / (double)n);
    C.losses[2] = (float)(-0.5 * ks / (double)n);
    C.losses[7] = w;
  }
}

// ---------------------------------------------------------------- NT-Xent
struct Branch {
  const float* mu;
  const float* lv;
  int ld;
  int ps;
  float* dmu;
  float* dlv;
  int gld;
  const float* gscale;
  float gmul;
  float* loss_out;
  float* lse;  // [2n]: lse_all, lse_pos (units of S/tau)
};
constexpr int MAXBR = 2;
struct NtArgs {
  Branch br[MAXBR];
  const int64_t* label;
  int n, d, sim;
  float tau;
  int accumulate;
  int nbr;
  int rpb;            // rows per 256-thread block of the LDS kernels (a multiple of 4: one row per wave per pass)
  int with_combine;   // rows kernel: the block with blockIdx.y == nbr runs the latent combine (cmb)
  CombineArgs cmb;
};

constexpr int NT_ROWS = 4;   // rows (waves) per 256-thread block
constexpr int NT_MAXN = 4096;      // largest batch whose row norms the global-walk kernels stage in LDS
constexpr int NT_MAXBIG = 1 << 17;  // largest batch at all (the BIG kernels: each gradient block re-counts the
                                    // finite rows, O(n) per block)

// similarity of row i (theta_i) and column j
template <int DM>
__device__ __forceinline__ float sim_ij(int sim, const float* mi, const float* li, float ni, const float* mj,
                                        const float* lj, float nj, int d) {
  float s = 0.f;
  if (sim == CV_SIM_COSINE) {
#pragma unroll
    for (int k = 0; k < DM; ++k)
      if (k < d) s += (mj[k] / nj) * (mi[k] / ni);
    return s;
  }
  if (sim == CV_SIM_L2) {
#pragma unroll
    for (int k = 0; k < DM; ++k)
      if (k < d) {
        const float df = mj[k] - mi[k];
        s += df * df;
      }
    return -s;
  }
  if (sim == CV_SIM_MODIFIED_L2) {
#pragma unroll
    for (int k = 0; k < DM; ++k)
      if (k < d) {
        const float df = mj[k] - mi[k];
        s += df * df / expf(0.5f * (lj[k] + li[k]));
      }
    return -s;
  }
  if (sim == CV_SIM_MAHALANOBIS) {
#pragma unroll
    for (int k = 0; k < DM; ++k)
      if (k < d) {
        const float df = mj[k] - mi[k];
        s += df * df / (0.5f * (expf(lj[k]) + expf(li[k])));
      }
    return -s;
  }
  // jeffrey: kl[i,j] = 0.5(L_j - L_i - d + sum D/v_j + sum v_j/(v_i + 1e-8)); S = -0.5(kl_ij + kl_ji)
  float Li = 0.f, Lj = 0.f, t2ij = 0.f, t3ij = 0.f, t2ji = 0.f, t3ji = 0.f;
#pragma unroll
  for (int k = 0; k < DM; ++k)
    if (k < d) {
      const float vi = expf(li[k]), vj = expf(lj[k]);
      const float df = mj[k] - mi[k];
      const float D = df * df;
      Li += li[k];
      Lj += lj[k];
      t2ij += D / vj;
      t3ij += vj / (vi + 1e-8f);
      t2ji += D / vi;
      t3ji += vi / (vj + 1e-8f);
    }
  const float kij = 0.5f * ((Lj - Li - (float)d) + t2ij + t3ij);
  const float kji = 0.5f * ((Li - Lj - (float)d) + t2ji + t3ji);
  return -(0.5f * (kij + kji));
}

__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) {
    m = mn;
    s = 0.f;
    return;
  }
  s = s * expf(m - mn) + s2 * expf(m2 - mn);
  m = mn;
}

template <int DM>
__device__ __forceinline__ void load_theta(const Branch& b, int r, int d, float* m, float* l, bool need_lv) {
#pragma unroll
  for (int k = 0; k < DM; ++k) {
    m[k] = (k < d) ? b.mu[(size_t)r * b.ld + k] : 0.f;
    l[k] = (need_lv && k < d) ? b.lv[(size_t)r * b.ld + k] : 0.f;
  }
}

__device__ __forceinline__ float row_norm(const Branch& b, int r, int d) {
  float s = 0.f;
  for (int k = 0; k < d; ++k) {
    const float v = b.mu[(size_t)r * b.ld + k];
    s += v * v;
  }
  return sqrtf(s);
}

// the norm of a row already in registers: the same operations, in the same order, as row_norm
template <int DM>
__device__ __forceinline__ float reg_norm(const float* m, int d) {
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < DM; ++k)
    if (k < d) s += m[k] * m[k];
  return sqrtf(s);
}

// Global-walk kernels (the branch does not fit the LDS-staged variants).  BIG: batches above NT_MAXN (the
// reference has no cap, losses.py:98-137): the row norms are recomputed from the loaded rows instead of being
// staged in LDS (bit-identical: reg_norm), so the kernels need no per-batch LDS at all.
template <int DM>
__device__ __forceinline__ void sim_grad_row(int sim, const float* mi, const float* li, float ni, bool clamped_i,
                                             const float* mj, const float* lj, float nj, float S, float H, int d,
                                             float* gm, float* gl) {
  if (sim == CV_SIM_COSINE) {
#pragma unroll
    for (int k = 0; k < DM; ++k)
      if (k < d) {
        const float uj = mj[k] / nj, ui = mi[k] / ni;
        gm[k] += H * (clamped_i ? uj : (uj - S * ui)) / ni;
      }
    return;
  }
  if (sim == CV_SIM_L2) {
#pragma unroll
    for (int k = 0; k < DM; ++k)
      if (k < d) gm[k] += H * 2.f * (mj[k] - mi[k]);
    return;
  }
  if (sim == CV_SIM_MODIFIED_L2) {
#pragma unroll
    for (int k = 0; k < DM; ++k)
      if (k < d) {
        const float df = mj[k] - mi[k];
        const float V = expf(0.5f * (lj[k] + li[k]));
        gm[k] += H * 2.f * df / V;
        gl[k] += H * 0.5f * df * df / V;
      }
    return;
  }
  if (sim == CV_SIM_MAHALANOBIS) {
#pragma unroll
    for (int k = 0; k < DM; ++k)
      if (k < d) {
        const float df = mj[k] - mi[k];
        const float vi = expf(li[k]);
        const float V = 0.5f * (expf(lj[k]) + vi);
        gm[k] += H * 2.f * df / V;
        gl[k] += H * df * df / (V * V) * 0.5f * vi;
      }
    return;
  }
  // jeffrey
#pragma unroll
  for (int k = 0; k < DM; ++k)
    if (k < d) {
      const float vi = expf(li[k]), vj = expf(lj[k]);
      const float df = mj[k] - mi[k];
      const float D = df * df;
      gm[k] += H * 0.5f * df * (1.f / vj + 1.f / vi);
      const float a = vi + 1e-8f;
      gl[k] += H * (-0.25f) * (-(vj * vi) / (a * a) - D / vi + vi / (vj + 1e-8f));
    }
}

// The latent heads are row-major [n][4d] (mu_c, lv_c, mu_s, lv_s): a lane walking its own column j
// reads d words 16d bytes apart, so every global load instruction of the kernels above touches 64
// cache lines.  These variants stage the branch's mu / logvar rows once per workgroup in LDS with an
// odd row pitch (d+1: lanes on consecutive rows hit distinct banks), together with the labels, the
// row norms and (backward) the row log-sum-exps, and give each workgroup NTL_ROWS rows.
constexpr int NTL_ROWS = 4;  // rows per 256-thread workgroup (one per wave)

struct NtLds {
  float* mu;   // [n][d+1]
  float* lv;   // [n][d+1] (similarities that use logvar)
  float* nrm;  // [n] clamped norms (cosine)
  float* raw;  // [n] raw norms (cosine, backward)
  float* lse;  // [2n] (backward)
  long long* lab;
};

inline size_t ntl_bytes(int n, int d, bool need_lv, bool grad) {
  const size_t pd = (size_t)d + 1;
  return (size_t)n * 8 + (size_t)n * pd * 4 * (need_lv ? 2 : 1) + (size_t)n * 4 * (grad ? 4 : 1);
}

__device__ __forceinline__ NtLds ntl_carve(char* s, int n, int d, bool need_lv, bool grad) {
  NtLds L;
  const int pd = d + 1;
  L.lab = (long long*)s;
  float* p = (float*)(s + (size_t)n * 8);
  L.mu = p;
  p += (size_t)n * pd;
  L.lv = nullptr;
  if (need_lv) {
    L.lv = p;
    p += (size_t)n * pd;
  }
  L.nrm = p;
  p += n;
  L.raw = grad ? p : nullptr;
  if (grad) p += n;
  L.lse = grad ? p : nullptr;
  return L;
}

__device__ __forceinline__ void ntl_stage(const Branch& b, const int64_t* label, int n, int d, bool need_lv,
                                          bool cosine, bool grad, NtLds& L) {
  const int t = threadIdx.x, pd = d + 1;
  const FDiv fd = FDiv::make(d);
  // batches of 8 loads in flight per thread before the LDS writes (one latency per batch)
  constexpr int U = 8;
  const int nd = n * d;
  // the labels / row log-sum-exps of this thread's first rows are requested first, so the wait of the
  // first row batch covers them too
  constexpr int UL = 2;
  long long lb0[UL];
  float la0[UL], lp0[UL];
#pragma unroll
  for (int q = 0; q < UL; ++q) {
    const int i = t + q * 256;
    lb0[q] = (i < n) ? label[i] : 0;
    la0[q] = (grad && i < n) ? b.lse[i] : 0.f;
    lp0[q] = (grad && i < n) ? b.lse[n + i] : 0.f;
  }
  // float4 rows when the branch is 16-byte aligned (every VAE / VAE64 head block): n x d/4 vector loads,
  // one batch of U per thread covers n*d <= 8192 (MNIST bs=512 d=8, VAE64 bs=256 d=32) in one latency
  const bool vec = (d % 4 == 0) && (b.ld % 4 == 0) && ((reinterpret_cast<uintptr_t>(b.mu) & 15) == 0) &&
                   (!need_lv || (reinterpret_cast<uintptr_t>(b.lv) & 15) == 0);
  const int d4 = d / 4, nq = vec ? n * d4 : 0;
  const FDiv fd4 = FDiv::make(vec ? d4 : 1);
  for (int base = t; base < nq; base += 256 * U) {
    f32x4 vm[U], vl[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int i = base + q * 256, ic = i < nq ? i : 0;
      const int r = fd4.div(ic), k4 = ic - r * d4;
      vm[q] = *reinterpret_cast<const f32x4*>(b.mu + (size_t)r * b.ld + 4 * k4);
      vl[q] = need_lv ? *reinterpret_cast<const f32x4*>(b.lv + (size_t)r * b.ld + 4 * k4) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int i = base + q * 256;
      if (i < nq) {
        const int r = fd4.div(i), k4 = i - r * d4;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          L.mu[r * pd + 4 * k4 + c] = vm[q][c];
          if (need_lv) L.lv[r * pd + 4 * k4 + c] = vl[q][c];
        }
      }
    }
  }
  for (int base = vec ? nd : t; base < nd; base += 256 * U) {
    float vm[U], vl[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int i = base + q * 256;
      const int r = fd.div(i), k = i - r * d;
      vm[q] = (i < nd) ? b.mu[(size_t)r * b.ld + k] : 0.f;
      vl[q] = (need_lv && i < nd) ? b.lv[(size_t)r * b.ld + k] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int i = base + q * 256;
      const int r = fd.div(i), k = i - r * d;
      if (i < nd) {
        L.mu[r * pd + k] = vm[q];
        if (need_lv) L.lv[r * pd + k] = vl[q];
      }
    }
  }
#pragma unroll
  for (int q = 0; q < UL; ++q) {
    const int i = t + q * 256;
    if (i < n) {
      L.lab[i] = lb0[q];
      if (grad) {
        L.lse[i] = la0[q];
        L.lse[n + i] = lp0[q];
      }
    }
  }
  for (int base = t + UL * 256; base < n; base += 256 * U) {
    long long lb[U];
    float la[U], lp[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int i = base + q * 256;
      lb[q] = (i < n) ? label[i] : 0;
      la[q] = (grad && i < n) ? b.lse[i] : 0.f;
      lp[q] = (grad && i < n) ? b.lse[n + i] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int i = base + q * 256;
      if (i < n) {
        L.lab[i] = lb[q];
        if (grad) {
          L.lse[i] = la[q];
          L.lse[n + i] = lp[q];
        }
      }
    }
  }
  __syncthreads();
  if (cosine) {
    for (int j = t; j < n; j += 256) {
      float s = 0.f;
      for (int k = 0; k < d; ++k) {
        const float v = L.mu[j * pd + k];
        s += v * v;
      }
      const float r = sqrtf(s);
      L.nrm[j] = fmaxf(r, 1e-8f);
      if (grad) L.raw[j] = r;
    }
    __syncthreads();
    // cosine: rows become the unit vectors u_j = mu_j / max(|mu_j|, 1e-8) (the very quotients the
    // pair loops would otherwise recompute per pair)
    for (int i = t; i < nd; i += 256) {
      const int r = fd.div(i), k = i - r * d;
      L.mu[r * pd + k] = L.mu[r * pd + k] / L.nrm[r];
    }
  }
  __syncthreads();
}

template <int DM>
__device__ __forceinline__ float dot_u(const float* a, const float* b, int d) {
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < DM; ++k)
    if (k < d) s += b[k] * a[k];
  return s;
}

template <int DM>
__device__ __forceinline__ void ntl_theta(const NtLds& L, int r, int d, float* m, float* l, bool need_lv) {
  const int pd = d + 1;
#pragma unroll
  for (int k = 0; k < DM; ++k) {
    m[k] = (k < d) ? L.mu[r * pd + k] : 0.f;
    l[k] = (need_lv && k < d) ? L.lv[r * pd + k] : 0.f;
  }
}

// the row log-sum-exps of rows [bx * rpb, (bx + 1) * rpb) of branch `by` (by == nbr: the latent combine block)
template <int DM>
__device__ __forceinline__ void ntxent_rows_lds_body(const NtArgs& A, const int bx, const int by) {
  extern __shared__ __attribute__((aligned(16))) char ntl_smem[];
  if (by >= A.nbr) {  // the fused latent step's combine block (independent of the rows)
    if (A.with_combine && bx == 0) combine_body<256>(A.cmb, reinterpret_cast<double*>(ntl_smem));
    return;
  }
  const Branch& b = A.br[by];
  const int n = A.n, d = A.d;
  const bool cosine = A.sim == CV_SIM_COSINE;
  const bool need_lv = !(A.sim == CV_SIM_COSINE || A.sim == CV_SIM_L2);
  NtLds L = ntl_carve(ntl_smem, n, d, need_lv, false);
  ntl_stage(b, A.label, n, d, need_lv, cosine, false, L);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int iend = min(n, (bx + 1) * A.rpb);
  for (int i = bx * A.rpb + w; i < iend; i += 4) {
    float mi[DM], li[DM], mj[DM], lj[DM];
    ntl_theta<DM>(L, i, d, mi, li, need_lv);
    const long long lab = L.lab[i];
    float ma = -INFINITY, sa = 0.f, mp = -INFINITY, sp = 0.f;
    for (int j = lane; j < n; j += 64) {
      if (j == i) continue;
      ntl_theta<DM>(L, j, d, mj, lj, need_lv);
      const float S = cosine ? dot_u<DM>(mi, mj, d) : sim_ij<DM>(A.sim, mi, li, 1.f, mj, lj, 1.f, d);
      const float s = S / A.tau;
      lse_merge(ma, sa, s, 1.f);
      const bool pos = b.ps ? (L.lab[j] != lab) : (L.lab[j] == lab);
      if (pos) lse_merge(mp, sp, s, 1.f);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float m2 = __shfl_xor(ma, o, 64), s2 = __shfl_xor(sa, o, 64);
      const float m3 = __shfl_xor(mp, o, 64), s3 = __shfl_xor(sp, o, 64);
      lse_merge(ma, sa, m2, s2);
      lse_merge(mp, sp, m3, s3);
    }
    if (lane == 0) {
      b.lse[i] = (sa > 0.f) ? ma + logf(sa) : -INFINITY;
      b.lse[n + i] = (sp > 0.f) ? mp + logf(sp) : -INFINITY;
    }
  }
}

// the contrastive loss of branch `by` (block bx == 0) and the gradients of rows [bx * rpb, (bx + 1) * rpb)
template <int DM>
__device__ __forceinline__ void ntxent_grad_lds_body(const NtArgs& A, const int bx, const int by) {
  extern __shared__ __attribute__((aligned(16))) char ntl_smem[];
  __shared__ float scratch[16];
  __shared__ double dscratch[16];
  const Branch& b = A.br[by];
  const int n = A.n, d = A.d;
  const bool cosine = A.sim == CV_SIM_COSINE;
  const bool need_lv = !(A.sim == CV_SIM_COSINE || A.sim == CV_SIM_L2);
  NtLds L = ntl_carve(ntl_smem, n, d, need_lv, true);
  ntl_stage(b, A.label, n, d, need_lv, cosine, true, L);
  // finite-row count (and, in block 0, the loss)
  float cnt = 0.f;
  double lsum = 0.0;
  for (int j = threadIdx.x; j < n; j += 256) {
    const float l = L.lse[j] - L.lse[n + j];
    if (isfinite(l)) {
      cnt += 1.f;
      lsum += (double)l;
    }
  }
  const float nf = block_sum<256>(cnt, scratch);
  if (bx == 0) {
    const double tot = block_sum<256>(lsum, dscratch);
    if (threadIdx.x == 0 && b.loss_out) b.loss_out[0] = (nf > 0.f) ? (float)(tot / (double)nf) : NAN;
  }
  if (!b.dmu) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float gup = b.gmul * (b.gscale ? b.gscale[0] : 1.0f);
  const float c = (nf > 0.f) ? gup / (nf * A.tau) : 0.f;
  const int iend = min(n, (bx + 1) * A.rpb);
  for (int i = bx * A.rpb + w; i < iend; i += 4) {
    float mi[DM], li[DM], mj[DM], lj[DM], gm[DM], gl[DM];
    ntl_theta<DM>(L, i, d, mi, li, need_lv);
#pragma unroll
    for (int k = 0; k < DM; ++k) { gm[k] = 0.f; gl[k] = 0.f; }
    const float ni = cosine ? L.nrm[i] : 1.f;
    const bool clamped_i = cosine && !(L.raw[i] > 1e-8f);
    const long long lab = L.lab[i];
    const float la_i = L.lse[i], lp_i = L.lse[n + i];
    const bool fin_i = isfinite(la_i - lp_i);
    for (int j = lane; j < n; j += 64) {
      if (j == i) continue;
      ntl_theta<DM>(L, j, d, mj, lj, need_lv);
      const float S = cosine ? dot_u<DM>(mi, mj, d) : sim_ij<DM>(A.sim, mi, li, 1.f, mj, lj, 1.f, d);
      const float s = S / A.tau;
      const bool pos = b.ps ? (L.lab[j] != lab) : (L.lab[j] == lab);
      const float la_j = L.lse[j], lp_j = L.lse[n + j];
      const bool fin_j = isfinite(la_j - lp_j);
      float G = 0.f;
      if (fin_i) G += c * (expf(s - la_i) - (pos ? expf(s - lp_i) : 0.f));
      if (fin_j) G += c * (expf(s - la_j) - (pos ? expf(s - lp_j) : 0.f));
      if (G != 0.f) {
        if (cosine) {  // d S / d mu_i = (u_j - S u_i) / n_i (u_j when |mu_i| is clamped); 1/n_i applied once below
#pragma unroll
          for (int k = 0; k < DM; ++k)
            if (k < d) gm[k] += G * (clamped_i ? mj[k] : (mj[k] - S * mi[k]));
        } else {
          sim_grad_row<DM>(A.sim, mi, li, 1.f, false, mj, lj, 1.f, S, G, d, gm, gl);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < DM; ++k) {
      if (k < d) {
        gm[k] = wave_sum(gm[k]);
        if (cosine) gm[k] = gm[k] / ni;
        if (need_lv) gl[k] = wave_sum(gl[k]);
      }
    }
    // lane k writes component k (a coalesced row store instead of d scalar stores from lane 0)
    float om = 0.f, ol = 0.f;
#pragma unroll
    for (int k = 0; k < DM; ++k)
      if (k == lane) { om = gm[k]; ol = need_lv ? gl[k] : 0.f; }
    if (lane < d) {
      float* pm = b.dmu + (size_t)i * b.gld + lane;
      *pm = A.accumulate ? *pm + om : om;
      if (b.dlv) {
        float* pl = b.dlv + (size_t)i * b.gld + lane;
        *pl = A.accumulate ? *pl + ol : ol;
      }
    }
  }
}

// Register-resident variants for small batches (cosine similarity, n <= 64 * JM, d <= DM, 16-byte rows: MNIST's
// bs = 512, d = 8; VAE64's bs <= 256, d = 32).  The LDS kernels above stage the whole branch per workgroup (two dependent HBM/L2 round trips,
// three barriers and two LDS passes before the first pair), then walk one row per wave: at these sizes the staging
// is the kernel.  Here every lane requests its JM columns (rows j = lane + 64 m as float4s, the label, and for the
// gradients the two log-sum-exps) and the wave's own row in ONE batch of loads, normalises in registers and runs
// the same pair loop.  The arithmetic, and its order, is the LDS kernels' (unit vectors = row / max(|row|, 1e-8),
// the same dot products, the same per-lane merge order j ascending, the same shuffle tree and 1/n_i placement), so
// the results are bit-identical to them (tests/test_gpu_ntxent_reg.py).
constexpr int NTR_JM = 8;  // columns per lane of the d <= 8 form (n <= 512); the d <= 32 form takes 4 (n <= 256)
int ntr_rows();  // rows per 256-thread workgroup of the register variants (cv_latent.hip; CV_NT_ROWS A/B)
__host__ __device__ inline bool ntr_fits(int n, int d, int sim) {
  return sim == CV_SIM_COSINE && d % 4 == 0 && ((n <= 64 * NTR_JM && d <= 8) || (n <= 256 && d <= 32));
}

template <int DM>
__device__ __forceinline__ void ntr_row(const float* p, int d, float* m) {
#pragma unroll
  for (int k4 = 0; k4 < DM / 4; ++k4) {
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (4 * k4 < d) v = *reinterpret_cast<const f32x4*>(p + 4 * k4);
#pragma unroll
    for (int c = 0; c < 4; ++c) m[4 * k4 + c] = v[c];
  }
}

// m <- m / max(|m|, 1e-8) (the LDS kernels' staged unit vectors); returns the clamped norm, *raw the norm itself
template <int DM>
__device__ __forceinline__ float ntr_unit(float* m, int d, float* raw = nullptr) {
#if defined(CV_NT_ABLATE) && CV_NT_ABLATE == 1
  if (raw) *raw = 1.f;  // diagnostic build: no normalisation (results invalid: a timing probe only)
  return 1.f;
#endif
  const float r = reg_norm<DM>(m, d);
  const float nr = fmaxf(r, 1e-8f);
#pragma unroll
  for (int k = 0; k < DM; ++k)
    if (k < d) m[k] = m[k] / nr;
  if (raw) *raw = r;
  return nr;
}

template <int DM, int JM>
__device__ __forceinline__ void ntxent_rows_reg_body(const NtArgs& A, const int bx, const int by) {
  extern __shared__ __attribute__((aligned(16))) char ntl_smem[];
  if (by >= A.nbr) {
    if (A.with_combine && bx == 0) combine_body<256>(A.cmb, reinterpret_cast<double*>(ntl_smem));
    return;
  }
  const Branch& b = A.br[by];
  const int n = A.n, d = A.d;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i0 = bx * A.rpb + w;  // (the wave's rows: i0, i0 + 4, ... below (bx + 1) rpb)
  if (i0 >= n) return;
  // the columns (rows j = lane + 64 m) are the same for every row of the workgroup: loaded and normalised once
  float mj[JM][DM];
  long long labj[JM];
#pragma unroll
  for (int m = 0; m < JM; ++m) {
    const int j = lane + 64 * m, jc = j < n ? j : 0;
    ntr_row<DM>(b.mu + (size_t)jc * b.ld, d, mj[m]);
    labj[m] = A.label[jc];
  }
#pragma unroll
  for (int m = 0; m < JM; ++m) ntr_unit<DM>(mj[m], d);
  const int iend = min(n, (bx + 1) * A.rpb);
  for (int i = i0; i < iend; i += 4) {
    float mi[DM];
    ntr_row<DM>(b.mu + (size_t)i * b.ld, d, mi);
    const long long lab = A.label[i];
    ntr_unit<DM>(mi, d);
    float ma = -INFINITY, sa = 0.f, mp = -INFINITY, sp = 0.f;
#pragma unroll
    for (int m = 0; m < JM; ++m) {
      const int j = lane + 64 * m;
      const float s = dot_u<DM>(mi, mj[m], d) / A.tau;
      if (j < n && j != i) {
        lse_merge(ma, sa, s, 1.f);
        const bool pos = b.ps ? (labj[m] != lab) : (labj[m] == lab);
        if (pos) lse_merge(mp, sp, s, 1.f);
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float m2 = __shfl_xor(ma, o, 64), s2 = __shfl_xor(sa, o, 64);
      const float m3 = __shfl_xor(mp, o, 64), s3 = __shfl_xor(sp, o, 64);
      lse_merge(ma, sa, m2, s2);
      lse_merge(mp, sp, m3, s3);
    }
    if (lane == 0) {
      b.lse[i] = (sa > 0.f) ? ma + logf(sa) : -INFINITY;
      b.lse[n + i] = (sp > 0.f) ? mp + logf(sp) : -INFINITY;
    }
  }
}

template <int DM, int JM>
__device__ __forceinline__ void ntxent_grad_reg_body(const NtArgs& A, const int bx, const int by) {
  __shared__ float scratch[16];
  __shared__ double dscratch[16];
  const Branch& b = A.br[by];
  const int n = A.n, d = A.d;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // every column load first (their latency overlaps the finite-row count and its barriers); the columns are the
  // same for every row of the workgroup
  float mj[JM][DM], laj[JM], lpj[JM];
  long long labj[JM];
#pragma unroll
  for (int m = 0; m < JM; ++m) {
    const int j = lane + 64 * m, jc = j < n ? j : 0;
    ntr_row<DM>(b.mu + (size_t)jc * b.ld, d, mj[m]);
    labj[m] = A.label[jc];
    laj[m] = b.lse[jc];
    lpj[m] = b.lse[n + jc];
  }
  // finite-row count (and, in block 0, the loss)
  float cnt = 0.f;
  double lsum = 0.0;
  for (int j = threadIdx.x; j < n; j += 256) {
    const float l = b.lse[j] - b.lse[n + j];
    if (isfinite(l)) {
      cnt += 1.f;
      lsum += (double)l;
    }
  }
  const float nf = block_sum<256>(cnt, scratch);
  if (bx == 0) {
    const double tot = block_sum<256>(lsum, dscratch);
    if (threadIdx.x == 0 && b.loss_out) b.loss_out[0] = (nf > 0.f) ? (float)(tot / (double)nf) : NAN;
  }
  if (!b.dmu) return;
  const float gup = b.gmul * (b.gscale ? b.gscale[0] : 1.0f);
  const float c = (nf > 0.f) ? gup / (nf * A.tau) : 0.f;
#pragma unroll
  for (int m = 0; m < JM; ++m) ntr_unit<DM>(mj[m], d);
  const int iend = min(n, (bx + 1) * A.rpb);
  for (int i = bx * A.rpb + w; i < iend; i += 4) {
    float mi[DM];
    ntr_row<DM>(b.mu + (size_t)i * b.ld, d, mi);
    const long long lab = A.label[i];
    const float la_i = b.lse[i], lp_i = b.lse[n + i];
    float rawi;
    const float ni = ntr_unit<DM>(mi, d, &rawi);
    const bool clamped_i = !(rawi > 1e-8f);
    const bool fin_i = isfinite(la_i - lp_i);
    float gm[DM];
#pragma unroll
    for (int k = 0; k < DM; ++k) gm[k] = 0.f;
#pragma unroll
    for (int m = 0; m < JM; ++m) {
      const int j = lane + 64 * m;
      const float S = dot_u<DM>(mi, mj[m], d);
      const float s = S / A.tau;
      const bool pos = b.ps ? (labj[m] != lab) : (labj[m] == lab);
      const bool fin_j = isfinite(laj[m] - lpj[m]);
      float G = 0.f;
      if (fin_i) G += c * (expf(s - la_i) - (pos ? expf(s - lp_i) : 0.f));
      if (fin_j) G += c * (expf(s - laj[m]) - (pos ? expf(s - lpj[m]) : 0.f));
      if (j < n && j != i && G != 0.f) {
#pragma unroll
        for (int k = 0; k < DM; ++k)
          if (k < d) gm[k] += G * (clamped_i ? mj[m][k] : (mj[m][k] - S * mi[k]));
      }
    }
#pragma unroll
    for (int k = 0; k < DM; ++k)
      if (k < d) gm[k] = wave_sum(gm[k]) / ni;
    float om = 0.f;
#pragma unroll
    for (int k = 0; k < DM; ++k)
      if (k == lane) om = gm[k];
    if (lane < d) {
      float* pm = b.dmu + (size_t)i * b.gld + lane;
      *pm = A.accumulate ? *pm + om : om;
      if (b.dlv) {
        float* pl = b.dlv + (size_t)i * b.gld + lane;
        *pl = A.accumulate ? *pl + 0.f : 0.f;  // (the LDS kernel adds its zero logvar gradient)
      }
    }
  }
}

// An NT-Xent phase (0: row log-sum-exps, 1: losses + gradients) queued by cv_ntxent_aux to run as extra workgroups
// of this thread's next direct-kernel launch ON THE STREAM IT WAS QUEUED FOR (cv_aux.hip, cv_output_loss; a launch
// on another stream leaves it queued); cv_ntxent_aux_flush launches it alone, on that stream, if none took it, and
// cv_ntxent_aux_discard drops it (the engine's error path: a program that raised between the queue and its flush
// must not leave a request whose pointers belong to that step).
struct AuxPend {
  int set, phase;
  hipStream_t stream;
  NtArgs a;
};
extern thread_local AuxPend g_aux;
bool ntxent_reg_ok(const NtArgs& a, int nbr);  // (cv_latent.hip)
bool aux_enabled();                            // (cv_aux.hip: CV_AUX / cv_debug_aux)
void aux_count_merged();                       // (cv_aux.hip: cv_debug_aux_count)

}  // namespace cv
