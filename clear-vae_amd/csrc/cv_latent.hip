// Latent-space kernels of the CLEAR-VAE step on gfx950:
//   reparameterisation (vae.py:56-79), KL + reparam chain rule (losses.py:48-49), the
//   reconstruction MSE of the autograd path (losses.py:45-47), and the SNN / NT-Xent contrastive
//   loss with its five similarity measures (losses.py:53-137) in two row-parallel passes:
//     rows : online log-sum-exp of S_ij/tau over all j and over positive pairs (one wave per row)
//     grad : dtheta_i = sum_j (G_ij + G_ji) dS_ij/dtheta_i with G = (q - p)/(nf*tau) on finite rows
//   (S is exactly symmetric for every measure, so only the row derivative is needed).
#include "cv_ntxent.hpp"

namespace cv {

// ---------------------------------------------------------------- reparameterisation
// offset[0] is read by every thread; the last workgroup to arrive (counted in offset[1]) advances it.
__global__ __launch_bounds__(256) void reparam_kernel(const float* __restrict__ heads, int n, int d,
                                                       const float* __restrict__ eps_in, uint64_t seed,
                                                       uint64_t* offset, float* __restrict__ z,
                                                       float* __restrict__ eps_out) {
  const uint64_t off = offset ? offset[0] : 0;
  const int zd = 2 * d;
  const long total = (long)n * zd;
  for (long p = (long)blockIdx.x * blockDim.x + threadIdx.x; 2 * p < total; p += (long)gridDim.x * blockDim.x) {
    float e2[2];
    if (!eps_in) normal2(seed, off, (uint64_t)p, e2[0], e2[1]);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const long e = 2 * p + q;
      if (e >= total) break;
      const int row = (int)(e / zd), j = (int)(e % zd);
      const int blk = (j < d) ? 0 : 2;  // c: mu at 0, lv at d ; s: mu at 2d, lv at 3d
      const int k = (j < d) ? j : j - d;
      const float mu = heads[(size_t)row * 4 * d + blk * d + k];
      const float lv = heads[(size_t)row * 4 * d + (blk + 1) * d + k];
      const float ep = eps_in ? eps_in[e] : e2[q];
      const float sd = expf(0.5f * lv);
      z[e] = mu + ep * sd;
      if (eps_out) eps_out[e] = ep;
    }
  }
  if (offset && !eps_in) {  // the last workgroup to finish advances the counter (offset[1]: arrivals)
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long prev = atomicAdd((unsigned long long*)(offset + 1), 1ull);
      if (prev == (unsigned long long)(gridDim.x - 1)) {
        offset[0] = off + 1;
        offset[1] = 0;
      }
    }
  }
}

__global__ void offset_advance_kernel(uint64_t* offset) { offset[0] += 1; }

// single factor (module path): z = mu + eps*exp(lv/2); grid-stride, offset advanced by the last block
__global__ __launch_bounds__(256) void sample_kernel(const float* __restrict__ mu, const float* __restrict__ lv,
                                                     long numel, const float* __restrict__ eps_in, uint64_t seed,
                                                     uint64_t* offset, float* __restrict__ z) {
  const uint64_t off = offset ? offset[0] : 0;
  for (long p = (long)blockIdx.x * 256 + threadIdx.x; 2 * p < numel; p += (long)gridDim.x * 256) {
    float e2[2];
    if (!eps_in) normal2(seed, off, (uint64_t)p, e2[0], e2[1]);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const long e = 2 * p + q;
      if (e >= numel) break;
      const float ep = eps_in ? eps_in[e] : e2[q];
      z[e] = mu[e] + ep * expf(0.5f * lv[e]);
    }
  }
  if (offset) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long prev = atomicAdd((unsigned long long*)(offset + 1), 1ull);
      if (prev == (unsigned long long)(gridDim.x - 1)) {
        offset[0] = off + 1;
        offset[1] = 0;
      }
    }
  }
}
__global__ __launch_bounds__(256) void sample_bwd_kernel(const float* __restrict__ mu, const float* __restrict__ z,
                                                         const float* __restrict__ dz, long numel, float* dmu,
                                                         float* dlv, int accumulate) {
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < numel; e += (long)gridDim.x * 256) {
    const float g = dz[e];
    const float gl = g * (z[e] - mu[e]) * 0.5f;
    dmu[e] = accumulate ? dmu[e] + g : g;
    dlv[e] = accumulate ? dlv[e] + gl : gl;
  }
}

// ---------------------------------------------------------------- KL (+ combination with dz)
// kl = -0.5/n * sum(1 + lv - mu^2 - exp(lv)); d kl/d mu = mu/n, d kl/d lv = -0.5/n (1 - exp(lv)).
// Deterministic: one workgroup, fixed-order tree reduction.
__global__ __launch_bounds__(1024) void kl_kernel(const float* __restrict__ mu, const float* __restrict__ lv, int ld,
                                                  int n, int d, float* kl_out, const float* gscale,
                                                  float* dmu, float* dlv, int gld, int accumulate) {
  __shared__ double scratch[16];
  double s = 0.0;
  const float g = gscale ? gscale[0] : 1.0f;
  const float inv_n = 1.0f / (float)n;
  for (int e = threadIdx.x; e < n * d; e += blockDim.x) {
    const int r = e / d, k = e % d;
    const float m = mu[(size_t)r * ld + k], l = lv[(size_t)r * ld + k];
    const float el = expf(l);
    s += (double)(1.0f + l - m * m - el);
    if (dmu) {
      const float gm = g * m * inv_n;
      const float gl = g * (-0.5f * inv_n) * (1.0f - el);
      float* pm = dmu + (size_t)r * gld + k;
      float* pl = dlv + (size_t)r * gld + k;
      *pm = accumulate ? *pm + gm : gm;
      *pl = accumulate ? *pl + gl : gl;
    }
  }
  const double tot = block_sum<1024>(s, scratch);
  if (threadIdx.x == 0 && kl_out) kl_out[0] = (float)(-0.5 * tot / (double)n);
}

__global__ __launch_bounds__(1024) void combine_kernel(const CombineArgs C) {
  __shared__ double scratch[16];
  combine_body<1024>(C, scratch);
}

// The combine over several workgroups (one batch of 8 elements per thread each): the element-wise d(heads) terms
// are the one-workgroup kernel's; each workgroup writes its two fp64 KL partials into its own slot of the caller's
// workspace, releases them (agent-scope fence) and takes the arrival ticket; the last workgroup to arrive acquires,
// sums the slots in workgroup order (the result does not depend on the arrival order: bit-reproducible run to run),
// writes the losses and resets the ticket for the next launch.  Nothing is shared between launches that do not share
// a workspace (two steps on two streams each own one).  A single workgroup walking n x 2d elements in 8-element
// batches was a chain of dependent round trips on the step's critical path (MNIST 10 us, VAE64 17 us).
// CV_COMBINE_WG=0, or no workspace: the one-workgroup kernel.
constexpr int CMB_NT = 256;
constexpr int CMB_MAXG = 64;
constexpr int CMB_SLOTS = 1024;  // KL partial slots of the workspace (combine_multi: CMB_MAXG; combine_dz: dz tiles)
__global__ __launch_bounds__(CMB_NT) void combine_multi_kernel(const CombineArgs C, double* __restrict__ work) {
  __shared__ double scratch[16];
  __shared__ int last;
  double kc, ks;
  const float w = combine_sums<CMB_NT>(C, blockIdx.x * CMB_NT * 8, gridDim.x * CMB_NT * 8, scratch, &kc, &ks);
  unsigned* ticket = reinterpret_cast<unsigned*>(work + 2 * CMB_SLOTS);
  if (threadIdx.x == 0) {
    work[2 * blockIdx.x] = kc;
    work[2 * blockIdx.x + 1] = ks;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  if (threadIdx.x < 64) {  // (one wave: the partials in workgroup order, a fixed-shape fp64 tree)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const int t = threadIdx.x;
    double a = 0.0, b = 0.0;
    if (t < (int)gridDim.x) {
      a = __hip_atomic_load(work + 2 * t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      b = __hip_atomic_load(work + 2 * t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      a += __shfl_down(a, o, 64);
      b += __shfl_down(b, o, 64);
    }
    if (t == 0) {
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (C.rec_in) {
        double r = 0.0;
        for (int q = 0; q < CV_REC_REPL; ++q) r += C.rec_in[q];
        C.losses[0] = (float)r;
      }
      C.losses[1] = (float)(-0.5 * a / (double)C.n);
      C.losses[2] = (float)(-0.5 * b / (double)C.n);
      C.losses[7] = w;
    }
  }
}

// The combine with the decoder-input gradient dz = d(h) W computed here, deterministically (trainer.py:452-480 through
// the decoder Linear, vae.py:33, and z = mu + eps exp(lv / 2), vae.py:56-60).  The decoder-input backward used to add
// dz in 16-feature partials with fp32 atomics (128 workgroups onto every element): the one order-dependent sum of the
// fused step (round 6: with it removed, replays of the MNIST and CelebA steps from the same state are bit-identical).
// Workgroup (s, rb, jt) contracts F / S storage columns (slice s) for dz rows 16 rb .. 16 rb + 15, columns 16 jt ..
// 16 jt + 15 on v_mfma_f32_16x16x4_f32 (lane l: a float4 of d(h) row l % 16 at 4 (l / 16) consecutive columns, and W
// of those columns' features at z column l % 16; step s2 contracts k = 4 (l / 16) + s2), its four waves' tiles added
// in wave order, and parks the tile in the workspace.  The last of a tile's S slices to arrive (release / acquire
// around the tile's ticket) adds the S tiles in slice order and runs the combine of its 256 elements (the arithmetic
// of combine_sums); the KL partials of the tiles go to the workspace's slots, summed in tile order by the last tile
// (combine_multi_kernel's protocol).  Every sum has a fixed order.
constexpr int CDZ_S = 8;  // most F slices (workgroups per 16 x 16 dz tile); default 4 (CV_CDZ_S)
__global__ __launch_bounds__(256) void combine_dz_kernel(const CombineArgs C, const float* __restrict__ gh,
                                                         const float* __restrict__ W, int F, int pix, int ch, int S,
                                                         float* __restrict__ dz_out, double* __restrict__ work) {
  __shared__ float red[4][16][17];
  __shared__ double scratch[16];
  __shared__ int last;
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int n = C.n, d = C.d, K = 2 * d;
  const int sl = blockIdx.x, rb = blockIdx.y, jt = blockIdx.z;
  const int ntile = gridDim.y * gridDim.z, tile = rb + gridDim.y * jt;
  const int row_l = 16 * rb + (l & 15), q = l >> 4, jl = 16 * jt + (l & 15);
  const bool rok = row_l < n, jok = jl < K;
  const float* grow = gh + (size_t)(rok ? row_l : 0) * F;
  const int per = F / S, c_beg = sl * per + w * (per >> 2), c_end = c_beg + (per >> 2);  // (host: F % (64 S) == 0)
  // (storage column col -> PyTorch feature (col % ch) pix + col / ch; ch % 4 == 0, so the 4 columns of a float4 are
  // features f0, f0 + pix, f0 + 2 pix, f0 + 3 pix)
  auto feat = [&](int col) { return pix <= 1 ? col : (col % ch) * pix + col / ch; };
  const int fstep = pix <= 1 ? 1 : pix;
  // the combine operands of this thread's element, requested before the contraction (used by the tile's last slice)
  const int i = t >> 4, jj = t & 15, row = 16 * rb + i, j = 16 * jt + jj;
  const bool eok = row < n && j < K;
  const int eblk = (j < d) ? 0 : 2, ek = (j < d) ? j : j - d;
  const size_t hm = eok ? (size_t)row * 4 * d + eblk * d + ek : 0, hl = hm + (eok ? d : 0);
  const float m = C.heads[hm], lv = C.heads[hl], zz = C.z[eok ? (size_t)row * K + j : 0];
  const float om = C.accumulate ? C.dheads[hm] : 0.f, ol = C.accumulate ? C.dheads[hl] : 0.f;
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int U = 4;  // 16-column chunks whose loads are in flight together
  for (int c0 = c_beg; c0 < c_end; c0 += 16 * U) {
    f32x4 a[U];
    float b[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int cc = c0 + 16 * u + 4 * q;
      const bool in = cc < c_end;
      a[u] = *reinterpret_cast<const f32x4*>(grow + (in ? cc : c_beg));
      const float* wp = W + (size_t)feat(in ? cc : c_beg) * K + jl;
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) b[u][s2] = (jok && in) ? wp[(size_t)s2 * fstep * K] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(rok ? a[u][s2] : 0.f, b[u][s2], acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[w][4 * q + r][l & 15] = acc[r];
  __syncthreads();
  unsigned* gticket = reinterpret_cast<unsigned*>(work + 2 * CMB_SLOTS);
  unsigned* tticket = gticket + 2;
  float* part = reinterpret_cast<float*>(work + 2 * CMB_SLOTS + 1 + CMB_SLOTS / 2);
  const float mine = ((red[0][i][jj] + red[1][i][jj]) + red[2][i][jj]) + red[3][i][jj];
  float g = mine;
  if (S > 1) {
    part[((size_t)tile * S + sl) * 256 + t] = mine;
    __syncthreads();
    if (t == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      last = __hip_atomic_fetch_add(tticket + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)S - 1;
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        __hip_atomic_store(tticket + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __syncthreads();
    if (!last) return;
    // the tile's last slice: dz = the S slice tiles in slice order, then the combine of its 256 elements
    float pv[CDZ_S];
#pragma unroll
    for (int s2 = 0; s2 < CDZ_S; ++s2)
      pv[s2] = s2 < S ? (s2 == sl ? mine : __hip_atomic_load(part + ((size_t)tile * S + s2) * 256 + t, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT)) : 0.f;
    g = pv[0];
#pragma unroll
    for (int s2 = 1; s2 < CDZ_S; ++s2)
      if (s2 < S) g += pv[s2];
  }
  const double tt = (double)C.anneal_step[0];
  const float wgt = (float)((double)C.beta / (1.0 + exp(-(tt - (double)C.loc) / (double)C.scale)));
  double sc = 0.0, ss = 0.0;
  if (eok) {
    if (dz_out) dz_out[(size_t)row * K + j] = g;
    const float inv_n = 1.0f / (float)n;
    const float el = expf(lv);
    const double term = (double)(1.0f + lv - m * m - el);
    if (j < d) sc = term; else ss = term;
    const float vm = wgt * m * inv_n + g;
    const float vl = wgt * (-0.5f * inv_n) * (1.0f - el) + g * (zz - m) * 0.5f;
    C.dheads[hm] = C.accumulate ? om + vm : vm;
    C.dheads[hl] = C.accumulate ? ol + vl : vl;
  }
  const double kc = block_sum<256>(sc, scratch);
  const double ks = block_sum<256>(ss, scratch);
  if (t == 0) {
    work[2 * tile] = kc;
    work[2 * tile + 1] = ks;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    last = __hip_atomic_fetch_add(gticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)ntile - 1;
  }
  __syncthreads();
  if (!last || t >= 64) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  double a = 0.0, bsum = 0.0;  // (lane t sums slots t, t + 64, ... in order; then a fixed shuffle tree)
  for (int s2 = t; s2 < ntile; s2 += 64) {
    a += __hip_atomic_load(work + 2 * s2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bsum += __hip_atomic_load(work + 2 * s2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_down(a, o, 64);
    bsum += __shfl_down(bsum, o, 64);
  }
  if (t == 0) {
    __hip_atomic_store(gticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (C.rec_in) {
      double r = 0.0;
      for (int q2 = 0; q2 < CV_REC_REPL; ++q2) r += C.rec_in[q2];
      C.losses[0] = (float)r;
    }
    C.losses[1] = (float)(-0.5 * a / (double)n);
    C.losses[2] = (float)(-0.5 * bsum / (double)n);
    C.losses[7] = wgt;
  }
}

static void combine_launch(const CombineArgs& C, double* work, hipStream_t st) {
  static int mode = -1;
  if (mode < 0) {
    const char* e = getenv("CV_COMBINE_WG");
    mode = (e && atoi(e) == 0) ? 0 : 1;
  }
  const long total = (long)C.n * 2 * C.d;
  long g = (total + CMB_NT * 8 - 1) / (CMB_NT * 8);
  if (g > CMB_MAXG) g = CMB_MAXG;
  if (!mode || g < 2 || !work) {
    hipLaunchKernelGGL(combine_kernel, dim3(1), dim3(1024), 0, st, C);
    return;
  }
  note_launch((const void*)combine_multi_kernel);
  hipLaunchKernelGGL(combine_multi_kernel, dim3((unsigned)g), dim3(CMB_NT), 0, st, C, work);
}

// ---------------------------------------------------------------- reconstruction MSE (autograd path)
__global__ __launch_bounds__(1024) void mse_kernel(const float* __restrict__ xh, const float* __restrict__ x, long total,
                                                   int n, float* rec_out, double* acc) {
  // multi-block: partial sums to acc (fp64 atomics); last block writes rec_out
  __shared__ double scratch[16];
  double s = 0.0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const float dd = xh[i] - x[i];
    s += (double)(dd * dd);
  }
  s = block_sum<1024>(s, scratch);
  if (threadIdx.x == 0) atomic_add_f64(acc, s);
}
__global__ void mse_finish_kernel(const double* acc, int n, float* rec_out) {
  if (threadIdx.x == 0) rec_out[0] = (float)(acc[0] / (double)n);
}
__global__ __launch_bounds__(256) void mse_bwd_kernel(const float* __restrict__ xh, const float* __restrict__ x,
                                                      long total, int n, const float* gscale, float* dxh) {
  const float g = (gscale ? gscale[0] : 1.0f) * 2.0f / (float)n;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x)
    dxh[i] = g * (xh[i] - x[i]);
}

template <int DM, bool BIG>
__global__ __launch_bounds__(256) void ntxent_rows_kernel(const NtArgs A) {
  __shared__ float nrm[BIG ? 1 : NT_MAXN];
  const Branch& b = A.br[blockIdx.y];
  const int n = A.n, d = A.d;
  const bool cosine = A.sim == CV_SIM_COSINE;
  const bool need_lv = !(A.sim == CV_SIM_COSINE || A.sim == CV_SIM_L2);
  if (cosine && !BIG)
    for (int j = threadIdx.x; j < n; j += 256) nrm[j] = fmaxf(row_norm(b, j, d), 1e-8f);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = blockIdx.x * NT_ROWS + w;
  if (i >= n) return;
  float mi[DM], li[DM], mj[DM], lj[DM];
  load_theta<DM>(b, i, d, mi, li, need_lv);
  const float ni = cosine ? (BIG ? fmaxf(reg_norm<DM>(mi, d), 1e-8f) : nrm[i]) : 1.f;
  const int64_t lab = A.label[i];
  float ma = -INFINITY, sa = 0.f, mp = -INFINITY, sp = 0.f;
  for (int j = lane; j < n; j += 64) {
    if (j == i) continue;
    load_theta<DM>(b, j, d, mj, lj, need_lv);
    const float nj = cosine ? (BIG ? fmaxf(reg_norm<DM>(mj, d), 1e-8f) : nrm[j]) : 1.f;
    const float s = sim_ij<DM>(A.sim, mi, li, ni, mj, lj, nj, d) / A.tau;
    lse_merge(ma, sa, s, 1.f);
    const bool pos = b.ps ? (A.label[j] != lab) : (A.label[j] == lab);
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

// d S_ij / d theta_i (row derivative), accumulated with weight H
template <int DM, bool BIG>
__global__ __launch_bounds__(256) void ntxent_grad_kernel(const NtArgs A) {
  __shared__ float nrm[BIG ? 1 : NT_MAXN];
  __shared__ float rawn[BIG ? 1 : NT_MAXN];
  __shared__ float scratch[16];
  __shared__ double dscratch[16];
  const Branch& b = A.br[blockIdx.y];
  const int n = A.n, d = A.d;
  const bool cosine = A.sim == CV_SIM_COSINE;
  const bool need_lv = !(A.sim == CV_SIM_COSINE || A.sim == CV_SIM_L2);
  // finite-row count (and, in block 0, the loss)
  float cnt = 0.f;
  double lsum = 0.0;
  for (int j = threadIdx.x; j < n; j += 256) {
    const float l = b.lse[j] - b.lse[n + j];
    if (isfinite(l)) {
      cnt += 1.f;
      lsum += (double)l;
    }
    if (cosine && !BIG) {
      const float r = row_norm(b, j, d);
      rawn[j] = r;
      nrm[j] = fmaxf(r, 1e-8f);
    }
  }
  const float nf = block_sum<256>(cnt, scratch);
  if (blockIdx.x == 0) {
    const double tot = block_sum<256>(lsum, dscratch);
    if (threadIdx.x == 0 && b.loss_out) b.loss_out[0] = (nf > 0.f) ? (float)(tot / (double)nf) : NAN;
  }
  __syncthreads();
  if (!b.dmu) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = blockIdx.x * NT_ROWS + w;
  if (i >= n) return;
  const float gup = b.gmul * (b.gscale ? b.gscale[0] : 1.0f);
  const float c = (nf > 0.f) ? gup / (nf * A.tau) : 0.f;
  float mi[DM], li[DM], mj[DM], lj[DM], gm[DM], gl[DM];
  load_theta<DM>(b, i, d, mi, li, need_lv);
#pragma unroll
  for (int k = 0; k < DM; ++k) { gm[k] = 0.f; gl[k] = 0.f; }
  const float rni = (cosine && BIG) ? reg_norm<DM>(mi, d) : 0.f;
  const float ni = cosine ? (BIG ? fmaxf(rni, 1e-8f) : nrm[i]) : 1.f;
  const bool clamped_i = cosine && !((BIG ? rni : rawn[i]) > 1e-8f);
  const int64_t lab = A.label[i];
  const float la_i = b.lse[i], lp_i = b.lse[n + i];
  const bool fin_i = isfinite(la_i - lp_i);
  for (int j = lane; j < n; j += 64) {
    if (j == i) continue;
    load_theta<DM>(b, j, d, mj, lj, need_lv);
    const float nj = cosine ? (BIG ? fmaxf(reg_norm<DM>(mj, d), 1e-8f) : nrm[j]) : 1.f;
    const float S = sim_ij<DM>(A.sim, mi, li, ni, mj, lj, nj, d);
    const float s = S / A.tau;
    const bool pos = b.ps ? (A.label[j] != lab) : (A.label[j] == lab);
    const float la_j = b.lse[j], lp_j = b.lse[n + j];
    const bool fin_j = isfinite(la_j - lp_j);
    float G = 0.f;
    if (fin_i) G += c * (expf(s - la_i) - (pos ? expf(s - lp_i) : 0.f));
    if (fin_j) G += c * (expf(s - la_j) - (pos ? expf(s - lp_j) : 0.f));
    if (G != 0.f) sim_grad_row<DM>(A.sim, mi, li, ni, clamped_i, mj, lj, nj, S, G, d, gm, gl);
  }
#pragma unroll
  for (int k = 0; k < DM; ++k) {
    if (k < d) {
      gm[k] = wave_sum(gm[k]);
      if (need_lv) gl[k] = wave_sum(gl[k]);
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < DM; ++k) {
      if (k < d) {
        float* pm = b.dmu + (size_t)i * b.gld + k;
        *pm = A.accumulate ? *pm + gm[k] : gm[k];
        if (b.dlv) {
          float* pl = b.dlv + (size_t)i * b.gld + k;
          const float v = need_lv ? gl[k] : 0.f;
          *pl = A.accumulate ? *pl + v : v;
        }
      }
    }
  }
}

// ---------------------------------------------------------------- NT-Xent, LDS-staged
template <int DM>
__global__ __launch_bounds__(256) void ntxent_rows_lds_kernel(const NtArgs A) {
  ntxent_rows_lds_body<DM>(A, blockIdx.x, blockIdx.y);
}

template <int DM>
__global__ __launch_bounds__(256) void ntxent_grad_lds_kernel(const NtArgs A) {
  ntxent_grad_lds_body<DM>(A, blockIdx.x, blockIdx.y);
}

// ---------------------------------------------------------------- NT-Xent rows + gradients in one launch
// (A/B knob CV_NT_FUSED=1; measured slower than the two launches — MNIST latent step 35.2 -> 42.2 us in-step: the
// wait holds every workgroup at the slowest one's log-sum-exps and the polling adds its own latency — so off.)
// The gradient of row i needs the log-sum-exps of every row j (the loss is symmetric in S), so the two passes
// above are two launches.  Here each workgroup computes its rows' log-sum-exps, publishes them (release, then an
// arrival count per branch), waits until every workgroup of its branch and the latent-combine workgroup have
// arrived (acquire), and runs the gradient pass for the same rows.  The host takes this path only when the whole
// grid fits the device's resident slots at once (occupancy query), so every awaited workgroup is running; the
// wait is bounded all the same (~0.1 s: a timeout sets g_nt_sync[7] and proceeds rather than hanging).  The last
// workgroup to finish resets the counters for the next launch (graph replays need no host zeroing).
__device__ unsigned g_nt_sync[8];  // [0..1] branch arrivals, [2] combine done, [3] grad finishes, [7] timeout flag

__device__ __forceinline__ unsigned nt_load(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int DM>
__global__ __launch_bounds__(256) void ntxent_fused_kernel(const NtArgs A) {
  extern __shared__ __attribute__((aligned(16))) char ntl_smem[];
  __shared__ float scratch[16];
  __shared__ double dscratch[16];
  const int t = threadIdx.x;
  if (blockIdx.y >= (unsigned)A.nbr) {  // the latent combine (KL + decoder chain seed of dheads)
    if (A.with_combine && blockIdx.x == 0) {
      combine_body<256>(A.cmb, reinterpret_cast<double*>(ntl_smem));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (every wave's dheads stores complete before the release)
      __syncthreads();
      if (t == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_fetch_add(g_nt_sync + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  const int br = blockIdx.y;
  const Branch& b = A.br[br];
  const int n = A.n, d = A.d;
  const bool cosine = A.sim == CV_SIM_COSINE;
  const bool need_lv = !(A.sim == CV_SIM_COSINE || A.sim == CV_SIM_L2);
  NtLds L = ntl_carve(ntl_smem, n, d, need_lv, true);
  ntl_stage(b, A.label, n, d, need_lv, cosine, true, L);  // (its lse copy is stale: reloaded below)
  const int lane = t & 63, w = t >> 6;
  const int iend = min(n, (int)(blockIdx.x + 1) * A.rpb);
  // ---- rows: log-sum-exps (ntxent_rows_lds_kernel's loop)
  for (int i = blockIdx.x * A.rpb + w; i < iend; i += 4) {
    float mi[DM], li[DM], mj[DM], lj[DM];
    ntl_theta<DM>(L, i, d, mi, li, need_lv);
    const long long lab = L.lab[i];
    float ma = -INFINITY, sa = 0.f, mp = -INFINITY, sp = 0.f;
    for (int j = lane; j < n; j += 64) {
      if (j == i) continue;
      ntl_theta<DM>(L, j, d, mj, lj, need_lv);
      const float S = cosine ? dot_u<DM>(mi, mj, d) : sim_ij<DM>(A.sim, mi, li, 1.f, mj, lj, 1.f, d);
      const float sv = S / A.tau;
      lse_merge(ma, sa, sv, 1.f);
      const bool pos = b.ps ? (L.lab[j] != lab) : (L.lab[j] == lab);
      if (pos) lse_merge(mp, sp, sv, 1.f);
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
  // ---- publish, wait for the branch's other workgroups and the combine
  __shared__ int timed_out;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(g_nt_sync + br, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned want = gridDim.x, wantc = A.with_combine ? 1u : 0u;
    int it = 0;
    while (nt_load(g_nt_sync + br) < want || nt_load(g_nt_sync + 2) < wantc) {
      __builtin_amdgcn_s_sleep(8);
      if (++it > (1 << 20)) {
        __hip_atomic_store(g_nt_sync + 7, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    timed_out = it > (1 << 20);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  for (int j = t; j < 2 * n; j += 256) L.lse[j] = __hip_atomic_load(b.lse + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  // ---- gradients (ntxent_grad_lds_kernel's body)
  float cnt = 0.f;
  double lsum = 0.0;
  for (int j = t; j < n; j += 256) {
    const float l = L.lse[j] - L.lse[n + j];
    if (isfinite(l)) {
      cnt += 1.f;
      lsum += (double)l;
    }
  }
  const float nf = block_sum<256>(cnt, scratch);
  if (blockIdx.x == 0) {
    const double tot = block_sum<256>(lsum, dscratch);
    if (t == 0 && b.loss_out) b.loss_out[0] = (nf > 0.f) ? (float)(tot / (double)nf) : NAN;
  }
  if (b.dmu) {
    const float gup = b.gmul * (b.gscale ? b.gscale[0] : 1.0f);
    const float c = (nf > 0.f) ? gup / (nf * A.tau) : 0.f;
    for (int i = blockIdx.x * A.rpb + w; i < iend; i += 4) {
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
        const float sv = S / A.tau;
        const bool pos = b.ps ? (L.lab[j] != lab) : (L.lab[j] == lab);
        const float la_j = L.lse[j], lp_j = L.lse[n + j];
        const bool fin_j = isfinite(la_j - lp_j);
        float G = 0.f;
        if (fin_i) G += c * (expf(sv - la_i) - (pos ? expf(sv - lp_i) : 0.f));
        if (fin_j) G += c * (expf(sv - la_j) - (pos ? expf(sv - lp_j) : 0.f));
        if (G != 0.f) {
          if (cosine) {
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
  // ---- the last workgroup out resets the counters for the next launch
  __syncthreads();
  if (t == 0) {
    const unsigned tot = (unsigned)A.nbr * gridDim.x;
    if (__hip_atomic_fetch_add(g_nt_sync + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == tot - 1) {
      __hip_atomic_store(g_nt_sync + 0, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(g_nt_sync + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(g_nt_sync + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(g_nt_sync + 3, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  (void)timed_out;
}

// fraction of the device's resident slots the fused grid may use (CV_NT_FILL, percent; default 100)
static double nt_fused_fill() {
  static double f = -1.0;
  if (f < 0) {
    const char* e = getenv("CV_NT_FILL");
    f = e ? atof(e) / 100.0 : 1.0;
  }
  return f;
}

// one launch for rows + gradients when the whole grid is resident at once; -1 otherwise
static int ntxent_launch_fused(const NtArgs& a, int nbr, hipStream_t st) {
  // measured slower (MNIST latent step 35.2 -> 42.2 us) and its bounded grid-wide wait proceeds on a timeout
  // (g_nt_sync[7]) with partial sums that no host code reads back: only in a diagnostic build
  // (-DCV_GRID_WAIT_AB=1), where CV_NT_FUSED=1 selects it for an A/B run; never in the shipped library
#if defined(CV_GRID_WAIT_AB) && CV_GRID_WAIT_AB
  static int mode = -1;
  if (mode < 0) {
    const char* e = getenv("CV_NT_FUSED");
    mode = e ? atoi(e) : 0;
  }
  if (!mode) return -1;
#else
  return -1;
#endif
  const bool need_lv = !(a.sim == CV_SIM_COSINE || a.sim == CV_SIM_L2);
  size_t lds = ntl_bytes(a.n, a.d, need_lv, true);
  if (lds > 144 * 1024) return -1;
  if (lds < 16 * sizeof(double)) lds = 16 * sizeof(double);
  NtArgs arg = a;
  arg.rpb = NTL_ROWS;
  arg.nbr = nbr;
  const dim3 grid(cdiv(a.n, arg.rpb), nbr + (a.with_combine ? 1 : 0));
  const void* kern;
  if (a.d <= 8) kern = (const void*)ntxent_fused_kernel<8>;
  else if (a.d <= 16) kern = (const void*)ntxent_fused_kernel<16>;
  else if (a.d <= 32) kern = (const void*)ntxent_fused_kernel<32>;
  else kern = (const void*)ntxent_fused_kernel<64>;
  if (lds > 64 * 1024 && hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  // every workgroup must be resident at once (half the device's slots, for the margin of other streams' kernels)
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = -1;
    (void)hipGetLastError();
  }
  int occ = 0;
  if (cus <= 0 || hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, 256, lds) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  if ((long)grid.x * grid.y > (long)occ * cus * nt_fused_fill()) return -1;
  void* params[] = {&arg};
  if (hipLaunchKernel(kern, grid, dim3(256), params, lds, st) != hipSuccess) {
    ::cv::set_error("ntxent_fused: launch failed");
    return 2;
  }
  return 0;
}

template <int DM, int JM>
__global__ __launch_bounds__(256) void ntxent_rows_reg_kernel(const NtArgs A) {
  ntxent_rows_reg_body<DM, JM>(A, blockIdx.x, blockIdx.y);
}

template <int DM, int JM>
__global__ __launch_bounds__(256) void ntxent_grad_reg_kernel(const NtArgs A) {
  ntxent_grad_reg_body<DM, JM>(A, blockIdx.x, blockIdx.y);
}

// the register-resident variants serve this batch (ntr_fits + 16-byte rows); CV_NT_REG=0: never (A/B)
static int g_nt_reg = -1;  // (cv_debug_nt_reg)
static int nt_reg_on() {
  if (g_nt_reg < 0) {
    const char* e = getenv("CV_NT_REG");
    g_nt_reg = (e && atoi(e) == 0) ? 0 : 1;
  }
  return g_nt_reg;
}
// rows per workgroup of the register variants: the workgroup's column loads serve all of them (a multiple of 4: one
// row per wave per pass).  CV_NT_ROWS overrides (A/B; MNIST step with the phases in the decoder grids: 4 / 8 rows
// 0.4992 / 0.4991 ms, 16 rows 0.5058, 32 rows 0.5369 — a longer aux workgroup becomes its grid's tail)
int ntr_rows() {
  static int r = -1;
  if (r < 0) {
    const char* e = getenv("CV_NT_ROWS");
    r = e ? atoi(e) : 4;
    if (r < 4 || r % 4) r = 4;
  }
  return r;
}

bool ntxent_reg_ok(const NtArgs& a, int nbr) {
  if (!nt_reg_on() || !ntr_fits(a.n, a.d, a.sim)) return false;
  for (int i = 0; i < nbr; ++i) {
    const Branch& b = a.br[i];
    if (b.ld % 4 || (reinterpret_cast<uintptr_t>(b.mu) & 15))
      return false;
  }
  return true;
}

template <template <int> class K>
struct DDispatch;

// LDS-staged variants when the branch fits (the common case); the global-walk kernels otherwise
static int ntxent_launch_lds(const NtArgs& a, int nbr, bool rows, hipStream_t st) {
  const bool need_lv = !(a.sim == CV_SIM_COSINE || a.sim == CV_SIM_L2);
  size_t lds = ntl_bytes(a.n, a.d, need_lv, !rows);
  if (lds > 144 * 1024) return -1;
  if (lds < 16 * sizeof(double)) lds = 16 * sizeof(double);  // (the combine block's reduction scratch)
  // one row per wave: the pair loops, not the per-block staging of the branch, dominate (16-row blocks,
  // i.e. a quarter of the blocks, measured 2x slower at MNIST bs=512)
  NtArgs arg = a;
  arg.rpb = NTL_ROWS;
  arg.nbr = nbr;
  const dim3 grid(cdiv(a.n, arg.rpb), nbr + ((rows && a.with_combine) ? 1 : 0));
  if (ntxent_reg_ok(a, nbr)) {
    arg.rpb = ntr_rows();
    const dim3 grid(cdiv(a.n, arg.rpb), nbr + ((rows && a.with_combine) ? 1 : 0));
    const void* kr = a.d <= 8 ? (rows ? (const void*)ntxent_rows_reg_kernel<8, NTR_JM> : (const void*)ntxent_grad_reg_kernel<8, NTR_JM>)
                              : (rows ? (const void*)ntxent_rows_reg_kernel<32, 4> : (const void*)ntxent_grad_reg_kernel<32, 4>);
    void* params[] = {&arg};
    note_launch(kr);
    if (hipLaunchKernel(kr, grid, dim3(256), params, 16 * sizeof(double), st) != hipSuccess) {
      ::cv::set_error("%s: launch failed", rows ? "ntxent_rows" : "ntxent_grad");
      return 2;
    }
    return 0;
  }
  const void* kern;
  if (a.d <= 8) kern = rows ? (const void*)ntxent_rows_lds_kernel<8> : (const void*)ntxent_grad_lds_kernel<8>;
  else if (a.d <= 16) kern = rows ? (const void*)ntxent_rows_lds_kernel<16> : (const void*)ntxent_grad_lds_kernel<16>;
  else if (a.d <= 32) kern = rows ? (const void*)ntxent_rows_lds_kernel<32> : (const void*)ntxent_grad_lds_kernel<32>;
  else kern = rows ? (const void*)ntxent_rows_lds_kernel<64> : (const void*)ntxent_grad_lds_kernel<64>;
  if (lds > 64 * 1024 && hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  void* params[] = {&arg};
  if (hipLaunchKernel(kern, grid, dim3(256), params, lds, st) != hipSuccess) {
    ::cv::set_error("%s: launch failed", rows ? "ntxent_rows" : "ntxent_grad");
    return 2;
  }
  return 0;
}

static int ntxent_launch(const NtArgs& a, int nbr, bool rows, hipStream_t st) {
  const int r = ntxent_launch_lds(a, nbr, rows, st);
  if (r >= 0) return r;
  if (rows && a.with_combine) {  // the global-walk kernels have no combine block
    hipLaunchKernelGGL(combine_kernel, dim3(1), dim3(1024), 0, st, a.cmb);
    CV_LAUNCH_CHECK("latent_combine");
  }
  dim3 grid(cdiv(a.n, NT_ROWS), nbr);
#define CV_NT_GLOBAL(DM_, BIG_)                                                          \
  if (rows) hipLaunchKernelGGL((ntxent_rows_kernel<DM_, BIG_>), grid, dim3(256), 0, st, a); \
  else hipLaunchKernelGGL((ntxent_grad_kernel<DM_, BIG_>), grid, dim3(256), 0, st, a);
#define CV_NT_DM(BIG_)                           \
  if (a.d <= 8) { CV_NT_GLOBAL(8, BIG_) }        \
  else if (a.d <= 16) { CV_NT_GLOBAL(16, BIG_) } \
  else if (a.d <= 32) { CV_NT_GLOBAL(32, BIG_) } \
  else { CV_NT_GLOBAL(64, BIG_) }
  if (a.n > NT_MAXN) {
    CV_NT_DM(true)
  } else {
    CV_NT_DM(false)
  }
#undef CV_NT_DM
#undef CV_NT_GLOBAL
  CV_LAUNCH_CHECK(rows ? "ntxent_rows" : "ntxent_grad");
  return 0;
}

}  // namespace cv

using namespace cv;

extern "C" int cv_reparam_forward(const float* heads, int n, int d, const float* eps, uint64_t seed, uint64_t* offset,
                                  float* z, float* eps_out, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(heads && z && n > 0 && d > 0, "reparam_forward: bad args");
  CV_REQUIRE(eps || offset, "reparam_forward: need injected eps or a device offset counter");
  long blocks = ((long)n * d + 255) / 256;  // one thread per pair of latents
  if (blocks > 64) blocks = 64;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(reparam_kernel, dim3((int)blocks), dim3(256), 0, S(stream), heads, n, d, eps, seed, offset, z,
                     eps_out);
  CV_LAUNCH_CHECK("reparam_forward");
  if (offset && eps) {  // injected noise: the counter still moves once per call
    hipLaunchKernelGGL(offset_advance_kernel, dim3(1), dim3(1), 0, S(stream), offset);
    CV_LAUNCH_CHECK("reparam_offset");
  }
  return 0;
}

extern "C" int cv_sample_forward(const float* mu, const float* logvar, long numel, const float* eps, uint64_t seed,
                                 uint64_t* offset, float* z, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(mu && logvar && z && numel > 0, "sample_forward: bad args");
  CV_REQUIRE(eps || offset, "sample_forward: need injected eps or a device offset counter");
  long g = (numel / 2 + 255) / 256 + 1;
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(sample_kernel, dim3(g), dim3(256), 0, S(stream), mu, logvar, numel, eps, seed,
                     eps ? nullptr : offset, z);
  CV_LAUNCH_CHECK("sample_forward");
  return 0;
}

extern "C" int cv_sample_backward(const float* mu, const float* z, const float* dz, long numel, float* dmu,
                                  float* dlogvar, int accumulate, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(mu && z && dz && dmu && dlogvar && numel > 0, "sample_backward: bad args");
  long g = (numel + 255) / 256;
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(sample_bwd_kernel, dim3(g), dim3(256), 0, S(stream), mu, z, dz, numel, dmu, dlogvar,
                     accumulate);
  CV_LAUNCH_CHECK("sample_backward");
  return 0;
}

extern "C" int cv_kl(const float* mu, const float* logvar, int ld, int n, int d, float* kl_out, const float* gscale,
                     float* dmu, float* dlogvar, int gld, int accumulate, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(mu && logvar && n > 0 && d > 0, "kl: bad args");
  CV_REQUIRE(!dmu == !dlogvar, "kl: dmu and dlogvar go together");
  hipLaunchKernelGGL(kl_kernel, dim3(1), dim3(1024), 0, S(stream), mu, logvar, ld, n, d, kl_out, gscale, dmu, dlogvar,
                     gld, accumulate);
  CV_LAUNCH_CHECK("kl");
  return 0;
}

extern "C" size_t cv_latent_combine_workspace_bytes(void) { return (2 * CMB_SLOTS + 1) * sizeof(double); }

// cv_latent_combine_dz's workspace: the KL slots, the tickets and the slice tiles of the dz contraction
extern "C" size_t cv_latent_combine_dz_workspace_bytes(int n, int d) {
  if (n <= 0 || d <= 0) return 0;
  const size_t tiles = (size_t)cdiv(n, 16) * cdiv(2 * d, 16);
  return (2 * CMB_SLOTS + 1 + CMB_SLOTS / 2) * sizeof(double) + tiles * CDZ_S * 256 * sizeof(float);
}

extern "C" int cv_latent_combine(const float* heads, const float* z, const float* dz, int n, int d, float beta,
                                 float loc, float scale, const int64_t* anneal_step, const double* rec_in,
                                 float* dheads, float* losses, double* work, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(heads && z && anneal_step && dheads && losses && n > 0 && d > 0, "latent_combine: bad args");
  const CombineArgs C{heads, z, dz, n, d, beta, loc, scale, anneal_step, rec_in, dheads, losses, 0};
  combine_launch(C, work, S(stream));
  CV_LAUNCH_CHECK("latent_combine");
  return 0;
}

extern "C" int cv_latent_combine_acc(const float* heads, const float* z, const float* dz, int n, int d, float beta,
                                     float loc, float scale, const int64_t* anneal_step, const double* rec_in,
                                     float* dheads, float* losses, double* work, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(heads && z && anneal_step && dheads && losses && n > 0 && d > 0, "latent_combine_acc: bad args");
  const CombineArgs C{heads, z, dz, n, d, beta, loc, scale, anneal_step, rec_in, dheads, losses, 1};
  combine_launch(C, work, S(stream));
  CV_LAUNCH_CHECK("latent_combine_acc");
  return 0;
}

extern "C" int cv_latent_combine_dz(const float* heads, const float* z, const float* dh, const float* weight,
                                    const cv_linear* lin, float beta, float loc, float scale,
                                    const int64_t* anneal_step, const double* rec_in, float* dheads, float* losses,
                                    float* dz_out, int accumulate, double* work, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(heads && z && dh && weight && lin && anneal_step && dheads && losses && work,
             "latent_combine_dz: null args");
  const int n = lin->n, K = lin->in_features, F = lin->out_features;
  CV_REQUIRE(n > 0 && K > 0 && K % 2 == 0 && F > 0 && F % 64 == 0, "latent_combine_dz: n=%d K=%d F=%d (F %% 64 == 0)",
             n, K, F);
  const int pix = lin->out_pix > 0 ? lin->out_pix : 1, ch = lin->out_ch;
  CV_REQUIRE(pix <= 1 || pix * ch == F, "latent_combine_dz: out_pix*out_ch != out_features");
  CV_REQUIRE(((uintptr_t)dh & 15) == 0, "latent_combine_dz: d(h) must be 16-byte aligned");
  static int ns0 = -1;  // F slices (CV_CDZ_S A/B: 1, 2, 4, 8)
  if (ns0 < 0) {
    const char* e = getenv("CV_CDZ_S");
    // (MNIST, same box, two rounds: 1 / 2 / 4 / 8 slices 0.4801 / 0.4779 / 0.4774 / 0.4801 ms against 0.4753 with the
    // atomic dz partials: determinism costs ~2 us there)
    ns0 = e ? atoi(e) : 4;
    if (ns0 < 1 || ns0 > CDZ_S) ns0 = CDZ_S;
  }
  int ns = ns0;
  while (ns > 1 && F % (64 * ns)) ns >>= 1;  // (F / ns: a multiple of 4 waves x 16 columns)
  CV_REQUIRE(pix <= 1 || ch % 4 == 0, "latent_combine_dz: out_ch %% 4 != 0");
  const dim3 grid((unsigned)ns, (unsigned)cdiv(n, 16), (unsigned)cdiv(K, 16));
  CV_REQUIRE((long)grid.y * grid.z <= CMB_SLOTS, "latent_combine_dz: %ld dz tiles > %d slots", (long)grid.y * grid.z,
             CMB_SLOTS);
  const CombineArgs C{heads, z, nullptr, n, K / 2, beta, loc, scale, anneal_step, rec_in, dheads, losses, accumulate};
  note_launch((const void*)combine_dz_kernel);
  hipLaunchKernelGGL(combine_dz_kernel, grid, dim3(256), 0, S(stream), C, dh, weight, F, pix, ch, ns, dz_out, work);
  CV_LAUNCH_CHECK("latent_combine_dz");
  return 0;
}

extern "C" int cv_mse_sum(const float* xhat, const float* x, int n, int per_sample, float* rec_out,
                          const float* gscale, float* dxhat, double* work, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(xhat && x && n > 0 && per_sample > 0, "mse_sum: bad args");
  const long total = (long)n * per_sample;
  long g = (total + 1023) / 1024;
  if (g > 512) g = 512;
  if (rec_out) {
    CV_REQUIRE(work != nullptr, "mse_sum: forward needs a zeroed fp64 work word");
    hipLaunchKernelGGL(mse_kernel, dim3(g), dim3(1024), 0, S(stream), xhat, x, total, n, rec_out, work);
    hipLaunchKernelGGL(mse_finish_kernel, dim3(1), dim3(64), 0, S(stream), work, n, rec_out);
  }
  if (dxhat) {
    long g2 = (total + 255) / 256;
    if (g2 > 2048) g2 = 2048;
    hipLaunchKernelGGL(mse_bwd_kernel, dim3(g2), dim3(256), 0, S(stream), xhat, x, total, n, gscale, dxhat);
  }
  CV_LAUNCH_CHECK("mse_sum");
  return 0;
}

static int ntxent_args(const cv_ntxent_branch* br, int nbr, const int64_t* label, int n, int d, int sim,
                       float temperature, int accumulate, NtArgs& a) {
  CV_REQUIRE(br && nbr >= 1 && nbr <= MAXBR && label && n > 0 && d > 0 && d <= 64, "ntxent: bad args (d<=64)");
  CV_REQUIRE(n <= NT_MAXBIG, "ntxent: batch %d > %d", n, NT_MAXBIG);
  CV_REQUIRE(sim >= CV_SIM_COSINE && sim <= CV_SIM_MAHALANOBIS, "unimplemented similarity measure.");
  memset(&a, 0, sizeof(a));
  for (int i = 0; i < nbr; ++i) {
    CV_REQUIRE(br[i].mu && br[i].lse, "ntxent: branch %d incomplete", i);
    const bool need_lv = !(sim == CV_SIM_COSINE || sim == CV_SIM_L2);
    CV_REQUIRE(!need_lv || br[i].logvar, "ntxent: this similarity needs logvar");
    a.br[i].mu = br[i].mu;
    a.br[i].lv = br[i].logvar;
    a.br[i].ld = br[i].ld;
    a.br[i].ps = br[i].ps;
    a.br[i].dmu = br[i].dmu;
    a.br[i].dlv = br[i].dlogvar;
    a.br[i].gld = br[i].gld;
    a.br[i].gscale = br[i].gscale;
    a.br[i].gmul = br[i].gmul;
    a.br[i].loss_out = br[i].loss_out;
    a.br[i].lse = br[i].lse;
  }
  a.label = label;
  a.n = n;
  a.d = d;
  a.sim = sim;
  a.tau = temperature;
  a.accumulate = accumulate;
  return 0;
}

extern "C" int cv_ntxent(const cv_ntxent_branch* br, int nbr, const int64_t* label, int n, int d, int sim,
                         float temperature, int phase, int accumulate, cv_stream_t stream) {
  clear_error();
  NtArgs a;
  if (ntxent_args(br, nbr, label, n, d, sim, temperature, accumulate, a)) return 1;
  if (phase == 0 || phase == 2) {
    if (ntxent_launch(a, nbr, true, S(stream))) return 2;
  }
  if (phase == 1 || phase == 2) {
    if (ntxent_launch(a, nbr, false, S(stream))) return 2;
  }
  return 0;
}

extern "C" int cv_ntxent_aux(const cv_ntxent_branch* br, int nbr, const int64_t* label, int n, int d, int sim,
                             float temperature, int phase, int accumulate, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(phase == 0 || phase == 1, "ntxent_aux: phase %d (0 rows, 1 gradients)", phase);
  NtArgs a;
  if (ntxent_args(br, nbr, label, n, d, sim, temperature, accumulate, a)) return 1;
  a.nbr = nbr;
  a.rpb = ntxent_reg_ok(a, nbr) ? ntr_rows() : NTL_ROWS;
  if (g_aux.set) {  // a phase no launch took (its flush was skipped): it runs now, on the stream it was queued for
    g_aux.set = 0;
    if (ntxent_launch(g_aux.a, g_aux.a.nbr, g_aux.phase == 0, g_aux.stream)) return 2;
  }
  g_aux.a = a;
  g_aux.phase = phase;
  g_aux.stream = S(stream);
  g_aux.set = 1;
  return 0;
}

extern "C" int cv_ntxent_aux_combine(const float* heads, const float* z, int n, int d, float beta, float loc,
                                     float scale, const int64_t* anneal_step, float* dheads, float* losses,
                                     cv_stream_t stream) {
  clear_error();
  (void)stream;
  CV_REQUIRE(heads && z && anneal_step && dheads && losses && n > 0 && d > 0, "ntxent_aux_combine: bad args");
  CV_REQUIRE(g_aux.set && g_aux.phase == 0, "ntxent_aux_combine: no queued phase-0 request");
  CV_REQUIRE(g_aux.a.n == n && g_aux.a.d == d, "ntxent_aux_combine: n / d differ from the queued request");
  g_aux.a.with_combine = 1;
  g_aux.a.cmb = CombineArgs{heads, z, nullptr, n, d, beta, loc, scale, anneal_step, nullptr, dheads, losses, 0};
  return 0;
}

extern "C" int cv_ntxent_aux_flush(cv_stream_t stream) {
  clear_error();
  (void)stream;
  if (!g_aux.set) return 0;
  g_aux.set = 0;
  // (on the stream the phase was queued for: a flush issued on another stream must not move it there)
  return ntxent_launch(g_aux.a, g_aux.a.nbr, g_aux.phase == 0, g_aux.stream) ? 2 : 0;
}

extern "C" int cv_ntxent_aux_discard(void) {
  const int had = g_aux.set;
  g_aux.set = 0;
  return had;
}

extern "C" int cv_ntxent_aux_pending(void) { return g_aux.set ? 1 + g_aux.phase : 0; }

extern "C" int cv_latent_step(const float* heads, const float* z, const float* dz, int n, int d, float beta,
                              float loc, float scale, const int64_t* anneal_step, const double* rec_in,
                              float* dheads, float* losses, const cv_ntxent_branch* br, int nbr,
                              const int64_t* label, int sim, float temperature, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(heads && z && anneal_step && dheads && losses && n > 0 && d > 0, "latent_step: bad args");
  NtArgs a;
  if (ntxent_args(br, nbr, label, n, d, sim, temperature, 1, a)) return 1;
  for (int i = 0; i < nbr; ++i)
    CV_REQUIRE(br[i].dmu == nullptr || (br[i].dmu >= dheads && br[i].dmu < dheads + (size_t)n * 4 * d),
               "latent_step: branch %d gradient must land in dheads", i);
  a.with_combine = 1;
  a.cmb = CombineArgs{heads, z, dz, n, d, beta, loc, scale, anneal_step, rec_in, dheads, losses, 0};
  // one launch when its grid is resident at once (ntxent_fused_kernel), else launch 1: row log-sum-exps of every
  // branch + the KL / decoder-chain seed of dheads (independent); launch 2: contrastive losses and their gradients
  // accumulated into dheads
  const int f = ntxent_launch_fused(a, nbr, S(stream));
  if (f >= 0) return f;
  if (ntxent_launch(a, nbr, true, S(stream))) return 2;
  if (ntxent_launch(a, nbr, false, S(stream))) return 2;
  return 0;
}

// test hook: the register-resident NT-Xent variants on (1) / off (0), -1 = query; returns the previous setting
extern "C" int cv_debug_nt_reg(int on) {
  const int prev = cv::nt_reg_on();
  if (on >= 0) cv::g_nt_reg = on ? 1 : 0;
  return prev;
}
