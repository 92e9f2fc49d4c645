// CLEAR-TC factor discriminator (the density-ratio total-correlation term) for gfx950.
//
// Reference arithmetic replaced (scotsun/clear-vae):
//   factor_cls = Linear(z, z) -> ReLU -> Linear(z, 1) -> Sigmoid          trainer_utils.py:133-138
//   mi_loss = relu(log(d / (1 - d))).mean(), d = factor_cls(z), and its
//     gradient into the VAE through z = mu + eps * exp(logvar / 2)         trainer.py:664-677
//   factor_shuffling "permute_1" (z_s rolled up by one row)              trainer.py:573-587
//   nn.BCELoss()(cat[factor_cls(z), factor_cls(shuffled z)], cat[1, 0])
//     and its gradient w.r.t. the discriminator parameters                trainer.py:680-698
//
// One wave per row, lane j = hidden unit j (z <= 64): the first layer's weights are staged once per
// workgroup in LDS with an odd row pitch, so the row walk (forward, lane j reads row j) and the column walk
// (backward, lane k reads column k) are both conflict-free.  The scalar chain (sigmoid, ratio, log, relu and
// their backward) is evaluated in the same fp32 order as autograd over the reference's expression.
// Reductions over rows go through per-workgroup partials folded in workgroup order by one reduction
// workgroup: deterministic.
#include "cv_common.hpp"

namespace cv {

constexpr int TC_MAXZ = 64;
constexpr int TC_W = 4;          // waves (rows in flight) per workgroup
constexpr int TC_MAXB = 64;      // row workgroups whose partials are folded
constexpr int TC_NP(int z) { return z * z + 2 * z + 1; }

struct TcArgs {
  cv_tc_disc D;
  const float* z;        // [n][zdim]
  int n;
  float lam;
  const float* heads;    // [n][4d] (mu_c | lv_c | mu_s | lv_s), with dheads (VAE step)
  float* dheads;
  int d;
  float* work;           // TC workspace (cv_tc_workspace_bytes)
  float* loss_out;
  cv_tc_grad G;          // factor step: discriminator gradients (overwritten)
};

// workspace layout (floats): [0, TC_MAXB) per-workgroup loss partials; then TC_MAXB * NP gradient partials
__host__ __device__ inline size_t tc_work_floats(int z) { return (size_t)TC_MAXB + (size_t)TC_MAXB * TC_NP(z); }

struct TcLds {
  float w1[TC_MAXZ][TC_MAXZ + 1];
  float zr[TC_W][TC_MAXZ];
  float gh[TC_W][TC_MAXZ];
  float red[TC_W][TC_MAXZ + 2];
};

__device__ __forceinline__ void tc_stage(const cv_tc_disc& D, TcLds& L) {
  const int Z = D.zdim;
  for (int e = threadIdx.x; e < Z * Z; e += 256) L.w1[e / Z][e % Z] = D.w1[e];
  __syncthreads();
}

// a = W2 . relu(W1 x + b1) + b2 for the wave's row (x already in L.zr[w]); returns a, leaves pre_j / h_j
__device__ __forceinline__ float tc_row_fwd(const cv_tc_disc& D, TcLds& L, int w, int lane, float& pre, float& hj) {
  const int Z = D.zdim;
  pre = 0.f;
  if (lane < Z) {
    float s = D.b1[lane];
    for (int k = 0; k < Z; ++k) s = fmaf(L.w1[lane][k], L.zr[w][k], s);
    pre = s;
  }
  hj = fmaxf(pre, 0.f);
  const float w2 = lane < Z ? D.w2[lane] : 0.f;
  return wave_sum(w2 * hj) + D.b2[0];
}

// VAE step: mi_loss rows + gradient of lam * mi_loss into d(heads).  Row groups of TC_W rows (one per wave)
// keep the trip count uniform across the block, so the barriers are reached by every wave.
__global__ __launch_bounds__(256) void tc_vae_kernel(const TcArgs A) {
  __shared__ TcLds L;
  __shared__ float part[TC_W];
  tc_stage(A.D, L);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, Z = A.D.zdim, d = A.d;
  const float inv_n = 1.0f / (float)A.n;
  float acc = 0.f;
  for (int base = blockIdx.x * TC_W; base < A.n; base += gridDim.x * TC_W) {
    const int r = base + w;
    const bool live = r < A.n;
    if (lane < Z) L.zr[w][lane] = live ? A.z[(size_t)r * Z + lane] : 0.f;
    __syncthreads();
    float pre, hj;
    const float a = tc_row_fwd(A.D, L, w, lane, pre, hj);
    const float dsc = 1.0f / (1.0f + expf(-a));   // nn.Sigmoid
    const float om = 1.0f - dsc;
    const float ratio = dsc / om;
    const float val = logf(ratio);
    if (live) acc += fmaxf(val, 0.f);               // F.relu (summed; the mean is taken below)
    if (A.dheads) {
      // autograd of relu(log(d / (1 - d))).mean() through the same ops, then Sigmoid's backward
      const float gval = (val > 0.f ? 1.f : 0.f) * inv_n;
      const float gratio = gval / ratio;
      const float gdsc = gratio / om + gratio * dsc / (om * om);
      const float ga = gdsc * dsc * om;
      if (lane < Z) L.gh[w][lane] = (pre > 0.f) ? ga * A.D.w2[lane] : 0.f;
      __syncthreads();
      if (live && lane < Z) {
        float gz = 0.f;
        for (int j = 0; j < Z; ++j) gz = fmaf(L.w1[j][lane], L.gh[w][j], gz);
        gz *= A.lam;
        // z = (z_c | z_s): lane k < d -> content factor, else style; z = mu + eps*exp(lv/2)
        const int blk = lane < d ? 0 : 2, k = lane < d ? lane : lane - d;
        const float zz = L.zr[w][lane];
        const float mu = A.heads[(size_t)r * 4 * d + blk * d + k];
        A.dheads[(size_t)r * 4 * d + blk * d + k] += gz;
        A.dheads[(size_t)r * 4 * d + (blk + 1) * d + k] += gz * (zz - mu) * 0.5f;
      }
    }
    __syncthreads();
  }
  if (lane == 0) part[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) A.work[blockIdx.x] = (part[0] + part[1]) + (part[2] + part[3]);
}

__global__ __launch_bounds__(64) void tc_mean_kernel(const float* work, int nb, int n, float* out) {
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int b = 0; b < nb; ++b) s += work[b];  // workgroup order: deterministic
    out[0] = s / (float)n;
  }
}

// factor step rows: 2n rows (joint z_r, then marginal (z_c(r), z_s(r+1 mod n))), BCE against (1, 0),
// per-workgroup gradient partials [W1 (Z*Z) | b1 (Z) | W2 (Z) | b2 (1)] and loss partials
__global__ __launch_bounds__(256) void tc_learn_rows_kernel(const TcArgs A) {
  __shared__ TcLds L;
  __shared__ float lpart[TC_W];
  tc_stage(A.D, L);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, Z = A.D.zdim, n = A.n, half = Z / 2;
  const float inv = 1.0f / (float)(2 * n);
  float gw1[TC_MAXZ];
#pragma unroll
  for (int k = 0; k < TC_MAXZ; ++k) gw1[k] = 0.f;
  float gb1 = 0.f, gw2 = 0.f, gb2 = 0.f, lsum = 0.f;
  for (int base = blockIdx.x * TC_W; base < 2 * n; base += gridDim.x * TC_W) {
    const int r = base + w;
    const bool live = r < 2 * n;
    const bool joint = r < n;
    const int i = joint ? r : r - n;
    if (lane < Z) {
      const int src = (joint || lane < half) ? i : (i + 1 == n ? 0 : i + 1);  // factor_shuffling permute_1
      L.zr[w][lane] = live ? A.z[(size_t)src * Z + lane] : 0.f;
    }
    __syncthreads();
    float pre, hj;
    const float a = tc_row_fwd(A.D, L, w, lane, pre, hj);
    if (live) {
      const float x = 1.0f / (1.0f + expf(-a));
      const float y = joint ? 1.f : 0.f;
      // nn.BCELoss: -(y max(log x, -100) + (1-y) max(log(1-x), -100)); backward (x-y) / max((1-x)x, 1e-12)
      lsum += -(y * fmaxf(logf(x), -100.f) + (1.f - y) * fmaxf(logf(1.f - x), -100.f));
      const float gx = (x - y) / fmaxf((1.f - x) * x, 1e-12f) * inv;
      const float ga = gx * x * (1.f - x);  // Sigmoid backward
      const float ghj = (lane < Z && pre > 0.f) ? ga * A.D.w2[lane] : 0.f;
      gb2 += ga;
      gw2 += ga * hj;
      gb1 += ghj;
      if (lane < Z) {
#pragma unroll
        for (int k = 0; k < TC_MAXZ; ++k)
          if (k < Z) gw1[k] = fmaf(ghj, L.zr[w][k], gw1[k]);
      }
    }
    __syncthreads();
  }
  // fold the waves in wave order into LDS (W1's image is free now) and write the block's partial
  for (int q = 0; q < TC_W; ++q) {
    if (w == q && lane < Z) {
#pragma unroll
      for (int k = 0; k < TC_MAXZ; ++k)
        if (k < Z) L.w1[lane][k] = (q == 0 ? 0.f : L.w1[lane][k]) + gw1[k];
      L.red[0][lane] = (q == 0 ? 0.f : L.red[0][lane]) + gb1;
      L.red[1][lane] = (q == 0 ? 0.f : L.red[1][lane]) + gw2;
    }
    if (w == q && lane == 0) L.red[2][0] = (q == 0 ? 0.f : L.red[2][0]) + gb2;  // (ga is wave-uniform)
    __syncthreads();
  }
  if (lane == 0) lpart[w] = lsum;
  __syncthreads();
  float* P = A.work + TC_MAXB + (size_t)blockIdx.x * TC_NP(Z);
  for (int e = threadIdx.x; e < Z * Z; e += 256) P[e] = L.w1[e / Z][e % Z];
  for (int e = threadIdx.x; e < Z; e += 256) {
    P[Z * Z + e] = L.red[0][e];
    P[Z * Z + Z + e] = L.red[1][e];
  }
  if (threadIdx.x == 0) {
    P[Z * Z + 2 * Z] = L.red[2][0];
    A.work[blockIdx.x] = (lpart[0] + lpart[1]) + (lpart[2] + lpart[3]);
  }
}

__global__ __launch_bounds__(256) void tc_learn_reduce_kernel(const TcArgs A, int nb) {
  const int Z = A.D.zdim, NP = TC_NP(Z);
  for (int e = blockIdx.x * 256 + threadIdx.x; e < NP; e += gridDim.x * 256) {
    float s = 0.f;
    int b = 0;
    for (; b + 16 <= nb; b += 16) {  // (16 partials in flight, workgroup order kept)
      float v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = A.work[TC_MAXB + (size_t)(b + q) * NP + e];
#pragma unroll
      for (int q = 0; q < 16; ++q) s += v[q];
    }
    for (; b < nb; ++b) s += A.work[TC_MAXB + (size_t)b * NP + e];
    if (e < Z * Z) A.G.w1[e] = s;
    else if (e < Z * Z + Z) A.G.b1[e - Z * Z] = s;
    else if (e < Z * Z + 2 * Z) A.G.w2[e - Z * Z - Z] = s;
    else A.G.b2[0] = s;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && A.loss_out) {
    float s = 0.f;
    for (int b = 0; b < nb; ++b) s += A.work[b];
    A.loss_out[0] = s / (float)(2 * A.n);
  }
}

static int tc_blocks(int rows) {
  int b = cdiv(rows, TC_W * 2);
  return b < 1 ? 1 : (b > TC_MAXB ? TC_MAXB : b);
}

static int check_disc(const cv_tc_disc* D) {
  CV_REQUIRE(D && D->w1 && D->b1 && D->w2 && D->b2, "tc: discriminator weights missing");
  CV_REQUIRE(D->zdim > 0 && D->zdim <= TC_MAXZ && D->zdim % 2 == 0, "tc: latent width %d must be even, <= %d",
             D->zdim, TC_MAXZ);
  return 0;
}

}  // namespace cv

using namespace cv;

extern "C" size_t cv_tc_workspace_bytes(int zdim) { return tc_work_floats(zdim > 0 ? zdim : 1) * sizeof(float); }

extern "C" int cv_tc_forward(const cv_tc_disc* D, const float* z, int n, float lam, const float* heads,
                             float* dheads, int d, void* work, float* mi_out, cv_stream_t stream) {
  clear_error();
  if (check_disc(D)) return 1;
  CV_REQUIRE(z && n > 0 && work && mi_out, "tc_forward: bad args");
  CV_REQUIRE(!dheads || (heads && 2 * d == D->zdim), "tc_forward: the gradient chain needs heads and d = z/2");
  TcArgs a;
  memset(&a, 0, sizeof(a));
  a.D = *D;
  a.z = z;
  a.n = n;
  a.lam = lam;
  a.heads = heads;
  a.dheads = dheads;
  a.d = d;
  a.work = (float*)work;
  const int nb = tc_blocks(n);
  hipLaunchKernelGGL(tc_vae_kernel, dim3(nb), dim3(256), 0, S(stream), a);
  CV_LAUNCH_CHECK("tc_forward");
  hipLaunchKernelGGL(tc_mean_kernel, dim3(1), dim3(64), 0, S(stream), (const float*)work, nb, n, mi_out);
  CV_LAUNCH_CHECK("tc_forward.mean");
  return 0;
}

extern "C" int cv_tc_learning_step(const cv_tc_disc* D, const float* z, int n, void* work, float* loss_out,
                                   const cv_tc_grad* g, cv_stream_t stream) {
  clear_error();
  if (check_disc(D)) return 1;
  CV_REQUIRE(z && n > 1 && work && g && g->w1 && g->b1 && g->w2 && g->b2, "tc_learning_step: bad args");
  TcArgs a;
  memset(&a, 0, sizeof(a));
  a.D = *D;
  a.z = z;
  a.n = n;
  a.work = (float*)work;
  a.loss_out = loss_out;
  a.G = *g;
  const int nb = tc_blocks(2 * n);
  hipLaunchKernelGGL(tc_learn_rows_kernel, dim3(nb), dim3(256), 0, S(stream), a);
  CV_LAUNCH_CHECK("tc_learning_step.rows");
  const int np = TC_NP(D->zdim);
  hipLaunchKernelGGL(tc_learn_reduce_kernel, dim3(cdiv(np, 256)), dim3(256), 0, S(stream), a, nb);
  CV_LAUNCH_CHECK("tc_learning_step.reduce");
  return 0;
}
