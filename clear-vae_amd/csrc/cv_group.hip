// GVAE / ML-VAE group evidence on gfx950 (reference code/src/models/vae.py:159-223 and the
// HierarchicalVAETrainer step, code/src/trainer.py:326-353), as segmented reductions over the batch's
// labels with no host round trip:
//   segment : pos(s) = #{j: label_j < label_s} + #{j < s: label_j == label_s}  (the reference's order:
//             groups by sorted unique label, members by ascending index, vae.py:163-172 + 202-223),
//             order[pos(s)] = s, group ids / segment starts by a block scan of the label boundaries
//   evidence: per (group, dim) one wave: GVAE mean / logsumexp - log|g|; ML-VAE precision-weighted
//             mean and -logsumexp(-logvar)
//   reparam : z_c[s] = mu_g + eps[pos(s)] * exp(lv_g/2) (eps rows in group order, as the reference's
//             per-group torch.randn), z_s[s] = mu_s + eps * exp(lv_s/2)
//   backward: KL over the m group rows, the B/m adjustment of rec / kl_s (trainer.py:322-324, 345-347),
//             the reparam chain summed per segment, then back through the evidence to every member.
// One workgroup of 1024 threads does the whole problem (n <= 32768, d <= 64; labels staged in LDS up to 4096), so
// the segmentation needs no grid-wide synchronisation and every reduction has a fixed order.
#include "cv_common.hpp"

namespace cv {

constexpr int GR_NT = 1024;
constexpr int GR_NW = GR_NT / 64;
constexpr int GR_MAXN = 4096;     // largest batch whose labels the forward stages in LDS
constexpr int GR_MAXBIG = 32768;  // largest batch at all (the segmentation is O(n^2) in one workgroup)
constexpr int GR_MAXD = 64;

struct GroupLayout {
  int* hdr;     // [0] = m (groups), [1] = n
  int* gid;     // [n] group of sample s
  int* pos;     // [n] position of s in group order
  int* order;   // [n] sample at group-order position r
  int* start;   // [n + 1] first position of group g (start[m] = n)
  float* gstat; // [n][2d] group rows mu_g | lv_g (first m valid)
};

__host__ __device__ inline GroupLayout group_layout(void* work, int n) {
  char* p = (char*)work;
  GroupLayout L;
  L.hdr = (int*)p;
  p += 64;
  L.gid = (int*)p;
  p += 4 * (size_t)n;
  L.pos = (int*)p;
  p += 4 * (size_t)n;
  L.order = (int*)p;
  p += 4 * (size_t)n;
  L.start = (int*)p;
  p += 4 * ((size_t)n + 1);
  p = (char*)(((uintptr_t)p + 15) & ~(uintptr_t)15);
  L.gstat = (float*)p;
  return L;
}

static size_t group_bytes(int n, int d) { return 64 + 16 * (size_t)n + 4 + 16 + 8 * (size_t)n * d; }

// exclusive prefix sum over the block (blockDim.x == NT); total in `total`
template <int NT>
__device__ __forceinline__ int block_excl_scan(int v, int* scratch, int& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  __syncthreads();
  if (lane == 63) scratch[w] = x;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) {
    const int c = scratch[i];
    if (i < w) base += c;
    tot += c;
  }
  total = tot;
  return base + x - v;
}

__device__ __forceinline__ float normal_at(uint64_t seed, uint64_t off, uint64_t e) {
  float a, b;
  normal2(seed, off, e >> 1, a, b);
  return (e & 1) ? b : a;
}

struct GroupFwd {
  int mode;
  const float* mu;
  const float* lv;
  int ld;
  const int64_t* label;
  int n, d;
  GroupLayout L;
  float* scale_out;
  const float* mu_s;
  const float* lv_s;
  int lds;
  const float* eps;
  int ld_eps;
  uint64_t seed;
  uint64_t* offset;
  float* z;
};

// BIG: batches above GR_MAXN (the reference has no cap, vae.py:159-223): the labels are read from global memory
// (L2-resident) instead of an LDS copy; every other step already walks the batch in workgroup strides
template <bool BIG>
__global__ __launch_bounds__(GR_NT) void group_forward_kernel(const GroupFwd A) {
  __shared__ int64_t lab_s[BIG ? 1 : GR_MAXN];
  __shared__ int scan[GR_NW];
  const int n = A.n, d = A.d, t = threadIdx.x;
  const GroupLayout& L = A.L;
  const uint64_t off = (A.offset && !A.eps) ? A.offset[0] : 0;
  const int64_t* lab = BIG ? A.label : lab_s;
  if (!BIG)
    for (int s = t; s < n; s += GR_NT) lab_s[s] = A.label[s];
  __syncthreads();
  // 1. group-order position of every sample
  for (int s = t; s < n; s += GR_NT) {
    const int64_t ls = lab[s];
    int lt = 0, eq = 0;
    for (int j = 0; j < n; ++j) {
      const int64_t lj = lab[j];
      lt += lj < ls;
      eq += (lj == ls) & (j < s);
    }
    const int p = lt + eq;
    L.pos[s] = p;
    L.order[p] = s;
  }
  __syncthreads();
  // 2. segment boundaries in group order -> group ids and starts (block scan over contiguous chunks)
  const int R = (n + GR_NT - 1) / GR_NT;
  const int r0 = t * R, r1 = min(n, r0 + R);
  int c = 0;
  for (int r = r0; r < r1; ++r) c += (r == 0 || lab[L.order[r]] != lab[L.order[r - 1]]);
  int m = 0;
  int g = block_excl_scan<GR_NT>(c, scan, m) - 1;
  for (int r = r0; r < r1; ++r) {
    if (r == 0 || lab[L.order[r]] != lab[L.order[r - 1]]) {
      ++g;
      L.start[g] = r;
    }
    L.gid[L.order[r]] = g;
  }
  if (t == 0) {
    L.start[m] = n;
    L.hdr[0] = m;
    L.hdr[1] = n;
    if (A.scale_out) A.scale_out[0] = (float)n / (float)m;
  }
  __syncthreads();
  // 3. evidence per (group, dim): one wave each
  const int lane = t & 63, w = t >> 6;
  for (int q = w; q < m * d; q += GR_NW) {
    const int gg = q / d, k = q - gg * d;
    const int s0 = L.start[gg], s1 = L.start[gg + 1];
    const float sgn = A.mode == CV_GROUP_MLVAE ? -1.f : 1.f;  // ML-VAE: the log precisions -logvar
    float mx = -INFINITY, sm = 0.f;
    for (int r = s0 + lane; r < s1; r += 64) {
      const int s = L.order[r];
      mx = fmaxf(mx, sgn * A.lv[(size_t)s * A.ld + k]);
      sm += A.mu[(size_t)s * A.ld + k];
    }
    mx = wave_max(mx);
    float se = 0.f;
    for (int r = s0 + lane; r < s1; r += 64) se += expf(sgn * A.lv[(size_t)L.order[r] * A.ld + k] - mx);
    se = wave_sum(se);
    const float lse = mx + logf(se);
    float mu_g, lv_g;
    if (A.mode == CV_GROUP_MLVAE) {
      float wm = 0.f;  // sum mu * exp(-lv) * exp(-lse): the precision-weighted mean
      for (int r = s0 + lane; r < s1; r += 64) {
        const int s = L.order[r];
        wm += A.mu[(size_t)s * A.ld + k] * expf(-A.lv[(size_t)s * A.ld + k] - lse);
      }
      mu_g = wave_sum(wm);
      lv_g = -lse;
    } else {
      mu_g = wave_sum(sm) / (float)(s1 - s0);
      lv_g = lse - logf((float)(s1 - s0));
    }
    if (lane == 0) {
      L.gstat[(size_t)gg * 2 * d + k] = mu_g;
      L.gstat[(size_t)gg * 2 * d + d + k] = lv_g;
    }
  }
  if (!A.z) return;
  __syncthreads();
  // 4. grouped reparameterisation (z_c) and the per-sample one (z_s)
  const int zd = 2 * d;
  for (int e = t; e < n * zd; e += GR_NT) {
    const int s = e / zd, j = e - s * zd;
    float mu, lv, ep;
    if (j < d) {
      const int gg = L.gid[s], r = L.pos[s];
      mu = L.gstat[(size_t)gg * zd + j];
      lv = L.gstat[(size_t)gg * zd + d + j];
      ep = A.eps ? A.eps[(size_t)r * A.ld_eps + j] : normal_at(A.seed, off, (uint64_t)r * zd + j);
    } else {
      mu = A.mu_s[(size_t)s * A.lds + j - d];
      lv = A.lv_s[(size_t)s * A.lds + j - d];
      ep = A.eps ? A.eps[(size_t)s * A.ld_eps + j] : normal_at(A.seed, off, (uint64_t)e);
    }
    A.z[e] = mu + ep * expf(0.5f * lv);
  }
  if (A.offset && !A.eps) {
    __syncthreads();
    if (t == 0) A.offset[0] = off + 1;
  }
}

// d(member heads) of one (group, dim) from d(mu_g), d(lv_g): lanes stride the group's members
__device__ __forceinline__ void evidence_members(int mode, const GroupLayout& L, int s0, int s1, const float* mu,
                                                 const float* lv, int ld, int k, float mu_g, float lv_g, float dmu_g,
                                                 float dlv_g, float* dmu, float* dlv, int ldo, int lane) {
  const float lcnt = logf((float)(s1 - s0));
  for (int r = s0 + lane; r < s1; r += 64) {
    const int s = L.order[r];
    const float l = lv[(size_t)s * ld + k];
    float gm, gl;
    if (mode == CV_GROUP_MLVAE) {
      const float ws = expf(lv_g - l);  // softmax weight of the log precision -lv
      gm = dmu_g * ws;
      gl = ws * (dlv_g - dmu_g * (mu[(size_t)s * ld + k] - mu_g));
    } else {
      gm = dmu_g / (float)(s1 - s0);
      gl = dlv_g * expf(l - lv_g - lcnt);  // softmax weight of lv
    }
    dmu[(size_t)s * ldo + k] = gm;
    dlv[(size_t)s * ldo + k] = gl;
  }
}

struct GroupBwd {
  int mode;
  const float* heads;
  const float* z;
  const float* dz;
  GroupLayout L;
  int n, d;
  float beta, loc, scale;
  const int64_t* anneal_step;
  const double* rec_in;
  float* dheads;
  float* losses;
};

// Fused HierarchicalVAETrainer latent step: heads / dheads [n][4d] = mu_c | lv_c | mu_s | lv_s.
__global__ __launch_bounds__(GR_NT) void group_backward_kernel(const GroupBwd A) {
  __shared__ double scratch[GR_NW];
  const int n = A.n, d = A.d, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const GroupLayout& L = A.L;
  const int m = L.hdr[0];
  const int zd = 2 * d, hd = 4 * d;
  const double tt = (double)A.anneal_step[0];
  // LogisticAnnealer.slope (trainer.py:32-34) in double
  const float wk = (float)((double)A.beta / (1.0 + exp(-(tt - (double)A.loc) / (double)A.scale)));
  const float inv_m = 1.0f / (float)m, inv_n = 1.0f / (float)n;
  const float adj = (float)n / (float)m;  // _group_adjust: rec and kl_s times B/m
  double kc = 0.0, ks = 0.0;
  // content half: KL over the group rows + the reparam chain summed over each segment
  for (int q = w; q < m * d; q += GR_NW) {
    const int g = q / d, k = q - g * d;
    const int s0 = L.start[g], s1 = L.start[g + 1];
    const float mu_g = L.gstat[(size_t)g * zd + k], lv_g = L.gstat[(size_t)g * zd + d + k];
    float a = 0.f, b = 0.f;
    for (int r = s0 + lane; r < s1; r += 64) {
      const int s = L.order[r];
      const float gz = A.dz[(size_t)s * zd + k];
      a += gz;
      b += gz * (A.z[(size_t)s * zd + k] - mu_g) * 0.5f;
    }
    a = wave_sum(a);
    b = wave_sum(b);
    const float el = expf(lv_g);
    const float dmu_g = wk * mu_g * inv_m + a;
    const float dlv_g = wk * (-0.5f * inv_m) * (1.0f - el) + b;
    if (lane == 0) kc += (double)(1.0f + lv_g - mu_g * mu_g - el);
    evidence_members(A.mode, L, s0, s1, A.heads, A.heads + d, hd, k, mu_g, lv_g, dmu_g, dlv_g, A.dheads,
                     A.dheads + d, hd, lane);
  }
  // style half: per-sample KL (times B/m) + reparam chain
  for (int e = t; e < n * d; e += GR_NT) {
    const int s = e / d, k = e - s * d;
    const float mu = A.heads[(size_t)s * hd + 2 * d + k], l = A.heads[(size_t)s * hd + 3 * d + k];
    const float el = expf(l);
    ks += (double)(1.0f + l - mu * mu - el);
    const float gz = A.dz[(size_t)s * zd + d + k];
    const float zz = A.z[(size_t)s * zd + d + k];
    A.dheads[(size_t)s * hd + 2 * d + k] = adj * wk * mu * inv_n + gz;
    A.dheads[(size_t)s * hd + 3 * d + k] = adj * wk * (-0.5f * inv_n) * (1.0f - el) + gz * (zz - mu) * 0.5f;
  }
  const double kct = block_sum<GR_NT>(kc, scratch);
  const double kst = block_sum<GR_NT>(ks, scratch);
  if (t == 0) {
    double r = 0.0;
    if (A.rec_in)
      for (int q = 0; q < CV_REC_REPL; ++q) r += A.rec_in[q];
    A.losses[0] = (float)((double)adj * r);
    A.losses[1] = (float)(-0.5 * kct / (double)m);
    A.losses[2] = (float)((double)adj * (-0.5 * kst / (double)n));
    A.losses[7] = wk;
  }
}

struct EvidenceBwd {
  int mode;
  const float* mu;
  const float* lv;
  int ld;
  GroupLayout L;
  int n, d;
  const float* dmu_g;
  const float* dlv_g;
  float* dmu;
  float* dlv;
  int ldo;
};

// module path: d(mu_c), d(lv_c) [n][d] from d(mu_g), d(lv_g) [m][d] (accumulate_group_evidence backward)
__global__ __launch_bounds__(GR_NT) void evidence_backward_kernel(const EvidenceBwd A) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, d = A.d;
  const GroupLayout& L = A.L;
  const int m = L.hdr[0];
  for (int q = w; q < m * d; q += GR_NW) {
    const int g = q / d, k = q - g * d;
    const float mu_g = L.gstat[(size_t)g * 2 * d + k], lv_g = L.gstat[(size_t)g * 2 * d + d + k];
    const float dm = A.dmu_g ? A.dmu_g[(size_t)g * d + k] : 0.f;
    const float dl = A.dlv_g ? A.dlv_g[(size_t)g * d + k] : 0.f;
    evidence_members(A.mode, L, L.start[g], L.start[g + 1], A.mu, A.lv, A.ld, k, mu_g, lv_g, dm, dl, A.dmu, A.dlv,
                     A.ldo, lane);
  }
}

}  // namespace cv

using namespace cv;

extern "C" size_t cv_group_workspace_bytes(int n, int d) { return n > 0 && d > 0 ? group_bytes(n, d) : 0; }

extern "C" int cv_group_forward(int mode, const float* mu_c, const float* lv_c, int ld, const int64_t* label, int n,
                                int d, void* work, float* scale_out, const float* mu_s, const float* lv_s, int lds,
                                const float* eps, int ld_eps, uint64_t seed, uint64_t* offset, float* z,
                                cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(mode == CV_GROUP_MLVAE || mode == CV_GROUP_GVAE, "group_forward: mode %d (MLVAE=0, GVAE=1)", mode);
  CV_REQUIRE(mu_c && lv_c && label && work && n > 0 && n <= GR_MAXBIG && d > 0 && d <= GR_MAXD && ld >= d,
             "group_forward: bad args (n <= %d, d <= %d)", GR_MAXBIG, GR_MAXD);
  CV_REQUIRE(!z || (mu_s && lv_s && lds >= d && (eps || offset)),
             "group_forward: z needs mu_s / lv_s and injected eps or a device offset counter");
  CV_REQUIRE(!eps || ld_eps >= 2 * d, "group_forward: eps rows hold 2d values");
  GroupFwd A;
  A.mode = mode;
  A.mu = mu_c;
  A.lv = lv_c;
  A.ld = ld;
  A.label = label;
  A.n = n;
  A.d = d;
  A.L = group_layout(work, n);
  A.scale_out = scale_out;
  A.mu_s = mu_s;
  A.lv_s = lv_s;
  A.lds = lds;
  A.eps = eps;
  A.ld_eps = ld_eps;
  A.seed = seed;
  A.offset = offset;
  A.z = z;
  if (n > GR_MAXN) hipLaunchKernelGGL(group_forward_kernel<true>, dim3(1), dim3(GR_NT), 0, S(stream), A);
  else hipLaunchKernelGGL(group_forward_kernel<false>, dim3(1), dim3(GR_NT), 0, S(stream), A);
  CV_LAUNCH_CHECK("group_forward");
  return 0;
}

extern "C" int cv_group_backward(int mode, const float* heads, const float* z, const float* dz, const void* work,
                                 int n, int d, float beta, float loc, float scale, const int64_t* anneal_step,
                                 const double* rec_in, float* dheads, float* losses, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(mode == CV_GROUP_MLVAE || mode == CV_GROUP_GVAE, "group_backward: mode %d", mode);
  CV_REQUIRE(heads && z && dz && work && anneal_step && dheads && losses && n > 0 && n <= GR_MAXBIG && d > 0 &&
                 d <= GR_MAXD,
             "group_backward: bad args");
  GroupBwd A;
  A.mode = mode;
  A.heads = heads;
  A.z = z;
  A.dz = dz;
  A.L = group_layout(const_cast<void*>(work), n);
  A.n = n;
  A.d = d;
  A.beta = beta;
  A.loc = loc;
  A.scale = scale;
  A.anneal_step = anneal_step;
  A.rec_in = rec_in;
  A.dheads = dheads;
  A.losses = losses;
  hipLaunchKernelGGL(group_backward_kernel, dim3(1), dim3(GR_NT), 0, S(stream), A);
  CV_LAUNCH_CHECK("group_backward");
  return 0;
}

extern "C" int cv_group_evidence_backward(int mode, const float* mu_c, const float* lv_c, int ld, const void* work,
                                          int n, int d, const float* dmu_g, const float* dlv_g, float* dmu_c,
                                          float* dlv_c, int ldo, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(mode == CV_GROUP_MLVAE || mode == CV_GROUP_GVAE, "group_evidence_backward: mode %d", mode);
  CV_REQUIRE(mu_c && lv_c && work && dmu_c && dlv_c && n > 0 && n <= GR_MAXBIG && d > 0 && d <= GR_MAXD &&
                 ld >= d && ldo >= d,
             "group_evidence_backward: bad args");
  EvidenceBwd A;
  A.mode = mode;
  A.mu = mu_c;
  A.lv = lv_c;
  A.ld = ld;
  A.L = group_layout(const_cast<void*>(work), n);
  A.n = n;
  A.d = d;
  A.dmu_g = dmu_g;
  A.dlv_g = dlv_g;
  A.dmu = dmu_c;
  A.dlv = dlv_c;
  A.ldo = ldo;
  hipLaunchKernelGGL(evidence_backward_kernel, dim3(1), dim3(GR_NT), 0, S(stream), A);
  CV_LAUNCH_CHECK("group_evidence_backward");
  return 0;
}
