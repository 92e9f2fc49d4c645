// The latent-side linear blocks of the fused step, each in one launch:
//   decoder input forward : z = mu + eps * exp(logvar / 2)               (VAE.sample, code/src/models/vae.py:56-60)
//                           h = Linear(z) -> BatchNorm1d -> ReLU -> ah   (vae.py:33-35; Unflatten :36 = storage order)
//   decoder input backward: ReLU mask, BatchNorm1d backward sums and transform, Linear weight gradient
//                           (dz = d(h) W stays a DENSE GEMM: it reduces over every feature)
//   encoder heads backward: d(flat) = dheads W with the last block's ReLU mask and BN backward sums, the heads'
//                           weight and bias gradients (vae.py:25-30)
//
// A workgroup owns DF = 16 storage columns of the [n][F] activation for ALL n rows.  The BatchNorm1d
// statistics of its features are therefore complete inside the workgroup: the decoder-input forward applies the
// normalisation in the same launch (it was Linear + a separate cv_bn_apply pass over h), its backward finishes
// the BN sums and goes straight on to the weight gradient (it was a mask launch with fp64 atomics plus a
// weight-gradient launch re-folding them), and every weight-gradient column is complete inside one workgroup
// (one writer, no split-K partials, deterministic).  The decoder-input forward recomputes the
// reparameterisation of the whole batch (n x 2d latents, Philox + one exp each) in every workgroup instead of
// reading a z that a separate launch would have to produce first; workgroup b stores its share of z.
//
// Arithmetic on v_mfma_f32_16x16x4_f32: the small operand (z, dheads: n x K, K <= 128) is staged in LDS at
// pitch KR + 4 (zero-padded to KR columns and 16-row tiles), the workgroup's 16 weight columns are B fragments
// in registers, and each wave walks 16-row tiles.  A fragment read is one ds_read_b128 of 4 consecutive k that
// feed 4 MFMAs (step s of a 16-k chunk contracts k = 4 (lane / 16) + s on both operands).  The weight gradients
// reuse the tile's output registers directly as the batch-side MFMA operand: lane l holds rows 4 (l / 16) + r,
// column l % 16 of a 16x16 tile, which is exactly the (k = l / 16, column l % 16) fragment of step s = r.
// Batch sums are accumulated in fp64 per lane and combined in a fixed order.
#include <type_traits>
#include "cv_common.hpp"
#include "cv_ntxent.hpp"

namespace cv {
namespace dl {

#ifndef CV_DL_NT
#define CV_DL_NT 512
#endif
constexpr int NTD = CV_DL_NT;  // 8 waves: the workgroup is alone on its CU (128 of them), so its waves hide
                               // each other's load latency and split the per-workgroup Philox draws
                               // (256 / 512 / 1024 threads: MNIST forward 22.6 / 17.0 / 17.5 us, heads backward
                               // 18.2 / 14.7 / 14.0 us; VAE64 forward 35.6 / 26.3 / 28.6 us)
constexpr int DF = 16;          // storage columns per workgroup
constexpr int NW = NTD / 64;    // waves
constexpr int ZMAX = 16384;     // latents staged in LDS (n * KR)

// CV_DL_PRE (A/B; default 1): the backward kernels issue their first batch of activation loads before staging the
// small operand (z / dheads) in LDS, so the cold activation reads' latency runs under the staging
static int dl_pre() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CV_DL_PRE");
    v = e ? atoi(e) : 1;
  }
  return v;
}

__device__ __forceinline__ int feature_of(int col, int pix, int ch) {  // PyTorch feature c*pix + p
  if (pix <= 1) return col;
  const int p = col / ch;
  return (col - p * ch) * pix + p;
}

__device__ __forceinline__ f32x4 lds4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// dst[row][KR + 4] <- src[row][K] for rows < nt*16 (zero outside [n) x [K)); 16 loads in flight per thread
template <int KR>
__device__ __forceinline__ void stage_pad(const float* __restrict__ src, int n, int K, float* dst) {
  constexpr int U = 16, P = KR + 4;
  const long total = (long)((n + 15) & ~15) * KR;
  for (long e0 = threadIdx.x; e0 < total; e0 += (long)NTD * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long e = e0 + (long)NTD * u;
      const int row = (int)(e / KR), j = (int)(e % KR);
      v[u] = (e < total && row < n && j < K) ? src[(size_t)row * K + j] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long e = e0 + (long)NTD * u;
      if (e >= total) break;
      dst[(e / KR) * P + e % KR] = v[u];
    }
  }
}

// C (16 x 16) = A[row0 .. row0 + 16)[0 .. KR) (LDS, pitch KR + 4) x B (b: this lane's B fragments,
// b[c][s] = B[16 c + 4 (lane / 16) + s][lane % 16]); lane l receives C[4 (l / 16) + r][l % 16] in [r]
template <int KR>
__device__ __forceinline__ f32x4 mma_rows(const float* sA, int row0, const f32x4* b) {
  const int l = threadIdx.x & 63;
  const float* a = sA + (row0 + (l & 15)) * (KR + 4) + 4 * (l >> 4);
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < KR / 16; ++c) {
    const f32x4 av = lds4(a + 16 * c);
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], b[c][s], acc, 0, 0, 0);
  }
  return acc;
}

// acc[jt] (16 x 16 tiles jt) += S[rows][jt*16 + i]^T (LDS, pitch KR + 4) x V[rows][lane column], rows = the 16 rows
// of the tile at row0, V = this lane's tile registers (v[r] = row 4 (lane / 16) + r): lane l receives
// [i = 4 (l / 16) + r][column l % 16]
template <int KR>
__device__ __forceinline__ void mma_rows_t(const float* sS, int row0, f32x4 v, f32x4* acc) {
  const int l = threadIdx.x & 63;
  const float* a = sS + (row0 + 4 * (l >> 4)) * (KR + 4) + (l & 15);
#pragma unroll
  for (int jt = 0; jt < KR / 16; ++jt)
#pragma unroll
    for (int s = 0; s < 4; ++s)
      acc[jt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s * (KR + 4) + 16 * jt], v[s], acc[jt], 0, 0, 0);
}

// fold a per-lane value over the 4 lanes of a column (l, l^16, l^32, l^48)
template <class T>
__device__ __forceinline__ T col_fold(T v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

struct FwdArgs {
  const float* heads;   // [n][4d] (mu_c | lv_c | mu_s | lv_s); nullptr: z is an input
  const float* eps;     // injected noise [n][2d] (test hook) or nullptr: Philox(seed, offset[0])
  uint64_t seed;
  uint64_t* offset;     // device (counter, arrival word); advanced once per launch (nullptr: none)
  float* z;             // [n][2d]
  const float* w;       // Linear weight [F][K], K = 2d
  const float* bias;    // [F]
  cv_bn bn;             // BatchNorm1d (train: batch statistics of h; eval: running statistics)
  double* stat_out;     // train: the complete sums (sum h, sum h^2) go to replica 0 of [REPL][2][F]
  float* h;             // [n][F] storage order (Linear output = BN input)
  float* ah;            // [n][F] storage order (ReLU output)
  int n, d, F, pix, ch;
};

// KR: K = 2d rounded up to a multiple of 16
// (bx, gx: the workgroup's feature block and the number of blocks: its own blockIdx / gridDim, or its share of a
// grid that also runs an NT-Xent phase, declinear_fwd_aux_kernel)
template <int KR>
__device__ __forceinline__ void declinear_fwd_body(const FwdArgs& A, const int bx, const int gx) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int P = KR + 4;
  const int K = 2 * A.d, n = A.n, F = A.F, nt = (n + 15) >> 4;
  float* sz = smem;  // [nt * 16][P]
  __shared__ double red[2][NTD / 64][DF];
  __shared__ BnFwdC kf[DF];
  const int t = threadIdx.x, l = t & 63, w = t >> 6, lr = l & 15, lq = l >> 4;
  const int col0 = bx * DF, col = col0 + lr;
  const int f = feature_of(col, A.pix, A.ch);
  const uint64_t off = A.offset ? A.offset[0] : 0;
  // ---- B fragments: W[f][k] (k = 16 c + 4 lq + s), and the bias (requested first: used last)
  f32x4 b[KR / 16];
#pragma unroll
  for (int c = 0; c < KR / 16; ++c)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int k = 16 * c + 4 * lq + s;
      b[c][s] = k < K ? A.w[(size_t)f * K + k] : 0.f;
    }
  const float bv = A.bias ? A.bias[f] : 0.f;
  // ---- latents: z = mu + eps * exp(lv / 2) (the arithmetic of reparam_kernel, element for element); every
  // global load of a batch is issued before the first use
  if (A.heads) {
    const int d = A.d;
    for (long e = t; e < (long)nt * 16 * KR; e += NTD) {  // the zero padding (disjoint from the latents)
      const int row = (int)(e / KR), j = (int)(e % KR);
      if (row >= n || j >= K) sz[row * P + j] = 0.f;
    }
    const long npair = (long)n * K / 2;  // (K even: a pair never straddles a row)
    constexpr int U = 8;
    for (long p0 = t; p0 < npair; p0 += (long)NTD * U) {
      float2 mu[U], lv[U], ep[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long p = p0 + (long)NTD * u;
        const long e = 2 * (p < npair ? p : 0);
        const int row = (int)(e / K), j = (int)(e - (long)row * K);
        const int blk = (j < d) ? 0 : 2, k = (j < d) ? j : j - d;
        const float* hr = A.heads + (size_t)row * 4 * d;
        mu[u] = *reinterpret_cast<const float2*>(hr + blk * d + k);  // (k even, d even: 8-byte aligned)
        lv[u] = *reinterpret_cast<const float2*>(hr + (blk + 1) * d + k);
        if (A.eps) ep[u] = *reinterpret_cast<const float2*>(A.eps + e);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long p = p0 + (long)NTD * u;
        if (p >= npair) break;
        if (!A.eps) normal2(A.seed, off, (uint64_t)p, ep[u].x, ep[u].y);
        const long e = 2 * p;
        const int row = (int)(e / K), j = (int)(e - (long)row * K);
        const float v0 = mu[u].x + ep[u].x * expf(0.5f * lv[u].x);
        const float v1 = mu[u].y + ep[u].y * expf(0.5f * lv[u].y);
        sz[row * P + j] = v0;
        sz[row * P + j + 1] = v1;
        if ((int)((p >> 6) % gx) == bx) {  // this workgroup's share of z
          A.z[e] = v0;
          A.z[e + 1] = v1;
        }
      }
    }
  } else {
    stage_pad<KR>(A.z, n, K, sz);
  }
  __syncthreads();
  // ---- pass 1: h and its batch sums
  double s1 = 0.0, s2 = 0.0;
  for (int tile = w; tile < nt; tile += NTD / 64) {
    const f32x4 acc = mma_rows<KR>(sz, 16 * tile, b);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * tile + 4 * lq + r;
      if (row >= n) continue;
      const float v = acc[r] + bv;
      A.h[(size_t)row * F + col] = v;
      s1 += (double)v;
      s2 += (double)v * (double)v;
    }
  }
  const bool train = A.bn.train != 0;
  s1 = col_fold(s1);
  s2 = col_fold(s2);
  if (lq == 0) {
    red[0][w][lr] = s1;
    red[1][w][lr] = s2;
  }
  __syncthreads();
  if (t < DF) {
    const int fc = feature_of(col0 + t, A.pix, A.ch);
    double S = 0.0, Q = 0.0;
    if (train) {
#pragma unroll
      for (int ww = 0; ww < NTD / 64; ++ww) {
        S += red[0][ww][t];
        Q += red[1][ww][t];
      }
      if (A.stat_out) {
        A.stat_out[fc] = S;
        A.stat_out[F + fc] = Q;
      }
    }
    kf[t] = bn_fwd_const_s(A.bn, fc, S, Q);
  }
  __syncthreads();
  // ---- pass 2: ah = ReLU(BN(h)), h recomputed (same arithmetic, same bits)
  const BnFwdC k = kf[lr];
  for (int tile = w; tile < nt; tile += NTD / 64) {
    const f32x4 acc = mma_rows<KR>(sz, 16 * tile, b);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * tile + 4 * lq + r;
      if (row < n) A.ah[(size_t)row * F + col] = bn_relu(acc[r] + bv, k);
    }
  }
  // ---- the last workgroup to finish advances the noise counter (every workgroup read it above)
  if (A.offset) {
    __syncthreads();
    if (t == 0) {
      const unsigned long long prev = atomicAdd((unsigned long long*)(A.offset + 1), 1ull);
      if (prev == (unsigned long long)(gx - 1)) {
        A.offset[0] = off + 1;
        A.offset[1] = 0;
      }
    }
  }
}
template <int KR>
__global__ __launch_bounds__(NTD) void declinear_fwd_kernel(const FwdArgs A) {
  declinear_fwd_body<KR>(A, blockIdx.x, gridDim.x);
}

struct BwdArgs {
  float* ga;            // [n][F] storage order: in d(ReLU output), out d(h) = BN1d-backward(mask * ga)
  const float* h;       // [n][F] BN input
  cv_bn bn;             // BatchNorm1d, train mode (forward sums in bn.stat)
  double* gstat_out;    // the complete backward sums (sum dz, sum dz*xhat) go to replica 0 of [REPL][2][F]
  const float* z;       // [n][K] the Linear's input
  float* gw;            // [F][K] += dW
  const float* w;       // [F][K] the Linear's weight (dz != nullptr)
  float* dz;            // [n][K] += d(h) W over the workgroup's 16 features (fp32 atomics; caller zeroes), or nullptr
  int n, K, F, pix, ch;
  int hold;  // keep pass 1's single load batch in registers for pass 2 (CV_DL_HOLD, A/B; default 1)
  int rot;   // rotate the row tiles' order by workgroup (CV_DL_ROT, A/B; default 1)
  int pre;   // dl_pre()
};

constexpr int TB = 4;  // 16-row tiles whose elementwise loads are in flight together (per wave)

template <int KR>
__device__ __forceinline__ void declinear_bwd_body(const BwdArgs& A, const int bx) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int P = KR + 4;
  const int K = A.K, n = A.n, F = A.F, nt = (n + 15) >> 4;
  float* sz = smem;                    // [nt * 16][P]
  float* sred = smem + nt * 16 * P;    // [NW waves][DF][KR]: the weight-gradient fold, then [NW][16][17] transposes
  __shared__ double red[2][NTD / 64][DF];
  __shared__ double fs[2][DF];
  __shared__ BnFwdC kf[DF];
  __shared__ BnBwdC kb[DF];
  const int t = threadIdx.x, l = t & 63, w = t >> 6, lr = l & 15, lq = l >> 4;
  const int col0 = bx * DF, col = col0 + lr;
  // Row-tile order rotated by workgroup: every workgroup adds its dz partials onto the same [n][K] rows, so in a
  // common order all of them hit one 16-row block at a time; the wave offset and the slot rotation spread them over
  // NW TB blocks.  Register slot i holds tile tile0 + NW ((i + sr) % TB): static slots, rotated tiles.
  const int wr = A.rot ? (w + bx) % NW : w, sr = A.rot ? (bx / NW) & (TB - 1) : 0;
  auto tile_at = [&](int tile0, int i) { return tile0 + NW * ((i + sr) & (TB - 1)); };
  auto load = [&](int tile0, float (*hv)[4], float (*dv)[4]) {
#pragma unroll
    for (int i = 0; i < TB; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * tile_at(tile0, i) + 4 * lq + r;
        const size_t o = (size_t)(row < n ? row : 0) * F + col;
        hv[i][r] = A.h[o];
        dv[i][r] = A.ga[o];
      }
  };
  float hv[TB][4], dv[TB][4];
  if (A.pre && wr < nt) load(wr, hv, dv);  // (in flight under the staging)
  stage_pad<KR>(A.z, n, K, sz);
  if (t < DF) {  // forward constants of the workgroup's features (replica fold, one thread per feature)
    const int fc = feature_of(col0 + t, A.pix, A.ch);
    double s, q;
    bn_sums(A.bn.stat, F, fc, s, q);
    fs[0][t] = s;
    fs[1][t] = q;
    kf[t] = bn_fwd_const_s(A.bn, fc, s, q);
  }
  __syncthreads();
  const BnFwdC k = kf[lr];
  // this lane's elements: rows 16 tile + 4 lq + r of column col, tiles w, w + 4, ...
  // ---- pass 1: ReLU mask, backward sums.  When every wave's rows fit one load batch (nt <= NW TB: MNIST / VAE64
  // at n <= 512), the batch stays in registers for pass 2 instead of being loaded again.
  double s1 = 0.0, s2 = 0.0;
  const bool held = A.hold && nt <= NW * TB;
  for (int tile0 = wr; tile0 < nt; tile0 += NW * TB) {
    if (!(A.pre && tile0 == wr)) load(tile0, hv, dv);
#pragma unroll
    for (int i = 0; i < TB; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * tile_at(tile0, i) + 4 * lq + r;
        if (row >= n) continue;
        const float dm = bn_out(hv[i][r], k) <= 0.f ? 0.f : dv[i][r];
        s1 += (double)dm;
        s2 += (double)(dm * ((hv[i][r] - k.mu) * k.istd));
      }
  }
  s1 = col_fold(s1);
  s2 = col_fold(s2);
  if (lq == 0) {
    red[0][w][lr] = s1;
    red[1][w][lr] = s2;
  }
  __syncthreads();
  if (t < DF) {
    const int fc = feature_of(col0 + t, A.pix, A.ch);
    double G1 = 0.0, G2 = 0.0;
#pragma unroll
    for (int ww = 0; ww < NTD / 64; ++ww) {
      G1 += red[0][ww][t];
      G2 += red[1][ww][t];
    }
    if (A.gstat_out) {
      A.gstat_out[fc] = G1;
      A.gstat_out[F + fc] = G2;
    }
    kb[t] = bn_bwd_const_s(A.bn, fc, fs[0][t], fs[1][t], G1, G2);
  }
  __syncthreads();
  // ---- pass 2: d(h) written in place; dW[col][k] += sum_rows d(h)[row][col] z[row][k] on the MFMA pipe
  const BnBwdC bb = kb[lr];
  f32x4 acc[KR / 16];
#pragma unroll
  for (int j = 0; j < KR / 16; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // dz partials: B fragments W[f(col0 + 4 lq + s)][16 jt + lr]; the d(h) tile goes through a wave-private LDS
  // transpose into the (row, feature) A fragment
  f32x4 wz[KR / 16];
  float* stp = sred + (size_t)NW * DF * KR + (size_t)w * 16 * 17;  // (past the fold area: waves end at different times)
  if (A.dz) {
#pragma unroll
    for (int jt = 0; jt < KR / 16; ++jt)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int fc = feature_of(col0 + 4 * lq + s, A.pix, A.ch), j = 16 * jt + lr;
        wz[jt][s] = j < K ? A.w[(size_t)fc * K + j] : 0.f;
      }
  }
  for (int tile0 = wr; tile0 < nt; tile0 += NW * TB) {
    if (!held) load(tile0, hv, dv);
#pragma unroll
    for (int i = 0; i < TB; ++i) {
      const int tile = tile_at(tile0, i);
      if (tile >= nt) continue;
      f32x4 dp;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * tile + 4 * lq + r;
        const float dm = bn_out(hv[i][r], k) <= 0.f ? 0.f : dv[i][r];
        dp[r] = row < n ? bn_bwd(dm, hv[i][r], bb) : 0.f;
        if (row < n) A.ga[(size_t)row * F + col] = dp[r];
      }
      // dW^T tile: [k][col] += z[rows][k]^T d(h)[rows][col]
      mma_rows_t<KR>(sz, 16 * tile, dp, acc);
      if (A.dz) {  // dz[rows][j] += sum over the 16 features d(h)[rows][f] W[f][j]
#pragma unroll
        for (int r = 0; r < 4; ++r) stp[(4 * lq + r) * 17 + lr] = dp[r];
        __builtin_amdgcn_wave_barrier();  // (one wave's LDS operations complete in order)
        f32x4 at;
#pragma unroll
        for (int s = 0; s < 4; ++s) at[s] = stp[lr * 17 + 4 * lq + s];
#pragma unroll
        for (int jt = 0; jt < KR / 16; ++jt) {
          f32x4 c = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < 4; ++s) c = __builtin_amdgcn_mfma_f32_16x16x4f32(at[s], wz[jt][s], c, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * tile + 4 * lq + r, j = 16 * jt + lr;
            if (row < n && j < K) atomicAdd(A.dz + (size_t)row * K + j, c[r]);
          }
        }
        __builtin_amdgcn_wave_barrier();  // (the next tile's transpose overwrites stp)
      }
    }
  }
  // lane l holds dW[col lr][k = 16 jt + 4 lq + r]: fold the waves in order
#pragma unroll
  for (int jt = 0; jt < KR / 16; ++jt)
#pragma unroll
    for (int r = 0; r < 4; ++r) sred[(w * DF + lr) * KR + 16 * jt + 4 * lq + r] = acc[jt][r];
  __syncthreads();
  for (int e = t; e < DF * K; e += NTD) {
    const int cl = e / K, kk = e - cl * K;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < NTD / 64; ++ww) v += sred[(ww * DF + cl) * KR + kk];
    A.gw[(size_t)feature_of(col0 + cl, A.pix, A.ch) * K + kk] += v;
  }
}
template <int KR>
__global__ __launch_bounds__(NTD) void declinear_bwd_kernel(const BwdArgs A) {
  declinear_bwd_body<KR>(A, blockIdx.x);
}

// The decoder-input launches with an NT-Xent phase (cv_ntxent_aux) as extra workgroups of the same grid: the row
// log-sum-exps in the forward's, the losses and gradients in the backward's.  Those grids hold one 512-thread
// workgroup per 16 features (128 for both models' 2048 features): half the CUs are idle while they run, which the
// NT-Xent workgroups take (the decoder ConvTranspose2d grids that served the phases before were full, and the
// phases cost ~9 us each there in taken slots).  The feature blocks are dispatched first; an NT-Xent
// workgroup runs the register-resident 256-thread body on its first four waves (waves 4..7 leave at once: a
// barrier waits only on the waves still running).  Results are those of the standalone launches, bit for bit (the
// same bodies on the same data).
template <int KR, int DM, int JM>
__global__ __launch_bounds__(NTD) void declinear_fwd_aux_kernel(const FwdArgs A, const NtArgs PA, const int nd,
                                                                const int agx) {
  const int v = blockIdx.x;
  if (v < nd) {
    declinear_fwd_body<KR>(A, v, nd);
    return;
  }
  if (threadIdx.x >= 256) return;
  ntxent_rows_reg_body<DM, JM>(PA, (v - nd) % agx, (v - nd) / agx);
}
template <int KR, int DM, int JM>
__global__ __launch_bounds__(NTD) void declinear_bwd_aux_kernel(const BwdArgs A, const NtArgs PA, const int nd,
                                                                const int agx) {
  const int v = blockIdx.x;
  if (v < nd) {
    declinear_bwd_body<KR>(A, v);
    return;
  }
  if (threadIdx.x >= 256) return;
  ntxent_grad_reg_body<DM, JM>(PA, (v - nd) % agx, (v - nd) / agx);
}

// ---------------------------------------------------------------- encoder heads backward
struct HeadsArgs {
  const float* dheads;  // [n][J], J = 4d
  const float* w;       // [J][F] PyTorch feature order
  const float* y;       // [n][F] storage order: the last encoder block's BN input
  cv_bn bn;             // that BatchNorm2d (C channels, pix pixels per channel)
  float* gin;           // [n][F] storage order: d(BN output) = (dheads W) * [ReLU active]
  double* gstat_out;    // [REPL][2][C] backward sums (+=)
  float* gw;            // [J][F] +=
  float* gb;            // [J] += (workgroup 0)
  int n, J, F, pix, ch;
  cv_latent_chain chain;  // chain.dz != nullptr: the decoder chain term is added to dheads while staging it
  int pre;                // dl_pre()
};

// stage_pad of dheads [n][J = 4d] with the decoder chain term of cv_latent_combine added (cv_latent_chain): column
// block b = j / d, latent k = j % d, z index zi = (b / 2) d + k; mu blocks + dz[zi], logvar blocks + dz[zi] (z[zi] -
// mu[zi]) / 2 (the combine's arithmetic: (g (z - m)) 0.5)
template <int KR>
__device__ __forceinline__ void stage_pad_chain(const float* __restrict__ src, int n, int K, const cv_latent_chain& c,
                                                float* dst) {
  constexpr int U = 8, P = KR + 4;
  const int d = c.d, zd = 2 * d;
  const long total = (long)((n + 15) & ~15) * KR;
  for (long e0 = threadIdx.x; e0 < total; e0 += (long)NTD * U) {
    float v[U], g[U], zz[U], m[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long e = e0 + (long)NTD * u;
      const int row = (int)(e / KR), j = (int)(e % KR);
      const bool ok = e < total && row < n && j < K;
      const int r = ok ? row : 0, jj = ok ? j : 0;
      const int b = jj / d, k = jj - b * d, zi = (b >> 1) * d + k;
      v[u] = ok ? src[(size_t)row * K + j] : 0.f;
      g[u] = ok ? c.dz[(size_t)r * zd + zi] : 0.f;
      zz[u] = (b & 1) ? c.z[(size_t)r * zd + zi] : 0.f;
      m[u] = (b & 1) ? c.heads[(size_t)r * K + (b - 1) * d + k] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long e = e0 + (long)NTD * u;
      if (e >= total) break;
      const int j = (int)(e % KR);
      const int b = j < K ? j / d : 0;
      dst[(e / KR) * P + j] = (b & 1) ? v[u] + g[u] * (zz[u] - m[u]) * 0.5f : v[u] + g[u];
    }
  }
}

template <int JR>
__global__ __launch_bounds__(NTD) void heads_bwd_kernel(const HeadsArgs A) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int P = JR + 4;
  const int J = A.J, n = A.n, F = A.F, C = A.ch;
  // row split (gridDim.y > 1): this workgroup takes the row tiles [tb0, tb0 + tpb) of its 16 features; the weight
  // and bias gradients then meet in device atomics (two adds onto the step's zeroed gradient: order-independent)
  const int tpb = (((n + 15) >> 4) + (int)gridDim.y - 1) / (int)gridDim.y, rbeg = 16 * tpb * (int)blockIdx.y;
  const int nl = max(0, min(n, rbeg + 16 * tpb) - rbeg), nt = (nl + 15) >> 4;
  const bool split = gridDim.y > 1;
  float* sd = smem;  // [nt * 16][P]; after the tiles: the weight-gradient fold, then the finalisation scratch
  __shared__ BnFwdC kf[DF];
  __shared__ double red[2][NTD / 64][DF];
  __shared__ int flag;
  const int t = threadIdx.x, l = t & 63, w = t >> 6, lr = l & 15, lq = l >> 4;
  const int col0 = blockIdx.x * DF, col = col0 + lr;
  const int f = feature_of(col, A.pix, C);
  float yv[TB][4];
  auto loady = [&](int tile0) {
#pragma unroll
    for (int i = 0; i < TB; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rbeg + 16 * (tile0 + NW * i) + 4 * lq + r;
        yv[i][r] = A.y[(size_t)(row < n ? row : 0) * F + col];
      }
  };
  if (A.pre && w < nt) loady(w);  // (in flight under the staging)
  f32x4 b[JR / 16];  // B fragments: W[j][f], j = 16 c + 4 lq + s
#pragma unroll
  for (int c = 0; c < JR / 16; ++c)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int j = 16 * c + 4 * lq + s;
      b[c][s] = j < J ? A.w[(size_t)j * F + f] : 0.f;
    }
  if (A.chain.dz) {
    stage_pad_chain<JR>(A.dheads, n, J, A.chain, sd);
    if (blockIdx.x == 0 && t == 0 && A.chain.rec_in && A.chain.losses) {
      double r = 0.0;
      for (int q = 0; q < CV_REC_REPL; ++q) r += A.chain.rec_in[q];
      A.chain.losses[0] = (float)r;
    }
  } else {
    stage_pad<JR>(A.dheads + (size_t)rbeg * J, nl, J, sd);
  }
  if (t < DF) {  // the layer's forward constants: finalised by its producer, or folded from the replicas
    const int cc = (col0 + t) % C;
    const cv_bn& bn = A.bn;
    if (bn.train && bn.cfwd && bn.ticket && bn.ticket[0] != 0u)
      kf[t] = BnFwdC{bn.cfwd[cc], bn.cfwd[C + cc], bn.cfwd[2 * C + cc], bn.cfwd[3 * C + cc]};
    else
      kf[t] = bn_fwd_const(bn, cc);
  }
  __syncthreads();
  const BnFwdC k = kf[lr];
  f32x4 acc[JR / 16];
#pragma unroll
  for (int j = 0; j < JR / 16; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  double s1 = 0.0, s2 = 0.0;
  for (int tile0 = w; tile0 < nt; tile0 += NW * TB) {
    if (!(A.pre && tile0 == w)) loady(tile0);
#pragma unroll
    for (int i = 0; i < TB; ++i) {
      const int tile = tile0 + NW * i;
      if (tile >= nt) break;
      const f32x4 g = mma_rows<JR>(sd, 16 * tile, b);
      f32x4 a;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rbeg + 16 * tile + 4 * lq + r;
        const float o = bn_out(yv[i][r], k);
        const float dz = o > 0.f ? g[r] : 0.f;
        a[r] = row < n ? fmaxf(o, 0.f) : 0.f;
        if (row < n) {
          A.gin[(size_t)row * F + col] = dz;
          s1 += (double)dz;
          s2 += (double)(dz * ((yv[i][r] - k.mu) * k.istd));
        }
      }
      // dW tile: [j][col] += dheads[rows][j]^T ReLU(BN(y))[rows][col]
      mma_rows_t<JR>(sd, 16 * tile, a, acc);
    }
  }
  // head biases: workgroup 0 sums the staged dheads columns, NTD / JR row groups per column (a serial walk of n
  // rows per column by JR threads was this launch's tail), folded in LDS in group order
  __shared__ float gbr[NTD];
  if (blockIdx.x == 0 && A.gb) {
    constexpr int RG = NTD / JR;
    const int j = t % JR, rgp = t / JR;
    float v = 0.f;
    if (j < J)
      for (int r = rgp; r < nl; r += RG) v += sd[r * P + j];
    gbr[t] = v;
    __syncthreads();
    if (t < J) {
      float u = 0.f;
#pragma unroll
      for (int q = 0; q < RG; ++q) u += gbr[q * JR + t];
      if (split) atomicAdd(A.gb + t, u);
      else A.gb[t] += u;
    }
  }
  s1 = col_fold(s1);
  s2 = col_fold(s2);
  if (lq == 0) {
    red[0][w][lr] = s1;
    red[1][w][lr] = s2;
  }
  __syncthreads();  // (every wave is done with sd: it becomes the fold area)
  float* sred = smem;  // [NW waves][JR][DF]
#pragma unroll
  for (int jt = 0; jt < JR / 16; ++jt)
#pragma unroll
    for (int r = 0; r < 4; ++r) sred[(w * JR + 16 * jt + 4 * lq + r) * DF + lr] = acc[jt][r];
  if (t < DF && A.gstat_out) {
    double a = 0.0, q = 0.0;
#pragma unroll
    for (int ww = 0; ww < NTD / 64; ++ww) {
      a += red[0][ww][t];
      q += red[1][ww][t];
    }
    const int cc = (col0 + t) % C;
    const int repl = blockIdx.x % CV_STAT_REPL(C);
    atomic_add_f64(A.gstat_out + (size_t)repl * 2 * C + cc, a);
    atomic_add_f64(A.gstat_out + (size_t)repl * 2 * C + C + cc, q);
  }
  __syncthreads();
  for (int e = t; e < J * DF; e += NTD) {  // e = j * DF + column: 16 consecutive columns per head output
    const int j = e / DF, cl = e - j * DF;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < NTD / 64; ++ww) v += sred[(ww * JR + j) * DF + cl];
    float* gp = A.gw + (size_t)j * F + feature_of(col0 + cl, A.pix, C);
    if (split) atomicAdd(gp, v);
    else *gp += v;
  }
  __syncthreads();  // (the fold area becomes the finalisation scratch)
  if (A.gstat_out) bn_finalize<NTD>(A.bn, A.gstat_out, true, reinterpret_cast<double*>(smem), &flag);
}

// ---------------------------------------------------------------- encoder heads forward (+ reparameterisation)
// heads = ReLU(BN(y)) W^T + b over the Flatten of the last conv block (vae.py:25-30), and, optionally, the
// reparameterisation z = mu + eps * exp(logvar / 2) of the workgroup's rows (vae.py:56-60, the arithmetic and
// the Philox pair indexing of reparam_kernel).  A workgroup owns 16 rows and one column group: the 16-column tile
// of some mu block and the tile of its logvar partner (d % 16 == 0), or, for d = 8, the one tile holding both
// (mu | logvar of 8 latents), so each latent's mu and logvar meet in one workgroup.  Its 8 waves split K (the
// F flattened features, staged straight from global in 16-byte rows with the BN + ReLU transform of the
// storage channel) and fold their partial tiles in LDS in wave order.  B comes from the heads weight packed
// [F (storage order)][4d] by the step's pack launch (cv_conv_pack with cs = 4d, cb = C, kh x kw = the pixels).
struct HeadsFwdArgs {
  const float* y;       // [n][F] storage order (pixel-major, C channels)
  cv_bn bn;             // the last conv block's BatchNorm2d (train: finalised cfwd or replica sums)
  const float* wp;      // [F][J] packed heads weight (row = storage feature)
  const float* bias;    // [J]
  float* heads;         // [n][J]
  const float* eps;     // reparameterisation: injected [n][2d] or Philox(seed, offset[0]); z == nullptr: none
  uint64_t seed;
  uint64_t* offset;
  float* z;             // [n][2d]
  int n, d, J, F, ch, ngrp, jt;  // jt: 16-column tiles per group (1: d = 8, 2: d % 16 == 0)
  int rows;                      // rows per workgroup: 16 (one MFMA row tile), or 8 (the tile's upper half idle)
};

constexpr int HF_NT = 1024;
template <int JT>
__global__ __launch_bounds__(HF_NT) void heads_fwd_kernel(const HeadsFwdArgs A) {
  constexpr int NWV = HF_NT / 64;
  __shared__ float cst[3][512];        // BN sc, mu, beta per channel (C <= 512)
  __shared__ float red[NWV][JT][16][17];
  __shared__ float hs[16][2 * 16 + 1];  // the group's summed tiles (+ bias)
  const int t = threadIdx.x, l = t & 63, w = t >> 6, lr = l & 15, lq = l >> 4;
  const int n = A.n, F = A.F, C = A.ch, d = A.d, J = A.J;
  const int rb = blockIdx.x / A.ngrp, gi = blockIdx.x - rb * A.ngrp;
  const int row0 = A.rows * rb;
  // the group's columns: tile 0 (and tile 1, the logvar partner)
  int c0[2];
  if (JT == 1) {
    c0[0] = 16 * gi;  // d = 8: [mu | logvar] of half gi
    c0[1] = c0[0];
  } else {
    const int per = d / 16, h = gi / per, m = gi - h * per;
    c0[0] = h * 2 * d + 16 * m;
    c0[1] = c0[0] + d;
  }
  const uint64_t off = (A.z && A.offset) ? A.offset[0] : 0;
  // BN constants of every channel (finalised by the producing conv, else folded)
  {
    const cv_bn& b = A.bn;
    const bool fin = b.train && b.cfwd && b.ticket && b.ticket[0] != 0u;
    for (int c = t; c < C; c += HF_NT) {
      BnFwdC k;
      if (fin) k = BnFwdC{b.cfwd[c], b.cfwd[C + c], b.cfwd[2 * C + c], b.cfwd[3 * C + c]};
      else k = bn_fwd_const(b, c);
      cst[0][c] = k.sc;
      cst[1][c] = k.mu;
      cst[2][c] = k.be;
    }
  }
  __syncthreads();
  // wave w contracts K slice [w F / NWV, (w + 1) F / NWV) in 16-wide chunks; lane (lr, lq) feeds row lr and
  // k = 16 c + 4 lq + s
  const int kper = F / NWV;  // (host: F % (16 * NWV) == 0)
  const int kb = w * kper;
  const int row = row0 + lr;
  const bool live = lr < A.rows && row < n;
  const float* yr = A.y + (size_t)(live ? row : 0) * F;
  f32x4 acc[JT];
#pragma unroll
  for (int j = 0; j < JT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int CB = 4;  // chunks per load batch
  for (int k0 = kb; k0 < kb + kper; k0 += 16 * CB) {
    f32x4 av[CB];
    float bv[CB][JT][4];
#pragma unroll
    for (int q = 0; q < CB; ++q) {
      const int k = k0 + 16 * q + 4 * lq;
      av[q] = *reinterpret_cast<const f32x4*>(yr + k);
#pragma unroll
      for (int j = 0; j < JT; ++j)
#pragma unroll
        for (int s = 0; s < 4; ++s) bv[q][j][s] = A.wp[(size_t)(k + s) * J + c0[j] + lr];
    }
#pragma unroll
    for (int q = 0; q < CB; ++q) {
      const int k = k0 + 16 * q + 4 * lq;
      const int c = k % C;  // 4 consecutive channels of one pixel (C % 4 == 0)
      f32x4 a = av[q];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        a[s] = fmaxf(fmaf(a[s] - cst[1][c + s], cst[0][c + s], cst[2][c + s]), 0.f);
        if (!live) a[s] = 0.f;
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int j = 0; j < JT; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], bv[q][j][s], acc[j], 0, 0, 0);
    }
  }
#pragma unroll
  for (int j = 0; j < JT; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w][j][4 * lq + r][lr] = acc[j][r];
  __syncthreads();
  for (int e = t; e < JT * 256; e += HF_NT) {  // fold the waves in order, add the bias, store
    const int j = e / 256, rr = (e / 16) % 16, cc = e % 16;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < NWV; ++ww) v += red[ww][j][rr][cc];
    const int col = c0[j] + cc;
    v += A.bias ? A.bias[col] : 0.f;
    hs[rr][16 * j + cc] = v;
    if (rr < A.rows && row0 + rr < n) A.heads[(size_t)(row0 + rr) * J + col] = v;
  }
  if (!A.z) return;
  __syncthreads();
  // reparameterisation of the group's latents (pair p = elements 2p, 2p + 1 of z [n][2d], as reparam_kernel)
  const int half = (JT == 1) ? gi : (c0[0] >= 2 * d ? 1 : 0);  // 0: z_c, 1: z_s
  const int lat0 = (JT == 1) ? 0 : c0[0] - half * 2 * d;      // first latent of the group within its half
  const int nl = (JT == 1) ? d : 16;                           // latents of the group
  for (int e = 2 * t; e < A.rows * nl; e += 2 * HF_NT) {
    const int rr = e / nl, m = e - rr * nl;  // (nl even: a pair stays in one row)
    const int grow = row0 + rr;
    if (grow >= n) continue;
    const int zj = half * d + lat0 + m;  // z column of the first element
    const long ez = (long)grow * 2 * d + zj;
    float e2[2];
    if (A.eps) {
      e2[0] = A.eps[ez];
      e2[1] = A.eps[ez + 1];
    } else {
      normal2(A.seed, off, (uint64_t)(ez >> 1), e2[0], e2[1]);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float mu = hs[rr][m + q];
      const float lv = hs[rr][(JT == 1 ? d : 16) + m + q];
      A.z[ez + q] = mu + e2[q] * expf(0.5f * lv);
    }
  }
  if (A.offset) {  // the last workgroup to finish advances the noise counter
    __syncthreads();
    if (t == 0) {
      const unsigned long long prev = atomicAdd((unsigned long long*)(A.offset + 1), 1ull);
      if (prev == (unsigned long long)(gridDim.x - 1)) {
        A.offset[0] = off + 1;
        A.offset[1] = 0;
      }
    }
  }
}

template <class Fn>
static int pick_kr(int K, Fn fn) {
  if (K <= 16) return fn(std::integral_constant<int, 16>());
  if (K <= 32) return fn(std::integral_constant<int, 32>());
  if (K <= 64) return fn(std::integral_constant<int, 64>());
  if (K <= 128) return fn(std::integral_constant<int, 128>());
  return -1;
}

// CV_AUX_DL (default 1): a queued NT-Xent phase rides in the decoder-input launch that follows it (0: it stays queued
// for its flush, A/B)
static int aux_dl_on() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CV_AUX_DL");
    v = e ? atoi(e) : 1;
  }
  return v;
}

// The queued NT-Xent phase (cv_ntxent_aux) this decoder-input launch on stream st can serve as extra workgroups:
// the merged kernel for (KR, phase) and the phase's arguments, or nullptr (not served: it stays queued)
template <int KR>
static const void* aux_dl_pick(int phase, hipStream_t st, NtArgs& pa, int& agx) {
  if (!g_aux.set || g_aux.phase != phase || g_aux.stream != st || !aux_dl_on() || !aux_enabled()) return nullptr;
  pa = g_aux.a;
  if (pa.with_combine || !ntxent_reg_ok(pa, pa.nbr)) return nullptr;
  const bool d8 = pa.d <= 8, d32 = pa.d <= 32 && pa.n <= 256;
  const void* fn = nullptr;
  if constexpr (KR == 16) {
    if (d8) fn = phase == 0 ? (const void*)declinear_fwd_aux_kernel<16, 8, NTR_JM> : (const void*)declinear_bwd_aux_kernel<16, 8, NTR_JM>;
  } else if constexpr (KR == 32 || KR == 64) {
    if (d32) fn = phase == 0 ? (const void*)declinear_fwd_aux_kernel<KR, 32, 4> : (const void*)declinear_bwd_aux_kernel<KR, 32, 4>;
  }
  if (!fn) return nullptr;
  agx = (pa.n + pa.rpb - 1) / pa.rpb;
  return fn;
}

static int set_lds(const void* kern, size_t bytes) {
  if (bytes <= 64 * 1024) return 0;
  if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess) {
    (void)hipGetLastError();
    return 1;
  }
  return 0;
}

}  // namespace dl
}  // namespace cv

using namespace cv;
using namespace cv::dl;

extern "C" int cv_decoder_input_supported(int n, int d, int features) {
  const int K = 2 * d;
  const int KR = K <= 16 ? 16 : K <= 32 ? 32 : K <= 64 ? 64 : 128;
  // (d even: a latent pair never straddles the c / s halves, and the heads' pairs are 8-byte aligned)
  return (n >= 1 && d >= 2 && d % 2 == 0 && K <= 128 && (long)((n + 15) & ~15) * KR <= ZMAX && features % DF == 0)
             ? 1 : 0;
}

extern "C" int cv_decoder_input_forward(const cv_linear* g, const float* heads, const float* eps, uint64_t seed,
                                        uint64_t* offset, float* z, const float* weight, const float* bias,
                                        const cv_bn* bn, double* stat_out, float* h, float* ah, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(g && z && weight && bn && h && ah, "decoder_input_forward: null args");
  CV_REQUIRE(g->in_features % 2 == 0 && g->out_features == bn->C, "decoder_input_forward: bad shapes");
  const int d = g->in_features / 2, F = g->out_features;
  CV_REQUIRE(cv_decoder_input_supported(g->n, d, F), "decoder_input_forward: n=%d, K=%d, F=%d outside the fused "
             "contract (d even, n*K <= %d, K <= 128, F %% %d == 0)", g->n, 2 * d, F, ZMAX, DF);
  CV_REQUIRE(!heads || eps || offset, "decoder_input_forward: need injected eps or a device offset counter");
  const int pix = g->out_pix > 0 ? g->out_pix : 1, ch = g->out_ch;
  CV_REQUIRE(pix <= 1 || pix * ch == F, "decoder_input_forward: out_pix*out_ch != out_features");
  FwdArgs a;
  a.heads = heads;
  a.eps = eps;
  a.seed = seed;
  a.offset = heads ? offset : nullptr;
  a.z = z;
  a.w = weight;
  a.bias = bias;
  a.bn = *bn;
  a.stat_out = bn->train ? stat_out : nullptr;
  a.h = h;
  a.ah = ah;
  a.n = g->n;
  a.d = d;
  a.F = F;
  a.pix = pix;
  a.ch = ch;
  return pick_kr(2 * d, [&](auto kr) -> int {
    constexpr int KR = decltype(kr)::value;
    const size_t lds = (size_t)((g->n + 15) & ~15) * (KR + 4) * sizeof(float);
    const void* kern = (const void*)declinear_fwd_kernel<KR>;
    NtArgs pa;
    int agx = 0;
    if (const void* fx = aux_dl_pick<KR>(0, S(stream), pa, agx)) {  // + the queued row log-sum-exps phase
      if (!set_lds(fx, lds)) {
        int nd = F / DF;
        void* params[] = {&a, &pa, &nd, &agx};
        g_aux.set = 0;
        note_launch(fx);
        if (hipLaunchKernel(fx, dim3((unsigned)(nd + agx * pa.nbr)), dim3(NTD), params, lds, S(stream)) != hipSuccess) {
          (void)hipGetLastError();
          set_error("decoder_input_forward + NT-Xent: launch failed");
          return 2;
        }
        aux_count_merged();
        return 0;
      }
      (void)hipGetLastError();
    }
    if (set_lds(kern, lds)) {
      set_error("decoder_input_forward: LDS carve-out of %zu bytes refused", lds);
      return 1;
    }
    hipLaunchKernelGGL(declinear_fwd_kernel<KR>, dim3(F / DF), dim3(NTD), lds, S(stream), a);
    CV_LAUNCH_CHECK("decoder_input_forward");
    return 0;
  });
}

extern "C" int cv_decoder_input_backward(const cv_linear* g, float* ga, const float* h, const cv_bn* bn,
                                         double* gstat_out, const float* z, float* gweight, const float* weight,
                                         float* dz, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(g && ga && h && bn && z && gweight && (!dz || weight), "decoder_input_backward: null args");
  CV_REQUIRE(bn->train && bn->stat && g->out_features == bn->C && g->in_features % 2 == 0,
             "decoder_input_backward: BN1d must be train-mode with its forward sums, C = out_features");
  const int K = g->in_features, F = g->out_features;
  CV_REQUIRE(cv_decoder_input_supported(g->n, K / 2, F), "decoder_input_backward: outside the fused contract");
  const int pix = g->out_pix > 0 ? g->out_pix : 1;
  BwdArgs a;
  a.ga = ga;
  a.h = h;
  a.bn = *bn;
  a.gstat_out = gstat_out;
  a.z = z;
  a.gw = gweight;
  a.w = weight;
  a.dz = dz;
  {
    static int abl = -1;  // CV_DL_ABLATE=1: timing probe only (wrong dz): drop the dz partial atomics
    if (abl < 0) {
      const char* e = getenv("CV_DL_ABLATE");
      abl = e ? atoi(e) : 0;
    }
    if (abl & 1) a.dz = nullptr;
    static int hold = -1;
    if (hold < 0) {
      const char* e = getenv("CV_DL_HOLD");
      hold = e ? atoi(e) : 1;
    }
    a.hold = hold;
    static int rot = -1;
    if (rot < 0) {
      const char* e = getenv("CV_DL_ROT");
      rot = e ? atoi(e) : 1;
    }
    a.rot = rot;
    a.pre = dl_pre();
  }
  a.n = g->n;
  a.K = K;
  a.F = F;
  a.pix = pix;
  a.ch = g->out_ch;
  return pick_kr(K, [&](auto kr) -> int {
    constexpr int KR = decltype(kr)::value;
    const size_t fold = (size_t)(NTD / 64) * (DF * KR + 16 * 17);  // the weight-gradient fold + the dz transposes
    const size_t lds = ((size_t)((g->n + 15) & ~15) * (KR + 4) + fold) * sizeof(float);
    const void* kern = (const void*)declinear_bwd_kernel<KR>;
    NtArgs pa;
    int agx = 0;
    if (const void* fx = aux_dl_pick<KR>(1, S(stream), pa, agx)) {  // + the queued losses / gradients phase
      if (!set_lds(fx, lds)) {
        int nd = F / DF;
        void* params[] = {&a, &pa, &nd, &agx};
        g_aux.set = 0;
        note_launch(fx);
        if (hipLaunchKernel(fx, dim3((unsigned)(nd + agx * pa.nbr)), dim3(NTD), params, lds, S(stream)) != hipSuccess) {
          (void)hipGetLastError();
          set_error("decoder_input_backward + NT-Xent: launch failed");
          return 2;
        }
        aux_count_merged();
        return 0;
      }
      (void)hipGetLastError();
    }
    if (set_lds(kern, lds)) {
      set_error("decoder_input_backward: LDS carve-out of %zu bytes refused", lds);
      return 1;
    }
    hipLaunchKernelGGL(declinear_bwd_kernel<KR>, dim3(F / DF), dim3(NTD), lds, S(stream), a);
    CV_LAUNCH_CHECK("decoder_input_backward");
    return 0;
  });
}

static size_t heads_lds(int n, int J) {
  const int JR = J <= 32 ? 32 : J <= 64 ? 64 : 128;
  size_t a = (size_t)((n + 15) & ~15) * (JR + 4) * sizeof(float);
  const size_t fold = (size_t)(NTD / 64) * DF * 128 * sizeof(float), fin = 4 * NTD * sizeof(double);
  if (a < fold) a = fold;
  if (a < fin) a = fin;
  return a;
}

extern "C" int cv_heads_backward_supported(int n, int in_features, int in_ch, int out_features) {
  return (n >= 1 && out_features >= 1 && out_features <= 128 && in_features % DF == 0 && in_ch % DF == 0 &&
          heads_lds(n, out_features) <= 150 * 1024) ? 1 : 0;
}

static int heads_backward(const cv_linear* g, const float* dheads, const cv_latent_chain* chain, const float* weight,
                          const float* y, const cv_bn* bn, float* gin, double* gstat_out, float* gweight, float* gbias,
                          cv_stream_t stream);

extern "C" int cv_heads_backward(const cv_linear* g, const float* dheads, const float* weight, const float* y,
                                 const cv_bn* bn, float* gin, double* gstat_out, float* gweight, float* gbias,
                                 cv_stream_t stream) {
  return heads_backward(g, dheads, nullptr, weight, y, bn, gin, gstat_out, gweight, gbias, stream);
}

extern "C" int cv_heads_backward_chain(const cv_linear* g, const float* dheads, const cv_latent_chain* chain,
                                       const float* weight, const float* y, const cv_bn* bn, float* gin,
                                       double* gstat_out, float* gweight, float* gbias, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(chain && chain->heads && chain->z && chain->dz && chain->d > 0, "heads_backward_chain: null chain");
  CV_REQUIRE(g && g->out_features == 4 * chain->d, "heads_backward_chain: out_features %d != 4 d (d = %d)",
             g ? g->out_features : -1, chain->d);
  return heads_backward(g, dheads, chain, weight, y, bn, gin, gstat_out, gweight, gbias, stream);
}

static int heads_backward(const cv_linear* g, const float* dheads, const cv_latent_chain* chain, const float* weight,
                          const float* y, const cv_bn* bn, float* gin, double* gstat_out, float* gweight, float* gbias,
                          cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(g && dheads && weight && y && bn && gin && gweight, "heads_backward: null args");
  const int pix = g->in_pix > 0 ? g->in_pix : 1, ch = pix > 1 ? g->in_ch : g->in_features;
  CV_REQUIRE(pix * ch == g->in_features && bn->C == ch, "heads_backward: in_pix*in_ch != in_features or BN C != in_ch");
  CV_REQUIRE(cv_heads_backward_supported(g->n, g->in_features, ch, g->out_features),
             "heads_backward: n=%d, out_features=%d outside the fused contract", g->n, g->out_features);
  HeadsArgs a;
  a.dheads = dheads;
  a.w = weight;
  a.y = y;
  a.bn = *bn;
  a.gin = gin;
  a.gstat_out = gstat_out;
  a.gw = gweight;
  a.gb = gbias;
  a.n = g->n;
  a.J = g->out_features;
  a.F = g->in_features;
  a.pix = pix;
  a.ch = ch;
  memset(&a.chain, 0, sizeof(a.chain));
  if (chain) a.chain = *chain;
  a.pre = dl_pre();
  // row splits (CV_HEADS_RS, A/B; default 1): the 128 feature workgroups leave half the CUs idle, but splitting
  // their rows measured slower — MNIST 0.4948 -> 0.4980 ms (2 splits) / 0.5056 (4), CelebA neutral / +0.7 % time —
  // the per-workgroup prologue (B fragments, the finalised constants) and the atomics outweigh the shorter tile loop.
  // The chained staging takes whole batches.
  static int rs_ovr = -2;
  if (rs_ovr == -2) {
    const char* e = getenv("CV_HEADS_RS");
    rs_ovr = e ? atoi(e) : -1;
  }
  int rs = rs_ovr > 0 ? rs_ovr : 1;
  if (chain || rs > (a.n + 15) / 16) rs = 1;
  const int rows_per = 16 * (((a.n + 15) / 16 + rs - 1) / rs);
  const size_t lds = heads_lds(rows_per, a.J);
  auto go = [&](auto jr) -> int {
    constexpr int JR = decltype(jr)::value;
    const void* kern = (const void*)heads_bwd_kernel<JR>;
    if (set_lds(kern, lds)) {
      set_error("heads_backward: LDS carve-out of %zu bytes refused", lds);
      return 1;
    }
    hipLaunchKernelGGL(heads_bwd_kernel<JR>, dim3(a.F / DF, rs), dim3(NTD), lds, S(stream), a);
    CV_LAUNCH_CHECK("heads_backward");
    return 0;
  };
  if (a.J <= 32) return go(std::integral_constant<int, 32>());
  if (a.J <= 64) return go(std::integral_constant<int, 64>());
  return go(std::integral_constant<int, 128>());
}

extern "C" int cv_heads_forward_supported(int n, int in_features, int in_ch, int d) {
  return (n >= 1 && in_ch % 4 == 0 && in_ch <= 512 && in_features % (16 * (HF_NT / 64)) == 0 &&
          (d == 8 || (d % 16 == 0 && d <= 64))) ? 1 : 0;
}

extern "C" int cv_heads_forward(const cv_linear* g, const float* y, const cv_bn* bn, const float* wpacked,
                                const float* bias, float* heads, const float* eps, uint64_t seed, uint64_t* offset,
                                float* z, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(g && y && bn && wpacked && heads, "heads_forward: null args");
  const int pix = g->in_pix > 0 ? g->in_pix : 1, ch = pix > 1 ? g->in_ch : g->in_features;
  CV_REQUIRE(pix * ch == g->in_features && bn->C == ch && g->out_features % 4 == 0,
             "heads_forward: in_pix*in_ch != in_features, BN C != in_ch or 4d not a multiple of 4");
  const int d = g->out_features / 4;
  CV_REQUIRE(cv_heads_forward_supported(g->n, g->in_features, ch, d), "heads_forward: n=%d, F=%d, C=%d, d=%d outside "
             "the fused contract", g->n, g->in_features, ch, d);
  CV_REQUIRE(!z || eps || offset, "heads_forward: the reparameterisation needs injected eps or an offset counter");
  HeadsFwdArgs a;
  a.y = y;
  a.bn = *bn;
  a.wp = wpacked;
  a.bias = bias;
  a.heads = heads;
  a.eps = eps;
  a.seed = seed;
  a.offset = z ? offset : nullptr;
  a.z = z;
  a.n = g->n;
  a.d = d;
  a.J = g->out_features;
  a.F = g->in_features;
  a.ch = ch;
  a.jt = d == 8 ? 1 : 2;
  a.ngrp = d == 8 ? 2 : 2 * (d / 16);
  // CV_HEADS_FWD_ROWS=8 (A/B): 8-row workgroups, twice the grid where 16-row ones leave most CUs idle (MNIST bs =
  // 512 and VAE64 bs = 256: 64 workgroups) — measured neutral (MNIST 0.4953 vs 0.4942 ms, CelebA 2.1267 vs
  // 2.1271 ms: the per-workgroup constants and weight loads, not the row count, set its length), so 16
  static int rows_ovr = -2;
  if (rows_ovr == -2) {
    const char* e = getenv("CV_HEADS_FWD_ROWS");
    rows_ovr = e ? atoi(e) : -1;
  }
  a.rows = rows_ovr == 8 ? 8 : 16;
  const dim3 grid(cdiv(g->n, a.rows) * a.ngrp);
  if (a.jt == 1) hipLaunchKernelGGL(heads_fwd_kernel<1>, grid, dim3(HF_NT), 0, S(stream), a);
  else hipLaunchKernelGGL(heads_fwd_kernel<2>, grid, dim3(HF_NT), 0, S(stream), a);
  CV_LAUNCH_CHECK("heads_forward");
  return 0;
}
