// Shared device/host helpers for libclearvae_hip.so (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>
#include <string.h>
#include "../../include/clearvae.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace cv {

// ---------------------------------------------------------------- host error plumbing
void set_error(const char* fmt, ...);
// launch log (cv_debug_kernel_log): the conv / linear launch sites record the kernel they issue
void note_launch(const void* kernel);
void clear_error();

#define CV_REQUIRE(cond, ...)                \
  do {                                       \
    if (!(cond)) {                           \
      ::cv::set_error(__VA_ARGS__);          \
      return 1;                              \
    }                                        \
  } while (0)

#define CV_LAUNCH_CHECK(name)                                                   \
  do {                                                                          \
    hipError_t e_ = hipGetLastError();                                          \
    if (e_ != hipSuccess) {                                                     \
      ::cv::set_error("%s: launch failed: %s", name, hipGetErrorString(e_));    \
      return 2;                                                                 \
    }                                                                           \
  } while (0)

static inline hipStream_t S(cv_stream_t s) { return reinterpret_cast<hipStream_t>(s); }
static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// Division by a runtime-invariant divisor as multiply-high + add + shift ("division by invariant
// integers"): valid for 0 <= n < 2^31.  The igemm hot loops divide by channel / tap / pixel counts
// per K tile; as v_div sequences those were ~20x the MFMA instruction count (PMC SQ_INSTS_VALU).
struct FDiv {
  uint32_t d, m, s;
  __host__ __device__ static FDiv make(uint32_t d) {
    FDiv f;
    f.d = d < 1 ? 1 : d;
    uint32_t s = 0;
    while ((1ull << s) < f.d) ++s;
    f.s = s;
    f.m = (uint32_t)((((1ull << 32) * ((1ull << s) - f.d)) / f.d) + 1);
    return f;
  }
  __device__ __forceinline__ int div(int n) const {
    const uint32_t t = __umulhi((uint32_t)n, m);
    return (int)((t + (uint32_t)n) >> s);
  }
  __device__ __forceinline__ int mod(int n) const { return n - div(n) * (int)d; }
};

// generic conv geometry: small grid S (hs x ws x cs), big grid B (hb x wb x cb), yb = ys*s - p + kh.
// Conv2d: small = output, big = input; ConvTranspose2d: small = input, big = output.
struct Geo {
  int n, hs, ws, cs, hb, wb, cb, kh, kw, s, p;
};

// direct (VALU) kernels for convs with <= 4 channels on one side (cv_narrow.hip); return -1 when
// the geometry is not one they serve, else 0 / error code
int narrow_gather(const Geo& g, const cv_operand* in, const float* wg, const float* bias, float* out,
                  const cv_epilogue* ep, hipStream_t st);
int narrow_scatter(const Geo& g, const cv_operand* in, const float* ws, const float* bias, float* out,
                   const cv_epilogue* ep, hipStream_t st);
// LDS-banded kernels for the image-side convs (<= 4 big-grid channels, 32 small-grid channels;
// cv_edge.hip); -1 when the geometry is not one they serve
int edge_gather(const Geo& g, const cv_operand* in, const float* wg, const float* bias, float* out,
                const cv_epilogue* ep, hipStream_t st);
int edge_scatter(const Geo& g, const cv_operand* in, const float* ws, const float* bias, float* out,
                 const cv_epilogue* ep, hipStream_t st);
int edge_wgrad(const Geo& g, const cv_operand* small, const cv_operand* big, float* gw, float* gbias, float* work,
               size_t work_bytes, hipStream_t st);
size_t edge_wgrad_ws_bytes(const Geo& g, bool bias);
int edge_scatter_out(const Geo& g, const cv_operand* in, const float* ws, const float* bias, float* out,
                     const cv_epilogue* ep, const cv_bn* obn, const float* x, float* xhat, double* rec_out, float* dv,
                     double* gstat, const float* rec_scale, hipStream_t st);
int edge_bwd(const Geo& g, const cv_operand* gout, const float* wg, float* gin, const cv_epilogue* ep,
             const cv_operand* x, float* gw, float* work, size_t work_bytes, hipStream_t st);

// class-fused direct SCATTER (cv_direct.hip): stride-2 Conv2d backward-data / ConvTranspose2d forward with the
// small-grid operand staged in LDS once per workgroup; wk = the k-contiguous packing [tap][cb][cs]; -1 when the
// call is not one it serves
int direct_scatter(const Geo& g, const cv_operand* in, const float* wk, const float* bias, float* out,
                   const cv_epilogue* ep, hipStream_t st, int mma);
// the same for a stride-2 GATHER (Conv2d forward / ConvTranspose2d backward-data); wk = the `scatter` packing
// [tap][cs][cb]
// dual launch (cv_dual.hip): between dual_begin and dual_end this thread's next direct backward-data launch and
// next GEMM-core weight-gradient launch are captured; dual_end issues them as one grid when the pair is served,
// else back to back (issue = false: drops them, after an error)
void dual_begin();
int dual_end(hipStream_t st, bool issue, hipStream_t side = nullptr);
// the capture between dual_begin and dual_end will issue its weight gradient on a side stream (tile plan without the
// dual grid's row cap where no dual grid will be served)
void dual_side(bool on);
// the largest weight-gradient tile rows for the current capture (0: no cap)
int dual_wgrad_bm_cap();
int direct_gather(const Geo& g, const cv_operand* in, const float* wk, const float* bias, float* out,
                  const cv_epilogue* ep, hipStream_t st, int mma);

// ---------------------------------------------------------------- wave64 reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide sum for blockDim.x == NT (multiple of 64); scratch >= NT/64 entries; result in all threads
template <int NT, class T>
__device__ __forceinline__ T block_sum(T v, T* scratch) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  T r = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += scratch[i];
  return r;
}

// ---------------------------------------------------------------- BatchNorm constants
// Per-feature constants derived from the fp64 replica sums (or running stats in eval mode).
struct BnFwdC { float sc, mu, be, istd; };      // a = max((x - mu)*sc + be, 0), sc = gamma*istd
struct BnBwdC { float sc, mu, istd, c1, c2; };   // dy = sc*(dz - c1 - (y-mu)*istd*c2)

// mean / istd of feature c from its (replica-folded) fp64 sums (train) or the running stats (eval)
__device__ __forceinline__ void bn_mean_istd_s(const cv_bn& b, int c, double s, double q, float& mean, float& istd) {
  if (b.train) {
    const double inv_n = 1.0 / (double)b.count;
    const double m = s * inv_n;
    double var = q * inv_n - m * m;
    if (var < 0.0) var = 0.0;
    mean = (float)m;
    istd = (float)(1.0 / sqrt(var + (double)b.eps));
  } else {
    mean = b.running_mean[c];
    istd = (float)(1.0 / sqrt((double)b.running_var[c] + (double)b.eps));
  }
}

__device__ __forceinline__ BnFwdC bn_fwd_const_s(const cv_bn& b, int c, double s, double q) {
  float mean, istd;
  bn_mean_istd_s(b, c, s, q, mean, istd);
  const float g = b.gamma ? b.gamma[c] : 1.f, be = b.beta ? b.beta[c] : 0.f;
  BnFwdC r;
  r.sc = g * istd;
  r.mu = mean;
  r.be = be;
  r.istd = istd;
  return r;
}

__device__ __forceinline__ BnBwdC bn_bwd_const_s(const cv_bn& b, int c, double s, double q, double gs, double gq) {
  float mean, istd;
  bn_mean_istd_s(b, c, s, q, mean, istd);
  const float g = b.gamma ? b.gamma[c] : 1.f;
  BnBwdC r;
  r.sc = g * istd;
  r.mu = mean;
  r.istd = istd;
  r.c1 = b.train ? (float)(gs / (double)b.count) : 0.f;
  r.c2 = b.train ? (float)(gq / (double)b.count) : 0.f;
  return r;
}

// replica fold of one feature: replicas r0, r0+G, ... < R of [R][2][C] (loads issued 4 at a time)
__device__ __forceinline__ void bn_sums_g(const double* st, int C, int c, int r0, int G, int R, double& s, double& q) {
  s = 0.0;
  q = 0.0;
  if (!st) return;
  int r = r0;
  for (; r + 3 * G < R; r += 4 * G) {
    const double* p0 = st + (size_t)r * 2 * C + c;
    const size_t d = (size_t)G * 2 * C;
    const double a0 = p0[0], a1 = p0[d], a2 = p0[2 * d], a3 = p0[3 * d];
    const double b0 = p0[C], b1 = p0[d + C], b2 = p0[2 * d + C], b3 = p0[3 * d + C];
    s += (a0 + a1) + (a2 + a3);
    q += (b0 + b1) + (b2 + b3);
  }
  for (; r < R; r += G) {
    s += st[(size_t)r * 2 * C + c];
    q += st[(size_t)r * 2 * C + C + c];
  }
}

__device__ __forceinline__ void bn_sums(const double* st, int C, int c, double& s, double& q) {
  bn_sums_g(st, C, c, 0, 1, CV_STAT_REPL(C), s, q);
}

__device__ __forceinline__ void bn_mean_istd(const cv_bn& b, int c, float& mean, float& istd) {
  double s = 0.0, q = 0.0;
  if (b.train) bn_sums(b.stat, b.C, c, s, q);
  bn_mean_istd_s(b, c, s, q, mean, istd);
}

__device__ __forceinline__ BnFwdC bn_fwd_const(const cv_bn& b, int c) {
  double s = 0.0, q = 0.0;
  if (b.train) bn_sums(b.stat, b.C, c, s, q);
  return bn_fwd_const_s(b, c, s, q);
}

__device__ __forceinline__ BnBwdC bn_bwd_const(const cv_bn& b, int c) {
  double s = 0.0, q = 0.0, gs = 0.0, gq = 0.0;
  if (b.train) {
    bn_sums(b.stat, b.C, c, s, q);
    bn_sums(b.gstat, b.C, c, gs, gq);
  }
  return bn_bwd_const_s(b, c, s, q, gs, gq);
}

// Block-cooperative replica fold: calls fn(f, s, q, gs, gq) once per feature f < b.C with the
// replica-summed fp64 sums (zeros in eval mode).  Narrow layers (many replicas) spread each
// feature's replicas over G threads and combine the partials through `scratch` (>= 4*NT doubles of
// LDS that is not live yet).  Every thread of the block must call it; it ends with a barrier.
template <int NT, typename Fn>
__device__ __forceinline__ void bn_fold(const cv_bn& b, bool with_g, double* scratch, Fn fn) {
  const int C = b.C, t = threadIdx.x;
  const int R = CV_STAT_REPL(C);
  int G = 1;
  if (b.train)
    while (2 * G * C <= NT && 2 * G <= R) G *= 2;
  if (G == 1) {
    for (int f = t; f < C; f += NT) {
      double s = 0.0, q = 0.0, gs = 0.0, gq = 0.0;
      if (b.train) {
        bn_sums(b.stat, C, f, s, q);
        if (with_g) bn_sums(b.gstat, C, f, gs, gq);
      }
      fn(f, s, q, gs, gq);
    }
  } else {
    const int f = t / G, j = t - f * G;
    double s = 0.0, q = 0.0, gs = 0.0, gq = 0.0;
    if (f < C) {
      bn_sums_g(b.stat, C, f, j, G, R, s, q);
      if (with_g) bn_sums_g(b.gstat, C, f, j, G, R, gs, gq);
    }
    scratch[t] = s;
    scratch[NT + t] = q;
    scratch[2 * NT + t] = gs;
    scratch[3 * NT + t] = gq;
    __syncthreads();
    if (t < C) {
      double a = 0.0, bq = 0.0, c = 0.0, d = 0.0;
      for (int i = 0; i < G; ++i) {
        a += scratch[t * G + i];
        bq += scratch[NT + t * G + i];
        c += scratch[2 * NT + t * G + i];
        d += scratch[3 * NT + t * G + i];
      }
      fn(t, a, bq, c, d);
    }
  }
  __syncthreads();
}

// Last-arriver finalisation of a BatchNorm layer's constants (include/clearvae.h, cv_bn.ticket).
// EVERY thread of EVERY workgroup of a launch that produces BN sums calls this exactly once, after its
// own statistics atomics, in uniform control flow.  The last workgroup to arrive folds the replicas
// (`produced` = the sums this launch accumulated: the forward sums, or the backward sums with b.stat
// holding the forward ones) and writes cfwd = [sc][mu][beta][istd] or cbwd = [sc][c1][mu][istd][c2].
// Hand-off (cdna_hip_programming.md, Guideline 16): every wave drains its atomics (vmcnt(0)) before
// the barrier, one lane adds to the ticket (agent scope), the electee acquires before its loads.
// scratch: >= 4*NT doubles of LDS that are no longer live; flag: one int of LDS.
// bn_finalize_at: the launch's workgroups counted as `nblk` with this one as `me` (a launch that runs another
// kernel's workgroups beside these, cv_dual.hip, counts only its own role's).
template <int NT>
__device__ __forceinline__ void bn_finalize_at(cv_bn b, const double* produced, bool bwd, double* scratch, int* flag,
                                               unsigned me, unsigned nblk) {
  float* out = bwd ? b.cbwd : b.cfwd;
#ifdef CV_NO_FINALIZE  // A/B build: no producer-side finalisation (every consumer folds the replicas)
  return;
#endif
  if (!b.ticket || !out || !b.train || !produced) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    // two-level arrival count: <= 64 groups of gsz consecutive workgroups; the last of a group
    // arrives at ticket[dir], the last group elects the finalising workgroup
    const unsigned gsz = (nblk + 63) / 64, ngrp = (nblk + gsz - 1) / gsz, grp = me / gsz;
    const unsigned gcnt = (grp + 1 == ngrp) ? nblk - grp * gsz : gsz;
    unsigned* gctr = b.ticket + 2 + (bwd ? 64 : 0) + grp;
    bool last = false;
    if (__hip_atomic_fetch_add(gctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gcnt - 1)
      last = __hip_atomic_fetch_add(b.ticket + (bwd ? 1 : 0), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             ngrp - 1;
    *flag = last ? 1 : 0;
    if (last) {  // acquire once, before the barrier that publishes the flag to the block
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!*flag) return;
  if (bwd) b.gstat = produced;
  else b.stat = produced;
  const int C = b.C;
  if (!bwd) {
    bn_fold<NT>(b, false, scratch, [&](int f, double s, double q, double, double) {
      const BnFwdC k = bn_fwd_const_s(b, f, s, q);
      out[f] = k.sc;
      out[C + f] = k.mu;
      out[2 * C + f] = k.be;
      out[3 * C + f] = k.istd;
    });
  } else {
    bn_fold<NT>(b, true, scratch, [&](int f, double s, double q, double gs, double gq) {
      const BnBwdC k = bn_bwd_const_s(b, f, s, q, gs, gq);
      out[f] = k.sc;
      out[C + f] = k.c1;
      out[2 * C + f] = k.mu;
      out[3 * C + f] = k.istd;
      out[4 * C + f] = k.c2;
    });
  }
}

template <int NT>
__device__ __forceinline__ void bn_finalize(cv_bn b, const double* produced, bool bwd, double* scratch, int* flag) {
  bn_finalize_at<NT>(b, produced, bwd, scratch, flag, blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z),
                     gridDim.x * gridDim.y * gridDim.z);
}

// (x - mu) first: the subtraction is exact for x near mu, so the sign test of a near-zero BN output
// (the ReLU mask) agrees with an fp64 evaluation far more often than x*sc + (beta - mu*sc) does.
__device__ __forceinline__ float bn_out(float x, BnFwdC k) { return fmaf(x - k.mu, k.sc, k.be); }
__device__ __forceinline__ float bn_relu(float x, BnFwdC k) { return fmaxf(bn_out(x, k), 0.f); }
__device__ __forceinline__ float bn_bwd(float dz, float y, BnBwdC k) {
  return k.sc * (dz - k.c1 - (y - k.mu) * k.istd * k.c2);
}

__device__ __forceinline__ void atomic_add_f64(double* p, double v) { atomicAdd(p, v); }

// ---------------------------------------------------------------- Philox4x32-10 + Box-Muller
struct u32x4 { uint32_t x, y, z, w; };
__device__ __forceinline__ u32x4 philox(uint64_t key, uint64_t ctr_hi, uint64_t ctr_lo) {
  uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
  uint32_t c0 = (uint32_t)ctr_lo, c1 = (uint32_t)(ctr_lo >> 32);
  uint32_t c2 = (uint32_t)ctr_hi, c3 = (uint32_t)(ctr_hi >> 32);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
    const uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
    const uint32_t n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
    c0 = n0; c1 = l1; c2 = n2; c3 = l0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}
__device__ __forceinline__ float u01(uint32_t v) {  // (0,1]
  return ((float)(v >> 8) + 1.0f) * (1.0f / 16777216.0f);
}
// two standard normals from one Philox draw
__device__ __forceinline__ void normal2(uint64_t seed, uint64_t offset, uint64_t idx, float& a, float& b) {
  const u32x4 r = philox(seed, offset, idx);
  const float u1 = u01(r.x), u2 = u01(r.y);
  const float rad = sqrtf(-2.0f * logf(u1));
  float s, c;
  sincosf(6.283185307179586f * u2, &s, &c);
  a = rad * c;
  b = rad * s;
}

}  // namespace cv
