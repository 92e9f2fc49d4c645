// Specialised implicit-GEMM core on fp32 MFMA (v_mfma_f32_16x16x4_f32) for gfx950.
//
// Serves the same four contractions as cv_igemm.hip (GATHER / SCATTER / WGRAD / DENSE, see there),
// restricted to vectorisable operands (channel counts that are multiples of 4, NHWC), which is every
// conv / linear layer of VAE and VAE64 except the image-facing ones.  What differs from the generic
// kernel, and why (per-block timeline stamps of the generic kernel: ~1.6 us per K tile = ~3,600
// cycles for 16 MFMAs per wave, and a 4-13 us prologue):
//   * the operand transforms (BN+ReLU forward, BN backward) and the epilogue statistics mode are
//     template parameters, so the staging code has no per-element branches;
//   * both LDS operand images are k-contiguous, [row][BK + 4]: a lane's ds_read_b128 returns the
//     4 consecutive k of its row, which feed 4 successive MFMAs (step s of a 16-k chunk uses
//     k = 4*(lane/16) + s for lane group lane/16 on both operands, so the contraction is unchanged).
//     One b128 read per 4 MFMAs instead of one b32 read per MFMA; the row pitch of 36 floats makes
//     the 16 rows of a fragment read land on 16 disjoint 4-bank groups (conflict free);
//   * every global load of a K tile is issued unconditionally (out-of-range lanes read element 0
//     and are zeroed by a select afterwards; the tail tiles re-read the last tile), so the number of
//     loads in flight is static and the compiler's vmcnt waits let D-1 tiles stay in flight across
//     the MFMA phases (a register ring of D stages; D=2 is the classic double buffer);
//   * the BatchNorm constants are folded from the fp64 replica sums into SoA LDS arrays (float4
//     reads at store time) AFTER the first tiles' loads are issued, so the fold's latency hides
//     under them.
#pragma once
#include <stdlib.h>
#include "cv_igemm.hpp"

namespace cv {
namespace fast {

constexpr int LDK = BK + 4;  // LDS row pitch (floats) of both k-contiguous operand images
// bf16 operand images (MT = MMA_BF16): the same [row][k] images with k-contiguous bf16 and an 80-byte
// row pitch, so the 16 rows of a ds_read_b128 fragment start on 16 disjoint 4-bank groups
constexpr int LDKH = BK + 8;
enum { MMA_F32 = 0, MMA_BF16 = 1 };
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ bf16x4 to_bf16x4(f32x4 v) { return __builtin_convertvector(v, bf16x4); }

__device__ __forceinline__ f32x4 lds4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ f32x4 g4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// Transposed operand staging.  Global memory holds the WGRAD A operand and every non-k-contiguous B operand
// as rows of k with the GEMM's m / n dimension contiguous, while the LDS images are [m or n][k].  A lane
// quad (lanes 4i..4i+3) fetches 4 consecutive k of one channel quad; quad_transpose turns that 4x4 block
// around with two DPP quad-permutation stages, so each lane stores 4 consecutive k of ONE row as a single
// 16-byte (bf16: 8-byte) LDS write.  16 lanes then write 16 consecutive rows of the 36-float pitch image:
// 16 disjoint 4-bank groups.  (The round-1 scalar transposed stores walked rows 4 apart: 4- to 8-way
// bank conflicts, SQ_LDS_BANK_CONFLICT = 87% of the LDS cycles of the weight-gradient GEMMs.)
__device__ __forceinline__ float dpp_quad_xor1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
}
__device__ __forceinline__ float dpp_quad_xor2(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
}
// lane q of a quad holds M[q][0..3]; returns M[0..3][q] (every lane of the wave must execute it)
__device__ __forceinline__ f32x4 quad_transpose(f32x4 v, int q) {
  const bool x = q & 1;
  const float r0 = dpp_quad_xor1(x ? v[0] : v[1]), r1 = dpp_quad_xor1(x ? v[2] : v[3]);
  if (x) { v[0] = r0; v[2] = r1; } else { v[1] = r0; v[3] = r1; }
  const bool X = q & 2;
  const float u0 = dpp_quad_xor2(X ? v[0] : v[2]), u1 = dpp_quad_xor2(X ? v[1] : v[3]);
  if (X) { v[0] = u0; v[1] = u1; } else { v[2] = u0; v[3] = u1; }
  return v;
}

// SoA constants: BNRELU [sc][mu][be], BNBWD [sc][c1][mu][istd][c2], each nf floats
template <int XF>
__host__ __device__ constexpr int soa_arrays() {
  return XF == CV_XF_BNRELU ? 3 : XF == CV_XF_BNBWD ? 5 : 0;
}

// same arithmetic, in the same order, as bn_relu / bn_bwd of cv_common.hpp
template <int XF>
__device__ __forceinline__ f32x4 xform4(f32x4 x, f32x4 y, const float* c, int nf, int ch) {
  if constexpr (XF == CV_XF_BNRELU) {
    const f32x4 sc = lds4(c + ch), mu = lds4(c + nf + ch), be = lds4(c + 2 * nf + ch);
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = fmaxf(fmaf(x[j] - mu[j], sc[j], be[j]), 0.f);
  } else if constexpr (XF == CV_XF_BNBWD) {
    const f32x4 sc = lds4(c + ch), c1 = lds4(c + nf + ch), mu = lds4(c + 2 * nf + ch);
    const f32x4 is = lds4(c + 3 * nf + ch), c2 = lds4(c + 4 * nf + ch);
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = sc[j] * (x[j] - c1[j] - (y[j] - mu[j]) * is[j] * c2[j]);
  }
  return x;
}

// per-thread register copy of the constants of one channel quad (BNRELU: sc, mu, be; BNBWD: sc, c1,
// mu, istd, c2), reloaded only when the quad changes
struct XC {
  f32x4 k[5];
};
template <int XF>
__device__ __forceinline__ XC load_xc(const float* c, int nf, int ch) {
  XC r;
#pragma unroll
  for (int q = 0; q < soa_arrays<XF>(); ++q) r.k[q] = lds4(c + q * nf + ch);
  return r;
}
template <int XF>
__device__ __forceinline__ f32x4 apply_xc(f32x4 x, f32x4 y, const XC& c) {
  if constexpr (XF == CV_XF_BNRELU) {
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = fmaxf(fmaf(x[j] - c.k[1][j], c.k[0][j], c.k[2][j]), 0.f);
  } else if constexpr (XF == CV_XF_BNBWD) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      x[j] = c.k[0][j] * (x[j] - c.k[1][j] - (y[j] - c.k[2][j]) * c.k[3][j] * c.k[4][j]);
  }
  return x;
}

template <int XF>
__device__ __forceinline__ void fill_soa(const cv_bn& bn, int nf, float* dst, double* scratch) {
  if constexpr (XF == CV_XF_BNRELU) {
    bn_fold<NT>(bn, false, scratch, [&](int f, double s, double q, double, double) {
      if (f < nf) {
        const BnFwdC k = bn_fwd_const_s(bn, f, s, q);
        dst[f] = k.sc;
        dst[nf + f] = k.mu;
        dst[2 * nf + f] = k.be;
      }
    });
  } else if constexpr (XF == CV_XF_BNBWD) {
    bn_fold<NT>(bn, true, scratch, [&](int f, double s, double q, double gs, double gq) {
      if (f < nf) {
        const BnBwdC k = bn_bwd_const_s(bn, f, s, q, gs, gq);
        dst[f] = k.sc;
        dst[nf + f] = k.c1;
        dst[2 * nf + f] = k.mu;
        dst[3 * nf + f] = k.istd;
        dst[4 * nf + f] = k.c2;
      }
    });
  }
}

// Finalised constants of a train-mode layer (cv_bn.cfwd / cbwd, written by the producer's last
// workgroup): a float4 copy into LDS instead of the replica fold.  The SoA order of cfwd starts with
// [sc][mu][beta] and cbwd is [sc][c1][mu][istd][c2], exactly the LDS images above.
// Split in two phases so every constant set of a prologue (A transform, B transform, the STAT_BWD
// epilogue's forward constants) is in flight together with the first tile's loads and the prologue pays
// ONE memory round trip: soa_issue loads the constants and the ticket into registers (nothing waits),
// soa_commit checks the ticket and writes LDS (a zero ticket: the producer did not finalise, and the
// caller folds the replica sums instead).
struct SoaPre {
  f32x4 tmp[3];
  unsigned tk;
  bool ok;
};
template <int XF>
__device__ __forceinline__ SoaPre soa_issue(const cv_bn& bn, int nf) {
  SoaPre p;
  const float* src = (XF == CV_XF_BNRELU) ? bn.cfwd : bn.cbwd;
  p.ok = bn.train && src && bn.ticket && nf == bn.C;
  p.tk = 0u;
  if (!p.ok) return p;
  const int n4 = soa_arrays<XF>() * nf / 4;
  const f32x4* s4 = reinterpret_cast<const f32x4*>(src);
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int i = threadIdx.x + q * NT;
    p.tmp[q] = s4[i < n4 ? i : 0];
  }
  p.tk = bn.ticket[XF == CV_XF_BNRELU ? 0 : 1];
  return p;
}
template <int XF>
__device__ __forceinline__ bool soa_commit(const SoaPre& p, const cv_bn& bn, int nf, float* dst) {
  if (!p.ok || p.tk == 0u) return false;
  const float* src = (XF == CV_XF_BNRELU) ? bn.cfwd : bn.cbwd;
  const int n4 = soa_arrays<XF>() * nf / 4;
  const f32x4* s4 = reinterpret_cast<const f32x4*>(src);
  f32x4* d4 = reinterpret_cast<f32x4*>(dst);
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int i = threadIdx.x + q * NT;
    if (i < n4) d4[i] = p.tmp[q];
  }
  for (int i = threadIdx.x + 3 * NT; i < n4; i += NT) d4[i] = s4[i];
  return true;
}
// the STAT_BWD epilogue's forward constants (AoS BnFwdC in LDS) from cfwd = [sc][mu][beta][istd]
struct EpiPre {
  float v[4];
  unsigned tk;
  bool ok;
};
__device__ __forceinline__ EpiPre epi_issue(const cv_bn& eb, int ce_n) {
  EpiPre p;
  p.ok = eb.train && eb.cfwd && eb.ticket && eb.C == ce_n;
  p.tk = 0u;
  if (!p.ok) return p;
  const int f = (int)threadIdx.x < ce_n ? (int)threadIdx.x : 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) p.v[q] = eb.cfwd[q * eb.C + f];
  p.tk = eb.ticket[0];
  return p;
}
__device__ __forceinline__ bool epi_commit(const EpiPre& p, const cv_bn& eb, int ce_n, BnFwdC* d) {
  if (!p.ok || p.tk == 0u) return false;
  if ((int)threadIdx.x < ce_n) d[threadIdx.x] = BnFwdC{p.v[0], p.v[1], p.v[2], p.v[3]};
  for (int f = threadIdx.x + NT; f < ce_n; f += NT)
    d[f] = BnFwdC{eb.cfwd[f], eb.cfwd[eb.C + f], eb.cfwd[2 * eb.C + f], eb.cfwd[3 * eb.C + f]};
  return true;
}

// DENSE B modes (the XB slot of a DENSE instance)
enum { DB_KCONT = 0, DB_NCONT = 1, DB_KPERM = 2 };

template <int OP, int BM, int BN>
struct Shape {
  static constexpr int WN = (BN >= 32) ? 2 : 1;
  static constexpr int WM = 4 / WN;
  static constexpr int TM = BM / WM, TN = BN / WN;
  static constexpr int FM = TM / 16, FN = TN / 16;
  static constexpr int RA = BM / 32;                  // A float4 slots per thread (BM*BK/4/NT)
  static constexpr int RB = (BN * BK / 4 + NT - 1) / NT;  // B float4 slots per thread
};

// LDS floats: 2 A images + 2 B images + epilogue reduction + constants
__host__ __device__ inline size_t fast_lds_floats(int BM, int BN, int nfa, int nfb, int nfe) {
  const int WN = (BN >= 32) ? 2 : 1, WM = 4 / WN;
  return 2 * (size_t)BM * LDK + 2 * (size_t)BN * LDK + 2 * WM * BN + nfa + nfb + nfe;
}

#ifndef CV_FAST_QTB
#define CV_FAST_QTB 0
#endif
// resident waves per SIMD the register allocation must allow: the narrow-tile variants serve the
// launches with thousands of short workgroups, where a third resident workgroup per CU removes a round
#ifndef CV_FAST_MINW_SMALL
#define CV_FAST_MINW_SMALL 3
#endif
#ifndef CV_FAST_MINW_64
#define CV_FAST_MINW_64 1
#endif
// MT: MMA_F32 (v_mfma_f32_16x16x4_f32, fp32 operands) or MMA_BF16 (operands rounded to bf16 when
// staged into LDS after the fp32 transform, v_mfma_f32_16x16x32_bf16, fp32 accumulation)
// (the deep-ring instances, D >= 4, serve under-filled launches only: 2 resident workgroups suffice there)
// The one-tile body on the workgroup's block coordinates (bx0, by0, bz0) of a (gx0, gy0, gz0) grid: gemm_kernel's
// own blockIdx, or its share of a dual launch (cv_dual.hip)
template <int OP, int BM, int BN, int XA, int XB, int EPI, int D, int MT>
__device__ __forceinline__ void gemm_body(const Args& P, const int bx0, const int by0, const int bz0, const int gx0,
                                          const int gy0, const int gz0) {
#define CV_GZ gz0
#define CV_FIN_ME (unsigned)(bx0 + gx0 * (by0 + gy0 * bz0))
#define CV_FIN_NBLK (unsigned)(gx0 * gy0 * gz0)
#include "cv_gemm_prelude.inc"

  // ---------------- one tile per workgroup
  const int gx = gx0, gy = gy0;
  const int nwg = gx * gy * gz0;
  const int hw_id = bx0 + gx * (by0 + gy * bz0);
  int bx = bx0, by = by0, bz = bz0;
#define CV_TILE_EXIT \
  do {              \
    finalize(true); \
    return;         \
  } while (0)
#define CV_TILE_CONSTS_BEGIN {
#define CV_TILE_CONSTS_END }
#define CV_TILE_FINALIZE finalize(true)
#include "cv_gemm_tile.inc"
#undef CV_TILE_EXIT
#undef CV_TILE_CONSTS_BEGIN
#undef CV_TILE_CONSTS_END
#undef CV_TILE_FINALIZE
#undef CV_GZ
#undef CV_FIN_ME
#undef CV_FIN_NBLK
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

template <int OP, int BM, int BN, int XA, int XB, int EPI, int D, int MT>
__global__ __launch_bounds__(NT, (BM == 64 && BN <= 32) ? (D >= 4 ? 2 : CV_FAST_MINW_SMALL)
                                                        : (BM == 64 ? CV_FAST_MINW_64 : 1))
void gemm_kernel(const Args P) {
  gemm_body<OP, BM, BN, XA, XB, EPI, D, MT>(P, blockIdx.x, blockIdx.y, blockIdx.z, gridDim.x, gridDim.y, gridDim.z);
}

// Two tiles per workgroup (GATHER / SCATTER launches with more tiles than one round of resident slots):
// a 1-D grid of G >= tiles / 2 workgroups, workgroup w takes tiles w and w + G of the tile grid
// P.tiles_x * P.tiles_y * P.tiles_z.  The BN constants are staged once per workgroup, the last-arriver
// finalisation runs once per workgroup, and the second round of workgroups — each paying the whole
// prologue (first-tile burst) and epilogue again — disappears.  The two tiles are two inlined copies of
// the tile body, not a loop (a loop back-edge kept ~50 more VGPRs live, measured); the narrow tiles ask
// for 4 resident workgroups so the MNIST backward-data launch (1568 tiles) fits 1024 slots.
template <int OP, int BM, int BN, int XA, int XB, int EPI, int D, int MT>
__global__ __launch_bounds__(NT, (BM == 64 && BN <= 32) ? 4 : (BM == 64 ? CV_FAST_MINW_64 : 1))
void gemm_kernel2(const Args P) {
#define CV_GZ ((int)gridDim.z)
#define CV_FIN_ME (blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z))
#define CV_FIN_NBLK (gridDim.x * gridDim.y * gridDim.z)
#include "cv_gemm_prelude.inc"

  const int gx = P.tiles_x, gy = P.tiles_y;
  const int nwg = gx * gy * P.tiles_z;
  const int hw_id = blockIdx.x;
  bool first = true;
  auto tile_body = [&](int tile) {
    int bx = tile % gx, by = (tile / gx) % gy, bz = tile / (gx * gy);
    // thread indices re-derived per tile (shadowing the prelude's): the captured copies cost 5 VGPRs of
    // spills on the BN-backward narrow tiles
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int wm = wid / WN, wn = wid % WN;
#define CV_TILE_EXIT return
#define CV_TILE_CONSTS_BEGIN \
  if (first) {               \
    first = false;
#define CV_TILE_CONSTS_END }
#define CV_TILE_FINALIZE ((void)0)
#include "cv_gemm_tile.inc"
#undef CV_TILE_EXIT
#undef CV_TILE_CONSTS_BEGIN
#undef CV_TILE_CONSTS_END
#undef CV_TILE_FINALIZE
  };
  // the host clamps the grid to at most `tiles` workgroups; the guard keeps a workgroup without a tile
  // (a grid larger than the tile count) from decoding a bogus tile (a parity class bz >= tiles_z)
  // (the tile body is inlined at exactly two call sites: more would grow the kernel past its register budget)
  const int G = (int)gridDim.x;
  int t1 = hw_id < nwg ? hw_id : -1, t2 = hw_id + G < nwg ? hw_id + G : -1;
  if (OP == OP_SCATTER && P.bal_ncls) {
    // K-balanced pairing: tiles sorted by their class's taps (heaviest class first); the workgroups with one
    // tile take the heaviest, and the others pair the i-th heaviest remaining tile with the i-th lightest
    const int S0 = nwg - G, single = G - S0, per = gx * gy;
    const int p1 = hw_id >= S0 ? hw_id - S0 : single + hw_id, p2 = single + 2 * S0 - 1 - hw_id;
    const int k1 = p1 / per, k2 = p2 / per;
    t1 = p1 - k1 * per + per * P.cls_order[k1];
    t2 = hw_id < S0 ? p2 - k2 * per + per * P.cls_order[k2] : -1;
  }
  if (t1 >= 0) tile_body(t1);
  if (t2 >= 0) tile_body(t2);
  finalize(true);
#undef CV_GZ
#undef CV_FIN_ME
#undef CV_FIN_NBLK
}

#ifndef CV_FAST_DEPTH_BNBWD
#define CV_FAST_DEPTH_BNBWD 2
#endif
#ifndef CV_FAST_DEPTH_WGRAD
#define CV_FAST_DEPTH_WGRAD 3
#endif
#ifndef CV_FAST_DEPTH
#define CV_FAST_DEPTH 2
#endif

// Resident-workgroup slots of a kernel on the device (occupancy x CUs), cached per (kernel, LDS bytes);
// 0 when unknown.
inline bool persist_enabled() {  // CV_PERSIST=0: no two-tile launch (one workgroup per tile), the A/B baseline
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("CV_PERSIST");
    on = (e && atoi(e) == 0) ? 0 : 1;
  }
  return on != 0;
}
inline long resident_slots(const void* kern, size_t lds) {
  static int cus = -1;
  if (cus < 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 0;
    (void)hipGetLastError();
  }
  if (cus <= 0) return 0;
  struct Ent {
    const void* k;
    size_t lds;
    int nb;
  };
  static Ent cache[512];
  static int n = 0;
  for (int i = 0; i < n; ++i)
    if (cache[i].k == kern && cache[i].lds == lds) return (long)cache[i].nb * cus;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, NT, lds) != hipSuccess) {
    (void)hipGetLastError();
    nb = 0;
  }
  if (n < 512) cache[n++] = Ent{kern, lds, nb};
  return (long)nb * cus;
}

// Deep operand ring for under-filled launches (CV_DEEP=0: off, the A/B baseline): a GATHER / SCATTER launch
// whose workgroups fill less than half of one round of resident slots leaves ~1-2 workgroups per CU, so
// nothing hides the K loop's load latency but the register ring itself; those launches take a 4-deep ring
// (3 K tiles in flight), which costs registers the under-filled launch does not need for occupancy.
inline bool deep_enabled() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("CV_DEEP");
    on = (e && atoi(e) == 0) ? 0 : 1;
  }
  return on != 0;
}
#ifndef CV_FAST_DEPTH_DEEP
#define CV_FAST_DEPTH_DEEP 4
#endif

// XCD-grouped tile order (Args::xcd), A/B knobs.  CV_XCD=1: GATHER / SCATTER tiles grouped per XCD (measured
// and rejected: MNIST 0.579 -> 0.617 ms/step); CV_XCD_WGRAD=1: the weight gradients' M-tile-fastest order
// instead of N-tile-fastest
inline int env_flag(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? (atoi(e) != 0) : dflt;
}
// CV_BAL=1: the two-tile SCATTER launches pair their tiles K-balanced (Args::bal_ncls) instead of w and w + G
// in class-major order; measured neutral (MNIST 0.5802 vs 0.5813 ms/step: the per-tile prologue / epilogue,
// not the classes' 1 / 2 / 2 / 4 taps, sets the workgroups' length), so off by default
// deep ring when the launch's tiles fill at most num/den of one round of resident slots (CV_DEEP_FILL=<percent>,
// default 50: "less than half a round")
inline long deep_num() {
  static long v = -1;
  if (v < 0) {
    const char* e = getenv("CV_DEEP_FILL");
    v = e ? atol(e) : 50;
  }
  return v;
}
inline long deep_den() { return 100; }
inline int bal_enabled() {
  static int on = env_flag("CV_BAL", 0);
  return on;
}
inline int xcd_enabled() {
  static int on = env_flag("CV_XCD", 0);
  return on;
}
inline int xcd_wgrad_enabled() {
  static int on = env_flag("CV_XCD_WGRAD", 0);
  return on;
}

// Launch capture (host): while `want` is set, the weight-gradient launch of launch_fast is recorded here instead
// of issued (cv_dual.hip issues it beside a direct backward-data launch, or alone).
struct GemmCap {
  bool want = false, got = false;
  int key[7];  // BM, BN, XA, XB, EPI, D, MT
  Args a;
  dim3 grid;
  size_t lds = 0;
  const void* kern = nullptr;
};
extern thread_local GemmCap* g_gemm_cap;

template <int OP, int BM, int BN, int XA, int XB, int EPI, int MT>
int launch_fast(const Args& a0, dim3 grid, hipStream_t st) {
  Args a = a0;
  a.xcd = (OP == OP_WGRAD) ? xcd_wgrad_enabled() : (!a0.fix_part ? xcd_enabled() : 0);
  constexpr int XFB = (OP == OP_WGRAD) ? XB : CV_XF_NONE;
  const bool bn1d = (OP == OP_DENSE) && XA != CV_XF_NONE && a.ca_n == a.K;
  const int nfa = (XA == CV_XF_NONE) ? 0 : (bn1d ? a.kchunk : a.ca_n);
  const int nfb = (XFB == CV_XF_NONE) ? 0 : a.cb_n;
  const size_t lds = fast_lds_floats(BM, BN, soa_arrays<XA>() * nfa, soa_arrays<XFB>() * nfb,
                                     EPI == CV_STAT_BWD ? 4 * a.ce_n : 0) * sizeof(float);
  CV_REQUIRE(lds <= 160 * 1024, "gemm: LDS request %zu bytes exceeds 160 KiB", lds);
  // the BN-backward A operand doubles the ring's registers: a 2-deep ring keeps the narrow tiles at
  // 3 resident workgroups per CU without spilling
  // the long-K weight-gradient tiles keep a 3-deep ring (one workgroup per CU there anyway)
  constexpr int DEPTH = (XA == CV_XF_BNBWD && BM == 64 && BN <= 32) ? CV_FAST_DEPTH_BNBWD
                        : (OP == OP_WGRAD && BM == 128)            ? CV_FAST_DEPTH_WGRAD
                                                                   : CV_FAST_DEPTH;
  auto kern = gemm_kernel<OP, BM, BN, XA, XB, EPI, DEPTH, MT>;
  auto carve = [&](const void* k) -> int {
    if (lds > 64 * 1024) {
      const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        cv::set_error("gemm: LDS carve-out of %zu bytes refused: %s", lds, hipGetErrorString(e));
        return 1;
      }
    }
    return 0;
  };
  if (carve((const void*)kern)) return 1;
  if (g_fast_occ_query) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)kern, NT, lds) != hipSuccess) {
      (void)hipGetLastError();
      nb = 0;
    }
    *g_fast_occ_query = nb;
    return 0;
  }
  if constexpr ((OP == OP_GATHER || OP == OP_SCATTER) && MT == MMA_F32 && DEPTH < CV_FAST_DEPTH_DEEP) {
    const long tiles = (long)grid.x * grid.y * grid.z;
    const long slots1 = deep_enabled() ? resident_slots((const void*)kern, lds) : 0;
    if (slots1 > 0 && tiles * deep_den() <= slots1 * deep_num()) {
      auto kern4 = gemm_kernel<OP, BM, BN, XA, XB, EPI, CV_FAST_DEPTH_DEEP, MT>;
      if (carve((const void*)kern4)) return 1;
      note_launch((const void*)kern4);
      hipLaunchKernelGGL(kern4, grid, dim3(NT), lds, st, a);
      CV_LAUNCH_CHECK("gemm_deep");
      return 0;
    }
  }
  if constexpr (OP == OP_GATHER || OP == OP_SCATTER) {
    const long tiles = (long)grid.x * grid.y * grid.z;
    // (a K-split launch keeps one tile per workgroup: its slices meet through the tile's ticket)
    if (persist_enabled() && !a.fix_part && tiles > resident_slots((const void*)kern, lds)) {
      auto kern2 = gemm_kernel2<OP, BM, BN, XA, XB, EPI, DEPTH, MT>;
      const long slots = resident_slots((const void*)kern2, lds);
      if (slots > 0) {
        if (carve((const void*)kern2)) return 1;
        Args p = a;
        p.tiles_x = (int)grid.x;
        p.tiles_y = (int)grid.y;
        p.tiles_z = (int)grid.z;
        // every tile is w or w + G, and no workgroup is without a first tile (G <= tiles): the two-tile
        // entry asks for more resident workgroups than the one-tile one, so slots can exceed tiles here
        long G = slots > (tiles + 1) / 2 ? slots : (tiles + 1) / 2;
        if (p.xcd) G = (G + 7) & ~7L;  // (tile w + G on the same XCD as tile w: the XCD-grouped order needs it)
        if (G > tiles) G = tiles;
        p.bal_ncls = 0;
        if (OP == OP_SCATTER && bal_enabled() && !p.xcd) {  // classes of unequal taps: K-balanced pairing
          const int s = p.g.s, ncls = s * s;
          int taps[4], ord[4];
          bool uneq = false;
          for (int c = 0; c < ncls && ncls <= 4; ++c) {
            const int ry = c / s, rx = c % s;
            taps[c] = ((p.g.kh > ry) ? (p.g.kh - ry + s - 1) / s : 0) * ((p.g.kw > rx) ? (p.g.kw - rx + s - 1) / s : 0);
            ord[c] = c;
            if (taps[c] != taps[0]) uneq = true;
          }
          if (uneq && ncls <= 4 && (int)grid.z == ncls) {
            for (int i = 0; i < ncls; ++i)  // stable: heaviest first
              for (int j = i + 1; j < ncls; ++j)
                if (taps[ord[j]] > taps[ord[i]]) { const int q = ord[i]; ord[i] = ord[j]; ord[j] = q; }
            p.bal_ncls = ncls;
            for (int i = 0; i < ncls; ++i) p.cls_order[i] = ord[i];
          }
        }
        note_launch((const void*)kern2);
        hipLaunchKernelGGL(kern2, dim3((unsigned)G), dim3(NT), lds, st, p);
        CV_LAUNCH_CHECK("gemm2");
        return 0;
      }
    }
  }
  if (OP == OP_WGRAD && g_gemm_cap && g_gemm_cap->want && !g_gemm_cap->got) {
    GemmCap& c = *g_gemm_cap;
    c.got = true;
    const int key[7] = {BM, BN, XA, XB, EPI, DEPTH, MT};
    for (int i = 0; i < 7; ++i) c.key[i] = key[i];
    c.a = a;
    c.grid = grid;
    c.lds = lds;
    c.kern = (const void*)kern;
    return 0;
  }
  note_launch((const void*)kern);
  hipLaunchKernelGGL(kern, grid, dim3(NT), lds, st, a);
  CV_LAUNCH_CHECK("gemm");
  return 0;
}

// dispatch over the transform / epilogue modes of one (op, tile)
template <int OP, int BM, int BN, int MT>
int dispatch_modes(const Args& a, int xb, dim3 grid, hipStream_t st) {
  const int xa = a.a.xf, ep = a.ep.stat_mode;
#define CV_FAST_EP(XA_, XB_)                                                            \
  if (ep == CV_STAT_NONE) return launch_fast<OP, BM, BN, XA_, XB_, CV_STAT_NONE, MT>(a, grid, st); \
  if (ep == CV_STAT_FWD) return launch_fast<OP, BM, BN, XA_, XB_, CV_STAT_FWD, MT>(a, grid, st);   \
  return launch_fast<OP, BM, BN, XA_, XB_, CV_STAT_BWD, MT>(a, grid, st);
#define CV_FAST_XA(XB_)                        \
  if (xa == CV_XF_NONE) { CV_FAST_EP(CV_XF_NONE, XB_) } \
  if (xa == CV_XF_BNRELU) { CV_FAST_EP(CV_XF_BNRELU, XB_) } \
  CV_FAST_EP(CV_XF_BNBWD, XB_)
  if constexpr (OP == OP_WGRAD) {  // no epilogue statistics; B transform
#undef CV_FAST_EP
#define CV_FAST_EP(XA_, XB_) return launch_fast<OP, BM, BN, XA_, XB_, CV_STAT_NONE, MT>(a, grid, st);
    if (xb == CV_XF_NONE) { CV_FAST_XA(CV_XF_NONE) }
    if (xb == CV_XF_BNRELU) { CV_FAST_XA(CV_XF_BNRELU) }
    CV_FAST_XA(CV_XF_BNBWD)
  } else if constexpr (OP == OP_DENSE) {
#undef CV_FAST_EP
#define CV_FAST_EP(XA_, XB_)                                                            \
  if (ep == CV_STAT_NONE) return launch_fast<OP, BM, BN, XA_, XB_, CV_STAT_NONE, MT>(a, grid, st); \
  if (ep == CV_STAT_FWD) return launch_fast<OP, BM, BN, XA_, XB_, CV_STAT_FWD, MT>(a, grid, st);   \
  return launch_fast<OP, BM, BN, XA_, XB_, CV_STAT_BWD, MT>(a, grid, st);
    if (xb == DB_KCONT) { CV_FAST_XA(DB_KCONT) }
    if (xb == DB_NCONT) { CV_FAST_XA(DB_NCONT) }
    CV_FAST_XA(DB_KPERM)
  } else {
    CV_FAST_XA(0)
  }
#undef CV_FAST_EP
#undef CV_FAST_XA
}

template <int OP, int MT>
int dispatch_tiles(const Args& a, int xb, int BM, int BN, dim3 grid, hipStream_t st) {
  if (BM == 64 && BN == 16) return dispatch_modes<OP, 64, 16, MT>(a, xb, grid, st);
  if (BM == 64 && BN == 32) return dispatch_modes<OP, 64, 32, MT>(a, xb, grid, st);
  if (BM == 64 && BN == 64) return dispatch_modes<OP, 64, 64, MT>(a, xb, grid, st);
  if constexpr (OP != OP_DENSE) {
    if (BM == 128 && BN == 16) return dispatch_modes<OP, 128, 16, MT>(a, xb, grid, st);
    if (BM == 128 && BN == 32) return dispatch_modes<OP, 128, 32, MT>(a, xb, grid, st);
    if (BM == 128 && BN == 64) return dispatch_modes<OP, 128, 64, MT>(a, xb, grid, st);
  }
  return -1;
}

}  // namespace fast
}  // namespace cv
