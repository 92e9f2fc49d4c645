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
template <int OP, int BM, int BN, int XA, int XB, int EPI, int D, int MT>
__global__ __launch_bounds__(NT, (BM == 64 && BN <= 32) ? CV_FAST_MINW_SMALL : (BM == 64 ? CV_FAST_MINW_64 : 1))
void gemm_kernel(const Args P) {
  static_assert(D >= 2, "the register ring needs at least two stages (D=1 is not a valid schedule)");
  using SH = Shape<OP, BM, BN>;
  constexpr int WN = SH::WN, WM = SH::WM, TM = SH::TM, TN = SH::TN, FM = SH::FM, FN = SH::FN;
  constexpr int RA = SH::RA, RB = SH::RB;
  static_assert(FM >= 1 && FN >= 1 && RA >= 1, "tile too small");
  constexpr bool ROWS = OP != OP_WGRAD;
  constexpr int XFB = (OP == OP_WGRAD) ? XB : CV_XF_NONE;  // B transform (WGRAD only)
  constexpr bool AY = XA == CV_XF_BNBWD, BYY = XFB == CV_XF_BNBWD;
  constexpr int DBM = (OP == OP_DENSE) ? XB : DB_NCONT;    // B staging mode
  constexpr bool BKC = (DBM == DB_KCONT || DBM == DB_KPERM);
  // quad-transposed staging of the non-k-contiguous B operand (CV_FAST_QTB=1); off by default: it makes
  // every B load instruction touch twice the cache lines and measured slower on the forward / backward-data
  // GEMMs, while the WGRAD A operand (worst conflicts) always uses it
  constexpr bool QTB = (CV_FAST_QTB != 0) && !BKC;

  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* As = smem;                       // [2][BM][LDK]
  float* Bs = As + 2 * BM * LDK;          // [2][BN][LDK]
  float* red = Bs + 2 * BN * LDK;         // [2][WM][BN]
  // bf16 images live at the start of the same regions ([2][BM][LDKH] / [2][BN][LDKH] halves)
  __bf16* Ah = reinterpret_cast<__bf16*>(As);
  __bf16* Bh = reinterpret_cast<__bf16*>(Bs);
  const bool bn1d = (OP == OP_DENSE) && XA != CV_XF_NONE && P.ca_n == P.K;
  const int nfa = (XA == CV_XF_NONE) ? 0 : (bn1d ? P.kchunk : P.ca_n);
  const int nfb = (XFB == CV_XF_NONE) ? 0 : P.cb_n;
  float* cA = red + 2 * WM * BN;
  float* cB = cA + soa_arrays<XA>() * nfa;
  float* cE = cB + soa_arrays<XFB>() * nfb;  // STAT_BWD: BnFwdC of the epilogue's BN layer

  CV_STAMP(st0);
#ifdef CV_STAMPS
  const unsigned long long mt0 = __builtin_amdgcn_s_memtime();
#endif
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const Geo& g = P.g;

  // producer side of the BN constants hand-off: every workgroup arrives once (early exits too)
  auto finalize = [&](bool) {
    if constexpr (EPI != CV_STAT_NONE) {
      bn_finalize<NT>(P.ep.ebn, P.ep.stat_out, EPI == CV_STAT_BWD, reinterpret_cast<double*>(As),
                      reinterpret_cast<int*>(As + 4096));
    }
  };

  // ---------------- block -> (m0, n0, k-range, class): identical to the generic kernel
  const int gx = gridDim.x, gy = gridDim.y;
  const int nwg = gx * gy * gridDim.z;
  const int hw_id = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (OP == OP_WGRAD) {
    const int xcd = hw_id & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (hw_id >> 3);
    by = lid % gy;
    bx = (lid / gy) % gx;
    bz = lid / (gx * gy);
  }
  const int m0 = bx * BM, n0 = by * BN;
  int M = P.M, K = P.K;
  const int N = P.N + ((OP == OP_WGRAD && P.gbias) ? 1 : 0);
  int kbeg = 0, kend = K;
  int ry = 0, rx = 0, yb0 = 0, xb0 = 0, cy = 1, cx = 1, ntx = 1;
  FDiv f_cx = FDiv::make(1), f_cycx = FDiv::make(1), f_ntx = FDiv::make(1);
  if (OP == OP_SCATTER) {
    const int s = g.s, cls = bz;
    ry = cls / s;
    rx = cls % s;
    yb0 = (((ry - g.p) % s) + s) % s;
    xb0 = (((rx - g.p) % s) + s) % s;
    cy = (g.hb > yb0) ? (g.hb - yb0 + s - 1) / s : 0;
    cx = (g.wb > xb0) ? (g.wb - xb0 + s - 1) / s : 0;
    const int nty = (g.kh > ry) ? (g.kh - ry + s - 1) / s : 0;
    ntx = (g.kw > rx) ? (g.kw - rx + s - 1) / s : 0;
    M = g.n * cy * cx;
    K = nty * ntx * g.cs;
    kend = K;
    if (m0 >= M) {
      finalize(true);
      return;
    }
    f_cx = FDiv::make(cx);
    f_cycx = FDiv::make(cy * cx);
    f_ntx = FDiv::make(ntx);
  } else {
    kbeg = bz * P.kchunk;
    kend = min(K, kbeg + P.kchunk);
    if (kbeg >= kend) {
      finalize(true);
      return;
    }
  }
  const int nt = (kend - kbeg + BK - 1) / BK;
  // GATHER / SCATTER visit K tiles tap-inner: tile j = (channel block j / ntap, tap j % ntap), so a
  // thread's channel quad (and its BN constants) changes only every ntap tiles
  const int ntap = (OP == OP_GATHER) ? g.kh * g.kw : (OP == OP_SCATTER ? (ntx > 0 ? K / g.cs : 1) : 1);
  const FDiv f_ntap = FDiv::make(ntap);
  const int CK = (OP == OP_GATHER) ? g.cb : g.cs;  // channels per tap of the K index

  // ---------------- per-thread A rows (row-oriented ops): rows (t>>3) + 32 i, k quad t & 7.
  // GATHER / SCATTER: a K tile never straddles a tap (channels % BK == 0, checked on the host), so
  // the tap of a tile is wave-uniform (scalar unit); per row we keep the element offset of tap 0,
  // channel 0 (r_base, may be negative for padded rows) and a bitmask of the taps that land inside
  // the image (r_vm), so a tile costs one add and one bit test per row.
  const int aq = t & 7, ar = t >> 3;
  int r_base[RA];
  unsigned r_vm[RA];
  int cy0 = 0, cx0 = 0;
  if constexpr (OP == OP_SCATTER) {
    cy0 = (yb0 + g.p - ry) / g.s;  // small row of class tap jy = 0 is cy0 + ty (exact division)
    cx0 = (xb0 + g.p - rx) / g.s;
  }
  if constexpr (ROWS) {
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const int r = m0 + ar + 32 * i;
      const bool ok = r < M;
      const int rr = ok ? r : 0;
      unsigned vm = 0;
      if constexpr (OP == OP_GATHER) {
        const int hw = g.hs * g.ws;
        const int n = P.f_hws.div(rr);
        const int rem = rr - n * hw;
        const int ys = P.f_ws.div(rem), xs = rem - ys * g.ws;
        const int y0 = ys * g.s - g.p, x0 = xs * g.s - g.p;
        r_base[i] = ((n * g.hb + y0) * g.wb + x0) * g.cb;
        for (int kh = 0; kh < g.kh; ++kh)
          for (int kw = 0; kw < g.kw; ++kw)
            if ((unsigned)(y0 + kh) < (unsigned)g.hb && (unsigned)(x0 + kw) < (unsigned)g.wb) vm |= 1u << (kh * g.kw + kw);
      } else if constexpr (OP == OP_SCATTER) {
        const int hw = cy * cx;
        const int n = f_cycx.div(rr);
        const int rem = rr - n * hw;
        const int ty = f_cx.div(rem), tx = rem - ty * cx;
        const int y0 = cy0 + ty, x0 = cx0 + tx;  // small pixel of class tap (0, 0)
        r_base[i] = ((n * g.hs + y0) * g.ws + x0) * g.cs;
        const int nty = ntx > 0 ? (K / g.cs) / ntx : 0;
        for (int jy = 0; jy < nty; ++jy)
          for (int jx = 0; jx < ntx; ++jx)
            if ((unsigned)(y0 - jy) < (unsigned)g.hs && (unsigned)(x0 - jx) < (unsigned)g.ws) vm |= 1u << (jy * ntx + jx);
      } else {
        r_base[i] = rr * P.lda;
        vm = 1u;
      }
      r_vm[i] = ok ? vm : 0u;
    }
  }

  auto lf = [&](int kk) -> int {  // DENSE: PyTorch feature index of storage-order k'
    if (P.a_pix <= 1) return kk;
    const int pix = P.f_ach.div(kk), c = kk - pix * P.a_ch;
    return c * P.a_pix + pix;
  };

  struct Stage {
    f32x4 a[RA], ay[AY ? RA : 1];
    f32x4 b[RB], by[BYY ? RB : 1];
    unsigned am, bm, bone;  // validity masks; bone: WGRAD bias-column slots
    int ach;                // channel index of the A transform constants
    int cb0;                // GATHER / SCATTER: channel block of the tile (wave-uniform)
  };

  // ---------------- global -> registers (every load unconditional)
  auto fetch = [&](Stage& S, int j) {
#if defined(CV_ABLATE) && CV_ABLATE == 2
    j = 0;  // diagnostic build: every tile re-reads the first tile (L1/L2-hot)
#endif
    int k0, tap = 0, cb0 = 0;
    if constexpr (OP == OP_GATHER || OP == OP_SCATTER) {
      const int cblk = f_ntap.div(j);  // wave-uniform
      tap = j - cblk * ntap;
      cb0 = cblk * BK;
      k0 = tap * CK + cb0;
    } else {
      k0 = kbeg + j * BK;
    }
    S.cb0 = cb0;
    S.am = 0;
    S.bm = 0;
    S.bone = 0;
    const float* ax = P.a.x;
    const float* ayp = P.a.y;
    if constexpr (ROWS) {
      const int kq = k0 + 4 * aq;
      const bool kok = kq < kend;
      if constexpr (OP == OP_GATHER) {
        const int kh = P.f_kw.div(tap), kw = tap - kh * g.kw;
        const int toff = (kh * g.wb + kw) * g.cb + cb0 + 4 * aq;
        S.ach = cb0 + 4 * aq;
#pragma unroll
        for (int i = 0; i < RA; ++i) {
          const bool ok = kok && ((r_vm[i] >> tap) & 1u);
          const int off = ok ? r_base[i] + toff : 0;
          S.a[i] = g4(ax + off);
          if constexpr (AY) S.ay[i] = g4(ayp + off);
          S.am |= (ok ? 1u : 0u) << i;
        }
      } else if constexpr (OP == OP_SCATTER) {
        const int jy = f_ntx.div(tap), jx = tap - jy * ntx;
        const int toff = cb0 + 4 * aq - (jy * g.ws + jx) * g.cs;
        S.ach = cb0 + 4 * aq;
#pragma unroll
        for (int i = 0; i < RA; ++i) {
          const bool ok = kok && ((r_vm[i] >> tap) & 1u);
          const int off = ok ? r_base[i] + toff : 0;
          S.a[i] = g4(ax + off);
          if constexpr (AY) S.ay[i] = g4(ayp + off);
          S.am |= (ok ? 1u : 0u) << i;
        }
      } else {  // DENSE, storage-order k'
        S.ach = bn1d ? kq - kbeg : (P.a_pix > 1 ? P.f_ach.mod(kq) : kq);
#pragma unroll
        for (int i = 0; i < RA; ++i) {
          const bool ok = r_vm[i] && kok;
          const int off = ok ? r_base[i] + kq : 0;
          S.a[i] = g4(ax + off);
          if constexpr (AY) S.ay[i] = g4(ayp + off);
          S.am |= (ok ? 1u : 0u) << i;
        }
      }
    } else {  // WGRAD A(m = cs, k = small pixel): float4 along cs
      constexpr int MQ = BM / 4;
#pragma unroll
      for (int e = 0; e < RA; ++e) {
        const int idx = t + NT * e;
        const int rest = idx >> 2, mq = rest % MQ, kk = 4 * (rest / MQ) + (idx & 3);  // lane quads: 4 k
        const int pix = k0 + kk, c0 = m0 + 4 * mq;
        const bool ok = pix < kend && c0 < g.cs;
        int off = pix * g.cs + c0;
        off = ok ? off : 0;
        S.a[e] = g4(ax + off);
        if constexpr (AY) S.ay[e] = g4(ayp + off);
        S.am |= (ok ? 1u : 0u) << e;
      }
      S.ach = 0;
    }

    // B
#pragma unroll
    for (int e = 0; e < RB; ++e) {
      const int idx = t + NT * e;
      if constexpr (BKC) {  // DENSE layout 0: 4 consecutive k of one output column
        const int n = idx >> 3, kq = k0 + 4 * (idx & 7), col = n0 + n;
        const bool ok = n < BN && col < N && kq < kend;
        if constexpr (DBM == DB_KCONT) {
          int off = col * P.ldb + kq;
          off = ok ? off : 0;
          S.b[e] = g4(P.w + off);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            int off = col * P.ldb + lf(kq + j);
            off = ok ? off : 0;
            S.b[e][j] = P.w[off];
          }
        }
        S.bm |= (ok ? 1u : 0u) << e;
      } else {
        constexpr int NQ = BN / 4;
        int nq, kk;
        if constexpr (QTB) {  // lane quads: 4 consecutive k of one column quad (quad_transpose staging)
          const int rest = idx >> 2;
          nq = rest % NQ;
          kk = 4 * (rest / NQ) + (idx & 3);
        } else {  // consecutive lanes: consecutive column quads of one k (coalesced rows, scalar staging)
          nq = idx % NQ;
          kk = idx / NQ;
        }
        const int col = n0 + 4 * nq, k = k0 + kk;
        bool ok = kk < BK && k < kend && col < N;
        int off = 0;
        if constexpr (OP == OP_GATHER) {
          off = k0 * g.cs + (kk * g.cs + col);
        } else if constexpr (OP == OP_SCATTER) {
          const int jy = f_ntx.div(tap), jx = tap - jy * ntx;
          const int kh = ry + g.s * jy, kw = rx + g.s * jx;
          off = ((kh * g.kw + kw) * g.cs + cb0) * g.cb + (kk * g.cb + col);
        } else if constexpr (OP == OP_DENSE) {
          off = lf(k) * P.ldb + col;
        } else {  // WGRAD: B(k = small pixel, col = (tap, cb)) = T(big[gather(pix, tap)][cb])
          const int hw = g.hs * g.ws;
          const int nimg = P.f_hws.div(k), rem = k - nimg * hw;
          const int ys = P.f_ws.div(rem), xs = rem - ys * g.ws;
          const int nreal = P.N;
          const int tap = P.f_cb.div(col), c0 = col - tap * g.cb;
          const int kh = P.f_kw.div(tap), kw = tap - kh * g.kw;
          const int yb = ys * g.s - g.p + kh, xb = xs * g.s - g.p + kw;
          if (ok && col == nreal) S.bone |= 1u << e;
          ok = ok && col < nreal && (unsigned)yb < (unsigned)g.hb && (unsigned)xb < (unsigned)g.wb;
          off = ((nimg * g.hb + yb) * g.wb + xb) * g.cb + c0;
        }
        off = ok ? off : 0;
        const float* bx_ = (OP == OP_WGRAD) ? P.b.x : P.w;
        S.b[e] = g4(bx_ + off);
        if constexpr (BYY) S.by[e] = g4(P.b.y + off);
        S.bm |= (ok ? 1u : 0u) << e;
      }
    }
  };

  // ---------------- transform + registers -> LDS
  XC xa, xb;        // register copies of the transform constants
  int xa_cb0 = -1;  // channel block xa belongs to (GATHER / SCATTER)
  auto store = [&](Stage& S, int buf) {
    float* Ab = As + buf * BM * LDK;
    float* Bb = Bs + buf * BN * LDK;
    __bf16* Abh = Ah + buf * BM * LDKH;
    __bf16* Bbh = Bh + buf * BN * LDKH;
    if constexpr (ROWS) {
      if constexpr (XA != CV_XF_NONE && OP != OP_DENSE) {
        if (S.cb0 != xa_cb0) {  // wave-uniform: a new channel block
          xa = load_xc<XA>(cA, nfa, S.ach);
          xa_cb0 = S.cb0;
        }
      }
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        f32x4 v = S.a[i];
        if constexpr (OP == OP_DENSE) {
          if constexpr (XA == CV_XF_BNRELU) v = xform4<XA>(v, v, cA, nfa, S.ach);
          if constexpr (XA == CV_XF_BNBWD) v = xform4<XA>(v, S.ay[i], cA, nfa, S.ach);
        } else {
          if constexpr (XA == CV_XF_BNRELU) v = apply_xc<XA>(v, v, xa);
          if constexpr (XA == CV_XF_BNBWD) v = apply_xc<XA>(v, S.ay[i], xa);
        }
        if (!((S.am >> i) & 1u)) v = zero4();
        if constexpr (MT == MMA_BF16) *reinterpret_cast<bf16x4*>(Abh + (ar + 32 * i) * LDKH + 4 * aq) = to_bf16x4(v);
        else *reinterpret_cast<f32x4*>(Ab + (ar + 32 * i) * LDK + 4 * aq) = v;
      }
    } else {
      constexpr int MQ = BM / 4;
#pragma unroll
      for (int e = 0; e < RA; ++e) {
        const int idx = t + NT * e;
        const int rest = idx >> 2, mq = rest % MQ, k4 = 4 * (rest / MQ), q = idx & 3;
        f32x4 v = S.a[e];
        if constexpr (XA == CV_XF_BNRELU) v = apply_xc<XA>(v, v, xa);
        if constexpr (XA == CV_XF_BNBWD) v = apply_xc<XA>(v, S.ay[e], xa);
        if (!((S.am >> e) & 1u)) v = zero4();
        v = quad_transpose(v, q);  // lane q: row 4mq + q, k = k4 .. k4 + 3
        if constexpr (MT == MMA_BF16) *reinterpret_cast<bf16x4*>(Abh + (4 * mq + q) * LDKH + k4) = to_bf16x4(v);
        else *reinterpret_cast<f32x4*>(Ab + (4 * mq + q) * LDK + k4) = v;
      }
    }
#pragma unroll
    for (int e = 0; e < RB; ++e) {
      const int idx = t + NT * e;
      f32x4 v = S.b[e];
      if constexpr (BKC) {
        const int n = idx >> 3, kq = idx & 7;
        if (!((S.bm >> e) & 1u)) v = zero4();
        if (n < BN) {
          if constexpr (MT == MMA_BF16) *reinterpret_cast<bf16x4*>(Bbh + n * LDKH + 4 * kq) = to_bf16x4(v);
          else *reinterpret_cast<f32x4*>(Bb + n * LDK + 4 * kq) = v;
        }
      } else {
        constexpr int NQ = BN / 4;
        if constexpr (XFB == CV_XF_BNRELU) v = apply_xc<XFB>(v, v, xb);
        if constexpr (XFB == CV_XF_BNBWD) v = apply_xc<XFB>(v, S.by[e], xb);
        if (!((S.bm >> e) & 1u)) v = zero4();
        if (OP == OP_WGRAD && ((S.bone >> e) & 1u)) v = f32x4{1.f, 0.f, 0.f, 0.f};
        if constexpr (QTB) {
          const int rest = idx >> 2, nq = rest % NQ, k4 = 4 * (rest / NQ), q = idx & 3;
          v = quad_transpose(v, q);  // lane q: column 4nq + q, k = k4 .. k4 + 3 (whole quads valid or not)
          if (k4 < BK) {
            if constexpr (MT == MMA_BF16) *reinterpret_cast<bf16x4*>(Bbh + (4 * nq + q) * LDKH + k4) = to_bf16x4(v);
            else *reinterpret_cast<f32x4*>(Bb + (4 * nq + q) * LDK + k4) = v;
          }
        } else {
          const int nq = idx % NQ, kk = idx / NQ;
          if (kk < BK) {
            if constexpr (MT == MMA_BF16) {
              const bf16x4 h = to_bf16x4(v);
#pragma unroll
              for (int j = 0; j < 4; ++j) Bbh[(4 * nq + j) * LDKH + kk] = h[j];
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j) Bb[(4 * nq + j) * LDK + kk] = v[j];
            }
          }
        }
      }
    }
  };

  // ---------------- prologue: first D-1 tiles in flight, then the BN constants
  Stage stg[D];
#pragma unroll
  for (int d = 0; d < D - 1; ++d) fetch(stg[d], max(min(d, nt - 1), 0));

  double* fold_scratch = reinterpret_cast<double*>(As);
  static_assert(2 * BM * LDK * sizeof(float) >= 4 * NT * sizeof(double) + 16, "fold scratch");
#if defined(CV_ABLATE) && CV_ABLATE == 3
  if (false)  // diagnostic build: no constants fold (garbage constants)
#endif
  {
  // every finalised constant set is requested before the first wait (one round trip with the tile loads)
  SoaPre pa{}, pb{};
  EpiPre pe{};
  if constexpr (XA != CV_XF_NONE) {
    if (!bn1d) pa = soa_issue<XA>(P.a.bn, nfa);
  }
  if constexpr (EPI == CV_STAT_BWD) pe = epi_issue(P.ep.ebn, P.ce_n);
  if constexpr (XA != CV_XF_NONE) {
    if (bn1d) {
      const float* src = (XA == CV_XF_BNRELU) ? P.a.bn.cfwd : P.a.bn.cbwd;
      const int C1 = P.a.bn.C;
      for (int idx = t; idx < kend - kbeg; idx += NT) {
        int f = kbeg + idx;
        if (P.a_pix > 1) {
          const int pix = f / P.a_ch, c = f - pix * P.a_ch;
          f = c * P.a_pix + pix;
        }
        if (P.a.bn.train && src && P.a.bn.ticket && P.a.bn.ticket[XA == CV_XF_BNRELU ? 0 : 1] != 0u) {
#pragma unroll
          for (int q = 0; q < soa_arrays<XA>(); ++q) cA[q * nfa + idx] = src[q * C1 + f];
        } else if constexpr (XA == CV_XF_BNRELU) {
          const BnFwdC k = bn_fwd_const(P.a.bn, f);
          cA[idx] = k.sc;
          cA[nfa + idx] = k.mu;
          cA[2 * nfa + idx] = k.be;
        } else {
          const BnBwdC k = bn_bwd_const(P.a.bn, f);
          cA[idx] = k.sc;
          cA[nfa + idx] = k.c1;
          cA[2 * nfa + idx] = k.mu;
          cA[3 * nfa + idx] = k.istd;
          cA[4 * nfa + idx] = k.c2;
        }
      }
    } else if (!soa_commit<XA>(pa, P.a.bn, nfa, cA)) {
      fill_soa<XA>(P.a.bn, nfa, cA, fold_scratch);
    }
  }
  if constexpr (XFB != CV_XF_NONE) {  // WGRAD only (long K): issued after A's commit, fewer live registers
    pb = soa_issue<XFB>(P.b.bn, nfb);
    if (!soa_commit<XFB>(pb, P.b.bn, nfb, cB)) fill_soa<XFB>(P.b.bn, nfb, cB, fold_scratch);
  }
  if constexpr (EPI == CV_STAT_BWD) {
    BnFwdC* d = reinterpret_cast<BnFwdC*>(cE);
    const cv_bn& eb = P.ep.ebn;
    if (!epi_commit(pe, eb, P.ce_n, d)) {
      bn_fold<NT>(eb, false, fold_scratch, [&](int f, double s, double q, double, double) {
        if (f < P.ce_n) d[f] = bn_fwd_const_s(eb, f, s, q);
      });
    }
  }
  }
  __syncthreads();
  if constexpr (OP == OP_WGRAD) {  // a thread's channel quads are fixed for the whole K range
    if constexpr (XA != CV_XF_NONE) {
      const int c0 = m0 + 4 * ((t >> 2) % (BM / 4));  // (the fetch's lane-quad mapping)
      xa = load_xc<XA>(cA, nfa, c0 < nfa ? c0 : 0);
    }
    if constexpr (XFB != CV_XF_NONE) {
      const int col = n0 + 4 * ((QTB ? (t >> 2) : t) % (BN / 4));
      xb = load_xc<XFB>(cB, nfb, col < P.N ? P.f_cb.mod(col) : 0);
    }
  }
  store(stg[0], 0);
  __syncthreads();
  CV_STAMP(st1);

  // ---------------- output element offsets; STAT_BWD prefetches the BN inputs at its outputs here,
  // so their latency hides under the main loop instead of opening the epilogue
  auto ep_off = [&](int row, int col) -> int {
    if constexpr (OP == OP_GATHER) {
      return row * g.cs + col;
    } else if constexpr (OP == OP_SCATTER) {
      const int hw = cy * cx;
      const int nimg = f_cycx.div(row), rem = row - nimg * hw;
      const int ty = f_cx.div(rem), tx = rem - ty * cx;
      return ((nimg * g.hb + yb0 + g.s * ty) * g.wb + xb0 + g.s * tx) * g.cb + col;
    } else {
      const int oc = (P.o_pix > 1) ? P.f_opix.mod(col) * P.o_ch + P.f_opix.div(col) : col;
      return row * P.ldo + oc;
    }
  };
  float eyv[EPI == CV_STAT_BWD ? FM : 1][EPI == CV_STAT_BWD ? FN : 1][4];
  if constexpr (EPI == CV_STAT_BWD && OP != OP_WGRAD) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = n0 + wn * TN + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * TM + i * 16 + (lane >> 4) * 4 + r;
          const bool ok = row < M && col < N;
          eyv[i][j][r] = P.ep.ey[ok ? ep_off(row, col) : 0];
        }
      }
  }

  // ---------------- main loop: one barrier per K tile, D-1 tiles of loads in flight
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = zero4();

  const int fr = lane & 15, fk = 4 * (lane >> 4);
  const float* Af = As + (wm * TM + fr) * LDK + fk;
  const float* Bf = Bs + (wn * TN + fr) * LDK + fk;
  auto mma = [&](int buf) {
#if defined(CV_ABLATE) && CV_ABLATE == 1
    return;  // diagnostic build: no fragment reads / MFMAs
#endif
    if constexpr (MT == MMA_BF16) {
      // lane l: A[row l&15][k = 8(l>>4) .. +7], B[k = 8(l>>4) .. +7][col l&15]; one MFMA per BK=32
      static_assert(BK == 32, "one 16x16x32 step per K tile");
      const __bf16* Ab = Ah + buf * BM * LDKH + (wm * TM + fr) * LDKH + 8 * (lane >> 4);
      const __bf16* Bb = Bh + buf * BN * LDKH + (wn * TN + fr) * LDKH + 8 * (lane >> 4);
      bf16x8 av[FM], bv[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) av[i] = *reinterpret_cast<const bf16x8*>(Ab + i * 16 * LDKH);
#pragma unroll
      for (int j = 0; j < FN; ++j) bv[j] = *reinterpret_cast<const bf16x8*>(Bb + j * 16 * LDKH);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
      return;
    }
    const float* Ab = Af + buf * BM * LDK;
    const float* Bb = Bf + buf * BN * LDK;
    f32x4 av[BK / 16][FM], bv[BK / 16][FN];
#pragma unroll
    for (int kc = 0; kc < BK / 16; ++kc) {
#pragma unroll
      for (int i = 0; i < FM; ++i) av[kc][i] = lds4(Ab + i * 16 * LDK + kc * 16);
#pragma unroll
      for (int j = 0; j < FN; ++j) bv[kc][j] = lds4(Bb + j * 16 * LDK + kc * 16);
    }
#pragma unroll
    for (int kc = 0; kc < BK / 16; ++kc)
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kc][i][s], bv[kc][j][s], acc[i][j], 0, 0, 0);
  };
  // Steady state: whole groups of D tiles with no exits inside the unrolled group (an exit would
  // merge control flow and force conservative vmcnt waits); each step fetches tile tt+D-1 (clamped).
  int tt = 0;
  for (; tt + D <= nt; tt += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      fetch(stg[(d + D - 1) % D], min(tt + d + D - 1, nt - 1));
      mma((tt + d) & 1);
      if (tt + d + 1 < nt) store(stg[(d + 1) % D], (tt + d + 1) & 1);
      __syncthreads();
    }
  }
  // Tail: the remaining r < D tiles are already staged (slots 0..r-1); no more loads.
  const int rem = nt - tt;
#pragma unroll
  for (int r = 1; r < D; ++r) {
    if (rem == r) {
#pragma unroll
      for (int d = 0; d < r; ++d) {
        mma((tt + d) & 1);
        if (d + 1 < r) store(stg[(d + 1) % D], (tt + d + 1) & 1);
        __syncthreads();
      }
    }
  }
  CV_STAMP(st2);

  // ---------------- epilogue (same semantics as the generic kernel)
  constexpr bool STATS = EPI != CV_STAT_NONE;
  float s1[FN], s2[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    s1[j] = 0.f;
    s2[j] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = n0 + wn * TN + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * TM + i * 16 + (lane >> 4) * 4 + r;
        float v = acc[i][j][r];
        if (row >= M || col >= N) continue;
        if constexpr (OP == OP_WGRAD) {
          if (P.part) {
            P.part[((size_t)bz * M + row) * N + col] = v;
            continue;
          }
          const int tap = P.f_cb.div(col), c = col - tap * g.cb;
          float* dst = (col >= P.N) ? P.gbias + row : P.out + ((size_t)row * g.cb + c) * (g.kh * g.kw) + tap;
          if (gridDim.z == 1) *dst += v;
          else atomicAdd(dst, v);
          continue;
        } else {
          const int off = ep_off(row, col);
          if (P.bias && (!P.accumulate || bz == 0)) v += P.bias[col];
          if (P.accumulate) {
            atomicAdd(P.out + off, v);
            continue;
          }
          if constexpr (EPI == CV_STAT_BWD) {
            const int f = P.f_sdiv.div(col);
            const float yv = eyv[i][j][r];
            const BnFwdC k = reinterpret_cast<const BnFwdC*>(cE)[f];
            if (P.ep.erelu && bn_out(yv, k) <= 0.f) v = 0.f;
            P.out[off] = v;
            s1[j] += v;
            s2[j] += v * ((yv - k.mu) * k.istd);
          } else {
            P.out[off] = v;
            if constexpr (STATS) {
              s1[j] += v;
              s2[j] += v * v;
            }
          }
        }
      }
    }
  }

  if constexpr (OP != OP_WGRAD && STATS) {
    if (!P.accumulate) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        s1[j] += __shfl_xor(s1[j], 16, 64);
        s1[j] += __shfl_xor(s1[j], 32, 64);
        s2[j] += __shfl_xor(s2[j], 16, 64);
        s2[j] += __shfl_xor(s2[j], 32, 64);
      }
      if (lane < 16) {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int c = wn * TN + j * 16 + lane;
          red[wm * BN + c] = s1[j];
          red[WM * BN + wm * BN + c] = s2[j];
        }
      }
      __syncthreads();
      if (t < BN) {
        const int col = n0 + t;
        if (col < N) {
          double a = 0.0, b = 0.0;
#pragma unroll
          for (int w = 0; w < WM; ++w) {
            a += (double)red[w * BN + t];
            b += (double)red[WM * BN + w * BN + t];
          }
          const int f = P.f_sdiv.div(col);
          const int C = (EPI == CV_STAT_BWD) ? P.ce_n : P.ep.ebn.C;
          const int repl = hw_id % CV_STAT_REPL(C);
          double* so = P.ep.stat_out + (size_t)repl * 2 * C;
          atomic_add_f64(so + f, a);
          atomic_add_f64(so + C + f, b);
        }
      }
    }
    finalize(true);
  }
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

#ifndef CV_FAST_DEPTH_BNBWD
#define CV_FAST_DEPTH_BNBWD 2
#endif
#ifndef CV_FAST_DEPTH_WGRAD
#define CV_FAST_DEPTH_WGRAD 3
#endif
#ifndef CV_FAST_DEPTH
#define CV_FAST_DEPTH 2
#endif

template <int OP, int BM, int BN, int XA, int XB, int EPI, int MT>
int launch_fast(const Args& a, dim3 grid, hipStream_t st) {
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
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      cv::set_error("gemm: LDS carve-out of %zu bytes refused: %s", lds, hipGetErrorString(e));
      return 1;
    }
  }
  if (g_fast_occ_query) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)kern, NT, lds) != hipSuccess) {
      (void)hipGetLastError();
      nb = 0;
    }
    *g_fast_occ_query = nb;
    return 0;
  }
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
