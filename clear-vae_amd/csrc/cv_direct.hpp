// Device side of the direct stride-2 conv (cv_direct.hip: the design notes, the host planner and the C-ABI hooks);
// shared with the dual launch (cv_dual.hip), which runs a direct workgroup and a weight-gradient workgroup side by
// side in one grid.
#pragma once
#include "cv_gemm.hpp"

namespace cv {
namespace direct {

constexpr int CK = 32;     // channels per LDS chunk = K elements of one weight stage
constexpr int PP = CK + 4; // LDS pitch (floats) of a region pixel's chunk and of a weight column's chunk
constexpr int MAXST = 64;  // stages (taps x channel chunks) per workgroup
constexpr int RQ = 4;      // region float4 per thread per staging round
#ifndef CV_DIRECT_NSL
#define CV_DIRECT_NSL 4
#endif
constexpr int NSL = CV_DIRECT_NSL;  // weight ring slots per wave (stages in flight: NSL - 1 issued ahead)
constexpr int RING = NSL * 4 * 16 * CK;  // ring floats per workgroup: 4 waves x NSL slots x 16 columns x CK

#ifdef CV_STAMPS
// instrumented builds only (make stamps): per-workgroup phase timeline [wg][8] u64 = {entry, constants staged,
// region staged, stages done, epilogue stores done, exit, HW_ID, XCC_ID} (s_memrealtime, 100 MHz)
static __device__ unsigned long long* g_dstamps;
#define CV_DSTAMP(v) const unsigned long long v = __builtin_amdgcn_s_memrealtime()
#else
#define CV_DSTAMP(v)
#endif

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

// wait until at most n of this wave's vector-memory operations are outstanding (n wave-uniform, 0..15)
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
  }
}

struct DArgs {
  Geo g;
  cv_operand a;          // the staged operand (transform XA): SCATTER small grid, GATHER big grid
  const float* wk;       // weights, k-contiguous packing [tap][co][ci]
  const float* bias;     // [co] or null
  float* out;            // output NHWC: SCATTER big grid [n][hb][wb][cb], GATHER small grid [n][hs][ws][cs]
  cv_epilogue ep;        // statistics epilogue of the output (ep.ebn.C = co)
  int ci, co;            // staged (contracted) channels, output channels
  int nbx, nby;          // output units per image row / column (SCATTER: 2x2 blocks; GATHER: small pixels)
  int br, ipw, nband;    // unit rows per workgroup, images per workgroup, bands per image
  int r1, c1;            // region rows per image (GATHER: all four planes), region columns (band + tap halo)
  int oy0, ox0;          // SCATTER: small-grid row / column of region row / column 0 (rows relative to the band)
  int pr;                // GATHER: rows of one parity plane (r1 = 4 pr)
  int M, nfrag;          // units per workgroup (ipw * br * nbx), 16-row fragments
  int rpix, nck;         // region pixels per chunk, channel chunks (ci / 32)
  int nst, ncls;         // weight stages (the classes' taps x channel chunks), classes (4 or 1)
  int cend[4];           // one past each class's last stage
  int dbg;               // stamps builds only (CV_DIRECT_DBG): 1 = no weight DMA in the loop, 2 = no MFMA, 4 = no
                         // fragment reads — timing ablations, results invalid
  int wofs[MAXST];       // stage -> weight offset tap * co * ci + chunk * 32
  int aofs[MAXST];       // stage -> LDS float offset of its A operand: (chunk * rpix + toff(tap)) * PP
  FDiv f_nbx, f_blk, f_rpi, f_rc, f_c4, f_pl;  // nbx, br * nbx, r1 * c1, c1, ci / 4, pr * c1
};

// OP: OP_SCATTER or OP_GATHER; XA: transform of the staged operand; EPI: statistics epilogue; CBT: output channels
// per workgroup (32: two column waves x two row waves; 64: four column waves); FMX: 16-row fragments per wave
// The kernel body, on the workgroup's block coordinates (bx, by) of a (gx, gy) grid — the direct kernel's own
// blockIdx, or its share of a dual launch (cv_dual.hip)
template <int OP, int XA, int EPI, int CBT, int FMX>
__device__ __forceinline__ void direct_body(const DArgs& P, const int bx, const int by, const int gx, const int gy) {
  constexpr int WN = CBT / 16, WM = 4 / WN;  // every wave owns 16 columns
  constexpr bool SC = OP == OP_SCATTER;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const Geo& g = P.g;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ci = P.ci, co = P.co;
  const int grp = bx / P.nband, band = bx - grp * P.nband;
  const int img0 = grp * P.ipw, by0 = band * P.br;
  const int n0 = by * CBT;
  CV_DSTAMP(st0);
  // staged tensor's grid
  const int sh = SC ? g.hs : g.hb, sw = SC ? g.ws : g.wb;

  float* Rg = smem;                             // [nck][rpix][PP]
  float* Bs = Rg + P.nck * P.rpix * PP;         // [wave][NSL][16][CK], quads swizzled
  float* cA = Bs + RING;                        // A transform constants (SoA, ci each)
  float* cE = cA + fast::soa_arrays<XA>() * ci; // STAT_BWD: BnFwdC[co] of the output's BatchNorm
  float* red = cE + (EPI == CV_STAT_BWD ? 4 * co : 0);  // [WM][2][CBT]

  // ---------------- region staging: float4 u = (pixel, channel quad); a thread's channel quad is fixed (NT % (ci/4) == 0)
  const int c4n = ci >> 2, total4 = P.rpix * c4n;
  const int rpi = P.r1 * P.c1;
  struct Rs {
    f32x4 x[RQ], y[XA == CV_XF_BNBWD ? RQ : 1];
    unsigned ok;
  };
  auto rload = [&](Rs& S, int u0) {
    S.ok = 0u;
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      const int u = u0 + t + q * NT;
      const int pix = P.f_c4.div(u), c4 = u - pix * c4n;
      const int il = P.f_rpi.div(pix), rem = pix - il * rpi;
      int y, x;
      if constexpr (SC) {  // small-grid pixel of region (row, column)
        const int ry = P.f_rc.div(rem), rx = rem - ry * P.c1;
        y = by0 + P.oy0 + ry;
        x = P.ox0 + rx;
      } else {  // big-grid pixel of parity plane q, plane (row, column)
        const int q = P.f_pl.div(rem), r2 = rem - q * (P.pr * P.c1);
        const int pry = P.f_rc.div(r2), prx = r2 - pry * P.c1;
        y = 2 * (by0 + pry) + (q >> 1) - g.p;
        x = 2 * prx + (q & 1) - g.p;
      }
      const int n = img0 + il;
      const bool ok = u < total4 && n < g.n && (unsigned)y < (unsigned)sh && (unsigned)x < (unsigned)sw;
      const int off = ok ? ((n * sh + y) * sw + x) * ci + 4 * c4 : 0;
      S.x[q] = fast::g4(P.a.x + off);
      if constexpr (XA == CV_XF_BNBWD) S.y[q] = fast::g4(P.a.y + off);
      S.ok |= (ok ? 1u : 0u) << q;
    }
  };
  Rs S0;
  rload(S0, 0);

  // ---------------- constants (requested with the first region loads in flight: one round trip)
  fast::SoaPre pa{};
  fast::EpiPre pe{};
  if constexpr (XA != CV_XF_NONE) pa = fast::soa_issue<XA>(P.a.bn, ci);
  if constexpr (EPI == CV_STAT_BWD) pe = fast::epi_issue(P.ep.ebn, co);
  double* scratch = reinterpret_cast<double*>(Bs);  // (>= 4 * NT doubles; the weight ring is not live yet)
  if constexpr (XA != CV_XF_NONE) {
    if (!fast::soa_commit<XA>(pa, P.a.bn, ci, cA)) fast::fill_soa<XA>(P.a.bn, ci, cA, scratch);
  }
  if constexpr (EPI == CV_STAT_BWD) {
    BnFwdC* d = reinterpret_cast<BnFwdC*>(cE);
    const cv_bn& eb = P.ep.ebn;
    if (!fast::epi_commit(pe, eb, co, d)) {
      bn_fold<NT>(eb, false, scratch, [&](int f, double s, double q, double, double) {
        if (f < co) d[f] = bn_fwd_const_s(eb, f, s, q);
      });
    }
  }
  __syncthreads();  // (the ring doubled as bn scratch above)
  CV_DSTAMP(st1);
  // ---------------- weight stages: every wave streams ITS OWN 16 columns (n0 + wn * 16 + 0..15) through a private
  // NSL-slot ring — no workgroup barrier between stages, each wave waits only for its own DMA (waves of one
  // column group, WM = 2, fetch the same columns twice: L2 traffic, not HBM).  Slot j % NSL holds stage j as
  // [16][CK], quad q of local column cl at q ^ ((cl >> 1) & 7); two 1 KB instructions (8 columns each) per stage.
  constexpr int WPW = 2;
  float* ring = Bs + wid * (NSL * 16 * CK);
  auto issue_at = [&](int wofs, int j) {
    float* slot = ring + (j % NSL) * 16 * CK;
    const float* src = P.wk + wofs + (n0 + wn * 16) * ci;
#pragma unroll
    for (int i = 0; i < WPW; ++i) {
      const int cl = 8 * i + (lane >> 3), q = (lane & 7) ^ ((cl >> 1) & 7);
      __builtin_amdgcn_global_load_lds((gbl_void*)(src + cl * ci + 4 * q), (lds_void*)(slot + i * 8 * CK), 16,
                                       0, 0);
    }
  };
  {
    const int pre = P.nst < NSL - 1 ? P.nst : NSL - 1;
    for (int k = 0; k < pre; ++k) issue_at(P.wofs[k], k);
  }
  fast::XC xc;
  if constexpr (XA != CV_XF_NONE) xc = fast::load_xc<XA>(cA, ci, 4 * (t % c4n));
  auto rstore = [&](const Rs& S, int u0) {
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      const int u = u0 + t + q * NT;
      if (u >= total4) continue;
      const int pix = P.f_c4.div(u), c4 = u - pix * c4n;
      f32x4 v = S.x[q];
      if constexpr (XA == CV_XF_BNRELU) v = fast::apply_xc<XA>(v, v, xc);
      if constexpr (XA == CV_XF_BNBWD) v = fast::apply_xc<XA>(v, S.y[q], xc);
      if (!((S.ok >> q) & 1u)) v = fast::zero4();  // zero halo = the convolution's padding
      *reinterpret_cast<f32x4*>(Rg + ((c4 >> 3) * P.rpix + pix) * PP + (c4 & 7) * 4) = v;
    }
  };
  for (int u0 = 0; u0 < total4; u0 += RQ * NT) {
    Rs S1;
    const bool more = u0 + RQ * NT < total4;
    if (more) rload(S1, u0 + RQ * NT);
    rstore(S0, u0);
    if (more) S0 = S1;
  }

  // ---------------- per-lane units.  The MFMA runs transposed — weights as its row operand, the staged units as
  // its column operand — so a lane's accumulator holds 4 CONSECUTIVE output channels of one unit: the epilogue
  // moves float4s (stores, pre-BN loads), 4x fewer memory instructions than one channel per lane.
  // Lane: unit m = f * 16 + (lane & 15) of fragment f, channels n0 + wn * 16 + 4 * (lane >> 4) + (0..3).
  const int fr = lane & 15, fk = 4 * (lane >> 4);
  const int blk = P.br * P.nbx;
  int abase[FMX];
  int ob[FMX];        // output element offset of unit m's pixel (SCATTER: block pixel (2by, 2bx)), channel 0; -1: none
  unsigned obf = 0u;  // fragment i: bit 2i = row 2by+1 inside the image, bit 2i+1 = column 2bx+1 inside
#pragma unroll
  for (int i = 0; i < FMX; ++i) {
    const int m = (wm + WM * i) * 16 + fr;
    int base = 0, o = -1;
    if (m < P.M) {
      const int il = P.f_blk.div(m), rem = m - il * blk;
      const int byl = P.f_nbx.div(rem), bx = rem - byl * P.nbx;
      base = (il * P.r1 + byl) * P.c1 + bx;  // (GATHER: plane 0; the tap's plane is in its offset)
      const int n = img0 + il, by = by0 + byl;
      if (n < g.n && by < P.nby) {
        if constexpr (SC) {
          o = ((n * g.hb + 2 * by) * g.wb + 2 * bx) * co;
          obf |= ((2 * by + 1 < g.hb) ? 1u : 0u) << (2 * i);
          obf |= ((2 * bx + 1 < g.wb) ? 1u : 0u) << (2 * i + 1);
        } else {
          o = ((n * g.hs + by) * g.ws + bx) * co;
        }
      }
    }
    abase[i] = base * PP + fk;
    ob[i] = o;
  }
  const int ch = wn * 16 + fk;  // this lane's first output channel within the tile
  f32x4 bias4 = fast::zero4();
  if (P.bias) bias4 = fast::g4(P.bias + n0 + ch);
  constexpr int NC = SC ? 4 : 1;  // classes
  auto pix_ok = [&](int c, int i) -> bool {
    const int dy = SC ? c >> 1 : 0, dx = SC ? c & 1 : 0;
    return ob[i] >= 0 && (!dy || ((obf >> (2 * i)) & 1u)) && (!dx || ((obf >> (2 * i + 1)) & 1u));
  };
  auto cofs = [&](int c) -> int { return (SC ? ((c >> 1) * g.wb + (c & 1)) * co : 0) + n0 + ch; };
  f32x4 eyv[EPI == CV_STAT_BWD ? NC : 1][EPI == CV_STAT_BWD ? FMX : 1];
  if constexpr (EPI == CV_STAT_BWD) {  // every class's pre-BN values, before the ring starts
    // (loaded inside the stage loop instead, under its counted waits, they measured slower: MNIST conv2
    // backward-data 34.4 -> 35.4 us, VAE64 37-47 % of the STAT_BWD calls +1-5 %)
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int i = 0; i < FMX; ++i) eyv[c][i] = fast::g4(P.ep.ey + (pix_ok(c, i) ? ob[i] + cofs(c) : 0));
  }
  // The ring's first NSL - 1 stages landed: an explicit count, so the first fragment read below does not depend on
  // how the barrier's fence is lowered for LDS-DMA.  Only the NC * FMX pre-BN loads issued after the DMA may
  // remain in flight (vector-memory loads retire in order).
  wait_vm(EPI == CV_STAT_BWD ? NC * FMX : 0);
  __syncthreads();  // region visible
  CV_DSTAMP(st2);

  f32x4 acc[NC][FMX];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int i = 0; i < FMX; ++i) acc[c][i] = fast::zero4();
  const int bsw = (fr >> 1) & 7;
  const float* Bw = ring + fr * CK;
  // Software pipeline: while stage j's MFMAs run, stage j + 1's fragments are read from LDS (its DMA waited for
  // first) and the stage tables' next entries are already in registers — the MFMAs never wait on an LDS or a
  // scalar load.  (A fragment past the last unit reads region pixel 0 and is discarded by the epilogue: no
  // per-MFMA branch, which would split every MFMA into its own exec-masked block.)
  struct Frag {
    f32x4 a[CK / 16][FMX], b[CK / 16];
  };
  auto frag = [&](int aofs, int j, Frag& F) {
    const float* Ab = Rg + aofs;
    const float* Bb = Bw + (j % NSL) * 16 * CK;
#pragma unroll
    for (int kc = 0; kc < CK / 16; ++kc) {
#pragma unroll
      for (int i = 0; i < FMX; ++i) F.a[kc][i] = fast::lds4(Ab + abase[i] + kc * 16);
      F.b[kc] = fast::lds4(Bb + 4 * ((kc * 4 + (lane >> 4)) ^ bsw));
    }
  };
  const int nst = P.nst, last = nst - 1;
  Frag fa, fb;  // ping-pong fragment sets (the loop is unrolled by two so neither is ever copied)
  frag(P.aofs[0], 0, fa);  // (stage 0 landed: the barrier above drained every DMA)
  int ao_n = P.aofs[last < 1 ? last : 1];             // stage j + 1's region offset
  int wo_n = P.wofs[last < NSL - 1 ? last : NSL - 1];  // stage j + NSL - 1's weight offset
  // one stage: stage j's MFMAs on `cur` while stage j + 1's fragments load into `nxt`
#ifdef CV_STAMPS
  const int dbg = P.dbg;
#else
  constexpr int dbg = 0;
#endif
  auto step = [&](int j, f32x4* ac, const Frag& cur, Frag& nxt) {
    // slot (j - 1) % NSL is free: stage j - 1's fragments were read (and returned) during stage j - 2
    if (!(dbg & 1) && j + NSL - 1 < nst) issue_at(wo_n, j + NSL - 1);
    wo_n = P.wofs[j + NSL < last ? j + NSL : last];
    if (j < last) {
      const int ahead = last - 1 - j < NSL - 2 ? last - 1 - j : NSL - 2;
      if (!(dbg & 1)) wait_vm(ahead * WPW);  // stage j + 1 landed (this wave's own DMA; later stages in flight)
      if (!(dbg & 4)) frag(ao_n, j + 1, nxt);
      ao_n = P.aofs[j + 2 < last ? j + 2 : last];
    }
    if (!(dbg & 2)) {
#pragma unroll
      for (int kc = 0; kc < CK / 16; ++kc)
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < FMX; ++i)
            ac[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.b[kc][s], cur.a[kc][i][s], ac[i], 0, 0, 0);
    }
  };
  int j = 0;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int jend = P.cend[c];
    for (; j + 1 < jend; j += 2) {
      step(j, acc[c], fa, fb);
      step(j + 1, acc[c], fb, fa);
    }
    if (j < jend) {  // odd tail: the next stage's fragments land in fb; one copy per class
      step(j, acc[c], fa, fb);
      fa = fb;
      ++j;
    }
  }
  CV_DSTAMP(st3);
  // epilogues of every class (dy, dx): float4 per (unit, 4 channels)
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  BnFwdC kc4[EPI == CV_STAT_BWD ? 4 : 1];
  if constexpr (EPI == CV_STAT_BWD) {
#pragma unroll
    for (int r = 0; r < 4; ++r) kc4[r] = reinterpret_cast<const BnFwdC*>(cE)[n0 + ch + r];
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
#pragma unroll
    for (int i = 0; i < FMX; ++i) {
      if (!pix_ok(c, i)) continue;
      f32x4 v = acc[c][i];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] += bias4[r];
        if constexpr (EPI == CV_STAT_BWD) {
          const float yv = eyv[c][i][r];
          if (P.ep.erelu && bn_out(yv, kc4[r]) <= 0.f) v[r] = 0.f;
          s1[r] += v[r];
          s2[r] += v[r] * ((yv - kc4[r].mu) * kc4[r].istd);
        } else if constexpr (EPI == CV_STAT_FWD) {
          s1[r] += v[r];
          s2[r] += v[r] * v[r];
        }
      }
      *reinterpret_cast<f32x4*>(P.out + ob[i] + cofs(c)) = v;
    }
  }

  CV_DSTAMP(st4);
  // ---------------- statistics: the 16 lanes of one channel quad (xor 1..8), the WM row waves, one fp64 replica
  if constexpr (EPI != CV_STAT_NONE) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[r] += __shfl_xor(s1[r], o, 64);
        s2[r] += __shfl_xor(s2[r], o, 64);
      }
    }
    if (fr == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        red[(wm * 2 + 0) * CBT + ch + r] = s1[r];
        red[(wm * 2 + 1) * CBT + ch + r] = s2[r];
      }
    }
    __syncthreads();
    if (t < CBT) {
      double a = 0.0, b = 0.0;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        a += (double)red[(w * 2 + 0) * CBT + t];
        b += (double)red[(w * 2 + 1) * CBT + t];
      }
      const int C = P.ep.ebn.C;
      const int repl = (bx + gx * by) % CV_STAT_REPL(C);
      double* so = P.ep.stat_out + (size_t)repl * 2 * C;
      atomic_add_f64(so + n0 + t, a);
      atomic_add_f64(so + C + n0 + t, b);
    }
    bn_finalize_at<NT>(P.ep.ebn, P.ep.stat_out, EPI == CV_STAT_BWD, reinterpret_cast<double*>(smem),
                       reinterpret_cast<int*>(smem + 8 * NT + 4), (unsigned)(bx + gx * by), (unsigned)(gx * gy));
  }
#ifdef CV_STAMPS
  if (t == 0 && g_dstamps) {
    const unsigned long long st5 = __builtin_amdgcn_s_memrealtime();
    unsigned long long* o = g_dstamps + (size_t)(bx + gx * by) * 8;
    o[0] = st0; o[1] = st1; o[2] = st2; o[3] = st3; o[4] = st4; o[5] = st5;
    o[6] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
    o[7] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11));
  }
#endif
}

// Launch capture (host): while `want` is set, direct_run records its launch here instead of issuing it, so the
// caller can issue it together with another kernel's workgroups in one grid (cv_dual.hip) or on its own.
struct DirectCap {
  bool want = false, got = false;
  int key[5];  // OP, XA, EPI, CBT, FMX
  DArgs a;
  dim3 grid;
  size_t lds = 0;
  const void* kern = nullptr;
};
extern thread_local DirectCap* g_direct_cap;

}  // namespace direct
}  // namespace cv
