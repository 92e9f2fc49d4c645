// Class-fused direct SCATTER on fp32 MFMA (v_mfma_f32_16x16x4_f32, gfx950): the stride-2 Conv2d backward-data
// and ConvTranspose2d forward (vae.py:15-46 / :113-156 through aten::convolution_backward and conv_transpose2d)
// with the small-grid operand staged into LDS ONCE per workgroup.
//
// Why: the implicit-GEMM core (cv_gemm.hpp) runs a stride-2 SCATTER as four GEMMs, one per output
// parity class, each re-loading and re-transforming the small-grid operand once per tap of its class: every
// small-grid element is fetched and BN-backward-transformed K*K times (9 for MNIST's k3, 16 for VAE64's k4), and
// every workgroup pays a global-memory round trip per 32-deep K step.  Here a workgroup owns a band of 2x2 output
// blocks (block (by, bx) = output pixels (2by + dy, 2bx + dx), one per parity class (dy, dx)) and all of its
// output channels (or a 32 / 64-wide tile of them):
//   1. the small-grid rows the band reads (plus a zero halo = the convolution's padding) are loaded, transformed
//      (BN+ReLU forward, or the BN backward of the layer below) and written to LDS once, channel-chunked
//      [cs/32][pixel][32 + 4] so a fragment read of 16 consecutive blocks is bank-conflict free;
//   2. the classes run one after another, each on its own accumulators: for class (dy, dx) and each tap (kh, kw)
//      the A fragment of block m is the LDS region pixel base(m) + toff(tap) — a uniform shift per tap, no
//      address arithmetic per element — and the tap's weights [cb][cs] (k-contiguous `gather` packing
//      [tap][cb][cs]) stream by LDS-DMA (global_load_lds_dwordx4, no VGPR round trip) through a ring PRIVATE to
//      each wave (its own 16 output channels, NSL slots, NSL - 1 stages ahead): a wave waits only for its own
//      DMA with a counted vmcnt, so the stage loop has no workgroup barrier at all and the waves of a CU drift
//      freely against each other (a per-stage barrier measured 0.76 us per stage against 0.43 of MFMA work).
//      The DMA writes lane-linear, so the XOR swizzle of a column's 8 quads (quad q stored at q ^ ((col >> 1)
//      & 7)) is applied on the source address; it keeps the B fragment reads conflict free without a pad;
//   3. all classes' epilogues run after the last stage (bias, the STAT_FWD sums, or the STAT_BWD ReLU mask and
//      BN-backward sums of the layer above, with the pre-BN values loaded before the first stage): no ordinary
//      global load or store sits between two weight stages, so the counted vmcnt waits never drain the ring.
//      The MFMA runs transposed (weights as the row operand), so a lane holds 4 consecutive channels of one
//      output pixel and the epilogue moves float4s.
// The contraction is the GEMM core's: the same k order within a tap (4 k per lane group, 16-k halves), taps in
// (kh, kw) order, fp32 MFMA accumulation; only the order in which taps are summed differs from the per-class GEMM
// (tap-major there too), so results agree with the core to fp32 rounding (tests/test_gpu_direct.py).
//
// The same kernel serves the stride-2 GATHER (Conv2d forward, ConvTranspose2d backward-data: vae.py:15-26 /
// :113-130 forward, the decoder's backward) with one "class": the output units are small-grid pixels, the staged
// region is the big-grid band they read, stored as its four stride-parity planes (big pixel (Y, X), Y' = Y + p:
// plane (Y' & 1, X' & 1), plane pixel (Y' >> 1, X' >> 1)), so tap (kh, kw) reads plane (kh & 1, kw & 1) at a
// uniform shift (kh >> 1, kw >> 1) and 16 consecutive output pixels read 16 consecutive plane pixels (the
// stride-2 walk of the big grid would put every second lane on the same LDS banks).  Its B operand is the
// `scatter` packing [tap][cs][cb] (k = big-grid channel contiguous per output channel).
#include <cstdio>

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
template <int OP, int XA, int EPI, int CBT, int FMX>
__global__ __launch_bounds__(NT, 2) void direct_kernel(const DArgs P) {
  constexpr int WN = CBT / 16, WM = 4 / WN;  // every wave owns 16 columns
  constexpr bool SC = OP == OP_SCATTER;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const Geo& g = P.g;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ci = P.ci, co = P.co;
  const int grp = blockIdx.x / P.nband, band = blockIdx.x - grp * P.nband;
  const int img0 = grp * P.ipw, by0 = band * P.br;
  const int n0 = blockIdx.y * CBT;
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
  __syncthreads();  // region visible (and the ring's first NSL - 1 stages landed)
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
      const int repl = (int)(blockIdx.x + gridDim.x * blockIdx.y) % CV_STAT_REPL(C);
      double* so = P.ep.stat_out + (size_t)repl * 2 * C;
      atomic_add_f64(so + n0 + t, a);
      atomic_add_f64(so + C + n0 + t, b);
    }
    bn_finalize<NT>(P.ep.ebn, P.ep.stat_out, EPI == CV_STAT_BWD, reinterpret_cast<double*>(smem),
                    reinterpret_cast<int*>(smem + 8 * NT + 4));
  }
#ifdef CV_STAMPS
  if (t == 0 && g_dstamps) {
    const unsigned long long st5 = __builtin_amdgcn_s_memrealtime();
    unsigned long long* o = g_dstamps + (size_t)(blockIdx.x + gridDim.x * blockIdx.y) * 8;
    o[0] = st0; o[1] = st1; o[2] = st2; o[3] = st3; o[4] = st4; o[5] = st5;
    o[6] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
    o[7] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11));
  }
#endif
}

// ---------------------------------------------------------------- host side
static int enabled() {  // CV_DIRECT=0: the per-class GEMM core instead (A/B baseline)
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("CV_DIRECT");
    on = (e && atoi(e) == 0) ? 0 : 1;
  }
  return on;
}

static size_t lds_floats(const DArgs& a, int XA, int EPI, int CBT) {
  const size_t region = (size_t)a.nck * a.rpix * PP;
  size_t n = region + (size_t)RING + (size_t)xf_floats(XA, a.ci) + (EPI == CV_STAT_BWD ? 4 * a.co : 0) +
             2 * 4 * (size_t)CBT;
  const size_t fin = 8 * NT + 8;  // bn_finalize scratch (4 * NT doubles) + flag, at the start of the region
  return n > fin ? n : fin;
}

template <int OP, int XA, int EPI, int CBT>
static const void* pick(int fmx) {
  if (fmx <= 1) return (const void*)direct_kernel<OP, XA, EPI, CBT, 1>;
  if (fmx <= 2) return (const void*)direct_kernel<OP, XA, EPI, CBT, 2>;
  return (const void*)direct_kernel<OP, XA, EPI, CBT, 4>;
}

template <int OP>
static const void* pick_kernel(int xa, int epi, int cbt, int fmx) {
#define CV_DS_E(XA_, CBT_)                                                 \
  if (epi == CV_STAT_NONE) return pick<OP, XA_, CV_STAT_NONE, CBT_>(fmx);  \
  if (epi == CV_STAT_FWD) return pick<OP, XA_, CV_STAT_FWD, CBT_>(fmx);    \
  return pick<OP, XA_, CV_STAT_BWD, CBT_>(fmx);
#define CV_DS_X(CBT_)                                     \
  if (xa == CV_XF_NONE) { CV_DS_E(CV_XF_NONE, CBT_) }     \
  if (xa == CV_XF_BNRELU) { CV_DS_E(CV_XF_BNRELU, CBT_) } \
  CV_DS_E(CV_XF_BNBWD, CBT_)
  if (cbt == 32) { CV_DS_X(32) }
  CV_DS_X(64)
#undef CV_DS_X
#undef CV_DS_E
}

static long g_minwg = -1;  // fewest workgroups worth a direct launch (cv_debug_direct_minwg, CV_DIRECT_MINWG)
static int g_gather_rule = 1;  // GATHER only where it beats the GEMM core (0: every geometry; cv_debug_direct_gather_rule)

// build the launch (tile choice, class taps, stage tables); false when the geometry is not served
static bool plan(const Geo& g, int op, DArgs& a, int& cbt, long& nwg) {
  const int K = g.kh;
  const bool sc = op == OP_SCATTER;
  a.g = g;
  a.ci = sc ? g.cs : g.cb;
  a.co = sc ? g.cb : g.cs;
  cbt = (a.co % 64 == 0) ? 64 : 32;
  a.nck = a.ci / CK;
  // taps per class, and the region offset of each: SCATTER output pixel Y = 2 by + dy reads small row
  // y = by + (dy + p - kh) / 2 for kh = dy + p (mod 2); GATHER output row y reads big row 2y - p + kh = plane
  // (kh & 1) row y + (kh >> 1)
  int ncls = sc ? 4 : 1;
  int ntap[4], tkh[4][16], tkw[4][16], toy[4][16], tox[4][16];
  int oymin = 1 << 20, oymax = -(1 << 20);
  for (int c = 0; c < ncls; ++c) {
    const int dy = c >> 1, dx = c & 1;
    ntap[c] = 0;
    for (int kh = 0; kh < K; ++kh) {
      if (sc && ((dy + g.p - kh) % 2 + 2) % 2) continue;
      for (int kw = 0; kw < K; ++kw) {
        if (sc && ((dx + g.p - kw) % 2 + 2) % 2) continue;
        if (ntap[c] >= 16) return false;
        const int oy = sc ? (dy + g.p - kh) / 2 : (kh >> 1), ox = sc ? (dx + g.p - kw) / 2 : (kw >> 1);
        tkh[c][ntap[c]] = kh;
        tkw[c][ntap[c]] = kw;
        toy[c][ntap[c]] = oy;
        tox[c][ntap[c]] = ox;
        ++ntap[c];
        oymin = oy < oymin ? oy : oymin;
        oymax = oy > oymax ? oy : oymax;
      }
    }
  }
  const int oxmin = oymin, oxmax = oymax;  // (square kernel, same padding)
  a.ncls = ncls;
  a.oy0 = oymin;
  a.ox0 = oxmin;
  if (sc) {
    a.nbx = cdiv(g.wb, 2);
    a.nby = cdiv(g.hb, 2);
  } else {
    a.nbx = g.ws;
    a.nby = g.hs;
  }
  a.c1 = a.nbx + (oxmax - oxmin);
  const int halo = oymax - oymin;  // extra region rows per band (GATHER: per plane)
  // tile: ~64 units per workgroup (a band of rows of one image, or several whole small images), halved while the
  // grid has fewer than two workgroups per CU or region + ring exceed ~80 KB of LDS, keeping >= 16 rows per row wave
  const int nbimg = a.nby * a.nbx;
  const long ntile_n = a.co / cbt;
  // units per workgroup (CV_DIRECT_UNITS, default 64) and the grid below which tiles are halved
  // (CV_DIRECT_MINGRID, default 512 = two workgroups per CU); 64-channel tiles (one row wave) keep <= 64 units
  static int U = -1, MG = -1;
  if (U < 0) {
    const char* e = getenv("CV_DIRECT_UNITS");
    const char* f = getenv("CV_DIRECT_MINGRID");
    U = e ? atoi(e) : 64;
    MG = f ? atoi(f) : 512;
  }
  const int units = cbt == 64 && U > 64 ? 64 : U;
  if (2 * nbimg >= units) {
    a.ipw = 1;
    a.br = units / a.nbx < 1 ? 1 : units / a.nbx;
    if (a.br > a.nby) a.br = a.nby;
  } else {
    a.br = a.nby;
    a.ipw = units / nbimg < 1 ? 1 : units / nbimg;
  }
  auto rows_of = [&](int br) -> int { return sc ? br + halo : 4 * (br + halo); };
  auto grid_of = [&]() -> long { return (long)cdiv(g.n, a.ipw) * cdiv(a.nby, a.br) * ntile_n; };
  auto region_floats = [&]() -> long { return (long)a.nck * a.ipw * rows_of(a.br) * a.c1 * PP; };
  const int mmin = 16 * (cbt == 32 ? 2 : 1);
  auto halve = [&]() -> bool {
    if (a.ipw > 1 && (a.ipw + 1) / 2 * a.br * a.nbx >= mmin) { a.ipw = (a.ipw + 1) / 2; return true; }
    if (a.ipw == 1 && a.br > 1 && (a.br + 1) / 2 * a.nbx >= mmin) { a.br = (a.br + 1) / 2; return true; }
    return false;
  };
  // LDS: region + the weight ring within ~80 KB (two workgroups per CU) where the tile can shrink that far; past
  // that one workgroup per CU (the caller's LDS check, 160 KB)
  const long ring = RING;
  while ((grid_of() < MG || region_floats() > 20 * 1024 - ring) && halve()) {
  }
  if (region_floats() > 36 * 1024 - ring) return false;
  if (g_minwg < 0) {
    const char* e = getenv("CV_DIRECT_MINWG");
    g_minwg = e ? atol(e) : 256;
  }
  if (grid_of() < g_minwg) return false;
  // GATHER pays its region (four parity planes of the big grid) per 16-64 output pixels: measured slower than the
  // GEMM core unless one resident round of workgroups covers the call and a tile holds >= 32 pixels (MNIST
  // conv2 / convT2 backward-data win; the 16-pixel tiles and VAE64's multi-round grids lose)
  if (!sc && g_gather_rule && (grid_of() > 512 || (long)a.ipw * a.br * a.nbx < 32)) return false;
  a.br = cdiv(a.nby, cdiv(a.nby, a.br));  // even bands
  a.nband = cdiv(a.nby, a.br);
  a.pr = a.br + halo;
  a.r1 = rows_of(a.br);
  a.M = a.ipw * a.br * a.nbx;
  a.nfrag = cdiv(a.M, 16);
  a.rpix = a.ipw * a.r1 * a.c1;
  // stages: classes in order, taps in (kh, kw) order, channel chunks innermost
  int j = 0;
  for (int c = 0; c < ncls; ++c) {
    for (int i = 0; i < ntap[c]; ++i) {
      const int tap = tkh[c][i] * K + tkw[c][i];
      const int plane = sc ? 0 : ((tkh[c][i] & 1) * 2 + (tkw[c][i] & 1)) * a.pr * a.c1;
      const int toff = plane + (toy[c][i] - oymin) * a.c1 + (tox[c][i] - oxmin);
      for (int ck = 0; ck < a.nck; ++ck) {
        if (j >= MAXST) return false;
        a.wofs[j] = tap * a.co * a.ci + ck * CK;
        a.aofs[j] = (ck * a.rpix + toff) * PP;
        ++j;
      }
    }
    a.cend[c] = j;
  }
  a.nst = j;
  if (a.nst < 1) return false;
  a.f_nbx = FDiv::make(a.nbx);
  a.f_blk = FDiv::make(a.br * a.nbx);
  a.f_rpi = FDiv::make(a.r1 * a.c1);
  a.f_rc = FDiv::make(a.c1);
  a.f_c4 = FDiv::make(a.ci / 4);
  a.f_pl = FDiv::make(a.pr * a.c1);
  nwg = grid_of();
  return true;
}

}  // namespace direct

#ifdef CV_STAMPS
extern "C" int cv_debug_set_stamps_direct(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(cv::direct::g_dstamps), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}
#endif

static int g_direct_launches = 0;  // test hook cv_debug_direct_count

// A stride-2 SCATTER (op = OP_SCATTER: Conv2d backward-data, ConvTranspose2d forward) or GATHER (OP_GATHER: Conv2d
// forward, ConvTranspose2d backward-data) contraction by the direct kernel; -1 when the call is not one it serves
// (then the caller runs the implicit-GEMM core).  wk: the k-contiguous packing [tap][co][ci] of the same weights —
// `gather` [tap][cb][cs] for SCATTER, `scatter` [tap][cs][cb] for GATHER.
static int direct_run(int op, const Geo& g, const cv_operand* in, const float* wk, const float* bias, float* out,
                      const cv_epilogue* ep, hipStream_t st, int mma) {
  using namespace direct;
  if (!wk || !enabled() || mma != CV_MMA_FP32) return -1;
  const int ci = op == OP_SCATTER ? g.cs : g.cb, co = op == OP_SCATTER ? g.cb : g.cs;
  if (g.s != 2 || g.kh != g.kw || (g.kh != 3 && g.kh != 4) || g.p < 0 || g.p > 2) return -1;
  if (in->nchw || ci % CK || ci > 128 || co % 32 || NT % (ci / 4)) return -1;
  if ((long)g.n * g.hb * g.wb * g.cb >= (1L << 31) || (long)g.n * g.hs * g.ws * g.cs >= (1L << 31)) return -1;
  const int epi = (ep && ep->stat_mode != CV_STAT_NONE) ? ep->stat_mode : CV_STAT_NONE;
  if (epi != CV_STAT_NONE && (ep->stat_div > 1 || !ep->stat_out)) return -1;
  if (epi == CV_STAT_BWD && (!ep->ey || ep->ebn.C != co)) return -1;
  if (epi == CV_STAT_FWD && ep->ebn.ticket && ep->ebn.C != co) return -1;
  if (in->xf != CV_XF_NONE && in->bn.C != ci) return -1;
  DArgs a;
  memset(&a, 0, sizeof(a));
  int cbt = 32;
  long nwg = 0;
  if (!plan(g, op, a, cbt, nwg)) return -1;
#ifdef CV_STAMPS
  {
    const char* e = getenv("CV_DIRECT_DBG");
    a.dbg = e ? atoi(e) : 0;
  }
#endif
  a.a = *in;
  a.wk = wk;
  a.bias = bias;
  a.out = out;
  if (epi != CV_STAT_NONE) {
    a.ep = *ep;
    a.ep.stat_div = 1;
    a.ep.ebn.C = co;
  } else {
    a.ep.stat_mode = CV_STAT_NONE;
  }
  const int wm = cbt == 32 ? 2 : 1;
  const int fmx = cdiv(a.nfrag, wm);
  if (fmx > 4) return -1;
  {
    static int log = -1;
    if (log < 0) log = getenv("CV_DIRECT_LOG") ? 1 : 0;
    if (log)
      fprintf(stderr, "direct %s n=%d big=%dx%dx%d small=%dx%dx%d k=%d ci=%d co=%d cbt=%d ipw=%d br=%d nby=%d M=%d "
              "nfrag=%d fmx=%d nst=%d wgs=%ld region_kb=%.1f\n", op == OP_SCATTER ? "scatter" : "gather", g.n, g.hb,
              g.wb, g.cb, g.hs, g.ws, g.cs, g.kh, a.ci, a.co, cbt, a.ipw, a.br, a.nby, a.M, a.nfrag, fmx, a.nst, nwg,
              a.nck * a.rpix * PP * 4.0 / 1024);
  }
  const void* kern = op == OP_SCATTER ? pick_kernel<OP_SCATTER>(in->xf, epi, cbt, fmx)
                                      : pick_kernel<OP_GATHER>(in->xf, epi, cbt, fmx);
  const size_t lds = lds_floats(a, in->xf, epi, cbt) * sizeof(float);
  if (lds > 160 * 1024) return -1;
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  const dim3 grid((unsigned)(nwg / (co / cbt)), (unsigned)(co / cbt));
  void* params[] = {&a};
  if (hipLaunchKernel(kern, grid, dim3(NT), params, lds, st) != hipSuccess) {
    (void)hipGetLastError();
    set_error("direct conv: launch failed");
    return 2;
  }
  ++g_direct_launches;
  return 0;
}

int direct_scatter(const Geo& g, const cv_operand* in, const float* wk, const float* bias, float* out,
                   const cv_epilogue* ep, hipStream_t st, int mma) {
  return direct_run(OP_SCATTER, g, in, wk, bias, out, ep, st, mma);
}

int direct_gather(const Geo& g, const cv_operand* in, const float* wk, const float* bias, float* out,
                  const cv_epilogue* ep, hipStream_t st, int mma) {
  return direct_run(OP_GATHER, g, in, wk, bias, out, ep, st, mma);
}

}  // namespace cv

extern "C" int cv_debug_direct_minwg(int minwg) {
  const int prev = (int)cv::direct::g_minwg;
  cv::direct::g_minwg = minwg;
  return prev;
}

extern "C" int cv_debug_direct_gather_rule(int on) {
  const int prev = cv::direct::g_gather_rule;
  cv::direct::g_gather_rule = on;
  return prev;
}

extern "C" int cv_debug_direct_count(int reset) {
  const int n = cv::g_direct_launches;
  if (reset) cv::g_direct_launches = 0;
  return n;
}
