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

#include "cv_direct.hpp"

namespace cv {
int direct_aux_launch(const int* dkey, const direct::DArgs& da, dim3 dgrid, size_t dlds, hipStream_t st);
}  // namespace cv

namespace cv {
namespace direct {

template <int OP, int XA, int EPI, int CBT, int FMX>
__global__ __launch_bounds__(NT, 2) void direct_kernel(const DArgs P) {
  direct_body<OP, XA, EPI, CBT, FMX>(P, blockIdx.x, blockIdx.y, gridDim.x, gridDim.y);
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
  static int force32 = -1;  // CV_DIRECT_CBT32=1: 32-channel output tiles everywhere (A/B knob)
  if (force32 < 0) {
    const char* e = getenv("CV_DIRECT_CBT32");
    force32 = (e && atoi(e) == 1) ? 1 : 0;
  }
  cbt = (a.co % 64 == 0 && !force32) ? 64 : 32;
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
  if (g_direct_cap && g_direct_cap->want && !g_direct_cap->got) {
    DirectCap& c = *g_direct_cap;
    c.got = true;
    c.key[0] = op;
    c.key[1] = in->xf;
    c.key[2] = epi;
    c.key[3] = cbt;
    c.key[4] = fmx <= 1 ? 1 : (fmx <= 2 ? 2 : 4);
    c.a = a;
    c.grid = grid;
    c.lds = lds;
    c.kern = kern;
    ++g_direct_launches;
    return 0;
  }
  {  // a queued NT-Xent phase rides in this grid (cv_aux.hip) where the pair is served
    const int key[5] = {op, in->xf, epi, cbt, fmx <= 1 ? 1 : (fmx <= 2 ? 2 : 4)};
    const int ar = direct_aux_launch(key, a, grid, lds, st);
    if (ar >= 0) {
      ++g_direct_launches;
      return ar;
    }
  }
  void* params[] = {&a};
  note_launch(kern);
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
