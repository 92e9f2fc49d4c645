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
//   2. the classes run one after another on one accumulator set: for class (dy, dx) and each of its taps (kh, kw)
//      the A fragment of block m is the LDS region pixel base(m) + toff(tap) — a uniform shift per tap, no
//      address arithmetic per element — and the tap's weights [cb][cs] stream through a 2-stage LDS ring
//      (k-contiguous `gather` packing [tap][cb][cs], one 16-byte load and one ds_write_b128 per thread);
//   3. each class's epilogue writes its output pixels (bias, the STAT_FWD sums, or the STAT_BWD ReLU mask and
//      BN-backward sums of the layer above, with the pre-BN values prefetched while the class computes).
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
#include "cv_gemm.hpp"

namespace cv {
namespace direct {

constexpr int CK = 32;     // channels per LDS chunk = K elements of one weight stage
constexpr int PP = CK + 4; // LDS pitch (floats) of a region pixel's chunk and of a weight column's chunk
constexpr int MAXST = 64;  // stages (taps x channel chunks) per workgroup
constexpr int RQ = 4;      // region float4 per thread per staging round

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
  // staged tensor's grid
  const int sh = SC ? g.hs : g.hb, sw = SC ? g.ws : g.wb;

  float* Rg = smem;                             // [nck][rpix][PP]
  float* Bs = Rg + P.nck * P.rpix * PP;         // [2][CBT][PP]
  float* cA = Bs + 2 * CBT * PP;                // A transform constants (SoA, ci each)
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
  __syncthreads();
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

  // ---------------- weight stages: [CBT][PP] per stage, 2-stage LDS ring, loads one stage ahead
  constexpr int WQ = CBT * 8 / NT;  // float4 per thread per stage
  f32x4 wr[WQ];
  auto wload = [&](int j) {
    const float* src = P.wk + P.wofs[j] + n0 * ci;
#pragma unroll
    for (int q = 0; q < WQ; ++q) {
      const int idx = t + q * NT, col = idx >> 3, kq = idx & 7;
      wr[q] = fast::g4(src + col * ci + 4 * kq);
    }
  };
  auto wstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < WQ; ++q) {
      const int idx = t + q * NT, col = idx >> 3, kq = idx & 7;
      *reinterpret_cast<f32x4*>(Bs + buf * CBT * PP + col * PP + 4 * kq) = wr[q];
    }
  };
  wload(0);
  wstore(0);
  if (P.nst > 1) wload(1);

  // ---------------- per-lane rows: A fragment row (lane & 15) and the 4 epilogue rows of every fragment
  const int fr = lane & 15, fk = 4 * (lane >> 4);
  const int blk = P.br * P.nbx;
  int abase[FMX];
  int ob[FMX][4];    // output element offset of block row m's pixel (2by, 2bx), channel 0; -1: no such block
  unsigned obf[FMX]; // per row r: bit 2r = row 2by+1 inside the image, bit 2r+1 = column 2bx+1 inside
#pragma unroll
  for (int i = 0; i < FMX; ++i) {
    const int f = wm + WM * i;
    {
      const int m = f * 16 + fr;
      int base = 0;
      if (m < P.M) {
        const int il = P.f_blk.div(m), rem = m - il * blk;
        const int byl = P.f_nbx.div(rem), bx = rem - byl * P.nbx;
        base = (il * P.r1 + byl) * P.c1 + bx;  // (GATHER: plane 0; the tap's plane is in its offset)
      }
      abase[i] = base * PP + fk;
    }
    obf[i] = 0u;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = f * 16 + 4 * (lane >> 4) + r;
      int o = -1;
      if (m < P.M) {
        const int il = P.f_blk.div(m), rem = m - il * blk;
        const int byl = P.f_nbx.div(rem), bx = rem - byl * P.nbx;
        const int n = img0 + il, by = by0 + byl;
        if (n < g.n && by < P.nby) {
          if constexpr (SC) {
            o = ((n * g.hb + 2 * by) * g.wb + 2 * bx) * co;
            obf[i] |= ((2 * by + 1 < g.hb) ? 1u : 0u) << (2 * r);
            obf[i] |= ((2 * bx + 1 < g.wb) ? 1u : 0u) << (2 * r + 1);
          } else {
            o = ((n * g.hs + by) * g.ws + bx) * co;
          }
        }
      }
      ob[i][r] = o;
    }
  }
  const int col = n0 + wn * 16 + fr;  // this lane's output channel
  const float bcol = P.bias ? P.bias[col] : 0.f;
  __syncthreads();  // region and weight stage 0 visible

  f32x4 acc[FMX];
  float s1 = 0.f, s2 = 0.f;
  float eyv[EPI == CV_STAT_BWD ? FMX : 1][4];
  const float* Bw = Bs + (wn * 16 + fr) * PP + fk;
  int j = 0;
  for (int c = 0; c < P.ncls; ++c) {
    const int dy = SC ? c >> 1 : 0, dx = SC ? c & 1 : 0;
    const int cofs = (SC ? (dy * g.wb + dx) * co : 0) + col;
    auto pix_ok = [&](int i, int r) -> bool {
      return ob[i][r] >= 0 && (!dy || ((obf[i] >> (2 * r)) & 1u)) && (!dx || ((obf[i] >> (2 * r + 1)) & 1u));
    };
    if constexpr (EPI == CV_STAT_BWD) {  // the class's pre-BN values, in flight while it computes
#pragma unroll
      for (int i = 0; i < FMX; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) eyv[i][r] = P.ep.ey[pix_ok(i, r) ? ob[i][r] + cofs : 0];
    }
#pragma unroll
    for (int i = 0; i < FMX; ++i) acc[i] = fast::zero4();
    const int jend = P.cend[c];
    for (; j < jend; ++j) {
      const int buf = j & 1;
      if (j + 1 < P.nst) wstore(buf ^ 1);  // stage j + 1, loaded during stage j - 1
      if (j + 2 < P.nst) wload(j + 2);
      const float* Ab = Rg + P.aofs[j];
      const float* Bb = Bw + buf * CBT * PP;
#pragma unroll
      for (int kc = 0; kc < CK / 16; ++kc) {
        f32x4 av[FMX];
#pragma unroll
        for (int i = 0; i < FMX; ++i)
          if (wm + WM * i < P.nfrag) av[i] = fast::lds4(Ab + abase[i] + kc * 16);
        const f32x4 bv = fast::lds4(Bb + kc * 16);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < FMX; ++i)
            if (wm + WM * i < P.nfrag) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i][s], bv[s], acc[i], 0, 0, 0);
      }
      __syncthreads();
    }
    // epilogue of class (dy, dx)
#pragma unroll
    for (int i = 0; i < FMX; ++i) {
      if (wm + WM * i >= P.nfrag) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (!pix_ok(i, r)) continue;
        const int off = ob[i][r] + cofs;
        float v = acc[i][r] + bcol;
        if constexpr (EPI == CV_STAT_BWD) {
          const float yv = eyv[i][r];
          const BnFwdC k = reinterpret_cast<const BnFwdC*>(cE)[col];
          if (P.ep.erelu && bn_out(yv, k) <= 0.f) v = 0.f;
          P.out[off] = v;
          s1 += v;
          s2 += v * ((yv - k.mu) * k.istd);
        } else {
          P.out[off] = v;
          if constexpr (EPI == CV_STAT_FWD) {
            s1 += v;
            s2 += v * v;
          }
        }
      }
    }
  }

  // ---------------- statistics: lanes of one column (l, l+16, l+32, l+48), the WM row waves, one fp64 replica
  if constexpr (EPI != CV_STAT_NONE) {
    s1 += __shfl_xor(s1, 16, 64);
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 16, 64);
    s2 += __shfl_xor(s2, 32, 64);
    if (lane < 16) {
      red[(wm * 2 + 0) * CBT + wn * 16 + lane] = s1;
      red[(wm * 2 + 1) * CBT + wn * 16 + lane] = s2;
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
  size_t n = region + 2 * (size_t)CBT * PP + (size_t)xf_floats(XA, a.ci) + (EPI == CV_STAT_BWD ? 4 * a.co : 0) +
             2 * 4 * (size_t)CBT;
  const size_t fin = 8 * NT + 8;  // bn_finalize scratch (4 * NT doubles) + flag, at the start of the region
  return n > fin ? n : fin;
}

template <int OP, int XA, int EPI, int CBT>
static const void* pick(int fmx) {
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
  // grid has fewer than two workgroups per CU or the region exceeds ~64 KB of LDS, keeping >= 16 rows per row wave
  const int nbimg = a.nby * a.nbx;
  const long ntile_n = a.co / cbt;
  if (nbimg >= 32) {
    a.ipw = 1;
    a.br = 64 / a.nbx < 1 ? 1 : 64 / a.nbx;
    if (a.br > a.nby) a.br = a.nby;
  } else {
    a.br = a.nby;
    a.ipw = 64 / nbimg < 1 ? 1 : 64 / nbimg;
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
  while ((grid_of() < 512 || region_floats() > 16 * 1024) && halve()) {
  }
  if (region_floats() > 20 * 1024) return false;
  if (g_minwg < 0) {
    const char* e = getenv("CV_DIRECT_MINWG");
    g_minwg = e ? atol(e) : 256;
  }
  if (grid_of() < g_minwg) return false;
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
  const void* kern = op == OP_SCATTER ? pick_kernel<OP_SCATTER>(in->xf, epi, cbt, fmx)
                                      : pick_kernel<OP_GATHER>(in->xf, epi, cbt, fmx);
  const size_t lds = lds_floats(a, in->xf, epi, cbt) * sizeof(float);
  if (lds > 96 * 1024) return -1;
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

extern "C" int cv_debug_direct_count(int reset) {
  const int n = cv::g_direct_launches;
  if (reset) cv::g_direct_launches = 0;
  return n;
}
