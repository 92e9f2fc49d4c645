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
#include "cv_gemm.hpp"

namespace cv {
namespace direct {

constexpr int CK = 32;     // channels per LDS chunk = K elements of one weight stage
constexpr int PP = CK + 4; // LDS pitch (floats) of a region pixel's chunk and of a weight column's chunk
constexpr int MAXST = 64;  // stages (taps x channel chunks) per workgroup
constexpr int RQ = 4;      // region float4 per thread per staging round

struct DArgs {
  Geo g;
  cv_operand a;          // small-grid operand (transform XA)
  const float* wk;       // weights, k-contiguous packing [tap][cb][cs]
  const float* bias;     // [cb] or null
  float* out;            // big grid NHWC [n][hb][wb][cb]
  cv_epilogue ep;        // statistics epilogue of the output (ep.ebn.C = cb)
  int nbx, nby;          // 2x2 output blocks per image row / column
  int br, ipw, nband;    // block rows per workgroup, images per workgroup, bands per image
  int rr, rc;            // region rows per image, region columns (band + tap halo)
  int oy0, ox0;          // small-grid row / column of region row / column 0, relative to the band (rows) / image
  int M, nfrag;          // blocks per workgroup (ipw * br * nbx), 16-row fragments
  int rpix, nck;         // region pixels per chunk, channel chunks (cs / 32)
  int nst;               // weight stages: the classes' taps x channel chunks
  int cend[4];           // one past each class's last stage
  int wofs[MAXST];       // stage -> weight offset tap * cb * cs + chunk * 32
  int aofs[MAXST];       // stage -> LDS float offset of its A operand: (chunk * rpix + toff(tap)) * PP
  FDiv f_nbx, f_blk, f_rpi, f_rc, f_c4;  // nbx, br * nbx, rr * rc, rc, cs / 4
};

// XA: transform of the small-grid operand; EPI: statistics epilogue; CBT: output channels per workgroup (32: two
// column waves x two row waves; 64: four column waves); FMX: 16-row fragments per wave (at most)
template <int XA, int EPI, int CBT, int FMX>
__global__ __launch_bounds__(NT, 2) void dscatter_kernel(const DArgs P) {
  constexpr int WN = CBT / 16, WM = 4 / WN;  // every wave owns 16 columns
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const Geo& g = P.g;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int cs = g.cs, cb = g.cb;
  const int grp = blockIdx.x / P.nband, band = blockIdx.x - grp * P.nband;
  const int img0 = grp * P.ipw, by0 = band * P.br;
  const int n0 = blockIdx.y * CBT;

  float* Rg = smem;                             // [nck][rpix][PP]
  float* Bs = Rg + P.nck * P.rpix * PP;         // [2][CBT][PP]
  float* cA = Bs + 2 * CBT * PP;                // A transform constants (SoA, cs each)
  float* cE = cA + fast::soa_arrays<XA>() * cs; // STAT_BWD: BnFwdC[cb] of the output's BatchNorm
  float* red = cE + (EPI == CV_STAT_BWD ? 4 * cb : 0);  // [WM][2][CBT]

  // ---------------- region staging: float4 u = (pixel, channel quad); a thread's channel quad is fixed (NT % (cs/4) == 0)
  const int c4n = cs >> 2, total4 = P.rpix * c4n;
  const int rpi = P.rr * P.rc;
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
      const int ry = P.f_rc.div(rem), rx = rem - ry * P.rc;
      const int y = by0 + P.oy0 + ry, x = P.ox0 + rx, n = img0 + il;
      const bool ok = u < total4 && n < g.n && (unsigned)y < (unsigned)g.hs && (unsigned)x < (unsigned)g.ws;
      const int off = ok ? ((n * g.hs + y) * g.ws + x) * cs + 4 * c4 : 0;
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
  if constexpr (XA != CV_XF_NONE) pa = fast::soa_issue<XA>(P.a.bn, cs);
  if constexpr (EPI == CV_STAT_BWD) pe = fast::epi_issue(P.ep.ebn, cb);
  double* scratch = reinterpret_cast<double*>(Bs);  // (>= 4 * NT doubles; the weight ring is not live yet)
  if constexpr (XA != CV_XF_NONE) {
    if (!fast::soa_commit<XA>(pa, P.a.bn, cs, cA)) fast::fill_soa<XA>(P.a.bn, cs, cA, scratch);
  }
  if constexpr (EPI == CV_STAT_BWD) {
    BnFwdC* d = reinterpret_cast<BnFwdC*>(cE);
    const cv_bn& eb = P.ep.ebn;
    if (!fast::epi_commit(pe, eb, cb, d)) {
      bn_fold<NT>(eb, false, scratch, [&](int f, double s, double q, double, double) {
        if (f < cb) d[f] = bn_fwd_const_s(eb, f, s, q);
      });
    }
  }
  __syncthreads();
  fast::XC xc;
  if constexpr (XA != CV_XF_NONE) xc = fast::load_xc<XA>(cA, cs, 4 * (t % c4n));
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
    const float* src = P.wk + P.wofs[j] + n0 * cs;
#pragma unroll
    for (int q = 0; q < WQ; ++q) {
      const int idx = t + q * NT, col = idx >> 3, kq = idx & 7;
      wr[q] = fast::g4(src + col * cs + 4 * kq);
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
        base = (il * P.rr + byl) * P.rc + bx;
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
          o = ((n * g.hb + 2 * by) * g.wb + 2 * bx) * cb;
          obf[i] |= ((2 * by + 1 < g.hb) ? 1u : 0u) << (2 * r);
          obf[i] |= ((2 * bx + 1 < g.wb) ? 1u : 0u) << (2 * r + 1);
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
  for (int c = 0; c < 4; ++c) {
    const int dy = c >> 1, dx = c & 1;
    const int cofs = (dy * g.wb + dx) * cb + col;
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
  size_t n = region + 2 * (size_t)CBT * PP + (size_t)xf_floats(XA, a.g.cs) + (EPI == CV_STAT_BWD ? 4 * a.g.cb : 0) +
             2 * 4 * (size_t)CBT;
  const size_t fin = 8 * NT + 8;  // bn_finalize scratch (4 * NT doubles) + flag, at the start of the region
  return n > fin ? n : fin;
}

template <int XA, int EPI, int CBT>
static const void* pick(int fmx) {
  if (fmx <= 2) return (const void*)dscatter_kernel<XA, EPI, CBT, 2>;
  return (const void*)dscatter_kernel<XA, EPI, CBT, 4>;
}

static const void* pick_kernel(int xa, int epi, int cbt, int fmx) {
#define CV_DS_E(XA_, CBT_)                                               \
  if (epi == CV_STAT_NONE) return pick<XA_, CV_STAT_NONE, CBT_>(fmx);    \
  if (epi == CV_STAT_FWD) return pick<XA_, CV_STAT_FWD, CBT_>(fmx);      \
  return pick<XA_, CV_STAT_BWD, CBT_>(fmx);
#define CV_DS_X(CBT_)                               \
  if (xa == CV_XF_NONE) { CV_DS_E(CV_XF_NONE, CBT_) }     \
  if (xa == CV_XF_BNRELU) { CV_DS_E(CV_XF_BNRELU, CBT_) } \
  CV_DS_E(CV_XF_BNBWD, CBT_)
  if (cbt == 32) { CV_DS_X(32) }
  CV_DS_X(64)
#undef CV_DS_X
#undef CV_DS_E
}

// build the launch (tile choice, class taps, stage tables); false when the geometry is not served
static bool plan(const Geo& g, DArgs& a, int& cbt, long& nwg) {
  const int K = g.kh;
  cbt = (g.cb % 64 == 0) ? 64 : 32;
  a.g = g;
  a.nbx = cdiv(g.wb, 2);
  a.nby = cdiv(g.hb, 2);
  a.nck = g.cs / CK;
  // class taps: output pixel Y = 2 by + dy reads small row y = by + (dy + p - kh) / 2 for kh = dy + p (mod 2)
  int oymin = 1 << 20, oymax = -(1 << 20);
  int ntap[4], tkh[4][4], tkw[4][4], toy[4][4], tox[4][4];
  for (int c = 0; c < 4; ++c) {
    const int dy = c >> 1, dx = c & 1;
    ntap[c] = 0;
    for (int kh = 0; kh < K; ++kh) {
      if (((dy + g.p - kh) % 2 + 2) % 2) continue;
      for (int kw = 0; kw < K; ++kw) {
        if (((dx + g.p - kw) % 2 + 2) % 2) continue;
        if (ntap[c] >= 4) return false;
        const int oy = (dy + g.p - kh) / 2, ox = (dx + g.p - kw) / 2;  // exact (even numerators)
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
  a.oy0 = oymin;
  a.ox0 = oxmin;
  a.rc = a.nbx + (oxmax - oxmin);
  // tile: ~64 blocks per workgroup (a band of block rows of one image, or several whole small images), halved
  // while the grid has fewer than two workgroups per CU and the region must fit ~48 KB of LDS
  const int nbimg = a.nby * a.nbx;
  const long ntile_n = g.cb / cbt;
  if (nbimg >= 32) {
    a.ipw = 1;
    a.br = 64 / a.nbx < 1 ? 1 : 64 / a.nbx;
    if (a.br > a.nby) a.br = a.nby;
  } else {
    a.br = a.nby;
    a.ipw = 64 / nbimg < 1 ? 1 : 64 / nbimg;
  }
  auto grid_of = [&]() -> long { return (long)cdiv(g.n, a.ipw) * cdiv(a.nby, a.br) * ntile_n; };
  auto region_floats = [&]() -> long { return (long)a.nck * a.ipw * (a.br + (oymax - oymin)) * a.rc * PP; };
  while ((grid_of() < 512 || region_floats() > 12 * 1024) && a.ipw * a.br * a.nbx > 16) {
    if (a.ipw > 1) a.ipw = (a.ipw + 1) / 2;
    else if (a.br > 1) a.br = (a.br + 1) / 2;
    else break;
  }
  if (region_floats() > 20 * 1024) return false;
  a.br = cdiv(a.nby, cdiv(a.nby, a.br));  // even bands
  a.nband = cdiv(a.nby, a.br);
  a.rr = a.br + (oymax - oymin);
  a.M = a.ipw * a.br * a.nbx;
  a.nfrag = cdiv(a.M, 16);
  a.rpix = a.ipw * a.rr * a.rc;
  // stages: classes in order, taps in (kh, kw) order, channel chunks innermost
  int j = 0;
  for (int c = 0; c < 4; ++c) {
    for (int i = 0; i < ntap[c]; ++i) {
      const int tap = tkh[c][i] * K + tkw[c][i];
      const int toff = (toy[c][i] - oymin) * a.rc + (tox[c][i] - oxmin);
      for (int ck = 0; ck < a.nck; ++ck) {
        if (j >= MAXST) return false;
        a.wofs[j] = tap * g.cb * g.cs + ck * CK;
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
  a.f_rpi = FDiv::make(a.rr * a.rc);
  a.f_rc = FDiv::make(a.rc);
  a.f_c4 = FDiv::make(g.cs / 4);
  nwg = grid_of();
  return true;
}

}  // namespace direct

static int g_direct_launches = 0;  // test hook cv_debug_direct_count

// The SCATTER contraction by the class-fused direct kernel; -1 when the call is not one it serves (then the
// caller runs the per-class GEMM core).  wk: the k-contiguous packing [tap][cb][cs] of the same weights.
int direct_scatter(const Geo& g, const cv_operand* in, const float* wk, const float* bias, float* out,
                   const cv_epilogue* ep, hipStream_t st, int mma) {
  using namespace direct;
  if (!wk || !enabled() || mma != CV_MMA_FP32) return -1;
  if (g.s != 2 || g.kh != g.kw || (g.kh != 3 && g.kh != 4) || g.p < 0 || g.p > 2) return -1;
  if (in->nchw || g.cs % CK || g.cs > 128 || g.cb % 32 || NT % (g.cs / 4)) return -1;
  if ((long)g.n * g.hb * g.wb * g.cb >= (1L << 31) || (long)g.n * g.hs * g.ws * g.cs >= (1L << 31)) return -1;
  const int epi = (ep && ep->stat_mode != CV_STAT_NONE) ? ep->stat_mode : CV_STAT_NONE;
  if (epi != CV_STAT_NONE && (ep->stat_div > 1 || !ep->stat_out)) return -1;
  if (epi == CV_STAT_BWD && (!ep->ey || ep->ebn.C != g.cb)) return -1;
  if (epi == CV_STAT_FWD && ep->ebn.ticket && ep->ebn.C != g.cb) return -1;
  if (in->xf != CV_XF_NONE && in->bn.C != g.cs) return -1;
  DArgs a;
  memset(&a, 0, sizeof(a));
  int cbt = 32;
  long nwg = 0;
  if (!plan(g, a, cbt, nwg)) return -1;
  a.a = *in;
  a.wk = wk;
  a.bias = bias;
  a.out = out;
  if (epi != CV_STAT_NONE) {
    a.ep = *ep;
    a.ep.stat_div = 1;
    a.ep.ebn.C = g.cb;
  } else {
    a.ep.stat_mode = CV_STAT_NONE;
  }
  const int wm = cbt == 32 ? 2 : 1;
  const int fmx = cdiv(a.nfrag, wm);
  if (fmx > 4) return -1;
  const void* kern = pick_kernel(in->xf, epi, cbt, fmx);
  const size_t lds = lds_floats(a, in->xf, epi, cbt) * sizeof(float);
  if (lds > 96 * 1024) return -1;
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  const dim3 grid((unsigned)(nwg / (g.cb / cbt)), (unsigned)(g.cb / cbt));
  void* params[] = {&a};
  if (hipLaunchKernel(kern, grid, dim3(NT), params, lds, st) != hipSuccess) {
    (void)hipGetLastError();
    set_error("direct_scatter: launch failed");
    return 2;
  }
  ++g_direct_launches;
  return 0;
}

}  // namespace cv

extern "C" int cv_debug_direct_count(int reset) {
  const int n = cv::g_direct_launches;
  if (reset) cv::g_direct_launches = 0;
  return n;
}
