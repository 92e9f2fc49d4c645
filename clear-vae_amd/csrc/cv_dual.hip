// Dual launch: a layer's stride-2 backward-data (the direct kernel, cv_direct.hpp) and its weight gradient (the
// GEMM core's WGRAD tile, cv_gemm.hpp) as ONE grid whose workgroups alternate between the two.
//
// Why: both read only what earlier calls produced (the layer's output gradient, its input), so
// they may run at the same time; and they are complementary — the direct kernel's workgroups spend their first
// and last thirds on HBM bursts (staging its region, writing its output) around an MFMA-bound stage loop, the
// WGRAD tiles are latency-bound K loops.  Run back to back each leaves most of the chip idle most of the time;
// run side by side as two free-running streams they took 36-44 us instead of 51-62 us (MNIST conv2 / conv3 /
// convT1, tools/overlap_probe.py), but a second stream costs ~10 us per cross-stream edge in the replayed step
// graph, more than the overlap buys.  One grid has no edge: workgroup v < 2 min(nd, ng) is direct workgroup v/2
// when v is even and WGRAD workgroup v/2 when odd (the dispatcher hands every CU some of each), the rest go to the
// role with more workgroups.  Each role sees its own block coordinates and workgroup count (the direct kernel's
// BatchNorm finalisation counts its own workgroups, bn_finalize_at), and the grid's LDS and registers are the
// larger of the two.  Served pairs are the instantiations below; any other pair is launched back to back.
// Measured: the one-grid form recovers only part of the free-running streams' overlap (MNIST conv2 pair
// 62.9 -> 58.7 us, convT2 63.3 -> 58.3 us in-step) — the roles share each CU's LDS and register budget at the
// larger of the two — and is used only where the direct grid is a single resident round.
#include "cv_direct.hpp"

namespace cv {
namespace fast {
thread_local GemmCap* g_gemm_cap = nullptr;
}  // namespace fast
namespace direct {
thread_local DirectCap* g_direct_cap = nullptr;
}  // namespace direct

namespace dual {

constexpr long kMaxDirect = 512;  // direct workgroups of a served dual grid (one resident round)
// CV_DUAL_MAXD (A/B): a larger cap (VAE64's 1024-workgroup conv2 pair measured slower as a dual grid in round 4,
// with the roles alternating)
static long max_direct() {
  static long v = -1;
  if (v < 0) {
    const char* e = getenv("CV_DUAL_MAXD");
    v = e ? atol(e) : kMaxDirect;
    if (v < 1) v = kMaxDirect;
  }
  return v;
}

struct DualMap {
  int nd, dgx, dgy;       // direct workgroups and their grid
  int ng, ggx, ggy, ggz;  // WGRAD workgroups and their grid
  int order;              // 0: roles alternate over the first 2 min(nd, ng); 1: direct first; 2: WGRAD first
};

template <int DOP, int DXA, int DEPI, int DCBT, int DFMX, int BM, int BN, int XA, int XB, int EPI, int D, int MT>
__global__ __launch_bounds__(NT, 2) void dual_kernel(const direct::DArgs PD, const Args PG, const DualMap m) {
  const int v = blockIdx.x;
  const int k = m.nd < m.ng ? m.nd : m.ng;
  int role, idx;
  if (m.order == 1) {
    role = v < m.nd ? 0 : 1;
    idx = role ? v - m.nd : v;
  } else if (m.order == 2) {
    role = v < m.ng ? 1 : 0;
    idx = role ? v : v - m.ng;
  } else if (v < 2 * k) {
    role = v & 1;
    idx = v >> 1;
  } else {
    role = m.nd > m.ng ? 0 : 1;
    idx = k + (v - 2 * k);
  }
  if (role == 0) {
    direct::direct_body<DOP, DXA, DEPI, DCBT, DFMX>(PD, idx % m.dgx, idx / m.dgx, m.dgx, m.dgy);
  } else {
    const int r = idx / m.ggx;
    fast::gemm_body<OP_WGRAD, BM, BN, XA, XB, EPI, D, MT>(PG, idx % m.ggx, r % m.ggy, r / m.ggy, m.ggx, m.ggy, m.ggz);
  }
}

struct Ent {
  int dk[5];  // direct OP, XA, EPI, CBT, FMX
  int gk[7];  // WGRAD BM, BN, XA, XB, EPI, D, MT
  const void* fn;
};
#define CV_DUAL(a, b, c, d, e, f, g, h, i, j, k, l) \
  Ent{{a, b, c, d, e}, {f, g, h, i, j, k, l}, (const void*)dual_kernel<a, b, c, d, e, f, g, h, i, j, k, l>}
// the pairs of the bench configurations' backward passes (fp32, 64-row WGRAD tiles — forced inside a dual capture,
// dual_wgrad_bm_cap — so both roles fit two workgroups per CU): MNIST conv2 / conv3 (backward-data SCATTER with the
// BN-backward transform and STAT_BWD + the weight gradient of the BN+ReLU input and the BN-backward output gradient)
// and MNIST convT2 (GATHER)
static const Ent k_pairs[] = {
    CV_DUAL(OP_SCATTER, CV_XF_BNBWD, CV_STAT_BWD, 32, 2, 64, 64, CV_XF_BNBWD, CV_XF_BNRELU, CV_STAT_NONE, 2, 0),
    CV_DUAL(OP_GATHER, CV_XF_BNBWD, CV_STAT_BWD, 64, 4, 64, 64, CV_XF_BNRELU, CV_XF_BNBWD, CV_STAT_NONE, 2, 0),
    CV_DUAL(OP_SCATTER, CV_XF_BNBWD, CV_STAT_BWD, 64, 1, 64, 64, CV_XF_BNBWD, CV_XF_BNRELU, CV_STAT_NONE, 2, 0),
    // VAE64's conv3 pair (bs = 256) and PACS's conv2 pair (bs = 32)
    CV_DUAL(OP_SCATTER, CV_XF_BNBWD, CV_STAT_BWD, 64, 2, 64, 64, CV_XF_BNBWD, CV_XF_BNRELU, CV_STAT_NONE, 2, 0),
    CV_DUAL(OP_SCATTER, CV_XF_BNBWD, CV_STAT_BWD, 32, 1, 64, 64, CV_XF_BNBWD, CV_XF_BNRELU, CV_STAT_NONE, 2, 0),
};
#undef CV_DUAL

static const void* lookup(const int* dk, const int* gk) {
  for (const Ent& e : k_pairs) {
    bool ok = true;
    for (int i = 0; i < 5; ++i) ok = ok && e.dk[i] == dk[i];
    for (int i = 0; i < 7 && gk; ++i) ok = ok && e.gk[i] == gk[i];  // (gk null: any weight-gradient side)
    if (ok) return e.fn;
  }
  return nullptr;
}

static int g_on = -1;     // CV_DUAL=0: back to back (A/B); cv_debug_dual overrides
static int g_issued = 0;  // dual grids issued (test hook cv_debug_dual_count)

static int enabled() {
  if (g_on < 0) {
    const char* e = getenv("CV_DUAL");
    g_on = (e && atoi(e) == 0) ? 0 : 1;
  }
  return g_on;
}

static int launch_one(const void* kern, dim3 grid, size_t lds, void* arg, hipStream_t st, const char* what) {
  void* params[] = {arg};
  note_launch(kern);
  if (hipLaunchKernel(kern, grid, dim3(NT), params, lds, st) != hipSuccess) {
    (void)hipGetLastError();
    set_error("%s: launch failed", what);
    return 2;
  }
  return 0;
}

}  // namespace dual

// Issue the captured launches: one dual grid when the pair is served, else each on its own (direct first; the
// weight gradient on `side` when given: cv_conv_backward_deferred_kpack_side, which has made `side` wait for the
// work before the call).
// With a side stream the weight gradient overlaps this and the next layers' backward-data as its own launch, which
// beats the dual grid on the larger pairs (same box, two rounds: MNIST 0.4735 -> 0.4439 ms, CelebA 1.893 -> 1.845,
// C3 3.542 -> 3.497; PACS 0.804 -> 0.809 and C5 bf16 1.095 -> 1.100 slightly slower): a dual grid is then served only
// below side_dual_max() direct workgroups (CV_SIDE_DUAL_MAX, default 256; 0: never).
static long side_dual_max() {
  static long v = -1;
  if (v < 0) {
    const char* e = getenv("CV_SIDE_DUAL_MAX");
    v = e ? atol(e) : 256;
    if (v < 0) v = 0;
  }
  return v;
}
// ... or at batches of at most side_dual_n() images (CV_SIDE_DUAL_N, default 32: PACS's shard, 0.8015 -> 0.7955 ms
// with its conv2 pair dual; at 128 the C5 fp32 twin lost 3 % that way, 1.268 -> 1.307 ms, and bf16 was neutral)
static int side_dual_n() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CV_SIDE_DUAL_N");
    v = e ? atoi(e) : 32;
    if (v < 0) v = 0;
  }
  return v;
}
static bool side_keeps_dual(const direct::DirectCap& d) {
  return (long)d.grid.x * d.grid.y < side_dual_max() || d.a.g.n <= side_dual_n();
}

static int dual_issue(direct::DirectCap& d, fast::GemmCap& g, hipStream_t st, hipStream_t side = nullptr) {
  using namespace dual;
  if (d.got && g.got && enabled() && (!side || side_keeps_dual(d))) {
    const void* fn = lookup(d.key, g.key);
    const long nd = (long)d.grid.x * d.grid.y, ng = (long)g.grid.x * g.grid.y * g.grid.z;
    // (a direct grid of more than one resident round — VAE64's conv2 at 256 images, 1024 workgroups — measured
    // slower as a dual grid, 174 -> 215 us; MNIST's pairs at 512 direct workgroups gain 4-5 us each)
    if (fn && nd <= max_direct() && nd + ng < (1L << 31)) {
      const size_t lds = d.lds > g.lds ? d.lds : g.lds;
      bool ok = true;
      if (lds > 64 * 1024 && hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
        (void)hipGetLastError();
        ok = false;
      }
      {
        static int log = -1;
        if (log < 0) log = getenv("CV_DUAL_LOG") ? 1 : 0;
        if (log) {
          int occ = -1, occd = -1, occg = -1;
          (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, NT, lds);
          (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occd, d.kern, NT, d.lds);
          (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occg, g.kern, NT, g.lds);
          (void)hipGetLastError();
          fprintf(stderr, "dual nd=%ld ng=%ld (grid %ux%ux%u) lds d=%zu g=%zu occ dual=%d direct=%d gemm=%d\n", nd, ng,
                  g.grid.x, g.grid.y, g.grid.z, d.lds, g.lds, occ, occd, occg);
        }
      }
      if (ok) {
        // CV_DUAL_ORDER (A/B): 1 the direct role's workgroups first (default: the MNIST step 0.4984 -> 0.4907 ms,
        // the conv2 / conv3 pairs 58 -> 55 us in-step), 0 the roles alternating, 2 the WGRAD role first (0.4913 ms)
        static int order = -1;
        if (order < 0) {
          const char* e = getenv("CV_DUAL_ORDER");
          order = e ? atoi(e) : 1;
          if (order < 0 || order > 2) order = 1;
        }
        DualMap m{(int)nd, (int)d.grid.x, (int)d.grid.y, (int)ng, (int)g.grid.x, (int)g.grid.y, (int)g.grid.z, order};
        void* params[] = {&d.a, &g.a, &m};
        d.got = g.got = false;
        note_launch(fn);
        if (hipLaunchKernel(fn, dim3((unsigned)(nd + ng)), dim3(NT), params, lds, st) != hipSuccess) {
          (void)hipGetLastError();
          set_error("dual launch failed");
          return 2;
        }
        ++g_issued;
        return 0;
      }
    }
  }
  {
    static int log = -1;
    if (log < 0) log = getenv("CV_DUAL_LOG") ? 1 : 0;
    if (log && d.got && g.got)
      fprintf(stderr, "dual-unserved dkey=%d,%d,%d,%d,%d gkey=%d,%d,%d,%d,%d,%d,%d nd=%ld ng=%ld\n", d.key[0], d.key[1],
              d.key[2], d.key[3], d.key[4], g.key[0], g.key[1], g.key[2], g.key[3], g.key[4], g.key[5], g.key[6],
              (long)d.grid.x * d.grid.y, (long)g.grid.x * g.grid.y * g.grid.z);
  }
  int r = 0;
  if (d.got) {
    d.got = false;
    r = launch_one(d.kern, d.grid, d.lds, &d.a, st, "direct conv");
    if (r) return r;
  }
  if (g.got) {
    g.got = false;
    r = launch_one(g.kern, g.grid, g.lds, &g.a, side ? side : st, "gemm");
  }
  return r;
}

static thread_local direct::DirectCap t_dcap;
static thread_local fast::GemmCap t_gcap;

static thread_local bool t_side = false;  // (this capture issues the weight gradient on a side stream)
void dual_side(bool on) { t_side = on; }

int dual_wgrad_bm_cap() {  // (only when the captured direct launch belongs to a served pair)
  if (!direct::g_direct_cap || !t_dcap.got || !dual::enabled()) return 0;
  const long nd = (long)t_dcap.grid.x * t_dcap.grid.y;
  if (t_side && !side_keeps_dual(t_dcap)) return 0;
  return (nd <= dual::max_direct() && dual::lookup(t_dcap.key, nullptr)) ? 64 : 0;
}

// Workgroup slots the weight-gradient role of a served dual grid has in the grid's first resident round (0: no
// target): CUs x the dual kernel's workgroups per CU (LDS-bound: the larger of the direct role's carve-out and
// ~40 KB for the 64x64 WGRAD tile's) minus the direct role's workgroups.  CV_DUAL_WTARGET=1 (A/B, default off):
// the WGRAD split is cut so the whole grid is resident at once.
long dual_wgrad_slots() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("CV_DUAL_WTARGET");
    on = e ? atoi(e) : 0;
  }
  if (!on || !dual_wgrad_bm_cap()) return 0;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = -1;
    (void)hipGetLastError();
  }
  if (cus <= 0) return 0;
  const size_t lds = t_dcap.lds > 40 * 1024 ? t_dcap.lds : 40 * 1024;
  long per = (long)(160 * 1024 / lds);
  if (per > 4) per = 4;  // (the roles' registers: 4 workgroups of 4 waves)
  const long nd = (long)t_dcap.grid.x * t_dcap.grid.y;
  const long free = per * cus - nd;
  return free >= 128 ? free : 0;
}

void dual_begin() {
  t_dcap = direct::DirectCap();
  t_gcap = fast::GemmCap();
  t_dcap.want = t_gcap.want = true;
  direct::g_direct_cap = &t_dcap;
  fast::g_gemm_cap = &t_gcap;
}

int dual_end(hipStream_t st, bool issue, hipStream_t side) {
  direct::g_direct_cap = nullptr;
  fast::g_gemm_cap = nullptr;
  if (!issue) {  // (an error between begin and end: nothing captured is launched)
    t_dcap.got = t_gcap.got = false;
    return 0;
  }
  return dual_issue(t_dcap, t_gcap, st, side);
}

}  // namespace cv

extern "C" int cv_debug_dual(int on) {
  const int prev = cv::dual::enabled();
  if (on >= 0) cv::dual::g_on = on ? 1 : 0;
  return prev;
}

extern "C" int cv_debug_dual_count(int reset) {
  const int n = cv::dual::g_issued;
  if (reset) cv::dual::g_issued = 0;
  return n;
}
