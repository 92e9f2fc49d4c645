// Auxiliary-role launches: an NT-Xent phase (cv_ntxent.hpp; cv_latent.hip) issued as extra workgroups of a direct
// conv launch (cv_direct.hpp) in ONE grid.
//
// Why: the contrastive terms (trainer.py:474-479 through losses.py:98-137) depend only on the heads,
// yet their two launches (row log-sum-exps, then the losses and gradients) sat on the step's critical path between
// the decoder backward and the heads backward: 31 us of the MNIST step in two small grids (256 workgroups each).
// A second stream in the replayed graph costs more than that in fork / join edges (measured, cvhip/engine.py
// LATENT_SIDE), so the phases ride in grids that already run: the rows phase in the first decoder ConvTranspose2d's
// forward, the gradient phase in the second's (the gradients accumulate into a d(heads) the step's first launch
// zeroed; the KL / decoder-chain seed, cv_latent_combine_acc, adds onto them later).  The roles alternate over the
// first 2 x min(direct, aux) workgroups so every CU gets some of each; the grid's LDS and registers are the larger
// of the two roles'.  Served: the direct kernels of MNIST's decoder forward (the instantiations below); any other
// launch leaves the phase queued and cv_ntxent_aux_flush runs it on its own.
#include "cv_direct.hpp"
#include "cv_ntxent.hpp"

namespace cv {
thread_local AuxPend g_aux;

namespace aux {

struct AuxMap {
  int nd, dgx, dgy;  // direct workgroups and their grid
  int na, agx;       // aux workgroups and their grid's x extent (row blocks per branch)
  int order;         // 0: roles alternate over the first 2 min(nd, na); 1: direct first; 2: aux first
};

template <int OP, int XA, int EPI, int CBT, int FMX, int PHASE, int DM, bool REG>
__global__ __launch_bounds__(NT, 2) void direct_aux_kernel(const direct::DArgs PD, const NtArgs PA, const AuxMap m) {
  const int v = blockIdx.x;
  const int k = m.nd < m.na ? m.nd : m.na;
  int role, idx;
  if (m.order == 1) {
    role = v < m.nd ? 0 : 1;
    idx = role ? v - m.nd : v;
  } else if (m.order == 2) {
    role = v < m.na ? 1 : 0;
    idx = role ? v : v - m.na;
  } else if (v < 2 * k) {
    role = v & 1;
    idx = v >> 1;
  } else {
    role = m.nd > m.na ? 0 : 1;
    idx = k + (v - 2 * k);
  }
  if (role == 0) {
    direct::direct_body<OP, XA, EPI, CBT, FMX>(PD, idx % m.dgx, idx / m.dgx, m.dgx, m.dgy);
  } else if constexpr (PHASE == 0) {
    if constexpr (REG) ntxent_rows_reg_body<DM, NTR_JM>(PA, idx % m.agx, idx / m.agx);
    else ntxent_rows_lds_body<DM>(PA, idx % m.agx, idx / m.agx);
  } else {
    if constexpr (REG) ntxent_grad_reg_body<DM, NTR_JM>(PA, idx % m.agx, idx / m.agx);
    else ntxent_grad_lds_body<DM>(PA, idx % m.agx, idx / m.agx);
  }
}

struct Ent {
  int dk[5];  // direct OP, XA, EPI, CBT, FMX
  int phase, dm, reg;
  const void* fn;
};
#define CV_AUX(a, b, c, d, e, ph, dm)                                                             \
  Ent{{a, b, c, d, e}, ph, dm, 0, (const void*)direct_aux_kernel<a, b, c, d, e, ph, dm, false>}, \
      Ent{{a, b, c, d, e}, ph, dm, 1, (const void*)direct_aux_kernel<a, b, c, d, e, ph, dm, true>}
// MNIST's decoder forward: ConvT1 (SCATTER, untransformed input: the decoder Linear's BN1d + ReLU output) and ConvT2
// (SCATTER, BN+ReLU input), both with the STAT_FWD epilogue; d <= 8 (the bench's z = 16; a d = 16 gradient phase
// spilled 12 registers in this grid, so larger latents take the standalone launches)
static const Ent k_aux[] = {
    CV_AUX(OP_SCATTER, CV_XF_NONE, CV_STAT_FWD, 64, 1, 0, 8),   CV_AUX(OP_SCATTER, CV_XF_NONE, CV_STAT_FWD, 64, 1, 1, 8),
    CV_AUX(OP_SCATTER, CV_XF_BNRELU, CV_STAT_FWD, 32, 2, 0, 8), CV_AUX(OP_SCATTER, CV_XF_BNRELU, CV_STAT_FWD, 32, 2, 1, 8),
};
#undef CV_AUX

static int g_on = -1;      // CV_AUX=0: the NT-Xent phases launch on their own (A/B); cv_debug_aux overrides
static int g_merged = 0;   // merged launches issued (test hook cv_debug_aux_count)

static int enabled() {
  if (g_on < 0) {
    const char* e = getenv("CV_AUX");
    g_on = (e && atoi(e) == 0) ? 0 : 1;
  }
  return g_on;
}

}  // namespace aux

bool aux_enabled() { return aux::enabled() != 0; }
void aux_count_merged() { ++aux::g_merged; }

// the pending NT-Xent phase with this direct launch as one grid: 0 / 2 (launched / launch error), -1 (not served:
// the caller launches the direct kernel alone and the phase stays queued)
int direct_aux_launch(const int* dkey, const direct::DArgs& da, dim3 dgrid, size_t dlds, hipStream_t st) {
  using namespace aux;
  if (!g_aux.set || !enabled() || g_aux.stream != st) return -1;  // (queued for another stream: not this launch's)
  const NtArgs& pa = g_aux.a;
  if ((pa.with_combine && g_aux.phase != 0) || pa.d > 8 || pa.n > NT_MAXN) return -1;
  const int dm = 8;
  const int reg = (pa.d <= 8 && ntxent_reg_ok(pa, pa.nbr)) ? 1 : 0;  // (the DM = 8 instantiations below)
  const void* fn = nullptr;
  for (const Ent& e : k_aux) {
    bool ok = e.phase == g_aux.phase && e.dm == dm && e.reg == reg;
    for (int i = 0; i < 5; ++i) ok = ok && e.dk[i] == dkey[i];
    if (ok) fn = e.fn;
  }
  if (!fn) return -1;
  const bool need_lv = !(pa.sim == CV_SIM_COSINE || pa.sim == CV_SIM_L2);
  size_t alds = reg ? 0 : ntl_bytes(pa.n, pa.d, need_lv, g_aux.phase == 1);
  if (alds < 16 * sizeof(double)) alds = 16 * sizeof(double);
  const size_t lds = dlds > alds ? dlds : alds;
  if (lds > 144 * 1024) return -1;
  if (lds > 64 * 1024 && hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  const long nd = (long)dgrid.x * dgrid.y;
  const int agx = (pa.n + pa.rpb - 1) / pa.rpb;
  const long na = (long)agx * pa.nbr + (pa.with_combine ? 1 : 0);  // (+ the combine block: bx 0, by nbr)
  // CV_AUX_ORDER (A/B): 1 the direct role's workgroups first (default: the MNIST step 0.4910 -> 0.4814 ms — dispatched
  // first, the conv workgroups take their two slots per CU and the NT-Xent workgroups fill the third), 0 the roles
  // alternating, 2 the NT-Xent workgroups first (0.4840 ms)
  static int order = -1;
  if (order < 0) {
    const char* e = getenv("CV_AUX_ORDER");
    order = e ? atoi(e) : 1;
    if (order < 0 || order > 2) order = 1;
  }
  AuxMap m{(int)nd, (int)dgrid.x, (int)dgrid.y, (int)na, agx, order};
  {
    static int log = -1;
    if (log < 0) log = getenv("CV_AUX_LOG") ? 1 : 0;
    if (log) {
      int occ = -1;
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, NT, lds);
      (void)hipGetLastError();
      fprintf(stderr, "aux phase=%d reg=%d nd=%ld na=%ld dlds=%zu alds=%zu occ=%d\n", g_aux.phase, reg, nd, na, dlds,
              alds, occ);
    }
  }
  direct::DArgs a = da;
  NtArgs b = pa;
  void* params[] = {&a, &b, &m};
  g_aux.set = 0;
  note_launch(fn);
  if (hipLaunchKernel(fn, dim3((unsigned)(nd + na)), dim3(NT), params, lds, st) != hipSuccess) {
    (void)hipGetLastError();
    set_error("direct + NT-Xent launch failed");
    return 2;
  }
  ++g_merged;
  return 0;
}

}  // namespace cv

extern "C" int cv_debug_aux(int on) {
  const int prev = cv::aux::enabled();
  if (on >= 0) cv::aux::g_on = on ? 1 : 0;
  return prev;
}

extern "C" int cv_debug_aux_count(int reset) {
  const int n = cv::aux::g_merged;
  if (reset) cv::aux::g_merged = 0;
  return n;
}
