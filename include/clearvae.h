/*
 * clearvae.h — C-ABI of libclearvae_hip.so, the MI355X (gfx950) hot path of CLEAR-VAE training.
 *
 * The reference (scotsun/clear-vae) is pure PyTorch eager and has no FFI; every entry point below
 * replaces a group of ATen calls made by the reference's Python code.  Each declaration cites the
 * reference lines (paths relative to the reference's repo root) whose arithmetic it implements.
 * The Python binding is clear-vae_amd/cvhip/_lib.py (ctypes); see INTEGRATION.md.
 *
 * Conventions
 *   - every pointer is a device pointer owned by the caller (PyTorch's caching allocator); the library
 *     never allocates, frees or synchronises, so every call can be captured into a HIP graph;
 *   - activations are NHWC fp32 ("pixels x channels" row-major); weights keep PyTorch's layouts
 *     (Conv2d [Cout][Cin][kh][kw], ConvTranspose2d [Cin][Cout][kh][kw], Linear [out][in]);
 *   - BatchNorm batch statistics are accumulated in fp64 by the producing kernel's epilogue into
 *     CV_STAT_REPL(C) replicas of [2][C] doubles (sum, sum of squares / sum dz, sum dz*xhat); when the
 *     layer carries a ticket (cv_bn.ticket), the last workgroup of the producing launch folds them into
 *     per-channel constants (cv_bn.cfwd / cv_bn.cbwd) that consuming GEMMs load in their prologue,
 *     otherwise each consumer folds the replicas itself (the normalised activation is never written
 *     to HBM);
 *   - return value 0 = success; otherwise cv_last_error() describes the failure (host-side checks
 *     run before any launch, so a failing call enqueues nothing).
 */
#ifndef CLEARVAE_H
#define CLEARVAE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* cv_stream_t; /* a hipStream_t (torch.cuda.current_stream().cuda_stream) */

/* Replicas of a C-feature statistics buffer: narrow layers get more replicas so that the fp64
 * atomics of thousands of producer workgroups do not serialise on a few addresses. */
#define CV_REC_REPL 32
#define CV_STAT_REPL(C) ((C) >= 256 ? 8 : (C) >= 64 ? 16 : 32)
#define CV_TICKET_WORDS 130

/* ---- BatchNorm as seen by a fused prologue/epilogue (nn.BatchNorm1d/2d, vae.py:17-44, 115-154) ---- */
typedef struct cv_bn {
  const float* gamma;        /* [C] PyTorch order                                              */
  const float* beta;         /* [C]                                                            */
  const double* stat;        /* [CV_STAT_REPL(C)][2][C] forward sums (sum x, sum x^2)         */
  const double* gstat;       /* [CV_STAT_REPL(C)][2][C] backward sums (sum dz, sum dz*xhat)   */
  const float* running_mean; /* [C]                                                            */
  const float* running_var;  /* [C]                                                            */
  int C;                     /* normalised features                                            */
  int count;                 /* elements per feature in the batch (N*H*W, or N for BN1d)       */
  int train;                 /* 1: batch statistics, 0: running statistics (eval mode)         */
  float eps;
  /* Finalised constants (train mode; optional).  A launch of the specialised GEMM core that produces
   * this layer's forward sums (CV_STAT_FWD epilogue with this layer as ebn) elects its last workgroup
   * with ticket[0] and writes cfwd = [sc][mu][beta][istd] (4*C floats, sc = gamma*istd); one that
   * produces the backward sums (CV_STAT_BWD epilogue) uses ticket[1] and writes
   * cbwd = [sc][c1][mu][istd][c2] (5*C floats, c1 = sum dz / n, c2 = sum dz*xhat / n).  A consuming
   * GEMM uses cfwd / cbwd only when the matching ticket is non-zero (its producer finalised) and
   * otherwise folds the replica sums itself; every other producer leaves the ticket at zero.  The
   * arrivals are counted in two levels (<= 64 groups of workgroups, CV_TICKET_WORDS words:
   * ticket[0..1] = groups done, then 64 group counters per direction) so thousands of workgroups do
   * not serialise on one address.  All words must be zero before the producing launch (they live in
   * the zeroed statistics arena). */
  float* cfwd;
  float* cbwd;
  unsigned int* ticket;      /* [CV_TICKET_WORDS] */
} cv_bn;

/* transform applied while an operand is staged into LDS */
enum { CV_XF_NONE = 0, CV_XF_BNRELU = 1, CV_XF_BNBWD = 2 };
/*   CV_XF_BNRELU : v = max(x*gamma*istd + (beta - mean*gamma*istd), 0)               (BN fwd + ReLU)
 *   CV_XF_BNBWD  : v = gamma*istd*(dz - sum(dz)/n - xhat*sum(dz*xhat)/n), xhat from y  (BN bwd)      */

typedef struct cv_operand {
  const float* x;  /* primary tensor: activation, or dz (masked upstream gradient) for BNBWD    */
  const float* y;  /* BNBWD only: the BN layer's input (pre-BN values), same layout as x        */
  int xf;          /* CV_XF_*                                                                  */
  int nchw;        /* 1: x is NCHW (network input, channels not a multiple of 4); else NHWC    */
  cv_bn bn;        /* constants source for the transform                                       */
} cv_operand;

/* epilogue statistics of the produced tensor */
enum { CV_STAT_NONE = 0, CV_STAT_FWD = 1, CV_STAT_BWD = 2 };
/*   CV_STAT_FWD: out is the input of a BN layer; accumulate (sum v, sum v^2) into stat_out.
 *   CV_STAT_BWD: out is d(post-ReLU activation) of BN layer `ebn` whose input is `ey`; the kernel
 *                stores dz = v * [relu active] and accumulates (sum dz, sum dz*xhat) into stat_out. */

typedef struct cv_epilogue {
  int stat_mode;      /* CV_STAT_*                                                  */
  double* stat_out;   /* [REPL][2][C]                                               */
  int stat_div;       /* feature index = column / stat_div (1 = per column)         */
  const float* ey;    /* STAT_BWD: pre-BN values at the output positions            */
  cv_bn ebn;          /* the BN layer fed by this output: STAT_BWD needs its batch statistics;
                         with ebn.ticket set (either mode) the producer finalises its constants */
  int erelu;          /* STAT_BWD: 1 if ReLU follows that BN                        */
} cv_epilogue;

/* Operand precision of a conv / linear contraction.  CV_MMA_BF16 (BASELINE configs[4], "bf16"): the
 * specialised MFMA core rounds both operands to bf16 as it stages them into LDS (after the fp32 BatchNorm
 * transform) and contracts on v_mfma_f32_16x16x32_bf16 with fp32 accumulation; activations, BatchNorm
 * statistics and epilogues stay fp32.  Calls the core does not serve (image-facing edge layers) stay
 * fp32.  The reference is fp32 only (CV_MMA_FP32, the default). */
enum { CV_MMA_FP32 = 0, CV_MMA_BF16 = 1 };

/* ---- convolution geometry (nn.Conv2d / nn.ConvTranspose2d, vae.py:15-46, 113-156) ---- */
typedef struct cv_conv {
  int n;                          /* batch                                         */
  int c_in, h_in, w_in;           /* layer input  (NHWC)                           */
  int c_out, h_out, w_out;        /* layer output (NHWC)                           */
  int kh, kw, stride, pad;
  int transposed;                 /* 0 Conv2d, 1 ConvTranspose2d                   */
  int mma;                        /* CV_MMA_*: operand precision of the contraction */
} cv_conv;

/* GEMM-native copies of a conv / convT weight, refreshed once per optimizer step.  With
 * w(cs, cb, tap) = W[cs][cb][kh][kw] (PyTorch layout; cs = out channels for Conv2d, in channels for
 * ConvTranspose2d): gather = Wg[tap][cb][cs], scatter = Ws[tap][cs][cb].  Conv2d forward and
 * ConvTranspose2d backward-data read `gather`; Conv2d backward-data and ConvTranspose2d forward read
 * `scatter`.  Up to 16 weights per call (one launch). */
typedef struct cv_conv_pack {
  const float* src; float* gather; float* scatter;
  int cs, cb, kh, kw;
} cv_conv_pack;
int cv_pack_conv_weights(const cv_conv_pack* items, int n, cv_stream_t stream);
/* cv_pack_conv_weights plus, in the same launch, zeroing of up to 8 buffers (4-byte granular) that are not
 * touched by the packing: the first launch of a training step clears the step's accumulators with it. */
int cv_pack_conv_weights_zero(const cv_conv_pack* items, int n, void* const* zero_ptrs, const size_t* zero_bytes,
                              int zero_count, cv_stream_t stream);
/* (cv_pack_conv_weights_zero / _zero_copy accept n = 0 items when they have buffers to zero or copy) */
/* torch.optim.Adam over a flat parameter arena (cv_adam_step, trainer.py:483) with the weight packing of
 * cv_pack_conv_weights in the same launch: the packing workgroups update their tile's parameters and pack the new
 * values (the items' src must lie inside params[0, numel)), the rest of the arena is updated by the launch's other
 * workgroups; the last workgroup advances step[0] (and aux_counter).  The packed copies are then current for the
 * next step's forward without a packing launch. */
int cv_adam_pack_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t numel,
                      const float* hyper, int64_t* step, const float* grad_scale, int64_t* aux_counter,
                      const cv_conv_pack* items, int n, cv_stream_t stream);
/* cv_adam_pack_step over a part of the arena (params .. params + numel, the items inside it) that leaves the step
 * counters as they are when advance = 0: a split update whose parts run at different points of the step (the
 * decoder's parameters as soon as the step has read them, beside the encoder backward); the part with advance = 1
 * (issued after the others, same step) advances step[0] and aux_counter.  Every part computes the bias correction
 * from the same step[0]. */
int cv_adam_pack_step_part(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t numel,
                           const float* hyper, int64_t* step, const float* grad_scale, int64_t* aux_counter,
                           const cv_conv_pack* items, int n, int advance, cv_stream_t stream);
/* cv_pack_conv_weights_zero plus up to 4 device copies (16-byte aligned and sized) in the same launch: the fused
 * step's first launch of a replayed step also moves the batch (X, labels: trainer.py:447-450's `X.to(device)` of a
 * device-resident batch) into the step graph's static input buffers, so the copy is not a launch of its own. */
int cv_pack_conv_weights_zero_copy(const cv_conv_pack* items, int n, void* const* zero_ptrs, const size_t* zero_bytes,
                                   int zero_count, void* const* copy_dst, const void* const* copy_src,
                                   const size_t* copy_bytes, int copy_count, cv_stream_t stream);

/* y = conv(T(x)) + bias.  Replaces nn.Conv2d/ConvTranspose2d.forward (vae.py:15-46) with the
 * preceding BatchNorm2d+ReLU fused into the operand load and the following BatchNorm2d's batch
 * statistics fused into the epilogue.  wpacked: the `gather` (Conv2d) or `scatter`
 * (ConvTranspose2d) packing of cv_pack_conv_weights. */
int cv_conv_forward(const cv_conv* g, const cv_operand* in, const float* wpacked, const float* bias,
                    float* out, const cv_epilogue* ep, cv_stream_t stream);

/* dx = conv^T(T(dy)).  Replaces the grad_input half of aten::convolution_backward.
 * wpacked: `scatter` (Conv2d) or `gather` (ConvTranspose2d) packing. */
int cv_conv_backward_data(const cv_conv* g, const cv_operand* gout, const float* wpacked,
                          float* gin, const cv_epilogue* ep, cv_stream_t stream);

/* The same calls given also wkpack = the OTHER packing of the same weight (the one wpacked is not: for a
 * stride-2 SCATTER contraction — Conv2d backward-data, ConvTranspose2d forward — the `gather` packing
 * [tap][cb][cs]; for a GATHER — Conv2d forward, ConvTranspose2d backward-data — the `scatter` packing
 * [tap][cs][cb]; i.e. the contraction's B operand k-contiguous per output channel; NULL allowed).  Results are
 * those of the calls without it; with it the library may run the contraction as one direct launch that stages
 * the operand's band in LDS once per workgroup and walks all taps (and, for SCATTER, all four stride-parity
 * classes) from there (cv_direct.hip) instead of implicit GEMMs that re-load it per tap.  Replaces the same
 * ATen calls (vae.py:15-46, 113-156). */
int cv_conv_forward_kpack(const cv_conv* g, const cv_operand* in, const float* wpacked, const float* wkpack,
                          const float* bias, float* out, const cv_epilogue* ep, cv_stream_t stream);
int cv_conv_backward_data_kpack(const cv_conv* g, const cv_operand* gout, const float* wpacked,
                                const float* wkpack, float* gin, const cv_epilogue* ep, cv_stream_t stream);

/* dw += sum_pixels T(x) (x) T(dy).  Replaces the grad_weight half of aten::convolution_backward.
 * gbias (optional, Conv2d only) += sum_pixels T(dy).  The pixel sum is split over workgroups
 * (split_k <= 0: automatic); the partial tiles go to `work` (cv_conv_wgrad_workspace_bytes) and one
 * reduction launch adds them into gweight/gbias.  With work == NULL the partials are fp32 atomics
 * into gweight/gbias instead (correct, slower).  Either way the result is added to gweight/gbias. */
size_t cv_conv_wgrad_workspace_bytes(const cv_conv* g, int split_k);
int cv_conv_backward_weight(const cv_conv* g, const cv_operand* in, const cv_operand* gout,
                            float* gweight, float* gbias, int split_k, float* work, size_t work_bytes,
                            cv_stream_t stream);

/* Deferred weight gradients: the same contraction as cv_conv_backward_weight (split_k automatic, `work`
 * required) but the split-K partial tiles stay in `work` and their layout is written to *defer (host
 * struct, filled at enqueue time) instead of launching the reduction; cv_step_reduce sums them later,
 * together with every other deferred gradient of the step, in one launch.  defer->split == 0: the
 * launch wrote gweight / gbias directly (nothing to reduce).  `work` must stay untouched until then. */
typedef struct cv_wgrad_defer {
  const float* part;   /* [split][M][ntot] partial tiles                                   */
  int split, M, N, ntot, cb, kk;
  float* gweight;      /* += sum over splits, element (m, col = tap*cb + c) -> [m][c][tap]  */
  float* gbias;        /* column N (if ntot > N): += row sums                              */
} cv_wgrad_defer;
int cv_conv_backward_weight_deferred(const cv_conv* g, const cv_operand* in, const cv_operand* gout,
                                     float* gweight, float* gbias, float* work, size_t work_bytes,
                                     cv_wgrad_defer* defer, cv_stream_t stream);

/* Both halves of a conv / convT backward (aten::convolution_backward, trainer.py:482): dx as
 * cv_conv_backward_data and the deferred weight gradient as cv_conv_backward_weight_deferred, in one launch for
 * the image-side ConvTranspose2d (vae.py:43 / :153: the edge kernels' geometry, ep's BatchNorm = in's
 * transform), otherwise the two launches in that order. */
int cv_conv_backward_deferred(const cv_conv* g, const cv_operand* gout, const float* wpacked, float* gin,
                              const cv_epilogue* ep, const cv_operand* in, float* gweight, float* gbias, float* work,
                              size_t work_bytes, cv_wgrad_defer* defer, cv_stream_t stream);
/* cv_conv_backward_deferred with the other packing of the weight (see cv_conv_forward_kpack) */
int cv_conv_backward_deferred_kpack(const cv_conv* g, const cv_operand* gout, const float* wpacked,
                                    const float* wkpack, float* gin, const cv_epilogue* ep, const cv_operand* in,
                                    float* gweight, float* gbias, float* work, size_t work_bytes,
                                    cv_wgrad_defer* defer, cv_stream_t stream);
/* cv_conv_backward_deferred_kpack with the weight-gradient launch on `side` where the pair is not one dual grid:
 * `side` waits for the work issued on `stream` before the call (an event; in a capture the side stream joins the
 * graph there), then runs the weight gradient beside this and the next layers' backward-data launches.  The caller
 * joins `side` back into `stream` before the deferred partials are read (cv_step_reduce).  Dual grids, the
 * image-side ConvTranspose2d's fused launch and the self-reducing split (CV_WGRAD_SELF) stay on `stream`;
 * side = NULL or = stream: cv_conv_backward_deferred_kpack. */
int cv_conv_backward_deferred_kpack_side(const cv_conv* g, const cv_operand* gout, const float* wpacked,
                                         const float* wkpack, float* gin, const cv_epilogue* ep,
                                         const cv_operand* in, float* gweight, float* gbias, float* work,
                                         size_t work_bytes, cv_wgrad_defer* defer, cv_stream_t side,
                                         cv_stream_t stream);

/* ---- fully connected layers (nn.Linear heads vae.py:27-30; decoder Linear vae.py:33) ----
 * A linear layer whose input (or output) is the NCHW-flattened view of an NHWC activation with
 * `*_pix` pixels and `*_ch` channels (nn.Flatten vae.py:25 / nn.Unflatten vae.py:36).              */
typedef struct cv_linear {
  int n;               /* batch rows                         */
  int in_features, out_features;
  int in_pix, in_ch;   /* in_features = in_pix*in_ch, or in_pix = 1 for a plain row-major input   */
  int out_pix, out_ch; /* same for the output                                                      */
  int mma;             /* CV_MMA_*                                                                  */
} cv_linear;

int cv_linear_forward(const cv_linear* g, const cv_operand* in, const float* weight,
                      const float* bias, float* out, int accumulate, const cv_epilogue* ep,
                      cv_stream_t stream);
int cv_linear_backward_data(const cv_linear* g, const cv_operand* gout, const float* weight,
                            float* gin, int accumulate, const cv_epilogue* ep, cv_stream_t stream);
/* dW += sum_n gout[n] (x) T(in[n]) (+ gbias), same split/workspace contract as the conv version. */
size_t cv_linear_wgrad_workspace_bytes(const cv_linear* g, int split_k);
int cv_linear_backward_weight(const cv_linear* g, const cv_operand* gout, const cv_operand* in,
                              float* gweight, float* gbias, int split_k, float* work, size_t work_bytes,
                              cv_stream_t stream);

int cv_linear_backward_weight_deferred(const cv_linear* g, const cv_operand* gout, const cv_operand* in,
                                       float* gweight, float* gbias, float* work, size_t work_bytes,
                                       cv_wgrad_defer* defer, cv_stream_t stream);

/* Decoder Linear -> BatchNorm1d -> ReLU backward (vae.py:33-35).  da: gradient w.r.t. the ReLU
 * output in the Unflatten/NHWC order (g->out_pix, g->out_ch); h: the Linear output (BN1d input),
 * same order.  Two launches: (1) mask da in place (da <- dz) and accumulate the BN1d backward sums
 * into gstat_out (fp64, replicas; caller zeroes); (2) accumulate the Linear weight gradient
 * dW[f][k] += sum_n BNbwd(dz)[n][f] * zin[n][k] (caller zeroes).  gweight == NULL runs only (1);
 * gstat_out == NULL runs only (2) on an already masked da with bn->gstat holding the sums (so the
 * weight gradient can run off the critical path, on another stream, after (1)). */
int cv_declinear_backward_weight(const cv_linear* g, float* da, const float* h, const cv_bn* bn,
                                 double* gstat_out, const float* zin, float* gweight,
                                 cv_stream_t stream);

/* The decoder's input block in one launch each way (cv_declinear.hip): a workgroup owns 16 features of the
 * [n][out_features] activation for the whole batch, so the BatchNorm1d statistics are complete inside it.
 * Forward (VAE.sample vae.py:56-60, then decoder Linear -> BatchNorm1d -> ReLU vae.py:33-35): heads != NULL:
 * z = mu + eps*exp(lv/2) from heads [n][4d] exactly as cv_reparam_forward (eps injected, or Philox(seed,
 * offset[0]) with offset advanced once), written to z; heads == NULL: z [n][2d] is the input.  h = Linear(z)
 * (storage order out_pix/out_ch), ah = ReLU(BN1d(h)); train: the complete batch sums of h are written to
 * replica 0 of stat_out [REPL][2][F] (the other replicas must be zero).  Replaces cv_reparam_forward +
 * cv_linear_forward + cv_bn_apply.
 * Backward (trainer.py:482 through vae.py:33-35): ga [n][F] = d(ReLU output) is overwritten with d(h) (ReLU
 * mask, then the BN1d backward transform); gstat_out replica 0 receives the complete backward sums; gweight
 * [F][2d] += d(h)^T z; with dz != NULL also dz [n][2d] += d(h) W (weight = the Linear's [F][2d]; each workgroup
 * adds its 16 features' share with fp32 atomics, the caller zeroes dz), else dz is left to
 * cv_linear_backward_data on d(h).  Replaces the two launches of cv_declinear_backward_weight (and the dz GEMM).  Contract: cv_decoder_input_supported(n, d, F) (n*2d <= 16384,
  * 2d <= 128, F % 16 == 0, d even). */
int cv_decoder_input_supported(int n, int d, int features);
int cv_decoder_input_forward(const cv_linear* g, const float* heads, const float* eps, uint64_t seed,
                             uint64_t* offset, float* z, const float* weight, const float* bias, const cv_bn* bn,
                             double* stat_out, float* h, float* ah, cv_stream_t stream);
int cv_decoder_input_backward(const cv_linear* g, float* ga, const float* h, const cv_bn* bn, double* gstat_out,
                              const float* z, float* gweight, const float* weight, float* dz, cv_stream_t stream);

/* Encoder heads forward in one launch (the four nn.Linear heads vae.py:27-30 over the Flatten of the last conv
 * block vae.py:25, its BatchNorm2d + ReLU applied to y on load): heads [n][4d] = ReLU(BN(y)) W^T + bias with W
 * packed [in_features (storage order)][4d] (cv_conv_pack of the [4d][C][Hh][Wh] view, `gather` order), and, when
 * z != NULL, the reparameterisation of its rows exactly as cv_reparam_forward (vae.py:56-60).  Replaces
 * cv_linear_forward of the heads (+ cv_reparam_forward).  Contract: cv_heads_forward_supported(n,
 * in_features, in_ch, d) (d = 8 or a multiple of 16 up to 64, in_ch % 4 == 0, in_ch <= 512). */
int cv_heads_forward_supported(int n, int in_features, int in_ch, int d);
int cv_heads_forward(const cv_linear* g, const float* y, const cv_bn* bn, const float* wpacked, const float* bias,
                     float* heads, const float* eps, uint64_t seed, uint64_t* offset, float* z, cv_stream_t stream);

/* Encoder heads backward in one launch (the four nn.Linear heads vae.py:27-30 as one [4d][F] weight over the
 * Flatten of the last conv block, vae.py:25; trainer.py:482): gin [n][F] (storage order in_pix/in_ch) =
 * (dheads W) * [BN(y) > 0] with that BatchNorm2d's backward sums added to gstat_out (fp64 replicas; the layer's
 * cbwd constants are finalised by the last workgroup when bn carries a ticket), gweight [4d][F] +=
 * dheads^T ReLU(BN(y)), gbias [4d] += column sums of dheads.  Replaces cv_linear_backward_data with a
 * CV_STAT_BWD epilogue plus cv_linear_backward_weight(_deferred) of the heads.  Contract:
 * cv_heads_backward_supported(n, in_features, in_ch, out_features) (4d <= 128, dheads staged in LDS). */
int cv_heads_backward_supported(int n, int in_features, int in_ch, int out_features);
int cv_heads_backward(const cv_linear* g, const float* dheads, const float* weight, const float* y, const cv_bn* bn,
                      float* gin, double* gstat_out, float* gweight, float* gbias, cv_stream_t stream);
/* The decoder gradient chained through the reparameterisation z = mu + eps * exp(logvar / 2) (vae.py:56-60),
 * applied by cv_heads_backward_chain while it stages dheads: column block b of a row (mu_c, lv_c, mu_s, lv_s) gets
 * + dz[z index] (mu blocks) or + dz * (z - mu) / 2 (logvar blocks), z index = (b / 2) * d + k — the chain term of
 * cv_latent_combine, so that the KL part of the combine can run earlier in the step (cv_ntxent_aux_combine) and
 * the decoder's dz is consumed where dheads is.  dheads itself is not rewritten.  rec_in / losses (optional):
 * losses[0] = the sum of the CV_REC_REPL replicas of rec_in. */
typedef struct cv_latent_chain {
  const float* heads;  /* [n][4d] */
  const float* z;      /* [n][2d] */
  const float* dz;     /* [n][2d] */
  int d;
  const double* rec_in;
  float* losses;
} cv_latent_chain;
int cv_heads_backward_chain(const cv_linear* g, const float* dheads, const cv_latent_chain* chain, const float* weight,
                            const float* y, const cv_bn* bn, float* gin, double* gstat_out, float* gweight,
                            float* gbias, cv_stream_t stream);

/* out = max(BN(x), 0) elementwise for a BatchNorm1d over `features` PyTorch-order features whose
 * tensor is stored in the Unflatten/NHWC order (pix, ch) (vae.py:34-36); rows = batch. */
int cv_bn_apply(const cv_bn* bn, const float* x, float* out, int rows, int features, int pix, int ch,
                int relu, cv_stream_t stream);

/* ---- BatchNorm running statistics (nn.BatchNorm*, momentum 0.1, unbiased running var) ---- */
int cv_bn_update_running(const cv_bn* bn, int nlayers, float momentum,
                         int64_t* const* num_batches_tracked, cv_stream_t stream);
/* nsets forwards' momentum updates of the same nlayers BatchNorms in one launch, applied in set order: bn is
 * [nsets][nlayers] (set-major; layer i of every set names the same running buffers, count and C, with its own
 * batch sums in .stat); num_batches_tracked advances by nsets (CLEAR-MIM's five estimator forwards,
 * trainer.py:873-888). */
int cv_bn_update_running_sets(const cv_bn* bn, int nlayers, int nsets, float momentum, int64_t* const* nbt,
                              cv_stream_t stream);
/* copy batch stats into (mean, invstd) float arrays (for tests / PyTorch-visible save_mean) */
int cv_bn_batch_stats(const cv_bn* bn, float* mean, float* invstd, cv_stream_t stream);

/* ---- decoder output: BatchNorm2d(C) + Sigmoid (vae.py:44-45) ---- */
/* xhat = sigmoid(BN(y)), written NCHW [n][c][h][w]; y is NHWC [n][h][w][c]. */
int cv_output_forward(const cv_bn* bn, const float* y, int n, int c, int hw, float* xhat,
                      cv_stream_t stream);
/* fused output + reconstruction loss (losses.py:36-47): rec = mean_n sum_chw (xhat - x)^2,
 * accumulated into the CV_REC_REPL fp64 replicas rec_out[0..CV_REC_REPL) (caller zeroes; rec is
 * their sum), and when dv_out != NULL the gradient of
 * (rec_scale*rec) w.r.t. the BN output: dv = rec_scale*2(xhat-x)/n * xhat(1-xhat) (NHWC), plus the
 * BN backward sums into gstat_out.  rec_scale may be NULL (1.0). x is NCHW. */
int cv_output_loss(const cv_bn* bn, const float* y, const float* x, int n, int c, int hw,
                   float* xhat, double* rec_out, float* dv_out, double* gstat_out,
                   const float* rec_scale, cv_stream_t stream);
/* The last ConvTranspose2d (vae.py:43 / :153) and cv_output_loss in one call: y = convT(T(in)) + bias with its
 * output BatchNorm's sums (ep, CV_STAT_FWD into bn->stat), then the decoder output, the reconstruction term and
 * its backward seed exactly as cv_output_loss.  One launch when the edge kernel serves the layer and its whole
 * grid is resident at once (the workgroups meet at a bounded grid-wide wait for the BN sums); else the two
 * calls. */
int cv_convt_output_loss(const cv_conv* g, const cv_operand* in, const float* wpacked, const float* bias, float* y,
                         const cv_epilogue* ep, const cv_bn* bn, const float* x, float* xhat, double* rec_out,
                         float* dv_out, double* gstat_out, const float* rec_scale, cv_stream_t stream);
/* backward of xhat = sigmoid(BN(y)) given dxhat (NCHW): dv (NHWC) + BN backward sums. */
int cv_output_backward(const cv_bn* bn, const float* y, const float* xhat, const float* dxhat,
                       int n, int c, int hw, float* dv_out, double* gstat_out, cv_stream_t stream);

/* ---- reparameterisation (vae.py:56-79) ---- */
/* heads: [n][4d] = (mu_c | logvar_c | mu_s | logvar_s); z: [n][2d] = (z_c | z_s).
 * eps == NULL: eps ~ N(0,1) from a counter-based Philox4x32-10 stream keyed by (seed, offset[0]);
 * offset is a device uint64[2] (counter, zeroed arrival word) advanced by the kernel (graph-replay
 * safe).  eps != NULL: [n][2d]
 * injected noise (test hook).  eps_out (optional) receives the noise used. */
int cv_reparam_forward(const float* heads, int n, int d, const float* eps, uint64_t seed,
                       uint64_t* offset, float* z, float* eps_out, cv_stream_t stream);

/* VAE.sample for one factor (vae.py:56-60): z = mu + eps*exp(0.5*logvar), [n][d] contiguous;
 * eps injected or drawn from Philox(seed, offset[0]) (offset advanced).  Backward:
 * dmu = dz, dlogvar = dz*(z-mu)/2 (accumulated into dmu/dlogvar when accumulate != 0). */
int cv_sample_forward(const float* mu, const float* logvar, long numel, const float* eps,
                      uint64_t seed, uint64_t* offset, float* z, cv_stream_t stream);
int cv_sample_backward(const float* mu, const float* z, const float* dz, long numel, float* dmu,
                       float* dlogvar, int accumulate, cv_stream_t stream);

/* ---- latent-space losses (losses.py:41-137) ---- */
enum { CV_SIM_COSINE = 0, CV_SIM_L2 = 1, CV_SIM_MODIFIED_L2 = 2, CV_SIM_JEFFREY = 3,
       CV_SIM_MAHALANOBIS = 4 };

/* KL term of vae_loss (losses.py:48-49): kl = -0.5 * mean_n sum_d(1 + lv - mu^2 - exp(lv));
 * with dmu/dlogvar != NULL also writes (or accumulates) gscale[0] * d kl / d(mu, logvar). */
int cv_kl(const float* mu, const float* logvar, int ld, int n, int d, float* kl_out,
          const float* gscale, float* dmu, float* dlogvar, int gld, int accumulate,
          cv_stream_t stream);

/* Fused-step seed of d(heads): KL(c), KL(s) with the LogisticAnnealer weight
 * w = beta/(1+exp(-(t-loc)/scale)), t = anneal_step[0] (trainer.py:22-38, 474-477), plus the decoder
 * gradient dz chained through z = mu + eps*exp(lv/2).  losses[0] = sum of the CV_REC_REPL
 * replicas rec_in[] of cv_output_loss (if given),
 * losses[1], losses[2] = kl_c, kl_s; losses[7] = w.  dheads is overwritten. */
int cv_latent_combine(const float* heads, const float* z, const float* dz, int n, int d, float beta,
                      float loc, float scale, const int64_t* anneal_step, const double* rec_in,
                      float* dheads, float* losses, double* work, cv_stream_t stream);
/* cv_latent_combine with dheads += instead of overwritten: the fused step whose NT-Xent gradients were already
 * accumulated into a zeroed dheads — the default schedule (cvhip/engine.py LATENT_AUX: the NT-Xent phases ride in the
 * decoder's ConvTranspose2d forward grids and this call follows the decoder backward), or the opt-in side stream
 * (LATENT_SIDE, joined before this call). */
int cv_latent_combine_acc(const float* heads, const float* z, const float* dz, int n, int d, float beta,
                          float loc, float scale, const int64_t* anneal_step, const double* rec_in,
                          float* dheads, float* losses, double* work, cv_stream_t stream);
/* work (or NULL): a caller-owned device workspace of cv_latent_combine_workspace_bytes(), zeroed once before its
 * first use (it is left zeroed after every call).  With it, batches of n x 2d >= 4096 elements run over several
 * workgroups whose KL partials are summed in workgroup order by the last to arrive (bit-reproducible, independent of
 * arrival order); NULL runs the one-workgroup kernel.  Two launches that may overlap in time (two streams) need two
 * workspaces. */
size_t cv_latent_combine_workspace_bytes(void);
/* cv_latent_combine(_acc) (accumulate 0 / 1) with the decoder-input gradient computed here: dz = d(h) W, d(h) the
 * decoder Linear's output gradient [n][F] in storage order (cv_decoder_input_backward's `ga` after the call, with
 * dz = NULL there), W the Linear weight [F][2d] (lin: the decoder Linear's geometry, out_pix / out_ch its Unflatten;
 * F % 64 == 0).  Deterministic: every dz element is one fixed-order sum (the atomics of the decoder-input backward's
 * dz partials were the fused step's only order-dependent sum).  dz_out (or NULL) receives dz.  work (required): a
 * caller-owned device workspace of cv_latent_combine_dz_workspace_bytes(n, d), zeroed once before its first use. */
size_t cv_latent_combine_dz_workspace_bytes(int n, int d);
int cv_latent_combine_dz(const float* heads, const float* z, const float* dh, const float* weight, const cv_linear* lin,
                         float beta, float loc, float scale, const int64_t* anneal_step, const double* rec_in,
                         float* dheads, float* losses, float* dz_out, int accumulate, double* work, cv_stream_t stream);

/* reconstruction term (losses.py:45-47) for the autograd path: rec = mean_n sum (xhat - x)^2;
 * work: one zeroed fp64 word.  dxhat != NULL: dxhat = gscale[0] * 2 (xhat - x) / n. */
int cv_mse_sum(const float* xhat, const float* x, int n, int per_sample, float* rec_out,
               const float* gscale, float* dxhat, double* work, cv_stream_t stream);

/* SNN / NT-Xent contrastive loss (losses.py:98-137) for up to 2 branches sharing labels
 * (content: pairs with equal labels; style with ps=1: pairs with different labels,
 * trainer.py:456-472).  phase 0: row log-sum-exps into lse; phase 1: loss (mean over finite rows,
 * losses.py:125-126) and, when dmu != NULL, the gradient gmul*gscale[0]*dloss/d(mu, logvar);
 * phase 2: both. */
typedef struct cv_ntxent_branch {
  const float* mu; const float* logvar; int ld;   /* [n] rows of stride ld               */
  int ps;
  float* dmu; float* dlogvar; int gld;            /* gradient outputs (may be NULL)       */
  const float* gscale; float gmul;                /* upstream gradient                    */
  float* loss_out;                                /* [1]                                  */
  float* lse;                                     /* workspace [2n]                       */
} cv_ntxent_branch;
int cv_ntxent(const cv_ntxent_branch* br, int nbr, const int64_t* label, int n, int d, int sim,
              float temperature, int phase, int accumulate, cv_stream_t stream);
/* An NT-Xent phase of cv_ntxent (phase 0: the row log-sum-exps; 1: the losses and gradients, accumulated into the
 * branches' d(mu) / d(logvar) when accumulate) queued to run as extra workgroups of this thread's next direct-kernel
 * conv launch on the SAME `stream` (cv_aux.hip: MNIST's decoder ConvTranspose2d forwards serve it; a launch on another
 * stream leaves it queued); the call after that conv must be cv_ntxent_aux_flush, which launches the phase on its own,
 * on the stream it was queued for, if no launch took it.  One phase at a time (a phase still queued when the next is
 * queued is launched first, on its own stream); the phases read only the heads and labels (trainer.py:474-479,
 * losses.py:98-137), so the fused step queues them into its decoder forward.  The branch gradients must not be read
 * before the flush.  cv_ntxent_aux_discard drops a queued phase without launching it (returns 1 if one was queued):
 * the engine calls it when a program raises between the queue and its flush.  cv_ntxent_aux_pending: 0, or 1 + the
 * queued phase (test hook). */
int cv_ntxent_aux(const cv_ntxent_branch* br, int nbr, const int64_t* label, int n, int d, int sim, float temperature,
                  int phase, int accumulate, cv_stream_t stream);
int cv_ntxent_aux_flush(cv_stream_t stream);
int cv_ntxent_aux_discard(void);
int cv_ntxent_aux_pending(void);
/* Attach the KL part of the latent combine (cv_latent_combine with dz = NULL and rec_in = NULL: losses[1], [2], [7]
 * and dheads = the KL gradient, overwritten — dheads must not hold anything yet) to the queued phase-0 request, as
 * one more workgroup of the same grid (or of the flush launch).  The decoder chain term follows in
 * cv_heads_backward_chain.  Requires a queued phase 0 (else an error). */
int cv_ntxent_aux_combine(const float* heads, const float* z, int n, int d, float beta, float loc, float scale,
                          const int64_t* anneal_step, float* dheads, float* losses, cv_stream_t stream);

/* The fused step's latent terms in two launches (trainer.py:452-480): cv_latent_combine (KL with the
 * annealer weight, the decoder gradient chained through z) and cv_ntxent phase 2 with accumulate = 1
 * on the same dheads.  The combine runs as an extra workgroup of the row-log-sum-exp launch (it does
 * not depend on it); every branch's dmu / dlogvar must point into dheads. */
int cv_latent_step(const float* heads, const float* z, const float* dz, int n, int d, float beta,
                   float loc, float scale, const int64_t* anneal_step, const double* rec_in,
                   float* dheads, float* losses, const cv_ntxent_branch* br, int nbr,
                   const int64_t* label, int sim, float temperature, cv_stream_t stream);

/* ---- MI upper bounds (mi_estimator.py:108-198) ---- */
enum { CV_MI_NONE = 0, CV_MI_CLUBSAMPLE = 1, CV_MI_L1OUT = 2 };

/* q(y|x) MLPs (mi_estimator.py:111-122): p_mu = L(dx,h)-ReLU-L(h,dy);
 * p_logvar = L(dx,h)-ReLU-L(h,dy)-Tanh; Linear weights [out][in]; h = hidden_size // 2. */
typedef struct cv_mlp {
  const float *w1, *b1, *w2, *b2;   /* p_mu     */
  const float *w3, *b3, *w4, *b4;   /* p_logvar */
  int dx, h, dy;
} cv_mlp;
typedef struct cv_mlp_grad {
  float *w1, *b1, *w2, *b2, *w3, *b3, *w4, *b4;
} cv_mlp_grad;

size_t cv_mi_workspace_bytes(int n);
/* CLUBSample.forward (mi_estimator.py:133-143; perm injected, or generated on device from
 * (seed, offset)) and L1OutUB.forward (mi_estimator.py:170-191, with the reference's [N,N,N]
 * broadcasting reduced to its O(N d) closed form).  Writes mi_out[0]; leaves perm / column sums
 * in `work` for cv_mi_backward. */
int cv_mi_forward(int kind, const cv_mlp* mlp, const float* x, int ldx, const float* y, int ldy,
                  int n, const int64_t* perm, uint64_t seed, uint64_t* offset, void* work,
                  float* mi_out, cv_stream_t stream);
/* gradient of gmul*gscale[0]*mi w.r.t. x and y (written or accumulated) and, when g != NULL, the MLP
 * parameters (accumulated).  Chain mode (dheads != NULL): x = z_c, y = z_s are the two halves of z
 * and the gradient is accumulated into d(heads) through z = mu + eps*exp(lv/2). */
int cv_mi_backward(int kind, const cv_mlp* mlp, const float* x, int ldx, const float* y, int ldy,
                   int n, void* work, const float* gscale, float gmul, float* dx, float* dy,
                   int gld, int accumulate, const cv_mlp_grad* g, const float* heads,
                   const float* z, float* dheads, int d, cv_stream_t stream);
/* learning_loss = -loglikeli (mi_estimator.py:129-131, 193-198): loss and MLP gradients
 * (overwritten); with params != NULL also the Adam update of the estimator arena
 * (trainer.py:885-887), whose grads arena must then hold g's buffers.  `work`: a
 * cv_mi_workspace_bytes(n) buffer, zeroed once at allocation (its arrival counters reset
 * themselves). */
int cv_mi_learning_step(const cv_mlp* mlp, const float* x, int ldx, const float* y, int ldy, int n,
                        void* work, float* loss_out, const cv_mlp_grad* g, float* params,
                        const float* grads,
                        float* exp_avg, float* exp_avg_sq, int64_t numel, const float* hyper,
                        int64_t* step, cv_stream_t stream);

/* ---- CLEAR-TC factor discriminator (trainer.py:573-699, trainer_utils.py:133-138) ----
 * factor_cls = Linear(z, z) -> ReLU -> Linear(z, 1) -> Sigmoid, Linear weights [out][in]; z <= 64, even. */
typedef struct cv_tc_disc {
  const float *w1, *b1, *w2, *b2;
  int zdim;
} cv_tc_disc;
typedef struct cv_tc_grad {
  float *w1, *b1, *w2, *b2;
} cv_tc_grad;
size_t cv_tc_workspace_bytes(int zdim);
/* mi_out[0] = relu(log(d / (1 - d))).mean(), d = factor_cls(z) (trainer.py:664-665), z [n][zdim].  With
 * dheads != NULL also accumulates the gradient of lam * mi_loss into d(heads) through
 * z = mu + eps*exp(logvar/2) (heads / dheads [n][4d] = mu_c | lv_c | mu_s | lv_s, d = zdim/2). */
int cv_tc_forward(const cv_tc_disc* D, const float* z, int n, float lam, const float* heads, float* dheads, int d,
                  void* work, float* mi_out, cv_stream_t stream);
/* The discriminator's step loss (trainer.py:683-694): BCE of factor_cls on z (target 1) and on
 * factor_shuffling(z) "permute_1" (target 0); loss_out[0] and the parameter gradients (overwritten).
 * The optimizer update is cv_adam_step on the discriminator's arena. */
int cv_tc_learning_step(const cv_tc_disc* D, const float* z, int n, void* work, float* loss_out,
                        const cv_tc_grad* g, cv_stream_t stream);

/* ---- GVAE / ML-VAE group evidence (vae.py:159-223; HierarchicalVAETrainer, trainer.py:291-353) ----
 * Segmented by label on the device (n <= 4096, d <= 64): groups in sorted-label order, members in
 * ascending index (the reference's order).  `work`: cv_group_workspace_bytes(n, d) bytes holding
 * int32 m at byte 0, then int32 gid[n], pos[n], order[n], start[n+1] at byte 64 onwards and the group rows
 * mu_g | lv_g [n][2d] fp32 (first m valid) at the next 16-byte boundary. */
enum { CV_GROUP_MLVAE = 0, CV_GROUP_GVAE = 1 };
size_t cv_group_workspace_bytes(int n, int d);
/* accumulate_group_evidence (vae.py:159-190) into `work`; scale_out (or NULL) = n/m, the
 * _group_adjust factor B/m (trainer.py:322-324).  With z != NULL also groupwise_reparam_each + sample
 * (vae.py:193-223, 56-60): z [n][2d] = mu_g[gid] + eps_c * exp(lv_g/2) | mu_s + eps_s * exp(lv_s/2), where
 * row r of the c-noise belongs to the sample at group-order position r (the reference's per-group
 * torch.randn order).  eps [n][ld_eps] injected (c columns [0,d) in group order, s columns [d,2d) per
 * sample) or NULL: Philox from (seed, offset[0]), offset[0] += 1. */
int cv_group_forward(int mode, const float* mu_c, const float* lv_c, int ld, const int64_t* label, int n, int d,
                     void* work, float* scale_out, const float* mu_s, const float* lv_s, int lds,
                     const float* eps, int ld_eps, uint64_t seed, uint64_t* offset, float* z, cv_stream_t stream);
/* The fused step's latent terms (trainer.py:342-349): kl_c over the m group rows, rec and kl_s times
 * B/m, the annealer weight beta/(1+exp(-(t-loc)/scale)) at t = anneal_step[0], and d(heads) [n][4d]
 * (written) from dz [n][2d] through the reparameterisation and the evidence.  losses[0..2] = rec
 * (sum of the CV_REC_REPL rec_in replicas, times B/m), kl_c, kl_s (times B/m); losses[7] = weight. */
int cv_group_backward(int mode, const float* heads, const float* z, const float* dz, const void* work, int n,
                      int d, float beta, float loc, float scale, const int64_t* anneal_step,
                      const double* rec_in, float* dheads, float* losses, cv_stream_t stream);
/* accumulate_group_evidence backward (module path): d(mu_c), d(lv_c) [n][ldo] (written) from d(mu_g),
 * d(lv_g) [m][d] (either may be NULL = zero) and the `work` of the matching cv_group_forward. */
int cv_group_evidence_backward(int mode, const float* mu_c, const float* lv_c, int ld, const void* work, int n,
                               int d, const float* dmu_g, const float* dlv_g, float* dmu_c, float* dlv_c, int ldo,
                               cv_stream_t stream);

/* ---- input pipeline (run_pacs_downstream_expr.py:88-98, run_camelyon17_downstream_expr.ipynb cell 6,
 * data_utils.py:55-73): transforms.Resize((h, w)) + ToTensor() of uint8 images, on the device ----
 * Resize of a PIL image is Image.resize(size, BILINEAR): Pillow's separable antialiased triangle filter
 * with 22-bit fixed-point coefficients and an 8-bit intermediate (src/libImaging/Resample.c).  The plan
 * (int32 words: header, then per output column / row the (first source index, taps) bounds and the
 * fixed-point coefficients) is built on the host with Pillow's double-precision recipe; copy it to the
 * device once. */
size_t cv_resize_plan_words(int in_h, int in_w, int out_h, int out_w);
int cv_resize_plan(int in_h, int in_w, int out_h, int out_w, int32_t* plan, size_t words);
/* source rows of the horizontal pass that a tile of `ty` output rows needs (host plan) */
int cv_resize_tile_rows(const int32_t* plan, int ty);
/* One batch: out [n][c][out_h][out_w] fp32 = Resize + ToTensor of images[index[i]] (uint8 [count][in_h][in_w][c],
 * HWC; index NULL = images 0..n-1), identical to Pillow + torchvision bit for bit; labels_out[i] =
 * labels[index[i]] and styles_out likewise when given.  ty output rows per workgroup, tile_rows =
 * cv_resize_tile_rows(plan, ty); stage = 1 copies each tile's source rows into LDS first (coalesced).
 * LDS per workgroup: the plan body + tile_rows * (out_w + stage * in_w) * c bytes, at most 64 KiB. */
int cv_load_batch_u8(const uint8_t* images, int in_h, int in_w, int c, const int64_t* index, int n,
                     const int32_t* plan, int out_h, int out_w, int ty, int tile_rows, int stage, float* out,
                     const int64_t* labels, int64_t* labels_out, const int64_t* styles, int64_t* styles_out,
                     cv_stream_t stream);

/* ---- Adam (torch.optim.Adam foreach semantics) over a flat fp32 arena ----
 * hyper: device float[8] = lr, beta1, beta2, eps, weight_decay; step: device int64[2] =
 * (steps taken, arrival counter = 0).  grad_scale (device float or NULL) multiplies the gradient
 * first (data-parallel averaging); aux_counter (or NULL) is incremented once per call
 * (LogisticAnnealer.step, trainer.py:484). */
int cv_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                 int64_t numel, const float* hyper, int64_t* step, const float* grad_scale,
                 int64_t* aux_counter, cv_stream_t stream);

/* End-of-backward reduction in ONE launch (the step before the optimizer, trainer.py:482-483):
 * the partial tiles of up to 24 deferred weight gradients (fixed split order: deterministic), the
 * BatchNorm affine gradients dgamma = sum dz*xhat, dbeta = sum dz of up to 16 layers (when dgamma or
 * dbeta is given; written, not accumulated) and, with running = 1, their running statistics
 * (nn.BatchNorm*, momentum, unbiased running var; num_batches_tracked += 1 when nbt is given). */
int cv_step_reduce(const cv_wgrad_defer* defers, int ndefer, const cv_bn* bn, int nbn, float* const* dgamma,
                   float* const* dbeta, int running, float momentum, int64_t* const* nbt, cv_stream_t stream);

/* cv_step_reduce + cv_adam_step (no grad_scale) in the same launch, for a single-process step: every
 * gradient the reduction finalises (deferred weights / biases, dgamma, dbeta — all inside the gradient arena
 * grads[0, numel)) is stepped as soon as it is produced, the rest of the arena (its gradients already final) by
 * trailing blocks; the last block advances step[0] and aux_counter.  step: device int64[66] = (steps taken, then
 * 65 zeroed arrival words, which reset themselves).  The reduced ranges must not overlap and, with the gaps
 * between them, form at most 32 plain ranges. */
int cv_step_reduce_adam(const cv_wgrad_defer* defers, int ndefer, const cv_bn* bn, int nbn, float* const* dgamma,
                        float* const* dbeta, int running, float momentum, int64_t* const* nbt, float* params,
                        float* grads, float* exp_avg, float* exp_avg_sq, int64_t numel, const float* hyper,
                        int64_t* step, int64_t* aux_counter, cv_stream_t stream);

/* BatchNorm affine gradients from the backward sums: dgamma = sum dz*xhat, dbeta = sum dz
 * (nn.BatchNorm weight/bias grads); written (not accumulated) for up to 16 layers. */
int cv_bn_param_grads(const cv_bn* bn, int nlayers, float* const* dgamma, float* const* dbeta,
                      cv_stream_t stream);

/* ---- misc ---- */
/* hipMemsetAsync(ptr, 0, bytes, stream) (graph-capturable) */
int cv_zero(void* ptr, size_t bytes, cv_stream_t stream);
/* zero up to 8 buffers (4-byte granular: sizes multiples of 4, 4-byte aligned) in one launch */
int cv_zero_many(void* const* ptrs, const size_t* bytes, int count, cv_stream_t stream);
/* device-to-device copy of up to 8 buffers (4-byte granular) in one launch (the step's input batch) */
int cv_copy_many(void* const* dst, const void* const* src, const size_t* bytes, int count, cv_stream_t stream);
/* Step graphs: capture the calls enqueued on `stream` between cv_graph_begin and cv_graph_end (thread-local
 * capture mode; the stream must not be the legacy default stream) into an executable graph, replay it with
 * cv_graph_launch on any stream, free it with cv_graph_destroy. */
int cv_graph_begin(cv_stream_t stream);
int cv_graph_end(cv_stream_t stream, void** exec_out);
int cv_graph_launch(void* exec, cv_stream_t stream);
int cv_graph_destroy(void* exec);
const char* cv_last_error(void);
int cv_version(void);
/* test hook: 1 routes every conv/linear GEMM to the generic implicit-GEMM kernel instead of the
 * specialised core (both compute the same contraction); returns the previous setting */
int cv_debug_force_generic_gemm(int on);
/* test hook: launches of the direct conv kernel (cv_conv_*_kpack) since the last reset */
int cv_debug_direct_count(int reset);
/* test hook: the fewest workgroups for which a stride-2 conv takes the direct kernel (default 256; smaller
 * grids run the GEMM core); returns the previous setting (-1: not yet initialised) */
int cv_debug_direct_minwg(int minwg);
/* test hook: 1 (default) serves a stride-2 GATHER by the direct kernel only where it measured faster than the GEMM
 * core (one resident round of workgroups, >= 32 output pixels per tile); 0 serves every geometry it can plan
 * (kernel tests); returns the previous setting */
int cv_debug_direct_gather_rule(int on);
/* test hook: 1 (default) issues a served backward-data + weight-gradient pair as one dual grid (cv_dual.hip), 0 runs
 * the two launches back to back (the arithmetic of each role is the same); a negative value only queries; returns
 * the previous setting */
int cv_debug_dual(int on);
/* test hook: 1 (default) lets the GEMM core take pixel-major tiles where they skip >= 10 % padding work
 * (cv_gemm_tile.inc), 0 never; a negative value only queries; returns the previous setting (-1: not yet read
 * from CV_PM) */
int cv_debug_pm(int on);
/* test hook: conv contractions planned with pixel-major tiles since the last reset */
int cv_debug_pm_count(int reset);
/* test hook: 1 (default) lets a queued NT-Xent phase ride in a served direct launch (cv_ntxent_aux), 0 launches it
 * on its own at the flush; a negative value only queries; returns the previous setting */
/* test hook: 1 (CV_WGRAD_SELF=1; measured slower, off by default) lets a deferred split-K weight gradient reduce its
 * own slices (the split's last slice adds the tile into gweight; the defer record says split 0), 0 (default) leaves
 * the partials for cv_step_reduce;
 * -1 queries; returns the previous setting (-1: not yet read from the environment) */
int cv_debug_wgrad_self(int on);
int cv_debug_aux(int on);
/* test hook: direct + NT-Xent grids issued since the last reset */
int cv_debug_aux_count(int reset);
/* Test hook: the register-resident NT-Xent variants (cosine, n <= 512, d <= 8; cv_ntxent.hpp) on (1) / off (0:
 * the LDS-staged kernels), -1 queries; returns the previous setting.  Diagnostics only. */
int cv_debug_nt_reg(int on);
/* test hook: dual grids issued since the last reset */
int cv_debug_dual_count(int reset);
/* measurement hook: 1 starts recording (on this thread) the kernels the conv / linear calls launch, clearing the
 * record; 0 stops; returns the previous setting.  cv_debug_kernel_names writes the recorded kernels' demangled
 * names, one per line, into buf (truncated to cap - 1 bytes, NUL-terminated) and returns how many were recorded
 * (bench.py: the PMC passes a roofline quotes must have been taken on the kernels the priced call issues). */
int cv_debug_kernel_log(int on);
int cv_debug_kernel_names(char* buf, size_t cap);

/* ---- GEMM workspace (in-launch split-K of under-filled long-K conv forward / ConvT backward-data
 * launches, e.g. VAE64's conv5 at 32-256 images per GPU): a caller-owned device buffer of at least
 * cv_gemm_workspace_bytes(), ZEROED before registration, for the current device (NULL: unregister).
 * Calls on one stream share it; without one the launches run unsplit.  CONTRACT: the split launches of a
 * device must be serialised — one stream at a time (the fused step engine issues them all on its step
 * stream; the autograd path on torch's current stream).  Two split launches in flight on different streams
 * would race on its fragment slabs and leave its self-resetting per-tile tickets non-zero, corrupting every
 * later split launch; a caller that runs conv layers on several streams concurrently registers NULL (no
 * split) or serialises them with events.  No reference counterpart
 * (the reference's convolutions are ATen's, code/src/models/vae.py:15-46 / :113-156). */
size_t cv_gemm_workspace_bytes(void);
int cv_set_gemm_workspace(void* work, size_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* CLEARVAE_H */
