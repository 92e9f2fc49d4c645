/* Host-side validation paths of the C-ABI (include/clearvae.h) under AddressSanitizer, without a GPU.
 *
 * Built by `make -C clear-vae_amd/csrc asan` against a host-only, ASan-instrumented build of the library
 * (hipcc --offload-host-only -fsanitize=address: the kernels are stubs, every host line is instrumented), and
 * run by tests/test_abi.py::test_host_validation_under_asan.  Every call below must be answered on the host:
 * a malformed geometry, a null or undersized buffer, an unsupported mode or batch is rejected with a non-zero
 * status and a cv_last_error() message before anything is enqueued, and the host-side builders (workspace
 * sizes, the Pillow resize plan) write exactly inside the buffers they are given.  Any out-of-bounds host
 * access in those paths is an ASan report and a non-zero exit. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "clearvae.h"

static int failures = 0;

#define EXPECT_ERR(call, what)                                                                  \
  do {                                                                                          \
    int rc_ = (call);                                                                           \
    const char* e_ = cv_last_error();                                                           \
    if (rc_ == 0 || !e_ || !e_[0]) {                                                            \
      fprintf(stderr, "FAIL %s: rc=%d err='%s'\n", what, rc_, e_ ? e_ : "(null)");             \
      ++failures;                                                                               \
    } else {                                                                                    \
      printf("ok   %-44s -> %s\n", what, e_);                                                   \
    }                                                                                           \
  } while (0)

#define EXPECT(cond, what)                                    \
  do {                                                        \
    if (!(cond)) {                                            \
      fprintf(stderr, "FAIL %s\n", what);                     \
      ++failures;                                             \
    } else {                                                  \
      printf("ok   %s\n", what);                              \
    }                                                         \
  } while (0)

int main(void) {
  EXPECT(cv_version() >= 1, "cv_version");
  /* a fake, never dereferenced device pointer: the calls below must fail before any launch */
  float* dp = (float*)(uintptr_t)0x1000;
  cv_stream_t st = NULL;

  /* ---- convolutions: geometry checks (MNIST conv2 with a wrong output size, bad stride / mma) */
  cv_conv bad = {8, 32, 14, 14, 64, 9, 9, 3, 3, 2, 1, 0, CV_MMA_FP32};
  cv_operand op;
  memset(&op, 0, sizeof(op));
  op.x = dp;
  EXPECT_ERR(cv_conv_forward(&bad, &op, dp, NULL, dp, NULL, st), "conv_forward: wrong output size");
  EXPECT_ERR(cv_conv_backward_data(&bad, &op, dp, dp, NULL, st), "conv_backward_data: wrong output size");
  cv_conv g = {8, 32, 14, 14, 64, 7, 7, 3, 3, 2, 1, 0, 7};
  EXPECT_ERR(cv_conv_forward(&g, &op, dp, NULL, dp, NULL, st), "conv_forward: bad mma precision");
  g.mma = CV_MMA_FP32;
  g.stride = 0;
  EXPECT_ERR(cv_conv_forward(&g, &op, dp, NULL, dp, NULL, st), "conv_forward: zero stride");
  g.stride = 2;
  EXPECT_ERR(cv_conv_forward(NULL, &op, dp, NULL, dp, NULL, st), "conv_forward: null geometry");
  EXPECT_ERR(cv_conv_forward(&g, NULL, dp, NULL, dp, NULL, st), "conv_forward: null operand");
  cv_operand bnop = op;
  bnop.xf = CV_XF_BNBWD; /* BN backward transform without y */
  bnop.bn.C = 32;
  EXPECT_ERR(cv_conv_forward(&g, &bnop, dp, NULL, dp, NULL, st), "conv_forward: BNBWD operand without y");
  bnop.xf = CV_XF_BNRELU;
  bnop.bn.C = 16; /* BN width != channels */
  EXPECT_ERR(cv_conv_forward(&g, &bnop, dp, NULL, dp, NULL, st), "conv_forward: BN width mismatch");
  size_t wb = cv_conv_wgrad_workspace_bytes(&g, 0);
  EXPECT(wb > 0 && wb % 4 == 0, "conv_wgrad_workspace_bytes");
  cv_wgrad_defer d;
  memset(&d, 0, sizeof(d));
  EXPECT_ERR(cv_conv_backward_weight_deferred(&g, &op, &op, dp, NULL, NULL, 0, &d, st),
             "conv_backward_weight_deferred: no workspace");
  EXPECT_ERR(cv_conv_backward_weight_deferred(&g, &op, &op, dp, NULL, dp, wb / 2, &d, st),
             "conv_backward_weight_deferred: workspace too small");

  /* ---- linear layers */
  cv_linear lin = {64, 2048, 128, 1, 0, 1, 0, 9};
  EXPECT_ERR(cv_linear_forward(&lin, &op, dp, NULL, dp, 0, NULL, st), "linear_forward: bad mma precision");
  lin.mma = CV_MMA_FP32;
  lin.in_pix = 3; /* in_features != in_pix * in_ch */
  lin.in_ch = 5;
  EXPECT_ERR(cv_linear_forward(&lin, &op, dp, NULL, dp, 0, NULL, st), "linear_forward: flatten mismatch");
  EXPECT(cv_decoder_input_supported(64, 8, 2048) == 1, "decoder_input_supported (MNIST)");
  EXPECT(cv_decoder_input_supported(64, 8, 2047) == 0, "decoder_input_supported (F % 16)");

  /* ---- latent terms */
  cv_ntxent_branch br;
  memset(&br, 0, sizeof(br));
  br.mu = dp;
  br.logvar = dp;
  br.ld = 32;
  br.loss_out = dp;
  br.lse = dp;
  int64_t* lp = (int64_t*)dp;
  EXPECT_ERR(cv_ntxent(&br, 1, lp, 64, 8, 99, 0.1f, 2, 0, st), "ntxent: unknown similarity");
  EXPECT_ERR(cv_ntxent(&br, 3, lp, 64, 8, 0, 0.1f, 2, 0, st), "ntxent: three branches");
  EXPECT_ERR(cv_ntxent(&br, 1, lp, 64, 65, 0, 0.1f, 2, 0, st), "ntxent: latent width 65 > 64");
  EXPECT(cv_mi_workspace_bytes(512) > 0, "mi_workspace_bytes");
  cv_mlp mlp;
  memset(&mlp, 0, sizeof(mlp));
  mlp.dx = mlp.dy = 8;
  mlp.h = 8;
  EXPECT_ERR(cv_mi_forward(7, &mlp, dp, 16, dp, 16, 64, NULL, 0, NULL, dp, dp, st), "mi_forward: unknown estimator");
  EXPECT(cv_group_workspace_bytes(64, 8) > 0, "group_workspace_bytes");
  EXPECT_ERR(cv_group_forward(5, dp, dp, 32, lp, 64, 8, dp, NULL, NULL, NULL, 0, NULL, 0, 0, NULL, NULL, st),
             "group_forward: unknown mode");
  EXPECT(cv_tc_workspace_bytes(16) > 0, "tc_workspace_bytes");

  /* ---- input pipeline: the host-built Pillow plan, exactly sized and undersized */
  const int sizes[][4] = {{96, 96, 64, 64}, {224, 224, 64, 64}, {227, 227, 64, 64}, {28, 28, 28, 28},
                          {17, 33, 64, 48}, {64, 64, 96, 96}};
  for (unsigned i = 0; i < sizeof(sizes) / sizeof(sizes[0]); ++i) {
    const int* s = sizes[i];
    size_t words = cv_resize_plan_words(s[0], s[1], s[2], s[3]);
    int32_t* plan = (int32_t*)malloc(words * sizeof(int32_t));
    char what[96];
    snprintf(what, sizeof(what), "resize_plan %dx%d -> %dx%d (%zu words)", s[0], s[1], s[2], s[3], words);
    EXPECT(words > 0 && plan && cv_resize_plan(s[0], s[1], s[2], s[3], plan, words) == 0, what);
    EXPECT(cv_resize_tile_rows(plan, 8) > 0, "resize_tile_rows");
    snprintf(what, sizeof(what), "resize_plan %dx%d: buffer one word short", s[0], s[1]);
    EXPECT_ERR(cv_resize_plan(s[0], s[1], s[2], s[3], plan, words - 1), what);
    free(plan);
  }
  EXPECT_ERR(cv_resize_plan(0, 96, 64, 64, NULL, 0), "resize_plan: empty image");

  /* ---- misc: bounded batched helpers, workspace registration */
  void* ptrs[9] = {dp, dp, dp, dp, dp, dp, dp, dp, dp};
  size_t nb[9] = {4, 4, 4, 4, 4, 4, 4, 4, 4};
  EXPECT_ERR(cv_zero_many(ptrs, nb, 9, st), "zero_many: more than 8 buffers");
  EXPECT_ERR(cv_copy_many(ptrs, (const void* const*)ptrs, nb, 9, st), "copy_many: more than 8 buffers");
  nb[0] = 6;
  EXPECT_ERR(cv_zero_many(ptrs, nb, 1, st), "zero_many: size not a multiple of 4");
  EXPECT(cv_gemm_workspace_bytes() > 4096, "gemm_workspace_bytes");
  EXPECT_ERR(cv_set_gemm_workspace(dp, 64), "set_gemm_workspace: too small");
  cv_wgrad_defer many[25];
  memset(many, 0, sizeof(many));
  EXPECT_ERR(cv_step_reduce(many, 25, NULL, 0, NULL, NULL, 0, 0.1f, NULL, st), "step_reduce: 25 deferred gradients");
  EXPECT_ERR(cv_adam_step(NULL, dp, dp, dp, 16, dp, lp, NULL, NULL, st), "adam_step: null params");

  /* a long error message (the last-error buffer must truncate, not overflow) */
  cv_conv huge = {1 << 30, 1 << 20, 1 << 12, 1 << 12, 1 << 20, 1 << 12, 1 << 12, 3, 3, 2, 1, 0, 0};
  EXPECT_ERR(cv_conv_forward(&huge, &op, dp, NULL, dp, NULL, st), "conv_forward: absurd sizes");

  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("all host validation checks passed\n");
  return 0;
}
