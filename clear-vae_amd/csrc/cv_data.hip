// Input pipeline on gfx950: the producer side of the training step.
//
// The reference feeds the model from torchvision transforms on the host: Resize((64, 64)) + ToTensor()
// on PIL images (code/run_pacs_downstream_expr.py:88-98, code/run_camelyon17_downstream_expr.ipynb cell 6;
// ToTensor alone for Styled-MNIST, code/src/utils/data_utils.py:55-73).  For PIL images Resize is
// Image.resize(size, BILINEAR), i.e. Pillow's two-pass separable resampling (src/libImaging/Resample.c,
// Pillow 12.2.0 here): a triangle filter widened by the downscale factor (antialiasing), coefficients
// normalised per output pixel and quantised to 22-bit fixed point, the horizontal pass rounded to 8
// bits before the vertical one.  ToTensor is u8 / 255 in fp32.
//
// Here the dataset lives in HBM as uint8 HWC images; one launch per batch gathers the sampled images
// (index array), runs both resampling passes with Pillow's integer arithmetic (the horizontal pass of
// the rows a tile of output rows needs staged in LDS), converts to fp32 NCHW / 255 straight into the
// step's input buffer, and gathers the labels / style labels.  Bit-exact with Pillow (oracle/resize_ref.py,
// tests/golden/resize_pil.npz).  The coefficient plan is built on the host with Pillow's double-precision
// recipe (cv_resize_plan) and copied to the device once per (input size, output size).
#include "cv_common.hpp"

#include <math.h>

namespace cv {

constexpr int RS_PREC = 22;  // Pillow PRECISION_BITS = 32 - 8 - 2
constexpr int RS_HDR = 16;   // plan header words

__device__ __forceinline__ int clip8(int ss) {
  const int v = ss >> RS_PREC;  // arithmetic shift, as Pillow's clip8 lookup index
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

struct LoadArgs {
  const uint8_t* images;
  int in_h, in_w, c;
  const int64_t* index;
  int n;
  const int32_t* plan;
  int out_h, out_w, ty;
  int stage;  // 1: the tile's source rows are first copied into LDS with coalesced loads
  float* out;
  const int64_t* labels;
  int64_t* labels_out;
  const int64_t* styles;
  int64_t* styles_out;
};

// KM > 0: both passes have at most KM taps (unrolled, coefficients in registers); KM = 0: any tap count
template <int KM>
__global__ __launch_bounds__(256) void load_batch_kernel(const LoadArgs A) {
  // LDS: [plan body][staged source rows (stage = 1)][horizontal-pass rows: rows][out_w][c], 16-byte aligned parts
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int img = blockIdx.y, tile = blockIdx.x;
  const int c = A.c, ow = A.out_w, oh = A.out_h;
  const int kh = A.plan[0], kv = A.plan[1], ybf = A.plan[2];
  const int pw = ow * (2 + kh) + oh * (2 + kv);  // bounds + coefficients: every tap loop reads them
  int32_t* P = reinterpret_cast<int32_t*>(lds);
  for (int i = threadIdx.x; i < pw; i += 256) P[i] = A.plan[RS_HDR + i];
  const int32_t* bh = P;
  const int32_t* kkh = bh + 2 * ow;
  const int32_t* bv = kkh + ow * kh;
  const int32_t* kkv = bv + 2 * oh;
  uint8_t* const base = lds + ((4 * pw + 15) & ~15);
  __syncthreads();
  const int yy0 = tile * A.ty, yy1 = min(oh, yy0 + A.ty);
  const int r0 = bv[2 * yy0], r1 = bv[2 * (yy1 - 1)] + bv[2 * (yy1 - 1) + 1];
  const int64_t src_i = A.index ? A.index[img] : img;
  const uint8_t* src = A.images + (size_t)src_i * A.in_h * A.in_w * c;
  const int rowb = A.in_w * c;
  const uint8_t* blk = src + (size_t)(ybf + r0) * rowb;  // the tile's source rows: one contiguous block
  const int nb = (r1 - r0) * rowb;
  uint8_t* tmp = base;
  if (A.stage) {
    tmp = base + ((nb + 15) & ~15);
    if (((uintptr_t)blk & 15) == 0) {  // 16-byte loads, then the byte tail
      const int n16 = nb >> 4;
      for (int i = threadIdx.x; i < n16; i += 256)
        reinterpret_cast<uint4*>(base)[i] = reinterpret_cast<const uint4*>(blk)[i];
      for (int i = (n16 << 4) + threadIdx.x; i < nb; i += 256) base[i] = blk[i];
    } else {
      for (int i = threadIdx.x; i < nb; i += 256) base[i] = blk[i];
    }
    __syncthreads();
    blk = base;
  }
  // horizontal pass (rows ybf + r0 .. ybf + r1 of the source): lane -> output column, the column's bounds and
  // coefficients held in registers across the tile's rows and channels (no per-element index division)
  const int lane = threadIdx.x & 63, sub = threadIdx.x >> 6;
  const int rows = r1 - r0;
  for (int xx = lane; xx < ow; xx += 64) {
    const int xmin = bh[2 * xx], xmax = bh[2 * xx + 1];
    int k[KM > 0 ? KM : 1];
    if (KM > 0) {
#pragma unroll
      for (int x = 0; x < (KM > 0 ? KM : 1); ++x) k[x] = x < xmax ? kkh[xx * kh + x] : 0;
    }
    for (int r = sub; r < rows; r += 4) {
      const uint8_t* row = blk + (size_t)r * rowb + xmin * c;
      for (int ch = 0; ch < c; ++ch) {
        int ss = 1 << (RS_PREC - 1);
        if (KM > 0) {
#pragma unroll
          for (int x = 0; x < (KM > 0 ? KM : 1); ++x)
            if (x < xmax) ss += (int)row[x * c + ch] * k[x];
        } else {
          for (int x = 0; x < xmax; ++x) ss += (int)row[x * c + ch] * kkh[xx * kh + x];
        }
        tmp[(r * ow + xx) * c + ch] = (uint8_t)clip8(ss);
      }
    }
  }
  __syncthreads();
  // vertical pass + ToTensor into NCHW fp32 (lane -> output column: coalesced stores)
  for (int xx = lane; xx < ow; xx += 64) {
    for (int yy = yy0 + sub; yy < yy1; yy += 4) {
      const int ymin = bv[2 * yy] - r0, ymax = bv[2 * yy + 1];
      const int32_t* kp = kkv + yy * kv;
      for (int ch = 0; ch < c; ++ch) {
        const uint8_t* col = tmp + (ymin * ow + xx) * c + ch;
        int ss = 1 << (RS_PREC - 1);
        if (KM > 0) {
#pragma unroll
          for (int y = 0; y < (KM > 0 ? KM : 1); ++y)
            if (y < ymax) ss += (int)col[y * ow * c] * kp[y];
        } else {
          for (int y = 0; y < ymax; ++y) ss += (int)col[y * ow * c] * kp[y];
        }
        A.out[(((size_t)img * c + ch) * oh + yy) * ow + xx] = __fdiv_rn((float)clip8(ss), 255.0f);
      }
    }
  }
  if (tile == 0 && threadIdx.x == 0) {
    if (A.labels_out) A.labels_out[img] = A.labels[src_i];
    if (A.styles_out) A.styles_out[img] = A.styles[src_i];
  }
}

// ---- host: Pillow's coefficient recipe (Resample.c precompute_coeffs + normalize_coeffs_8bpc) ----
#pragma clang fp contract(off)
static inline double bilinear_filter(double x) {
  if (x < 0.0) x = -x;
  if (x < 1.0) return 1.0 - x;
  return 0.0;
}

static int coeff_ksize(int in_size, int out_size) {
  const double scale = (double)in_size / (double)out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;
  return (int)ceil(support) * 2 + 1;
}

// bounds [out][2] = (first input index, taps), kk [out][ksize] fixed-point; returns ksize
static int precompute(int in_size, int out_size, int32_t* bounds, int32_t* kk) {
  const double in0 = 0.0, in1 = (double)in_size;
  const double scale = (in1 - in0) / (double)out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;
  const int ksize = (int)ceil(support) * 2 + 1;
  double k[4096];
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = in0 + (xx + 0.5) * scale;
    double ww = 0.0;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    int x = 0;
    for (; x < xmax; ++x) {
      const double w = bilinear_filter((x + xmin - center + 0.5) * ss);
      k[x] = w;
      ww += w;
    }
    for (x = 0; x < xmax; ++x)
      if (ww != 0.0) k[x] /= ww;
    for (; x < ksize; ++x) k[x] = 0;
    for (x = 0; x < ksize; ++x)
      kk[(size_t)xx * ksize + x] = k[x] < 0 ? (int32_t)(-0.5 + k[x] * (1 << RS_PREC))
                                            : (int32_t)(0.5 + k[x] * (1 << RS_PREC));
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
  }
  return ksize;
}
#pragma clang fp contract(on)

}  // namespace cv

using namespace cv;

extern "C" size_t cv_resize_plan_words(int in_h, int in_w, int out_h, int out_w) {
  if (in_h <= 0 || in_w <= 0 || out_h <= 0 || out_w <= 0) return 0;
  const int kh = coeff_ksize(in_w, out_w), kv = coeff_ksize(in_h, out_h);
  return RS_HDR + (size_t)out_w * (2 + kh) + (size_t)out_h * (2 + kv);
}

extern "C" int cv_resize_plan(int in_h, int in_w, int out_h, int out_w, int32_t* plan, size_t words) {
  clear_error();
  CV_REQUIRE(plan && in_h > 0 && in_w > 0 && out_h > 0 && out_w > 0 && out_h <= 4096 && out_w <= 4096,
             "resize_plan: bad sizes");
  const size_t need = cv_resize_plan_words(in_h, in_w, out_h, out_w);
  CV_REQUIRE(words >= need, "resize_plan: %zu words < %zu", words, need);
  const int kh = coeff_ksize(in_w, out_w), kv = coeff_ksize(in_h, out_h);
  CV_REQUIRE(kh <= 4096 && kv <= 4096, "resize_plan: downscale factor too large");
  memset(plan, 0, words * sizeof(int32_t));
  int32_t* bh = plan + RS_HDR;
  int32_t* kkh = bh + 2 * out_w;
  int32_t* bv = kkh + (size_t)out_w * kh;
  int32_t* kkv = bv + 2 * out_h;
  precompute(in_w, out_w, bh, kkh);
  precompute(in_h, out_h, bv, kkv);
  const int ybf = bv[0];
  for (int i = 0; i < out_h; ++i) bv[2 * i] -= ybf;  // rows relative to the first used source row
  plan[0] = kh;
  plan[1] = kv;
  plan[2] = ybf;
  plan[3] = bv[2 * (out_h - 1)] + bv[2 * (out_h - 1) + 1];  // source rows used
  plan[4] = out_w;
  plan[5] = out_h;
  plan[6] = in_w;
  plan[7] = in_h;
  return 0;
}

// rows of the horizontal pass a tile of `ty` output rows needs (host copy of the plan)
extern "C" int cv_resize_tile_rows(const int32_t* plan, int ty) {
  const int out_w = plan[4], out_h = plan[5], kh = plan[0];
  const int32_t* bv = plan + RS_HDR + (size_t)out_w * (2 + kh);
  int best = 0;
  for (int y0 = 0; y0 < out_h; y0 += ty) {
    const int y1 = y0 + ty < out_h ? y0 + ty : out_h;
    const int rows = bv[2 * (y1 - 1)] + bv[2 * (y1 - 1) + 1] - bv[2 * y0];
    if (rows > best) best = rows;
  }
  return best;
}

extern "C" int cv_load_batch_u8(const uint8_t* images, int in_h, int in_w, int c, const int64_t* index, int n,
                                const int32_t* plan, int out_h, int out_w, int ty, int tile_rows, int stage, float* out,
                                const int64_t* labels, int64_t* labels_out, const int64_t* styles,
                                int64_t* styles_out, cv_stream_t stream) {
  clear_error();
  CV_REQUIRE(images && plan && out && n > 0 && n <= 65535 && in_h > 0 && in_w > 0 && c >= 1 && c <= 4 &&
                 out_h > 0 && out_w > 0 && ty > 0 && tile_rows > 0,
             "load_batch_u8: bad args");
  CV_REQUIRE(!labels_out || labels, "load_batch_u8: labels_out needs labels");
  CV_REQUIRE(!styles_out || styles, "load_batch_u8: styles_out needs styles");
  const size_t pw = (size_t)out_w * (2 + coeff_ksize(in_w, out_w)) + (size_t)out_h * (2 + coeff_ksize(in_h, out_h));
  const size_t lds = ((4 * pw + 15) & ~(size_t)15) + (size_t)tile_rows * out_w * c +
                     (stage ? (((size_t)tile_rows * in_w * c + 15) & ~(size_t)15) : 0);
  CV_REQUIRE(lds <= 65536, "load_batch_u8: %zu bytes of LDS exceed 64 KiB (smaller ty / stage = 0)", lds);
  LoadArgs A;
  A.images = images;
  A.in_h = in_h;
  A.in_w = in_w;
  A.c = c;
  A.index = index;
  A.n = n;
  A.plan = plan;
  A.out_h = out_h;
  A.out_w = out_w;
  A.ty = ty;
  A.stage = stage;
  A.out = out;
  A.labels = labels;
  A.labels_out = labels_out;
  A.styles = styles;
  A.styles_out = styles_out;
  const int km = coeff_ksize(in_w, out_w) > coeff_ksize(in_h, out_h) ? coeff_ksize(in_w, out_w)
                                                                      : coeff_ksize(in_h, out_h);
  const dim3 grid(cdiv(out_h, ty), n);
  if (km <= 3)
    hipLaunchKernelGGL(load_batch_kernel<3>, grid, dim3(256), lds, S(stream), A);
  else if (km <= 5)
    hipLaunchKernelGGL(load_batch_kernel<5>, grid, dim3(256), lds, S(stream), A);
  else if (km <= 9)
    hipLaunchKernelGGL(load_batch_kernel<9>, grid, dim3(256), lds, S(stream), A);
  else
    hipLaunchKernelGGL(load_batch_kernel<0>, grid, dim3(256), lds, S(stream), A);
  CV_LAUNCH_CHECK("load_batch_u8");
  return 0;
}
