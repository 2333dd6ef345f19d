// remove_background pre/post-processing on device (src/s3od/predictor.py:79-139, src/s3od/utils.py).
//   preprocess: uint8 HWC image -> letterbox resize (cv2.resize INTER_LINEAR fixed-point, SIMD-path
//               rounding) into a zero-padded S x S canvas -> (x/255 - mean)/std (float64 math,
//               rounded to fp32 like numpy) -> fp32 NCHW [1,3,S,S]
//   postprocess: sigmoid -> unpad -> antialiased bilinear resize to the original size
//               (F.interpolate(..., antialias=True), separable triangle filter, horizontal first)
#include "common.hpp"

namespace {
constexpr int COEF_BITS = 11, COEF_SCALE = 1 << COEF_BITS;

// cv2 resizeGeneric_ coefficient for one destination index (INTER_LINEAR, fixed point)
DEV void cv_coef(int d, int ssize, int dsize, int& s0, int& s1, int& a0, int& a1) {
  double scale = (double)ssize / (double)dsize;
  float f = (float)((d + 0.5) * scale - 0.5);
  int s = (int)floorf(f);
  f -= (float)s;
  if (s < 0) { f = 0.f; s = 0; }
  if (s >= ssize - 1) { f = 0.f; s = ssize - 1; }
  s0 = s; s1 = min(s + 1, ssize - 1);
  int c0 = (int)rintf((1.f - f) * COEF_SCALE);      // saturate_cast<short>(float) rounds to nearest
  int c1 = (int)rintf(f * COEF_SCALE);
  a0 = c0; a1 = c1;
}
}  // namespace

// one thread per destination pixel of the resized (new_h x new_w) image; writes normalised fp32
// into the S x S canvas at (pad_h + y, pad_w + x).  The canvas must be pre-filled with the
// normalised value of a zero pixel (kernel below).
__global__ void preprocess_kernel(const unsigned char* __restrict__ img, int H0, int W0, int new_h, int new_w,
                                  int pad_h, int pad_w, int S, float* __restrict__ out) {
  int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= new_w || y >= new_h) return;
  const double mean[3] = {0.485, 0.456, 0.406}, stdv[3] = {0.229, 0.224, 0.225};
  int v[3];
  if (new_h == H0 && new_w == W0) {
    for (int c = 0; c < 3; c++) v[c] = img[((long)y * W0 + x) * 3 + c];
  } else {
    int sx0, sx1, ax0, ax1, sy0, sy1, by0, by1;
    cv_coef(x, W0, new_w, sx0, sx1, ax0, ax1);
    cv_coef(y, H0, new_h, sy0, sy1, by0, by1);
    for (int c = 0; c < 3; c++) {
      int r0 = img[((long)sy0 * W0 + sx0) * 3 + c] * ax0 + img[((long)sy0 * W0 + sx1) * 3 + c] * ax1;
      int r1 = img[((long)sy1 * W0 + sx0) * 3 + c] * ax0 + img[((long)sy1 * W0 + sx1) * 3 + c] * ax1;
      // VResizeLinearVec_32s8u: sat_u8((mulhi16(r0>>4, b0) + mulhi16(r1>>4, b1) + 2) >> 2)
      int t0 = ((short)(r0 >> 4) * (short)by0) >> 16;
      int t1 = ((short)(r1 >> 4) * (short)by1) >> 16;
      int o = (t0 + t1 + 2) >> 2;
      v[c] = o < 0 ? 0 : (o > 255 ? 255 : o);
    }
  }
  for (int c = 0; c < 3; c++) {
    float t = (float)v[c] / 255.0f;                  // float32 / python float -> float32 (numpy 2)
    double d = ((double)t - mean[c]) / stdv[c];       // - float64 mean, / float64 std
    out[((long)c * S + (pad_h + y)) * S + (pad_w + x)] = (float)d;
  }
}

__global__ void canvas_fill_kernel(float* out, int S) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 3L * S * S) return;
  int c = i / ((long)S * S);
  const double mean[3] = {0.485, 0.456, 0.406}, stdv[3] = {0.229, 0.224, 0.225};
  out[i] = (float)((0.0 - mean[c]) / stdv[c]);
}

// ---------------------------------------------------------------- antialiased bilinear
// PyTorch _upsample_bilinear2d_aa taps for output index i (align_corners=False, triangle filter with
// support max(scale, 1)).  The taps are not buffered: the span [xmin, xmin + xsize) is derived here and
// each weight is recomputed where it is used, so any downscale factor works (the reference resizes back
// to any original size, predictor.py:118-124).
struct AASpan {
  int xmin, xsize;
  float center, invscale, tot;
};

DEV float aa_tap(const AASpan& s, int j) {
  float x = (j + s.xmin - s.center + 0.5f) * s.invscale;
  return fabsf(x) < 1.f ? 1.f - fabsf(x) : 0.f;
}

DEV AASpan aa_span(int i, int in, int out) {
  AASpan s;
  float scale = (float)in / (float)out;
  float support = scale >= 1.f ? scale : 1.f;
  s.center = scale * (i + 0.5f);
  s.invscale = scale >= 1.f ? 1.f / scale : 1.f;
  s.xmin = max((int)(s.center - support + 0.5f), 0);
  s.xsize = min((int)(s.center + support + 0.5f), in) - s.xmin;
  float tot = 0.f;
  for (int j = 0; j < s.xsize; j++) tot += aa_tap(s, j);
  s.tot = tot;                // weights are w_j / tot (0 when tot == 0), as PyTorch normalises them
  return s;
}

DEV float aa_weight(const AASpan& s, int j) { return s.tot != 0.f ? aa_tap(s, j) / s.tot : 0.f; }

// pass 1: sigmoid + crop + horizontal resample: [NM][LH][LW] logits -> tmp [NM][h][W0]
__global__ void post_h_kernel(const float* __restrict__ logits, int LH, int LW, int pad_h, int pad_w, int h, int w, int W0,
                              float* __restrict__ tmp) {
  int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, c = blockIdx.z;
  if (x >= W0) return;
  AASpan sp = aa_span(x, w, W0);
  const float* row = logits + ((long)c * LH + (pad_h + y)) * LW + pad_w + sp.xmin;
  float acc = 0.f;
  for (int j = 0; j < sp.xsize; j++) acc += aa_weight(sp, j) * (1.f / (1.f + expf(-row[j])));
  tmp[((long)c * h + y) * W0 + x] = acc;
}

// pass 2: vertical resample -> out [NM][H0][W0]
__global__ void post_v_kernel(const float* __restrict__ tmp, int h, int H0, int W0, float* __restrict__ out) {
  int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, c = blockIdx.z;
  if (x >= W0) return;
  AASpan sp = aa_span(y, h, H0);
  const float* col = tmp + ((long)c * h + sp.xmin) * W0 + x;
  float acc = 0.f;
  for (int j = 0; j < sp.xsize; j++) acc += aa_weight(sp, j) * col[(long)j * W0];
  out[((long)c * H0 + y) * W0 + x] = acc;
}

extern "C" {

// img: device uint8 [H0][W0][3]; out: fp32 [1][3][S][S]
int s3od_preprocess(const void* img, int H0, int W0, int new_h, int new_w, int pad_h, int pad_w, int S, float* out, void* stream) {
  S3OD_REQUIRE(new_h + pad_h <= S && new_w + pad_w <= S, "preprocess: resized image does not fit the canvas");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(canvas_fill_kernel, dim3(cdiv(3L * S * S, 256)), dim3(256), 0, st, out, S);
  hipLaunchKernelGGL(preprocess_kernel, dim3(cdiv(new_w, 256), new_h), dim3(256), 0, st, (const unsigned char*)img, H0, W0,
                     new_h, new_w, pad_h, pad_w, S, out);
  return s3od_check_launch("preprocess");
}

// logits: fp32 [NM][LH][LW] (one image, NM masks; LH x LW = S x S, or S x 16*floor(new_w/16) for the
// reference's unpadded Quirk-2 input); tmp: fp32 [NM][h][W0]; out: fp32 [NM][H0][W0]
int s3od_sigmoid_unpad_resize(const float* logits, int NM, int LH, int LW, int pad_h, int pad_w, int h, int w, int H0, int W0,
                              float* tmp, float* out, void* stream) {
  S3OD_REQUIRE(NM >= 1 && NM <= 64 && h > 0 && w > 0, "postprocess: bad mask count / crop");
  S3OD_REQUIRE(H0 > 0 && W0 > 0 && H0 <= 65535 && h <= 65535, "postprocess: output size out of range");
  S3OD_REQUIRE(pad_h + h <= LH && pad_w + w <= LW, "postprocess: crop outside the logits");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(post_h_kernel, dim3(cdiv(W0, 256), h, NM), dim3(256), 0, st, logits, LH, LW, pad_h, pad_w, h, w, W0, tmp);
  hipLaunchKernelGGL(post_v_kernel, dim3(cdiv(W0, 256), H0, NM), dim3(256), 0, st, tmp, h, H0, W0, out);
  return s3od_check_launch("sigmoid_unpad_resize");
}

}  // extern "C"
