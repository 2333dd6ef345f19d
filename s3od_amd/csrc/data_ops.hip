// Training-batch construction on device (synth_sod/.../dataset.py:34-131 MaskDataset.__getitem__ and
// transforms.py:12-224 get_transforms, "test" and "regular" modes), one fused pass per sample:
//   LongestMaxSize + centred PadIfNeeded (letterbox, zero fill) -> geometric augmentation
//   (HorizontalFlip, VerticalFlip, RandomRotate90, RandomResizedCrop, Rotate: composed on the host
//   into ONE inverse affine map from output pixel to canvas coordinates) -> ColorJitter ->
//   multiplicative / Gaussian noise -> Normalize(ImageNet) ; mask: same geometry, nearest, /255.
// Reads the uint8 source once (L2-resident taps), writes fp32 NCHW image + fp32 mask: HBM-bound.
// Random parameters are drawn on the host per sample; Gaussian noise uses a counter-based hash
// RNG (seed, pixel, channel), so a batch is reproducible from its seed.
#include "common.hpp"

struct AugParams {
  float A[6];                 // canvas coords of an output pixel centre: (A0 x + A1 y + A2, A3 x + A4 y + A5)
  int H0, W0, new_h, new_w, pad_h, pad_w;   // letterbox geometry of the source in the S x S canvas
  float bright, contrast, sat, hue;          // ColorJitter factors (1, 1, 1, 0 = identity); hue in turns
  float gray_mean;            // mean grey of the (brightness-adjusted) canvas, for contrast
  float mult[3];              // multiplicative noise per channel (1 = off)
  float gauss_std;            // Gaussian noise std in [0,1] units (0 = off)
  unsigned seed;
};

namespace {
// value in [0,1] of canvas pixel (ix, iy) of channel c: inside the resized region -> bilinear
// sample of the source (cv2 INTER_LINEAR half-pixel mapping, edge replicate), else 0 (pad)
DEV float canvas_px(const unsigned char* img, const AugParams& P, int ix, int iy, int c) {
  int rx = ix - P.pad_w, ry = iy - P.pad_h;
  if (rx < 0 || ry < 0 || rx >= P.new_w || ry >= P.new_h) return 0.f;
  float u = (rx + 0.5f) * ((float)P.W0 / P.new_w) - 0.5f, v = (ry + 0.5f) * ((float)P.H0 / P.new_h) - 0.5f;
  u = fminf(fmaxf(u, 0.f), P.W0 - 1.f); v = fminf(fmaxf(v, 0.f), P.H0 - 1.f);
  int x0 = (int)u, y0 = (int)v, x1 = min(x0 + 1, P.W0 - 1), y1 = min(y0 + 1, P.H0 - 1);
  float fx = u - x0, fy = v - y0;
  float a = img[((long)y0 * P.W0 + x0) * 3 + c], b = img[((long)y0 * P.W0 + x1) * 3 + c];
  float d = img[((long)y1 * P.W0 + x0) * 3 + c], e = img[((long)y1 * P.W0 + x1) * 3 + c];
  return ((a * (1.f - fx) + b * fx) * (1.f - fy) + (d * (1.f - fx) + e * fx) * fy) * (1.f / 255.f);
}
DEV unsigned hash3(unsigned a, unsigned b, unsigned c) {
  unsigned h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ (c + 0x165667B1u) * 0xC2B2AE3Du;
  h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
  return h;
}
DEV float clamp01(float v) { return fminf(fmaxf(v, 0.f), 1.f); }
}  // namespace

__global__ void augment_sample_kernel(const unsigned char* __restrict__ img, const unsigned char* __restrict__ mask,
                                      AugParams P, int S, float* __restrict__ out_img, float* __restrict__ out_mask) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= S) return;
  const float cx = P.A[0] * (x + 0.5f) + P.A[1] * (y + 0.5f) + P.A[2] - 0.5f;
  const float cy = P.A[3] * (x + 0.5f) + P.A[4] * (y + 0.5f) + P.A[5] - 0.5f;
  // canvas bilinear (constant-0 border outside the canvas, like Rotate / crop borders)
  const float fx0 = floorf(cx), fy0 = floorf(cy);
  const int ix = (int)fx0, iy = (int)fy0;
  const float fx = cx - fx0, fy = cy - fy0;
  float rgb[3];
#pragma unroll
  for (int c = 0; c < 3; c++) {
    float acc = 0.f;
#pragma unroll
    for (int t = 0; t < 4; t++) {
      int tx = ix + (t & 1), ty = iy + (t >> 1);
      float w = ((t & 1) ? fx : 1.f - fx) * ((t >> 1) ? fy : 1.f - fy);
      if (w != 0.f && tx >= 0 && ty >= 0 && tx < S && ty < S) acc += w * canvas_px(img, P, tx, ty, c);
    }
    rgb[c] = acc;
  }
  // ColorJitter (fixed order brightness, contrast, saturation, hue), clipped like uint8 images
  if (P.bright != 1.f) for (int c = 0; c < 3; c++) rgb[c] = clamp01(rgb[c] * P.bright);
  if (P.contrast != 1.f) for (int c = 0; c < 3; c++) rgb[c] = clamp01((rgb[c] - P.gray_mean) * P.contrast + P.gray_mean);
  if (P.sat != 1.f) {
    float g = 0.299f * rgb[0] + 0.587f * rgb[1] + 0.114f * rgb[2];
    for (int c = 0; c < 3; c++) rgb[c] = clamp01((rgb[c] - g) * P.sat + g);
  }
  if (P.hue != 0.f) {   // rotation about the grey axis by 2*pi*hue
    float th = 6.283185307f * P.hue, cs = cosf(th), sn = sinf(th);
    const float k = 0.57735027f, a = (1.f - cs) / 3.f, b = k * sn;
    float r = rgb[0], g = rgb[1], bl = rgb[2];
    rgb[0] = clamp01((cs + a) * r + (a - b) * g + (a + b) * bl);
    rgb[1] = clamp01((a + b) * r + (cs + a) * g + (a - b) * bl);
    rgb[2] = clamp01((a - b) * r + (a + b) * g + (cs + a) * bl);
  }
  const double mean[3] = {0.485, 0.456, 0.406}, stdv[3] = {0.229, 0.224, 0.225};
  const long plane = (long)S * S, o = (long)y * S + x;
#pragma unroll
  for (int c = 0; c < 3; c++) {
    float v = rgb[c] * P.mult[c];
    if (P.gauss_std > 0.f) {
      unsigned h1 = hash3(P.seed, (unsigned)o, 2 * c), h2 = hash3(P.seed, (unsigned)o, 2 * c + 1);
      float u1 = ((h1 >> 8) + 1) * (1.f / 16777217.f), u2 = (h2 >> 8) * (1.f / 16777216.f);
      v += P.gauss_std * sqrtf(-2.f * logf(u1)) * cosf(6.283185307f * u2);
    }
    v = clamp01(v);
    out_img[c * plane + o] = (float)(((double)v - mean[c]) / stdv[c]);
  }
  if (out_mask) {   // nearest (cv2 INTER_NEAREST on the resize, nearest on the geometric warp)
    int nx = (int)floorf(cx + 0.5f), ny = (int)floorf(cy + 0.5f);
    float m = 0.f;
    int rx = nx - P.pad_w, ry = ny - P.pad_h;
    if (nx >= 0 && ny >= 0 && nx < S && ny < S && rx >= 0 && ry >= 0 && rx < P.new_w && ry < P.new_h) {
      int sx = min((int)floorf(rx * ((float)P.W0 / P.new_w)), P.W0 - 1);
      int sy = min((int)floorf(ry * ((float)P.H0 / P.new_h)), P.H0 - 1);
      m = mask[(long)sy * P.W0 + sx] * (1.f / 255.f);
    }
    out_mask[o] = m;
  }
}

extern "C" {

// img: device uint8 [H0][W0][3]; mask: device uint8 [H0][W0] (nullable with out_mask);
// params: host AugParams; out_img fp32 [3][S][S] (one batch slot), out_mask fp32 [S][S]
int s3od_augment_sample(const void* img, const void* mask, const void* params, int S, float* out_img, float* out_mask,
                        void* stream) {
  const AugParams P = *(const AugParams*)params;
  S3OD_REQUIRE(P.H0 > 0 && P.W0 > 0 && P.new_h > 0 && P.new_w > 0 && P.new_h + P.pad_h <= S && P.new_w + P.pad_w <= S,
               "augment_sample: bad letterbox geometry");
  S3OD_REQUIRE((mask == nullptr) == (out_mask == nullptr), "augment_sample: mask and out_mask go together");
  hipLaunchKernelGGL(augment_sample_kernel, dim3(cdiv(S, 256), S), dim3(256), 0, (hipStream_t)stream,
                     (const unsigned char*)img, (const unsigned char*)mask, P, S, out_img, out_mask);
  return s3od_check_launch("augment_sample");
}

}  // extern "C"
