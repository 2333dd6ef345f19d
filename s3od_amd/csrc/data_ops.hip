// Training-batch construction on device (synth_sod/.../dataset.py:34-131 MaskDataset.__getitem__ and
// transforms.py:12-224 get_transforms, "test" and "regular" modes), one fused pass per sample:
//   LongestMaxSize + centred PadIfNeeded (letterbox, zero fill) -> geometric augmentation
//   (HorizontalFlip, VerticalFlip, RandomRotate90, RandomResizedCrop, Rotate: composed on the host
//   into ONE inverse affine map from output pixel to canvas coordinates) -> ColorJitter ->
//   multiplicative / Gaussian noise -> Normalize(ImageNet) ; mask: same geometry, nearest, /255.
// Reads the uint8 source once (L2-resident taps), writes fp32 NCHW image + fp32 mask: HBM-bound.
// Random parameters are drawn on the host per sample; Gaussian noise uses a counter-based hash
// RNG (seed, pixel, channel), so a batch is reproducible from its seed.
// "synthetic" mode (transforms.py:65-220): the geometric pass also applies the Perspective /
// OpticalDistortion members of the distortion group and writes raw [0,1] RGB; two photometric
// passes (s3od_augment_synthetic) then apply the colour / noise / brightness-contrast / shadow group
// (per pixel), then downscale + blur + sharpen/emboss (one composed 2-D filter), colour-space,
// posterize and Normalize.
#include "common.hpp"

struct AugParams {
  float A[6];                 // canvas coords of an output pixel centre: (A0 x + A1 y + A2, A3 x + A4 y + A5) / den
  int H0, W0, new_h, new_w, pad_h, pad_w;   // letterbox geometry of the source in the S x S canvas
  float bright, contrast, sat, hue;          // ColorJitter factors (1, 1, 1, 0 = identity); hue in turns
  float gray_mean;            // mean grey of the (brightness-adjusted) canvas, for contrast
  float mult[3];              // multiplicative noise per channel (1 = off)
  float gauss_std;            // Gaussian noise std in [0,1] units (0 = off)
  unsigned seed;
  float persp[2];             // den = persp0 x + persp1 y + 1 (Perspective; 0, 0 = affine)
  float kdist;                // radial OpticalDistortion of the output coordinates (0 = off)
  int raw;                    // 1: write raw [0,1] RGB (no jitter / noise / Normalize): synthetic pipeline
};

// synthetic-mode photometric chain (host-drawn; every member has an identity setting)
struct SynthParams {
  float bright, contrast, sat, hue, gray_mean;   // ColorJitter (group 1)
  float hsv_h, hsv_s, hsv_v;                      // HueSaturationValue shifts: degrees, [0,1] units (group 1)
  float iso_int, iso_color;                       // ISONoise: luminance / colour noise std (group 2)
  float gauss_std;                                // GaussNoise std, [0,1] units (group 2)
  float mult[3];                                  // MultiplicativeNoise (group 2)
  float rbc_alpha, rbc_beta;                      // RandomBrightnessContrast (group 4)
  int n_shadow;                                   // RandomShadow triangles (group 4), 0..3
  float shadow[3][6];                             //   vertices (x0,y0,x1,y1,x2,y2) in output pixels
  float shadow_dim;                               //   multiplier inside a shadow
  float down;                                     // Downscale factor (group 3; 1 = off), nearest down + nearest up
  int ksize;                                      // composed blur (group 5) * sharpen / emboss (group 8) filter, odd <= 15
  int color_op;                                   // group 6: 0 none, 1 sepia, 2 gray, 3 channel shuffle
  int perm[3];                                    //   channel shuffle permutation
  int post_bits;                                  // Posterize bits (group 8; 8 = off)
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
// standard normal from the counter-based hash (Box-Muller on two hashed uniforms)
DEV float gauss(unsigned seed, unsigned pix, int c) {
  unsigned h1 = hash3(seed, pix, 2 * c), h2 = hash3(seed, pix, 2 * c + 1);
  float u1 = ((h1 >> 8) + 1) * (1.f / 16777217.f), u2 = (h2 >> 8) * (1.f / 16777216.f);
  return sqrtf(-2.f * logf(u1)) * cosf(6.283185307f * u2);
}
DEV void jitter(float* rgb, float bright, float contrast, float sat, float hue, float gray_mean) {
  if (bright != 1.f) for (int c = 0; c < 3; c++) rgb[c] = clamp01(rgb[c] * bright);
  if (contrast != 1.f) for (int c = 0; c < 3; c++) rgb[c] = clamp01((rgb[c] - gray_mean) * contrast + gray_mean);
  if (sat != 1.f) {
    float g = 0.299f * rgb[0] + 0.587f * rgb[1] + 0.114f * rgb[2];
    for (int c = 0; c < 3; c++) rgb[c] = clamp01((rgb[c] - g) * sat + g);
  }
  if (hue != 0.f) {   // rotation about the grey axis by 2*pi*hue
    float th = 6.283185307f * hue, cs = cosf(th), sn = sinf(th);
    const float k = 0.57735027f, a = (1.f - cs) / 3.f, b = k * sn;
    float r = rgb[0], g = rgb[1], bl = rgb[2];
    rgb[0] = clamp01((cs + a) * r + (a - b) * g + (a + b) * bl);
    rgb[1] = clamp01((a + b) * r + (cs + a) * g + (a - b) * bl);
    rgb[2] = clamp01((a - b) * r + (a + b) * g + (cs + a) * bl);
  }
}
// point-in-triangle (same-sign edge functions)
DEV bool in_tri(const float* t, float px, float py) {
  float d0 = (t[2] - t[0]) * (py - t[1]) - (t[3] - t[1]) * (px - t[0]);
  float d1 = (t[4] - t[2]) * (py - t[3]) - (t[5] - t[3]) * (px - t[2]);
  float d2 = (t[0] - t[4]) * (py - t[5]) - (t[1] - t[5]) * (px - t[4]);
  return (d0 >= 0.f && d1 >= 0.f && d2 >= 0.f) || (d0 <= 0.f && d1 <= 0.f && d2 <= 0.f);
}
}  // namespace

__global__ void augment_sample_kernel(const unsigned char* __restrict__ img, const unsigned char* __restrict__ mask,
                                      AugParams P, int S, float* __restrict__ out_img, float* __restrict__ out_mask) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= S) return;
  float xo = x + 0.5f, yo = y + 0.5f;
  if (P.kdist != 0.f) {       // radial distortion about the image centre (normalised radius)
    const float h = 0.5f * S, u = (xo - h) / h, v = (yo - h) / h, f = 1.f + P.kdist * (u * u + v * v);
    xo = h + u * f * h; yo = h + v * f * h;
  }
  const float den = P.persp[0] * xo + P.persp[1] * yo + 1.f;
  const float cx = (P.A[0] * xo + P.A[1] * yo + P.A[2]) / den - 0.5f;
  const float cy = (P.A[3] * xo + P.A[4] * yo + P.A[5]) / den - 0.5f;
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
  const long plane = (long)S * S, o = (long)y * S + x;
  if (P.raw) {
#pragma unroll
    for (int c = 0; c < 3; c++) out_img[c * plane + o] = rgb[c];
  } else {
    // ColorJitter (fixed order brightness, contrast, saturation, hue), clipped like uint8 images
    jitter(rgb, P.bright, P.contrast, P.sat, P.hue, P.gray_mean);
    const double mean[3] = {0.485, 0.456, 0.406}, stdv[3] = {0.229, 0.224, 0.225};
#pragma unroll
    for (int c = 0; c < 3; c++) {
      float v = rgb[c] * P.mult[c];
      if (P.gauss_std > 0.f) v += P.gauss_std * gauss(P.seed, (unsigned)o, c);
      v = clamp01(v);
      out_img[c * plane + o] = (float)(((double)v - mean[c]) / stdv[c]);
    }
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

// synthetic pass 1 (per pixel): colour group (ColorJitter | HueSaturationValue), noise group
// (ISONoise | GaussNoise | MultiplicativeNoise), RandomBrightnessContrast | RandomShadow.  In-place on
// the raw [0,1] image x [3][S][S].
__global__ void synth_pixel_kernel(float* __restrict__ x, SynthParams P, int S) {
  const int px = blockIdx.x * blockDim.x + threadIdx.x, py = blockIdx.y;
  if (px >= S) return;
  const long plane = (long)S * S, o = (long)py * S + px;
  float rgb[3] = {x[o], x[plane + o], x[2 * plane + o]};
  jitter(rgb, P.bright, P.contrast, P.sat, P.hue, P.gray_mean);
  if (P.hsv_h != 0.f || P.hsv_s != 0.f || P.hsv_v != 0.f) {
    float r = rgb[0], g = rgb[1], b = rgb[2];
    float mx = fmaxf(r, fmaxf(g, b)), mn = fminf(r, fminf(g, b)), d = mx - mn;
    float h = 0.f;
    if (d > 0.f) h = mx == r ? fmodf((g - b) / d + 6.f, 6.f) : (mx == g ? (b - r) / d + 2.f : (r - g) / d + 4.f);
    float sv = mx > 0.f ? d / mx : 0.f, vv = mx;
    h = fmodf(h * 60.f + P.hsv_h + 360.f, 360.f) / 60.f;
    sv = clamp01(sv + P.hsv_s); vv = clamp01(vv + P.hsv_v);
    float c = vv * sv, xx = c * (1.f - fabsf(fmodf(h, 2.f) - 1.f)), m = vv - c;
    int hi = min((int)h, 5);
    float rr = hi == 0 || hi == 5 ? c : (hi == 1 || hi == 4 ? xx : 0.f);
    float gg = hi == 1 || hi == 2 ? c : (hi == 0 || hi == 3 ? xx : 0.f);
    float bb = hi == 3 || hi == 4 ? c : (hi == 2 || hi == 5 ? xx : 0.f);
    rgb[0] = rr + m; rgb[1] = gg + m; rgb[2] = bb + m;
  }
  if (P.iso_int > 0.f || P.iso_color > 0.f) {   // luminance noise shared by the channels + per-channel colour noise
    float l = P.iso_int * gauss(P.seed, (unsigned)o, 3);
    for (int c = 0; c < 3; c++) rgb[c] = clamp01(rgb[c] + l + P.iso_color * gauss(P.seed ^ 0x5bd1e995u, (unsigned)o, c));
  }
  for (int c = 0; c < 3; c++) {
    float v = rgb[c] * P.mult[c];
    if (P.gauss_std > 0.f) v += P.gauss_std * gauss(P.seed, (unsigned)o, c);
    v = v * P.rbc_alpha + P.rbc_beta;
    rgb[c] = clamp01(v);
  }
  for (int t = 0; t < P.n_shadow; t++)
    if (in_tri(P.shadow[t], px + 0.5f, py + 0.5f)) { for (int c = 0; c < 3; c++) rgb[c] *= P.shadow_dim; break; }
#pragma unroll
  for (int c = 0; c < 3; c++) x[c * plane + o] = rgb[c];
}

// synthetic pass 2: out = Normalize(posterize(colour_op(clip(sum_t w_t * down(x)(p + t))))) with the composed
// ksize x ksize filter (GaussianBlur | MotionBlur | Defocus, then Sharpen | Emboss: both linear, so they
// compose into one kernel) and the Downscale nearest-down / nearest-up sampling of its taps.
__global__ void synth_filter_kernel(const float* __restrict__ x, const float* __restrict__ kw, SynthParams P, int S,
                                    float* __restrict__ out) {
  const int px = blockIdx.x * blockDim.x + threadIdx.x, py = blockIdx.y;
  if (px >= S) return;
  const long plane = (long)S * S, o = (long)py * S + px;
  const int r = P.ksize / 2;
  const int Sd = max(1, (int)(S * P.down));
  float rgb[3] = {0.f, 0.f, 0.f};
  for (int dy = -r; dy <= r; dy++) {
    int yy = min(max(py + dy, 0), S - 1);      // BORDER_REFLECT_101 approximated by clamp
    for (int dx = -r; dx <= r; dx++) {
      int xx = min(max(px + dx, 0), S - 1);
      float w = kw ? kw[(dy + r) * P.ksize + (dx + r)] : 1.f;
      int sx = xx, sy = yy;
      if (P.down < 1.f) {    // nearest down to Sd x Sd, nearest back up to S x S
        int dxs = min((int)(xx * (float)Sd / S), Sd - 1), dys = min((int)(yy * (float)Sd / S), Sd - 1);
        sx = min((int)((dxs + 0.5f) * S / Sd), S - 1); sy = min((int)((dys + 0.5f) * S / Sd), S - 1);
      }
      const long q = (long)sy * S + sx;
      rgb[0] += w * x[q]; rgb[1] += w * x[plane + q]; rgb[2] += w * x[2 * plane + q];
    }
  }
  for (int c = 0; c < 3; c++) rgb[c] = clamp01(rgb[c]);
  if (P.color_op == 1) {          // ToSepia
    float r0 = rgb[0], g0 = rgb[1], b0 = rgb[2];
    rgb[0] = clamp01(0.393f * r0 + 0.769f * g0 + 0.189f * b0);
    rgb[1] = clamp01(0.349f * r0 + 0.686f * g0 + 0.168f * b0);
    rgb[2] = clamp01(0.272f * r0 + 0.534f * g0 + 0.131f * b0);
  } else if (P.color_op == 2) {   // ToGray (weighted average)
    float g = 0.299f * rgb[0] + 0.587f * rgb[1] + 0.114f * rgb[2];
    rgb[0] = rgb[1] = rgb[2] = g;
  } else if (P.color_op == 3) {   // ChannelShuffle
    float t[3] = {rgb[P.perm[0]], rgb[P.perm[1]], rgb[P.perm[2]]};
    rgb[0] = t[0]; rgb[1] = t[1]; rgb[2] = t[2];
  }
  if (P.post_bits < 8) {          // Posterize: keep the top post_bits of the 8-bit value
    const int mask = (0xFF << (8 - P.post_bits)) & 0xFF;
    for (int c = 0; c < 3; c++) rgb[c] = (float)(((int)(rgb[c] * 255.f + 0.5f)) & mask) * (1.f / 255.f);
  }
  const double mean[3] = {0.485, 0.456, 0.406}, stdv[3] = {0.229, 0.224, 0.225};
#pragma unroll
  for (int c = 0; c < 3; c++) out[c * plane + o] = (float)(((double)rgb[c] - mean[c]) / stdv[c]);
}

extern "C" {

// raw: fp32 [3][S][S] in [0,1] from s3od_augment_sample with AugParams.raw = 1 (overwritten: scratch);
// params: host SynthParams; kw: device fp32 [ksize][ksize] filter (nullable when ksize == 1);
// out: fp32 [3][S][S] ImageNet-normalised
int s3od_augment_synthetic(float* raw, const void* params, const float* kw, int S, float* out, void* stream) {
  const SynthParams P = *(const SynthParams*)params;
  S3OD_REQUIRE(P.ksize >= 1 && P.ksize <= 15 && (P.ksize & 1), "augment_synthetic: ksize must be odd, 1..15");
  S3OD_REQUIRE(P.ksize == 1 || kw != nullptr, "augment_synthetic: filter weights missing");
  S3OD_REQUIRE(P.n_shadow >= 0 && P.n_shadow <= 3 && P.post_bits >= 1 && P.post_bits <= 8 && P.down > 0.f && P.down <= 1.f,
               "augment_synthetic: bad parameters");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(synth_pixel_kernel, dim3(cdiv(S, 256), S), dim3(256), 0, st, raw, P, S);
  hipLaunchKernelGGL(synth_filter_kernel, dim3(cdiv(S, 256), S), dim3(256), 0, st, raw, P.ksize > 1 ? kw : nullptr, P, S, out);
  return s3od_check_launch("augment_synthetic");
}

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
