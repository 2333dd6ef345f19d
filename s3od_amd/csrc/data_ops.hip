// Training-batch construction on device (synth_sod/.../dataset.py:34-131 MaskDataset.__getitem__ and
// transforms.py:12-224 get_transforms, "test" and "regular" modes), one fused pass per sample:
//   LongestMaxSize + centred PadIfNeeded (letterbox, zero fill) -> geometric augmentation
//   (HorizontalFlip, VerticalFlip, RandomRotate90, RandomResizedCrop, Rotate: composed on the host
//   into ONE inverse affine map from output pixel to canvas coordinates) -> ColorJitter ->
//   multiplicative / Gaussian noise -> Normalize(ImageNet) ; mask: same geometry, nearest, /255.
// Reads the uint8 source once (L2-resident taps), writes fp32 NCHW image + fp32 mask: HBM-bound.
// Random parameters are drawn on the host per sample; Gaussian noise uses a counter-based hash
// RNG (seed, pixel, channel), so a batch is reproducible from its seed.
// "synthetic" mode (transforms.py:65-220): the geometric pass also applies the distortion group
// (OpticalDistortion, GridDistortion (separable maps), ElasticTransform (displacement field from
// s3od_elastic_field), Perspective) and writes raw [0,1] RGB; s3od_augment_synthetic then runs the
// photometric groups in the reference's order: [CLAHE: histogram / LUT / apply passes] -> per pixel
// colour + noise (ColorJitter | HueSaturationValue, ISONoise (HLS, Poisson luminance) | GaussNoise |
// MultiplicativeNoise) -> [ImageCompression: 8x8 DCT quantise / dequantise, 4:2:0] -> one filter pass
// (Downscale sampling, RandomShadow | RandomBrightnessContrast per sampled tap, blur kernel | ZoomBlur,
// colour space, Sharpen | Emboss (composed with the blur kernel), Posterize, RandomSnow) ->
// [RandomRain: drop lines + 7x7 box blur + 0.7 brightness] -> Normalize.
// "regular" mode draws of Sharpen / ISONoise (transforms.py:44-62) run the same entry in order 1:
// raw geometry -> Sharpen filter -> ColorJitter + noise -> Normalize.
// Algorithms restated from albumentations 2.0.8 / OpenCV 4.12 (pinned in uv.lock; neither is in this
// image, so parity is against oracle/augment_oracle.py, a numpy restatement, not the libraries).
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
  const float* grid;          // GridDistortion maps (device [2][S]: x map then y map, index coords) or null
  const float* elastic;       // ElasticTransform displacement (device [2][S][S]: dx then dy) or null
};

// photometric chain (host-drawn; every member has an identity setting)
struct SynthParams {
  float bright, contrast, sat, hue, gray_mean;   // ColorJitter (group 1)
  float hsv_h, hsv_s, hsv_v;                      // HueSaturationValue shifts: degrees, [0,1] units (group 1)
  float clahe_clip;                               // CLAHE clip limit, 8x8 tiles on L of Lab (group 1; 0 = off)
  float iso_intensity, iso_color_shift;           // ISONoise (group 2; intensity 0 = off)
  float gauss_std;                                // GaussNoise std, [0,1] units (group 2)
  float mult[3];                                  // MultiplicativeNoise (group 2)
  int jpeg_quality;                               // ImageCompression quality (group 3; 0 = off)
  float down;                                     // Downscale factor (group 3; 1 = off), nearest down + nearest up
  float rbc_alpha, rbc_beta;                      // RandomBrightnessContrast (group 4)
  int n_shadow;                                   // RandomShadow polygons (group 4), 0..3
  float shadow[3][10];                            //   5 vertices (x0,y0,...,x4,y4) each, output pixels
  float shadow_dim;                               //   multiplier inside a polygon (1 - shadow_intensity)
  int ksize;                                      // composed blur (group 5) * sharpen / emboss (group 8) filter, odd <= 15
  int zoom_n;                                     // ZoomBlur (group 5): number of zoom factors (0 = off)
  float zoom[4];                                  //   factors (arange(1, max_factor, step_factor))
  int color_op;                                   // group 6: 0 none, 1 sepia, 2 gray, 3 channel shuffle
  int perm[3];                                    //   channel shuffle permutation
  int post_bits;                                  // Posterize bits (group 8; 8 = off)
  float snow_point, snow_coeff;                   // RandomSnow "bleach" (group 9; snow_point 0 = off)
  int rain_n, rain_slant, rain_len, rain_blur;    // RandomRain "default" (group 9; rain_n 0 = off)
  float rain_color, rain_bright;                  //   drop colour ([0,1], grey), brightness coefficient
  int order;                                      // 0: synthetic chain; 1: regular chain (filter, then colour + noise)
  unsigned seed;
  const int* rain_drops;                          // device [rain_n][2] drop start (x, y)
  float* ws;                                      // device workspace, augment_ws_floats(S) floats (null if unused)
};

// workspace layout (floats): scratch image [3][S][S] | JPEG Y [Sp][Sp] | JPEG Cb, Cr [Sp/2][Sp/2] each |
// CLAHE histograms int [64][256] | CLAHE LUTs [64][256] | 8 doubles of statistics;  Sp = 16 * ceil(S / 16)
static inline long ws_sp(int S) { return 16L * ((S + 15) / 16); }
static inline long ws_jpeg_y(int S) { return 3L * S * S; }
static inline long ws_jpeg_c(int S) { return ws_jpeg_y(S) + ws_sp(S) * ws_sp(S); }
static inline long ws_hist(int S) { return ws_jpeg_c(S) + 2 * (ws_sp(S) / 2) * (ws_sp(S) / 2); }
static inline long ws_lut(int S) { return ws_hist(S) + 64 * 256; }
static inline long ws_stats(int S) { long o = ws_lut(S) + 64 * 256; return (o + 1) & ~1L; }
static inline long ws_floats(int S) { return ws_stats(S) + 16; }

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
// uniform in (0, 1) from the hash
DEV float uni(unsigned seed, unsigned pix, unsigned c) { return ((hash3(seed, pix, c) >> 8) + 0.5f) * (1.f / 16777216.f); }
// Poisson(lam) by sequential inversion of one uniform (capped far in the tail)
DEV int poisson(float lam, float u) {
  float p = expf(-lam), F = p;
  int k = 0;
  const int cap = (int)(3.f * lam) + 40;
  while (u > F && k < cap) { k++; p = p * lam / (float)k; F += p; }
  return k;
}
// BORDER_REFLECT_101 index
DEV int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
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
DEV void hsv_shift(float* rgb, float dh, float ds, float dv) {
  float r = rgb[0], g = rgb[1], b = rgb[2];
  float mx = fmaxf(r, fmaxf(g, b)), mn = fminf(r, fminf(g, b)), d = mx - mn;
  float h = 0.f;
  if (d > 0.f) h = mx == r ? fmodf((g - b) / d + 6.f, 6.f) : (mx == g ? (b - r) / d + 2.f : (r - g) / d + 4.f);
  float sv = mx > 0.f ? d / mx : 0.f, vv = mx;
  h = fmodf(h * 60.f + dh + 360.f, 360.f) / 60.f;
  sv = clamp01(sv + ds); vv = clamp01(vv + dv);
  float c = vv * sv, xx = c * (1.f - fabsf(fmodf(h, 2.f) - 1.f)), m = vv - c;
  int hi = min((int)h, 5);
  float rr = hi == 0 || hi == 5 ? c : (hi == 1 || hi == 4 ? xx : 0.f);
  float gg = hi == 1 || hi == 2 ? c : (hi == 0 || hi == 3 ? xx : 0.f);
  float bb = hi == 3 || hi == 4 ? c : (hi == 2 || hi == 5 ? xx : 0.f);
  rgb[0] = rr + m; rgb[1] = gg + m; rgb[2] = bb + m;
}
// group 1 per-pixel members (ColorJitter | HueSaturationValue)
DEV void colour_group(float* rgb, const SynthParams& P) {
  jitter(rgb, P.bright, P.contrast, P.sat, P.hue, P.gray_mean);
  if (P.hsv_h != 0.f || P.hsv_s != 0.f || P.hsv_v != 0.f) hsv_shift(rgb, P.hsv_h, P.hsv_s, P.hsv_v);
}
// cv2 COLOR_RGB2HLS / HLS2RGB for float images (H in degrees [0, 360), L and S in [0, 1])
DEV void rgb2hls(const float* rgb, float& h, float& l, float& s) {
  float r = rgb[0], g = rgb[1], b = rgb[2];
  float vmax = fmaxf(r, fmaxf(g, b)), vmin = fminf(r, fminf(g, b)), diff = vmax - vmin;
  l = (vmax + vmin) * 0.5f;
  h = 0.f; s = 0.f;
  if (diff > 1.1920929e-7f) {
    s = l < 0.5f ? diff / (vmax + vmin) : diff / (2.f - vmax - vmin);
    float k = 60.f / diff;
    if (vmax == r) h = (g - b) * k;
    else if (vmax == g) h = (b - r) * k + 120.f;
    else h = (r - g) * k + 240.f;
    if (h < 0.f) h += 360.f;
  }
}
DEV void hls2rgb(float h, float l, float s, float* rgb) {
  if (s == 0.f) { rgb[0] = rgb[1] = rgb[2] = l; return; }
  const int sector_data[6][3] = {{1, 3, 0}, {1, 0, 2}, {3, 0, 1}, {0, 2, 1}, {0, 1, 3}, {2, 1, 0}};
  float p2 = l <= 0.5f ? l * (1.f + s) : l + s - l * s, p1 = 2.f * l - p2;
  h *= (1.f / 60.f);
  while (h < 0.f) h += 6.f;
  while (h >= 6.f) h -= 6.f;
  int sector = (int)floorf(h);
  h -= sector;
  float tab[4] = {p2, p1, p1 + (p2 - p1) * (1.f - h), p1 + (p2 - p1) * h};
  rgb[2] = tab[sector_data[sector][0]];   // cv2 writes b, g, r in that order from the table
  rgb[1] = tab[sector_data[sector][1]];
  rgb[0] = tab[sector_data[sector][2]];
}
// sRGB <-> CIE Lab (D65), cv2's float formulas (L in [0, 100])
DEV float srgb_lin(float v) { return v > 0.04045f ? powf((v + 0.055f) / 1.055f, 2.4f) : v / 12.92f; }
DEV float lin_srgb(float v) { return v > 0.0031308f ? 1.055f * powf(v, 1.f / 2.4f) - 0.055f : 12.92f * v; }
DEV float lab_f(float t) { return t > 0.008856f ? cbrtf(t) : 7.787f * t + 16.f / 116.f; }
DEV void rgb2lab(const float* rgb, float& L, float& A, float& B) {
  float r = srgb_lin(rgb[0]), g = srgb_lin(rgb[1]), b = srgb_lin(rgb[2]);
  float X = (0.412453f * r + 0.357580f * g + 0.180423f * b) / 0.950456f;
  float Y = 0.212671f * r + 0.715160f * g + 0.072169f * b;
  float Z = (0.019334f * r + 0.119193f * g + 0.950227f * b) / 1.088754f;
  float fx = lab_f(X), fy = lab_f(Y), fz = lab_f(Z);
  L = Y > 0.008856f ? 116.f * fy - 16.f : 903.3f * Y;
  A = 500.f * (fx - fy);
  B = 200.f * (fy - fz);
}
DEV void lab2rgb(float L, float A, float B, float* rgb) {
  float Y, fy;
  if (L <= 8.f) { Y = L / 903.3f; fy = 7.787f * Y + 16.f / 116.f; }
  else { fy = (L + 16.f) / 116.f; Y = fy * fy * fy; }
  float fx = A / 500.f + fy, fz = fy - B / 200.f;
  float X = fx > 0.206893f ? fx * fx * fx : (fx - 16.f / 116.f) / 7.787f;
  float Z = fz > 0.206893f ? fz * fz * fz : (fz - 16.f / 116.f) / 7.787f;
  X *= 0.950456f; Z *= 1.088754f;
  rgb[0] = clamp01(lin_srgb(3.240479f * X - 1.53715f * Y - 0.498535f * Z));
  rgb[1] = clamp01(lin_srgb(-0.969256f * X + 1.875991f * Y + 0.041556f * Z));
  rgb[2] = clamp01(lin_srgb(0.055648f * X - 0.204043f * Y + 1.057311f * Z));
}
DEV int lab_l8(float L) { return min(max((int)rintf(L * (255.f / 100.f)), 0), 255); }
// point-in-polygon, even-odd rule (cv2.fillPoly), at a pixel centre
DEV bool in_poly5(const float* v, float px, float py) {
  bool in = false;
#pragma unroll
  for (int i = 0, j = 4; i < 5; j = i++) {
    float xi = v[2 * i], yi = v[2 * i + 1], xj = v[2 * j], yj = v[2 * j + 1];
    if ((yi > py) != (yj > py) && px < (xj - xi) * (py - yi) / (yj - yi) + xi) in = !in;
  }
  return in;
}
DEV void normalize_store(float* out, long plane, long o, const float* rgb) {
  const double mean[3] = {0.485, 0.456, 0.406}, stdv[3] = {0.229, 0.224, 0.225};
#pragma unroll
  for (int c = 0; c < 3; c++) out[c * plane + o] = (float)(((double)rgb[c] - mean[c]) / stdv[c]);
}
DEV long floor_div(long a, long b) { long q = a / b; return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q; }
}  // namespace

__global__ void augment_sample_kernel(const unsigned char* __restrict__ img, const unsigned char* __restrict__ mask,
                                      AugParams P, int S, float* __restrict__ out_img, float* __restrict__ out_mask) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= S) return;
  const long plane = (long)S * S, o = (long)y * S + x;
  float xo = x + 0.5f, yo = y + 0.5f;
  // distortion group (transforms.py:161-181): remap of the geometric result, BORDER_CONSTANT 0
  bool outside = false;
  if (P.grid) { xo = P.grid[x] + 0.5f; yo = P.grid[S + y] + 0.5f; }
  if (P.elastic) { xo += P.elastic[o]; yo += P.elastic[plane + o]; }
  if (P.grid || P.elastic) outside = xo < -0.5f || yo < -0.5f || xo > S + 0.5f || yo > S + 0.5f;
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
    rgb[c] = outside ? 0.f : acc;
  }
  if (P.raw) {
#pragma unroll
    for (int c = 0; c < 3; c++) out_img[c * plane + o] = rgb[c];
  } else {
    // ColorJitter (fixed order brightness, contrast, saturation, hue), clipped like uint8 images
    jitter(rgb, P.bright, P.contrast, P.sat, P.hue, P.gray_mean);
#pragma unroll
    for (int c = 0; c < 3; c++) {
      float v = rgb[c] * P.mult[c];
      if (P.gauss_std > 0.f) v += P.gauss_std * gauss(P.seed, (unsigned)o, c);
      rgb[c] = clamp01(v);
    }
    normalize_store(out_img, plane, o, rgb);
  }
  if (out_mask) {   // nearest (cv2 INTER_NEAREST on the resize, nearest on the geometric warp)
    int nx = (int)floorf(cx + 0.5f), ny = (int)floorf(cy + 0.5f);
    float m = 0.f;
    int rx = nx - P.pad_w, ry = ny - P.pad_h;
    if (!outside && nx >= 0 && ny >= 0 && nx < S && ny < S && rx >= 0 && ry >= 0 && rx < P.new_w && ry < P.new_h) {
      int sx = min((int)floorf(rx * ((float)P.W0 / P.new_w)), P.W0 - 1);
      int sy = min((int)floorf(ry * ((float)P.H0 / P.new_h)), P.H0 - 1);
      m = mask[(long)sy * P.W0 + sx] * (1.f / 255.f);
    }
    out_mask[o] = m;
  }
}

// ---------------------------------------------------------------- ElasticTransform displacement
// generate_displacement_fields (albumentations 2.0.8, noise_distribution "gaussian", approximate=False):
// standard-normal field per axis, cv2.GaussianBlur(ksize x ksize, sigma, BORDER_REFLECT_101), * alpha
struct ElasticParams {
  float w[33];                // normalised 1-D Gaussian taps (ksize <= 33)
  int ksize;
  float alpha;
  unsigned seed;
};

__global__ void elastic_h_kernel(ElasticParams P, int S, float* __restrict__ tmp) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, c = blockIdx.z;
  if (x >= S) return;
  const int r = P.ksize / 2;
  float acc = 0.f;
  for (int j = -r; j <= r; j++) acc += P.w[j + r] * gauss(P.seed, (unsigned)((long)y * S + reflect101(x + j, S)), 8 + c);
  tmp[((long)c * S + y) * S + x] = acc;
}

__global__ void elastic_v_kernel(ElasticParams P, int S, const float* __restrict__ tmp, float* __restrict__ out) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, c = blockIdx.z;
  if (x >= S) return;
  const int r = P.ksize / 2;
  float acc = 0.f;
  for (int j = -r; j <= r; j++) acc += P.w[j + r] * tmp[((long)c * S + reflect101(y + j, S)) * S + x];
  out[((long)c * S + y) * S + x] = acc * P.alpha;
}

// ---------------------------------------------------------------- CLAHE (cv2.createCLAHE on L of Lab, 8x8 tiles)
__global__ void clahe_hist_kernel(const float* __restrict__ x, int S, int* __restrict__ hist) {
  __shared__ int h[256];
  const int tile = blockIdx.x, tx = tile % 8, ty = tile / 8, T = S / 8;
  h[threadIdx.x] = 0;
  __syncthreads();
  const long plane = (long)S * S;
  for (int i = threadIdx.x; i < T * T; i += blockDim.x) {
    const int px = tx * T + i % T, py = ty * T + i / T;
    const long o = (long)py * S + px;
    float rgb[3] = {x[o], x[plane + o], x[2 * plane + o]}, L, A, B;
    rgb2lab(rgb, L, A, B);
    atomicAdd(&h[lab_l8(L)], 1);
  }
  __syncthreads();
  hist[tile * 256 + threadIdx.x] = h[threadIdx.x];
}

// clip, redistribute and integrate one tile's histogram exactly as cv2's CLAHE_CalcLut_Body
__global__ void clahe_lut_kernel(int* __restrict__ hist, float clip, int S, float* __restrict__ lut) {
  if (threadIdx.x != 0) return;
  int* hh = hist + blockIdx.x * 256;
  const int T = S / 8, area = T * T;
  const int limit = max((int)(clip * area / 256), 1);
  int clipped = 0;
  for (int i = 0; i < 256; i++)
    if (hh[i] > limit) { clipped += hh[i] - limit; hh[i] = limit; }
  const int batch = clipped / 256;
  int residual = clipped - batch * 256;
  for (int i = 0; i < 256; i++) hh[i] += batch;
  if (residual != 0) {
    const int step = max(256 / residual, 1);
    for (int i = 0; i < 256 && residual > 0; i += step, residual--) hh[i]++;
  }
  const float scale = 255.f / area;
  int sum = 0;
  for (int i = 0; i < 256; i++) {
    sum += hh[i];
    lut[blockIdx.x * 256 + i] = fminf(fmaxf(rintf(sum * scale), 0.f), 255.f);
  }
}

__global__ void clahe_apply_kernel(float* __restrict__ x, int S, const float* __restrict__ lut) {
  const int px = blockIdx.x * blockDim.x + threadIdx.x, py = blockIdx.y;
  if (px >= S) return;
  const long plane = (long)S * S, o = (long)py * S + px;
  const int T = S / 8;
  const float inv = 1.f / T;
  float txf = px * inv - 0.5f, tyf = py * inv - 0.5f;
  int tx1 = (int)floorf(txf), ty1 = (int)floorf(tyf);
  const float xa = txf - tx1, ya = tyf - ty1;
  int tx2 = min(tx1 + 1, 7), ty2 = min(ty1 + 1, 7);
  tx1 = max(tx1, 0); ty1 = max(ty1, 0);
  float rgb[3] = {x[o], x[plane + o], x[2 * plane + o]}, L, A, B;
  rgb2lab(rgb, L, A, B);
  const int v = lab_l8(L);
  const float* l1 = lut + (ty1 * 8) * 256;
  const float* l2 = lut + (ty2 * 8) * 256;
  float res = (l1[tx1 * 256 + v] * (1.f - xa) + l1[tx2 * 256 + v] * xa) * (1.f - ya) +
              (l2[tx1 * 256 + v] * (1.f - xa) + l2[tx2 * 256 + v] * xa) * ya;
  const float l8 = fminf(fmaxf(rintf(res), 0.f), 255.f);
  lab2rgb(l8 * (100.f / 255.f), A, B, rgb);
#pragma unroll
  for (int c = 0; c < 3; c++) x[c * plane + o] = rgb[c];
}

// ---------------------------------------------------------------- per-pixel groups
// sum and sum of squares (fp64) of the HLS lightness after the colour group: ISONoise's
// cv2.meanStdDev(hls)[1] (population standard deviation)
__global__ void lightness_stats_kernel(const float* __restrict__ x, SynthParams P, int S, double* __restrict__ st) {
  const int px = blockIdx.x * blockDim.x + threadIdx.x, py = blockIdx.y;
  double a = 0.0, b = 0.0;
  if (px < S) {
    const long plane = (long)S * S, o = (long)py * S + px;
    float rgb[3] = {x[o], x[plane + o], x[2 * plane + o]}, h, l, s;
    colour_group(rgb, P);
    rgb2hls(rgb, h, l, s);
    a = l; b = (double)l * l;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) { a += __shfl_xor(a, off); b += __shfl_xor(b, off); }
  __shared__ double red[2][4];
  const int w = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) { red[0][w] = a; red[1][w] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double sa = 0.0, sb = 0.0;
    for (int i = 0; i < (int)(blockDim.x / 64); i++) { sa += red[0][i]; sb += red[1][i]; }
    atomicAdd(&st[0], sa);
    atomicAdd(&st[1], sb);
  }
}

// colour group (ColorJitter | HueSaturationValue) then noise group (ISONoise | GaussNoise |
// MultiplicativeNoise), per pixel.  in -> out (may alias); normalize: write ImageNet-normalised.
__global__ void synth_pixel_kernel(const float* in, float* out, SynthParams P, int S, const double* __restrict__ st,
                                   int normalize) {
  const int px = blockIdx.x * blockDim.x + threadIdx.x, py = blockIdx.y;
  if (px >= S) return;
  const long plane = (long)S * S, o = (long)py * S + px;
  float rgb[3] = {in[o], in[plane + o], in[2 * plane + o]};
  colour_group(rgb, P);
  if (P.iso_intensity > 0.f) {
    // iso_noise: hue += N(0, color_shift * 360 * intensity); L += Poisson(std_L * intensity * 255) / 255 * (1 - L)
    const double n = (double)S * S, mean = st[0] / n;
    const float sd = (float)sqrt(fmax(st[1] / n - mean * mean, 0.0));
    float h, l, s;
    rgb2hls(rgb, h, l, s);
    h += P.iso_color_shift * 360.f * P.iso_intensity * gauss(P.seed ^ 0x5bd1e995u, (unsigned)o, 0);
    if (h < 0.f) h += 360.f;
    if (h > 360.f) h -= 360.f;
    const int k = poisson(sd * P.iso_intensity * 255.f, uni(P.seed, (unsigned)o, 7));
    l += (k / 255.f) * (1.f - l);
    hls2rgb(h, l, s, rgb);
  }
#pragma unroll
  for (int c = 0; c < 3; c++) {
    float v = rgb[c] * P.mult[c];
    if (P.gauss_std > 0.f) v += P.gauss_std * gauss(P.seed, (unsigned)o, c);
    rgb[c] = clamp01(v);
  }
  if (normalize) {
    normalize_store(out, plane, o, rgb);
  } else {
#pragma unroll
    for (int c = 0; c < 3; c++) out[c * plane + o] = rgb[c];
  }
}

// ---------------------------------------------------------------- ImageCompression (JPEG, 4:2:0)
// IJG Annex K base tables (natural order); scaled per quality inside the kernel.  The DCT matrix and the
// tables are built per workgroup in LDS: a per-lane (divergent) index into a by-value kernel argument
// miscompiled here (the lanes read one lane's element), so no table rides in the kernel arguments.
__constant__ int kJpegBase[2][64] = {
    {16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55, 14, 13, 16, 24, 40, 57, 69, 56,
     14, 17, 22, 29, 51, 87, 80, 62, 18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
     49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99},
    {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99, 24, 26, 56, 99, 99, 99, 99, 99,
     47, 66, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
     99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99}};

// one 8x8 block per workgroup (64 threads): level-shifted samples -> DCT -> quantise -> dequantise ->
// IDCT -> rounded 8-bit samples into the Y [Sp][Sp] / Cb, Cr [Sp/2][Sp/2] planes
__global__ void jpeg_block_kernel(const float* __restrict__ x, int S, int quality, float* __restrict__ yplane,
                                  float* __restrict__ cplane) {
  __shared__ float f[8][8], t[8][8], dm[8][8];
  const int tid = threadIdx.x, i = tid & 7, j = tid >> 3;
  const int Sp = 16 * ((S + 15) / 16), nby = Sp / 8, nbc = Sp / 16;
  const long plane = (long)S * S;
  int b = blockIdx.x, comp, bx, by;
  if (b < nby * nby) { comp = 0; bx = b % nby; by = b / nby; }
  else { b -= nby * nby; comp = 1 + b / (nbc * nbc); b %= nbc * nbc; bx = b % nbc; by = b / nbc; }
  // dm[u][k] = c(u)/2 cos((2k+1) u pi / 16): the orthonormal 8-point DCT-II
  dm[j][i] = (j == 0 ? 0.70710678f : 1.f) * 0.5f * cosf((float)((2 * i + 1) * j) * 0.19634954f);
  const int q = max(quality, 1), qscale = q < 50 ? 5000 / q : 200 - 2 * q;
  const float qv = (float)min(max((kJpegBase[comp == 0 ? 0 : 1][j * 8 + i] * qscale + 50) / 100, 1), 255);
  float sample;
  if (comp == 0) {
    const int px = min(bx * 8 + i, S - 1), py = min(by * 8 + j, S - 1);
    const long o = (long)py * S + px;
    float r = rintf(clamp01(x[o]) * 255.f), g = rintf(clamp01(x[plane + o]) * 255.f), bl = rintf(clamp01(x[2 * plane + o]) * 255.f);
    sample = rintf(0.299f * r + 0.587f * g + 0.114f * bl);
  } else {
    int sum = 0;
    for (int dy = 0; dy < 2; dy++)
      for (int dx = 0; dx < 2; dx++) {
        const int px = min(2 * (bx * 8 + i) + dx, S - 1), py = min(2 * (by * 8 + j) + dy, S - 1);
        const long o = (long)py * S + px;
        float r = rintf(clamp01(x[o]) * 255.f), g = rintf(clamp01(x[plane + o]) * 255.f), bl = rintf(clamp01(x[2 * plane + o]) * 255.f);
        float c = comp == 1 ? -0.168736f * r - 0.331264f * g + 0.5f * bl + 128.f : 0.5f * r - 0.418688f * g - 0.081312f * bl + 128.f;
        sum += (int)fminf(fmaxf(rintf(c), 0.f), 255.f);
      }
    sample = (float)((sum + 2) >> 2);
  }
  f[j][i] = sample - 128.f;
  __syncthreads();
  float a = 0.f;                                      // rows: t[y][u] = sum_x dm[u][x] f[y][x]
#pragma unroll
  for (int k = 0; k < 8; k++) a += dm[i][k] * f[j][k];
  t[j][i] = a;
  __syncthreads();
  a = 0.f;                                            // columns: F[v][u] = sum_y dm[v][y] t[y][u]
#pragma unroll
  for (int k = 0; k < 8; k++) a += dm[j][k] * t[k][i];
  const float F = rintf(a / qv) * qv;
  __syncthreads();
  f[j][i] = F;
  __syncthreads();
  a = 0.f;                                            // inverse columns: t[y][u] = sum_v dm[v][y] F[v][u]
#pragma unroll
  for (int k = 0; k < 8; k++) a += dm[k][j] * f[k][i];
  t[j][i] = a;
  __syncthreads();
  a = 0.f;                                            // inverse rows: g[y][x] = sum_u dm[u][x] t[y][u]
#pragma unroll
  for (int k = 0; k < 8; k++) a += dm[k][i] * t[j][k];
  const float v = fminf(fmaxf(rintf(a + 128.f), 0.f), 255.f);
  if (comp == 0) yplane[(long)(by * 8 + j) * Sp + bx * 8 + i] = v;
  else cplane[(long)(comp - 1) * (Sp / 2) * (Sp / 2) + (long)(by * 8 + j) * (Sp / 2) + bx * 8 + i] = v;
}

// decoder side: h2v2 "fancy" (triangle) chroma upsampling, YCbCr -> RGB, 8-bit rounding, back to [0, 1]
__global__ void jpeg_rgb_kernel(const float* __restrict__ yplane, const float* __restrict__ cplane, int S,
                                float* __restrict__ x) {
  const int px = blockIdx.x * blockDim.x + threadIdx.x, py = blockIdx.y;
  if (px >= S) return;
  const int Sp = 16 * ((S + 15) / 16), Sc = Sp / 2, Wc = (S + 1) / 2;
  const long plane = (long)S * S, o = (long)py * S + px;
  const int nx = px >> 1, ny = py >> 1;
  const int fx = min(max((px & 1) ? nx + 1 : nx - 1, 0), Wc - 1), fy = min(max((py & 1) ? ny + 1 : ny - 1, 0), Wc - 1);
  float cc[2];
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const float* c = cplane + (long)k * Sc * Sc;
    const int s = 9 * (int)c[ny * Sc + nx] + 3 * (int)c[ny * Sc + fx] + 3 * (int)c[fy * Sc + nx] + (int)c[fy * Sc + fx];
    cc[k] = (float)((s + 8) >> 4) - 128.f;
  }
  const float Y = yplane[(long)py * Sp + px];
  float rgb[3] = {Y + 1.402f * cc[1], Y - 0.344136f * cc[0] - 0.714136f * cc[1], Y + 1.772f * cc[0]};
#pragma unroll
  for (int c = 0; c < 3; c++) x[c * plane + o] = fminf(fmaxf(rintf(rgb[c]), 0.f), 255.f) * (1.f / 255.f);
}

// ---------------------------------------------------------------- filter pass
namespace {
// value of integer pixel q after Downscale (nearest down, nearest up) and the lighting group
// (RandomShadow polygons | RandomBrightnessContrast), channel c
DEV float lit(const float* __restrict__ x, const SynthParams& P, int S, int Sd, int qx, int qy, int c) {
  int sx = qx, sy = qy;
  if (P.down < 1.f) {
    const int dxs = min((int)(qx * (float)Sd / S), Sd - 1), dys = min((int)(qy * (float)Sd / S), Sd - 1);
    sx = min((int)((dxs + 0.5f) * S / Sd), S - 1); sy = min((int)((dys + 0.5f) * S / Sd), S - 1);
  }
  float v = x[(long)c * S * S + (long)sy * S + sx];
  v = clamp01(v * P.rbc_alpha + P.rbc_beta);
  for (int t = 0; t < P.n_shadow; t++)
    if (in_poly5(P.shadow[t], qx + 0.5f, qy + 0.5f)) v = clamp01(v * P.shadow_dim);
  return v;
}
// blur-group input at integer pixel q: the lit value, or ZoomBlur's (img + sum_k zoom_k(img)) / (n + 1)
DEV float blur_in(const float* __restrict__ x, const SynthParams& P, int S, int Sd, int qx, int qy, int c) {
  const float v = lit(x, P, S, Sd, qx, qy, c);
  if (P.zoom_n == 0) return v;
  float acc = v;
  for (int k = 0; k < P.zoom_n; k++) {
    const int zs = (int)(S * P.zoom[k]), off = (zs - S) / 2;
    const float sc = (float)S / (float)zs;
    float fx = (qx + off + 0.5f) * sc - 0.5f, fy = (qy + off + 0.5f) * sc - 0.5f;
    int x0 = (int)floorf(fx), y0 = (int)floorf(fy);
    float ax = fx - x0, ay = fy - y0;
    if (x0 < 0) { x0 = 0; ax = 0.f; }
    if (x0 >= S - 1) { x0 = S - 1; ax = 0.f; }
    if (y0 < 0) { y0 = 0; ay = 0.f; }
    if (y0 >= S - 1) { y0 = S - 1; ay = 0.f; }
    const int x1 = min(x0 + 1, S - 1), y1 = min(y0 + 1, S - 1);
    acc += (lit(x, P, S, Sd, x0, y0, c) * (1.f - ax) + lit(x, P, S, Sd, x1, y0, c) * ax) * (1.f - ay) +
           (lit(x, P, S, Sd, x0, y1, c) * (1.f - ax) + lit(x, P, S, Sd, x1, y1, c) * ax) * ay;
  }
  return acc / (P.zoom_n + 1);
}
}  // namespace

// out = [Normalize](snow(posterize(colour_op(clip(sum_t w_t * blur_in(p + t)))))) with the composed
// ksize x ksize filter (GaussianBlur | MotionBlur | Defocus, then Sharpen | Emboss: both linear, so they
// compose into one kernel; BORDER_REFLECT_101).  normalize = 0 writes raw [0, 1] RGB (rain / regular chain).
__global__ void synth_filter_kernel(const float* __restrict__ x, const float* __restrict__ kw, SynthParams P, int S,
                                    float* __restrict__ out, int normalize) {
  const int px = blockIdx.x * blockDim.x + threadIdx.x, py = blockIdx.y;
  if (px >= S) return;
  const long plane = (long)S * S, o = (long)py * S + px;
  const int r = P.ksize / 2;
  const int Sd = max(1, (int)(S * P.down));
  float rgb[3] = {0.f, 0.f, 0.f};
  for (int dy = -r; dy <= r; dy++) {
    const int yy = reflect101(py + dy, S);
    for (int dx = -r; dx <= r; dx++) {
      const int xx = reflect101(px + dx, S);
      const float w = kw ? kw[(dy + r) * P.ksize + (dx + r)] : 1.f;
#pragma unroll
      for (int c = 0; c < 3; c++) rgb[c] += w * blur_in(x, P, S, Sd, xx, yy, c);
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
  if (P.snow_point > 0.f) {       // add_snow_bleach: HLS lightness below the snow point * brightness_coeff
    float h, l, s;
    rgb2hls(rgb, h, l, s);
    const float thr = P.snow_point * 0.5f + 1.f / 3.f;
    if (l < thr) { l = fminf(l * P.snow_coeff, 1.f); hls2rgb(h, l, s, rgb); }
  }
  if (normalize) {
    normalize_store(out, plane, o, rgb);
  } else {
#pragma unroll
    for (int c = 0; c < 3; c++) out[c * plane + o] = rgb[c];
  }
}

// ---------------------------------------------------------------- RandomRain ("default")
// add_rain: cv2.line(drop start, start + (slant, drop_length), drop_color, 1) for every drop.  The line is
// rasterised with round-half-up DDA steps (max(|slant|, length) + 1 points, 8-connected like LINE_8).
__global__ void rain_lines_kernel(float* __restrict__ x, SynthParams P, int S) {
  const int n = max(abs(P.rain_slant), P.rain_len);
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)P.rain_n * (n + 1)) return;
  const int d = (int)(t / (n + 1)), i = (int)(t % (n + 1));
  const int x0 = P.rain_drops[2 * d], y0 = P.rain_drops[2 * d + 1];
  const int px = x0 + (int)floor_div(2L * i * P.rain_slant + n, 2L * n);
  const int py = y0 + (int)floor_div(2L * i * P.rain_len + n, 2L * n);
  if (px < 0 || py < 0 || px >= S || py >= S) return;
  const long plane = (long)S * S, o = (long)py * S + px;
#pragma unroll
  for (int c = 0; c < 3; c++) x[c * plane + o] = P.rain_color;
}

// cv2.blur(rain_blur x rain_blur, BORDER_REFLECT_101), HSV V * brightness_coefficient (= RGB * coeff), Normalize
__global__ void rain_final_kernel(const float* __restrict__ x, SynthParams P, int S, float* __restrict__ out) {
  const int px = blockIdx.x * blockDim.x + threadIdx.x, py = blockIdx.y;
  if (px >= S) return;
  const long plane = (long)S * S, o = (long)py * S + px;
  const int r = P.rain_blur / 2;
  float rgb[3] = {0.f, 0.f, 0.f};
  for (int dy = -r; dy <= r; dy++) {
    const long row = (long)reflect101(py + dy, S) * S;
    for (int dx = -r; dx <= r; dx++) {
      const long q = row + reflect101(px + dx, S);
#pragma unroll
      for (int c = 0; c < 3; c++) rgb[c] += x[c * plane + q];
    }
  }
  const float k = P.rain_bright / (float)(P.rain_blur * P.rain_blur);
#pragma unroll
  for (int c = 0; c < 3; c++) rgb[c] = clamp01(rgb[c] * k);
  normalize_store(out, plane, o, rgb);
}

extern "C" {

// raw: fp32 [3][S][S] in [0,1] from s3od_augment_sample with AugParams.raw = 1 (overwritten: scratch);
// params: host SynthParams (order 0: the synthetic chain; order 1: the regular chain's Sharpen / ISONoise
// draws); kw: device fp32 [ksize][ksize] filter (nullable when ksize == 1); out: fp32 [3][S][S]
// ImageNet-normalised.  params.ws: device workspace of s3od_augment_ws_floats(S) floats, required for
// CLAHE, ISONoise, ImageCompression, RandomRain and order 1.
int s3od_augment_synthetic(float* raw, const void* params, const float* kw, int S, float* out, void* stream) {
  const SynthParams P = *(const SynthParams*)params;
  S3OD_REQUIRE(P.ksize >= 1 && P.ksize <= 15 && (P.ksize & 1), "augment_synthetic: ksize must be odd, 1..15");
  S3OD_REQUIRE(P.ksize == 1 || kw != nullptr, "augment_synthetic: filter weights missing");
  S3OD_REQUIRE(P.n_shadow >= 0 && P.n_shadow <= 3 && P.post_bits >= 1 && P.post_bits <= 8 && P.down > 0.f && P.down <= 1.f &&
               P.zoom_n >= 0 && P.zoom_n <= 4 && P.order >= 0 && P.order <= 1, "augment_synthetic: bad parameters");
  const bool need_ws = P.clahe_clip > 0.f || P.iso_intensity > 0.f || P.jpeg_quality > 0 || P.rain_n > 0 || P.order == 1;
  S3OD_REQUIRE(!need_ws || P.ws != nullptr, "augment_synthetic: workspace required for CLAHE / ISONoise / JPEG / rain / order 1");
  S3OD_REQUIRE(P.clahe_clip <= 0.f || S % 8 == 0, "augment_synthetic: CLAHE needs S divisible by its 8x8 tile grid");
  S3OD_REQUIRE(P.jpeg_quality >= 0 && P.jpeg_quality <= 100, "augment_synthetic: jpeg quality out of range");
  S3OD_REQUIRE(P.rain_n == 0 || (P.rain_drops != nullptr && P.rain_blur >= 1 && (P.rain_blur & 1) &&
                                  max(abs(P.rain_slant), P.rain_len) > 0), "augment_synthetic: bad rain parameters");
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid(cdiv(S, 256), S), blk(256);
  float* ws = P.ws;
  double* stats = ws ? (double*)(ws + ws_stats(S)) : nullptr;
  const float* kwp = P.ksize > 1 ? kw : nullptr;
  if (P.order == 1) {
    // regular chain: (ColorJitter | Sharpen) -> (GaussNoise | ISONoise | MultiplicativeNoise) -> Normalize
    float* scratch = ws;
    const float* src = raw;
    if (kwp) {
      SynthParams F = P;
      F.rbc_alpha = 1.f; F.rbc_beta = 0.f; F.n_shadow = 0; F.zoom_n = 0; F.color_op = 0; F.post_bits = 8; F.snow_point = 0.f;
      F.down = 1.f;
      hipLaunchKernelGGL(synth_filter_kernel, grid, blk, 0, st, raw, kwp, F, S, scratch, 0);
      src = scratch;
    }
    if (P.iso_intensity > 0.f) {
      (void)hipMemsetAsync(stats, 0, 2 * sizeof(double), st);
      hipLaunchKernelGGL(lightness_stats_kernel, grid, blk, 0, st, src, P, S, stats);
    }
    hipLaunchKernelGGL(synth_pixel_kernel, grid, blk, 0, st, src, out, P, S, (const double*)stats, 1);
    return s3od_check_launch("augment_synthetic (regular chain)");
  }
  if (P.clahe_clip > 0.f) {
    int* hist = (int*)(ws + ws_hist(S));
    float* lut = ws + ws_lut(S);
    hipLaunchKernelGGL(clahe_hist_kernel, dim3(64), dim3(256), 0, st, raw, S, hist);
    hipLaunchKernelGGL(clahe_lut_kernel, dim3(64), dim3(64), 0, st, hist, P.clahe_clip, S, lut);
    hipLaunchKernelGGL(clahe_apply_kernel, grid, blk, 0, st, raw, S, lut);
  }
  if (P.iso_intensity > 0.f) {
    (void)hipMemsetAsync(stats, 0, 2 * sizeof(double), st);
    hipLaunchKernelGGL(lightness_stats_kernel, grid, blk, 0, st, raw, P, S, stats);
  }
  hipLaunchKernelGGL(synth_pixel_kernel, grid, blk, 0, st, raw, raw, P, S, (const double*)stats, 0);
  if (P.jpeg_quality > 0) {
    // image_compression: cv2.imencode(".jpg", quality) + imdecode (standard tables, 4:2:0)
    const int Sp = (int)ws_sp(S);
    float* yp = ws + ws_jpeg_y(S);
    float* cp = ws + ws_jpeg_c(S);
    const int nblk = (Sp / 8) * (Sp / 8) + 2 * (Sp / 16) * (Sp / 16);
    hipLaunchKernelGGL(jpeg_block_kernel, dim3(nblk), dim3(64), 0, st, raw, S, P.jpeg_quality, yp, cp);
    hipLaunchKernelGGL(jpeg_rgb_kernel, grid, blk, 0, st, yp, cp, S, raw);
  }
  if (P.rain_n > 0) {
    float* scratch = ws;
    hipLaunchKernelGGL(synth_filter_kernel, grid, blk, 0, st, raw, kwp, P, S, scratch, 0);
    const long pts = (long)P.rain_n * (max(abs(P.rain_slant), P.rain_len) + 1);
    hipLaunchKernelGGL(rain_lines_kernel, dim3(cdiv(pts, 256)), blk, 0, st, scratch, P, S);
    hipLaunchKernelGGL(rain_final_kernel, grid, blk, 0, st, scratch, P, S, out);
  } else {
    hipLaunchKernelGGL(synth_filter_kernel, grid, blk, 0, st, raw, kwp, P, S, out, 1);
  }
  return s3od_check_launch("augment_synthetic");
}

// ElasticTransform displacement field: params = host ElasticParams; tmp, out: fp32 [2][S][S] (dx, dy)
int s3od_elastic_field(const void* params, int S, float* tmp, float* out, void* stream) {
  const ElasticParams P = *(const ElasticParams*)params;
  S3OD_REQUIRE(P.ksize >= 1 && P.ksize <= 33 && (P.ksize & 1), "elastic_field: ksize must be odd, 1..33");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(elastic_h_kernel, dim3(cdiv(S, 256), S, 2), dim3(256), 0, st, P, S, tmp);
  hipLaunchKernelGGL(elastic_v_kernel, dim3(cdiv(S, 256), S, 2), dim3(256), 0, st, P, S, tmp, out);
  return s3od_check_launch("elastic_field");
}

// scratch size (floats) of s3od_augment_synthetic's params.ws for canvas size S, written to *out
int s3od_augment_ws_floats(int S, long* out) {
  S3OD_REQUIRE(S > 0 && out != nullptr, "augment_ws_floats: bad arguments");
  *out = ws_floats(S);
  return 0;
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
