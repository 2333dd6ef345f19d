// Multi-mask segmentation loss (synth_sod/src/synth_sod/model_training/loss.py:79-275) fused:
//   pass 1  per-(b,m) sums over pixels (wavefront shuffles -> block -> fp64 atomics)
//   pass 2  one block: soft IoU (squares form, :155-164), argmax best mask, component losses
//           (best + lambda*all, :190-233), aux MSE(sigmoid(pred_iou), ious) (:265-272)
//   pass 3  per-pixel gradient w.r.t. the mask logits (and pred_iou gradient)
// Components: 0 focal (on sigmoid(logits): the reference's double sigmoid, loss.py:18,126-143),
//             1 IoU (:79-99), 2 BCE (torch.nn.BCELoss on sigmoid), 3 SSIM (:34-76, 11x11 Gaussian
//             sigma 1.5, zero padding): its per-map sum of the SSIM map comes from ssim_fwd_kernel and
//             its pixel gradient is added by ssim_grad_kernel (separable Gaussian filters in LDS).
#include "common.hpp"

namespace {
constexpr int NS = 8;   // sums: pt, p, t, p2, t2, focal, bce, ssim-map sum

DEV float sigm(float x) { return 1.f / (1.f + __expf(-x)); }
// binary_cross_entropy_with_logits(z, t), z = p in (0,1)
DEV float bce_logits(float z, float t) { return fmaxf(z, 0.f) - z * t + log1pf(__expf(-fabsf(z))); }
DEV float bce_prob(float p, float t) {   // torch BCELoss: logs clamped at -100
  float lp = fmaxf(logf(p), -100.f), l1p = fmaxf(logf(1.f - p), -100.f);
  return -(t * lp + (1.f - t) * l1p);
}
}  // namespace

__global__ void __launch_bounds__(256) loss_sums_kernel(const float* __restrict__ logits, const float* __restrict__ tgt,
                                                        double* __restrict__ sums, int M, long HW, int pix_per_block,
                                                        float alpha, float gamma) {
  const int bm = blockIdx.y, b = bm / M;
  const float* x = logits + (long)bm * HW;
  const float* t = tgt + (long)b * HW;
  long p0 = (long)blockIdx.x * pix_per_block, p1 = min(HW, p0 + pix_per_block);
  float s[NS] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (long i = p0 + threadIdx.x; i < p1; i += blockDim.x) {
    float p = sigm(x[i]), tt = t[i];
    s[0] += p * tt; s[1] += p; s[2] += tt; s[3] += p * p; s[4] += tt * tt;
    float L = bce_logits(p, tt);
    float pt = __expf(-L);
    float om = 1.f - pt;
    s[5] += alpha * (gamma == 2.f ? om * om : powf(om, gamma)) * L;
    s[6] += bce_prob(p, tt);
  }
  __shared__ float red[4][NS];
#pragma unroll
  for (int k = 0; k < NS; k++) {
    float v = warp_sum(s[k]);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < NS) {
    float v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    atomicAdd(sums + (long)bm * NS + threadIdx.x, (double)v);
  }
}

// out layout (floats): [0] total, [1] best_iou, [2] gt_ious mean, [3] mse,
//   [4 + 2c] comp c best, [5 + 2c] comp c full-mean   (c = 0..3 for focal, iou, bce, ssim)
//   [16 ..) ious [B*M], then best idx (as float) [B]
// coef: [B*M][4] = d total / d all_c[b,m] for c = focal, iou, bce, ssim ; and IoU-loss (I+s, U+s)
__global__ void loss_finalize_kernel(const double* sums, const float* pred_iou, int B, int M, long HW, float w_focal, float w_iou,
                                     float w_bce, float w_ssim, float w_mse, float lam, float* out, float* coef, float* iou_ws,
                                     float* d_iou_unit) {
  if (threadIdx.x != 0) return;
  const float sm = 1e-6f;
  float tot = 0.f, best_iou_sum = 0.f, gt_sum = 0.f, mse = 0.f;
  float cb[4] = {0, 0, 0, 0}, cf[4] = {0, 0, 0, 0};
  float* ious = out + 16;
  float* bestf = out + 16 + B * M;
  for (int b = 0; b < B; b++) {
    int best = 0; float bi = -1e30f;
    for (int m = 0; m < M; m++) {
      const double* s = sums + (long)(b * M + m) * NS;
      float inter = (float)s[0], p2 = (float)s[3], t2 = (float)s[4];
      float iou = (inter + sm) / (t2 + p2 - inter + sm);
      ious[b * M + m] = iou;
      gt_sum += iou;
      if (iou > bi) { bi = iou; best = m; }   // first max wins, like torch.argmax
    }
    bestf[b] = (float)best;
    best_iou_sum += bi;
    for (int m = 0; m < M; m++) {
      const double* s = sums + (long)(b * M + m) * NS;
      float I = (float)s[0], Ps = (float)s[1], Ts = (float)s[2];
      float U = Ps + Ts - I;
      float vals[4] = {(float)(s[5] / (double)HW), 1.f - (I + sm) / (U + sm), (float)(s[6] / (double)HW),
                       1.f - (float)(s[7] / (double)HW)};
      for (int c = 0; c < 4; c++) {
        if (m == best) cb[c] += vals[c];
        cf[c] += vals[c];
      }
      float k = (m == best ? 1.f / B : 0.f) + lam / (float)(B * M);
      coef[(b * M + m) * 4 + 0] = w_focal * k;
      coef[(b * M + m) * 4 + 1] = w_iou * k;
      coef[(b * M + m) * 4 + 2] = w_bce * k;
      coef[(b * M + m) * 4 + 3] = w_ssim * k;
      iou_ws[(b * M + m) * 2 + 0] = I + sm;
      iou_ws[(b * M + m) * 2 + 1] = U + sm;
      float sp = 1.f / (1.f + expf(-pred_iou[b * M + m]));
      float d = sp - ious[b * M + m];
      mse += d * d;
      d_iou_unit[b * M + m] = w_mse * 2.f * d / (float)(B * M) * sp * (1.f - sp);
    }
  }
  mse /= (float)(B * M);
  float ws[4] = {w_focal, w_iou, w_bce, w_ssim};
  for (int c = 0; c < 4; c++) {
    out[4 + 2 * c] = cb[c] / (float)B;
    out[5 + 2 * c] = cf[c] / (float)(B * M);
    tot += ws[c] * (out[4 + 2 * c] + lam * out[5 + 2 * c]);
  }
  tot += w_mse * mse;
  out[0] = tot; out[1] = best_iou_sum / (float)B; out[2] = gt_sum / (float)(B * M); out[3] = mse;
}

__global__ void loss_grad_kernel(const float* __restrict__ logits, const float* __restrict__ tgt, const float* __restrict__ coef,
                                 const float* __restrict__ iou_ws, const float* __restrict__ gscale, float* __restrict__ dlogits,
                                 int M, long HW, float alpha, float gamma) {
  const int bm = blockIdx.y, b = bm / M;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= HW) return;
  const float g = gscale ? *gscale : 1.f;
  const float cfoc = coef[bm * 4 + 0] / (float)HW, ciou = coef[bm * 4 + 1], cbce = coef[bm * 4 + 2] / (float)HW;
  const float Is = iou_ws[bm * 2 + 0], Us = iou_ws[bm * 2 + 1];
  float x = logits[(long)bm * HW + i], t = tgt[(long)b * HW + i];
  float p = sigm(x);
  float dp = 0.f;
  if (cfoc != 0.f) {
    float L = bce_logits(p, t), e = __expf(-L), om = 1.f - e;
    float dfdL = gamma == 2.f ? alpha * (2.f * om * e * L + om * om) : alpha * (gamma * powf(om, gamma - 1.f) * e * L + powf(om, gamma));
    dp += cfoc * dfdL * (sigm(p) - t);
  }
  if (ciou != 0.f) dp += ciou * -(t * Us - Is * (1.f - t)) / (Us * Us);
  if (cbce != 0.f) dp += cbce * (p - t) / fmaxf(p * (1.f - p), 1e-12f);
  dlogits[(long)bm * HW + i] = g * dp * p * (1.f - p);
}

__global__ void loss_iou_grad_kernel(const float* d_iou_unit, const float* gscale, float* d_iou, int n) {
  int i = threadIdx.x;
  if (i < n) d_iou[i] = (gscale ? *gscale : 1.f) * d_iou_unit[i];
}


// ------------------------------------------------------------------ SSIM (loss.py:34-76)
// ssim_map = ((2 mu1 mu2 + C1)(2 s12 + C2)) / ((mu1^2 + mu2^2 + C1)(s1 + s2 + C2)) with mu = G*x,
// s1 = G*(p^2) - mu1^2, s2 = G*(t^2) - mu2^2, s12 = G*(pt) - mu1 mu2 and G the normalised 11x11
// Gaussian (sigma 1.5) applied with zero padding; the loss of a map is 1 - mean(ssim_map).
// G is separable (outer product of the 1-D window), so each 2-D filter is a row pass then a
// column pass over an LDS tile with a halo.
struct Gauss11 { float g[11]; };
constexpr float SSIM_C1 = 0.01f * 0.01f, SSIM_C2 = 0.03f * 0.03f;
constexpr int ST = 32;                     // output tile edge

// the five filtered maps at one pixel -> ssim value and d ssim / d (mu1, e11, e12)
DEV float ssim_px(float mu1, float mu2, float e11, float e22, float e12, float* dmu1, float* de11, float* de12) {
  float m11 = mu1 * mu1, m22 = mu2 * mu2, m12 = mu1 * mu2;
  float A1 = 2.f * m12 + SSIM_C1, A2 = 2.f * (e12 - m12) + SSIM_C2;
  float B1 = m11 + m22 + SSIM_C1, B2 = (e11 - m11) + (e22 - m22) + SSIM_C2;
  float den = B1 * B2, m = A1 * A2 / den;
  if (dmu1) {
    *dmu1 = (2.f * mu2 * A2 - 2.f * mu2 * A1) / den - m * (2.f * mu1 / B1 - 2.f * mu1 / B2);
    *de11 = -m / B2;
    *de12 = 2.f * A1 / den;
  }
  return m;
}

// per (b,m) map: sums[bm*NS + 7] += sum over the tile of ssim_map(p = sigmoid(logits), t)
__global__ void __launch_bounds__(256) ssim_fwd_kernel(const float* __restrict__ logits, const float* __restrict__ tgt,
                                                       double* __restrict__ sums, int M, int H, int W, Gauss11 G) {
  constexpr int R = 5, E = ST + 2 * R;                     // 42
  __shared__ float xp[E][E], xt[E][E];
  __shared__ float hm[5][E][ST];                            // row-filtered p, t, pp, tt, pt
  const int bm = blockIdx.z, b = bm / M, tid = threadIdx.x;
  const int y0 = blockIdx.y * ST - R, x0 = blockIdx.x * ST - R;
  const float* lg = logits + (long)bm * H * W;
  const float* tg = tgt + (long)b * H * W;
  for (int i = tid; i < E * E; i += 256) {
    int r = i / E, c = i - r * E, y = y0 + r, x = x0 + c;
    bool in = (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
    xp[r][c] = in ? 1.f / (1.f + __expf(-lg[(long)y * W + x])) : 0.f;
    xt[r][c] = in ? tg[(long)y * W + x] : 0.f;
  }
  __syncthreads();
  for (int i = tid; i < E * ST; i += 256) {
    int r = i / ST, c = i - r * ST;
    float a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0;
#pragma unroll
    for (int k = 0; k < 11; k++) {
      float p = xp[r][c + k], t = xt[r][c + k], g = G.g[k];
      a0 += g * p; a1 += g * t; a2 += g * (p * p); a3 += g * (t * t); a4 += g * (p * t);
    }
    hm[0][r][c] = a0; hm[1][r][c] = a1; hm[2][r][c] = a2; hm[3][r][c] = a3; hm[4][r][c] = a4;
  }
  __syncthreads();
  float acc = 0.f;
  for (int i = tid; i < ST * ST; i += 256) {
    int r = i / ST, c = i - r * ST, y = y0 + R + r, x = x0 + R + c;
    if (y >= H || x >= W) continue;
    float v[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 11; k++) {
      float g = G.g[k];
#pragma unroll
      for (int q = 0; q < 5; q++) v[q] += g * hm[q][r + k][c];
    }
    acc += ssim_px(v[0], v[1], v[2], v[3], v[4], nullptr, nullptr, nullptr);
  }
  __shared__ float red[4];
  acc = warp_sum(acc);
  if ((tid & 63) == 0) red[tid >> 6] = acc;
  __syncthreads();
  if (tid == 0) atomicAdd(sums + (long)bm * NS + 7, (double)(red[0] + red[1] + red[2] + red[3]));
}

// dlogits += g * coef_ssim * d(1 - mean ssim_map)/dp * p(1-p):
//   d/dp(x) = -(1/HW) [ (G*Dmu1)(x) + 2 p(x) (G*De11)(x) + t(x) (G*De12)(x) ]
// with D* = d ssim_map / d(mu1, e11, e12) on image pixels (0 outside); G is symmetric, so the
// adjoint of the zero-padded filter is the same zero-padded filter.  Tile + halo 10 in LDS.
__global__ void __launch_bounds__(256) ssim_grad_kernel(const float* __restrict__ logits, const float* __restrict__ tgt,
                                                        const float* __restrict__ coef, const float* __restrict__ gscale,
                                                        float* __restrict__ dlogits, int M, int H, int W, Gauss11 G) {
  constexpr int R = 5, E1 = ST + 4 * R, E2 = ST + 2 * R;    // 52, 42
  extern __shared__ float sm[];
  float* xp = sm;                                           // [E1][E1]
  float* xt = xp + E1 * E1;                                 // [E1][E1]
  float* h1 = xt + E1 * E1;                                 // [5][E1][E2] row-filtered inputs
  float* dm = h1 + 5 * E1 * E2;                             // [3][E2][E2] D maps
  float* h2 = h1;                                           // [3][E2][ST] row-filtered D maps (reuses h1)
  const int bm = blockIdx.z, b = bm / M, tid = threadIdx.x;
  const float cs = coef[bm * 4 + 3];
  if (cs == 0.f) return;
  const long HW = (long)H * W;
  const int ty = blockIdx.y * ST, tx = blockIdx.x * ST;
  const int y1 = ty - 2 * R, x1 = tx - 2 * R;               // origin of the input halo
  const float* lg = logits + (long)bm * HW;
  const float* tg = tgt + (long)b * HW;
  for (int i = tid; i < E1 * E1; i += 256) {
    int r = i / E1, c = i - r * E1, y = y1 + r, x = x1 + c;
    bool in = (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
    xp[i] = in ? 1.f / (1.f + __expf(-lg[(long)y * W + x])) : 0.f;
    xt[i] = in ? tg[(long)y * W + x] : 0.f;
  }
  __syncthreads();
  for (int i = tid; i < E1 * E2; i += 256) {                // rows of the halo, columns of the D region
    int r = i / E2, c = i - r * E2;
    float a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0;
#pragma unroll
    for (int k = 0; k < 11; k++) {
      float p = xp[r * E1 + c + k], t = xt[r * E1 + c + k], g = G.g[k];
      a0 += g * p; a1 += g * t; a2 += g * (p * p); a3 += g * (t * t); a4 += g * (p * t);
    }
    h1[(0 * E1 + r) * E2 + c] = a0; h1[(1 * E1 + r) * E2 + c] = a1; h1[(2 * E1 + r) * E2 + c] = a2;
    h1[(3 * E1 + r) * E2 + c] = a3; h1[(4 * E1 + r) * E2 + c] = a4;
  }
  __syncthreads();
  for (int i = tid; i < E2 * E2; i += 256) {                // D maps on the tile + halo 5
    int r = i / E2, c = i - r * E2, y = ty - R + r, x = tx - R + c;
    float d0 = 0.f, d1 = 0.f, d2 = 0.f;
    if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) {
      float v[5] = {0, 0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < 11; k++) {
        float g = G.g[k];
#pragma unroll
        for (int q = 0; q < 5; q++) v[q] += g * h1[(q * E1 + r + k) * E2 + c];
      }
      ssim_px(v[0], v[1], v[2], v[3], v[4], &d0, &d1, &d2);
    }
    dm[(0 * E2 + r) * E2 + c] = d0; dm[(1 * E2 + r) * E2 + c] = d1; dm[(2 * E2 + r) * E2 + c] = d2;
  }
  __syncthreads();
  for (int i = tid; i < E2 * ST; i += 256) {
    int r = i / ST, c = i - r * ST;
    float a0 = 0, a1 = 0, a2 = 0;
#pragma unroll
    for (int k = 0; k < 11; k++) {
      float g = G.g[k];
      a0 += g * dm[(0 * E2 + r) * E2 + c + k]; a1 += g * dm[(1 * E2 + r) * E2 + c + k]; a2 += g * dm[(2 * E2 + r) * E2 + c + k];
    }
    h2[(0 * E2 + r) * ST + c] = a0; h2[(1 * E2 + r) * ST + c] = a1; h2[(2 * E2 + r) * ST + c] = a2;
  }
  __syncthreads();
  const float gs = (gscale ? *gscale : 1.f) * cs * (-1.f / (float)HW);
  for (int i = tid; i < ST * ST; i += 256) {
    int r = i / ST, c = i - r * ST, y = ty + r, x = tx + c;
    if (y >= H || x >= W) continue;
    float a0 = 0, a1 = 0, a2 = 0;
#pragma unroll
    for (int k = 0; k < 11; k++) {
      float g = G.g[k];
      a0 += g * h2[(0 * E2 + r + k) * ST + c]; a1 += g * h2[(1 * E2 + r + k) * ST + c]; a2 += g * h2[(2 * E2 + r + k) * ST + c];
    }
    float p = xp[(r + 2 * R) * E1 + c + 2 * R], t = xt[(r + 2 * R) * E1 + c + 2 * R];
    float dp = a0 + 2.f * p * a1 + t * a2;
    dlogits[(long)bm * HW + (long)y * W + x] += gs * dp * p * (1.f - p);
  }
}

static Gauss11 gauss11() {
  // torch: Tensor([exp(-(x - 5)^2 / (2 sigma^2)) for x]) (float64 -> float32), then / sum in float32
  Gauss11 G; float s = 0.f;
  for (int k = 0; k < 11; k++) { G.g[k] = (float)exp(-(double)((k - 5) * (k - 5)) / (2.0 * 1.5 * 1.5)); }
  for (int k = 0; k < 11; k++) s += G.g[k];
  for (int k = 0; k < 11; k++) G.g[k] = G.g[k] / s;
  return G;
}
constexpr int SSIM_GRAD_LDS = (2 * 52 * 52 + 5 * 52 * 42 + 3 * 42 * 42) * 4;

extern "C" {

// logits [B,M,H,W] f32, target [B,H,W] f32, pred_iou [B,M] f32.  weights for focal / iou / bce / mse
// (0 disables a component); lam = full_mask_lambda*exp(-decay*epoch).  ws: workspace of
// >= B*M*(8*2 + 4 + 2 + 1) floats (doubles for the sums).  out: >= 16 + B*M + B floats.
// w_ssim > 0 needs the map geometry: H*W == HW (W = image width).
int s3od_mask_loss_fwd(const float* logits, const float* target, const float* pred_iou, int B, int M, long HW, int W,
                       float w_focal, float w_iou, float w_bce, float w_ssim, float w_mse, float lam, float alpha, float gamma,
                       double* sums, float* coef, float* iou_ws, float* d_iou_unit, float* out, void* stream) {
  S3OD_REQUIRE(w_ssim == 0.f || (W > 0 && HW % W == 0), "mask_loss_fwd: SSIM needs the map width (HW=%ld W=%d)", HW, W);
  hipStream_t st = (hipStream_t)stream;
  (void)hipMemsetAsync(sums, 0, sizeof(double) * B * M * NS, st);
  const int ppb = 16384;
  hipLaunchKernelGGL(loss_sums_kernel, dim3(cdiv(HW, ppb), B * M), dim3(256), 0, st, logits, target, sums, M, HW, ppb, alpha, gamma);
  if (w_ssim != 0.f) {
    const int H = (int)(HW / W);
    hipLaunchKernelGGL(ssim_fwd_kernel, dim3(cdiv(W, ST), cdiv(H, ST), B * M), dim3(256), 0, st, logits, target, sums, M, H, W,
                       gauss11());
  }
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(64), 0, st, sums, pred_iou, B, M, HW, w_focal, w_iou, w_bce, w_ssim, w_mse,
                     lam, out, coef, iou_ws, d_iou_unit);
  return s3od_check_launch("mask_loss_fwd");
}

// gscale: device scalar upstream gradient (nullable = 1).  dlogits [B,M,H,W], d_iou [B,M]
// W: map width, needed when the SSIM component is on (w_ssim != 0 in the forward); 0 otherwise.
int s3od_mask_loss_bwd(const float* logits, const float* target, const float* coef, const float* iou_ws, const float* d_iou_unit,
                       const float* gscale, float* dlogits, float* d_iou, int B, int M, long HW, int W, int with_ssim,
                       float alpha, float gamma, void* stream) {
  S3OD_REQUIRE(!with_ssim || (W > 0 && HW % W == 0), "mask_loss_bwd: SSIM needs the map width (HW=%ld W=%d)", HW, W);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(loss_grad_kernel, dim3(cdiv(HW, 256), B * M), dim3(256), 0, st, logits, target, coef, iou_ws, gscale, dlogits,
                     M, HW, alpha, gamma);
  if (with_ssim) {
    static const bool attr = ((void)hipFuncSetAttribute((const void*)ssim_grad_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, SSIM_GRAD_LDS), true);   // once per process (thread-safe static init)
    (void)attr;
    const int H = (int)(HW / W);
    hipLaunchKernelGGL(ssim_grad_kernel, dim3(cdiv(W, ST), cdiv(H, ST), B * M), dim3(256), SSIM_GRAD_LDS, st, logits, target, coef,
                       gscale, dlogits, M, H, W, gauss11());
  }
  hipLaunchKernelGGL(loss_iou_grad_kernel, dim3(1), dim3(64), 0, st, d_iou_unit, gscale, d_iou, B * M);
  return s3od_check_launch("mask_loss_bwd");
}

}  // extern "C"
