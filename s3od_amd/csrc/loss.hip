// Multi-mask segmentation loss (synth_sod/src/synth_sod/model_training/loss.py:79-275) fused:
//   pass 1  per-(b,m) sums over pixels (wavefront shuffles -> block -> fp64 atomics)
//   pass 2  one block: soft IoU (squares form, :155-164), argmax best mask, component losses
//           (best + lambda*all, :190-233), aux MSE(sigmoid(pred_iou), ious) (:265-272)
//   pass 3  per-pixel gradient w.r.t. the mask logits (and pred_iou gradient)
// Components: 0 focal (on sigmoid(logits): the reference's double sigmoid, loss.py:18,126-143),
//             1 IoU (:79-99), 2 BCE (torch.nn.BCELoss on sigmoid).  SSIM is not fused here.
#include "common.hpp"

namespace {
constexpr int NS = 8;   // sums: pt, p, t, p2, t2, focal, bce, spare

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
//   [4 + 2c] comp c best, [5 + 2c] comp c full-mean   (c = 0..2 for focal, iou, bce)
//   [16 ..) ious [B*M], then best idx (as float) [B]
// coef: [B*M][4] = d total / d all_c[b,m] for c = focal, iou, bce ; and IoU-loss (I+s, U+s)
__global__ void loss_finalize_kernel(const double* sums, const float* pred_iou, int B, int M, long HW, float w_focal, float w_iou,
                                     float w_bce, float w_mse, float lam, float* out, float* coef, float* iou_ws, float* d_iou_unit) {
  if (threadIdx.x != 0) return;
  const float sm = 1e-6f;
  float tot = 0.f, best_iou_sum = 0.f, gt_sum = 0.f, mse = 0.f;
  float cb[3] = {0, 0, 0}, cf[3] = {0, 0, 0};
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
      float vals[3] = {(float)(s[5] / (double)HW), 1.f - (I + sm) / (U + sm), (float)(s[6] / (double)HW)};
      for (int c = 0; c < 3; c++) {
        if (m == best) cb[c] += vals[c];
        cf[c] += vals[c];
      }
      float k = (m == best ? 1.f / B : 0.f) + lam / (float)(B * M);
      coef[(b * M + m) * 4 + 0] = w_focal * k;
      coef[(b * M + m) * 4 + 1] = w_iou * k;
      coef[(b * M + m) * 4 + 2] = w_bce * k;
      iou_ws[(b * M + m) * 2 + 0] = I + sm;
      iou_ws[(b * M + m) * 2 + 1] = U + sm;
      float sp = 1.f / (1.f + expf(-pred_iou[b * M + m]));
      float d = sp - ious[b * M + m];
      mse += d * d;
      d_iou_unit[b * M + m] = w_mse * 2.f * d / (float)(B * M) * sp * (1.f - sp);
    }
  }
  mse /= (float)(B * M);
  float ws[3] = {w_focal, w_iou, w_bce};
  for (int c = 0; c < 3; c++) {
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

extern "C" {

// logits [B,M,H,W] f32, target [B,H,W] f32, pred_iou [B,M] f32.  weights for focal / iou / bce / mse
// (0 disables a component); lam = full_mask_lambda*exp(-decay*epoch).  ws: workspace of
// >= B*M*(8*2 + 4 + 2 + 1) floats (doubles for the sums).  out: >= 16 + B*M + B floats.
int s3od_mask_loss_fwd(const float* logits, const float* target, const float* pred_iou, int B, int M, long HW,
                       float w_focal, float w_iou, float w_bce, float w_mse, float lam, float alpha, float gamma,
                       double* sums, float* coef, float* iou_ws, float* d_iou_unit, float* out, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  (void)hipMemsetAsync(sums, 0, sizeof(double) * B * M * NS, st);
  const int ppb = 16384;
  hipLaunchKernelGGL(loss_sums_kernel, dim3(cdiv(HW, ppb), B * M), dim3(256), 0, st, logits, target, sums, M, HW, ppb, alpha, gamma);
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(64), 0, st, sums, pred_iou, B, M, HW, w_focal, w_iou, w_bce, w_mse, lam,
                     out, coef, iou_ws, d_iou_unit);
  return s3od_check_launch("mask_loss_fwd");
}

// gscale: device scalar upstream gradient (nullable = 1).  dlogits [B,M,H,W], d_iou [B,M]
int s3od_mask_loss_bwd(const float* logits, const float* target, const float* coef, const float* iou_ws, const float* d_iou_unit,
                       const float* gscale, float* dlogits, float* d_iou, int B, int M, long HW, float alpha, float gamma, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(loss_grad_kernel, dim3(cdiv(HW, 256), B * M), dim3(256), 0, st, logits, target, coef, iou_ws, gscale, dlogits,
                     M, HW, alpha, gamma);
  hipLaunchKernelGGL(loss_iou_grad_kernel, dim3(1), dim3(64), 0, st, d_iou_unit, gscale, d_iou, B * M);
  return s3od_check_launch("mask_loss_bwd");
}

}  // extern "C"
