// Memory-bound DPT-decoder kernels (NHWC activations): weight repack, BatchNorm fold /
// batch statistics / apply / backward, bilinear resize fwd/bwd, global average pool,
// IoU-score MLP head fwd/bwd, mask-head backward prologue, ReLU masks.
// Reference: src/s3od/model.py:109-467.
#include "common.hpp"

#define DISPATCH_T(dtype, ...)                                                  \
  do {                                                                          \
    if ((dtype) == S3OD_BF16) { typedef bf16 T; __VA_ARGS__ }                   \
    else if ((dtype) == S3OD_F32) { typedef float T; __VA_ARGS__ }              \
    else { s3od_set_error("bad dtype %d", (int)(dtype)); return 22; }           \
  } while (0)

// ---------------------------------------------------------------- weight repack
// src f32 [O][I][KH][KW] (PyTorch conv / conv-view of ConvTranspose) -> dst T [O][KH][KW][I]
template <typename T>
__global__ void repack_kernel(const float* __restrict__ src, T* __restrict__ dst, int O, int I, int KHW) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)O * I * KHW;
  if (idx >= total) return;
  int i = idx % I; long r = idx / I; int t = r % KHW; int o = r / KHW;
  dst[idx] = from_f<T>(src[((long)o * I + i) * KHW + t]);
}

// ConvTranspose2d weight [Cin_T][Cout_T][KH][KW] IS the conv-view weight [cout_c][cin_c][KH][KW]; no flip.

// ---------------------------------------------------------------- BatchNorm
// eval fold: y = (z - rm) * w / sqrt(rv + eps) + b = z*scale + shift  (z = conv + conv bias)
__global__ void bn_fold_kernel(const float* w, const float* b, const float* rm, const float* rv,
                               float eps, float* scale, float* shift, int C) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = w[c] / sqrtf(rv[c] + eps);
  scale[c] = s;
  shift[c] = b[c] - rm[c] * s;
}

// train: stats = (sum, sumsq) over count values of z = conv + bias. Writes mean/rstd (for backward),
// scale/shift (for apply) and updates running stats (momentum, unbiased var) like nn.BatchNorm2d.
__global__ void bn_finalize_kernel(const double* stats, long count, const float* w, const float* b, float* rm, float* rv,
                                   float momentum, float eps, float* mean_o, float* rstd_o, float* scale, float* shift, int C) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double mean = stats[c] / (double)count;
  double var = stats[C + c] / (double)count - mean * mean;
  if (var < 0) var = 0;
  float rstd = (float)(1.0 / sqrt(var + (double)eps));
  mean_o[c] = (float)mean; rstd_o[c] = rstd;
  scale[c] = w[c] * rstd;
  shift[c] = b[c] - (float)mean * w[c] * rstd;
  if (rm) {
    double unb = count > 1 ? var * (double)count / (double)(count - 1) : var;
    rm[c] = (1.f - momentum) * rm[c] + momentum * (float)mean;
    rv[c] = (1.f - momentum) * rv[c] + momentum * (float)unb;
  }
}

// y = act(x*scale[c] + shift[c]) (+res1 +res2); act 0 none / 1 relu.  NHWC, C % 8 == 0
template <typename T>
__global__ void affine_act_kernel(const T* __restrict__ x, const float* __restrict__ scale, const float* __restrict__ shift,
                                  int act, const T* __restrict__ r1, const T* __restrict__ r2, T* __restrict__ y, long total, int C) {
  long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= total) return;
  int c = i % C;
  float v[8], s[8], t[8];
  load8<T>(x + i, v); load8<float>(scale + c, s); load8<float>(shift + c, t);
#pragma unroll
  for (int e = 0; e < 8; e++) { v[e] = v[e] * s[e] + t[e]; if (act == 1) v[e] = fmaxf(v[e], 0.f); }
  if (r1) { float r[8]; load8<T>(r1 + i, r);
#pragma unroll
    for (int e = 0; e < 8; e++) v[e] += r[e]; }
  if (r2) { float r[8]; load8<T>(r2 + i, r);
#pragma unroll
    for (int e = 0; e < 8; e++) v[e] += r[e]; }
  store8<T>(y + i, v);
}

// BN backward, pass 1: per channel sums of dy' and dy'*xhat where dy' = dy (or dy*(y>0) if relu_y)
// xhat = (z - mean)*rstd.  Output double [2][C].
template <typename T>
__global__ void bn_bwd_reduce_kernel(const T* __restrict__ dy, const T* __restrict__ z, const T* __restrict__ y_relu,
                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                     double* __restrict__ sums, long npix, int C, int pix_per_block) {
  // block: 256 threads = (C/8) column groups x rows
  const int cg = C / 8, rows = 256 / cg;
  const int t = threadIdx.x, cgi = t % cg, ri = t / cg;
  if (ri >= rows) return;
  const int c = cgi * 8;
  float mu[8], rs[8];
  load8<float>(mean + c, mu); load8<float>(rstd + c, rs);
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long p0 = (long)blockIdx.x * pix_per_block, p1 = min(npix, p0 + pix_per_block);
#pragma unroll 4
  for (long p = p0 + ri; p < p1; p += rows) {
    float d[8], zz[8];
    load8<T>(dy + p * C + c, d); load8<T>(z + p * C + c, zz);
    if (y_relu) { float yy[8]; load8<T>(y_relu + p * C + c, yy);
#pragma unroll
      for (int e = 0; e < 8; e++) if (!(yy[e] > 0.f)) d[e] = 0.f; }
#pragma unroll
    for (int e = 0; e < 8; e++) { float xh = (zz[e] - mu[e]) * rs[e]; s1[e] += d[e]; s2[e] += d[e] * xh; }
  }
#pragma unroll
  for (int e = 0; e < 8; e++) { atomicAdd(sums + c + e, (double)s1[e]); atomicAdd(sums + C + c + e, (double)s2[e]); }
}

// BN backward, pass 2: dz = w*rstd*(dy' - s1/n - xhat*s2/n); also dw = s2, db = s1 (finalize)
template <typename T>
__global__ void bn_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ z, const T* __restrict__ y_relu,
                                    const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ w,
                                    const double* __restrict__ sums, T* __restrict__ dz, long total, int C, long npix) {
  long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= total) return;
  int c = i % C;
  float d[8], zz[8];
  load8<T>(dy + i, d); load8<T>(z + i, zz);
  if (y_relu) { float yy[8]; load8<T>(y_relu + i, yy);
#pragma unroll
    for (int e = 0; e < 8; e++) if (!(yy[e] > 0.f)) d[e] = 0.f; }
  float o[8];
#pragma unroll
  for (int e = 0; e < 8; e++) {
    int cc = c + e;
    float mu = mean[cc], rs = rstd[cc];
    float m1 = (float)(sums[cc] / (double)npix), m2 = (float)(sums[C + cc] / (double)npix);
    float xh = (zz[e] - mu) * rs;
    o[e] = w[cc] * rs * (d[e] - m1 - xh * m2);
  }
  store8<T>(dz + i, o);
}

__global__ void bn_param_grads_kernel(const double* sums, float* dw, float* db, int C) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  db[c] += (float)sums[c];
  dw[c] += (float)sums[C + c];
}

// ---------------------------------------------------------------- bilinear (align_corners=False)
// PyTorch upsample_bilinear2d: src = max(0, (dst + 0.5)*in/out - 0.5); i0 = floor, i1 = min(i0+1, in-1)
DEV void bil_coef(int o, int in, int out, int& i0, int& i1, float& w0, float& w1) {
  float scale = (float)in / (float)out;
  float src = ((float)o + 0.5f) * scale - 0.5f;
  if (src < 0.f) src = 0.f;
  i0 = (int)src; if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + 1 < in ? i0 + 1 : in - 1;
  w1 = src - (float)i0; w0 = 1.f - w1;
}

template <typename T>
__global__ void bilinear_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int B, int IH, int IW, int OH, int OW, int C) {
  long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  long total = (long)B * OH * OW * C;
  if (i >= total) return;
  int c = i % C; long pix = i / C;
  int ox = pix % OW; long r = pix / OW; int oy = r % OH; int b = r / OH;
  int y0, y1, x0, x1; float wy0, wy1, wx0, wx1;
  bil_coef(oy, IH, OH, y0, y1, wy0, wy1);
  bil_coef(ox, IW, OW, x0, x1, wx0, wx1);
  const T* base = x + (long)b * IH * IW * C + c;
  float a[8], bb[8], cc[8], d[8], o[8];
  load8<T>(base + ((long)y0 * IW + x0) * C, a); load8<T>(base + ((long)y0 * IW + x1) * C, bb);
  load8<T>(base + ((long)y1 * IW + x0) * C, cc); load8<T>(base + ((long)y1 * IW + x1) * C, d);
#pragma unroll
  for (int e = 0; e < 8; e++) o[e] = wy0 * (wx0 * a[e] + wx1 * bb[e]) + wy1 * (wx0 * cc[e] + wx1 * d[e]);
  store8<T>(y + i, o);
}

// gather-form backward: dx[i] = sum over outputs whose (i0 or i1) == i of weight * (dy + bcast[b,c])
template <typename T>
__global__ void bilinear_bwd_kernel(const T* __restrict__ dy, const float* __restrict__ bcast, T* __restrict__ dx,
                                    int B, int IH, int IW, int OH, int OW, int C) {
  long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  long total = (long)B * IH * IW * C;
  if (i >= total) return;
  int c = i % C; long pix = i / C;
  int ix = pix % IW; long r = pix / IW; int iy = r % IH; int b = r / IH;
  // candidate output ranges: src in [i-1, i+1)  ->  o in [(i-1+0.5)/s - 0.5, (i+1+0.5)/s - 0.5]
  float sy = (float)IH / (float)OH, sx = (float)IW / (float)OW;
  int oy_lo = max(0, (int)floorf(((float)iy - 0.5f) / sy - 0.5f) - 1), oy_hi = min(OH - 1, (int)ceilf(((float)iy + 1.5f) / sy - 0.5f) + 1);
  int ox_lo = max(0, (int)floorf(((float)ix - 0.5f) / sx - 0.5f) - 1), ox_hi = min(OW - 1, (int)ceilf(((float)ix + 1.5f) / sx - 0.5f) + 1);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float bc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (bcast) load8<float>(bcast + (long)b * C + c, bc);
  for (int oy = oy_lo; oy <= oy_hi; oy++) {
    int a0, a1; float u0, u1; bil_coef(oy, IH, OH, a0, a1, u0, u1);
    float wy = (a0 == iy ? u0 : 0.f) + (a1 == iy ? u1 : 0.f);
    if (wy == 0.f) continue;
    for (int ox = ox_lo; ox <= ox_hi; ox++) {
      int c0, c1; float v0, v1; bil_coef(ox, IW, OW, c0, c1, v0, v1);
      float wx = (c0 == ix ? v0 : 0.f) + (c1 == ix ? v1 : 0.f);
      if (wx == 0.f) continue;
      float d[8]; load8<T>(dy + (((long)b * OH + oy) * OW + ox) * C + c, d);
      float wgt = wy * wx;
#pragma unroll
      for (int e = 0; e < 8; e++) acc[e] += wgt * (d[e] + bc[e]);
    }
  }
  store8<T>(dx + i, acc);
}

// ---------------------------------------------------------------- pooled IoU head
// mean over pixels: x [B, HW, C] -> out [B, C] f32 (atomics; out must be zeroed)
template <typename T>
__global__ void avgpool_kernel(const T* __restrict__ x, float* __restrict__ out, int HW, int C, int pix_per_block) {
  const int cg = C / 8, rows = 256 / cg;
  const int t = threadIdx.x, cgi = t % cg, ri = t / cg;
  if (ri >= rows) return;
  const int b = blockIdx.y, c = cgi * 8;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long p0 = (long)blockIdx.x * pix_per_block, p1 = min((long)HW, p0 + pix_per_block);
#pragma unroll 4
  for (long p = p0 + ri; p < p1; p += rows) {
    float v[8]; load8<T>(x + ((long)b * HW + p) * C + c, v);
#pragma unroll
    for (int e = 0; e < 8; e++) s[e] += v[e];
  }
  float inv = 1.0f / (float)HW;
#pragma unroll
  for (int e = 0; e < 8; e++) atomicAdd(out + (long)b * C + c + e, s[e] * inv);
}

// classifier_head (src/s3od/model.py:185-191): Linear(256,64) -> ReLU -> Linear(64,3); one block per image
__global__ void iou_head_fwd_kernel(const float* pooled, const float* w1, const float* b1, const float* w2, const float* b2,
                                    float* hid, float* out) {
  __shared__ float h[64];
  int b = blockIdx.x, t = threadIdx.x;   // 64 threads
  const float* x = pooled + b * 256;
  float a = b1[t];
  for (int k = 0; k < 256; k++) a += w1[t * 256 + k] * x[k];
  a = fmaxf(a, 0.f);
  h[t] = a;
  if (hid) hid[b * 64 + t] = a;
  __syncthreads();
  if (t < 3) {
    float o = b2[t];
    for (int k = 0; k < 64; k++) o += w2[t * 64 + k] * h[k];
    out[b * 3 + t] = o;
  }
}

// backward of the head: given dout [B,3] -> dw2, db2, dw1, db1 (accumulate) and dpooled/HW [B,256] (bcast for p1)
__global__ void iou_head_bwd_kernel(const float* pooled, const float* hid, const float* w1, const float* w2, const float* dout,
                                    float* dw1, float* db1, float* dw2, float* db2, float* dpix, int B, float inv_hw) {
  // single block of 256 threads; B is small
  __shared__ float dh[64];
  int t = threadIdx.x;
  for (int b = 0; b < B; b++) {
    const float* d = dout + b * 3;
    if (t < 64) {
      float g = 0.f;
      for (int j = 0; j < 3; j++) { g += d[j] * w2[j * 64 + t]; atomicAdd(dw2 + j * 64 + t, d[j] * hid[b * 64 + t]); }
      dh[t] = hid[b * 64 + t] > 0.f ? g : 0.f;
      atomicAdd(db1 + t, dh[t]);
    }
    if (t < 3) atomicAdd(db2 + t, d[t]);
    __syncthreads();
    // dw1[j][k] += dh[j]*pooled[k];  dpooled[k] = sum_j dh[j] w1[j][k]
    float dp = 0.f;
    for (int j = 0; j < 64; j++) { atomicAdd(dw1 + j * 256 + t, dh[j] * pooled[b * 256 + t]); dp += dh[j] * w1[j * 256 + t]; }
    dpix[b * 256 + t] = dp * inv_hw;
    __syncthreads();
  }
}

// ---------------------------------------------------------------- mask-head backward prologue
// dlogits [B,3,HW] f32, h [M,96] T (post-ReLU) -> dh [M,96] T, dw2 [3][32], db2 [3] (accumulate)
template <typename T>
__global__ void mask_heads_bwd_kernel(const float* __restrict__ dlog, const T* __restrict__ hs, const float* __restrict__ w2,
                                      T* __restrict__ dh, float* __restrict__ dw2, float* __restrict__ db2, long M, int HW, int pix_per_block) {
  __shared__ float sw[96], sb[3];
  const int t = threadIdx.x;   // 96 threads: column j
  if (t < 96) sw[t] = 0.f;
  if (t < 3) sb[t] = 0.f;
  __syncthreads();
  const int k = t / 32;
  const float wk = w2[t];
  float accw = 0.f, accb = 0.f;
  long p0 = (long)blockIdx.x * pix_per_block, p1 = min(M, p0 + pix_per_block);
#pragma unroll 4
  for (long m = p0; m < p1; m++) {
    int b = m / HW; long pix = m - (long)b * HW;
    float dl = dlog[((long)b * 3 + k) * HW + pix];
    float hv = to_f<T>(hs[m * 96 + t]);
    dh[m * 96 + t] = from_f<T>(hv > 0.f ? dl * wk : 0.f);
    accw += dl * hv;
    if ((t & 31) == 0) accb += dl;
  }
  atomicAdd(dw2 + t, accw);
  if ((t & 31) == 0) atomicAdd(db2 + k, accb);
}

extern "C" {

int s3od_repack_weight(int dtype, const float* src, void* dst, int O, int I, int KH, int KW, void* stream) {
  long total = (long)O * I * KH * KW;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL(repack_kernel<T>, dim3(cdiv(total, 256)), dim3(256), 0, (hipStream_t)stream, src, (T*)dst, O, I, KH * KW);
  });
  return s3od_check_launch("repack_weight");
}

int s3od_bn_fold(const float* w, const float* b, const float* rm, const float* rv, float eps,
                 float* scale, float* shift, int C, void* stream) {
  hipLaunchKernelGGL(bn_fold_kernel, dim3(cdiv(C, 256)), dim3(256), 0, (hipStream_t)stream, w, b, rm, rv, eps, scale, shift, C);
  return s3od_check_launch("bn_fold");
}

int s3od_bn_finalize(const double* stats, long count, const float* w, const float* b, float* rm, float* rv, float momentum,
                     float eps, float* mean, float* rstd, float* scale, float* shift, int C, void* stream) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(cdiv(C, 256)), dim3(256), 0, (hipStream_t)stream, stats, count, w, b, rm, rv,
                     momentum, eps, mean, rstd, scale, shift, C);
  return s3od_check_launch("bn_finalize");
}

int s3od_affine_act(int dtype, const void* x, const float* scale, const float* shift, int act, const void* r1, const void* r2,
                    void* y, long total, int C, void* stream) {
  S3OD_REQUIRE(C % 8 == 0, "affine_act: C %% 8");
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL(affine_act_kernel<T>, dim3(cdiv(total / 8, 256)), dim3(256), 0, (hipStream_t)stream, (const T*)x, scale, shift,
                       act, (const T*)r1, (const T*)r2, (T*)y, total, C);
  });
  return s3od_check_launch("affine_act");
}

int s3od_bn_bwd(int dtype, const void* dy, const void* z, const void* y_relu, const float* mean, const float* rstd,
                const float* w, double* sums, void* dz, float* dw, float* db, long npix, int C, void* stream) {
  S3OD_REQUIRE(C % 8 == 0 && 256 % (C / 8) == 0, "bn_bwd: C");
  hipStream_t st = (hipStream_t)stream;
  (void)hipMemsetAsync(sums, 0, sizeof(double) * 2 * C, st);
  const int ppb = 4096;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<T>, dim3(cdiv(npix, ppb)), dim3(256), 0, st, (const T*)dy, (const T*)z, (const T*)y_relu,
                       mean, rstd, sums, npix, C, ppb);
    hipLaunchKernelGGL(bn_bwd_apply_kernel<T>, dim3(cdiv(npix * C / 8, 256)), dim3(256), 0, st, (const T*)dy, (const T*)z,
                       (const T*)y_relu, mean, rstd, w, sums, (T*)dz, npix * C, C, npix);
  });
  hipLaunchKernelGGL(bn_param_grads_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, sums, dw, db, C);
  return s3od_check_launch("bn_bwd");
}

int s3od_bilinear_fwd(int dtype, const void* x, void* y, int B, int IH, int IW, int OH, int OW, int C, void* stream) {
  S3OD_REQUIRE(C % 8 == 0, "bilinear: C %% 8");
  long total = (long)B * OH * OW * C / 8;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL(bilinear_fwd_kernel<T>, dim3(cdiv(total, 256)), dim3(256), 0, (hipStream_t)stream, (const T*)x, (T*)y, B, IH, IW, OH, OW, C);
  });
  return s3od_check_launch("bilinear_fwd");
}

int s3od_bilinear_bwd(int dtype, const void* dy, const float* bcast, void* dx, int B, int IH, int IW, int OH, int OW, int C, void* stream) {
  S3OD_REQUIRE(C % 8 == 0, "bilinear: C %% 8");
  long total = (long)B * IH * IW * C / 8;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL(bilinear_bwd_kernel<T>, dim3(cdiv(total, 256)), dim3(256), 0, (hipStream_t)stream, (const T*)dy, bcast, (T*)dx,
                       B, IH, IW, OH, OW, C);
  });
  return s3od_check_launch("bilinear_bwd");
}

int s3od_avgpool(int dtype, const void* x, float* out, int B, int HW, int C, void* stream) {
  S3OD_REQUIRE(C % 8 == 0 && 256 % (C / 8) == 0, "avgpool: C");
  hipStream_t st = (hipStream_t)stream;
  (void)hipMemsetAsync(out, 0, sizeof(float) * B * C, st);
  const int ppb = 1024;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL(avgpool_kernel<T>, dim3(cdiv(HW, ppb), B), dim3(256), 0, st, (const T*)x, out, HW, C, ppb);
  });
  return s3od_check_launch("avgpool");
}

int s3od_iou_head_fwd(const float* pooled, const float* w1, const float* b1, const float* w2, const float* b2, float* hid,
                      float* out, int B, void* stream) {
  hipLaunchKernelGGL(iou_head_fwd_kernel, dim3(B), dim3(64), 0, (hipStream_t)stream, pooled, w1, b1, w2, b2, hid, out);
  return s3od_check_launch("iou_head_fwd");
}

int s3od_iou_head_bwd(const float* pooled, const float* hid, const float* w1, const float* w2, const float* dout, float* dw1,
                      float* db1, float* dw2, float* db2, float* dpix, int B, int HW, void* stream) {
  hipLaunchKernelGGL(iou_head_bwd_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, pooled, hid, w1, w2, dout, dw1, db1, dw2, db2,
                     dpix, B, 1.0f / (float)HW);
  return s3od_check_launch("iou_head_bwd");
}

int s3od_mask_heads_bwd(int dtype, const float* dlogits, const void* hsave, const float* w2, void* dh, float* dw2, float* db2,
                        int B, int HW, void* stream) {
  long M = (long)B * HW;
  const int ppb = 128;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL(mask_heads_bwd_kernel<T>, dim3(cdiv(M, ppb)), dim3(96), 0, (hipStream_t)stream, dlogits, (const T*)hsave, w2,
                       (T*)dh, dw2, db2, M, HW, ppb);
  });
  return s3od_check_launch("mask_heads_bwd");
}

}  // extern "C"
