// Memory-bound DPT-decoder kernels (NHWC activations): weight repack, BatchNorm fold /
// batch statistics / apply / backward, bilinear resize fwd/bwd, global average pool,
// IoU-score MLP head fwd/bwd, mask-head backward prologue, ReLU masks.
// Reference: src/s3od/model.py:109-467.
#include "common.hpp"
#include <type_traits>

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

// Multi-tensor form: every packed weight of the model in ONE launch (the fp32 masters change after
// each optimizer step, so the whole set is re-packed per step).  tab: device int64 [T][RPK_FIELDS] =
// {src ptr, dst ptr, O, I, KH*KW, dst element offset, mode, dst leading dim}; chunk_t / chunk_o map
// blocks -> (tensor, start).  mode 0: dst [O][KHW][I] (the conv / linear kernel layout);
// mode 1: dst [I][KHW][ld] with column o (+offset) and the taps reversed — the stride-1 conv's
// data-gradient weight (dx = conv(dy, w^T flipped)), several tensors may interleave their columns;
// mode 2: as mode 1 without the tap reversal (the ConvTranspose2d(4, s2) sub-pixel kernel's weight).
constexpr int RPK_FIELDS = 8;
template <typename T>
__global__ void __launch_bounds__(256) repack_multi_kernel(const long* __restrict__ tab, const int* __restrict__ chunk_t,
                                                           const long* __restrict__ chunk_o, int chunk) {
  const int t = chunk_t[blockIdx.x];
  const long o0 = chunk_o[blockIdx.x];
  const long* e = tab + (long)RPK_FIELDS * t;
  const float* src = (const float*)e[0];
  T* dst = (T*)e[1] + e[5];
  const int O = (int)e[2], I = (int)e[3], KHW = (int)e[4], mode = (int)e[6];
  const long ld = e[7];
  const long total = (long)O * I * KHW;
  const long o1 = min(total, o0 + chunk);
  // linears (KHW 1, mode 0) are a plain cast: 4 elements per thread (16-B loads) when both sides are aligned; the
  // general path's 64-bit div / mod per element made the whole-model repack VALU-bound (389 us per step)
  const bool aligned = (size_t)(src + o0) % 16 == 0 && (size_t)(dst + o0) % (4 * sizeof(T)) == 0;
  if (mode == 0 && KHW == 1 && aligned) {
    const long n4 = (o1 - o0) >> 2;
    const float4* s4 = (const float4*)(src + o0);
    for (long j = threadIdx.x; j < n4; j += blockDim.x) {
      const float4 f = s4[j];
      if constexpr (sizeof(T) == 4) ((float4*)(dst + o0))[j] = f;
      else ((bf16x4*)(dst + o0))[j] = bf16x4{(bf16)f.x, (bf16)f.y, (bf16)f.z, (bf16)f.w};
    }
    for (long idx = o0 + 4 * n4 + threadIdx.x; idx < o1; idx += blockDim.x) dst[idx] = from_f<T>(src[idx]);
    return;
  }
  if (total >= (1L << 31)) {                       // (no model tensor is this large) 64-bit index arithmetic
    for (long idx = o0 + threadIdx.x; idx < o1; idx += blockDim.x) {
      if (mode == 0) {
        int i = idx % I; long r = idx / I; int tp = r % KHW; int o = r / KHW;
        dst[idx] = from_f<T>(src[((long)o * I + i) * KHW + tp]);
      } else {
        int o = idx % O; long r = idx / O; int tp = r % KHW; int i = r / KHW;
        dst[((long)i * KHW + tp) * ld + o] = from_f<T>(src[((long)o * I + i) * KHW + (mode == 1 ? KHW - 1 - tp : tp)]);
      }
    }
    return;
  }
  for (int idx = (int)o0 + threadIdx.x; idx < (int)o1; idx += blockDim.x) {      // 32-bit index arithmetic
    if (mode == 0) {
      const int i = idx % I, r = idx / I, tp = r % KHW, o = r / KHW;
      dst[idx] = from_f<T>(src[(o * I + i) * KHW + tp]);
    } else {
      const int o = idx % O, r = idx / O, tp = r % KHW, i = r / KHW;
      dst[((long)i * KHW + tp) * ld + o] = from_f<T>(src[(o * I + i) * KHW + (mode == 1 ? KHW - 1 - tp : tp)]);
    }
  }
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
// stats enter as the conv epilogue's fp64 [S3OD_NREP][sum | sum of squares] replicas and are folded and cleared
// here (persistent workspace)
__global__ void bn_finalize_kernel(double* stats, long count, const float* w, const float* b, float* rm, float* rv,
                                   float momentum, float eps, float* mean_o, float* rstd_o, float* scale, float* shift, int C) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s1 = 0.0, s2 = 0.0;
  for (int r = 0; r < S3OD_NREP; r++) {
    double* st = stats + (long)r * 2 * C;
    s1 += st[c]; s2 += st[C + c];
    st[c] = 0.0; st[C + c] = 0.0;
  }
  double mean = s1 / (double)count;
  double var = s2 / (double)count - mean * mean;
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
  for (int e = 0; e < 8; e++) { v[e] = __builtin_fmaf(v[e], s[e], t[e]); if (act == 1) v[e] = fmaxf(v[e], 0.f); }
  if (r1) { float r[8]; load8<T>(r1 + i, r);
#pragma unroll
    for (int e = 0; e < 8; e++) v[e] += r[e]; }
  if (r2) { float r[8]; load8<T>(r2 + i, r);
#pragma unroll
    for (int e = 0; e < 8; e++) v[e] += r[e]; }
  store8<T>(y + i, v);
}

// Row-blocked NHWC reductions: a 256-thread block = CG = C/8 column groups x (256/CG) row phases,
// each thread owning 8 channels; per-thread partials are reduced over the row phases in LDS so a
// block issues one atomic per channel (not one per thread).
template <int NV> DEV void rowphase_reduce(float (&v)[NV][8], float* red, int t, int CG) {
  const int nph = 256 / CG;
#pragma unroll
  for (int j = 0; j < NV; j++) {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; e++) red[t * 8 + e] = v[j][e];
    __syncthreads();
    if (t < CG)
      for (int q = 1; q < nph; q++)
#pragma unroll
        for (int e = 0; e < 8; e++) v[j][e] += red[(q * CG + t) * 8 + e];
  }
}

// ReLU masks of the BN backward.  MODE 0: none; 1: dy' = dy*(y>0) with y read back; 2: y recomputed
// as T(fma(z, scale, shift)) — the exact value affine_act_kernel stored — so the y tensor is not read
// (two of the seven tensor passes of the two-pass backward).
template <typename T, int MODE> struct ReluMask {
  const T* y; float s[8], t[8];
  DEV void init(const T* y_, const float* as, const float* at, int c) {
    y = y_;
    if (MODE == 2) { load8<float>(as + c, s); load8<float>(at + c, t); }
  }
  DEV void load(long o, float* yy) const { if (MODE == 1) load8<T>(y + o, yy); }
  DEV bool on(const float* zz, const float* yy, int e) const {
    if (MODE == 0) return true;
    if (MODE == 1) return yy[e] > 0.f;
    return (float)(T)__builtin_fmaf(zz[e], s[e], t[e]) > 0.f;
  }
};

// BN backward, pass 1: per channel sums of dy' and dy'*xhat where dy' = dy masked by ReluMask,
// xhat = (z - mean)*rstd.  Output double [2][C].  Main loop keeps 4 pixel rows of loads in flight.
template <typename T, int MODE>
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(const T* __restrict__ dy, const T* __restrict__ z, const T* __restrict__ y_relu,
                                     const float* __restrict__ as, const float* __restrict__ at,
                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                     double* __restrict__ sums, long npix, int C, int pix_per_block) {
  __shared__ float red[256 * 8];
  const int cg = C / 8, rows = 256 / cg;
  const int t = threadIdx.x, cgi = t % cg, ri = t / cg;
  const int c = cgi * 8;
  float mu[8], rs[8];
  load8<float>(mean + c, mu); load8<float>(rstd + c, rs);
  ReluMask<T, MODE> rl; rl.init(y_relu, as, at, c);
  float acc[2][8] = {{0, 0, 0, 0, 0, 0, 0, 0}, {0, 0, 0, 0, 0, 0, 0, 0}};
  const long p0 = (long)blockIdx.x * pix_per_block, p1 = min(npix, p0 + pix_per_block);
  auto body = [&](const float* d0, const float* zz, const float* yy) {
#pragma unroll
    for (int e = 0; e < 8; e++) {
      float d = rl.on(zz, yy, e) ? d0[e] : 0.f;
      float xh = (zz[e] - mu[e]) * rs[e];
      acc[0][e] += d; acc[1][e] += d * xh;
    }
  };
  long p = p0 + ri;
  for (; p + 3 * rows < p1; p += 4 * rows) {
    float d[4][8], zz[4][8], yy[4][8];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const long o = (p + j * rows) * C + c;
      load8<T>(dy + o, d[j]); load8<T>(z + o, zz[j]);
      rl.load(o, yy[j]);
    }
#pragma unroll
    for (int j = 0; j < 4; j++) body(d[j], zz[j], yy[j]);
  }
  for (; p < p1; p += rows) {
    float d[8], zz[8], yy[8];
    const long o = p * C + c;
    load8<T>(dy + o, d); load8<T>(z + o, zz);
    rl.load(o, yy);
    body(d, zz, yy);
  }
  rowphase_reduce<2>(acc, red, t, cg);
  if (t < cg) {
    double* rep = sums + (long)(blockIdx.x % S3OD_NREP) * 3 * C;
#pragma unroll
    for (int e = 0; e < 8; e++) { atomicAdd(rep + c + e, (double)acc[0][e]); atomicAdd(rep + C + c + e, (double)acc[1][e]); }
  }
}

// fold the replicas of [s1 | s2] into replica 0 (replicas 1.. cleared as they are read)
__global__ void bn_fold_replicas_kernel(double* sums, int C) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * C) return;
  double s = sums[i];
  for (int r = 1; r < S3OD_NREP; r++) { s += sums[(long)r * 3 * C + i]; sums[(long)r * 3 * C + i] = 0.0; }
  sums[i] = s;
}

// BN backward, pass 2: dz = w*rstd*(dy' - s1/n - xhat*s2/n); optional dcb[c] += sum_p dz (the
// bias gradient of the conv that produced z).
template <typename T, int MODE>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ z, const T* __restrict__ y_relu,
                                    const float* __restrict__ as, const float* __restrict__ at,
                                    const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ w,
                                    double* __restrict__ sums, T* __restrict__ dz, float* __restrict__ dcb,
                                    long npix, int C, int pix_per_block) {
  __shared__ float red[256 * 8];
  const int cg = C / 8, rows = 256 / cg;
  const int t = threadIdx.x, cgi = t % cg, ri = t / cg;
  const int c = cgi * 8;
  float mu[8], rs[8], k1[8], m1[8], m2[8];
#pragma unroll
  for (int e = 0; e < 8; e++) {
    mu[e] = mean[c + e]; rs[e] = rstd[c + e]; k1[e] = w[c + e] * rs[e];
    m1[e] = (float)(sums[c + e] / (double)npix); m2[e] = (float)(sums[C + c + e] / (double)npix);
  }
  ReluMask<T, MODE> rl; rl.init(y_relu, as, at, c);
  float acc[1][8] = {{0, 0, 0, 0, 0, 0, 0, 0}};
  const long p0 = (long)blockIdx.x * pix_per_block, p1 = min(npix, p0 + pix_per_block);
  auto body = [&](long o, const float* d0, const float* zz, const float* yy) {
    float out[8];
#pragma unroll
    for (int e = 0; e < 8; e++) {
      float d = rl.on(zz, yy, e) ? d0[e] : 0.f;
      float xh = (zz[e] - mu[e]) * rs[e];
      out[e] = k1[e] * (d - m1[e] - xh * m2[e]);
      acc[0][e] += out[e];
    }
    store8<T>(dz + o, out);
  };
  // software-pipelined over 4-row batches: batch k+1's loads are issued before batch k's stores.  One vmcnt counts
  // loads and stores in issue order, so a batch loaded AFTER the previous batch's stores waited for those stores too.
  long p = p0 + ri;
  if (p + 3 * rows < p1) {
    Row8<T> cd[4], cz[4], cy[4];
    auto ld4 = [&](long pp, Row8<T> (&rd)[4], Row8<T> (&rz)[4], Row8<T> (&ry)[4]) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const long o = (pp + j * rows) * C + c;
        rd[j].load(dy + o); rz[j].load(z + o);
        if (MODE == 1) ry[j].load(y_relu + o);
      }
    };
    ld4(p, cd, cz, cy);
    for (;;) {
      const long pn = p + 4 * rows;
      const bool more = pn + 3 * rows < p1;
      Row8<T> nd[4], nz[4], ny[4];
      if (more) ld4(pn, nd, nz, ny);
#pragma unroll
      for (int j = 0; j < 4; j++) {
        float d[8], zz[8], yy[8];
        cd[j].get(d); cz[j].get(zz);
        if (MODE == 1) cy[j].get(yy);
        body((p + j * rows) * C + c, d, zz, yy);
      }
      p = pn;
      if (!more) break;
#pragma unroll
      for (int j = 0; j < 4; j++) { cd[j] = nd[j]; cz[j] = nz[j]; cy[j] = ny[j]; }
    }
  }
  for (; p < p1; p += rows) {
    float d[8], zz[8], yy[8];
    const long o = p * C + c;
    load8<T>(dy + o, d); load8<T>(z + o, zz);
    rl.load(o, yy);
    body(o, d, zz, yy);
  }
  if (dcb) {
    rowphase_reduce<1>(acc, red, t, cg);
    if (t < cg) {
      double* rep = sums + (long)(blockIdx.x % S3OD_NREP) * 3 * C + 2 * C;
#pragma unroll
      for (int e = 0; e < 8; e++) atomicAdd(rep + c + e, (double)acc[0][e]);
    }
  }
}

// last reader of the BN backward workspace: clears what is left (replica 0's [s1 | s2], every replica's
// conv-bias partials), so the workspace leaves all zero
__global__ void bn_param_grads_kernel(double* sums, float* dw, float* db, float* dcb, int C) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  db[c] += (float)sums[c];
  dw[c] += (float)sums[C + c];
  sums[c] = 0.0; sums[C + c] = 0.0;
  double s = 0.0;
  for (int r = 0; r < S3OD_NREP; r++) { s += sums[(long)r * 3 * C + 2 * C + c]; sums[(long)r * 3 * C + 2 * C + c] = 0.0; }
  if (dcb) dcb[c] += (float)s;
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

// exact 2x upsampling: one thread = 8 channels of the 2x2 output block (2k..2k+1, 2j..2j+1), read
// from the clamped 3x3 input neighbourhood of (k, j) (9 loads for 4 outputs instead of 16).  Output
// row 2k takes neighbourhood rows (0, 1) and 2k+1 rows (1, 2) with bil_coef's weights; at the borders
// bil_coef's clamped taps coincide with the clamped neighbourhood rows (or carry weight 0), so every
// output is computed by the same expression as bilinear_fwd_kernel.
template <typename T>
__global__ void bilinear_up2_kernel(const T* __restrict__ x, T* __restrict__ y, int B, int IH, int IW, int C) {
  long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  long total = (long)B * IH * IW * C;
  if (i >= total) return;
  const int c = i % C; long pix = i / C;
  const int j = pix % IW; long r = pix / IW; const int k = r % IH; const int b = r / IH;
  const int OH = 2 * IH, OW = 2 * IW;
  const int ry[3] = {max(k - 1, 0), k, min(k + 1, IH - 1)}, rx[3] = {max(j - 1, 0), j, min(j + 1, IW - 1)};
  const T* base = x + (long)b * IH * IW * C + c;
  float n[3][3][8];
#pragma unroll
  for (int a = 0; a < 3; a++)
#pragma unroll
    for (int e = 0; e < 3; e++) load8<T>(base + ((long)ry[a] * IW + rx[e]) * C, n[a][e]);
#pragma unroll
  for (int dy = 0; dy < 2; dy++) {
    int y0, y1; float wy0, wy1;
    bil_coef(2 * k + dy, IH, OH, y0, y1, wy0, wy1);
#pragma unroll
    for (int dx = 0; dx < 2; dx++) {
      int x0, x1; float wx0, wx1;
      bil_coef(2 * j + dx, IW, OW, x0, x1, wx0, wx1);
      const float* a = n[dy][dx]; const float* bb = n[dy][dx + 1];
      const float* cc = n[dy + 1][dx]; const float* d = n[dy + 1][dx + 1];
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; e++) o[e] = wy0 * (wx0 * a[e] + wx1 * bb[e]) + wy1 * (wx0 * cc[e] + wx1 * d[e]);
      store8<T>(y + (((long)b * OH + 2 * k + dy) * OW + 2 * j + dx) * C + c, o);
    }
  }
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
  if (OH == 2 * IH && OW == 2 * IW) {
    // exact 2x (the fusion blocks at square-multiple inputs): the only outputs that can reach input
    // row iy are 2iy-1 .. 2iy+2 (same per column).  All 16 candidate rows are loaded together
    // (clamped address, weight 0 outside), then summed in the generic loop's order -- identical
    // result, but one memory round trip instead of a dependent chain of them.
    float wy[4], wx[4];
    int oyc[4], oxc[4];
#pragma unroll
    for (int t = 0; t < 4; t++) {
      const int oy = 2 * iy - 1 + t, ox = 2 * ix - 1 + t;
      wy[t] = 0.f; wx[t] = 0.f;
      if (oy >= 0 && oy < OH) {
        int a0, a1; float u0, u1; bil_coef(oy, IH, OH, a0, a1, u0, u1);
        wy[t] = (a0 == iy ? u0 : 0.f) + (a1 == iy ? u1 : 0.f);
      }
      if (ox >= 0 && ox < OW) {
        int c0, c1; float v0, v1; bil_coef(ox, IW, OW, c0, c1, v0, v1);
        wx[t] = (c0 == ix ? v0 : 0.f) + (c1 == ix ? v1 : 0.f);
      }
      oyc[t] = min(max(oy, 0), OH - 1); oxc[t] = min(max(ox, 0), OW - 1);
    }
    float d[4][4][8];
#pragma unroll
    for (int ty = 0; ty < 4; ty++)
#pragma unroll
      for (int tx = 0; tx < 4; tx++) load8<T>(dy + (((long)b * OH + oyc[ty]) * OW + oxc[tx]) * C + c, d[ty][tx]);
#pragma unroll
    for (int ty = 0; ty < 4; ty++) {
      if (wy[ty] == 0.f) continue;
#pragma unroll
      for (int tx = 0; tx < 4; tx++) {
        if (wx[tx] == 0.f) continue;
        const float wgt = wy[ty] * wx[tx];
#pragma unroll
        for (int e = 0; e < 8; e++) acc[e] += wgt * (d[ty][tx][e] + bc[e]);
      }
    }
    store8<T>(dx + i, acc);
    return;
  }
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
// mean over pixels: x [B, HW, C] -> out [B, C] f32.  Deterministic (the classifier's pooled input feeds pred_iou and,
// through d_iou, the broadcast gradient of the whole backward: fp32 atomics here made bf16 gradients differ run to
// run by ~1e-3 after the chain's bf16 roundings amplified the last-bit differences).  Pass 1: block (k, b) sums pixels
// [k PPB, (k+1) PPB) into part[b][k][C]; pass 2 adds the partials in k order and scales.
constexpr int AVGPOOL_PPB = 1024;
template <typename T>
__global__ void __launch_bounds__(256) avgpool_part_kernel(const T* __restrict__ x, float* __restrict__ part, int HW, int C) {
  __shared__ float red[256 * 8];
  const int cg = C / 8, rows = 256 / cg;
  const int t = threadIdx.x, cgi = t % cg, ri = t / cg;
  const int b = blockIdx.y, c = cgi * 8;
  float s[1][8] = {{0, 0, 0, 0, 0, 0, 0, 0}};
  long p0 = (long)blockIdx.x * AVGPOOL_PPB, p1 = min((long)HW, p0 + AVGPOOL_PPB);
#pragma unroll 4
  for (long p = p0 + ri; p < p1; p += rows) {
    float v[8]; load8<T>(x + ((long)b * HW + p) * C + c, v);
#pragma unroll
    for (int e = 0; e < 8; e++) s[0][e] += v[e];
  }
  rowphase_reduce<1>(s, red, t, cg);
  if (t < cg) {
    float* dst = part + ((long)b * gridDim.x + blockIdx.x) * C + c;
#pragma unroll
    for (int e = 0; e < 8; e++) dst[e] = s[0][e];
  }
}
__global__ void avgpool_fold_kernel(const float* __restrict__ part, float* __restrict__ out, int nk, int C, float inv) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;   // over B * C
  const int b = i / C, c = i - b * C;
  float s = 0.f;
  for (int k = 0; k < nk; k++) s += part[((long)b * nk + k) * C + c];
  out[i] = s * inv;
}

// classifier_head (src/s3od/model.py:185-191): Linear(256,64) -> ReLU -> Linear(64,NM); one block per image
__global__ void iou_head_fwd_kernel(const float* pooled, const float* w1, const float* b1, const float* w2, const float* b2,
                                    float* hid, float* out, int NM) {
  __shared__ float h[64];
  int b = blockIdx.x, t = threadIdx.x;   // 64 threads
  const float* x = pooled + b * 256;
  float a = b1[t];
  for (int k = 0; k < 256; k++) a += w1[t * 256 + k] * x[k];
  a = fmaxf(a, 0.f);
  h[t] = a;
  if (hid) hid[b * 64 + t] = a;
  __syncthreads();
  if (t < NM) {
    float o = b2[t];
    for (int k = 0; k < 64; k++) o += w2[t * 64 + k] * h[k];
    out[b * NM + t] = o;
  }
}

// backward of the head: given dout [B,NM] -> dw2, db2, dw1, db1 (accumulate) and dpooled/HW [B,256] (bcast for p1)
// one block of 256 threads per image (fp32 atomics into the shared weight gradients)
__global__ void iou_head_bwd_kernel(const float* pooled, const float* hid, const float* w1, const float* w2, const float* dout,
                                    float* dw1, float* db1, float* dw2, float* db2, float* dpix, int B, float inv_hw, int NM) {
  __shared__ float dh[64];
  const int t = threadIdx.x, b = blockIdx.x;
  const float* d = dout + b * NM;
  if (t < 64) {
    float g = 0.f;
    for (int j = 0; j < NM; j++) { g += d[j] * w2[j * 64 + t]; atomicAdd(dw2 + j * 64 + t, d[j] * hid[b * 64 + t]); }
    dh[t] = hid[b * 64 + t] > 0.f ? g : 0.f;
    atomicAdd(db1 + t, dh[t]);
  }
  if (t < NM) atomicAdd(db2 + t, d[t]);
  __syncthreads();
  // dw1[j][k] += dh[j]*pooled[k];  dpooled[k] = sum_j dh[j] w1[j][k]
  float dp = 0.f;
  for (int j = 0; j < 64; j++) { atomicAdd(dw1 + j * 256 + t, dh[j] * pooled[b * 256 + t]); dp += dh[j] * w1[j * 256 + t]; }
  dpix[b * 256 + t] = dp * inv_hw;
}

// ---------------------------------------------------------------- mask-head backward prologue
// dlogits [B,NM,HW] f32, h [M,32NM] T (post-ReLU) -> dh [M,32NM] T = relu'(h) * dlogit_k * w2[k];
// accumulates dw2 [NM][32], db2 [NM] and db1 [32NM] (= column sums of dh, the 3x3 convs' bias gradient).
// block = 128 NM threads = 32 pixel rows x 4NM chunks of 8 channels (chunk j belongs to head j/4).
template <typename T, int NM>
__global__ void __launch_bounds__(128 * NM) mask_heads_bwd_kernel(const float* __restrict__ dlog, const T* __restrict__ hs,
                                                             const float* __restrict__ w2, T* __restrict__ dh,
                                                             float* __restrict__ dw2, float* __restrict__ db2, float* __restrict__ db1,
                                                             long M, int HW) {
  constexpr int NC = 4 * NM, C = 32 * NM, NT = 32 * NC;
  __shared__ float red[NT * 8];
  const int t = threadIdx.x, j = t % NC, pr = t / NC;
  const int k = j >> 2, c0 = j * 8;
  float wk[8];
  load8<float>(w2 + c0, wk);
  float aw[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ab[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float adb = 0.f;
  for (long m = (long)blockIdx.x * 32 + pr; m < M; m += (long)gridDim.x * 32) {
    int b = m / HW; long pix = m - (long)b * HW;
    float dl = dlog[((long)b * NM + k) * HW + pix];
    float hv[8], o[8];
    load8<T>(hs + m * C + c0, hv);
#pragma unroll
    for (int e = 0; e < 8; e++) {
      o[e] = hv[e] > 0.f ? dl * wk[e] : 0.f;
      aw[e] += dl * hv[e];
    }
    store8<T>(dh + m * C + c0, o);
#pragma unroll
    for (int e = 0; e < 8; e++) ab[e] += o[e];
    adb += dl;
  }
  // reduce over the 32 pixel rows: aw -> dw2, ab -> db1, adb (chunks 0,4,8,..) -> db2
  float* r = red;
  for (int pass = 0; pass < 3; pass++) {
    __syncthreads();
    if (pass == 0) { for (int e = 0; e < 8; e++) r[t * 8 + e] = aw[e]; }
    else if (pass == 1) { for (int e = 0; e < 8; e++) r[t * 8 + e] = ab[e]; }
    else r[t * 8] = adb;
    __syncthreads();
    if (t < C) {
      const int jj = t >> 3, e = t & 7;
      if (pass < 2) {
        float s = 0.f;
        for (int q = 0; q < 32; q++) s += r[((q * NC) + jj) * 8 + e];
        atomicAdd((pass == 0 ? dw2 : db1) + t, s);
      } else if (t < NM) {
        float s = 0.f;
        for (int q = 0; q < 32; q++) s += r[((q * NC) + 4 * t) * 8];
        atomicAdd(db2 + t, s);
      }
    }
  }
}

extern "C" {

int s3od_repack_weight(int dtype, const float* src, void* dst, int O, int I, int KH, int KW, void* stream) {
  long total = (long)O * I * KH * KW;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL(repack_kernel<T>, dim3(cdiv(total, 256)), dim3(256), 0, (hipStream_t)stream, src, (T*)dst, O, I, KH * KW);
  });
  return s3od_check_launch("repack_weight");
}

// tab: device int64 [ntensors][8] (src f32*, dst T* (or f32* for dtype F32 / fp32 biases), O, I, KH*KW,
// dst element offset, mode (0 kernel layout, 1 transposed + tap-reversed), dst leading dim (mode 1));
// chunk_t / chunk_o: device table of nchunks blocks (chunk elements each)
int s3od_repack_multi(int dtype, const long* tab, const int* chunk_t, const long* chunk_o, int nchunks, int chunk, void* stream) {
  S3OD_REQUIRE(nchunks >= 0 && chunk > 0, "repack_multi: bad chunk table");
  if (nchunks == 0) return 0;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL(repack_multi_kernel<T>, dim3(nchunks), dim3(256), 0, (hipStream_t)stream, tab, chunk_t, chunk_o, chunk);
  });
  return s3od_check_launch("repack_multi");
}

int s3od_bn_fold(const float* w, const float* b, const float* rm, const float* rv, float eps,
                 float* scale, float* shift, int C, void* stream) {
  hipLaunchKernelGGL(bn_fold_kernel, dim3(cdiv(C, 256)), dim3(256), 0, (hipStream_t)stream, w, b, rm, rv, eps, scale, shift, C);
  return s3od_check_launch("bn_fold");
}

// stats: [S3OD_NREP][2][C] fp64 replicas of the conv epilogue's (sum, sum of squares) of z, folded and left all zero
int s3od_bn_finalize(double* stats, long count, const float* w, const float* b, float* rm, float* rv, float momentum,
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

// sums: S3OD_NREP * 3 * C doubles (replicated [s1 | s2 | conv-bias] accumulators), all zero on entry; left all zero
static int bn_bwd_impl(int dtype, const void* dy, const void* z, const void* y_relu, const float* as, const float* at,
                       const float* mean, const float* rstd, const float* w, double* sums, void* dz, float* dw, float* db,
                       float* dcb, long npix, int C, void* stream) {
  S3OD_REQUIRE(C % 8 == 0 && 256 % (C / 8) == 0, "bn_bwd: C");
  hipStream_t st = (hipStream_t)stream;
  // blocks per pass (tools/hbm_bench.py bn, bs 16 x 256 channels): 1024 for >= 256K pixels (1M: 606 -> 542 us,
  // 256K: 173 -> 150 us), 512 below (64K: 1024 blocks of 64 pixels pay more in atomics: 61 -> 82 us)
  const int rows = 256 / (C / 8);
  const int nb_knob = S3OD_KNOB("S3OD_BN_BLOCKS", 0);
  long ppb = max(64L, npix / (nb_knob > 0 ? nb_knob : (npix >= 262144 ? 1024 : 512)));
  ppb = (ppb + rows - 1) / rows * rows;
  const int nb = cdiv(npix, ppb);
  DISPATCH_T(dtype, {
    auto go = [&](auto mode) {
      constexpr int R = decltype(mode)::value;
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, R>), dim3(nb), dim3(256), 0, st, (const T*)dy, (const T*)z, (const T*)y_relu,
                         as, at, mean, rstd, sums, npix, C, (int)ppb);
      hipLaunchKernelGGL(bn_fold_replicas_kernel, dim3(cdiv(2 * C, 256)), dim3(256), 0, st, sums, C);
      hipLaunchKernelGGL((bn_bwd_apply_kernel<T, R>), dim3(nb), dim3(256), 0, st, (const T*)dy, (const T*)z,
                         (const T*)y_relu, as, at, mean, rstd, w, sums, (T*)dz, dcb, npix, C, (int)ppb);
    };
    if (as) go(std::integral_constant<int, 2>{});
    else if (y_relu) go(std::integral_constant<int, 1>{});
    else go(std::integral_constant<int, 0>{});
  });
  hipLaunchKernelGGL(bn_param_grads_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, sums, dw, db, dcb, C);
  return s3od_check_launch("bn_bwd");
}

int s3od_bn_bwd(int dtype, const void* dy, const void* z, const void* y_relu, const float* mean, const float* rstd,
                const float* w, double* sums, void* dz, float* dw, float* db, float* dcb, long npix, int C, void* stream) {
  return bn_bwd_impl(dtype, dy, z, y_relu, nullptr, nullptr, mean, rstd, w, sums, dz, dw, db, dcb, npix, C, stream);
}

int s3od_bn_relu_bwd(int dtype, const void* dy, const void* z, const float* scale, const float* shift, const float* mean,
                     const float* rstd, const float* w, double* sums, void* dz, float* dw, float* db, float* dcb, long npix,
                     int C, void* stream) {
  S3OD_REQUIRE(scale && shift, "bn_relu_bwd: scale/shift");
  return bn_bwd_impl(dtype, dy, z, nullptr, scale, shift, mean, rstd, w, sums, dz, dw, db, dcb, npix, C, stream);
}

int s3od_bilinear_fwd(int dtype, const void* x, void* y, int B, int IH, int IW, int OH, int OW, int C, void* stream) {
  S3OD_REQUIRE(C % 8 == 0, "bilinear: C %% 8");
  long total = (long)B * OH * OW * C / 8;
  DISPATCH_T(dtype, {
    if (OH == 2 * IH && OW == 2 * IW) {
      const long t2 = (long)B * IH * IW * C / 8;
      hipLaunchKernelGGL(bilinear_up2_kernel<T>, dim3(cdiv(t2, 256)), dim3(256), 0, (hipStream_t)stream, (const T*)x, (T*)y, B, IH, IW, C);
    } else {
      hipLaunchKernelGGL(bilinear_fwd_kernel<T>, dim3(cdiv(total, 256)), dim3(256), 0, (hipStream_t)stream, (const T*)x, (T*)y, B, IH, IW, OH, OW, C);
    }
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

// ws: fp32 [B][ceil(HW / 1024)][C] partial sums (caller-owned, contents dead between calls)
int s3od_avgpool(int dtype, const void* x, float* out, float* ws, int B, int HW, int C, void* stream) {
  S3OD_REQUIRE(C % 8 == 0 && 256 % (C / 8) == 0 && (B * C) % 64 == 0 && ws, "avgpool: C / workspace");
  hipStream_t st = (hipStream_t)stream;
  const int nk = cdiv(HW, AVGPOOL_PPB);
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL(avgpool_part_kernel<T>, dim3(nk, B), dim3(256), 0, st, (const T*)x, ws, HW, C);
  });
  hipLaunchKernelGGL(avgpool_fold_kernel, dim3(B * C / 64), dim3(64), 0, st, ws, out, nk, C, 1.0f / (float)HW);
  return s3od_check_launch("avgpool");
}

int s3od_iou_head_fwd(const float* pooled, const float* w1, const float* b1, const float* w2, const float* b2, float* hid,
                      float* out, int B, int NM, void* stream) {
  S3OD_REQUIRE(NM >= 1 && NM <= 64, "iou_head_fwd: %d outputs", NM);
  hipLaunchKernelGGL(iou_head_fwd_kernel, dim3(B), dim3(64), 0, (hipStream_t)stream, pooled, w1, b1, w2, b2, hid, out, NM);
  return s3od_check_launch("iou_head_fwd");
}

int s3od_iou_head_bwd(const float* pooled, const float* hid, const float* w1, const float* w2, const float* dout, float* dw1,
                      float* db1, float* dw2, float* db2, float* dpix, int B, int HW, int NM, void* stream) {
  S3OD_REQUIRE(NM >= 1 && NM <= 64, "iou_head_bwd: %d outputs", NM);
  hipLaunchKernelGGL(iou_head_bwd_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, pooled, hid, w1, w2, dout, dw1, db1, dw2, db2,
                     dpix, B, 1.0f / (float)HW, NM);
  return s3od_check_launch("iou_head_bwd");
}

int s3od_mask_heads_bwd(int dtype, const float* dlogits, const void* hsave, const float* w2, void* dh, float* dw2, float* db2,
                        float* db1, int B, int HW, int NM, void* stream) {
  S3OD_REQUIRE(NM == 1 || NM == 3, "mask_heads_bwd: %d heads not built (1 or 3)", NM);
  long M = (long)B * HW;
  const int nb = (int)min(1024L, (M + 31) / 32);
  DISPATCH_T(dtype, {
    if (NM == 3)
      hipLaunchKernelGGL((mask_heads_bwd_kernel<T, 3>), dim3(nb), dim3(384), 0, (hipStream_t)stream, dlogits, (const T*)hsave, w2,
                         (T*)dh, dw2, db2, db1, M, HW);
    else
      hipLaunchKernelGGL((mask_heads_bwd_kernel<T, 1>), dim3(nb), dim3(128), 0, (hipStream_t)stream, dlogits, (const T*)hsave, w2,
                         (T*)dh, dw2, db2, db1, M, HW);
  });
  return s3od_check_launch("mask_heads_bwd");
}

}  // extern "C"
