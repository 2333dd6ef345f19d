// Memory-bound ViT kernels: patch im2col, token prefix, RoPE table, LayerNorm fwd/bwd,
// tap cast, bias / LayerScale gradient reductions, QKV-gradient RoPE inverse.
// DINOv3 arithmetic follows tf:models/dinov3_vit/modeling_dinov3_vit.py (transformers).
#include "common.hpp"

#define DISPATCH_T(dtype, ...)                                                  \
  do {                                                                          \
    if ((dtype) == S3OD_BF16) { typedef bf16 T; __VA_ARGS__ }                   \
    else if ((dtype) == S3OD_F32) { typedef float T; __VA_ARGS__ }              \
    else { s3od_set_error("bad dtype %d", (int)(dtype)); return 22; }           \
  } while (0)

// ---------------------------------------------------------------- patch embed im2col
// x: [B,3,H,W] f32 NCHW -> cols [B*P, 768] T, k = c*256 + kh*16 + kw (conv weight flatten order)
template <typename T>
__global__ void patch_im2col_kernel(const float* __restrict__ x, T* __restrict__ cols, int B, int H, int W) {
  const int ph = H / 16, pw = W / 16, P = ph * pw;
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;   // one (b, p, c, kh) row of 16 pixels
  long total = (long)B * P * 48;
  if (idx >= total) return;
  int ckh = idx % 48; long bp = idx / 48;
  int p = bp % P; int b = bp / P;
  int c = ckh / 16, kh = ckh % 16;
  int py = p / pw, px = p % pw;
  const float* src = x + (((long)b * 3 + c) * H + py * 16 + kh) * W + px * 16;
  T* dst = cols + bp * 768 + c * 256 + kh * 16;
  float v[16];
#pragma unroll
  for (int i = 0; i < 4; i++) { float4 f = ((const float4*)src)[i]; v[4 * i] = f.x; v[4 * i + 1] = f.y; v[4 * i + 2] = f.z; v[4 * i + 3] = f.w; }
  store8<T>(dst, v);
  store8<T>(dst + 8, v + 8);
}

// hidden size D of the encoder: 768 (ViT-B/16, dinob) or 1024 (ViT-L/16, dinol); head dim 64
#define DISPATCH_D(D_, ...)                                                     \
  do {                                                                          \
    if ((D_) == 768) { constexpr int D = 768; __VA_ARGS__ }                     \
    else if ((D_) == 1024) { constexpr int D = 1024; __VA_ARGS__ }              \
    else { s3od_set_error("hidden size %d not built (768 or 1024)", (int)(D_)); return 22; } \
  } while (0)

// rows 0..4 of each image: cls + 4 register tokens (tf:…:88-90)
__global__ void token_prefix_kernel(float* x, const float* cls, const float* reg, int Ntok, int D) {
  int b = blockIdx.x, t = blockIdx.y;  // t in 0..4
  const float* src = t == 0 ? cls : reg + (t - 1) * D;
  float* dst = x + ((long)b * Ntok + t) * D;
  for (int i = threadIdx.x; i < D; i += blockDim.x) dst[i] = src[i];
}

// RoPE table (tf:…:96-121, 168-200): cos/sin [P,64]; rescale <= 0 means none (eval)
__global__ void rope_table_kernel(float* cs, float* sn, int ph, int pw, float rescale) {
  int p = blockIdx.x, j = threadIdx.x;  // 64 threads
  if (p >= ph * pw) return;
  int jj = j & 31;
  int f = jj & 15;
  // inv_freq = 1 / 100 ** arange(0, 1, 4/64)
  float expo = (float)f * (4.0f / 64.0f);
  float inv_freq = 1.0f / powf(100.0f, expo);
  int y = p / pw, xq = p % pw;
  float coord = jj < 16 ? ((float)y + 0.5f) / (float)ph : ((float)xq + 0.5f) / (float)pw;
  coord = 2.0f * coord - 1.0f;
  if (rescale > 0.f) coord = coord * rescale;
  float ang = (6.283185307179586f * coord) * inv_freq;
  cs[p * 64 + j] = cosf(ang);
  sn[p * 64 + j] = sinf(ang);
}

// ---------------------------------------------------------------- LayerNorm (D = 768 / 1024)
// one wave per row (NV = D/256 float4 per lane); fp32 statistics; y = (x-mean)*rstd*w + b stored as T
template <typename T, int D>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                      const float* __restrict__ b, T* __restrict__ y,
                                                      float* __restrict__ mean_o, float* __restrict__ rstd_o, int M, float eps) {
  constexpr int NV = D / 256;
  int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* xr = x + (long)row * D;
  float v[4 * NV];
#pragma unroll
  for (int i = 0; i < NV; i++) { float4 f = ((const float4*)xr)[lane + 64 * i]; v[4 * i] = f.x; v[4 * i + 1] = f.y; v[4 * i + 2] = f.z; v[4 * i + 3] = f.w; }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4 * NV; i++) s += v[i];
  float mean = warp_sum(s) * (1.0f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 4 * NV; i++) { float d = v[i] - mean; q += d * d; }
  float var = warp_sum(q) * (1.0f / D);
  float rstd = 1.0f / sqrtf(var + eps);
  if (y) {                                         // y == nullptr: statistics only
  T* yr = y + (long)row * D;
#pragma unroll
  for (int i = 0; i < NV; i++) {
    int c = 4 * (lane + 64 * i);
    float4 wf = *(const float4*)(w + c), bf = *(const float4*)(b + c);
    float o0 = (v[4 * i] - mean) * rstd * wf.x + bf.x, o1 = (v[4 * i + 1] - mean) * rstd * wf.y + bf.y;
    float o2 = (v[4 * i + 2] - mean) * rstd * wf.z + bf.z, o3 = (v[4 * i + 3] - mean) * rstd * wf.w + bf.w;
    if constexpr (sizeof(T) == 4) *(float4*)(yr + c) = make_float4(o0, o1, o2, o3);
    else { bf16x4 o = {(bf16)o0, (bf16)o1, (bf16)o2, (bf16)o3}; *(bf16x4*)(yr + c) = o; }
  }
  }
  if (lane == 0) { mean_o[row] = mean; rstd_o[row] = rstd; }
}

// LayerNorm backward. dx = dres + rstd*(g - mean(g) - xhat*mean(g*xhat)), g = dy*w
// dw += sum dy*xhat ; db += sum dy   (fp32 block partials -> replicated atomics [NREP][2D])
// LS: fused with the LayerScale backward of the layer below, which consumes this dx (ViT backward order:
// norm2 -> layer_scale1 of the same layer, norm1 -> layer_scale2 of the next lower layer): du = dx * lam (T),
// dlam += sum dx*u, dbias += sum du into a second replicated workspace ws2 -- saves that kernel's re-read of dx.
template <typename T, int D, bool LS = false>
__global__ void __launch_bounds__(256) ln_bwd_kernel(const T* __restrict__ dy, const float* __restrict__ x,
                                                      const float* __restrict__ mean, const float* __restrict__ rstd,
                                                      const float* __restrict__ w, const float* __restrict__ dres,
                                                      float* __restrict__ dx, float* __restrict__ ws,
                                                      int M, int rows_per_block, const T* __restrict__ u = nullptr,
                                                      const float* __restrict__ lam = nullptr, T* __restrict__ du = nullptr,
                                                      float* __restrict__ ws2 = nullptr) {
  constexpr int NV = D / 256, NE = 4 * NV, NS = LS ? 4 : 2;
  __shared__ float sred[NS][D];
  float* sdw = sred[0];
  float* sdb = sred[1];
  for (int i = threadIdx.x; i < D; i += 256)
#pragma unroll
    for (int k = 0; k < NS; k++) sred[k][i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float pw[NE], pb[NE], pl[LS ? NE : 1], pd[LS ? NE : 1], lv[LS ? NE : 1];
#pragma unroll
  for (int i = 0; i < NE; i++) { pw[i] = 0.f; pb[i] = 0.f; }
  if constexpr (LS) {
#pragma unroll
    for (int i = 0; i < NV; i++) {
      const float4 l4 = *(const float4*)(lam + 4 * (lane + 64 * i));
      lv[4 * i] = l4.x; lv[4 * i + 1] = l4.y; lv[4 * i + 2] = l4.z; lv[4 * i + 3] = l4.w;
    }
#pragma unroll
    for (int i = 0; i < NE; i++) { pl[i] = 0.f; pd[i] = 0.f; }
  }
  int r0 = blockIdx.x * rows_per_block;
  for (int row = r0 + wave; row < min(M, r0 + rows_per_block); row += 4) {
    const float* xr = x + (long)row * D;
    float mu = mean[row], rs = rstd[row];
    float xh[NE], g[NE], dyv[NE];
    float4 rr4[NV];
    bf16x4 uu4[LS ? NV : 1];
#pragma unroll
    for (int i = 0; i < NV; i++) {  // issue the residual-gradient (and LayerScale input) loads before the row reductions
      rr4[i] = dres ? *(const float4*)(dres + (long)row * D + 4 * (lane + 64 * i)) : make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (LS && sizeof(T) == 2) uu4[i] = *(const bf16x4*)(u + (long)row * D + 4 * (lane + 64 * i));
    }
#pragma unroll
    for (int i = 0; i < NV; i++) {
      int c = 4 * (lane + 64 * i);
      float4 xf = *(const float4*)(xr + c);
      float4 wf = *(const float4*)(w + c);
      float d4[4];
      if constexpr (sizeof(T) == 4) { float4 t = *(const float4*)(dy + (long)row * D + c); d4[0] = t.x; d4[1] = t.y; d4[2] = t.z; d4[3] = t.w; }
      else { bf16x4 t = *(const bf16x4*)(dy + (long)row * D + c); d4[0] = (float)t[0]; d4[1] = (float)t[1]; d4[2] = (float)t[2]; d4[3] = (float)t[3]; }
      float xs[4] = {xf.x, xf.y, xf.z, xf.w}, wv[4] = {wf.x, wf.y, wf.z, wf.w};
#pragma unroll
      for (int e = 0; e < 4; e++) { xh[4 * i + e] = (xs[e] - mu) * rs; dyv[4 * i + e] = d4[e]; g[4 * i + e] = d4[e] * wv[e]; }
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NE; i++) { s1 += g[i]; s2 += g[i] * xh[i]; }
    s1 = warp_sum(s1) * (1.0f / D);
    s2 = warp_sum(s2) * (1.0f / D);
#pragma unroll
    for (int i = 0; i < NV; i++) {
      int c = 4 * (lane + 64 * i);
      float o[4];
      float rr[4] = {rr4[i].x, rr4[i].y, rr4[i].z, rr4[i].w};
#pragma unroll
      for (int e = 0; e < 4; e++) {
        int k = 4 * i + e;
        o[e] = rr[e] + rs * (g[k] - s1 - xh[k] * s2);
        pw[k] += dyv[k] * xh[k];
        pb[k] += dyv[k];
      }
      *(float4*)(dx + (long)row * D + c) = make_float4(o[0], o[1], o[2], o[3]);
      if constexpr (LS) {
        float uv[4];
        if constexpr (sizeof(T) == 4) {
          const float4 t = *(const float4*)(u + (long)row * D + c);
          uv[0] = t.x; uv[1] = t.y; uv[2] = t.z; uv[3] = t.w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; e++) uv[e] = (float)uu4[i][e];
        }
        float dd[4];
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const int k = 4 * i + e;
          dd[e] = o[e] * lv[k];
          pl[k] += o[e] * uv[e];
          pd[k] += dd[e];
        }
        store4<T>(du + (long)row * D + c, dd);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NV; i++)
#pragma unroll
    for (int e = 0; e < 4; e++) {
      int c = 4 * (lane + 64 * i) + e;
      atomicAdd(&sdw[c], pw[4 * i + e]);
      atomicAdd(&sdb[c], pb[4 * i + e]);
    }
  if constexpr (LS) {
#pragma unroll
    for (int i = 0; i < NV; i++)
#pragma unroll
      for (int e = 0; e < 4; e++) {
        int c = 4 * (lane + 64 * i) + e;
        atomicAdd(&sred[2][c], pl[4 * i + e]);
        atomicAdd(&sred[3][c], pd[4 * i + e]);
      }
  }
  __syncthreads();
  float* rep = ws + (long)(blockIdx.x % S3OD_NREP) * 2 * D;   // replicated [dw | db] partials
  for (int i = threadIdx.x; i < D; i += 256) { atomicAdd(rep + i, sdw[i]); atomicAdd(rep + D + i, sdb[i]); }
  if constexpr (LS) {
    float* rep2 = ws2 + (long)(blockIdx.x % S3OD_NREP) * 2 * D;   // replicated [dlam | dbias] partials
    for (int i = threadIdx.x; i < D; i += 256) { atomicAdd(rep2 + i, sred[2][i]); atomicAdd(rep2 + D + i, sred[3][i]); }
  }
}

// a[i] += sum_r ws[r][i], b[i] += sum_r ws[r][D + i]   (fold of the replicated 2 x D partials; a/b may be null)
// sums the S3OD_NREP replicas of [a | b] partials and clears them (the workspace enters and leaves all zero)
__global__ void fold2_kernel(float* __restrict__ ws, float* __restrict__ a, float* __restrict__ b, int D) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * D) return;
  float s = 0.f;
  for (int r = 0; r < S3OD_NREP; r++) { s += ws[(long)r * 2 * D + i]; ws[(long)r * 2 * D + i] = 0.f; }
  if (i < D) { if (a) a[i] += s; }
  else if (b) b[i - D] += s;
}

// taps: x f32 [B, Ntok, D] -> T [B, P, D] (drop 1 + 4 prefix tokens; src/s3od/model.py:75-84)
template <typename T>
__global__ void cast_tap_kernel(const float* __restrict__ x, T* __restrict__ y, int B, int Ntok, int P, int D) {
  long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  long total = (long)B * P * D;
  if (i >= total) return;
  long row = i / D; int c = i % D;
  int b = row / P, p = row % P;
  float v[8];
  load8<float>(x + ((long)b * Ntok + (Ntok - P) + p) * D + c, v);
  store8<T>(y + i, v);
}

// column sums of a [M, N] T matrix (bias gradients): out[n] += sum_m a[m, n]
// block = 256 threads = tpr column-groups (8 columns each) x rp row phases; LDS reduction over
// the row phases, then per block either one fp32 atomic per column (part == nullptr) or the block's partial
// sums stored to part[blockIdx.y][N] for colsum_fold_kernel.
template <typename T>
__global__ void __launch_bounds__(256) colsum_kernel(const T* __restrict__ a, long lda, int M, int N, float* __restrict__ out,
                                                     int rows_per_block, float* __restrict__ part) {
  __shared__ float red[256 * 8];
  const int G = N / 8;
  const int tpr = G < 256 ? G : 256, rp = 256 / tpr;
  const int t = threadIdx.x, ci = t % tpr, ph = t / tpr;
  const int cg = blockIdx.x * tpr + ci;
  const bool act = ph < rp && cg < G;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (act) {
    long r0 = (long)blockIdx.y * rows_per_block, r1 = min((long)M, r0 + rows_per_block);
    const T* base = a + cg * 8;
    long r = r0 + ph;
    for (; r + 3 * rp < r1; r += 4 * rp) {     // 4 independent 16-B loads in flight per thread
      float v0[8], v1[8], v2[8], v3[8];
      load8<T>(base + r * lda, v0); load8<T>(base + (r + rp) * lda, v1);
      load8<T>(base + (r + 2 * rp) * lda, v2); load8<T>(base + (r + 3 * rp) * lda, v3);
#pragma unroll
      for (int e = 0; e < 8; e++) s[e] += (v0[e] + v1[e]) + (v2[e] + v3[e]);
    }
    for (; r < r1; r += rp) {
      float v[8]; load8<T>(base + r * lda, v);
#pragma unroll
      for (int e = 0; e < 8; e++) s[e] += v[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; e++) red[t * 8 + e] = s[e];
  __syncthreads();
  if (ph == 0 && cg < G) {
    for (int q = 1; q < rp; q++)
#pragma unroll
      for (int e = 0; e < 8; e++) s[e] += red[(q * tpr + ci) * 8 + e];
    if (part) {
      float* pr = part + (long)blockIdx.y * N + cg * 8;
      *(float4*)pr = make_float4(s[0], s[1], s[2], s[3]);
      *(float4*)(pr + 4) = make_float4(s[4], s[5], s[6], s[7]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; e++) atomicAdd(out + cg * 8 + e, s[e]);
    }
  }
}
// out[n] += sum over the nb partial rows in a fixed order (deterministic): block = 32 columns x 8 row groups, each
// thread sums rows rg, rg + 8, ... with 8 loads in flight, then the 8 group sums are added in group order
__global__ void __launch_bounds__(256) colsum_fold_kernel(const float* __restrict__ part, int nb, int N, float* __restrict__ out) {
  __shared__ float red[8][32];
  const int c = threadIdx.x & 31, rg = threadIdx.x >> 5, n = blockIdx.x * 32 + c;
  float s = 0.f;
  if (n < N) {
    int r = rg;
    for (; r + 56 < nb; r += 64) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; u++) v[u] = part[(long)(r + 8 * u) * N + n];
#pragma unroll
      for (int u = 0; u < 8; u++) s += v[u];
    }
    for (; r < nb; r += 8) s += part[(long)r * N + n];
  }
  red[rg][c] = s;
  __syncthreads();
  if (rg == 0 && n < N) {
    float t = red[0][c];
#pragma unroll
    for (int q = 1; q < 8; q++) t += red[q][c];
    out[n] += t;
  }
}

// LayerScale backward: du = dx * lam (T); dlam[n] += sum_m dx*u ; dbias[n] += sum_m du
// block = 4 * D/8 threads = D/8 column groups (8 columns) x 4 row phases; LDS reduction, 2 x D atomics per block
template <typename T, int D>
__global__ void __launch_bounds__(D / 2) scale_bwd_kernel(const float* __restrict__ dx, const T* __restrict__ u, const float* __restrict__ lam,
                                 T* __restrict__ du, float* __restrict__ ws, int M, int rows_per_block) {
  constexpr int NG = D / 8, NT = 4 * NG;
  __shared__ float red[NT * 8];
  const int t = threadIdx.x, g = t % NG, ph = t / NG;
  const int n = g * 8;
  int r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  float l[8]; load8<float>(lam + n, l);
  float sl[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll 4
  for (int r = r0 + ph; r < r1; r += 4) {
    float d[8], uu[8], o[8];
    load8<float>(dx + (long)r * D + n, d);
    load8<T>(u + (long)r * D + n, uu);
#pragma unroll
    for (int e = 0; e < 8; e++) { o[e] = d[e] * l[e]; sl[e] += d[e] * uu[e]; sb[e] += o[e]; }
    store8<T>(du + (long)r * D + n, o);
  }
  for (int pass = 0; pass < 2; pass++) {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; e++) red[t * 8 + e] = pass ? sb[e] : sl[e];
    __syncthreads();
    for (int c = t; c < D; c += NT) {
      const int gg = c >> 3, e = c & 7;
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < 4; q++) s += red[(q * NG + gg) * 8 + e];
      atomicAdd(ws + (long)(blockIdx.x % S3OD_NREP) * 2 * D + (pass ? D : 0) + c, s);
    }
  }
}

// dq,dk,dv [B,H,N,64] (dq w.r.t. the 1/8-scaled, rotated q) -> dqkv [B*N, 3D] T w.r.t. the
// pre-RoPE projections: d(pre) = cos*dy - R(sin*dy), R = rotate_half; dq additionally * 1/8.
// Also accumulates the q / v bias gradients (column sums of dqkv; k_proj has no bias).
// block = 3 * H * 8 threads = (which, head, 8-wide d chunk) x rows_per_block rows
template <typename T, int H>
__global__ void __launch_bounds__(24 * H) qkv_unrope_kernel(const T* __restrict__ dq, const T* __restrict__ dk, const T* __restrict__ dv,
                                  const float* __restrict__ cs, const float* __restrict__ sn,
                                  T* __restrict__ dqkv, float* __restrict__ ws,
                                  int B, int Ntok, int P, int rows_per_block) {
  constexpr int D = 64 * H;
  const int t = threadIdx.x;
  const int d8 = t & 7, h = (t >> 3) % H, which = t / (8 * H);
  const int d0 = d8 * 8;
  const int pd = d0 < 32 ? d0 + 32 : d0 - 32;
  const T* src = which == 0 ? dq : (which == 1 ? dk : dv);
  const long M = (long)B * Ntok;
  const long r0 = (long)blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  constexpr int RB = 4;   // rows whose loads are issued together
  for (long m0 = r0; m0 < r1; m0 += RB) {
    float v[RB][8], pv[RB][8], cr[RB][8], sr[RB][8];
    bool rot[RB];
#pragma unroll
    for (int j = 0; j < RB; j++) {
      const long m = min(m0 + j, r1 - 1);
      const int b = m / Ntok, tk = m - (long)b * Ntok;
      const T* row = src + (((long)b * H + h) * Ntok + tk) * 64;
      const int tp = max(tk - (Ntok - P), 0);
      rot[j] = which < 2 && tk >= Ntok - P;
      load8<T>(row + d0, v[j]);
      load8<T>(row + pd, pv[j]);
      load8<float>(cs + (long)tp * 64 + d0, cr[j]);
      load8<float>(sn + (long)tp * 64 + pd, sr[j]);
    }
#pragma unroll
    for (int j = 0; j < RB; j++) {
      const long m = m0 + j;
      if (m >= r1) break;
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; e++) {
        // y = x*cos + R(x)*sin  =>  dx = cos*dy + R^T(sin*dy);  R^T(z)[d] = z[d+32] (d<32), -z[d-32] (d>=32)
        float rt = d0 < 32 ? sr[j][e] * pv[j][e] : -sr[j][e] * pv[j][e];
        o[e] = rot[j] ? cr[j][e] * v[j][e] + rt : v[j][e];
        if (which == 0) o[e] *= 0.125f;
        acc[e] += o[e];
      }
      store8<T>(dqkv + m * 3 * D + which * D + h * 64 + d0, o);
    }
  }
  if (which != 1 && ws) {   // replicated partials: ws[blk % NREP][q D | v D]
    float* dst = ws + (long)(blockIdx.x % S3OD_NREP) * 2 * D + (which == 0 ? 0 : D) + h * 64 + d0;
#pragma unroll
    for (int e = 0; e < 8; e++) atomicAdd(dst + e, acc[e]);
  }
}

// d(cls) = sum_b dx[b,0], d(reg[t]) = sum_b dx[b,1+t]  (accumulate)
__global__ void token_prefix_bwd_kernel(const float* dx, float* dcls, float* dreg, int B, int Ntok, int D) {
  int t = blockIdx.x;  // 0..4
  float* dst = t == 0 ? dcls : dreg + (t - 1) * D;
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    float s = 0.f;
    for (int b = 0; b < B; b++) s += dx[((long)b * Ntok + t) * D + c];
    dst[c] += s;
  }
}

extern "C" {

int s3od_token_prefix_bwd(const float* dx, float* dcls, float* dreg, int B, int Ntok, int D, void* stream) {
  hipLaunchKernelGGL(token_prefix_bwd_kernel, dim3(5), dim3(256), 0, (hipStream_t)stream, dx, dcls, dreg, B, Ntok, D);
  return s3od_check_launch("token_prefix_bwd");
}

int s3od_patch_im2col(int dtype, const float* x, void* cols, int B, int H, int W, void* stream) {
  S3OD_REQUIRE(W % 4 == 0 && H >= 16 && W >= 16, "patch_im2col: W must be a multiple of 4 and H,W >= 16");
  long total = (long)B * (H / 16) * (W / 16) * 48;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL(patch_im2col_kernel<T>, dim3(cdiv(total, 256)), dim3(256), 0, (hipStream_t)stream, x, (T*)cols, B, H, W);
  });
  return s3od_check_launch("patch_im2col");
}

int s3od_token_prefix(float* x, const float* cls, const float* reg, int B, int Ntok, int D, void* stream) {
  hipLaunchKernelGGL(token_prefix_kernel, dim3(B, 5), dim3(256), 0, (hipStream_t)stream, x, cls, reg, Ntok, D);
  return s3od_check_launch("token_prefix");
}

int s3od_rope_table(float* cs, float* sn, int ph, int pw, float rescale, void* stream) {
  hipLaunchKernelGGL(rope_table_kernel, dim3(ph * pw), dim3(64), 0, (hipStream_t)stream, cs, sn, ph, pw, rescale);
  return s3od_check_launch("rope_table");
}

int s3od_layernorm_fwd(int dtype, const float* x, const float* w, const float* b, void* y, float* mean, float* rstd,
                       int M, int D_, float eps, void* stream) {
  DISPATCH_D(D_, {
    DISPATCH_T(dtype, {
      hipLaunchKernelGGL((ln_fwd_kernel<T, D>), dim3(cdiv(M, 4)), dim3(256), 0, (hipStream_t)stream, x, w, b, (T*)y, mean, rstd, M, eps);
    });
  });
  return s3od_check_launch("layernorm_fwd");
}

// ws: S3OD_NREP * 2 * D floats (replicated dw / db partials), all zero on entry; left all zero
int s3od_layernorm_bwd(int dtype, const void* dy, const float* x, const float* mean, const float* rstd, const float* w,
                       const float* dres, float* dx, float* dw, float* db, float* ws, int M, int D_, void* stream) {
  const int rpb = S3OD_KNOB("S3OD_LN_RPB", 32);
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_D(D_, {
    DISPATCH_T(dtype, {
      hipLaunchKernelGGL((ln_bwd_kernel<T, D>), dim3(cdiv(M, rpb)), dim3(256), 0, st, (const T*)dy, x, mean, rstd, w, dres, dx, ws, M, rpb);
    });
  });
  hipLaunchKernelGGL(fold2_kernel, dim3(cdiv(2 * D_, 256)), dim3(256), 0, st, ws, dw, db, D_);
  return s3od_check_launch("layernorm_bwd");
}

// s3od_layernorm_bwd fused with the LayerScale backward (s3od_layerscale_bwd) of the layer that consumes its dx:
// du = dx * lam, dlam += sum dx*u, dbias += sum du.  ws, ws2: S3OD_NREP * 2 * D floats each, all zero on entry and
// left all zero.  Replaces the pair s3od_layernorm_bwd + s3od_layerscale_bwd (tf:modeling_dinov3_vit.py:419-445).
int s3od_layernorm_ls_bwd(int dtype, const void* dy, const float* x, const float* mean, const float* rstd, const float* w,
                          const float* dres, float* dx, float* dw, float* db, float* ws, const void* u, const float* lam,
                          void* du, float* dlam, float* dbias, float* ws2, int M, int D_, void* stream) {
  S3OD_REQUIRE(u && lam && du && ws2 && ws != ws2, "layernorm_ls_bwd: bad arguments");
  // rows per block: 64 (bf16, M 65616: 221 us vs 240 us at 32 and 328 us at 16; the fused kernel runs at 3
  // waves/SIMD, so longer blocks amortise the 4 x D partial flush)
  const int rpb = S3OD_KNOB("S3OD_LNLS_RPB", 64);
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_D(D_, {
    DISPATCH_T(dtype, {
      hipLaunchKernelGGL((ln_bwd_kernel<T, D, true>), dim3(cdiv(M, rpb)), dim3(256), 0, st, (const T*)dy, x, mean, rstd, w, dres,
                         dx, ws, M, rpb, (const T*)u, lam, (T*)du, ws2);
    });
  });
  hipLaunchKernelGGL(fold2_kernel, dim3(cdiv(2 * D_, 256)), dim3(256), 0, st, ws, dw, db, D_);
  hipLaunchKernelGGL(fold2_kernel, dim3(cdiv(2 * D_, 256)), dim3(256), 0, st, ws2, dlam, dbias, D_);
  return s3od_check_launch("layernorm_ls_bwd");
}

int s3od_cast_tap(int dtype, const float* x, void* y, int B, int Ntok, int P, int D, void* stream) {
  S3OD_REQUIRE(D % 8 == 0, "cast_tap: D %% 8");
  long total = (long)B * P * D / 8;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL(cast_tap_kernel<T>, dim3(cdiv(total, 256)), dim3(256), 0, (hipStream_t)stream, x, (T*)y, B, Ntok, P, D);
  });
  return s3od_check_launch("cast_tap");
}

// row blocks of the column sum: <= ~512 of >= 64 rows.  Without a workspace each block adds its sums by fp32
// atomics, which serialise on one address in L2: 256 / 512 / 1024 of them cost ~50 / 100 / 200 us whatever the
// matrix size (tools/colsum_bench.py, profiles/r05w_colsum.txt); with one, the blocks store partial rows and a
// second pass adds them in a fixed order
static long colsum_rpb(int M, int gx, bool ws) { (void)ws; return max(64L, (long)M * gx / 512); }
// bytes of the partial-sum workspace s3od_colsum uses for these arguments
int s3od_colsum_ws(int M, int N, long* bytes) {
  S3OD_REQUIRE(bytes != nullptr && N % 8 == 0, "colsum_ws: bad arguments");
  const int G = N / 8, tpr = G < 256 ? G : 256, gx = cdiv(G, tpr);
  *bytes = 4L * cdiv(M, colsum_rpb(M, gx, true)) * N;
  return 0;
}

int s3od_colsum(int dtype, const void* a, long lda, int M, int N, float* out, float* ws, long ws_bytes, void* stream) {
  S3OD_REQUIRE(N % 8 == 0, "colsum: N %% 8");
  const int G = N / 8, tpr = G < 256 ? G : 256, gx = cdiv(G, tpr);
  long need = 0;
  if (ws) s3od_colsum_ws(M, N, &need);
  const bool two_pass = ws && ws_bytes >= need && N % 4 == 0 && !S3OD_OFF("S3OD_COLSUM_2P");
  const long rpb = colsum_rpb(M, gx, two_pass);
  const int nb = (int)cdiv(M, rpb);
  dim3 grid(gx, nb);
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL(colsum_kernel<T>, grid, dim3(256), 0, (hipStream_t)stream, (const T*)a, lda, M, N, out, (int)rpb,
                       two_pass ? ws : nullptr);
  });
  if (two_pass) hipLaunchKernelGGL(colsum_fold_kernel, dim3(cdiv(N, 32)), dim3(256), 0, (hipStream_t)stream, ws, nb, N, out);
  return s3od_check_launch("colsum");
}

// ws: S3OD_NREP * 2 * D floats (replicated dlam / dbias partials), all zero on entry; left all zero
int s3od_layerscale_bwd(int dtype, const float* dx, const void* u, const float* lam, void* du, float* dlam, float* dbias,
                        float* ws, int M, int D_, void* stream) {
  const int rpb = S3OD_KNOB("S3OD_LS_RPB", 16);
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_D(D_, {
    DISPATCH_T(dtype, {
      hipLaunchKernelGGL((scale_bwd_kernel<T, D>), dim3(cdiv(M, rpb)), dim3(D / 2), 0, st, dx, (const T*)u, lam, (T*)du, ws, M, rpb);
    });
  });
  hipLaunchKernelGGL(fold2_kernel, dim3(cdiv(2 * D_, 256)), dim3(256), 0, st, ws, dlam, dbias, D_);
  return s3od_check_launch("layerscale_bwd");
}

// H heads of 64 (D = 64 H); ws: S3OD_NREP * 2 * D floats, all zero on entry; left all zero
int s3od_qkv_unrope(int dtype, const void* dq, const void* dk, const void* dv, const float* cs, const float* sn,
                    void* dqkv, float* dbq, float* dbv, float* ws, int B, int Ntok, int P, int H, void* stream) {
  S3OD_REQUIRE(ws || (!dbq && !dbv), "qkv_unrope: bias gradients need the workspace");
  S3OD_REQUIRE(H == 12 || H == 16, "qkv_unrope: %d heads not built (12 or 16)", H);
  const long M = (long)B * Ntok;
  const int D_ = 64 * H;
  const int rpb = S3OD_KNOB("S3OD_UNROPE_RPB", 64);
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    if (H == 12)
      hipLaunchKernelGGL((qkv_unrope_kernel<T, 12>), dim3(cdiv(M, rpb)), dim3(24 * 12), 0, st, (const T*)dq, (const T*)dk,
                         (const T*)dv, cs, sn, (T*)dqkv, ws, B, Ntok, P, rpb);
    else
      hipLaunchKernelGGL((qkv_unrope_kernel<T, 16>), dim3(cdiv(M, rpb)), dim3(24 * 16), 0, st, (const T*)dq, (const T*)dk,
                         (const T*)dv, cs, sn, (T*)dqkv, ws, B, Ntok, P, rpb);
  });
  if (ws) hipLaunchKernelGGL(fold2_kernel, dim3(cdiv(2 * D_, 256)), dim3(256), 0, st, ws, dbq, dbv, D_);
  return s3od_check_launch("qkv_unrope");
}

}  // extern "C"
