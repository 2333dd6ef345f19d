// Implicit-GEMM engine for gfx950 (CDNA4): C[M,N] = sum_k A[m,k] * B[n,k].
//
// One kernel template serves every matmul-shaped op of the S3OD hot path:
//   * ViT linears (QKV / o_proj / MLP)        A,B dense, K-contiguous ("KC")
//   * their dgrad                              B = W read as [k=out][n=in]  ("MC")
//   * their wgrad                              A = dY^T, B = X  (both MC, split-K)
//   * decoder convs (1x1, 3x3 s1/s2)           A = NHWC gather (implicit im2col)
//   * conv dgrad / ConvTranspose forward       A = gather by output-parity class
//   * conv / ConvT wgrad                       B = NHWC gather
//
// Tiles: BM x BN x BK with BK*sizeof(T) = 128 bytes (bf16: BK=64, f32: BK=32); 256 threads
// = 4 waves in a 2x2 grid, each wave owning a (BM/2)x(BN/2) sub-tile of 16x16 MFMA blocks.
//   T = bf16 : v_mfma_f32_16x16x32_bf16 (fp32 accumulate)          -- fast path
//   T = float: v_mfma_f32_16x16x4_f32  (exact fp32 fma chains)     -- strict parity path
// Global->LDS: register staging (16 B per lane per chunk), double-buffered LDS, one
// barrier per K tile.  LDS images:
//   KC tile [rows][128 B], 16-B slots XOR-swizzled by ((row>>1)&7)  -> ds_read_b128 conflict-free
//   MC tile [BK][rows*sizeof(T)], 32-B slots XOR-swizzled by g(k)  -> ds_read_b64_tr_b16
// Epilogue: accumulators are staged through LDS as an fp32 tile and handed to a
// block-level functor (bias / BN-fold / activation / residual / RoPE / atomics ...).
#pragma once
#include "common.hpp"

template <typename T> struct KT { static constexpr int BK = 64; };
template <> struct KT<float> { static constexpr int BK = 32; };

DEV int kc_off(int r, int byte) { return r * 128 + ((((byte >> 4) ^ ((r >> 1) & 7)) << 4) | (byte & 15)); }
template <int RB> DEV int mc_off(int k, int byte) {
  constexpr int SLOTS = RB / 32;
  int g = ((k & 3) | (((k >> 3) & 1) << 2)) & (SLOTS - 1);
  return k * RB + ((((byte >> 5) ^ g) << 5) | (byte & 31));
}

// ------------------------------------------------------------------ geometry helpers
// GEMM rows enumerate pixels (b, y', x') of a "row grid" RH x RW.  For dense/FWD tiles the
// row grid is the output image; for parity-class dgrad it is the sub-grid y = py + s*y'.
struct ConvGeo {
  int B;
  int SH, SW, SC;     // gathered source tensor (NHWC), channels = SC (also its row stride)
  int RH, RW;         // row grid (pixels of the GEMM rows)
  int KH, KW, s, p;   // kernel / stride / pad of the *forward* conv
  // dgrad parity class (only for DGRAD mode)
  int py, px, kh0, kw0, nth, ntw, qy0, qx0;
};

static inline ConvGeo make_class(ConvGeo g, int OH, int OW, int py, int px) {
  // rows of class (py,px) of a dgrad output image OH x OW
  g.py = py; g.px = px;
  g.RH = (OH - py + g.s - 1) / g.s; g.RW = (OW - px + g.s - 1) / g.s;
  g.kh0 = (py + g.p) % g.s; g.kw0 = (px + g.p) % g.s;
  g.nth = g.kh0 < g.KH ? (g.KH - g.kh0 + g.s - 1) / g.s : 0;
  g.ntw = g.kw0 < g.KW ? (g.KW - g.kw0 + g.s - 1) / g.s : 0;
  g.qy0 = (py + g.p) / g.s; g.qx0 = (px + g.p) / g.s;
  return g;
}

// maps a GEMM row m to the linear output-pixel (row) index of the stored tensor
struct RowMap {
  int mode;          // 0 dense, 1 tokens (skip prefix), 2 parity class
  int P, prefix;     // tokens: m = b*P + p -> b*(P+prefix) + prefix + p
  int RH, RW, OH, OW, s, py, px;   // class: (b,y',x') -> (b, py+s*y', px+s*x') in OH x OW
  DEV long map(int m) const {
    if (mode == 0) return m;
    if (mode == 1) { int b = m / P; return (long)b * (P + prefix) + prefix + (m - b * P); }
    int hw = RH * RW; int b = m / hw; int r = m - b * hw; int yy = r / RW; int xx = r - yy * RW;
    return ((long)b * OH + (py + s * yy)) * OW + (px + s * xx);
  }
};

template <typename T> DEV uint4 relu16(uint4 v) {
  if constexpr (sizeof(T) == 2) {
    unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
      unsigned lo = (w[i] & 0x8000u) ? 0u : (w[i] & 0xFFFFu);
      unsigned hi = (w[i] & 0x80000000u) ? 0u : (w[i] & 0xFFFF0000u);
      w[i] = lo | hi;
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    float4 f = *(float4*)&v;
    f.x = fmaxf(f.x, 0.f); f.y = fmaxf(f.y, 0.f); f.z = fmaxf(f.z, 0.f); f.w = fmaxf(f.w, 0.f);
    return *(uint4*)&f;
  }
}

// ------------------------------------------------------------------ operand loaders
// Each loader fills NCH = R/32 16-byte chunks per thread for K tile kt.
// KC: chunk i of thread t -> row (t>>3) + 32 i, byte (t&7)*16 of the 128-B k-row.
// MC: chunk i of thread t -> k-row t/CPR + i*(256/CPR), 16-B column chunk t%CPR.

template <typename T, int R> struct DenseKC {          // X[row*ld + k]
  static constexpr bool KCL = true;
  static constexpr int NCH = R / 32, EPC = 16 / sizeof(T), BK = KT<T>::BK;
  const T* p; long ld; int nrows, K; int relu;
  const T* rowp[NCH]; int koff;
  DEV void setup(int t0, int tid) {
    koff = (tid & 7) * EPC;
#pragma unroll
    for (int i = 0; i < NCH; i++) { int r = t0 + (tid >> 3) + 32 * i; rowp[i] = r < nrows ? p + (long)r * ld : nullptr; }
  }
  DEV void load(int kt, uint4* v) {
    int k = kt * BK + koff;
#pragma unroll
    for (int i = 0; i < NCH; i++) {
      v[i] = (rowp[i] && k < K) ? *(const uint4*)(rowp[i] + k) : make_uint4(0, 0, 0, 0);
      if (relu) v[i] = relu16<T>(v[i]);
    }
  }
};

template <typename T, int R> struct DenseMC {          // X[k*ld + col]
  static constexpr bool KCL = false;
  static constexpr int NCH = R / 32, EPC = 16 / sizeof(T), BK = KT<T>::BK;
  static constexpr int CPR = R * sizeof(T) / 16, RSTEP = 256 / CPR;
  const T* p; long ld; int K, ncols;
  int col, kr; bool cval;
  DEV void setup(int t0, int tid) { col = t0 + (tid % CPR) * EPC; kr = tid / CPR; cval = col < ncols; }
  DEV void load(int kt, uint4* v) {
#pragma unroll
    for (int i = 0; i < NCH; i++) {
      int k = kt * BK + kr + i * RSTEP;
      v[i] = (cval && k < K) ? *(const uint4*)(p + (long)k * ld + col) : make_uint4(0, 0, 0, 0);
    }
  }
};

// conv forward A operand: rows = output pixels (b,oy,ox) of RH x RW, k = tap*SC + c
template <typename T, int R> struct ConvFwdA {
  static constexpr bool KCL = true;
  static constexpr int NCH = R / 32, EPC = 16 / sizeof(T), BK = KT<T>::BK;
  const T* x; ConvGeo g; int M; int relu;
  int rb[NCH], ry[NCH], rx[NCH];
  int tap, c;     // incremental k -> (tap, channel) state of this thread's chunk
  DEV void setup(int t0, int tid) {
    int hw = g.RH * g.RW;
#pragma unroll
    for (int i = 0; i < NCH; i++) {
      int m = t0 + (tid >> 3) + 32 * i;
      if (m < M) { int b = m / hw; int r = m - b * hw; int oy = r / g.RW; rb[i] = b; ry[i] = oy * g.s - g.p; rx[i] = (r - oy * g.RW) * g.s - g.p; }
      else { rb[i] = -1; ry[i] = 0; rx[i] = 0; }
    }
    tap = -1;
  }
  DEV void load(int kt, uint4* v) {
    int koff = (threadIdx.x & 7) * EPC;
    if (tap < 0) { int k = kt * BK + koff; tap = k / g.SC; c = k - tap * g.SC; }
    int kh = tap / g.KW, kw = tap - kh * g.KW;
    bool kval = tap < g.KH * g.KW;
#pragma unroll
    for (int i = 0; i < NCH; i++) {
      int iy = ry[i] + kh, ix = rx[i] + kw;
      bool ok = kval && rb[i] >= 0 && iy >= 0 && iy < g.SH && ix >= 0 && ix < g.SW;
      v[i] = ok ? *(const uint4*)(x + (((long)rb[i] * g.SH + iy) * g.SW + ix) * g.SC + c) : make_uint4(0, 0, 0, 0);
      if (relu) v[i] = relu16<T>(v[i]);
    }
    c += BK; while (c >= g.SC) { c -= g.SC; tap++; }
  }
};

// dgrad / ConvT A operand: rows = class pixels (b, y', x'), k = (jh*ntw + jw)*SC + c
template <typename T, int R> struct ConvDgradA {
  static constexpr bool KCL = true;
  static constexpr int NCH = R / 32, EPC = 16 / sizeof(T), BK = KT<T>::BK;
  const T* dy; ConvGeo g; int M;
  int rb[NCH], ry[NCH], rx[NCH];
  int tap, c;
  DEV void setup(int t0, int tid) {
    int hw = g.RH * g.RW;
#pragma unroll
    for (int i = 0; i < NCH; i++) {
      int m = t0 + (tid >> 3) + 32 * i;
      if (m < M) { int b = m / hw; int r = m - b * hw; int yy = r / g.RW; rb[i] = b; ry[i] = yy + g.qy0; rx[i] = (r - yy * g.RW) + g.qx0; }
      else { rb[i] = -1; ry[i] = 0; rx[i] = 0; }
    }
    tap = -1;
  }
  DEV void load(int kt, uint4* v) {
    int koff = (threadIdx.x & 7) * EPC;
    if (tap < 0) { int k = kt * BK + koff; tap = k / g.SC; c = k - tap * g.SC; }
    int jh = g.ntw ? tap / g.ntw : 0, jw = tap - jh * g.ntw;
    bool kval = tap < g.nth * g.ntw;
#pragma unroll
    for (int i = 0; i < NCH; i++) {
      int sy = ry[i] - jh, sx = rx[i] - jw;
      bool ok = kval && rb[i] >= 0 && sy >= 0 && sy < g.SH && sx >= 0 && sx < g.SW;
      v[i] = ok ? *(const uint4*)(dy + (((long)rb[i] * g.SH + sy) * g.SW + sx) * g.SC + c) : make_uint4(0, 0, 0, 0);
    }
    c += BK; while (c >= g.SC) { c -= g.SC; tap++; }
  }
};

// dgrad / ConvT B operand (MC): B[k=(jh,jw,c)][n] = W[c][kh0+s*jh][kw0+s*jw][n], W repacked [C][KH][KW][N]
template <typename T, int R> struct ConvDgradB {
  static constexpr bool KCL = false;
  static constexpr int NCH = R / 32, EPC = 16 / sizeof(T), BK = KT<T>::BK;
  static constexpr int CPR = R * sizeof(T) / 16, RSTEP = 256 / CPR;
  const T* w; ConvGeo g; int NC;     // NC = output channels of the dgrad (= conv input channels)
  int col, kr; bool cval;
  DEV void setup(int t0, int tid) { col = t0 + (tid % CPR) * EPC; kr = tid / CPR; cval = col < NC; }
  DEV void load(int kt, uint4* v) {
    int K = g.nth * g.ntw * g.SC;
#pragma unroll
    for (int i = 0; i < NCH; i++) {
      int k = kt * BK + kr + i * RSTEP;
      uint4 r = make_uint4(0, 0, 0, 0);
      if (cval && k < K) {
        int t = k / g.SC, c = k - t * g.SC;
        int jh = t / g.ntw, jw = t - jh * g.ntw;
        int kh = g.kh0 + g.s * jh, kw = g.kw0 + g.s * jw;
        r = *(const uint4*)(w + (((long)c * g.KH + kh) * g.KW + kw) * NC + col);
      }
      v[i] = r;
    }
  }
};

// wgrad B operand (MC gather): B[k=pix of the conv output grid RH x RW][n=(tap, cin)] = X[src][cin]
template <typename T, int R> struct WgradB {
  static constexpr bool KCL = false;
  static constexpr int NCH = R / 32, EPC = 16 / sizeof(T), BK = KT<T>::BK;
  static constexpr int CPR = R * sizeof(T) / 16, RSTEP = 256 / CPR;
  const T* x; ConvGeo g; int NPIX; int relu;   // g.SC = Cin of X, g.SH/SW = X dims, RH/RW = output grid
  int kr, kh, kw, cin; bool cval;
  int pb[NCH], py[NCH], pxx[NCH]; int started;
  DEV void setup(int t0, int tid) {
    int col = t0 + (tid % CPR) * EPC; kr = tid / CPR;
    int tap = col / g.SC; cin = col - tap * g.SC; kh = tap / g.KW; kw = tap - kh * g.KW;
    cval = tap < g.KH * g.KW; started = 0;
  }
  DEV void load(int kt, uint4* v) {
    if (!started) {
      started = 1;
#pragma unroll
      for (int i = 0; i < NCH; i++) {
        int k = kt * BK + kr + i * RSTEP; int hw = g.RH * g.RW;
        int b = k / hw; int r = k - b * hw; int oy = r / g.RW;
        pb[i] = b; py[i] = oy; pxx[i] = r - oy * g.RW;
      }
    }
#pragma unroll
    for (int i = 0; i < NCH; i++) {
      int iy = py[i] * g.s - g.p + kh, ix = pxx[i] * g.s - g.p + kw;
      bool ok = cval && pb[i] < g.B && iy >= 0 && iy < g.SH && ix >= 0 && ix < g.SW;
      v[i] = ok ? *(const uint4*)(x + (((long)pb[i] * g.SH + iy) * g.SW + ix) * g.SC + cin) : make_uint4(0, 0, 0, 0);
      if (relu) v[i] = relu16<T>(v[i]);
      // advance by BK pixels
      pxx[i] += BK;
      while (pxx[i] >= g.RW) { pxx[i] -= g.RW; if (++py[i] >= g.RH) { py[i] = 0; pb[i]++; } }
    }
    (void)NPIX;
  }
};

// ------------------------------------------------------------------ fragment readers
template <typename T, bool KCL, int R> struct Frag;

template <int R> struct Frag<bf16, true, R> {     // KC: ds_read_b128
  DEV static bf16x8 read(const char* lds, int row0, int kk, int lane) {
    int r = row0 + (lane & 15);
    int byte = kk * 64 + (lane >> 4) * 16;
    return *(const bf16x8*)(lds + kc_off(r, byte));
  }
};
template <int R> struct Frag<bf16, false, R> {    // MC: 2 x ds_read_b64_tr_b16
  static constexpr int RB = R * 2;
  DEV static bf16x8 read(const char* lds, int row0, int kk, int lane) {
    int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    int byte = (row0 + 4 * p) * 2;
    int k0 = kk * 32 + 8 * g + q;
    typedef __attribute__((address_space(3))) s16x4 lds_s4;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(lds + mc_off<RB>(k0, byte)));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(lds + mc_off<RB>(k0 + 4, byte)));
    bf16x8 r;
    bf16x4 a = __builtin_bit_cast(bf16x4, lo), b = __builtin_bit_cast(bf16x4, hi);
    r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3]; r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
    return r;
  }
};
template <int R> struct Frag<float, true, R> {    // KC f32: lane -> A[row l&15][k = kk*4 + l>>4]
  DEV static float read(const char* lds, int row0, int kk, int lane) {
    int r = row0 + (lane & 15);
    int byte = (kk * 4 + (lane >> 4)) * 4;
    return *(const float*)(lds + kc_off(r, byte));
  }
};
template <int R> struct Frag<float, false, R> {
  static constexpr int RB = R * 4;
  DEV static float read(const char* lds, int row0, int kk, int lane) {
    int k = kk * 4 + (lane >> 4);
    int byte = (row0 + (lane & 15)) * 4;
    return *(const float*)(lds + mc_off<RB>(k, byte));
  }
};

template <typename T> struct Mma;
template <> struct Mma<bf16> {
  static constexpr int KSTEPS = 2;  // BK=64 -> 2 x K32
  typedef bf16x8 frag;
  DEV static f32x4 mma(frag a, frag b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
};
template <> struct Mma<float> {
  static constexpr int KSTEPS = 8;  // BK=32 -> 8 x K4
  typedef float frag;
  DEV static f32x4 mma(frag a, frag b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
};

// ------------------------------------------------------------------ the kernel
template <typename T, int BM, int BN> struct GemmShape {
  static constexpr int BK = KT<T>::BK;
  static constexpr int ABYTES = BM * 128, BBYTES = BN * 128;
  static constexpr int STAGE = ABYTES + BBYTES;
  static constexpr int LDT = BN + 4;                       // fp32 C-tile row stride
  static constexpr int CBYTES = BM * LDT * 4;
  static constexpr int LDS = (2 * STAGE > CBYTES ? 2 * STAGE : CBYTES);
};

struct KRange { int kt0, kt1; };

// Block-level epilogue contract:  epi(tile, LDT, m0, n0, tid)
template <typename T, int BM, int BN, class LA, class LB, class EPI>
__global__ void __launch_bounds__(256) igemm_kernel(LA la, LB lb, EPI epi, int KTILES, int split) {
  typedef GemmShape<T, BM, BN> S;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  constexpr int MI = BM / 32, NI = BN / 32;   // 16x16 blocks per wave
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  // split-K range
  int per = (KTILES + split - 1) / split;
  int kt0 = blockIdx.z * per, kt1 = min(KTILES, kt0 + per);
  epi.prepare(blockIdx.z);
  la.setup(m0, tid);
  lb.setup(n0, tid);

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; i++)
#pragma unroll
    for (int j = 0; j < NI; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[LA::NCH], rb[LB::NCH];
  auto stage_store = [&](char* base) {
    char* la_ = base; char* lb_ = base + S::ABYTES;
#pragma unroll
    for (int i = 0; i < LA::NCH; i++) {
      int off;
      if constexpr (LA::KCL) off = kc_off((tid >> 3) + 32 * i, (tid & 7) * 16);
      else { constexpr int CPR = BM * sizeof(T) / 16; off = mc_off<BM * sizeof(T)>(tid / CPR + i * (256 / CPR), (tid % CPR) * 16); }
      *(uint4*)(la_ + off) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < LB::NCH; i++) {
      int off;
      if constexpr (LB::KCL) off = kc_off((tid >> 3) + 32 * i, (tid & 7) * 16);
      else { constexpr int CPR = BN * sizeof(T) / 16; off = mc_off<BN * sizeof(T)>(tid / CPR + i * (256 / CPR), (tid % CPR) * 16); }
      *(uint4*)(lb_ + off) = rb[i];
    }
  };

  if (kt0 < kt1) {
    la.load(kt0, ra); lb.load(kt0, rb);
    stage_store(smem);
    __syncthreads();
    int cur = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      const bool more = kt + 1 < kt1;
      if (more) { la.load(kt + 1, ra); lb.load(kt + 1, rb); }
      const char* As = smem + cur * S::STAGE;
      const char* Bs = As + S::ABYTES;
#pragma unroll
      for (int kk = 0; kk < Mma<T>::KSTEPS; kk++) {
        typename Mma<T>::frag af[MI], bfr[NI];
#pragma unroll
        for (int i = 0; i < MI; i++) af[i] = Frag<T, LA::KCL, BM>::read(As, wm * (BM / 2) + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < NI; j++) bfr[j] = Frag<T, LB::KCL, BN>::read(Bs, wn * (BN / 2) + j * 16, kk, lane);
#pragma unroll
        for (int i = 0; i < MI; i++)
#pragma unroll
          for (int j = 0; j < NI; j++) acc[i][j] = Mma<T>::mma(af[i], bfr[j], acc[i][j]);
      }
      if (more) stage_store(smem + (cur ^ 1) * S::STAGE);
      __syncthreads();
      cur ^= 1;
    }
  }
  // stage C tile to LDS (fp32)
  float* ct = (float*)smem;
#pragma unroll
  for (int i = 0; i < MI; i++)
#pragma unroll
    for (int j = 0; j < NI; j++) {
      int r = wm * (BM / 2) + i * 16 + (lane >> 4) * 4;
      int c = wn * (BN / 2) + j * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; e++) ct[(r + e) * S::LDT + c] = acc[i][j][e];
    }
  __syncthreads();
  epi(ct, S::LDT, m0, n0, tid, BM, BN);
}

// iterate 8-wide row segments of the staged tile: f(m, n, const float* v8)
template <class F> DEV void for_segments(const float* ct, int LDT, int BM, int BN, int m0, int n0, int M, int N, int tid, F f) {
  const int segs = BM * BN / 8, spr = BN / 8;
  for (int s = tid; s < segs; s += 256) {
    int r = s / spr, cs = s - r * spr;
    int m = m0 + r, n = n0 + cs * 8;
    if (m < M && n < N) f(m, n, ct + r * LDT + cs * 8, r, cs * 8);
  }
}

// ------------------------------------------------------------------ common epilogue
// out = act(acc*scale[n] + shift[n]) + res1 + res2 ; optional raw store (pre-act) and BN
// batch statistics (sum / sum of squares of the pre-activation value, fp64 atomics).
enum { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_GELU_BWD = 3, ACT_RELU_BWD = 4 };
// ACT_GELU_BWD: o = v * gelu'(res1)   (res1 = saved pre-activation, not added)
// ACT_RELU_BWD: o = v * (res1 > 0)    (res1 = saved activation output, not added)
template <typename TO, typename TR, typename TP = TO> struct EpiStd {
  // pre = acc + bias[n] ;  v = pre*scale[n] + shift[n] ;  out = act(v) (+res1 +res2)
  TO* out; long ldo; int coff;          // output row stride / channel offset
  const float* bias; const float* scale; const float* shift;
  const TR* res1; long ldr1; const TR* res2; long ldr2;
  TP* pre; long ldp;                    // optional: store pre (acc + bias), compute dtype
  double* stats;                        // optional: [2][N] (sum, sumsq) of pre (BN batch statistics)
  int act, M, N;
  RowMap rm;
  DEV void prepare(int) {}
  DEV void operator()(const float* ct, int LDT, int m0, int n0, int tid, int BM, int BN) const {
    for_segments(ct, LDT, BM, BN, m0, n0, M, N, tid, [&](int m, int n, const float* a, int, int) {
      float pv[8], v[8], o[8];
      long orow = rm.map(m);
#pragma unroll
      for (int e = 0; e < 8; e++) { pv[e] = a[e] + (bias ? bias[n + e] : 0.f); v[e] = pv[e] * (scale ? scale[n + e] : 1.f) + (shift ? shift[n + e] : 0.f); }
      if (pre) store8<TP>(pre + orow * ldp + n, pv);
      if (act >= ACT_GELU_BWD) {
        float r[8]; load8<TR>(res1 + orow * ldr1 + n, r);
#pragma unroll
        for (int e = 0; e < 8; e++) o[e] = act == ACT_GELU_BWD ? v[e] * gelu_erf_grad(r[e]) : (r[e] > 0.f ? v[e] : 0.f);
      } else {
#pragma unroll
        for (int e = 0; e < 8; e++) o[e] = act == ACT_RELU ? fmaxf(v[e], 0.f) : (act == ACT_GELU ? gelu_erf(v[e]) : v[e]);
        if (res1) { float r[8]; load8<TR>(res1 + orow * ldr1 + n, r);
#pragma unroll
          for (int e = 0; e < 8; e++) o[e] += r[e]; }
      }
      if (res2) { float r[8]; load8<TR>(res2 + orow * ldr2 + n, r);
#pragma unroll
        for (int e = 0; e < 8; e++) o[e] += r[e]; }
      store8<TO>(out + orow * ldo + coff + n, o);
    });
    if (stats) {
      // column statistics of pre over this tile's valid rows: 256 threads -> (col, row-phase)
      int nph = 256 / BN;
      int c = tid % BN, ph = tid / BN;
      int n = n0 + c;
      if (n < N) {
        float s = 0.f, q = 0.f;
        float bn_ = bias ? bias[n] : 0.f;
        for (int r = ph; r < BM; r += nph) {
          if (m0 + r >= M) break;
          float v = ct[r * LDT + c] + bn_;
          s += v; q += v * v;
        }
        atomicAdd(stats + n, (double)s);
        atomicAdd(stats + N + n, (double)q);
      }
    }
  }
};

// split-K wgrad epilogue: atomically accumulate into an fp32 gradient in PyTorch layout
//   dW[(m*Cx + cin)*taps + tap] += tile   where n = tap*Cx + cin   (Linear: taps=1)
struct EpiWgrad {
  float* dw; int M, N, Cx, taps;
  DEV void prepare(int) {}
  DEV void operator()(const float* ct, int LDT, int m0, int n0, int tid, int BM, int BN) const {
    const int total = BM * BN;
    for (int s = tid; s < total; s += 256) {
      int r = s / BN, c = s - r * BN;
      int m = m0 + r, n = n0 + c;
      if (m < M && n < N) {
        int tap = n / Cx, cin = n - tap * Cx;
        atomicAdd(dw + ((long)m * Cx + cin) * taps + tap, ct[r * LDT + c]);
      }
    }
  }
};

template <typename T, int BM, int BN, class LA, class LB, class EPI>
static int launch_igemm(LA la, LB lb, EPI epi, int M, int N, int KTILES, int split, int zdim_extra, hipStream_t st) {
  typedef GemmShape<T, BM, BN> S;
  auto kfn = igemm_kernel<T, BM, BN, LA, LB, EPI>;
  static bool attr = false;
  if (!attr) { (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, S::LDS); attr = true; }
  dim3 grid(cdiv(N, BN), cdiv(M, BM), split * zdim_extra);
  hipLaunchKernelGGL(kfn, grid, dim3(256), S::LDS, st, la, lb, epi, KTILES, split);
  return s3od_check_launch("igemm");
}
