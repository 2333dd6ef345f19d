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

constexpr int GEMM_THREADS = 512;          // 8 waves per workgroup (2 per SIMD)
constexpr int GEMM_WAVES = GEMM_THREADS / 64;
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
// Global -> LDS by LDS-DMA (global_load_lds_dwordx4): one wave instruction writes 1 KiB of LDS
// lane-linearly (wave base + lane*16), so the XOR swizzles are applied to the per-lane SOURCE
// address (guide §5.4 rule 21).  Out-of-range chunks (padding, tails) read a zero page.
// A tile of R rows is R*128 bytes: NIW = R*128/1024/GEMM_WAVES = R/64 instructions per wave.
//   KC image: instruction slot o = (wave*NIW + i)*1024 + lane*16 -> row o>>7, physical 16-B slot
//             (o>>4)&7, logical chunk = phys ^ ((row>>1)&7)
//   MC image: k-row o / RB, physical byte o % RB, logical 32-B slot = phys32 ^ g(k)
__device__ __attribute__((aligned(16))) uint4 g_s3od_zero[8];

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glob_void;
DEV void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((glob_void*)src, (lds_void*)lds_wave_base, 16, 0, 0);
}
DEV const void* zero_src() { return (const void*)g_s3od_zero; }

template <int RB> DEV int mc_logical_byte(int k, int phys) {
  constexpr int SLOTS = RB / 32;
  int g = ((k & 3) | (((k >> 3) & 1) << 2)) & (SLOTS - 1);
  return (((phys >> 5) ^ g) << 5) | (phys & 31);
}

template <typename T, int R> struct KCGeom {
  static constexpr int NIW = R * 128 / 1024 / GEMM_WAVES, EPC = 16 / sizeof(T), BK = KT<T>::BK;
  static_assert(NIW >= 1, "tile too small for the wave count");
  // row and logical element offset (within the k tile) of this lane's chunk of instruction i
  DEV static int row(int wave, int i, int lane) { return (wave * NIW + i) * 8 + (lane >> 3); }
  DEV static int kel(int wave, int i, int lane) { int r = row(wave, i, lane); return ((lane & 7) ^ ((r >> 1) & 7)) * EPC; }
};
template <typename T, int R> struct MCGeom {
  static constexpr int NIW = R * 128 / 1024 / GEMM_WAVES, RB = R * sizeof(T), BK = KT<T>::BK;
  DEV static int krow(int wave, int i, int lane) { return ((wave * NIW + i) * 1024 + lane * 16) / RB; }
  DEV static int col(int wave, int i, int lane) {
    int o = ((wave * NIW + i) * 1024 + lane * 16) % RB;
    return mc_logical_byte<RB>(krow(wave, i, lane), o) / (int)sizeof(T);
  }
};

template <typename T, int R> struct DenseKC {          // X[row*ld + k]
  static constexpr bool KCL = true, RELU = false;
  typedef KCGeom<T, R> G; static constexpr int NIW = G::NIW, BK = G::BK;
  const T* p; long ld; int nrows, K; int relu;
  const T* rowp[NIW]; int kel[NIW]; bool rv[NIW];
  DEV void setup(int t0, int tid) {
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      int r = t0 + G::row(wave, i, lane);
      rv[i] = r < nrows;
      rowp[i] = p + (long)(rv[i] ? r : 0) * ld;
      kel[i] = G::kel(wave, i, lane);
    }
  }
  DEV void issue(int kt, char* tile) {
    const int wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      int k = kt * BK + kel[i];
      const void* src = (rv[i] && k < K) ? (const void*)(rowp[i] + k) : zero_src();
      glds16(src, tile + (wave * NIW + i) * 1024);
    }
  }
};

template <typename T, int R> struct DenseMC {          // X[k*ld + col]
  static constexpr bool KCL = false, RELU = false;
  typedef MCGeom<T, R> G; static constexpr int NIW = G::NIW, BK = G::BK;
  const T* p; long ld; int K, ncols;
  int relu = 0;
  int kr[NIW], cl[NIW];
  DEV void setup(int t0, int tid) {
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int i = 0; i < NIW; i++) { kr[i] = G::krow(wave, i, lane); cl[i] = t0 + G::col(wave, i, lane); }
  }
  DEV void issue(int kt, char* tile) {
    const int wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      int k = kt * BK + kr[i];
      const void* src = (k < K && cl[i] < ncols) ? (const void*)(p + (long)k * ld + cl[i]) : zero_src();
      glds16(src, tile + (wave * NIW + i) * 1024);
    }
  }
};

// conv forward A operand: rows = output pixels (b,oy,ox) of RH x RW, k = tap*SC + c
template <typename T, int R, bool RELU_ = false> struct ConvFwdA {
  static constexpr bool KCL = true, RELU = RELU_;
  typedef KCGeom<T, R> G; static constexpr int NIW = G::NIW, BK = G::BK;
  const T* x; ConvGeo g; int M; int relu;
  int rb[NIW], ry[NIW], rx[NIW];
  int tap[NIW], c[NIW];     // incremental k -> (tap, channel) per chunk
  DEV void setup(int t0, int tid) {
    const int lane = tid & 63, wave = tid >> 6;
    int hw = g.RH * g.RW;
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      int m = t0 + G::row(wave, i, lane);
      if (m < M) { int b = m / hw; int r = m - b * hw; int oy = r / g.RW; rb[i] = b; ry[i] = oy * g.s - g.p; rx[i] = (r - oy * g.RW) * g.s - g.p; }
      else { rb[i] = -1; ry[i] = 0; rx[i] = 0; }
      tap[i] = -1; c[i] = G::kel(wave, i, lane);
    }
  }
  DEV void issue(int kt, char* tile) {
    const int wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      if (tap[i] < 0) { int k = kt * BK + c[i]; tap[i] = k / g.SC; c[i] = k - tap[i] * g.SC; }
      int kh = tap[i] / g.KW, kw = tap[i] - kh * g.KW;
      int iy = ry[i] + kh, ix = rx[i] + kw;
      bool ok = tap[i] < g.KH * g.KW && rb[i] >= 0 && iy >= 0 && iy < g.SH && ix >= 0 && ix < g.SW;
      const void* src = ok ? (const void*)(x + (((long)rb[i] * g.SH + iy) * g.SW + ix) * g.SC + c[i]) : zero_src();
      glds16(src, tile + (wave * NIW + i) * 1024);
      c[i] += BK; while (c[i] >= g.SC) { c[i] -= g.SC; tap[i]++; }
    }
  }
};

// dgrad / ConvT A operand: rows = class pixels (b, y', x'), k = (jh*ntw + jw)*SC + c
template <typename T, int R> struct ConvDgradA {
  static constexpr bool KCL = true, RELU = false;
  typedef KCGeom<T, R> G; static constexpr int NIW = G::NIW, BK = G::BK;
  const T* dy; ConvGeo g; int M;
  int relu = 0;
  int rb[NIW], ry[NIW], rx[NIW];
  int tap[NIW], c[NIW];
  DEV void setup(int t0, int tid) {
    const int lane = tid & 63, wave = tid >> 6;
    int hw = g.RH * g.RW;
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      int m = t0 + G::row(wave, i, lane);
      if (m < M) { int b = m / hw; int r = m - b * hw; int yy = r / g.RW; rb[i] = b; ry[i] = yy + g.qy0; rx[i] = (r - yy * g.RW) + g.qx0; }
      else { rb[i] = -1; ry[i] = 0; rx[i] = 0; }
      tap[i] = -1; c[i] = G::kel(wave, i, lane);
    }
  }
  DEV void issue(int kt, char* tile) {
    const int wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      if (tap[i] < 0) { int k = kt * BK + c[i]; tap[i] = k / g.SC; c[i] = k - tap[i] * g.SC; }
      int jh = g.ntw ? tap[i] / g.ntw : 0, jw = tap[i] - jh * g.ntw;
      int sy = ry[i] - jh, sx = rx[i] - jw;
      bool ok = tap[i] < g.nth * g.ntw && rb[i] >= 0 && sy >= 0 && sy < g.SH && sx >= 0 && sx < g.SW;
      const void* src = ok ? (const void*)(dy + (((long)rb[i] * g.SH + sy) * g.SW + sx) * g.SC + c[i]) : zero_src();
      glds16(src, tile + (wave * NIW + i) * 1024);
      c[i] += BK; while (c[i] >= g.SC) { c[i] -= g.SC; tap[i]++; }
    }
  }
};

// dgrad / ConvT B operand (MC): B[k=(jh,jw,c)][n] = W[c][kh0+s*jh][kw0+s*jw][n], W repacked [C][KH][KW][N]
template <typename T, int R> struct ConvDgradB {
  static constexpr bool KCL = false, RELU = false;
  typedef MCGeom<T, R> G; static constexpr int NIW = G::NIW, BK = G::BK;
  const T* w; ConvGeo g; int NC;     // NC = output channels of the dgrad (= conv input channels)
  int relu = 0;
  int kr[NIW], cl[NIW];
  DEV void setup(int t0, int tid) {
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int i = 0; i < NIW; i++) { kr[i] = G::krow(wave, i, lane); cl[i] = t0 + G::col(wave, i, lane); }
  }
  DEV void issue(int kt, char* tile) {
    const int wave = threadIdx.x >> 6;
    const int K = g.nth * g.ntw * g.SC;
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      int k = kt * BK + kr[i];
      const void* src = zero_src();
      if (k < K && cl[i] < NC) {
        int t = k / g.SC, cc = k - t * g.SC;
        int jh = t / g.ntw, jw = t - jh * g.ntw;
        int kh = g.kh0 + g.s * jh, kw = g.kw0 + g.s * jw;
        src = (const void*)(w + (((long)cc * g.KH + kh) * g.KW + kw) * NC + cl[i]);
      }
      glds16(src, tile + (wave * NIW + i) * 1024);
    }
  }
};

// wgrad B operand (MC gather): B[k=pix of the conv output grid RH x RW][n=(tap, cin)] = X[src][cin]
template <typename T, int R, bool RELU_ = false> struct WgradB {
  static constexpr bool KCL = false, RELU = RELU_;
  typedef MCGeom<T, R> G; static constexpr int NIW = G::NIW, BK = G::BK;
  const T* x; ConvGeo g; int NPIX; int relu;   // g.SC = Cin of X, g.SH/SW = X dims, RH/RW = output grid
  int kh[NIW], kw[NIW], cin[NIW], kr[NIW]; bool cval[NIW];
  int pb[NIW], py[NIW], pxx[NIW]; int started;
  DEV void setup(int t0, int tid) {
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      int col = t0 + G::col(wave, i, lane);
      kr[i] = G::krow(wave, i, lane);
      int tp = col / g.SC; cin[i] = col - tp * g.SC; kh[i] = tp / g.KW; kw[i] = tp - kh[i] * g.KW;
      cval[i] = tp < g.KH * g.KW;
    }
    started = 0;
  }
  DEV void issue(int kt, char* tile) {
    const int wave = threadIdx.x >> 6;
    if (!started) {
      started = 1;
      const int hw = g.RH * g.RW;
#pragma unroll
      for (int i = 0; i < NIW; i++) {
        int k = kt * BK + kr[i];
        int b = k / hw; int r = k - b * hw; int oy = r / g.RW;
        pb[i] = b; py[i] = oy; pxx[i] = r - oy * g.RW;
      }
    }
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      int iy = py[i] * g.s - g.p + kh[i], ix = pxx[i] * g.s - g.p + kw[i];
      bool ok = cval[i] && pb[i] < g.B && iy >= 0 && iy < g.SH && ix >= 0 && ix < g.SW;
      const void* src = ok ? (const void*)(x + (((long)pb[i] * g.SH + iy) * g.SW + ix) * g.SC + cin[i]) : zero_src();
      glds16(src, tile + (wave * NIW + i) * 1024);
      pxx[i] += BK;
      while (pxx[i] >= g.RW) { pxx[i] -= g.RW; if (++py[i] >= g.RH) { py[i] = 0; pb[i]++; } }
    }
    (void)NPIX;
  }
};

DEV bf16x8 relu_frag(bf16x8 v) {
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  u4 w = __builtin_bit_cast(u4, v);
#pragma unroll
  for (int i = 0; i < 4; i++) { unsigned m = (w[i] >> 15) & 0x00010001u; w[i] &= ~(m * 0xFFFFu); }
  return __builtin_bit_cast(bf16x8, w);
}
DEV float relu_frag(float v) { return fmaxf(v, 0.f); }

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
template <typename T, int BM, int BN, int NST_ = 3> struct GemmShape {
  static constexpr int BK = KT<T>::BK;
  static constexpr int ABYTES = BM * 128, BBYTES = BN * 128;
  static constexpr int STAGE = ABYTES + BBYTES;
  static constexpr int NST = NST_;
  static constexpr int LDT = BN + 4;                       // fp32 C-tile row stride
  static constexpr int CBYTES = BM * LDT * 4;
  static constexpr int LDS = (NST * STAGE > CBYTES ? NST * STAGE : CBYTES);
  // wave grid: 8 waves as WM x WN
  static constexpr int WM = BM >= 2 * BN ? 4 : (BN >= 2 * BM ? 2 : (BM >= BN ? 4 : 2));
  static constexpr int WN = GEMM_WAVES / WM;
  static constexpr int TM = BM / WM, TN = BN / WN;         // per-wave tile
  static constexpr int MI = TM / 16, NI = TN / 16;
  static_assert(MI >= 1 && NI >= 1 && TM % 16 == 0 && TN % 16 == 0, "bad wave tiling");
};

struct KRange { int kt0, kt1; };

template <int N> DEV void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
DEV void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Block-level epilogue contract:  epi(tile, LDT, m0, n0, tid, BM, BN)
//
// Main loop: 3 LDS stages filled by LDS-DMA two K-tiles ahead; one raw s_barrier per K tile,
// placed BEFORE the last k-step's MFMAs so the next tile's first fragments are read from LDS
// while the current tile's last MFMAs run (fragments double-buffered in registers).
// vmcnt is counted (the tile two steps ahead stays in flight across the barrier); there is
// no __syncthreads() in the loop (it would drain vmcnt to 0: guide §5).
// Block order is remapped so consecutive tiles of one row-panel share an XCD (guide T1).
template <typename T, int BM, int BN, int NST, class LA, class LB, class EPI>
__global__ void __launch_bounds__(GEMM_THREADS) igemm_kernel(LA la, LB lb, EPI epi, int KTILES, int split) {
  typedef GemmShape<T, BM, BN, NST> S;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / S::WN, wn = wave % S::WN;
  constexpr int MI = S::MI, NI = S::NI, KS = Mma<T>::KSTEPS;
  constexpr int NL = LA::NIW + LB::NIW;       // LDS-DMA instructions per thread per K tile
  int bx, by;
  {
    const int nwg = gridDim.x * gridDim.y;
    const int L = blockIdx.y * gridDim.x + blockIdx.x;
    const int q = nwg >> 3, r = nwg & 7, xcd = L & 7, idx = L >> 3;
    const int W = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
    bx = W % gridDim.x; by = W / gridDim.x;
  }
  const int m0 = by * BM, n0 = bx * BN;
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

  typedef typename Mma<T>::frag frag;
  frag fa[2][MI], fb[2][NI];
  auto read_frags = [&](int buf, const char* stage, int kk) {
    const char* As = stage;
    const char* Bs = stage + S::ABYTES;
#pragma unroll
    for (int i = 0; i < MI; i++) fa[buf][i] = Frag<T, LA::KCL, BM>::read(As, wm * S::TM + i * 16, kk, lane);
#pragma unroll
    for (int j = 0; j < NI; j++) fb[buf][j] = Frag<T, LB::KCL, BN>::read(Bs, wn * S::TN + j * 16, kk, lane);
  };
  auto mfmas = [&](int buf) {
    if constexpr (LA::RELU) {
#pragma unroll
      for (int i = 0; i < MI; i++) fa[buf][i] = relu_frag(fa[buf][i]);
    }
    if constexpr (LB::RELU) {
#pragma unroll
      for (int j = 0; j < NI; j++) fb[buf][j] = relu_frag(fb[buf][j]);
    }
#pragma unroll
    for (int i = 0; i < MI; i++)
#pragma unroll
      for (int j = 0; j < NI; j++) acc[i][j] = Mma<T>::mma(fa[buf][i], fb[buf][j], acc[i][j]);
  };

  const int nt = kt1 - kt0;
  constexpr int PD = NST - 1;                 // LDS-DMA prefetch distance (tiles in flight)
  if (nt > 0) {
    // prologue: tiles 0 .. PD-1
#pragma unroll
    for (int q = 0; q < PD; q++)
      if (q < nt) { la.issue(kt0 + q, smem + q * S::STAGE); lb.issue(kt0 + q, smem + q * S::STAGE + S::ABYTES); }
    if constexpr (PD == 2) { if (nt > 1) wait_vmcnt<NL>(); else wait_vmcnt<0>(); }
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    read_frags(0, smem, 0);
    int cur = 0;
    for (int t = 0; t < nt; ++t) {
      const bool pre = t + PD < nt;
      if (pre) {
        int st = cur + PD; if (st >= NST) st -= NST;
        char* nx = smem + st * S::STAGE;
        la.issue(kt0 + t + PD, nx);
        lb.issue(kt0 + t + PD, nx + S::ABYTES);
      }
      const char* stg = smem + cur * S::STAGE;
      int nxt = cur + 1; if (nxt >= NST) nxt -= NST;
#pragma unroll
      for (int kk = 0; kk < KS; kk++) {
        const int b = kk & 1;
        if (kk + 1 < KS) {
          read_frags(b ^ 1, stg, kk + 1);
        } else if (t + 1 < nt) {
          // tile t+1 landed (own DMAs): PD-1 newer tiles may stay in flight
          if constexpr (PD == 2) { if (pre) wait_vmcnt<NL>(); else wait_vmcnt<0>(); }
          else wait_vmcnt<0>();
          wait_lgkm0();
          __builtin_amdgcn_s_barrier();
          read_frags(b ^ 1, smem + nxt * S::STAGE, 0);
        }
        mfmas(b);
      }
      cur = nxt;
    }
  }
  __syncthreads();
  // stage C tile to LDS (fp32)
  float* ct = (float*)smem;
#pragma unroll
  for (int i = 0; i < MI; i++)
#pragma unroll
    for (int j = 0; j < NI; j++) {
      int r = wm * S::TM + i * 16 + (lane >> 4) * 4;
      int c = wn * S::TN + j * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; e++) ct[(r + e) * S::LDT + c] = acc[i][j][e];
    }
  __syncthreads();
  epi(ct, S::LDT, m0, n0, tid, BM, BN);
}

// iterate 8-wide row segments of the staged tile: f(m, n, const float* v8)
template <class F> DEV void for_segments(const float* ct, int LDT, int BM, int BN, int m0, int n0, int M, int N, int tid, F f) {
  const int segs = BM * BN / 8, spr = BN / 8;
  for (int s = tid; s < segs; s += GEMM_THREADS) {
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
      int nph = GEMM_THREADS / BN;
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
    for (int s = tid; s < total; s += GEMM_THREADS) {
      int r = s / BN, c = s - r * BN;
      int m = m0 + r, n = n0 + c;
      if (m < M && n < N) {
        int tap = n / Cx, cin = n - tap * Cx;
        atomicAdd(dw + ((long)m * Cx + cin) * taps + tap, ct[r * LDT + c]);
      }
    }
  }
};

template <typename T, int BM, int BN, class LA, class LB, class EPI, int NST = 3>
static int launch_igemm(LA la, LB lb, EPI epi, int M, int N, int KTILES, int split, int zdim_extra, hipStream_t st) {
  typedef GemmShape<T, BM, BN, NST> S;
  auto kfn = igemm_kernel<T, BM, BN, NST, LA, LB, EPI>;
  static bool attr = false;
  if (!attr) { (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, S::LDS); attr = true; }
  dim3 grid(cdiv(N, BN), cdiv(M, BM), split * zdim_extra);
  hipLaunchKernelGGL(kfn, grid, dim3(GEMM_THREADS), S::LDS, st, la, lb, epi, KTILES, split);
  return s3od_check_launch("igemm");
}
