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
#include <algorithm>

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

// ReLU of two packed bf16: a bf16 with the sign bit set is a negative int16, so a signed 16-bit max against
// 0 is ReLU (-0 -> +0) -- one v_pk_max_i16 per dword instead of a mask / select sequence
typedef short s16x2_t __attribute__((ext_vector_type(2)));
DEV unsigned relu_bf16x2(unsigned x) {
  return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(s16x2_t, x), (s16x2_t){0, 0}));
}
template <typename T> DEV uint4 relu16(uint4 v) {
  if constexpr (sizeof(T) == 2) {
    return make_uint4(relu_bf16x2(v.x), relu_bf16x2(v.y), relu_bf16x2(v.z), relu_bf16x2(v.w));
  } else {
    float4 f = *(float4*)&v;
    f.x = fmaxf(f.x, 0.f); f.y = fmaxf(f.y, 0.f); f.z = fmaxf(f.z, 0.f); f.w = fmaxf(f.w, 0.f);
    return *(uint4*)&f;
  }
}

// ------------------------------------------------------------------ operand loaders
// Global -> LDS by LDS-DMA through a buffer resource (buffer_load_dwordx4 ... lds): one wave
// instruction writes 1 KiB of LDS lane-linearly (M0 = wave base, + lane*16), so the XOR
// swizzles are applied to the per-lane SOURCE offset (guide §5.4 rule 21).
//   * the descriptor (base, byte size) is built from kernel arguments only -> SGPRs;
//   * each lane keeps a 32-bit byte offset that is advanced by a uniform step per K tile, so the
//     steady-state address cost is ~1 VALU per load (no 64-bit pointer math);
//   * out-of-range chunks (padding taps, row/column tails) use an offset beyond the descriptor's
//     size: the hardware range check returns zeros (no zero page, no per-load select);
//   * the wave index is readfirstlane'd so every M0 value is computed on the scalar unit.
// A tile of R rows is R*128 bytes: NIW = R*128/1024/GEMM_WAVES = R/64 instructions per wave.
//   KC image: instruction slot o = (wave*NIW + i)*1024 + lane*16 -> row o>>7, physical 16-B slot
//             (o>>4)&7, logical chunk = phys ^ ((row>>1)&7)
//   MC image: k-row o / RB, physical byte o % RB, logical 32-B slot = phys32 ^ g(k)
// Operands must be < 3.75 GiB (checked on the host by buf_ok()).
constexpr unsigned long BUF_MAX = 0xF0000000ul;
constexpr unsigned BUF_OOB = 0xF8000000u;      // any offset >= BUF_MAX reads zeros

typedef __attribute__((address_space(3))) void lds_void;
DEV __amdgpu_buffer_rsrc_t make_rsrc(const void* p, unsigned long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(unsigned)(bytes < BUF_MAX ? bytes : BUF_MAX), 0x00020000);
}
DEV void blds16(__amdgpu_buffer_rsrc_t r, unsigned voff, char* lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds_wave_base, 16, voff, 0, 0, 0);
}
DEV int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// Where a loader's 16-B-per-lane chunk i goes: every loader computes one buffer offset per chunk (source-side
// swizzle, OOB -> zeros) and hands it to the sink, which LDS-DMAs it straight into the lane-linear LDS image
// (buffer_load_dwordx4 ... lds).
struct DmaSink {
  char* base;                                    // tile + wave * NIW * 1024
  DEV void operator()(int i, __amdgpu_buffer_rsrc_t r, unsigned voff) const { blds16(r, voff, base + i * 1024); }
};
#define HD __host__ __device__

// 8 x 32-pixel output tiles of the 3x3 halo weight-gradient kernels (gemm_ops.hip, wgrad_dma.hip)
constexpr int HT_TH = 8, HT_TW = 32, HT_HR = HT_TH + 2, HT_HC = HT_TW + 2, HT_PX = HT_HR * HT_HC;
// LDS-DMA 3x3 weight gradient, 64 x 64 channel blocks (wgrad_dma.hip; needs H % 8 == 0, W % 32 == 0)
int wgrad3x3_dma_launch(bool relu_x, const bf16* dy, const bf16* x, float* ws, int B, int H, int W, int CinT, int CoT,
                        hipStream_t st);

template <int RB> DEV int mc_logical_byte(int k, int phys) {
  constexpr int SLOTS = RB / 32;
  int g = ((k & 3) | (((k >> 3) & 1) << 2)) & (SLOTS - 1);
  return (((phys >> 5) ^ g) << 5) | (phys & 31);
}

template <typename T, int R, int NW = GEMM_WAVES> struct KCGeom {
  static constexpr int NIW = R * 128 / 1024 / NW, EPC = 16 / sizeof(T), BK = KT<T>::BK;
  static_assert(NIW >= 1, "tile too small for the wave count");
  // row and logical element offset (within the k tile) of this lane's chunk of instruction i
  DEV static int row(int wave, int i, int lane) { return (wave * NIW + i) * 8 + (lane >> 3); }
  DEV static int kel(int wave, int i, int lane) { int r = row(wave, i, lane); return ((lane & 7) ^ ((r >> 1) & 7)) * EPC; }
};
template <typename T, int R, int NW = GEMM_WAVES> struct MCGeom {
  static constexpr int NIW = R * 128 / 1024 / NW, RB = R * sizeof(T), BK = KT<T>::BK;
  DEV static int krow(int wave, int i, int lane) { return ((wave * NIW + i) * 1024 + lane * 16) / RB; }
  DEV static int col(int wave, int i, int lane) {
    int o = ((wave * NIW + i) * 1024 + lane * 16) % RB;
    return mc_logical_byte<RB>(krow(wave, i, lane), o) / (int)sizeof(T);
  }
};

template <typename T, int R, int NW = GEMM_WAVES> struct DenseKC {          // X[row*ld + k]
  static constexpr int ROWS = R;
  static constexpr bool KCL = true, RELU = false;
  typedef KCGeom<T, R, NW> G; static constexpr int NIW = G::NIW, BK = G::BK;
  const T* p; long ld; int nrows, K; int relu;
  const T* pb; unsigned long nb;           // this block's row window (descriptor rebased per block)
  unsigned vo[NIW]; int kel[NIW];
  // the descriptor only ever spans the R rows of one block, so the tensor itself may exceed 4 GiB
  HD unsigned long bytes() const { return ((unsigned long)(R - 1) * ld + K) * sizeof(T); }
  HD bool buf_ok() const { return bytes() < BUF_MAX && (unsigned long)K * sizeof(T) < 0x4000000ul; }
  DEV void setup(int t0, int tid) {
    const int lane = tid & 63, wave = wave_id();
    const int rem = nrows - t0;
    pb = p + (long)t0 * ld;
    nb = rem > 0 ? ((unsigned long)(min(rem, R) - 1) * ld + K) * sizeof(T) : 0;
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      int r = G::row(wave, i, lane);
      kel[i] = G::kel(wave, i, lane);
      vo[i] = r < rem ? (unsigned)(((long)r * ld + kel[i]) * sizeof(T)) : BUF_OOB;
    }
  }
  DEV void issue(int kt, char* tile) { issue_to(kt, DmaSink{tile + wave_id() * NIW * 1024}); }
  template <class SK> DEV void issue_to(int kt, SK sk) {
    const auto rs = make_rsrc(pb, nb);
    const unsigned adv = (unsigned)(kt * BK * sizeof(T));
    if ((kt + 1) * BK > K) {          // K tail (uniform branch)
#pragma unroll
      for (int i = 0; i < NIW; i++) sk(i, rs, kt * BK + kel[i] < K ? vo[i] + adv : BUF_OOB);
      return;
    }
#pragma unroll
    for (int i = 0; i < NIW; i++) sk(i, rs, vo[i] + adv);
  }
};

template <typename T, int R, int NW = GEMM_WAVES> struct DenseMC {          // X[k*ld + col]
  static constexpr int ROWS = R;
  static constexpr bool KCL = false, RELU = false;
  typedef MCGeom<T, R, NW> G; static constexpr int NIW = G::NIW, BK = G::BK;
  const T* p; long ld; int K, ncols;
  int relu = 0;
  unsigned vo[NIW]; int kr[NIW]; bool cv[NIW];
  // the descriptor is rebased to each K tile's first row: only BK rows need to be addressable
  HD unsigned long total() const { return ((unsigned long)(K - 1) * ld + ncols) * sizeof(T); }
  HD unsigned long bytes() const { return ((unsigned long)BK * ld) * sizeof(T); }
  HD bool buf_ok() const { return bytes() < BUF_MAX; }
  DEV void setup(int t0, int tid) {
    const int lane = tid & 63, wave = wave_id();
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      kr[i] = G::krow(wave, i, lane);
      int cl = t0 + G::col(wave, i, lane);
      cv[i] = cl < ncols;
      vo[i] = (unsigned)(((long)kr[i] * ld + cl) * sizeof(T));
    }
  }
  DEV void issue(int kt, char* tile) { issue_to(kt, DmaSink{tile + wave_id() * NIW * 1024}); }
  template <class SK> DEV void issue_to(int kt, SK sk) {
    const long e0 = (long)kt * BK * ld;
    const auto rs = make_rsrc(p + e0, total() - (unsigned long)e0 * sizeof(T));
    if ((kt + 1) * BK > K) {          // K tail (uniform branch)
#pragma unroll
      for (int i = 0; i < NIW; i++) sk(i, rs, cv[i] && kt * BK + kr[i] < K ? vo[i] : BUF_OOB);
      return;
    }
#pragma unroll
    for (int i = 0; i < NIW; i++) sk(i, rs, cv[i] ? vo[i] : BUF_OOB);
  }
};

// Image window of a gather: a block (or K tile) whose rows cover pixels [first, last] of a batch of
// images of `hw` pixels reads images first/hw .. last/hw only.  The descriptor is rebased to the
// first of them, so only that window (not the whole batch) must stay below BUF_MAX.
HD inline unsigned long img_window_bytes(int rows, int hw, int B, unsigned long img_bytes) {
  long n = (long)(rows - 1) / hw + 2;
  return (unsigned long)(n < B ? n : B) * img_bytes;
}

// Incremental K-tile -> (tap, channel base) walker for gathers whose K is tap-major with
// SC % BK == 0: a whole K tile then lies inside one tap, so tap/channel are wave-uniform.
struct TapWalk {
  int nk = -1, tap = 0, c0 = 0, th = 0, tw = 0;
  // returns true when the tap changed (per-lane validity must be recomputed)
  DEV bool step(int kt, int BK, int SC, int TW) {
    if (kt != nk) {
      int k = kt * BK; tap = k / SC; c0 = k - tap * SC; th = tap / TW; tw = tap - th * TW;
      nk = kt + 1; return true;
    }
    nk = kt + 1;
    c0 += BK;
    if (c0 < SC) return false;
    c0 = 0; tap++;
    if (++tw == TW) { tw = 0; th++; }
    return true;
  }
  // generic (SC % BK != 0, 2 SC >= BK): advance by BK channels, a tile spans taps tap and tap+1
  DEV void step_any(int kt, int BK, int SC, int TW) {
    if (kt != nk) { int k = kt * BK; tap = k / SC; c0 = k - tap * SC; th = tap / TW; tw = tap - th * TW; }
    else { c0 += BK; while (c0 >= SC) { c0 -= SC; tap++; if (++tw == TW) { tw = 0; th++; } } }
    nk = kt + 1;
  }
  DEV void next_tap(int TW, int& th1, int& tw1) const { tw1 = tw + 1; th1 = th; if (tw1 == TW) { tw1 = 0; th1++; } }
};

// conv forward A operand: rows = output pixels (b,oy,ox) of RH x RW, k = tap*SC + c
template <typename T, int R, bool RELU_ = false, int NW = GEMM_WAVES> struct ConvFwdA {
  static constexpr int ROWS = R;
  static constexpr bool KCL = true, RELU = RELU_;
  typedef KCGeom<T, R, NW> G; static constexpr int NIW = G::NIW, BK = G::BK;
  const T* x; ConvGeo g; int M; int relu;
  const T* xb; unsigned long nb;          // image window of this block (rebased descriptor)
  int iy0[NIW], ix0[NIW], pix0[NIW];      // top-left input pixel (may be outside) and its element offset + kel
  int kl[NIW];
  unsigned base[NIW];
  TapWalk tw;
  HD unsigned long img_bytes() const { return (unsigned long)g.SH * g.SW * g.SC * sizeof(T); }
  HD unsigned long bytes() const { return img_window_bytes(R, g.RH * g.RW, g.B, img_bytes()); }
  HD bool buf_ok() const { return bytes() < BUF_MAX && 2 * g.SC >= BK; }
  DEV void setup(int t0, int tid) {
    const int lane = tid & 63, wave = wave_id();
    int hw = g.RH * g.RW;
    const int b0 = min(t0, M - 1) / hw, b1 = min(t0 + R - 1, M - 1) / hw;
    xb = x + (long)b0 * g.SH * g.SW * g.SC;
    nb = (unsigned long)(b1 - b0 + 1) * img_bytes();
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      int m = t0 + G::row(wave, i, lane);
      int kel = G::kel(wave, i, lane);
      kl[i] = kel;
      if (m < M) {
        int b = m / hw; int r = m - b * hw; int oy = r / g.RW;
        iy0[i] = oy * g.s - g.p; ix0[i] = (r - oy * g.RW) * g.s - g.p;
        pix0[i] = (((b - b0) * g.SH + iy0[i]) * g.SW + ix0[i]) * g.SC + kel;
      } else { iy0[i] = -0x4000000; ix0[i] = 0; pix0[i] = 0; }
    }
    tw = TapWalk{};
  }
  DEV void issue(int kt, char* tile) { issue_to(kt, DmaSink{tile + wave_id() * NIW * 1024}); }
  template <class SK> DEV void issue_to(int kt, SK sk) {
    const auto rs = make_rsrc(xb, nb);
    if (g.SC % BK) {                 // channels not a multiple of BK: per-lane tap (rare shapes)
      tw.step_any(kt, BK, g.SC, g.KW);
      int th1, tw1; tw.next_tap(g.KW, th1, tw1);
#pragma unroll
      for (int i = 0; i < NIW; i++) {
        int c = tw.c0 + kl[i];
        bool wr = c >= g.SC;
        int th = wr ? th1 : tw.th, tww = wr ? tw1 : tw.tw;
        int iy = iy0[i] + th, ix = ix0[i] + tww;
        bool ok = tw.tap + (int)wr < g.KH * g.KW && (unsigned)iy < (unsigned)g.SH && (unsigned)ix < (unsigned)g.SW;
        int off = pix0[i] - kl[i] + (th * g.SW + tww) * g.SC + (wr ? c - g.SC : c);
        sk(i, rs, ok ? (unsigned)off * (unsigned)sizeof(T) : BUF_OOB);
      }
      return;
    }
    if (tw.step(kt, BK, g.SC, g.KW)) {
      const bool tv = tw.tap < g.KH * g.KW;
      const int toff = (tw.th * g.SW + tw.tw) * g.SC;
#pragma unroll
      for (int i = 0; i < NIW; i++) {
        int iy = iy0[i] + tw.th, ix = ix0[i] + tw.tw;
        bool ok = tv && (unsigned)iy < (unsigned)g.SH && (unsigned)ix < (unsigned)g.SW;
        base[i] = ok ? (unsigned)(pix0[i] + toff) * (unsigned)sizeof(T) : BUF_OOB;
      }
    }
    const unsigned cb = (unsigned)(tw.c0 * sizeof(T));
#pragma unroll
    for (int i = 0; i < NIW; i++) sk(i, rs, base[i] + cb);
  }
};

// 3x3 / stride 1 / pad 1 conv forward A operand for the 256x256 ping-pong kernel (bf16, SC a power-of-two multiple
// of BK): rows = output pixels (b, oy, ox) of H x W, k = tap*SC + c.  Per lane and chunk only the element offset of
// the CENTRE pixel is kept, plus a 9-bit tap-validity mask (every chunk's mask in one register), so a K tile's
// offset is pix + a uniform (tap, channel) step and ConvFwdA's per-lane walker state (which spills beside the
// ping-pong body's 240 live registers) is gone.
template <int R, bool RELU_ = false, int NW = GEMM_WAVES> struct Conv3A {
  static constexpr int ROWS = R;
  static constexpr bool KCL = true, RELU = RELU_;
  typedef KCGeom<bf16, R, NW> G; static constexpr int NIW = G::NIW, BK = G::BK;
  static_assert(NIW <= 3, "the tap masks of at most 3 chunks share one register");
  const bf16* x; int B, H, W, SC, M, lgc;   // lgc = log2(SC / BK)
  const bf16* xb; unsigned long nb;        // image window of this block (rebased descriptor)
  int pix[NIW]; unsigned mask;
  HD unsigned long img_bytes() const { return (unsigned long)H * W * SC * 2; }
  HD bool buf_ok() const { return img_window_bytes(R, H * W, B, img_bytes()) < BUF_MAX && (BK << lgc) == SC; }
  DEV void setup(int t0, int tid) {
    const int lane = tid & 63, wave = wave_id(), hw = H * W;
    const int b0 = min(t0, M - 1) / hw, b1 = min(t0 + R - 1, M - 1) / hw;
    xb = x + (long)b0 * hw * SC;
    nb = (unsigned long)(b1 - b0 + 1) * img_bytes();
    mask = 0;
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      const int m = t0 + G::row(wave, i, lane);
      pix[i] = 0;
      if (m < M) {
        const int b = m / hw, r = m - b * hw, oy = r / W, ox = r - oy * W;
        pix[i] = ((b - b0) * hw + r) * SC + G::kel(wave, i, lane);
        unsigned mk = 0;
#pragma unroll
        for (int t = 0; t < 9; t++)
          if ((unsigned)(oy + t / 3 - 1) < (unsigned)H && (unsigned)(ox + t % 3 - 1) < (unsigned)W) mk |= 1u << t;
        mask |= mk << (10 * i);
      }
    }
  }
  DEV void issue(int kt, char* tile) { issue_to(kt, DmaSink{tile + wave_id() * NIW * 1024}); }
  template <class SK> DEV void issue_to(int kt, SK sk) {
    const auto rs = make_rsrc(xb, nb);
    const int tap = kt >> lgc, c0 = (kt - (tap << lgc)) * BK;
    const int ty = tap / 3, tx = tap - 3 * ty;
    const int toff = ((ty - 1) * W + (tx - 1)) * SC + c0;
#pragma unroll
    for (int i = 0; i < NIW; i++) sk(i, rs, ((mask >> (10 * i + tap)) & 1u) ? (unsigned)(pix[i] + toff) * 2u : BUF_OOB);
  }
};

// dgrad / ConvT A operand: rows = class pixels (b, y', x'), k = (jh*ntw + jw)*SC + c
template <typename T, int R, int NW = GEMM_WAVES> struct ConvDgradA {
  static constexpr int ROWS = R;
  static constexpr bool KCL = true, RELU = false;
  typedef KCGeom<T, R, NW> G; static constexpr int NIW = G::NIW, BK = G::BK;
  const T* dy; ConvGeo g; int M;
  int relu = 0;
  const T* yb; unsigned long nb;          // image window of this block (rebased descriptor)
  int ry[NIW], rx[NIW], pix0[NIW], kl[NIW];
  unsigned base[NIW];
  TapWalk tw;
  HD unsigned long img_bytes() const { return (unsigned long)g.SH * g.SW * g.SC * sizeof(T); }
  HD unsigned long bytes() const { return img_window_bytes(R, g.RH * g.RW, g.B, img_bytes()); }
  HD bool buf_ok() const { return bytes() < BUF_MAX && 2 * g.SC >= BK; }
  DEV void setup(int t0, int tid) {
    const int lane = tid & 63, wave = wave_id();
    int hw = g.RH * g.RW;
    const int b0 = min(t0, M - 1) / hw, b1 = min(t0 + R - 1, M - 1) / hw;
    yb = dy + (long)b0 * g.SH * g.SW * g.SC;
    nb = (unsigned long)(b1 - b0 + 1) * img_bytes();
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      int m = t0 + G::row(wave, i, lane);
      int kel = G::kel(wave, i, lane);
      kl[i] = kel;
      if (m < M) {
        int b = m / hw; int r = m - b * hw; int yy = r / g.RW;
        ry[i] = yy + g.qy0; rx[i] = (r - yy * g.RW) + g.qx0;
        pix0[i] = (((b - b0) * g.SH + ry[i]) * g.SW + rx[i]) * g.SC + kel;
      } else { ry[i] = -0x4000000; rx[i] = 0; pix0[i] = 0; }
    }
    tw = TapWalk{};
  }
  DEV void issue(int kt, char* tile) { issue_to(kt, DmaSink{tile + wave_id() * NIW * 1024}); }
  template <class SK> DEV void issue_to(int kt, SK sk) {
    const auto rs = make_rsrc(yb, nb);
    const int TW = g.ntw > 0 ? g.ntw : 1;
    if (g.SC % BK) {                 // channels not a multiple of BK: per-lane tap (rare shapes)
      tw.step_any(kt, BK, g.SC, TW);
      int th1, tw1; tw.next_tap(TW, th1, tw1);
#pragma unroll
      for (int i = 0; i < NIW; i++) {
        int c = tw.c0 + kl[i];
        bool wr = c >= g.SC;
        int th = wr ? th1 : tw.th, tww = wr ? tw1 : tw.tw;
        int sy = ry[i] - th, sx = rx[i] - tww;
        bool ok = tw.tap + (int)wr < g.nth * g.ntw && (unsigned)sy < (unsigned)g.SH && (unsigned)sx < (unsigned)g.SW;
        int off = pix0[i] - kl[i] - (th * g.SW + tww) * g.SC + (wr ? c - g.SC : c);
        sk(i, rs, ok ? (unsigned)off * (unsigned)sizeof(T) : BUF_OOB);
      }
      return;
    }
    if (tw.step(kt, BK, g.SC, TW)) {
      const bool tv = tw.tap < g.nth * g.ntw;
      const int toff = (tw.th * g.SW + tw.tw) * g.SC;
#pragma unroll
      for (int i = 0; i < NIW; i++) {
        int sy = ry[i] - tw.th, sx = rx[i] - tw.tw;
        bool ok = tv && (unsigned)sy < (unsigned)g.SH && (unsigned)sx < (unsigned)g.SW;
        base[i] = ok ? (unsigned)(pix0[i] - toff) * (unsigned)sizeof(T) : BUF_OOB;
      }
    }
    const unsigned cb = (unsigned)(tw.c0 * sizeof(T));
#pragma unroll
    for (int i = 0; i < NIW; i++) sk(i, rs, base[i] + cb);
  }
};

// dgrad / ConvT B operand (MC): B[k=(jh,jw,c)][n] = W[c][kh0+s*jh][kw0+s*jw][n], W repacked [C][KH][KW][N]
template <typename T, int R, int NW = GEMM_WAVES> struct ConvDgradB {
  static constexpr int ROWS = R;
  static constexpr bool KCL = false, RELU = false;
  typedef MCGeom<T, R, NW> G; static constexpr int NIW = G::NIW, BK = G::BK;
  const T* w; ConvGeo g; int NC;     // NC = output channels of the dgrad (= conv input channels)
  int relu = 0;
  unsigned lo[NIW]; bool cv[NIW]; int kr[NIW];
  TapWalk tw;
  HD unsigned long bytes() const { return (unsigned long)g.SC * g.KH * g.KW * NC * sizeof(T); }
  HD bool buf_ok() const { return bytes() < BUF_MAX && 2 * g.SC >= BK; }
  DEV void setup(int t0, int tid) {
    const int lane = tid & 63, wave = wave_id();
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      kr[i] = G::krow(wave, i, lane); int cl = t0 + G::col(wave, i, lane);
      cv[i] = cl < NC;
      lo[i] = (unsigned)(((long)kr[i] * g.KH * g.KW * NC + cl) * sizeof(T));
    }
    tw = TapWalk{};
  }
  DEV void issue(int kt, char* tile) { issue_to(kt, DmaSink{tile + wave_id() * NIW * 1024}); }
  template <class SK> DEV void issue_to(int kt, SK sk) {
    const auto rs = make_rsrc(w, bytes());
    const int TW = g.ntw > 0 ? g.ntw : 1;
    if (g.SC % BK) {                 // a tile spans taps tap / tap+1 (rows c0+kr >= SC wrap)
      tw.step_any(kt, BK, g.SC, TW);
      int th1, tw1; tw.next_tap(TW, th1, tw1);
      const int kh = g.kh0 + g.s * tw.th, kw = g.kw0 + g.s * tw.tw;
      const int kh1 = g.kh0 + g.s * th1, kw1 = g.kw0 + g.s * tw1;
      const bool tv0 = tw.tap < g.nth * g.ntw, tv1 = tw.tap + 1 < g.nth * g.ntw;
      const unsigned u0 = (unsigned)((((long)tw.c0 * g.KH + kh) * g.KW + kw) * NC * sizeof(T));
      const unsigned u1 = (unsigned)((((long)(tw.c0 - g.SC) * g.KH + kh1) * g.KW + kw1) * NC * sizeof(T));
#pragma unroll
      for (int i = 0; i < NIW; i++) {
        bool wr = tw.c0 + kr[i] >= g.SC;
        bool ok = cv[i] && (wr ? tv1 : tv0);
        sk(i, rs, ok ? lo[i] + (wr ? u1 : u0) : BUF_OOB);
      }
      return;
    }
    tw.step(kt, BK, g.SC, TW);
    const bool tv = tw.tap < g.nth * g.ntw;
    const int kh = g.kh0 + g.s * tw.th, kw = g.kw0 + g.s * tw.tw;
    const unsigned uo = (unsigned)((((long)tw.c0 * g.KH + kh) * g.KW + kw) * NC * sizeof(T));
#pragma unroll
    for (int i = 0; i < NIW; i++) sk(i, rs, (tv && cv[i]) ? lo[i] + uo : BUF_OOB);
  }
};

// wgrad B operand (MC gather): B[k=pix of the conv output grid RH x RW][n=(tap, cin)] = X[src][cin]
// Fast path (RW % BK == 0): the 64 pixels of a K tile share one output row, so (b, oy, ox0) are
// wave-uniform and interior tiles need no per-lane bounds test.
template <typename T, int R, bool RELU_ = false, int NW = GEMM_WAVES> struct WgradB {
  static constexpr int ROWS = R;
  static constexpr bool KCL = false, RELU = RELU_;
  typedef MCGeom<T, R, NW> G; static constexpr int NIW = G::NIW, BK = G::BK;
  const T* x; ConvGeo g; int NPIX; int relu;   // g.SC = Cin of X, g.SH/SW = X dims, RH/RW = output grid
  int kh[NIW], kw[NIW], kr[NIW], cin[NIW]; unsigned lo[NIW]; bool cval[NIW];
  int nk, pb, poy, pox;                         // uniform walker (fast path)
  int qb[NIW], qy[NIW], qx[NIW];                // per-lane walker (generic path)
  // the descriptor is rebased per K tile to the image of its first pixel (a tile of BK pixels
  // spans at most BK/hw + 2 images), so the batch itself may exceed 4 GiB
  HD unsigned long img_bytes() const { return (unsigned long)g.SH * g.SW * g.SC * sizeof(T); }
  HD unsigned long bytes() const { return img_window_bytes(BK, g.RH * g.RW, g.B, img_bytes()); }
  HD bool buf_ok() const { return bytes() < BUF_MAX; }
  DEV void setup(int t0, int tid) {
    const int lane = tid & 63, wave = wave_id();
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      int col = t0 + G::col(wave, i, lane);
      kr[i] = G::krow(wave, i, lane);
      int tp = col / g.SC; cin[i] = col - tp * g.SC; kh[i] = tp / g.KW; kw[i] = tp - kh[i] * g.KW;
      cval[i] = tp < g.KH * g.KW;
      // lane part of the source offset for an interior tile: (kh*SW + kw + kr*s)*SC + cin
      lo[i] = (unsigned)(((long)(kh[i] * g.SW + kw[i] + kr[i] * g.s) * g.SC + cin[i]) * sizeof(T));
    }
    nk = -1;
  }
  DEV void issue(int kt, char* tile) { issue_to(kt, DmaSink{tile + wave_id() * NIW * 1024}); }
  template <class SK> DEV void issue_to(int kt, SK sk) {
    if (g.RW % BK == 0) {
      if (kt != nk) { int k = kt * BK; int hw = g.RH * g.RW; pb = k / hw; int r = k - pb * hw; poy = r / g.RW; pox = r - poy * g.RW; }
      else { pox += BK; if (pox >= g.RW) { pox = 0; if (++poy >= g.RH) { poy = 0; pb++; } } }
      nk = kt + 1;
      const int iy0 = poy * g.s - g.p, ix0 = pox * g.s - g.p;
      const bool live = pb < g.B;
      const auto rs = make_rsrc(x + (long)(live ? pb : 0) * g.SH * g.SW * g.SC, img_bytes());
      const unsigned uo = (unsigned)(((long)iy0 * g.SW + ix0) * g.SC * (long)sizeof(T));
      const bool interior = iy0 >= 0 && iy0 + g.KH <= g.SH && ix0 >= 0 && ix0 + (BK - 1) * g.s + g.KW <= g.SW;
      if (live && interior) {
#pragma unroll
        for (int i = 0; i < NIW; i++) sk(i, rs, cval[i] ? lo[i] + uo : BUF_OOB);
      } else {
#pragma unroll
        for (int i = 0; i < NIW; i++) {
          int iy = iy0 + kh[i], ix = ix0 + kr[i] * g.s + kw[i];
          bool ok = live && cval[i] && (unsigned)iy < (unsigned)g.SH && (unsigned)ix < (unsigned)g.SW;
          sk(i, rs, ok ? lo[i] + uo : BUF_OOB);
        }
      }
      return;
    }
    // generic: per-lane pixel walker, descriptor rebased to the image of the tile's first pixel
    const int hw = g.RH * g.RW;
    const int b0 = min(kt * BK / hw, g.B - 1);
    const auto rs = make_rsrc(x + (long)b0 * g.SH * g.SW * g.SC, (unsigned long)(g.B - b0) * img_bytes());
    if (kt != nk) {
#pragma unroll
      for (int i = 0; i < NIW; i++) {
        int k = kt * BK + kr[i];
        int b = k / hw; int r = k - b * hw; int oy = r / g.RW;
        qb[i] = b; qy[i] = oy; qx[i] = r - oy * g.RW;
      }
    }
    nk = kt + 1;
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      int iy = qy[i] * g.s - g.p + kh[i], ix = qx[i] * g.s - g.p + kw[i];
      bool ok = cval[i] && qb[i] < g.B && (unsigned)iy < (unsigned)g.SH && (unsigned)ix < (unsigned)g.SW;
      unsigned v = (unsigned)(((((long)(qb[i] - b0) * g.SH + iy) * g.SW + ix) * g.SC + cin[i]) * (long)sizeof(T));
      sk(i, rs, ok ? v : BUF_OOB);
      qx[i] += BK;
      while (qx[i] >= g.RW) { qx[i] -= g.RW; if (++qy[i] >= g.RH) { qy[i] = 0; qb[i]++; } }
    }
    (void)NPIX;
  }
};

// 3x3 / stride 1 / pad 1 weight-gradient B operand for the ping-pong kernel (bf16, MC image):
// B[k = output pixel][n = tap*Cin + cin] = x[pixel shifted by the tap][cin].  With W % BK == 0 a K tile's 64 pixels
// are one run of an image row and Cin % 256 == 0 puts a 256-column tile inside ONE tap, so the tile is a contiguous
// 64-pixel run of x shifted by (dy, dx): per lane only its k-row and its channel offset are kept, the row / image
// walk is uniform (scalar) and just the first / last pixel of a row can fall outside the image (dx = -1 / +1).
template <int R, bool RELU_ = false, int NW = GEMM_WAVES> struct Wgrad3B {
  static constexpr int ROWS = R;
  static constexpr bool KCL = false, RELU = RELU_;
  typedef MCGeom<bf16, R, NW> G; static constexpr int NIW = G::NIW, BK = G::BK;
  const bf16* x; int B, H, W, Cin;
  int tdy, tdx;                                  // this block's tap offsets (uniform)
  int nk, pb, py, px0;                           // uniform walker: next K tile, its image / row / first column
  int kr[NIW]; unsigned lo[NIW];
  HD unsigned long img_bytes() const { return (unsigned long)H * W * Cin * 2; }
  HD bool buf_ok() const { return img_bytes() < BUF_MAX && W % BK == 0 && Cin % 256 == 0; }
  DEV void setup(int t0, int tid) {
    const int lane = tid & 63, wave = wave_id();
    const int tap = t0 / Cin, c0 = t0 - tap * Cin;
    tdy = tap / 3 - 1; tdx = tap - 3 * (tap / 3) - 1;
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      kr[i] = G::krow(wave, i, lane);
      lo[i] = (unsigned)((kr[i] * Cin + c0 + G::col(wave, i, lane)) * 2);
    }
    nk = -1;
  }
  DEV void issue(int kt, char* tile) { issue_to(kt, DmaSink{tile + wave_id() * NIW * 1024}); }
  template <class SK> DEV void issue_to(int kt, SK sk) {
    if (kt != nk) { const int p = kt * BK, hw = H * W; pb = p / hw; const int r = p - pb * hw; py = r / W; px0 = r - py * W; }
    else { px0 += BK; if (px0 >= W) { px0 = 0; if (++py >= H) { py = 0; pb++; } } }
    nk = kt + 1;
    const int yy = py + tdy;
    const bool rowok = pb < B && (unsigned)yy < (unsigned)H;
    const auto rs = make_rsrc(x + (long)(rowok ? pb : 0) * H * W * Cin, img_bytes());
    const int base = ((yy * W + px0 + tdx) * Cin) * 2;          // pixel (yy, px0 + dx), channel 0 (may be < 0)
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      const bool ok = rowok && (unsigned)(px0 + kr[i] + tdx) < (unsigned)W;
      sk(i, rs, ok ? (unsigned)(base + (int)lo[i]) : BUF_OOB);
    }
  }
};

DEV bf16x8 relu_frag(bf16x8 v) {
  return __builtin_bit_cast(bf16x8, relu16<bf16>(__builtin_bit_cast(uint4, v)));
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
template <typename T, int BM, int BN, int NST_ = 3, int WM_ = 0> struct GemmShape {
  static constexpr int BK = KT<T>::BK;
  static constexpr int ABYTES = BM * 128, BBYTES = BN * 128;
  static constexpr int STAGE = ABYTES + BBYTES;
  static constexpr int NST = NST_;
  static constexpr int LDT = BN + 4;                       // fp32 C-tile row stride
  // the fp32 C tile is staged through LDS in row chunks of CROWS (half the tile when the whole
  // tile would not fit beside the K stages, e.g. 256x256)
  static constexpr int CROWS = (BM * LDT * 4 <= NST * STAGE || BM * LDT * 4 <= 160 * 1024) ? BM : BM / 2;
  static constexpr int CBYTES = CROWS * LDT * 4;
  static constexpr int LDS = (NST * STAGE > CBYTES ? NST * STAGE : CBYTES);
  static_assert(LDS <= 160 * 1024, "LDS budget");
  // wave grid: 8 waves as WM x WN
  static constexpr int WM = WM_ ? WM_ : (BM >= 2 * BN ? 4 : (BN >= 2 * BM ? 2 : (BM >= BN ? 4 : 2)));
  static constexpr int WN = GEMM_WAVES / WM;
  static constexpr int TM = BM / WM, TN = BN / WN;         // per-wave tile
  static constexpr int MI = TM / 16, NI = TN / 16;
  static_assert(MI >= 1 && NI >= 1 && TM % 16 == 0 && TN % 16 == 0, "bad wave tiling");
};

struct KRange { int kt0, kt1; };

// workgroup barrier that orders LDS only (does not drain in-flight global loads / LDS-DMA)

// Block-level epilogue contract:  epi(tile, LDT, m0, n0, tid, BM, BN)
//
// Main loop: 3 LDS stages filled by LDS-DMA two K-tiles ahead; one raw s_barrier per K tile,
// placed BEFORE the last k-step's MFMAs so the next tile's first fragments are read from LDS
// while the current tile's last MFMAs run (fragments double-buffered in registers).
// vmcnt is counted (the tile two steps ahead stays in flight across the barrier); there is
// no __syncthreads() in the loop (it would drain vmcnt to 0: guide §5).
// Block order is remapped so consecutive tiles of one row-panel share an XCD (guide T1).
template <typename T, int BM, int BN, int NST, class LA, class LB, class EPI, int WM_ = 0>
__global__ void __launch_bounds__(GEMM_THREADS) igemm_kernel(LA la, LB lb, EPI epi, int KTILES, int split) {
  typedef GemmShape<T, BM, BN, NST, WM_> S;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
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
      for (int j = 0; j < NI; j++) acc[i][j] = Mma<T>::mma(fb[buf][j], fa[buf][i], acc[i][j]);
  };
  // (B, A operand order: acc[i][j] holds the 16x16 block TRANSPOSED, so lane (g, l) owns
  //  C[m = i*16 + l][n = j*16 + 4g .. 4g+3] -- four consecutive columns -> one 16-B LDS store)

  const int nt = kt1 - kt0;
  constexpr int PD = NST - 1;                 // LDS-DMA prefetch distance (tiles in flight)
  if (nt > 0) {
    // prologue: tiles 0 .. PD-1
#pragma unroll
    for (int q = 0; q < PD; q++)
      if (q < nt) {
        la.issue(kt0 + q, smem + q * S::STAGE);
        lb.issue(kt0 + q, smem + q * S::STAGE + S::ABYTES);
      }
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
  vm_drain();
  lds_barrier();
  // stage the C tile to LDS (fp32) in row chunks of CROWS and hand each chunk to the epilogue
  float* ct = (float*)smem;
#pragma unroll
  for (int c0 = 0; c0 < BM; c0 += S::CROWS) {
    if (c0) lds_barrier();
#pragma unroll
    for (int i = 0; i < MI; i++) {
      const int rb = wm * S::TM + i * 16;                    // wave-uniform
      if (rb < c0 || rb >= c0 + S::CROWS) continue;
#pragma unroll
      for (int j = 0; j < NI; j++) {
        int r = rb - c0 + (lane & 15);
        int c = wn * S::TN + j * 16 + (lane >> 4) * 4;
        *(float4*)(ct + r * S::LDT + c) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      }
    }
    lds_barrier();
    epi(ct, S::LDT, m0 + c0, n0, tid, S::CROWS, BN, GEMM_THREADS);
  }
}

// iterate 8-wide row segments of the staged tile: f(m, n, const float* v8, r, c).  When the
// thread count is a multiple of the segments per row (every config but the N=96 head), a thread
// keeps ONE column group and the loop has a compile-time trip count, so it unrolls and the LDS
// reads / global stores of all rows are in flight together.
template <class F> DEV void for_segments(const float* ct, int LDT, int BM, int BN, int m0, int n0, int M, int N, int tid, int NT, F f) {
  const int spr = BN / 8;
  if (NT % spr == 0 && BM % (NT / spr) == 0) {
    const int rpi = NT / spr, cs = tid % spr, r0 = tid / spr;
    const int n = n0 + cs * 8;
    if (n >= N) return;
#pragma unroll
    for (int it = 0; it < BM / rpi; it++) {
      const int r = r0 + it * rpi, m = m0 + r;
      if (m >= M) break;
      const float4* src = (const float4*)(ct + r * LDT + cs * 8);
      float4 x0 = src[0], x1 = src[1];
      float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      f(m, n, v, r, cs * 8);
    }
    return;
  }
  const int segs = BM * BN / 8;
  for (int s = tid; s < segs; s += NT) {
    int r = s / spr, cs = s - r * spr;
    int m = m0 + r, n = n0 + cs * 8;
    if (m < M && n < N) f(m, n, ct + r * LDT + cs * 8, r, cs * 8);
  }
}

// ------------------------------------------------------------------ common epilogue
// out = act(acc*scale[n] + shift[n]) + res1 + res2 ; optional raw store (pre-act) and BN
// batch statistics (sum / sum of squares of the pre-activation value, fp64 atomics).
enum { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_GELU_BWD = 3, ACT_RELU_BWD = 4, ACT_GELU_SG = 5, ACT_MUL = 6 };
// ACT_GELU_BWD: o = v * gelu'(res1)   (res1 = saved pre-activation, not added)
// ACT_RELU_BWD: o = v * (res1 > 0)    (res1 = saved activation output, not added)
// ACT_GELU_SG:  o = gelu(v) and `pre` receives gelu'(v) instead of the pre-activation (one erf serves both)
// ACT_MUL:      o = v * res1          (res1 = the saved gelu'(v) of ACT_GELU_SG, not added)
template <typename TO, typename TR, typename TP = TO, int EB = 4> struct EpiStd {
  // pre = acc + bias[n] ;  v = pre*scale[n] + shift[n] ;  out = act(v) (+res1 +res2)
  TO* out; long ldo; int coff;          // output row stride / channel offset
  const float* bias; const float* scale; const float* shift;
  const TR* res1; long ldr1; const TR* res2; long ldr2;
  TP* pre; long ldp;                    // optional: store pre (acc + bias), compute dtype
  double* stats;                        // optional: [2][N] (sum, sumsq) of pre (BN batch statistics)
  int act, M, N;
  RowMap rm;
  float* csum = nullptr;                // optional: out[n] column sums (bias gradient), fp32 atomics
  DEV void prepare(int) {}
  DEV void operator()(const float* ct, int LDT, int m0, int n0, int tid, int BM, int BN, int NT) const {
    // a thread always sees the same 8-column group (NT % (BN/8) == 0), so its column
    // partial sums live in registers until the block reduction below
    float cs8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // per-column affine terms of this thread's (fixed) 8-column group, loaded once
    float b8[8], s8[8], h8[8];
    {
      const int nn = n0 + (tid % (BN / 8)) * 8;
      const bool ok = nn < N;
#pragma unroll
      for (int e = 0; e < 8; e++) {
        b8[e] = (bias && ok) ? bias[nn + e] : 0.f;
        s8[e] = (scale && ok) ? scale[nn + e] : 1.f;
        h8[e] = (shift && ok) ? shift[nn + e] : 0.f;
      }
    }
    const bool fixed_cols = NT % (BN / 8) == 0;
    // one segment: 8 columns of row m (orow = its output row), a = the 8 staged accumulators, r1 = the 8 res1 values
    // (read only when res1 is set: an array, never a pointer select, which would keep it in scratch).  ACT is a
    // compile-time constant: the activation is dispatched once, outside the loops.
    auto seg = [&](auto ACTC, long orow, int n, const float (&a)[8], const float (&r1)[8], const float (&bb)[8],
                   const float (&ss)[8], const float (&hh)[8]) {
      constexpr int A = decltype(ACTC)::value;
      float pv[8], v[8], o[8];
#pragma unroll
      for (int e = 0; e < 8; e++) { pv[e] = a[e] + bb[e]; v[e] = pv[e] * ss[e] + hh[e]; }
      if (A != ACT_GELU_SG && pre) store8<TP>(pre + orow * ldp + n, pv);
      constexpr bool FAST = sizeof(TP) == 2;     // bf16 compute: branch-free GELU (common.hpp)
      if constexpr (A == ACT_GELU_BWD) {
#pragma unroll
        for (int e = 0; e < 8; e++) o[e] = v[e] * (FAST ? gelu_fast_grad(r1[e]) : gelu_erf_grad(r1[e]));
      } else if constexpr (A == ACT_RELU_BWD) {
#pragma unroll
        for (int e = 0; e < 8; e++) o[e] = r1[e] > 0.f ? v[e] : 0.f;
      } else if constexpr (A == ACT_MUL) {
#pragma unroll
        for (int e = 0; e < 8; e++) o[e] = v[e] * r1[e];
      } else if constexpr (A == ACT_GELU_SG) {
        float gd[8];
#pragma unroll
        for (int e = 0; e < 8; e++) {
          float f, ex;
          erf_as(v[e], f, ex);
          o[e] = 0.5f * v[e] * (1.0f + f);
          gd[e] = 0.5f * (1.0f + f) + v[e] * (0.39894228040143268f * ex);
        }
        if (pre) store8<TP>(pre + orow * ldp + n, gd);
      } else {
#pragma unroll
        for (int e = 0; e < 8; e++) o[e] = A == ACT_GELU ? (FAST ? gelu_fast(v[e]) : gelu_erf(v[e])) : A == ACT_RELU ? fmaxf(v[e], 0.f) : v[e];
        if (res1) {
#pragma unroll
          for (int e = 0; e < 8; e++) o[e] += r1[e];
        }
      }
      if (res2) { float r[8]; load8<TR>(res2 + orow * ldr2 + n, r);
#pragma unroll
        for (int e = 0; e < 8; e++) o[e] += r[e]; }
      store8<TO>(out + orow * ldo + coff + n, o);
      if (csum) {
#pragma unroll
        for (int e = 0; e < 8; e++) cs8[e] += o[e];
      }
    };
    auto dispatch = [&](auto body) {
      switch (act) {
        case ACT_RELU: body(std::integral_constant<int, ACT_RELU>{}); break;
        case ACT_GELU: body(std::integral_constant<int, ACT_GELU>{}); break;
        case ACT_GELU_BWD: body(std::integral_constant<int, ACT_GELU_BWD>{}); break;
        case ACT_RELU_BWD: body(std::integral_constant<int, ACT_RELU_BWD>{}); break;
        case ACT_GELU_SG: body(std::integral_constant<int, ACT_GELU_SG>{}); break;
        case ACT_MUL: body(std::integral_constant<int, ACT_MUL>{}); break;
        default: body(std::integral_constant<int, ACT_NONE>{}); break;
      }
    };
    const int spr_ = BN / 8;
    if (fixed_cols && BM % (NT / spr_) == 0) {
      // a thread's segments are rows r0 + it * rpi of one 8-column group.  They run in batches of EB: the batch's
      // staged accumulators (LDS) and res1 rows (global) are all read before its first store -- with a read per
      // segment, each LDS read latency is exposed in turn and each residual load waits (vmcnt, in issue order)
      // for every earlier segment's stores.  Rows outside the output read row 0 (address select, no branch).
      const int rpi = NT / spr_, cs = tid % spr_, r0 = tid / spr_, n = n0 + cs * 8, nit = BM / rpi;
      if (n < N) {
        dispatch([&](auto ACTC) {
#pragma unroll
          for (int it0 = 0; it0 < nit; it0 += EB) {
            __builtin_amdgcn_sched_barrier(0);     // no batch's reads hoisted above the previous batch (VGPRs)
            float av[EB][8];
            Row8<TR> q[EB];
            long orow[EB];
#pragma unroll
            for (int u = 0; u < EB; u++) {
              const int it = it0 + u, r = r0 + it * rpi, m = m0 + r;
              if (it < nit) {
                const float4* src = (const float4*)(ct + r * LDT + cs * 8);
                const float4 x0 = src[0], x1 = src[1];
                av[u][0] = x0.x; av[u][1] = x0.y; av[u][2] = x0.z; av[u][3] = x0.w;
                av[u][4] = x1.x; av[u][5] = x1.y; av[u][6] = x1.z; av[u][7] = x1.w;
                orow[u] = m < M ? rm.map(m) : 0;
                if (res1) q[u].load(res1 + orow[u] * ldr1 + n);
              }
            }
#pragma unroll
            for (int u = 0; u < EB; u++) {
              const int it = it0 + u;
              if (it < nit && m0 + r0 + it * rpi < M) {
                float r1v[8];
                q[u].get(r1v);                     // unused (never read) without res1
                seg(ACTC, orow[u], n, av[u], r1v, b8, s8, h8);
              }
            }
          }
        });
      }
    } else {
      dispatch([&](auto ACTC) {
        for_segments(ct, LDT, BM, BN, m0, n0, M, N, tid, NT, [&](int m, int n, const float* a, int, int) {
          float av[8], bb[8], ss[8], hh[8], r1v[8];
#pragma unroll
          for (int e = 0; e < 8; e++) {
            av[e] = a[e];
            bb[e] = bias ? bias[n + e] : 0.f; ss[e] = scale ? scale[n + e] : 1.f; hh[e] = shift ? shift[n + e] : 0.f;
            r1v[e] = 0.f;
          }
          const long orow = rm.map(m);
          if (res1) load8<TR>(res1 + orow * ldr1 + n, r1v);
          seg(ACTC, orow, n, av, r1v, bb, ss, hh);
        });
      });
    }
    if (stats) {
      // column statistics of pre over this tile's valid rows: thread -> (col, row phase).  The fp64 atomics of
      // every tile of the grid would all land on the same 2N words; they are spread over S3OD_NREP replicas
      // ([NREP][2][N], chosen by tile and row phase), which s3od_bn_finalize folds and clears
      const int nph = NT / BN;
      const int c = tid % BN, ph = tid / BN;
      const int n = n0 + c;
      if (n < N) {
        float s = 0.f, q = 0.f;
        const float bn_ = bias ? bias[n] : 0.f;
        for (int r = ph; r < BM; r += nph) {
          if (m0 + r >= M) break;
          const float v = ct[r * LDT + c] + bn_;
          s += v; q += v * v;
        }
        const int rep = (int)(((unsigned)(blockIdx.y * gridDim.x + blockIdx.x) * (unsigned)nph + ph + (m0 / BM)) % S3OD_NREP);
        double* st = stats + (long)rep * 2 * N;
        atomicAdd(st + n, (double)s);
        atomicAdd(st + N + n, (double)q);
      }
    }
    if (csum) {
      // reduce the per-thread 8-column partials over the row phases through the (consumed) C tile
      lds_barrier();
      float* red = (float*)ct;
#pragma unroll
      for (int e = 0; e < 8; e++) red[tid * 8 + e] = cs8[e];
      lds_barrier();
      const int spr = BN / 8, nph = NT / spr;
      if (tid < BN && n0 + tid < N) {
        const int g = tid >> 3, e = tid & 7;
        float s = 0.f;
        for (int ph = 0; ph < nph; ph++) s += red[(ph * spr + g) * 8 + e];
        atomicAdd(csum + n0 + tid, s);
      }
    }
  }
};

// split-K wgrad epilogue: atomically accumulate into an fp32 gradient in PyTorch layout
//   dW[(m*Cx + cin)*taps + tap] += tile   where n = tap*Cx + cin   (Linear: taps=1)
struct EpiWgrad {
  float* dw; int M, N, Cx, taps;
  DEV void prepare(int) {}
  DEV void operator()(const float* ct, int LDT, int m0, int n0, int tid, int BM, int BN, int NT) const {
    const int total = BM * BN;
    for (int s = tid; s < total; s += NT) {
      int r = s / BN, c = s - r * BN;
      int m = m0 + r, n = n0 + c;
      if (m < M && n < N) {
        int tap = n / Cx, cin = n - tap * Cx;
        atomicAdd(dw + ((long)m * Cx + cin) * taps + tap, ct[r * LDT + c]);
      }
    }
  }
};

// split-K wgrad epilogue without atomics: split z writes its whole fp32 tile to its own slab ws[z][M][N] with 16-B
// stores (every workgroup writes its tile, an empty K range writes zeros), and wgrad_reduce_kernel sums the slabs into
// dW.  The fp32 atomics of EpiWgrad run at the chip's ~1.3 TB/s atomic rate and all land at the end of every workgroup
// (one round); plain stores move the same bytes at the store rate.
struct EpiWgradPart {
  float* ws; int M, N;
  int z = 0;
  DEV void prepare(int zz) { z = zz; }
  DEV void operator()(const float* ct, int LDT, int m0, int n0, int tid, int BM, int BN, int NT) const {
    float* slab = ws + (long)z * M * N;
    for_segments(ct, LDT, BM, BN, m0, n0, M, N, tid, NT, [&](int m, int n, const float* a, int, int) {
      float4* d = (float4*)(slab + (long)m * N + n);
      d[0] = make_float4(a[0], a[1], a[2], a[3]);
      d[1] = make_float4(a[4], a[5], a[6], a[7]);
    });
  }
};

// ------------------------------------------------------------------ 256x256 ping-pong kernel (bf16)
// 8 waves = 2 (M) x 4 (N), each owning a 128x64 sub-tile (acc[8][4], 128 VGPRs); waves w and w+4
// share a SIMD (cyclic wave->SIMD placement), so the two M halves are SIMD partners.  The M half
// wr = 1 runs one barrier behind wr = 0: while one wave of a SIMD runs its 16-MFMA block, its
// partner issues the next block's LDS reads and LDS-DMA (MI355X_MICROARCH.md "Two waves per SIMD",
// cdna_hip_programming.md §5 "256² 8-phase template").
//
// Each K tile (BK = 64) is 4 phases = the wave's 4 C quadrants (64 rows x 32 cols) in the order
// (0,0) (0,1) (1,1) (1,0); a phase is  [LDS reads | DMA issue] barrier [16 MFMA] barrier.  All of a
// tile's fragments are read in its phases 0 and 1 (A0+B0, then B1+A1: 96 VGPRs), so its LDS buffer
// is free from phase 3 on and the DMA of tile t+2 can start there, a whole tile ahead.
// LDS: 2 buffers x 4 half images (A rows 0-127 / 128-255, B cols 0-127 / 128-255; 16 KB each), so
// the loaders run with R = 128.  Tile t+1's A halves are issued in phase 3 of tile t-1 and its B
// halves in phase 0 of tile t; phase 3 of tile t retires both with a counted vmcnt.
//   RAW: every wave's wait for tile t+1 sits in its phase-3 load segment of tile t, i.e. before the
//        barrier that precedes the first read of tile t+1 by either stagger half;
//   WAR: a buffer's last reads are in phase 1; it is restaged in phase 3 (>= 2 phases later, so
//        every reader's lgkmcnt(0) precedes a barrier the restaging wave has passed).
// Fragment addressing inside a 128-row half image with every read's row0 a multiple of 16: the
// per-lane part of the address is computed once and the row0 / kk parts become immediates.
//   KC [128][128 B]: kc_off(row0 + l, b) = row0*128 + kc_off(l, b)   ((r>>1)&7 depends on l only)
//   MC [64 k][256 B]: mc_off<256>(kk*32 + 8g + q, 2*row0 + 8p)
//                     = kk*8192 + (8g+q)*256 + 8p + (((row0>>4) ^ gk) << 5),  gk = q | (g&1)<<2
template <bool KCL> struct PPFrag;
template <> struct PPFrag<true> {
  int o[2];
  DEV void init(int lane, int) {
#pragma unroll
    for (int kk = 0; kk < 2; kk++) o[kk] = kc_off(lane & 15, kk * 64 + (lane >> 4) * 16);
  }
  DEV bf16x8 read(const char* img, int row0, int kk) const { return *(const bf16x8*)(img + o[kk] + row0 * 128); }
};
template <> struct PPFrag<false> {
  int base, gk;
  // h64: the reads' rows are offset by 64 * h64 (folded into the XOR: (4 h64 | m) ^ gk = m ^ (gk ^ 4 h64))
  DEV void init(int lane, int h64) {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    base = (8 * g + q) * 256 + 8 * p; gk = (q | ((g & 1) << 2)) ^ (h64 << 2);
  }
  DEV bf16x8 read(const char* img, int row0, int kk) const {
    typedef __attribute__((address_space(3))) s16x4 lds_s4;
    const char* a = img + base + ((((row0 >> 4) ^ gk)) << 5) + kk * 8192;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)a);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(a + 1024));
    bf16x4 x = __builtin_bit_cast(bf16x4, lo), y = __builtin_bit_cast(bf16x4, hi);
    bf16x8 r;
    r[0] = x[0]; r[1] = x[1]; r[2] = x[2]; r[3] = x[3]; r[4] = y[0]; r[5] = y[1]; r[6] = y[2]; r[7] = y[3];
    return r;
  }
};


// The epilogue stages C through the K-stage LDS in two 128-row chunks with LDS barriers only (a
// __syncthreads() would drain the stores).  (A persistent variant -- the next tile's first K
// stage issued behind this tile's stores -- measured within 5 % of this at 20 spilled VGPRs.)
// Dev timeline build (-DS3OD_TIMELINE, tools/pp_timeline.py; never in the production library): the ping-pong kernel
// records per block [start, main loop done, epilogue done, HW_ID / XCC_ID, C half 0 staged, half 0 done, half 1
// staged, -] (s_memrealtime, 100 MHz) into s3od_tl[linear block][8], set per translation unit by s3od_dbg_timeline()
#ifdef S3OD_TIMELINE
static __device__ unsigned long long* s3od_tl;
#define S3OD_TL(slot, v) do { if (s3od_tl && threadIdx.x == 0) s3od_tl[((long)blockIdx.z * gridDim.y * gridDim.x + \
    blockIdx.y * gridDim.x + blockIdx.x) * 8 + (slot)] = (v); } while (0)
#else
#define S3OD_TL(slot, v) do { } while (0)
#endif

// block -> (M tile, N tile) of a 2-D grid: an XCD-contiguous linear index W (the blocks one XCD receives get
// consecutive W), then row-major -- or, with G > 0, in groups of G M-tiles walked column-major, so the ~32 blocks an
// XCD runs at once cover a G x (32 / G) patch and share G A-panels and 32 / G B-panels in that XCD's L2 instead of one
// A-panel and 32 B-panels
DEV void tile_of_block(int G, int& mt, int& nt) {
  const int nN = gridDim.x, nM = gridDim.y, nwg = nN * nM;
  const int L = blockIdx.y * nN + blockIdx.x;
  const int q = nwg >> 3, r = nwg & 7, xcd = L & 7, idx = L >> 3;
  const int W = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  if (G <= 0) { mt = W / nN; nt = W % nN; return; }
  const int per = G * nN, g = W / per, w = W - g * per, m_first = g * G, gs = min(nM - m_first, G);
  mt = m_first + w % gs; nt = w / gs;
}

template <class LA, class LB, class EPI>
__global__ void __launch_bounds__(GEMM_THREADS, 1) igemm_pp_kernel(LA la0, LB lb0, EPI epi, int KTILES, int split, int flags) {
  typedef bf16 T;
  constexpr int BM = 256, BN = 256, HB = 128 * 128, STG = 4 * HB, LDT = BN + 4;
  static_assert(sizeof(T) == 2 && KT<T>::BK == 64, "ping-pong kernel is bf16 only");
  static_assert(128 * LDT * 4 <= 160 * 1024 && 2 * STG <= 128 * LDT * 4, "ping-pong LDS budget");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int wr = wave >> 2, wc = wave & 3;
  S3OD_TL(0, __builtin_amdgcn_s_memrealtime());
  S3OD_TL(3, ((unsigned long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11)) << 32) |
             (unsigned)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)));
  int m0, n0;
  {
    int mt, nt_;
    tile_of_block((flags >> 8) & 0xff, mt, nt_);
    m0 = mt * BM; n0 = nt_ * BN;
  }
  const int per = (KTILES + split - 1) / split;
  const int kt0 = blockIdx.z * per, kt1 = min(KTILES, kt0 + per);
  const int nt = kt1 - kt0;
  epi.prepare(blockIdx.z);
  LA la1 = la0; LB lb1 = lb0;
  la0.setup(m0, tid); la1.setup(m0 + 128, tid);
  lb0.setup(n0, tid); lb1.setup(n0 + 128, tid);
  constexpr int NA = LA::NIW * 2;              // DMA instructions per wave for the two A halves
  const bool stag = !(flags & 1);              // dev knob S3OD_PP_FLAGS bit 0: no stagger
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nt > 0) {
    // first K stage: buffer 0 whole + buffer 1's A halves
    la0.issue(kt0, smem); la1.issue(kt0, smem + HB); lb0.issue(kt0, smem + 2 * HB); lb1.issue(kt0, smem + 3 * HB);
    if (nt > 1) { la0.issue(kt0 + 1, smem + STG); la1.issue(kt0 + 1, smem + STG + HB); wait_vmcnt<NA>(); }
    else wait_vmcnt<0>();
    raw_barrier();
    if (wr && stag) raw_barrier();             // stagger: the wr = 1 half runs one barrier behind
    PPFrag<LA::KCL> pfa; pfa.init(lane, 0);
    PPFrag<LB::KCL> pfb; pfb.init(lane, wc & 1);                        // this wave's 64 B columns
    const int boff = LB::KCL ? (wc & 1) * 64 * 128 : 0;
    bf16x8 fa[2][4][2], fb[2][2][2];
    auto rdA = [&](const char* As, int qm) {
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int kk = 0; kk < 2; kk++) {
          fa[qm][i][kk] = pfa.read(As, qm * 64 + i * 16, kk);
          if constexpr (LA::RELU) fa[qm][i][kk] = relu_frag(fa[qm][i][kk]);
        }
    };
    auto rdB = [&](const char* Bs, int qn) {
#pragma unroll
      for (int j = 0; j < 2; j++)
#pragma unroll
        for (int kk = 0; kk < 2; kk++) {
          fb[qn][j][kk] = pfb.read(Bs, qn * 32 + j * 16, kk);
          if constexpr (LB::RELU) fb[qn][j][kk] = relu_frag(fb[qn][j][kk]);
        }
    };
    auto mm = [&](int qm, int qn) {
      raw_barrier();
      wait_lgkm0();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; kk++)
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
          for (int j = 0; j < 2; j++)
            acc[qm * 4 + i][qn * 2 + j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[qn][j][kk], fa[qm][i][kk], acc[qm * 4 + i][qn * 2 + j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      raw_barrier();
    };
    // DMA issue spread over the four load segments (round 5 issued both B halves in phase 0 and both A halves in
    // phase 3, making those load segments outlast the partner's 16 MFMAs): B half 0 / 1 of tile t+1 in phases 0 / 1
    // (their buffer's last reads were in tile t-1); A half 0 of tile t+2 in phase 2 -- read only by the wr = 0 waves,
    // whose last reads (phase 1) every wave has waited for before the barrier that opens its phase 2; A half 1 in
    // phase 3 -- read by the wr = 1 waves, which wait for their phase-1 reads one barrier later, still before any
    // wave's phase 3.
    for (int t = 0; t < nt; ++t) {
      char* cb = smem + (t & 1) * STG;
      char* nb = smem + ((t + 1) & 1) * STG;
      const char* As = cb + wr * HB;
      const char* Bs = cb + (2 + (wc >> 1)) * HB + boff;
      // phase 0: quadrant (0,0); B half 0 of tile t+1
      rdA(As, 0); rdB(Bs, 0);
      if (t + 1 < nt) lb0.issue(kt0 + t + 1, nb + 2 * HB);
      mm(0, 0);
      // phase 1: quadrant (0,1); the tile's last LDS reads; B half 1 of tile t+1
      rdB(Bs, 1); rdA(As, 1);
      if (t + 1 < nt) lb1.issue(kt0 + t + 1, nb + 3 * HB);
      mm(0, 1);
      // phase 2: quadrant (1,1); A half 0 of tile t+2 into this tile's buffer
      if (t + 2 < nt) la0.issue(kt0 + t + 2, cb);
      mm(1, 1);
      // phase 3: quadrant (1,0); A half 1 of tile t+2; retire tile t+1 (A issued in tile t-1, B in phases 0 / 1)
      if (t + 2 < nt) { la1.issue(kt0 + t + 2, cb + HB); wait_vmcnt<NA>(); }
      else if (t + 1 < nt) wait_vmcnt<0>();
      mm(1, 0);
    }
    if (!wr && stag) raw_barrier();            // re-align the two halves
  }
  S3OD_TL(1, __builtin_amdgcn_s_memrealtime());
  vm_drain();
  // The C tile goes through LDS (fp32) in two rounds of two 64-row quarters: round c stages rows [c*64, c*64+64) of
  // each wave row half (wave row wr -> buffer wr), then the epilogue runs on both.  After round 0 every wave's first
  // four accumulator row tiles are dead, so at most 64 accumulator VGPRs are live under the epilogue code (halves
  // staged one at a time kept the wr = 1 waves' 128 live through half 0's epilogue).
  float* ct0 = (float*)smem;
  float* ct1 = ct0 + 64 * LDT;
  // (a lambda on a compile-time round, not a loop: a loop this size stays rolled and indexes acc at run time,
  // which puts all of acc on the stack)
  auto round = [&](auto CC) {
    constexpr int c = decltype(CC)::value;
    lds_barrier();
    {
      float* dst = wr ? ct1 : ct0;
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int r = i * 16 + (lane & 15), col = wc * 64 + j * 16 + (lane >> 4) * 4;
          *(f32x4*)(dst + r * LDT + col) = acc[c * 4 + i][j];
        }
    }
    lds_barrier();
    S3OD_TL(4 + 2 * c, __builtin_amdgcn_s_memrealtime());
#ifdef S3OD_TIMELINE
    // dev (timeline build, S3OD_PP_FLAGS bit 1): a bare bf16 store loop instead of the epilogue functor
    if constexpr (std::is_same_v<EPI, EpiStd<bf16, bf16, bf16>>) {
      if (flags & 2) {
        const int cs = tid % 32, r0 = tid / 32;
#pragma unroll
        for (int it = 0; it < 8; it++) {
          const int r = r0 + (it & 3) * 16;
          const float* src_ = (it < 4 ? ct0 : ct1) + r * LDT + cs * 8;
          const float4 a = ((const float4*)src_)[0], b = ((const float4*)src_)[1];
          const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
          store8<bf16>(epi.out + (long)(m0 + (it < 4 ? 0 : 128) + c * 64 + r) * epi.ldo + n0 + cs * 8, v);
        }
        return;
      }
    }
#endif
    epi(ct0, LDT, m0 + c * 64, n0, tid, 64, BN, GEMM_THREADS);
    epi(ct1, LDT, m0 + 128 + c * 64, n0, tid, 64, BN, GEMM_THREADS);
    if (c == 0) S3OD_TL(5, __builtin_amdgcn_s_memrealtime());
  };
  round(std::integral_constant<int, 0>{});
  round(std::integral_constant<int, 1>{});
  S3OD_TL(2, __builtin_amdgcn_s_memrealtime());
}
constexpr int PP_LDS = 128 * (256 + 4) * 4;   // two 64-row C quarters (133 KB) >= the two 64 KB K stages

// the 4-wave 256x256 kernel (gemm_q.hip, its own translation unit: AGPR accumulators); instantiated there for the
// linears' (loader, epilogue) combinations
template <class LA, class LB, class EPI>
int launch_igemm_q(LA la, LB lb, EPI epi, int M, int N, int KTILES, int split, int zdim_extra, hipStream_t st);

// WM_: waves along M (0 = by tile shape); e.g. 512x64 tiles use WM_=8 for 64x64 per-wave tiles; WM_ = -1: gemm_q.hip
template <typename T, int BM, int BN, class LA, class LB, class EPI, int NST = 3, int WM_ = 0>
static int launch_igemm(LA la, LB lb, EPI epi, int M, int N, int KTILES, int split, int zdim_extra, hipStream_t st) {
  if constexpr (WM_ < 0) {
    static_assert(BM == 256 && BN == 256 && sizeof(T) == 2, "q config");
    return launch_igemm_q(la, lb, epi, M, N, KTILES, split, zdim_extra, st);
  } else if constexpr (LA::ROWS * 2 == BM) {    // half-row loaders: the 256x256 ping-pong kernel
    static_assert(BM == 256 && BN == 256 && LB::ROWS == 128 && sizeof(T) == 2, "ping-pong config");
    if (!la.buf_ok() || !lb.buf_ok()) {
      s3od_set_error("igemm: operand window too large for a buffer descriptor or gather channels < %d", KT<T>::BK / 2);
      return 22;
    }
    auto kfn = igemm_pp_kernel<LA, LB, EPI>;
    static const bool attr = ((void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, PP_LDS), true);   // once per process (thread-safe static init)
    (void)attr;
    const int flags = S3OD_KNOB("S3OD_PP_FLAGS", 0) | (S3OD_KNOB("S3OD_GEMM_GROUP", 0) & 0xff) << 8;
    dim3 grid(cdiv(N, BN), cdiv(M, BM), split * zdim_extra);
    hipLaunchKernelGGL(kfn, grid, dim3(GEMM_THREADS), PP_LDS, st, la, lb, epi, KTILES, split, flags);
    return s3od_check_launch("igemm_pp");
  } else {
    if (!la.buf_ok() || !lb.buf_ok()) {
      s3od_set_error("igemm: operand window too large for a buffer descriptor or gather channels < %d", KT<T>::BK / 2);
      return 22;
    }
    typedef GemmShape<T, BM, BN, NST, WM_> S;
    auto kfn = igemm_kernel<T, BM, BN, NST, LA, LB, EPI, WM_>;
    static const bool attr = ((void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, S::LDS), true);   // once per process (thread-safe static init)
    (void)attr;
    dim3 grid(cdiv(N, BN), cdiv(M, BM), split * zdim_extra);
    hipLaunchKernelGGL(kfn, grid, dim3(GEMM_THREADS), S::LDS, st, la, lb, epi, KTILES, split);
    return s3od_check_launch("igemm");
  }
}
