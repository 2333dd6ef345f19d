// C-ABI entry points built on the implicit-GEMM engine (gemm.hpp).
#include "gemm.hpp"
// blaslt.hip: row-major D = A . B (+ C) through hipBLASLt; 0 = done, nonzero = not run (no algorithm / error)
int blaslt_gemm_rm(const void* A, long lda, const void* B, long ldb, const void* C, long ldc, void* D, long ldd, int M,
                   int N, int K, hipStream_t st);
#include <type_traits>
#include <utility>

#define DISPATCH_T(dtype, ...)                                                  \
  do {                                                                          \
    if ((dtype) == S3OD_BF16) { typedef bf16 T; __VA_ARGS__ }                   \
    else if ((dtype) == S3OD_F32) { typedef float T; __VA_ARGS__ }              \
    else { s3od_set_error("bad dtype %d", (int)(dtype)); return 22; }           \
  } while (0)

static RowMap dense_rm() { RowMap r{}; r.mode = 0; return r; }

// Tile configuration (dev knob for the micro-benchmarks): S3OD_GEMM_CFG=<n> forces one config for
// every GEMM entry point; default (-1) = per-op choice below.
//   0: 256x128, 3 stages (1 WG/CU)   1: 128x128, 2 stages (2 WG/CU)   2: 128x128, 3 stages
//   3: 256x128, 2 stages (BN is clamped to 64 for 64-channel convs: 256x64 x 2 stages = 80 KB)
//   4: 256x256, 2 stages (1 WG/CU, per-wave 64x128; C staged in two 128-row halves)
#include <stdlib.h>
static int gemm_cfg() { return S3OD_KNOB("S3OD_GEMM_CFG", -1); }
// W = waves that issue the operand loads (the loaders are built for that many waves)
// PP_: the 256x256 ping-pong kernel (bf16 only), whose loaders stage half tiles (LM / LN rows)
template <int BM_, int BN_, int NST_, int W_ = GEMM_WAVES, int WM_ = 0, bool PP_ = false> struct TileCfg {
  static constexpr int BM = BM_, BN = BN_, NST = NST_, W = W_, WM = WM_;
  static constexpr bool PP = PP_;
  static constexpr bool SLAB = PP_ || WM_ < 0;   // split-K partials into caller slabs (the 256x256 kernels)
  static constexpr int LM = PP_ ? BM_ / 2 : BM_, LN = PP_ ? BN_ / 2 : BN_;
};
// a conv whose output-channel tile is narrower than 256 cannot run the ping-pong kernel
template <class C, int BNW> using ConvCfg = std::conditional_t<(C::PP && BNW < 256), TileCfg<128, 128, 2>, C>;
// call f(TileCfg) for the selected config; `def` = per-op default config index
// the M-tail launches (below) force the 128x128 config through this override
static thread_local int tl_cfg = -1;
struct TailCfg {
  int saved;
  TailCfg() : saved(tl_cfg) { tl_cfg = 1; }
  ~TailCfg() { tl_cfg = saved; }
};
// M tail: rows past the last full 256-row panel (M = 16 * 4101 = 65616 leaves 80) would cost a whole
// extra round of full-K tiles (e.g. o_proj 3078 tiles on 512 slots = 7 rounds, 6 without the tail);
// they run as a second, small launch on 128x128 tiles instead.  Dev knob S3OD_M_TAIL=0 disables.
static bool split_tail(int M) {
  const int knob = S3OD_KNOB("S3OD_M_TAIL", 1);
  return knob && tl_cfg < 0 && M > 256 && (M & 255) != 0;
}
// the 256x256 ping-pong kernel (one workgroup per CU) only pays when its tiles fill whole rounds of
// the 256 CUs: at bs 8 (M = 32808) o_proj / down-projection / QKV have 384 / 384 / 1152 tiles = 1.5 /
// 1.5 / 4.5 rounds, where the 128x128 config (2 per CU) runs whole rounds (o_proj 138 us at 281 TF/s)
static bool pp_pays(int M, int N) {
  const long tiles = (long)(M / 256) * cdiv(N, 256), rounds = (tiles + 255) / 256;
  return tiles >= 256 && (double)tiles / (double)(rounds * 256) >= 0.95;
}
// Q: the op may run config 6, the 4-wave 256x256 kernel (gemm_q.hip: instantiated for the linears only)
template <typename T, bool Q = false, class F> static int with_cfg(int def, F f) {
  int c = tl_cfg >= 0 ? tl_cfg : gemm_cfg(); if (c < 0) c = def;
  switch (c) {
    case 6:
      if constexpr (Q && sizeof(T) == 2) return f(TileCfg<256, 256, 2, 4, -1>{});
      else return f(TileCfg<128, 128, 2>{});
    case 1: return f(TileCfg<128, 128, 2>{});
    case 2: return f(TileCfg<128, 128, 3>{});
    case 3: return f(TileCfg<256, 128, 2>{});
    case 4: return f(TileCfg<256, 256, 2>{});
    case 5:
      if constexpr (sizeof(T) == 2) return f(TileCfg<256, 256, 2, GEMM_WAVES, 0, true>{});
      else return f(TileCfg<128, 128, 2>{});
    default: return f(TileCfg<256, 128, 3>{});
  }
}

// ------------------------------------------------------------------ QKV + RoPE epilogue
// n in [0,2304): q | k | v ; RoPE on patch tokens for q,k (tf:…/modeling_dinov3_vit.py:238-268);
// q pre-multiplied by the softmax scale 1/8 (exact in any binary float format).
template <typename T> struct EpiQKV {
  T* q; T* k; T* v; const float* bias; const float* cs; const float* sn;
  int M, Ntok, P, H;
  int moff = 0;                       // global token row of local row 0 (M-tail launch)
  DEV void prepare(int) {}
  DEV void operator()(const float* ct, int LDT, int m0, int n0, int tid, int BM, int BN, int NT) const {
    // this thread's fixed 8-column group: bias of its columns and of their RoPE partners (d +- 32)
    float b8[8], bp8[8];
    {
      const int nn = n0 + (tid % (BN / 8)) * 8, dd = nn & 63, dc = dd < 32 ? 32 : -32;
#pragma unroll
      for (int e = 0; e < 8; e++) { b8[e] = bias ? bias[nn + e] : 0.f; bp8[e] = bias ? bias[nn + dc + e] : 0.f; }
    }
    const bool fixed_cols = NT % (BN / 8) == 0;
    for_segments(ct, LDT, BM, BN, m0, n0, M, 3 * H * 64, tid, NT, [&](int m, int n, const float* a, int r, int c) {
      int which = n / (H * 64), nn = n - which * H * 64, h = nn >> 6, d0 = nn & 63;
      int b = (m + moff) / Ntok, t = (m + moff) - b * Ntok;
      float val[8];
#pragma unroll
      for (int e = 0; e < 8; e++) val[e] = a[e] + (fixed_cols ? b8[e] : (bias ? bias[n + e] : 0.f));
      if (which < 2 && t >= Ntok - P) {
        int dc = d0 < 32 ? 32 : -32;
        const float4* pa = (const float4*)(ct + r * LDT + c + dc);
        float4 p0 = pa[0], p1 = pa[1];
        float pv[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
        int tp = t - (Ntok - P);
        const float4* cr = (const float4*)(cs + (long)tp * 64 + d0);
        const float4* sr = (const float4*)(sn + (long)tp * 64 + d0);
        float4 c0 = cr[0], c1 = cr[1], s0 = sr[0], s1 = sr[1];
        float cv[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
        for (int e = 0; e < 8; e++) {
          float q = pv[e] + (fixed_cols ? bp8[e] : (bias ? bias[n + dc + e] : 0.f));
          float rot = d0 < 32 ? -q : q;
          val[e] = val[e] * cv[e] + rot * sv[e];
        }
      }
      if (which == 0) {
#pragma unroll
        for (int e = 0; e < 8; e++) val[e] *= S3OD_QSCALE;
      }
      T* dst = which == 0 ? q : (which == 1 ? k : v);
      store8<T>(dst + (((long)b * H + h) * Ntok + t) * 64 + d0, val);
    });
  }
};

// ------------------------------------------------------------------ fused mask heads
// per pixel: h = relu(conv3x3_64->32NM(feat) + b1) ; logit_k = h[32k:32k+32] . w2[k] + b2[k]
// (src/s3od/model.py:440-452,461-467; the NM Sequential heads run as one N=32NM GEMM)
template <typename T> struct EpiHeads {
  float* logits; T* hsave; const float* b1; const float* w2; const float* b2;
  int M, HW, NM;
  RowMap rm;                                                  // staged row -> pixel (mode 0 dense)
  DEV void prepare(int) {}
  DEV void operator()(const float* ct, int LDT, int m0, int n0, int tid, int BM, int BN, int NT) const {
    const int C = 32 * NM, SPR = 4 * NM;                      // channels / 8-channel segments per row
    // h = relu(acc + b1) is formed on the fly from the staged fp32 tile (no in-place pass)
    if (hsave) {
      const int segs = BM * SPR;
      for (int s = tid; s < segs; s += NT) {
        int r = s / SPR, c = (s - r * SPR) * 8, m = m0 + r;
        if (m >= M) continue;
        const long px = rm.map(m);
        if (px < 0) continue;
        const float4* src = (const float4*)(ct + r * LDT + c);
        float4 x0 = src[0], x1 = src[1];
        float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
        for (int e = 0; e < 8; e++) v[e] = fmaxf(v[e] + b1[c + e], 0.f);
        store8<T>(hsave + px * C + c, v);
      }
    }
    // logit_k = b2[k] + sum_j relu(acc[32k + j] + b1[32k + j]) * w2[32k + j]; k is wave-uniform
    for (int s = tid; s < NM * BM; s += NT) {
      int k = s / BM, r = s - k * BM;
      int m = m0 + r;
      if (m >= M) continue;
      const long px = rm.map(m);
      if (px < 0) continue;
      const float4* row = (const float4*)(ct + r * LDT + 32 * k);
      const float* bb = b1 + 32 * k;
      const float* ww = w2 + 32 * k;
      float acc = b2[k];
#pragma unroll
      for (int q = 0; q < 8; q++) {
        float4 x = row[q];
        acc += fmaxf(x.x + bb[4 * q + 0], 0.f) * ww[4 * q + 0];
        acc += fmaxf(x.y + bb[4 * q + 1], 0.f) * ww[4 * q + 1];
        acc += fmaxf(x.z + bb[4 * q + 2], 0.f) * ww[4 * q + 2];
        acc += fmaxf(x.w + bb[4 * q + 3], 0.f) * ww[4 * q + 3];
      }
      const long b = px / HW, pix = px - b * HW;
      logits[(b * NM + k) * HW + pix] = acc;
    }
  }
};


// ---------------------------------------------------------------- register-weight 3x3 conv, 64 -> 64
// The full-resolution 64-channel convs (upsample_2x.2 forward and its stride-1 data gradient) move
// 4.3 / 6.4 GB per call at bs 16 (1024^2): HBM-bound at ~5.5 TB/s if loads, MFMAs and stores overlap.
//   * one workgroup of 4 waves per CU (one wave per SIMD); wave w = output rows 4 (w>>1) .. +3 of the
//     tile x output channels 32 (w&1) .. +31 and holds those channels' 9 taps x 64 weights as MFMA A
//     fragments in registers (144 VGPRs), so the only LDS traffic is the input halo (B fragments);
//   * tile = 8 x 32 output pixels; its (8+2) x (32+2) x 64 halo arrives by LDS-DMA (44 x 1 KiB pieces,
//     11 per wave, zeros outside the image via the buffer range check) into a 3-deep ring, issued two
//     tiles ahead, so the only per-tile synchronisation is one s_barrier behind a counted vmcnt;
//   * the epilogue runs from the accumulators: bias / ReLU (forward) or the ReLU' mask of res1 (data
//     gradient, its rows loaded at the start of the tile), the lane pair (lg, lg^1) trades 4-channel
//     groups so every lane stores one 16-B run of 8 channels per 16-pixel block; column sums of the
//     output (bias gradient) go through LDS atomics, one global flush per workgroup.
// Input channels CI = 64 (tile 8 x 32) or 96 (the mask heads' data gradient: tile 8 x 16, 192-B halo rows).
template <int CI> struct RwShape {
  static constexpr int TH = 8, TW = CI == 64 ? 32 : 16, HC = TW + 2, PX = (TH + 2) * HC;   // halo pixels
  static constexpr int ROWB = CI * 2, KK = CI / 32, NPC = TW / 16, PB = 4 * NPC;          // 16-px blocks per wave
  static constexpr int PIECES = ((PX * ROWB + 4095) / 4096) * 4, PPW = PIECES / 4;        // 1 KiB DMA pieces
  static constexpr int BUF = PIECES * 1024, LDS = 3 * BUF + 2048;       // + bias / column sums / head partials
  // grouped mask heads: 3 tile slots of head partials [wave 4][row 4][block 2][head 3][lane 16] floats after that
  static constexpr int PSLOT = 4 * 4 * 2 * 3 * 16, LDS_H = LDS + 3 * PSLOT * 4;
  static_assert(LDS <= 160 * 1024 && (CI != 64 || LDS_H <= 160 * 1024), "register-weight conv LDS budget");
  // 16-B slot of logical chunk c in halo row px (an involution; conflict-free ds_read_b128 for every tap offset,
  // checked against the gfx950 lane groups): CI 64: c ^ (px & 7); CI 96: XOR of the low 2 bits, groups of 4 kept
  DEV static int slot(int c, int px) {
    if constexpr (CI == 64) return c ^ (px & 7);
    else return (c & ~3) | ((c & 3) ^ ((px ^ (px >> 1)) & 3));
  }
};

// MODE 0: out = acc + bias;  MODE 2: out = ReLU(acc + bias);  MODE 1: out = res1 > 0 ? acc : 0, colsum += out;
// MODE 3: the 3 mask heads (src/s3od/model.py:440-452,461-467): 96 output channels (48 per wave, NB = 3),
//   h = ReLU(acc + b1) -> hsave (bf16 [px][96]) and logit_k = b2[k] + h[32k .. 32k+31] . w2[k] -> logits [B][3][H][W];
//   head 1 straddles the two waves of a row group: the odd wave's part goes through LDS (one extra barrier)
// Every wave issues a FIXED sequence of vector-memory instructions per tile (PPW DMA pieces, PB mask loads, PB stores:
// dummy pieces / out-of-image lanes use an out-of-range buffer offset instead of a branch), so the counted vmcnt
// that retires a tile's halo is a per-phase constant.
// GB > 0 (MODE 0 / 2; mode 1 is launched ungrouped, see launch_rw): the tile's PB blocks run in groups of GB (all 9 * KK steps of one group's GB x NB accumulators,
// then the next group's), and each group's epilogue (ReLU / mask, lane-pair trade, pack, store) is issued between the
// NEXT group's MFMAs -- the last group's carried into the next tile's first group (a dummy group with out-of-range
// stores before the first tile) -- so with one wave per SIMD the matrix pipe no longer idles through the epilogue.
// Same MFMA chain per accumulator (outputs bit-identical to GB = 0); per tile still PB stores after the halo issue,
// so the counted waits are unchanged.
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
template <int MODE, int CI, int GB>
__global__ void __launch_bounds__(256, 1) conv3x3_c64_rw_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                                 const float* __restrict__ bias,
                                                                 const bf16* __restrict__ res1, float* __restrict__ colsum,
                                                                 bf16* __restrict__ out, int H, int W, int tiles_x,
                                                                 int tiles_y, int ntiles, const float* __restrict__ w2,
                                                                 const float* __restrict__ b2, float* __restrict__ logits) {
  typedef RwShape<CI> S;
  constexpr int PB = S::PB, PPW = S::PPW, NPC = S::NPC, HC = S::HC, ROWB = S::ROWB;
  constexpr int NB = MODE == 3 ? 3 : 2, CO = 32 * NB;     // 16-channel blocks per wave / output channels
  static_assert(MODE != 3 || (CI == 64 && NPC == 2), "mask heads: 64 input channels, 8 x 32 tiles");
  static_assert(GB == 0 || (MODE != 3 && PB % GB == 0) || (MODE == 3 && GB == NPC), "grouped epilogue: whole groups (heads: one row)");
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int lr = lane & 15, lg = lane >> 4, odd = lg & 1;
  const int row0 = 4 * (wave >> 1), ch0 = 16 * NB * (wave & 1);   // this wave's output rows / channels
  // tiles: XCD x = blockIdx % 8 owns the contiguous range [x*n/8, (x+1)*n/8) (neighbouring tiles share halo
  // rows in that XCD's L2); its workgroups stride through it
  const int nwg = gridDim.x, xcd = blockIdx.x & 7, wpx = (nwg + 7 - xcd) >> 3, wi = blockIdx.x >> 3;
  const int t_beg = (int)((long)ntiles * xcd / 8), t_end = (int)((long)ntiles * (xcd + 1) / 8);
  const long img_i = (long)H * W * CI, img_o = (long)H * W * CO;    // elements per image

  // weights -> registers: lane (lr, lg) holds w[co = ch0 + 16 nb + lr][tap][ci = 32 kk + 8 lg .. +7]
  bf16x8 wr[9][S::KK][NB];
#pragma unroll
  for (int tap = 0; tap < 9; tap++)
#pragma unroll
    for (int kk = 0; kk < S::KK; kk++)
#pragma unroll
      for (int nb = 0; nb < NB; nb++)
        wr[tap][kk][nb] = *(const bf16x8*)(w + ((long)(ch0 + nb * 16 + lr) * 9 + tap) * CI + kk * 32 + lg * 8);

  // DMA lane constants: piece p = PPW wave + i covers LDS bytes [1024 p, 1024 p + 1024) of a ring slot, laid out
  // [px][16-B slot]; lane writes bytes 16 lane .. +15 of the piece = logical chunk slot^-1 of pixel px
  int dm[PPW];
#pragma unroll
  for (int i = 0; i < PPW; i++) {
    const int b = (wave * PPW + i) * 1024 + lane * 16, px = b / ROWB, ch = S::slot((b % ROWB) >> 4, px);
    dm[i] = px < S::PX ? ((px / HC) << 16) | ((px % HC) << 4) | ch : -1;
  }
  auto issue = [&](int tile, int slot) {            // tile >= t_end: dummy pieces (zeros into a free slot)
    const bool live = tile < t_end;
    const int tc = live ? tile : t_beg;
    const int txi = tc % tiles_x, t2 = tc / tiles_x, tyi = t2 % tiles_y, bb = t2 / tiles_y;
    const int ty0 = tyi * S::TH - 1, tx0 = txi * S::TW - 1;
    const auto r = make_rsrc(x + bb * img_i, (unsigned long)img_i * 2);
    char* dst = smem + slot * S::BUF + wave * PPW * 1024;
#pragma unroll
    for (int i = 0; i < PPW; i++) {
      const int v = dm[i], gy = ty0 + (v >> 16), gx = tx0 + ((v >> 4) & 0xfff);
      const bool ok = live && v >= 0 && (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
      blds16(r, ok ? (unsigned)((gy * W + gx) * ROWB + (v & 15) * 16) : 0x80000000u, dst + i * 1024);
    }
  };
  // halo fragment addresses: px = L + off (L = row0 * HC + lr per lane, off compile-time per (block, tap)); the
  // slot term depends on the lane and on off & 7 only, so yb[off & 7][kk] + ROWB * off = per-lane base + immediate
  int yb[8][S::KK];
  {
    const int L = row0 * HC + lr;
#pragma unroll
    for (int j = 0; j < 8; j++)
#pragma unroll
      for (int kk = 0; kk < S::KK; kk++) yb[j][kk] = L * ROWB + 16 * S::slot(kk * 4 + lg, L + j);
  }
  // after the lane-pair trade in the epilogue a lane owns channels cb .. cb+7 of its pixel
  const int cb = ch0 + (odd ? 16 : 0) + 8 * (lg >> 1);
  // 64 floats after the ring: the bias (MODE 0/2, the accumulators' initial value) or the column sums (MODE 1)
  // MODE 3: aux[0..95] = b1, aux[96..191] = w2, aux[192..194] = b2, aux[256..511] = head-1 partials [8 rows][32 px]
  float* aux = (float*)(smem + 3 * S::BUF);
  if (tid < CO) aux[tid] = (MODE != 1 && bias) ? bias[tid] : 0.f;
  if constexpr (MODE == 3) {
    if (tid < 96) aux[96 + tid] = w2[tid];
    if (tid < 3) aux[192 + tid] = b2[tid];
  }
  __syncthreads();
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

  // GB > 0: the carried group (accumulators, store offsets, masks, output descriptor); a dummy before the first tile
  constexpr int GBC = GB > 0 ? GB : 1;
  f32x4 cacc[GBC][NB];
  unsigned cpo[GBC];
  u32x4v crm[GBC];
#pragma unroll
  for (int q = 0; q < GBC; q++) {
    cpo[q] = 0x80000000u;
    crm[q] = u32x4v{0u, 0u, 0u, 0u};
#pragma unroll
    for (int nb = 0; nb < NB; nb++) cacc[q][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  int cbb = 0;                                        // batch index of the carried group's tile
  // epilogue of one 16-px block: lane holds out[px = block, lr][co = ch0 + 16 nb + 4 lg .. +3]; v_permlane16_swap
  // trades rows 1 / 3 of the first operand with rows 0 / 2 of the second (row = 16 lanes = one lg): the even lg keeps
  // its nb 0 and receives the odd partner's nb 0, the odd lg keeps nb 1 and receives the even's -> channels cb .. cb+7
  // (the output descriptor is built here from the batch index: in a round-5 build a descriptor carried across tiles
  // in SGPRs lost its range word in the grouped mode-1 instance, whose in-tile group stores were dropped)
  auto epi_blk = [&](const f32x4 (&a)[NB], unsigned p, u32x4v mraw, int bbx) {
    const auto r = make_rsrc(out + bbx * img_o, out ? (unsigned long)img_o * 2 : 0ul);
    float o[8];
#pragma unroll
    for (int e = 0; e < 4; e++) {
      float v0 = a[0][e], v1 = a[1][e];
      if (MODE == 2) { v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); }
      const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(v0), __float_as_uint(v1), false, false);
      o[e] = __uint_as_float(sw[0]);               // channels cb + 0..3
      o[4 + e] = __uint_as_float(sw[1]);           // channels cb + 4..7
    }
    if constexpr (MODE == 1) {
      const bf16x8 m = __builtin_bit_cast(bf16x8, mraw);
#pragma unroll
      for (int e = 0; e < 8; e++) o[e] = (float)m[e] > 0.f ? o[e] : 0.f;   // out-of-image lanes: mask reads 0
#pragma unroll
      for (int e = 0; e < 8; e++) cs[e] += o[e];     // column sums of channels cb .. cb+7 (lane partials)
    }
    bf16x8 ob;
#pragma unroll
    for (int e = 0; e < 8; e++) ob[e] = (bf16)o[e];
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, ob), r, p, 0, 0);
  };
  // MODE 3, grouped: a block's epilogue (h = ReLU(acc) -> hsave, the three head partials summed over the 4 lg lanes
  // -> LDS slot `slot` [wave][row r][block c][head][lr]); the logits of tile t are stored two tiles later, after the
  // per-tile barrier has made both waves' partials visible (3 slots: a slot is rewritten only after every wave has
  // passed the barrier behind its reads), in the same summation order as the ungrouped path (bit-identical)
  int cslot = 2, cgi = 0;                             // the carried group's partial slot / row (dummy: slot of tile -1)
  float* pslots = (float*)(smem + 3 * S::BUF + 2048);
  auto pix = [&](int slot, int w, int r, int c, int h, int l) { return ((((slot * 4 + w) * 4 + r) * 2 + c) * 3 + h) * 16 + l; };
  auto epi_head = [&](const f32x4 (&a)[NB], unsigned p, int bbx, int slot, int r, int c) {
    const auto rs = make_rsrc(out + bbx * img_o, out ? (unsigned long)img_o * 2 : 0ul);
    float v[NB][4];
#pragma unroll
    for (int nb = 0; nb < NB; nb++)
#pragma unroll
      for (int e = 0; e < 4; e++) v[nb][e] = fmaxf(a[nb][e], 0.f);
    float o[8];
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[0][e]), __float_as_uint(v[1][e]), false, false);
      o[e] = __uint_as_float(sw[0]);
      o[4 + e] = __uint_as_float(sw[1]);
    }
    bf16x8 ob;
#pragma unroll
    for (int e = 0; e < 8; e++) ob[e] = (bf16)o[e];
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, ob), rs, p, 0, 0);
    if constexpr (NB == 3) {
      const unsigned p2 = p == 0x80000000u ? p : p - cb * 2 + (ch0 + 32 + 4 * lg) * 2;
      const bf16x4 o2 = {(bf16)v[2][0], (bf16)v[2][1], (bf16)v[2][2], (bf16)v[2][3]};
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, o2), rs, p2, 0, 0);
    }
#pragma unroll
    for (int nb = 0; nb < NB; nb++) {
      float d = 0.f;
#pragma unroll
      for (int e = 0; e < 4; e++) d += v[nb][e] * aux[96 + ch0 + 16 * nb + 4 * lg + e];
      d += __shfl_xor(d, 16);
      d += __shfl_xor(d, 32);
      if (lg == 0) pslots[pix(slot, wave, r, c, nb, lr)] = d;
    }
  };
  auto store_logits = [&](int tt, bool valid, int slot) {
    const int tc = valid ? tt : t_beg;
    const int txi = tc % tiles_x, t2 = tc / tiles_x, tyi = t2 % tiles_y, bb = t2 / tiles_y;
    const auto rl = make_rsrc(logits + (long)bb * 3 * H * W, (unsigned long)3 * H * W * 4);
    const int c = lg & 1;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int gy = tyi * S::TH + row0 + r, gx = txi * S::TW + c * 16 + lr;
      const bool ok = valid && lg < 2 && gy < H && gx < W;
      const unsigned base = (unsigned)(gy * W + gx) * 4;
      if (!(wave & 1)) {
        const float l0 = aux[192] + pslots[pix(slot, wave, r, c, 0, lr)] + pslots[pix(slot, wave, r, c, 1, lr)];
        const float l1 = aux[193] + pslots[pix(slot, wave, r, c, 2, lr)] + pslots[pix(slot, wave + 1, r, c, 0, lr)];
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(l0), rl, ok ? base : 0x80000000u, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(l1), rl, ok ? base + (unsigned)H * W * 4 : 0x80000000u, 0, 0);
      } else {
        const float l2 = aux[194] + pslots[pix(slot, wave, r, c, 1, lr)] + pslots[pix(slot, wave, r, c, 2, lr)];
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(l2), rl, ok ? base + 2u * H * W * 4 : 0x80000000u, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(0u, rl, 0x80000000u, 0, 0);   // keeps the per-tile store count uniform
      }
    }
  };
  (void)epi_head; (void)store_logits; (void)pix;

  int tile = t_beg + wi, k = 0;
  issue(tile, 0);
  issue(tile + wpx, 1);
  for (; tile < t_end; tile += wpx, k++) {
    const int txi = tile % tiles_x, t2 = tile / tiles_x, tyi = t2 % tiles_y, bb = t2 / tiles_y;
    const auto ro = make_rsrc(out + bb * img_o, out ? (unsigned long)img_o * 2 : 0ul);   // MODE 3: hsave is optional
    unsigned po[PB];                                  // byte offset of this lane's 8-channel run per 16-px block (or OOB)
#pragma unroll
    for (int pb = 0; pb < PB; pb++) {
      const int gy = tyi * S::TH + row0 + pb / NPC, gx = txi * S::TW + (pb % NPC) * 16 + lr;
      po[pb] = (gy < H && gx < W) ? (unsigned)((gy * W + gx) * (CO * 2) + cb * 2) : 0x80000000u;
    }
    // data-gradient mask runs of this tile, issued before the next halo's DMA (their wait leaves it in flight)
    u32x4v rm_[PB];
    if constexpr (MODE == 1) {
      const auto rr = make_rsrc(res1 + bb * img_o, (unsigned long)img_o * 2);
#pragma unroll
      for (int pb = 0; pb < PB; pb++) rm_[pb] = __builtin_amdgcn_raw_buffer_load_b128(rr, po[pb], 0, 0);
    }
    // retire this tile's halo (own pieces): the vector-memory ops issued after them are a per-phase constant
    //   k = 0: next halo [+ masks];  k = 1: [masks,] halo, stores [, masks];  k >= 2: stores [, masks], halo, stores [, masks]
    //   (MODE 3 stores 2 PB hsave runs + 8 logit rows = 3 PB per tile)
    constexpr int NS = MODE == 3 ? 3 * PB : PB;       // stores per tile
    if (k == 0) { if constexpr (MODE == 1) wait_vmcnt<PPW + PB>(); else wait_vmcnt<PPW>(); }
    else if (k == 1) { if constexpr (MODE == 1) wait_vmcnt<PB + PPW + PB + PB>(); else wait_vmcnt<PPW + NS>(); }
    else { if constexpr (MODE == 1) wait_vmcnt<PB + PB + PPW + PB + PB>(); else wait_vmcnt<NS + PPW + NS>(); }
    if constexpr (MODE == 3 && GB > 0) wait_lgkm0();  // this wave's head partials written before the barrier
    __builtin_amdgcn_s_barrier();                     // every wave's pieces landed; every wave done with slot k-1
    asm volatile("" ::: "memory");
    issue(tile + 2 * wpx, (k + 2) % 3);
    const char* hb = smem + (k % 3) * S::BUF;
    constexpr int NST = 9 * S::KK;
    if constexpr (GB > 0) {
      if constexpr (MODE == 3) store_logits(tile - 2 * wpx, k >= 2, (k + 1) % 3);
      // fragments of group gi's GB blocks for step st; the group's MFMAs; the carried group's epilogue in the first
      // GB step pairs
      auto rd_g = [&](int gi, int st, bf16x8 (&fa)[GB]) {
        const int tap = st / S::KK, kk = st % S::KK, dy = tap / 3, dx = tap - 3 * (tap / 3);
#pragma unroll
        for (int q = 0; q < GB; q++) {
          const int pb = gi * GB + q, off = (pb / NPC + dy) * HC + (pb % NPC) * 16 + dx;
          fa[q] = *(const bf16x8*)(hb + yb[off & 7][kk] + off * ROWB);
        }
      };
#pragma unroll
      for (int gi = 0; gi < PB / GB; gi++) {
        f32x4 acc[GB][NB];
#pragma unroll
        for (int nb = 0; nb < NB; nb++) {
          const f32x4 b0 = MODE != 1 ? *(const f32x4*)(aux + ch0 + nb * 16 + 4 * lg) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int q = 0; q < GB; q++) acc[q][nb] = b0;
        }
        auto mm_g = [&](int st, const bf16x8 (&fa)[GB]) {
#pragma unroll
          for (int q = 0; q < GB; q++)
#pragma unroll
            for (int nb = 0; nb < NB; nb++)
              acc[q][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[st / S::KK][st % S::KK][nb], fa[q], acc[q][nb], 0, 0, 0);
        };
        bf16x8 fa0[GB], fa1[GB];
        rd_g(gi, 0, fa0);
#pragma unroll
        for (int st = 0; st < NST; st += 2) {
          if (st + 1 < NST) rd_g(gi, st + 1, fa1);
          __builtin_amdgcn_sched_barrier(0);
          mm_g(st, fa0);
          if (st / 2 < GB) {
            if constexpr (MODE == 3) epi_head(cacc[st / 2], cpo[st / 2], cbb, cslot, cgi, st / 2);
            else epi_blk(cacc[st / 2], cpo[st / 2], crm[st / 2], cbb);
          }
          __builtin_amdgcn_sched_barrier(0);
          if (st + 2 < NST) rd_g(gi, st + 2, fa0);
          __builtin_amdgcn_sched_barrier(0);
          if (st + 1 < NST) mm_g(st + 1, fa1);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int q = 0; q < GB; q++) {
#pragma unroll
          for (int nb = 0; nb < NB; nb++) cacc[q][nb] = acc[q][nb];
          cpo[q] = po[gi * GB + q];
          if constexpr (MODE == 1) crm[q] = rm_[gi * GB + q];
        }
        cbb = bb;
        cslot = k % 3;
        cgi = gi;
      }
      continue;
    }
    f32x4 acc[PB][NB];                                // acc[pb][nb]: D[co = ch0 + 16 nb + 4 lg + e][px = block pb, lr]
#pragma unroll
    for (int nb = 0; nb < NB; nb++) {
      const f32x4 b0 = MODE != 1 ? *(const f32x4*)(aux + ch0 + nb * 16 + 4 * lg) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int pb = 0; pb < PB; pb++) acc[pb][nb] = b0;
    }
    // 9 * KK (tap, k-chunk) steps of 2 PB MFMAs; the next step's PB halo fragments are read before this step's MFMAs
    auto rd = [&](int st, bf16x8 (&fa)[PB]) {
      const int tap = st / S::KK, kk = st % S::KK, dy = tap / 3, dx = tap - 3 * (tap / 3);
#pragma unroll
      for (int pb = 0; pb < PB; pb++) {
        const int off = (pb / NPC + dy) * HC + (pb % NPC) * 16 + dx;
        fa[pb] = *(const bf16x8*)(hb + yb[off & 7][kk] + off * ROWB);
      }
    };
    auto mm = [&](int st, const bf16x8 (&fa)[PB]) {
#pragma unroll
      for (int pb = 0; pb < PB; pb++)
#pragma unroll
        for (int nb = 0; nb < NB; nb++)
          acc[pb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[st / S::KK][st % S::KK][nb], fa[pb], acc[pb][nb], 0, 0, 0);
    };
    bf16x8 fa0[PB], fa1[PB];
    rd(0, fa0);
#pragma unroll
    for (int st = 0; st < NST; st += 2) {
      if (st + 1 < NST) rd(st + 1, fa1);
      __builtin_amdgcn_sched_barrier(0);
      mm(st, fa0);
      __builtin_amdgcn_sched_barrier(0);
      if (st + 2 < NST) rd(st + 2, fa0);
      __builtin_amdgcn_sched_barrier(0);
      if (st + 1 < NST) mm(st + 1, fa1);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (MODE == 3) {
      // h = ReLU(acc) (b1 was the initial value); hsave: channels cb .. cb+7 (nb 0 / 1 traded as below) and
      // ch0 + 32 + 4 lg .. +3 (nb 2); head partials: per 16-channel block, summed over the 4 lg lanes
      float hp[PB][3];
#pragma unroll
      for (int pb = 0; pb < PB; pb++) {
        float v[3][4];
#pragma unroll
        for (int nb = 0; nb < 3; nb++)
#pragma unroll
          for (int e = 0; e < 4; e++) v[nb][e] = fmaxf(acc[pb][nb][e], 0.f);
        float o[8];
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[0][e]), __float_as_uint(v[1][e]), false, false);
          o[e] = __uint_as_float(sw[0]);
          o[4 + e] = __uint_as_float(sw[1]);
        }
        bf16x8 ob;
#pragma unroll
        for (int e = 0; e < 8; e++) ob[e] = (bf16)o[e];
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, ob), ro, po[pb], 0, 0);
        const unsigned p2 = po[pb] == 0x80000000u ? po[pb] : po[pb] - cb * 2 + (ch0 + 32 + 4 * lg) * 2;
        const bf16x4 o2 = {(bf16)v[2][0], (bf16)v[2][1], (bf16)v[2][2], (bf16)v[2][3]};
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, o2), ro, p2, 0, 0);
#pragma unroll
        for (int nb = 0; nb < 3; nb++) {
          float d = 0.f;
#pragma unroll
          for (int e = 0; e < 4; e++) d += v[nb][e] * aux[96 + ch0 + 16 * nb + 4 * lg + e];
          d += __shfl_xor(d, 16);
          d += __shfl_xor(d, 32);
          hp[pb][nb] = d;
        }
      }
      // wave half 0 (channels 0-47): head 0 = blocks 0 + 1, head 1 = block 2 + the odd wave's block 0;
      // half 1 (48-95): head 2 = blocks 1 + 2
      float* part = aux + 256 + (row0 + 0) * 32;
      if (wave & 1) {
#pragma unroll
        for (int pb = 0; pb < PB; pb++)
          if (lg == 0) part[(pb / NPC) * 32 + (pb % NPC) * 16 + lr] = hp[pb][0];
      }
      lds_barrier();
      const auto rl = make_rsrc(logits + (long)bb * 3 * H * W, (unsigned long)3 * H * W * 4);
#pragma unroll
      for (int r = 0; r < 4; r++) {
        // lanes lg 0 / 1 store the row's two 16-pixel blocks (64 + 64 contiguous bytes); lg 2 / 3 are out of range
        const int gy = tyi * S::TH + row0 + r, gx = txi * S::TW + (lg & 1) * 16 + lr;
        const bool ok = lg < 2 && gy < H && gx < W;
        const int pb = 2 * r + (lg & 1);
        const unsigned base = (unsigned)(gy * W + gx) * 4;
        if (!(wave & 1)) {
          const float l0 = aux[192] + hp[2 * r][0] + hp[2 * r][1], l0b = aux[192] + hp[2 * r + 1][0] + hp[2 * r + 1][1];
          const float l1 = aux[193] + hp[2 * r][2] + part[r * 32 + lr], l1b = aux[193] + hp[2 * r + 1][2] + part[r * 32 + 16 + lr];
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((lg & 1) ? l0b : l0), rl, ok ? base : 0x80000000u, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((lg & 1) ? l1b : l1), rl, ok ? base + (unsigned)H * W * 4 : 0x80000000u, 0, 0);
        } else {
          const float l2 = aux[194] + hp[2 * r][1] + hp[2 * r][2], l2b = aux[194] + hp[2 * r + 1][1] + hp[2 * r + 1][2];
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((lg & 1) ? l2b : l2), rl, ok ? base + 2u * H * W * 4 : 0x80000000u, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b32(0u, rl, 0x80000000u, 0, 0);   // keeps the per-tile store count uniform
        }
        (void)pb;
      }
    } else {
#pragma unroll
      for (int pb = 0; pb < PB; pb++) epi_blk(acc[pb], po[pb], rm_[pb], bb);
    }
  }
  if constexpr (GB > 0) {                             // the last tile's carried group
    if constexpr (MODE == 3) {
#pragma unroll
      for (int q = 0; q < GB; q++) epi_head(cacc[q], cpo[q], cbb, cslot, cgi, q);
      lds_barrier();                                  // the last two tiles' partials complete: store their logits
      store_logits(tile - 2 * wpx, k >= 2, (k + 1) % 3);
      store_logits(tile - wpx, k >= 1, (k + 2) % 3);
    } else {
#pragma unroll
      for (int q = 0; q < GB; q++) epi_blk(cacc[q], cpo[q], crm[q], cbb);
    }
  }
  if (MODE == 1 && colsum) {                          // 16 lanes (lr) -> 1, LDS atomics, one global add per channel
#pragma unroll
    for (int e = 0; e < 8; e++) {
      float c = cs[e];
      c += __shfl_xor(c, 1); c += __shfl_xor(c, 2); c += __shfl_xor(c, 4); c += __shfl_xor(c, 8);
      if (lr == 0) atomicAdd(aux + cb + e, c);
    }
    __syncthreads();
    if (tid < 64) atomicAdd(colsum + tid, aux[tid]);
  }
  wait_vmcnt<0>();        // no LDS-DMA (dummy pieces included) may still be landing when the workgroup retires
}

// S3OD_CONV_RW=0 disables the path (an A/B inside one process under S3OD_AB=1)
static bool rw_ok(int dtype, int B, int H, int W) {
  return dtype == S3OD_BF16 && !S3OD_OFF("S3OD_CONV_RW") && (long)H * W * 192 < (1L << 31) && B > 0;
}
template <int MODE, int CI, int GB>
static int launch_rw_g(const bf16* x, const bf16* w, const float* bias, const bf16* res1, float* colsum, bf16* out,
                       int B, int H, int W, hipStream_t st, const float* w2, const float* b2, float* logits) {
  typedef RwShape<CI> S;
  auto kfn = conv3x3_c64_rw_kernel<MODE, CI, GB>;
  constexpr int LDS = MODE == 3 && GB > 0 ? S::LDS_H : S::LDS;
  static const bool attr = ((void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, LDS), true);   // once per process (thread-safe static init)
  (void)attr;
  const int tx = cdiv(W, S::TW), ty = cdiv(H, S::TH);
  const long tiles = (long)B * tx * ty;
  if (tiles >= (1L << 31)) { s3od_set_error("conv rw: too many tiles"); return 22; }
    const int nwg = (int)std::min<long>(std::max<long>(tiles, 8), (long)s3od_cu_count());   // one persistent WG per CU, >= 8 so every XCD owns its range
  hipLaunchKernelGGL(kfn, dim3(nwg), dim3(256), LDS, st, x, w, bias, res1, colsum, out, H, W, tx, ty, (int)tiles, w2, b2,
                     logits);
  return s3od_check_launch("conv3x3_c64_rw");
}
// modes 0 / 2 (forward): the grouped epilogue (S3OD_RW_GB = blocks per group: 2 default, or 0 = the epilogue after all
// MFMAs).  Measured (tools/conv64_bench.py, bs 16 x 1024^2 64 -> 64 + ReLU, same box): GB 0 1290-1309 us, GB 2 1225-1242,
// GB 4 1251-1280 (profiles/r05t_rw_grouped_epilogue.txt; GB 4 removed in round 6).
// Mode 1 (the ReLU'-masked data gradient) runs ungrouped: its grouped instances were the only register-weight convs
// that spill (GB 2: 62 SGPRs into VGPR lanes + 6 VGPRs into AGPRs; GB 4: 40 + 16), and GB 4 produced wrong outputs
// (in-tile group stores dropped / masks misapplied) although its vector-memory order matches the hand-counted waits
// (ISA audit); GB 2 saved only 60-110 us per step.  tests/test_kernel_resources_cpu.py keeps every
// counted-vmcnt production kernel free of scratch and VGPR spills.
template <int MODE, int CI>
static int launch_rw(const bf16* x, const bf16* w, const float* bias, const bf16* res1, float* colsum, bf16* out,
                     int B, int H, int W, hipStream_t st, const float* w2 = nullptr, const float* b2 = nullptr,
                     float* logits = nullptr) {
  if constexpr (MODE == 3) {
    // mask heads grouped by output row (S3OD_RW_HGB=2, opt-in): bit-identical but slower, 2160-2174 -> 2421-2424 us at
    // bs 16 x 1024^2 (the weights' AGPR reads double the loop's VALU; profiles/r05t_rw_grouped_epilogue.txt)
    if (S3OD_KNOB("S3OD_RW_HGB", 0) == 2) return launch_rw_g<3, CI, 2>(x, w, bias, res1, colsum, out, B, H, W, st, w2, b2, logits);
  } else if constexpr (MODE != 1) {
    if (S3OD_KNOB("S3OD_RW_GB", 2) == 2) return launch_rw_g<MODE, CI, 2>(x, w, bias, res1, colsum, out, B, H, W, st, w2, b2, logits);
  }
  return launch_rw_g<MODE, CI, 0>(x, w, bias, res1, colsum, out, B, H, W, st, w2, b2, logits);
}

// ---------------------------------------------------------------- register-weight ConvTranspose2d(128, 64, 4, s2, p1)
// upsample_2x.0 of the output head (src/s3od/model.py:146-153: 512^2 x 128 -> 1024^2 x 64, bias, ReLU) moves 3.2 GB
// per call at bs 16; the generic path (conv data gradient, one implicit GEMM per output parity class) ran it at
// 2.56 ms.  Sub-pixel decomposition: output pixel (2j + py, 2i + px) = bias + sum over the 2 x 2 taps
// ky = 1 - py + 2a, kx = 1 - px + 2c of x[j + py - a][i + px - c] . W[:, :, ky, kx], i.e. four 2x2 convs of x.
//   * tile = 8 x 16 input pixels (-> 16 x 32 output pixels); its (8+2) x (16+2) x 128 halo arrives by LDS-DMA into a
//     3-deep ring, rows padded to 288 B (two dummy 16-B slots, conflict-free ds_read_b128 for every tap offset);
//   * wave w: output row parity py = w >> 1, output channels 32 (w & 1) .. +31, both column parities in turn; its
//     2 classes x 4 taps x 128 x 32 weights sit in registers as MFMA A fragments (256 VGPRs, gathered once);
//   * epilogue as in the 3x3 kernel: bias is the accumulators' initial value, ReLU, lane-pair channel trade,
//     one 16-B store per lane per 16-pixel block (stride-2 output columns; the other parity's wave fills the gaps).
namespace ct {
constexpr int TH = 8, TW = 16, HC = TW + 2, PX = (TH + 2) * HC, ROWB = 288;          // 18 slots of 16 B per pixel
constexpr int PIECES = ((PX * ROWB + 4095) / 4096) * 4, PPW = PIECES / 4, BUF = PIECES * 1024, LDS = 3 * BUF + 1024;
static_assert(LDS <= 160 * 1024, "convT LDS budget");
}  // namespace ct
template <bool RELU>
__global__ void __launch_bounds__(256, 1) convT4s2_rw_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wt,
                                                              const float* __restrict__ bias, bf16* __restrict__ out,
                                                              int H, int W, int tiles_x, int tiles_y, int ntiles) {
  using namespace ct;
  constexpr int NS = 16;                                            // stores per tile per wave (2 classes x 8 rows)
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int lr = lane & 15, lg = lane >> 4, odd = lg & 1;
  const int py = wave >> 1, ch0 = 32 * (wave & 1);
  const int nwg = gridDim.x, xcd = blockIdx.x & 7, wpx = (nwg + 7 - xcd) >> 3, wi = blockIdx.x >> 3;
  const int t_beg = (int)((long)ntiles * xcd / 8), t_end = (int)((long)ntiles * (xcd + 1) / 8);
  const long img_i = (long)H * W * 128, img_o = (long)4 * H * W * 64;

  // weights: wt = [co = 64][ky][kx][ci = 128] (ConvTranspose2d weight [128][64][4][4] transposed, s3od_repack_multi
  // mode 2); wr[pxc][s][nb], s = (2a + c) * 4 + kk: lane (lr, lg) holds W[co = ch0 + 16 nb + lr][ky][kx][ci = 32 kk + 8 lg ..]
  bf16x8 wr[2][16][2];
#pragma unroll
  for (int pxc = 0; pxc < 2; pxc++)
#pragma unroll
    for (int s = 0; s < 16; s++)
#pragma unroll
      for (int nb = 0; nb < 2; nb++) {
        const int a = s >> 3, c = (s >> 2) & 1, kk = s & 3, ky = 1 - py + 2 * a, kx = 1 - pxc + 2 * c;
        wr[pxc][s][nb] = *(const bf16x8*)(wt + ((ch0 + nb * 16 + lr) * 16 + ky * 4 + kx) * 128 + kk * 32 + lg * 8);
      }
  int dm[PPW];
#pragma unroll
  for (int i = 0; i < PPW; i++) {
    const int b = (wave * PPW + i) * 1024 + lane * 16, px = b / ROWB, ch = (b % ROWB) >> 4;
    dm[i] = (px < PX && ch < 16) ? ((px / HC) << 16) | ((px % HC) << 4) | ch : -1;
  }
  auto issue = [&](int tile, int slot) {
    const bool live = tile < t_end;
    const int tc = live ? tile : t_beg;
    const int txi = tc % tiles_x, t2 = tc / tiles_x, tyi = t2 % tiles_y, bb = t2 / tiles_y;
    const int ty0 = tyi * TH - 1, tx0 = txi * TW - 1;
    const auto r = make_rsrc(x + bb * img_i, (unsigned long)img_i * 2);
    char* dst = smem + slot * BUF + wave * PPW * 1024;
#pragma unroll
    for (int i = 0; i < PPW; i++) {
      const int v = dm[i], gy = ty0 + (v >> 16), gx = tx0 + ((v >> 4) & 0xfff);
      const bool ok = live && v >= 0 && (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
      blds16(r, ok ? (unsigned)((gy * W + gx) * 256 + (v & 15) * 16) : 0x80000000u, dst + i * 1024);
    }
  };
  // halo pixel of (row r, tap a, column parity pxc, tap c) for lane lr: (r + 1 + py - a) * HC + lr + 1 + pxc - c
  const int lbase = (lr + HC * py) * ROWB + lg * 16;
  const int cb = ch0 + (odd ? 16 : 0) + 8 * (lg >> 1);
  float* aux = (float*)(smem + 3 * BUF);
  if (tid < 64) aux[tid] = bias ? bias[tid] : 0.f;
  __syncthreads();

  int tile = t_beg + wi, k = 0;
  issue(tile, 0);
  issue(tile + wpx, 1);
  for (; tile < t_end; tile += wpx, k++) {
    const int txi = tile % tiles_x, t2 = tile / tiles_x, tyi = t2 % tiles_y, bb = t2 / tiles_y;
    const auto ro = make_rsrc(out + bb * img_o, (unsigned long)img_o * 2);
    if (k == 0) wait_vmcnt<PPW>();
    else if (k == 1) wait_vmcnt<PPW + NS>();
    else wait_vmcnt<NS + PPW + NS>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(tile + 2 * wpx, (k + 2) % 3);
    const char* hb = smem + (k % 3) * BUF + lbase;
#pragma unroll
    for (int pxc = 0; pxc < 2; pxc++) {
      f32x4 acc[8][2];
#pragma unroll
      for (int nb = 0; nb < 2; nb++) {
        const f32x4 b0 = *(const f32x4*)(aux + ch0 + nb * 16 + 4 * lg);
#pragma unroll
        for (int r = 0; r < 8; r++) acc[r][nb] = b0;
      }
      auto rd = [&](int s, bf16x8 (&fa)[8]) {
        const int a = s >> 3, c = (s >> 2) & 1, kk = s & 3;
#pragma unroll
        for (int r = 0; r < 8; r++) fa[r] = *(const bf16x8*)(hb + ((r + 1 - a) * HC + 1 + pxc - c) * ROWB + kk * 64);
      };
      auto mm = [&](int s, const bf16x8 (&fa)[8]) {
#pragma unroll
        for (int r = 0; r < 8; r++)
#pragma unroll
          for (int nb = 0; nb < 2; nb++)
            acc[r][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[pxc][s][nb], fa[r], acc[r][nb], 0, 0, 0);
      };
      bf16x8 fa0[8], fa1[8];
      rd(0, fa0);
#pragma unroll
      for (int s = 0; s < 16; s += 2) {
        rd(s + 1, fa1);
        __builtin_amdgcn_sched_barrier(0);
        mm(s, fa0);
        __builtin_amdgcn_sched_barrier(0);
        if (s + 2 < 16) rd(s + 2, fa0);
        __builtin_amdgcn_sched_barrier(0);
        mm(s + 1, fa1);
        __builtin_amdgcn_sched_barrier(0);
      }
      const int gx = txi * TW + lr;
#pragma unroll
      for (int r = 0; r < 8; r++) {
        const int gy = tyi * TH + r;
        const unsigned po = (gy < H && gx < W) ? (unsigned)(((2 * gy + py) * 2 * W + 2 * gx + pxc) * 128 + cb * 2) : 0x80000000u;
        float o[8];
#pragma unroll
        for (int e = 0; e < 4; e++) {
          float v0 = acc[r][0][e], v1 = acc[r][1][e];
          if (RELU) { v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); }
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(v0), __float_as_uint(v1), false, false);
          o[e] = __uint_as_float(sw[0]);
          o[4 + e] = __uint_as_float(sw[1]);
        }
        bf16x8 ob;
#pragma unroll
        for (int e = 0; e < 8; e++) ob[e] = (bf16)o[e];
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, ob), ro, po, 0, 0);
      }
    }
  }
  wait_vmcnt<0>();
}

// ---------------------------------------------------------------- register-weight Conv2d(64, 128, 4, s2, p1)
// The data gradient of upsample_2x.0 (the ConvTranspose2d's input gradient is this strided conv of dy with the
// same conv-view weight [128][4][4][64]; 1024^2 x 64 -> 512^2 x 128 at bs 16, plus the column sums that are
// output_conv1's bias gradient).  Same design as the kernels above:
//   * tile = 4 x 16 output pixels; its (2*4+2) x (2*16+2) x 64 input halo lands by LDS-DMA in a 3-deep ring, pixel
//     rows padded to 144 B (9 slots, one dummy): the stride-2 tap reads are conflict-free without a swizzle;
//   * wave w = output channels 32 w .. +31 with their 16 taps x 64 weights in registers (256 VGPRs) as MFMA A
//     fragments, read straight from the conv-view pack; all waves share the tile's 4 x 16 pixels;
//   * epilogue: lane-pair channel trade, one 16-B store per lane per 16-pixel row, column sums in fp32 (LDS atomics,
//     one global add per channel and workgroup).
static bool convt_rw_ok(int dtype, int B, int H, int W);
namespace cs2 {
constexpr int TH = 4, TW = 16, HR = 2 * TH + 2, HC = 2 * TW + 2, PX = HR * HC, ROWB = 144;
constexpr int PIECES = ((PX * ROWB + 4095) / 4096) * 4, PPW = PIECES / 4, BUF = PIECES * 1024, LDS = 3 * BUF + 1024;
static_assert(LDS <= 160 * 1024, "conv s2 LDS budget");
}  // namespace cs2
__global__ void __launch_bounds__(256, 1) conv4s2_rw_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                             float* __restrict__ colsum, bf16* __restrict__ out, int H,
                                                             int W, int tiles_x, int tiles_y, int ntiles) {
  using namespace cs2;
  constexpr int NS = TH;                                            // stores per tile per wave
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int lr = lane & 15, lg = lane >> 4, odd = lg & 1;
  const int ch0 = 32 * wave;
  const int nwg = gridDim.x, xcd = blockIdx.x & 7, wpx = (nwg + 7 - xcd) >> 3, wi = blockIdx.x >> 3;
  const int t_beg = (int)((long)ntiles * xcd / 8), t_end = (int)((long)ntiles * (xcd + 1) / 8);
  const int Hi = 2 * H, Wi = 2 * W;
  const long img_i = (long)Hi * Wi * 64, img_o = (long)H * W * 128;
  // wr[tap][kk][nb]: lane (lr, lg) holds w[co = ch0 + 16 nb + lr][tap][ci = 32 kk + 8 lg .. +7]
  bf16x8 wr[16][2][2];
#pragma unroll
  for (int tap = 0; tap < 16; tap++)
#pragma unroll
    for (int kk = 0; kk < 2; kk++)
#pragma unroll
      for (int nb = 0; nb < 2; nb++)
        wr[tap][kk][nb] = *(const bf16x8*)(w + ((ch0 + nb * 16 + lr) * 16 + tap) * 64 + kk * 32 + lg * 8);
  int dm[PPW];
#pragma unroll
  for (int i = 0; i < PPW; i++) {
    const int b = (wave * PPW + i) * 1024 + lane * 16, px = b / ROWB, ch = (b % ROWB) >> 4;
    dm[i] = (px < PX && ch < 8) ? ((px / HC) << 16) | ((px % HC) << 4) | ch : -1;
  }
  auto issue = [&](int tile, int slot) {
    const bool live = tile < t_end;
    const int tc = live ? tile : t_beg;
    const int txi = tc % tiles_x, t2 = tc / tiles_x, tyi = t2 % tiles_y, bb = t2 / tiles_y;
    const int iy0 = 2 * tyi * TH - 1, ix0 = 2 * txi * TW - 1;
    const auto r = make_rsrc(x + bb * img_i, (unsigned long)img_i * 2);
    char* dst = smem + slot * BUF + wave * PPW * 1024;
#pragma unroll
    for (int i = 0; i < PPW; i++) {
      const int v = dm[i], gy = iy0 + (v >> 16), gx = ix0 + ((v >> 4) & 0xfff);
      const bool ok = live && v >= 0 && (unsigned)gy < (unsigned)Hi && (unsigned)gx < (unsigned)Wi;
      blds16(r, ok ? (unsigned)((gy * Wi + gx) * 128 + (v & 15) * 16) : 0x80000000u, dst + i * 1024);
    }
  };
  // halo pixel of output (row r, column lr) and tap (ky, kx): (2 r + ky) * HC + 2 lr + kx
  const int lbase = 2 * lr * ROWB + lg * 16;
  const int cb = ch0 + (odd ? 16 : 0) + 8 * (lg >> 1);
  float* aux = (float*)(smem + 3 * BUF);
  if (tid < 128) aux[tid] = 0.f;
  __syncthreads();
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

  int tile = t_beg + wi, k = 0;
  issue(tile, 0);
  issue(tile + wpx, 1);
  for (; tile < t_end; tile += wpx, k++) {
    const int txi = tile % tiles_x, t2 = tile / tiles_x, tyi = t2 % tiles_y, bb = t2 / tiles_y;
    const auto ro = make_rsrc(out + bb * img_o, (unsigned long)img_o * 2);
    if (k == 0) wait_vmcnt<PPW>();
    else if (k == 1) wait_vmcnt<PPW + NS>();
    else wait_vmcnt<NS + PPW + NS>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(tile + 2 * wpx, (k + 2) % 3);
    const char* hb = smem + (k % 3) * BUF + lbase;
    f32x4 acc[TH][2];
#pragma unroll
    for (int r = 0; r < TH; r++) { acc[r][0] = f32x4{0.f, 0.f, 0.f, 0.f}; acc[r][1] = f32x4{0.f, 0.f, 0.f, 0.f}; }
    auto rd = [&](int s, bf16x8 (&fa)[TH]) {
      const int tap = s >> 1, kk = s & 1, ky = tap >> 2, kx = tap & 3;
#pragma unroll
      for (int r = 0; r < TH; r++) fa[r] = *(const bf16x8*)(hb + ((2 * r + ky) * HC + kx) * ROWB + kk * 64);
    };
    auto mm = [&](int s, const bf16x8 (&fa)[TH]) {
#pragma unroll
      for (int r = 0; r < TH; r++)
#pragma unroll
        for (int nb = 0; nb < 2; nb++)
          acc[r][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[s >> 1][s & 1][nb], fa[r], acc[r][nb], 0, 0, 0);
    };
    bf16x8 fa0[TH], fa1[TH];
    rd(0, fa0);
#pragma unroll
    for (int s = 0; s < 32; s += 2) {
      rd(s + 1, fa1);
      __builtin_amdgcn_sched_barrier(0);
      mm(s, fa0);
      __builtin_amdgcn_sched_barrier(0);
      if (s + 2 < 32) rd(s + 2, fa0);
      __builtin_amdgcn_sched_barrier(0);
      mm(s + 1, fa1);
      __builtin_amdgcn_sched_barrier(0);
    }
    const int gx = txi * TW + lr;
#pragma unroll
    for (int r = 0; r < TH; r++) {
      const int gy = tyi * TH + r;
      const bool ok = gy < H && gx < W;
      const unsigned po = ok ? (unsigned)(((gy * W + gx) * 128 + cb) * 2) : 0x80000000u;
      float o[8];
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[r][0][e]), __float_as_uint(acc[r][1][e]), false, false);
        o[e] = __uint_as_float(sw[0]);
        o[4 + e] = __uint_as_float(sw[1]);
      }
      if (ok) {
#pragma unroll
        for (int e = 0; e < 8; e++) cs[e] += o[e];
      }
      bf16x8 ob;
#pragma unroll
      for (int e = 0; e < 8; e++) ob[e] = (bf16)o[e];
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, ob), ro, po, 0, 0);
    }
  }
  if (colsum) {
#pragma unroll
    for (int e = 0; e < 8; e++) {
      float c = cs[e];
      c += __shfl_xor(c, 1); c += __shfl_xor(c, 2); c += __shfl_xor(c, 4); c += __shfl_xor(c, 8);
      if (lr == 0) atomicAdd(aux + cb + e, c);
    }
    __syncthreads();
    if (tid < 128) atomicAdd(colsum + tid, aux[tid]);
  }
  wait_vmcnt<0>();
}
static int launch_conv4s2_rw(const bf16* x, const bf16* w, float* colsum, bf16* out, int B, int H, int W, hipStream_t st) {
  auto kfn = conv4s2_rw_kernel;
  static const bool attr = ((void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, cs2::LDS), true);   // once per process (thread-safe static init)
  (void)attr;
  const int tx = cdiv(W, cs2::TW), ty = cdiv(H, cs2::TH);
  const long tiles = (long)B * tx * ty;
  if (tiles >= (1L << 31)) { s3od_set_error("conv s2 rw: too many tiles"); return 22; }
    const int nwg = (int)std::min<long>(std::max<long>(tiles, 8), (long)s3od_cu_count());
  hipLaunchKernelGGL(kfn, dim3(nwg), dim3(256), cs2::LDS, st, x, w, colsum, out, H, W, tx, ty, (int)tiles);
  return s3od_check_launch("conv4s2_rw");
}

// S3OD_CONVT_RW=0 disables the path (under S3OD_AB=1: per call)
static bool convt_rw_ok(int dtype, int B, int H, int W) {
  return dtype == S3OD_BF16 && !S3OD_OFF("S3OD_CONVT_RW") && B > 0 && (long)4 * H * W * 128 < (1L << 31);
}
static int launch_convt_rw(const bf16* x, const bf16* wt, const float* bias, bool relu, bf16* out, int B, int H, int W,
                           hipStream_t st) {
  auto kfn = relu ? convT4s2_rw_kernel<true> : convT4s2_rw_kernel<false>;
  static const bool attr0 = ((void)hipFuncSetAttribute((const void*)convT4s2_rw_kernel<false>,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, ct::LDS), true);
  static const bool attr1 = ((void)hipFuncSetAttribute((const void*)convT4s2_rw_kernel<true>,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, ct::LDS), true);
  (void)attr0; (void)attr1;
  const int tx = cdiv(W, ct::TW), ty = cdiv(H, ct::TH);
  const long tiles = (long)B * tx * ty;
  if (tiles >= (1L << 31)) { s3od_set_error("convT rw: too many tiles"); return 22; }
    const int nwg = (int)std::min<long>(std::max<long>(tiles, 8), (long)s3od_cu_count());   // >= 8: every XCD owns a tile range
  hipLaunchKernelGGL(kfn, dim3(nwg), dim3(256), ct::LDS, st, x, wt, bias, out, H, W, tx, ty, (int)tiles);
  return s3od_check_launch("convT4s2_rw");
}

// ---------------------------------------------------------------- halo-tile 3x3 weight gradient
// dW[co][tap][ci] = sum_px dy[px][co] * x[px + tap][ci] for a 3x3 / stride 1 / pad 1 conv with Cin = 64
// and Cout = 64 / 96 (the full-resolution decoder convs).  The implicit-GEMM wgrad tiles N = 9*64 into
// 128-column blocks, so every 64-pixel K tile is fetched once per N block: ~7x the unique bytes go
// through L2 (measured: 57 % of wave time parked on vmcnt).  Here a persistent workgroup owns ALL
// 9 x 64 x Cout outputs in registers and sweeps 8 x 32-pixel tiles: dy (256 px x Cout) and the x halo
// (10 x 34 px x 64) are staged once per tile (register-prefetched one tile ahead) and every MFMA
// operand is read with ds_read_b64_tr_b16 (K = pixels, permuted identically on both operands).
// Waves: 4 (one per SIMD, up to 512 registers: the whole 9 x 64 x Cout fp32 block lives in registers),
// 9 of the 36 (tap, ci-block) pairs each, all co blocks per wave so each B fragment feeds NCO MFMAs.  The partial sums are flushed once per
// workgroup with fp32 atomics into the [co][tap][ci] workspace (wgrad_permute_add_kernel follows).
template <int CO> struct WgShape {
  static constexpr int DYB = 256 * CO * 2;                 // dy tile image [px][CO]
  static constexpr int HXB = HT_PX * 128;                  // x halo image [px][64]
  static constexpr int LDS = DYB + HXB;
  static constexpr int DCH = 256 * CO / 8, HCH = HT_PX * 8;           // 16-B chunks to stage
  static constexpr int NT = 256;                                       // 4 waves, one per SIMD
  static constexpr int PT = (DCH + HCH + NT - 1) / NT;                 // 16-B chunks per thread
  static_assert(LDS <= 160 * 1024, "halo wgrad LDS budget");
};
template <int CO> DEV int dy_at(int row, int byte) {       // conflict-free for the transposed reads
  if constexpr (CO == 64) return row * 128 + ((((byte >> 4) ^ (row & 7)) << 4) | (byte & 15));
  else return row * 192 + ((((byte >> 4) ^ ((row >> 1) & 3)) << 4) | (byte & 15));
}
DEV int hx_at(int row, int byte) { return row * 128 + ((((byte >> 4) ^ (row & 7)) << 4) | (byte & 15)); }
// 16 columns x 32 rows fragment, transposed (rows = K, permuted: 4g + q and 16 + 4g + q)
template <class AT> DEV bf16x8 trf(const char* img, int r0, int col0, int lane, AT at) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int byte = (col0 + 4 * p) * 2;
  typedef __attribute__((address_space(3))) s16x4 lds4;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(img + at(r0 + 4 * g + q, byte)));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(img + at(r0 + 16 + 4 * g + q, byte)));
  bf16x4 a = __builtin_bit_cast(bf16x4, lo), b = __builtin_bit_cast(bf16x4, hi);
  return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

template <int CO, bool RELU>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
conv3x3_wgrad_halo_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x, float* __restrict__ ws, int H, int W,
                          int tiles_x, int tiles_y, int ntiles, int CinT, int CoT, int nci, int wpc) {
  typedef WgShape<CO> S;
  constexpr int NCO = CO / 16, CPD = CO / 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* dyi = smem;
  char* hxi = smem + S::DYB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // channel block of this workgroup: (co0 .. co0+CO) x (ci0 .. ci0+64) of a CoT x CinT conv; the wpc
  // workgroups of one block split the tiles into contiguous ranges (neighbouring tiles share halo rows)
  const int combo = blockIdx.x / wpc, wi = blockIdx.x - combo * wpc;
  const int co0 = (combo / nci) * CO, ci0 = (combo % nci) * 64;
  const int t_beg = (int)((long)ntiles * wi / wpc), t_end = (int)((long)ntiles * (wi + 1) / wpc);
  constexpr int NP = 9;                                  // (tap, ci-block) pairs of this wave: 9*wave ..
  const int pair0 = NP * wave;
  f32x4 acc[NP][NCO];
#pragma unroll
  for (int i = 0; i < NP; i++)
#pragma unroll
    for (int j = 0; j < NCO; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 pf[S::PT];
  auto prefetch = [&](int tile) {
    const int txi = tile % tiles_x, t2 = tile / tiles_x, tyi = t2 % tiles_y, b = t2 / tiles_y;
    const int ty0 = tyi * HT_TH, tx0 = txi * HT_TW;
#pragma unroll
    for (int i = 0; i < S::PT; i++) {
      const int c = tid + S::NT * i;
      pf[i] = make_uint4(0, 0, 0, 0);
      if (c < S::DCH) {                                   // dy tile: px = ty*32 + tx
        const int px = c / CPD, ch = c - px * CPD, gy = ty0 + px / HT_TW, gx = tx0 + px % HT_TW;
        if (gy < H && gx < W) pf[i] = *(const uint4*)(dy + (((long)b * H + gy) * W + gx) * CoT + co0 + ch * 8);
      } else if (c < S::DCH + S::HCH) {                   // x halo
        const int c2 = c - S::DCH, px = c2 >> 3, ch = c2 & 7, hy = px / HT_HC, hx = px - hy * HT_HC;
        const int gy = ty0 - 1 + hy, gx = tx0 - 1 + hx;
        if (gy >= 0 && gy < H && gx >= 0 && gx < W) {
          pf[i] = *(const uint4*)(x + (((long)b * H + gy) * W + gx) * CinT + ci0 + ch * 8);
          if (RELU) pf[i] = relu16<bf16>(pf[i]);
        }
      }
    }
  };
  int tile = t_beg;
  if (tile < t_end) prefetch(tile);
  for (; tile < t_end; tile++) {
#pragma unroll
    for (int i = 0; i < S::PT; i++) {
      const int c = tid + S::NT * i;
      if (c < S::DCH) { const int px = c / CPD, ch = c - px * CPD; *(uint4*)(dyi + dy_at<CO>(px, ch * 16)) = pf[i]; }
      else if (c < S::DCH + S::HCH) { const int c2 = c - S::DCH; *(uint4*)(hxi + hx_at(c2 >> 3, (c2 & 7) * 16)) = pf[i]; }
    }
    __syncthreads();
    if (tile + 1 < t_end) prefetch(tile + 1);
    for (int ty = 0; ty < HT_TH; ty++) {                  // K step = one output row of 32 pixels
      bf16x8 fa[NCO];
#pragma unroll
      for (int cb = 0; cb < NCO; cb++) fa[cb] = trf(dyi, ty * HT_TW, cb * 16, lane, dy_at<CO>);
#pragma unroll
      for (int j = 0; j < NP; j++) {
        const int pr = pair0 + j, tap = pr >> 2, cib = pr & 3, tdy = tap / 3, tdx = tap - tdy * 3;
        const bf16x8 fb = trf(hxi, (ty + tdy) * HT_HC + tdx, cib * 16, lane, hx_at);
#pragma unroll
        for (int cb = 0; cb < NCO; cb++) acc[j][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[cb], fb, acc[j][cb], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  // flush: lane holds D[co = cb*16 + 4g + r][ci = cib*16 + li] of pair j -> ws[co][tap*64 + ci]
  const int g = lane >> 4, li = lane & 15;
#pragma unroll
  for (int j = 0; j < NP; j++) {
    const int pr = pair0 + j, tap = pr >> 2, cib = pr & 3;
#pragma unroll
    for (int cb = 0; cb < NCO; cb++)
#pragma unroll
      for (int r = 0; r < 4; r++)
        atomicAdd(ws + (long)(co0 + cb * 16 + 4 * g + r) * (9 * CinT) + tap * CinT + ci0 + cib * 16 + li, acc[j][cb][r]);
  }
}

template <int CO, bool RELU>
static int launch_wgrad_halo(const bf16* dy, const bf16* x, float* ws, int B, int H, int W, int CinT, int CoT, hipStream_t st) {
  typedef WgShape<CO> S;
  auto kfn = conv3x3_wgrad_halo_kernel<CO, RELU>;
  static const bool attr = ((void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, S::LDS), true);   // once per process (thread-safe static init)
  (void)attr;
  const int tx = cdiv(W, HT_TW), ty = cdiv(H, HT_TH);
  const long tiles = (long)B * tx * ty;
    // one persistent workgroup per CU (registers) over all channel blocks: each block gets ~ncu/blocks of them
  const int nci = CinT / 64, nblk = (CoT / CO) * nci;
  const int wpc = (int)std::max<long>(1, std::min<long>(tiles, std::max(1, s3od_cu_count() / nblk)));
  hipLaunchKernelGGL(kfn, dim3(nblk * wpc), dim3(S::NT), S::LDS, st, dy, x, ws, H, W, tx, ty, (int)tiles, CinT, CoT, nci, wpc);
  return s3od_check_launch("conv3x3_wgrad_halo");
}

// Weight gradient of the 4x4 / stride-2 / pad-1 conv view of upsample_2x.0 (ConvTranspose2d(128, 64, 4, 2, 1)):
// dW[co][ky][kx][ci] = sum_p dy[p][co] * x[2p - 1 + (ky, kx)][ci], dy on the OH x OW grid (128 channels), x on the
// 2OH x 2OW grid (64).  The same LDS-DMA / register-accumulator scheme as the 3x3 kernel above with 16 taps:
//   * tile = 2 x 32 dy pixels; its x halo (2*2+2) x (2*32+2) is stored column-DE-INTERLEAVED (even / odd halo
//     columns in two 33-pixel sub-rows), so a tap's 32 stride-2 pixels are 32 consecutive image rows and the
//     transposed reads keep the swizzle of the 3x3 kernel;
//   * workgroup = a 64-output-channel block; wave w = taps 4w .. 4w+3 x 4 ci blocks (256 accumulator VGPRs).
namespace wg4 {
constexpr int TH = 2, TW = 32, HR = 2 * TH + 2, HS = TW + 1, HPX = HR * 2 * HS;   // halo rows, sub-row length
constexpr int AB = TH * TW * 128, HB = HPX * 128, PIECES = ((AB + HB + 4095) / 4096) * 4, PPW = PIECES / 4;
constexpr int BUF = PIECES * 1024, LDS = 2 * BUF;
static_assert(AB % 1024 == 0 && LDS <= 160 * 1024, "wgrad 4s2 layout");
}  // namespace wg4
__global__ void __launch_bounds__(256, 1)
conv4s2_wgrad_dma_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x, float* __restrict__ ws, int OH, int OW,
                         int tiles_x, int tiles_y, int ntiles, int CinT, int CoT, int nci, int wpc, int ymaj) {
  using namespace wg4;
  constexpr int NCO = 4, NP = 16;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int combo = blockIdx.x / wpc, wi = blockIdx.x - combo * wpc;
  const int t_beg = (int)((long)ntiles * wi / wpc), t_end = (int)((long)ntiles * (wi + 1) / wpc);
  const int co0 = (combo / nci) * 64, ci0 = (combo % nci) * 64;
  const int pair0 = NP * wave, IH = 2 * OH, IW = 2 * OW;
  f32x4 acc[NP][NCO];
#pragma unroll
  for (int i = 0; i < NP; i++)
#pragma unroll
    for (int j = 0; j < NCO; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // dm = (row << 16) | (column << 4) | logical chunk: dy pieces -> tile row / column; halo -> halo row / halo column
  int dm[PPW];
#pragma unroll
  for (int i = 0; i < PPW; i++) {
    const int p = wave * PPW + i, b = p * 1024 + lane * 16;
    if (p < AB / 1024) {
      const int row = b >> 7, c = ((b >> 4) & 7) ^ (row & 7);
      dm[i] = ((row / TW) << 16) | ((row % TW) << 4) | c;
    } else {
      const int hb = b - AB, row = hb >> 7, c = ((hb >> 4) & 7) ^ (row & 7);
      const int hr = row / (2 * HS), rem = row - hr * 2 * HS, sub = rem / HS, idx = rem - sub * HS;
      dm[i] = row < HPX ? (hr << 16) | ((2 * idx + sub) << 4) | c : -1;
    }
  }
  auto issue = [&](int tile, int slot) {
    // ymaj: consecutive tiles walk down a column (the halo's top 2 of 6 rows were the previous tile's: L2)
    int txi, tyi, b;
    if (ymaj) { tyi = tile % tiles_y; const int t2 = tile / tiles_y; txi = t2 % tiles_x; b = t2 / tiles_x; }
    else { txi = tile % tiles_x; const int t2 = tile / tiles_x; tyi = t2 % tiles_y; b = t2 / tiles_y; }
    const int oy0 = tyi * TH, ox0 = txi * TW;
    const long img_d = (long)OH * OW * CoT, img_x = (long)IH * IW * CinT;
    const auto rd = make_rsrc(dy + b * img_d, (unsigned long)img_d * 2);
    const auto rx = make_rsrc(x + b * img_x, (unsigned long)img_x * 2);
    char* dst = smem + slot * BUF + wave * PPW * 1024;
#pragma unroll
    for (int i = 0; i < PPW; i++) {
      const int p = wave * PPW + i, v = dm[i];
      if (p < AB / 1024) {                               // wave-uniform
        const int gy = oy0 + (v >> 16), gx = ox0 + ((v >> 4) & 0xfff);
        const bool ok = gy < OH && gx < OW;
        blds16(rd, ok ? (unsigned)(((gy * OW + gx) * CoT + co0) * 2 + (v & 15) * 16) : 0x80000000u, dst + i * 1024);
      } else {
        const int gy = 2 * oy0 - 1 + (v >> 16), gx = 2 * ox0 - 1 + ((v >> 4) & 0xfff);
        const bool ok = v >= 0 && (unsigned)gy < (unsigned)IH && (unsigned)gx < (unsigned)IW;
        blds16(rx, ok ? (unsigned)(((gy * IW + gx) * CinT + ci0) * 2 + (v & 15) * 16) : 0x80000000u, dst + i * 1024);
      }
    }
  };
  int tile = t_beg, k = 0;
  if (tile < t_end) issue(tile, 0);
  for (; tile < t_end; tile++, k++) {
    wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (tile + 1 < t_end) issue(tile + 1, (k + 1) & 1);
    const char* dyi = smem + (k & 1) * BUF;
    const char* hxi = dyi + AB;
    for (int ty = 0; ty < TH; ty++) {                     // K step = one dy row of 32 pixels
      bf16x8 fa[NCO];
#pragma unroll
      for (int cb = 0; cb < NCO; cb++) fa[cb] = trf(dyi, ty * TW, cb * 16, lane, dy_at<64>);
#pragma unroll
      for (int j = 0; j < NP; j++) {
        const int pr = pair0 + j, tap = pr >> 2, cib = pr & 3, ky = tap >> 2, kx = tap & 3;
        // halo column 2 k + kx of halo row 2 ty + ky = sub-row (kx & 1), entry k + (kx >> 1)
        const bf16x8 fb = trf(hxi, ((2 * ty + ky) * 2 + (kx & 1)) * HS + (kx >> 1), cib * 16, lane, hx_at);
#pragma unroll
        for (int cb = 0; cb < NCO; cb++) acc[j][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[cb], fb, acc[j][cb], 0, 0, 0);
      }
    }
  }
  const int g = lane >> 4, li = lane & 15;
#pragma unroll
  for (int j = 0; j < NP; j++) {
    const int pr = pair0 + j, tap = pr >> 2, cib = pr & 3;
#pragma unroll
    for (int cb = 0; cb < NCO; cb++)
#pragma unroll
      for (int r = 0; r < 4; r++)
        atomicAdd(ws + (long)(co0 + cb * 16 + 4 * g + r) * (16 * CinT) + tap * CinT + ci0 + cib * 16 + li, acc[j][cb][r]);
  }
}
static int launch_wgrad4s2(const bf16* dy, const bf16* x, float* ws, int B, int OH, int OW, int CinT, int CoT, hipStream_t st) {
  auto kfn = conv4s2_wgrad_dma_kernel;
  static const bool attr = ((void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, wg4::LDS), true);   // once per process (thread-safe static init)
  (void)attr;
  const int tx = cdiv(OW, wg4::TW), ty = cdiv(OH, wg4::TH);
  const long tiles = (long)B * tx * ty;
  if (tiles >= (1L << 31)) { s3od_set_error("wgrad 4s2: too many tiles"); return 22; }
    const int nci = CinT / 64, nblk = (CoT / 64) * nci;
  const int wpc = (int)std::max<long>(1, std::min<long>(tiles, std::max(1, s3od_cu_count() / nblk)));
  hipLaunchKernelGGL(kfn, dim3(nblk * wpc), dim3(256), wg4::LDS, st, dy, x, ws, OH, OW, tx, ty, (int)tiles, CinT, CoT, nci, wpc,
                     S3OD_KNOB("S3OD_WGD_YMAJ", 1));
  return s3od_check_launch("conv4s2_wgrad_dma");
}

template <int BM, int BN> struct Tile {};

// split-K factor of a wgrad GEMM from a time model: ceil(tiles*sp / slots) rounds of ceil(KT/sp)
// K tiles each, plus the split-K fp32 atomics at the chip-wide atomic rate (~1.3 TB/s, guide
// "Global float atomics").  slots = resident workgroups (256 CUs x WGs per CU by LDS).
template <typename T, int BM, int BN, int NST> static int wgrad_split(int tiles, int KT) {
  typedef GemmShape<T, BM, BN, NST> S;
  const int per_cu = (160 * 1024) / S::LDS > 0 ? (160 * 1024) / S::LDS : 1;
  const long slots = 256L * per_cu;
  const double ck = 2.0 * BM * BN * S::BK / (3.9e6 / per_cu);      // us per K tile per WG
  const double atom = (double)BM * BN * 4 / 1.3e6;                 // us of chip atomics per WG
  int best = 1; double bt = 1e30;
  for (int sp = 1; sp <= (KT >= 8 ? KT / 4 : 1); sp++) {
    long wgs = (long)tiles * sp;
    double t = (double)((wgs + slots - 1) / slots) * ((KT + sp - 1) / sp) * ck + wgs * atom;
    if (t < bt * 0.999) { bt = t; best = sp; }
  }
  return best;
}

// dW (+)= the sum of the split-K slabs ws[sp][M][N] (EpiWgradPart), scattered to the PyTorch layout
// dW[(m*Cx + cin)*taps + tap] for n = tap*Cx + cin (Linear: taps = 1, Cx = N).  One thread per 4 consecutive n.
__global__ void wgrad_reduce_kernel(const float* __restrict__ ws, int sp, int M, int N, float* __restrict__ dw, int Cx, int taps) {
  const long i4 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const long MN = (long)M * N;
  if (i4 >= MN) return;
  // the slabs' loads go out 8 at a time before any add (a load-add chain waits out one memory latency per slab:
  // 81 us for 7 slabs of 3072 x 768 in the step, 4x the bytes' HBM time); summation order z = 0, 1, .. unchanged
  float4 s = *(const float4*)(ws + i4);
  for (int z0 = 1; z0 < sp; z0 += 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; u++)
      if (z0 + u < sp) v[u] = *(const float4*)(ws + (long)(z0 + u) * MN + i4);
#pragma unroll
    for (int u = 0; u < 8; u++)
      if (z0 + u < sp) { s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w; }
  }
  const int m = (int)(i4 / N), n = (int)(i4 - (long)m * N);
  if (taps == 1) {
    float4* d = (float4*)(dw + i4);
    const float4 o = *d;
    *d = make_float4(o.x + s.x, o.y + s.y, o.z + s.z, o.w + s.w);
    return;
  }
  const float sv[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const int tap = (n + e) / Cx, cin = (n + e) - tap * Cx;
    dw[((long)m * Cx + cin) * taps + tap] += sv[e];
  }
}

// S3OD_WGRAD_SLAB=0 (under S3OD_AB=1: per call): the fp32-atomic split-K epilogue instead of the slabs (A/B)
static bool slab_ok() { return !S3OD_OFF("S3OD_WGRAD_SLAB"); }

// M-tail launches (split_tail: the <= 255 rows past the last full 256-row panel).  On 128x128 tiles a tail has only
// N/128 workgroups (6 for N 768), each a full-K main loop on an otherwise idle chip (13-45 us at K 768-3072).  bf16:
// a skinny full-K kernel instead -- one wave per 16 x 16 output block (240 waves for 80 x 768), operands straight from
// global memory (80 rows of A and the B panel stay in L2), and the SAME v_mfma_f32_16x16x32_bf16 chain over K, in the
// same order and fragment layout as the ping-pong / 128x128 kernels (lane (g, l) holds row l, k = 32 kk + 8 g .. +7,
// zero past K), so every tail row is bit-identical to what a full panel computes: outputs do not depend on where a
// row falls, i.e. on the batch size.  (A split-K tail was as fast but broke that: bf16 bs-8 vs bs-1 rel-L2 1e-2.)
// Block = 4 waves = 16 rows x 64 columns; the fp32 tile is staged in LDS and the op's own epilogue functor runs on it.
template <bool BKC, int U, class EPI>
__global__ void __launch_bounds__(256) tail_gemm_kernel(const bf16* __restrict__ A, long lda, const bf16* __restrict__ Bp,
                                                        long ldb, int M, int N, int K, EPI epi) {
  constexpr int LDT = 64 + 4;
  __shared__ __attribute__((aligned(16))) float ct[2048];     // 16 x 68 C tile; the column-sum reduction reads 256 x 8
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, l = lane & 15;
  const int m0 = blockIdx.y * 16, nb0 = blockIdx.x * 64, am = m0 + l, bn = nb0 + wave * 16 + l;
  const bool aok = am < M, bok = bn < N;
  // rows past M / columns past N read row 0 / column 0 instead (clamped addresses, no branches in the loop): an
  // output element only sees its own A row and B column, and those rows / columns are never stored
  const bf16* ar = A + (long)(aok ? am : 0) * lda;
  const long bo = bok ? bn : 0;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  // N-contiguous B (dgrad: w [K][N]): a fragment wants 8 k of one column, so the wave stages each k-step's 32 x 16
  // block through LDS -- lane j fetches 16 B of row k = j / 2 (columns 8 (j & 1) ..), the fragment is read back as 8
  // bf16 of column l (row stride 24 elements = 48 B: 16-B aligned stores; no bank conflicts on the reads)
  constexpr int RS = 24;
  static_assert(sizeof(float) * 2048 + (BKC ? 2 : 2 * 4 * U * 32 * RS) <= 160 * 1024, "tail_gemm: LDS budget (gfx950: 160 KiB)");
  __shared__ bf16 bst[BKC ? 1 : 4 * U * 32 * RS];
  bf16* wst = bst + (BKC ? 0 : wave * U * 32 * RS);
  const int bj = lane >> 1, bc = 8 * (lane & 1);
  const long bcol = (nb0 + wave * 16 + bc < N) ? nb0 + wave * 16 + bc : 0;   // whole 16-B chunks: N % 8 == 0
  auto load = [&](int k, bf16x8& fa, bf16x8& fb) {            // K % 8 == 0: a lane's 8 k are all in range or all out
    fa = *(const bf16x8*)(ar + k);
    if constexpr (BKC) fb = *(const bf16x8*)(Bp + bo * ldb + k);
  };
  // a lone wave's chain is load-latency bound: the loads of U k-steps are issued together, then their U MFMAs run
  // in k order ((B, A) operand order, as Mma<bf16> in the kernels)
  const int KF = K / 32;
  int kk = 0;
  for (; kk + U <= KF; kk += U) {
    bf16x8 fa[U], fb[U];
    uint4 braw[BKC ? 1 : U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      load((kk + u) * 32 + 8 * g, fa[u], fb[u]);
      if constexpr (!BKC) braw[u] = *(const uint4*)(Bp + (long)((kk + u) * 32 + bj) * ldb + bcol);
    }
    if constexpr (!BKC) {
      // the wave's LDS block is written and read back by different lanes of the same wave: order the previous
      // batch's reads before these stores and these stores before the reads (wave-scope fence + wave barrier: the
      // C++ model does not order cross-lane LDS traffic within a wave by itself)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int u = 0; u < U; u++) *(uint4*)(wst + (u * 32 + bj) * RS + bc) = braw[u];
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int u = 0; u < U; u++)
#pragma unroll
        for (int e = 0; e < 8; e++) fb[u][e] = wst[(u * 32 + 8 * g + e) * RS + l];
    }
    __builtin_amdgcn_sched_barrier(0);                        // all U loads in flight before the first MFMA waits
#pragma unroll
    for (int u = 0; u < U; u++) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[u], fa[u], acc, 0, 0, 0);
  }
  for (; kk < KF; kk++) {
    bf16x8 fa, fb;
    load(kk * 32 + 8 * g, fa, fb);
    if constexpr (!BKC) {
#pragma unroll
      for (int e = 0; e < 8; e++) fb[e] = Bp[(long)(kk * 32 + 8 * g + e) * ldb + bo];
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb, fa, acc, 0, 0, 0);
  }
  if (K % 32) {                                               // K tail: lanes past K contribute zeros
    bf16x8 fa, fb;
    const int k = KF * 32 + 8 * g;
    if (k < K) {
      load(k, fa, fb);
      if constexpr (!BKC) {
#pragma unroll
        for (int e = 0; e < 8; e++) fb[e] = Bp[(long)(k + e) * ldb + bo];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; e++) { fa[e] = (bf16)0.f; fb[e] = (bf16)0.f; }
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb, fa, acc, 0, 0, 0);
  }
  *(f32x4*)(ct + l * LDT + wave * 16 + 4 * g) = acc;          // lane (g, l) owns C[m0 + l][n + 4g .. 4g+3]
  __syncthreads();
  epi.prepare(0);
  epi(ct, LDT, m0, nb0, tid, 16, 64, 256);
}
template <class LA, class LB, class EPI>
static int launch_tail_gemm(const LA& la, const LB& lb, EPI e, int M, int N, hipStream_t st) {
  // U = k-steps whose loads are in flight together: the largest that divides K / 32 (a remainder runs one step at a
  // time, each paying the full latency).  K-contiguous B: up to 24 (U = 32: 283 VGPRs, spills); N-contiguous B (LDS
  // staging, 4 U KB per wave): up to 16.
  const int KF = la.K / 32;
  auto go = [&](auto u) {
    hipLaunchKernelGGL((tail_gemm_kernel<LB::KCL, decltype(u)::value, EPI>), dim3(cdiv(N, 64), cdiv(M, 16)), dim3(256), 0, st,
                       (const bf16*)la.p, la.ld, (const bf16*)lb.p, lb.ld, M, N, la.K, e);
    return s3od_check_launch("igemm tail");
  };
  if constexpr (LB::KCL) {
    if (KF % 24 == 0) return go(std::integral_constant<int, 24>{});
    if (KF % 16 == 0) return go(std::integral_constant<int, 16>{});
  } else {
    if (KF % 16 == 0) return go(std::integral_constant<int, 16>{});
    if (KF % 12 == 0) return go(std::integral_constant<int, 12>{});
  }
  return go(std::integral_constant<int, 8>{});
}
// the launch of one with_cfg config: the skinny tail kernel for a bf16 M-tail launch (tl_cfg == 1, A K-contiguous, no
// ReLU-on-load); f32 tails stay on the 128x128 kernel (same summation order too).  S3OD_TAIL_SKINNY=0 (under S3OD_AB=1: per call):
// the 128x128 tail launch in bf16 as well.
template <typename T, class C, class LA, class LB, class EPI>
static int launch_op(LA la, LB lb, EPI e, int M, int N, int KTILES, hipStream_t st) {
  if constexpr (!C::PP && sizeof(T) == 2 && LA::KCL)
    if (tl_cfg == 1 && M < 256 && !la.relu && !lb.relu && !S3OD_OFF("S3OD_TAIL_SKINNY"))
      return launch_tail_gemm(la, lb, e, M, N, st);
  return launch_igemm<T, C::BM, C::BN, LA, LB, EPI, C::NST, C::WM>(la, lb, e, M, N, KTILES, 1, 1, st);
}

// dw[(co*Cin + ci)*taps + tap] += ws[(co*taps + tap)*Cin + ci]   (one thread per dw element)
// ws enters all zero (split-K atomics land in it) and leaves all zero: each element is cleared as it is read,
// so a persistent workspace needs no memset per call
__global__ void wgrad_permute_add_kernel(float* __restrict__ ws, float* __restrict__ dw, int Cout, int Cin, int taps) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)Cout * Cin * taps) return;
  int tap = i % taps; long r = i / taps;
  int ci = r % Cin; int co = r / Cin;
  const long src = ((long)co * taps + tap) * Cin + ci;
  dw[i] += ws[src];
  ws[src] = 0.f;
}

extern "C" {

#ifdef S3OD_TIMELINE
// dev timeline build only (tools/pp_timeline.py): where the ping-pong kernels of this file record their blocks
int s3od_dbg_timeline(unsigned long long* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(s3od_tl), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}
#endif

// ---------------------------------------------------------------------------------- linear
// pre = sum_k x[m,k] w[n,k] + bias[n];  out[rm(m), n] = act(pre*scale[n] + shift[n]) (+res1 +res2)
// x: [M,K] (ld ldx) dtype T, w: [N,K] T, res: T or f32 (res_f32), out T or f32 (out_f32).
// row_mode 0: dense; 1: token rows (m = b*P + p -> b*(P+prefix) + prefix + p)
int s3od_linear_fwd(int dtype, int M, int N, int K, const void* x, long ldx, const void* w,
                    const float* bias, const float* scale, const float* shift, int act,
                    const void* res1, long ldr1, const void* res2, long ldr2, int res_f32,
                    void* out, long ldo, int out_f32, void* pre, long ldp,
                    int row_mode, int P, int prefix, void* stream) {
  S3OD_REQUIRE(K % 8 == 0 && N % 8 == 0, "linear_fwd: K and N must be multiples of 8 (K=%d N=%d)", K, N);
  if (row_mode == 0 && split_tail(M)) {
    const int M1 = M & ~255, M2 = M - M1;
    int rc = s3od_linear_fwd(dtype, M1, N, K, x, ldx, w, bias, scale, shift, act, res1, ldr1, res2, ldr2, res_f32,
                             out, ldo, out_f32, pre, ldp, row_mode, P, prefix, stream);
    if (rc) return rc;
    const long es = dtype == S3OD_BF16 ? 2 : 4, eo = out_f32 ? 4 : es, er = res_f32 ? 4 : es;
    TailCfg tail;
    return s3od_linear_fwd(dtype, M2, N, K, (const char*)x + M1 * ldx * es, ldx, w, bias, scale, shift, act,
                           res1 ? (const char*)res1 + M1 * ldr1 * er : nullptr, ldr1,
                           res2 ? (const char*)res2 + M1 * ldr2 * er : nullptr, ldr2, res_f32,
                           (char*)out + M1 * ldo * eo, ldo, out_f32, pre ? (char*)pre + M1 * ldp * es : nullptr, ldp,
                           row_mode, P, prefix, stream);
  }
  RowMap rm = dense_rm(); rm.mode = row_mode; rm.P = P; rm.prefix = prefix;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    const int KTILES = cdiv(K, KT<T>::BK);
    auto go = [&](auto tile, auto tout, auto tres) -> int {
      typedef decltype(tout) TO; typedef decltype(tres) TR;
      // measured (tools/lin_sweep.py, bs 16 1024^2): the 256x256 ping-pong kernel for the large ViT
      // linears (o_proj 241 -> 215 us, up 576 -> 563, down 487 -> 418); else 256x128 x 3 stages for
      // K >= 2048, 128x128 otherwise.  Since the quarter-staged ping-pong epilogue (round 6) the plain bias-only
      // DPT projections M=65536 K=768 run on it too (tools/lib_ab.py: N 1024 160 -> 156 us, 512 90 -> 87, 256 54 -> 52)
      const int def = (pp_pays(M, N) && N % 256 == 0) ? 5 : (K >= 2048 ? 0 : 1);
      return with_cfg<T, true>(def, [&](auto C) -> int {
        constexpr int BM = decltype(C)::BM, BN = decltype(C)::BN, NST = decltype(C)::NST;
        DenseKC<T, decltype(C)::LM, decltype(C)::W> la{(const T*)x, ldx, M, K, 0};
        DenseKC<T, decltype(C)::LN, decltype(C)::W> lb{(const T*)w, (long)K, N, K, 0};
        EpiStd<TO, TR, T> e{(TO*)out, ldo, 0, bias, scale, shift, (const TR*)res1, ldr1, (const TR*)res2, ldr2,
                            (T*)pre, ldp, nullptr, act, M, N, rm};
        const int epi_probe = S3OD_KNOB("S3OD_EPI_PROBE", 0);   // dev: 1 = skip the epilogue's stores
        if (epi_probe == 1) e.M = 0;
        return launch_op<T, decltype(C)>(la, lb, e, M, N, KTILES, st);
      });
    };
    if (out_f32 && res_f32) return go(0, float{}, float{});
    if (out_f32) return go(0, float{}, T{});
    if (res_f32) return go(0, T{}, float{});
    return go(0, T{}, T{});
  });
  return 0;
}

// dx[rm(m), n] = sum_k dy[m,k] w[k,n] (+ res)  (w: [K=out][N=in]); act=ACT_GELU_BWD multiplies by
// gelu'(aux); with act=ACT_NONE a non-null aux is ADDED (aux may alias dx: in-place accumulate).
int s3od_linear_dgrad(int dtype, int M, int N, int K, const void* dy, long lddy, const void* w,
                      int act, const void* aux, long ldaux, void* dx, long lddx, int out_f32,
                      int row_mode, int P, int prefix, float* colsum, void* stream) {
  S3OD_REQUIRE(K % 8 == 0 && N % 8 == 0, "linear_dgrad: K,N %% 8");
  if (row_mode == 0 && split_tail(M)) {
    const int M1 = M & ~255, M2 = M - M1;
    int rc = s3od_linear_dgrad(dtype, M1, N, K, dy, lddy, w, act, aux, ldaux, dx, lddx, out_f32, row_mode, P, prefix,
                               colsum, stream);
    if (rc) return rc;
    const long es = dtype == S3OD_BF16 ? 2 : 4, eo = out_f32 ? 4 : es;
    TailCfg tail;
    return s3od_linear_dgrad(dtype, M2, N, K, (const char*)dy + M1 * lddy * es, lddy, w, act,
                             aux ? (const char*)aux + M1 * ldaux * eo : nullptr, ldaux, (char*)dx + M1 * lddx * eo, lddx,
                             out_f32, row_mode, P, prefix, colsum, stream);
  }
  // plain bf16 data gradients -- no activation derivative, no column sums, dense rows; aux an accumulate -- are plain
  // library GEMMs: hipBLASLt (blaslt.hip), 1.24-1.35x faster on the ViT backward's long-K shapes.  Only the whole
  // 256-row panels: left a tail, hipBLASLt adds a 16x16-tile kernel over the full K for it, which beside the side
  // stream's weight gradients took 300-370 us in the step (profiles/r06z_summary.md) -- the M-tail stays on the skinny
  // tail kernel above (TailCfg).  S3OD_DGRAD_BLASLT=0 (or no algorithm for the shape) keeps everything here.
  if (tl_cfg != 1 && dtype == S3OD_BF16 && act == ACT_NONE && !out_f32 && row_mode == 0 && !colsum &&
      S3OD_KNOB("S3OD_DGRAD_BLASLT", 1) &&
      blaslt_gemm_rm(dy, lddy, w, N, aux, ldaux, dx, lddx, M, N, K, (hipStream_t)stream) == 0)
    return s3od_check_launch("linear_dgrad (hipBLASLt)");
  RowMap rm = dense_rm(); rm.mode = row_mode; rm.P = P; rm.prefix = prefix;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    const int KTILES = cdiv(K, KT<T>::BK);
    // ping-pong 256x256 for the long-K dgrads (up 441 -> 374 us, qkv 334 -> 292) and the K = 768 ones with an
    // activation-derivative epilogue (down-projection x gelu': 519 -> 500 us, round 6); 128x128 for plain K = 768
    // (o_proj 118 vs 118 us)
    const int def = (pp_pays(M, N) && N % 256 == 0 && (K >= 2048 || act != ACT_NONE)) ? 5 : 1;
    return with_cfg<T, true>(def, [&](auto C) -> int {
      constexpr int BM = decltype(C)::BM, BN = decltype(C)::BN, NST = decltype(C)::NST;
      DenseKC<T, decltype(C)::LM, decltype(C)::W> la{(const T*)dy, lddy, M, K, 0};
      DenseMC<T, decltype(C)::LN, decltype(C)::W> lb{(const T*)w, (long)N, K, N};
      if (out_f32) {
        // f32 output: aux is an f32 tensor to add (e.g. the residual-stream gradient, in place)
        EpiStd<float, float> e{(float*)dx, lddx, 0, nullptr, nullptr, nullptr, (const float*)aux, ldaux, nullptr, 0, nullptr, 0, nullptr, act, M, N, rm, colsum};
        return launch_op<T, decltype(C)>(la, lb, e, M, N, KTILES, st);
      }
      EpiStd<T, T> e{(T*)dx, lddx, 0, nullptr, nullptr, nullptr, (const T*)aux, ldaux, nullptr, 0, nullptr, 0, nullptr, act, M, N, rm, colsum};
      return launch_op<T, decltype(C)>(la, lb, e, M, N, KTILES, st);
    });
  });
  return 0;
}

// default tile config of a linear weight gradient: the 256x256 ping-pong kernel with split-K slabs for the large
// outputs (3072x768 441 -> 403 us, 768x3072 457 -> 398, 2304x768 335 -> 308), 256x128 x 3 stages with fp32 atomics
// otherwise.  S3OD_LWG_ROWS_PP=1 also puts the small outputs over >= 64K rows on the ping-pong kernel: faster alone
// (tools/wgrad_sweep.py: 768x768 127 -> 110 us, 1024x768 154 -> 144, 256x256 x 1M rows 283 -> 268;
// profiles/r05t_wgrad_sweep.txt) but null in the step, where these run on the side stream beside the data gradients
// (tools/ab_step.py medians 151.4 vs 151.0 ms), so off by default
static int linear_wgrad_def_cfg(int Nout, int Kin, int rows) {
  const bool big_rows = rows >= 65536 && S3OD_KNOB("S3OD_LWG_ROWS_PP", 0);
  return ((long)Nout * Kin > 1024L * 1024 || big_rows) ? 5 : 0;
}
// split-K slab floats a linear weight gradient uses (0: the fp32-atomic epilogue, no slab): the ping-pong kernel's
// split-K partials go to sp caller-owned fp32 slabs [sp][Nout][Kin], summed by wgrad_reduce_kernel
static long linear_wgrad_slab_floats(int dtype, int Nout, int Kin, int rows, int split) {
  if (dtype != S3OD_BF16 || !slab_ok() || Kin % 4 != 0) return 0;
  const int KTILES = cdiv(rows, KT<bf16>::BK);
  const int def = linear_wgrad_def_cfg(Nout, Kin, rows);
  return with_cfg<bf16, true>(def, [&](auto C) -> long {
    if constexpr (!decltype(C)::SLAB) return 0;
    else {
      const int sp = split > 0 ? split : wgrad_split<bf16, 256, 256, 2>(cdiv(Nout, 256) * cdiv(Kin, 256), KTILES);
      return sp > 1 ? (long)sp * Nout * Kin : 0;
    }
  });
}

// bytes of the slab workspace s3od_linear_wgrad uses for these arguments (0 = none needed)
int s3od_linear_wgrad_ws(int dtype, int Nout, int Kin, int rows, int split, long* bytes) {
  S3OD_REQUIRE(bytes != nullptr, "linear_wgrad_ws: null output");
  *bytes = 4 * linear_wgrad_slab_floats(dtype, Nout, Kin, rows, split);
  return 0;
}

// dw[n_out, k_in] += sum_rows dy[row, n_out] x[row, k_in]  (split over rows: fp32 atomics into dw, or -- when the
// caller passes a slab of >= s3od_linear_wgrad_ws bytes -- per-split fp32 slabs summed into dw by a second kernel)
int s3od_linear_wgrad(int dtype, int Nout, int Kin, int rows, const void* dy, long lddy,
                      const void* x, long ldx, float* dw, int split, float* slab, long slab_bytes, void* stream) {
  S3OD_REQUIRE(Nout % 8 == 0 && Kin % 8 == 0, "linear_wgrad: dims %% 8");
  hipStream_t st = (hipStream_t)stream;
  const long need = slab ? linear_wgrad_slab_floats(dtype, Nout, Kin, rows, split) : 0;
  if (need == 0 || slab_bytes < 4 * need) slab = nullptr;
  DISPATCH_T(dtype, {
    const int KTILES = cdiv(rows, KT<T>::BK);
    const int def = linear_wgrad_def_cfg(Nout, Kin, rows);
    return with_cfg<T, true>(def, [&](auto C) -> int {
      constexpr int BM = decltype(C)::BM, BN = decltype(C)::BN, NST = decltype(C)::NST;
      int sp = split > 0 ? split : wgrad_split<T, BM, BN, NST>(cdiv(Nout, BM) * cdiv(Kin, BN), KTILES);
      DenseMC<T, decltype(C)::LM, decltype(C)::W> la{(const T*)dy, lddy, rows, Nout};
      DenseMC<T, decltype(C)::LN, decltype(C)::W> lb{(const T*)x, ldx, rows, Kin};
      if constexpr (decltype(C)::SLAB) {
        if (slab) {
          EpiWgradPart e{slab, Nout, Kin};
          int rc = launch_igemm<T, BM, BN, decltype(la), decltype(lb), decltype(e), NST, decltype(C)::WM>(la, lb, e, Nout, Kin, KTILES, sp, 1, st);
          if (rc) return rc;
          hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(cdiv((long)Nout * Kin / 4, 256)), dim3(256), 0, st, slab, sp, Nout, Kin, dw, Kin, 1);
          return s3od_check_launch("linear_wgrad reduce");
        }
      }
      EpiWgrad e{dw, Nout, Kin, Kin, 1};
      const int epi_probe = S3OD_KNOB("S3OD_EPI_PROBE", 0);   // dev: 1 = skip the split-K atomics (timing only)
      if (epi_probe == 1) e.M = 0;
      return launch_igemm<T, BM, BN, decltype(la), decltype(lb), decltype(e), NST, decltype(C)::WM>(la, lb, e, Nout, Kin, KTILES, sp, 1, st);
    });
  });
  return 0;
}

// fused QKV projection + bias + RoPE + head split. x: [B*Ntok, D] T ; w: [3D, D] T ; D = 64 H
int s3od_qkv_rope_fwd(int dtype, int B, int Ntok, int P, int H, const void* x, const void* w, const float* bias,
                      const float* cos_t, const float* sin_t, void* q, void* k, void* v, void* stream) {
  const int D = 64 * H, N = 3 * D, Mall = B * Ntok;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    auto part = [&](int m_first, int M) -> int {
      return with_cfg<T>(pp_pays(M, N) ? 5 : 1, [&](auto C) -> int {
        constexpr int BM = decltype(C)::BM, BN = decltype(C)::BN, NST = decltype(C)::NST;
        DenseKC<T, decltype(C)::LM, decltype(C)::W> la{(const T*)x + (long)m_first * D, (long)D, M, D, 0};
        DenseKC<T, decltype(C)::LN, decltype(C)::W> lb{(const T*)w, (long)D, N, D, 0};
        EpiQKV<T> e{(T*)q, (T*)k, (T*)v, bias, cos_t, sin_t, M, Ntok, P, H};
        e.moff = m_first;
        return launch_op<T, decltype(C)>(la, lb, e, M, N, cdiv(D, KT<T>::BK), st);
      });
    };
    if (!split_tail(Mall)) return part(0, Mall);
    const int M1 = Mall & ~255;
    int rc = part(0, M1);
    if (rc) return rc;
    TailCfg tail;
    return part(M1, Mall - M1);
  });
  return 0;
}

// the 3x3 s1 p1 convs whose output channels fill 256-wide tiles and whose pixel tiles fill whole rounds of the
// chip run on the ping-pong kernel when there are >= 8 rounds of tiles or K >= 9 * 512 (measured, tools/conv_cfg_bench.py,
// bs 16: 256^2 RCU 1.38 vs 1.51-1.66 ms with BN sums, plain 1.21 vs 1.34-1.38 ms; 128^2 512 -> 256 0.56 vs 0.69-0.81 ms;
// the 128^2 256 -> 256 RCU 0.39 vs 0.37-0.38 ms with BN sums stays on 128x128 tiles), and from 2 rounds without BN
// statistics (eval: 4 rounds = the C5 256^2 bs-4 RCUs, C5 74.72 -> 74.47 ms, C2 24.99 -> 24.91 ms per batch; 2 rounds =
// the C2 128^2 bs-8 RCUs, C2 25.37 -> 25.25 ms; 1 round mixed; profiles/r04b_conv_pp_rounds_ab.txt).
// S3OD_CONV_PP=0 (under S3OD_AB=1: per call): the 128x128 implicit GEMM (A/B runs); S3OD_CONV_PP=2: the eval threshold with BN
// statistics too; S3OD_CONV_PP_MIN: the eval threshold in 256x256 tiles (default 512).
static bool conv_pp_ok(const ConvGeo& g, int M, int N, bool stats) {
  const int nch = g.SC / 64;
  const long tiles = (long)(M / 256) * (N / 256);
  const int min_ns = S3OD_KNOB("S3OD_CONV_PP_MIN", 512) > 0 ? S3OD_KNOB("S3OD_CONV_PP_MIN", 512) : 512;
  const bool rounds = tiles >= 2048 || g.SC >= 512 || (tiles >= min_ns && (!stats || S3OD_KNOB("S3OD_CONV_PP", -1) == 2));
  // 128-channel inputs (the output_conv1 data gradient, K = 9 x 128): the ping-pong kernel's per-tap A tiles are half
  // width there and the generic path measured faster in the whole step (150.1 -> 147.5 ms median, same box)
  if (g.SC < 256 && !S3OD_KNOB("S3OD_CONV_PP_SC128", 0)) return false;
  return tl_cfg < 0 && gemm_cfg() < 0 && g.KH == 3 && g.KW == 3 && g.s == 1 && g.p == 1 && g.RH == g.SH && g.RW == g.SW &&
         g.SC % 64 == 0 && (nch & (nch - 1)) == 0 && N % 256 == 0 && pp_pays(M, N) && rounds && !S3OD_OFF("S3OD_CONV_PP");
}

// implicit-GEMM conv forward (im2col gathered per K tile by ConvFwdA); also the stride-1 3x3 data gradient run as a
// forward conv of dy with the transposed, tap-reversed weight (s3od_conv_dgrad with wT)
static int conv_fwd_igemm(int dtype, ConvGeo g, int M, int N, int K, int Cin, int Cout, const void* x, int relu_in,
                          const void* wp, const float* bias, const float* scale, const float* shift, int act,
                          const void* res1, const void* res2, void* out, void* pre, double* stats, float* colsum,
                          hipStream_t st) {
  DISPATCH_T(dtype, {
    const int KTILES = cdiv(K, KT<T>::BK);
    if constexpr (sizeof(T) == 2) {
      if (conv_pp_ok(g, M, N, stats != nullptr)) {
        // 3x3 s1 p1 with 256-multiple output channels: the 256x256 ping-pong kernel (one workgroup per CU covers
        // all 256 output channels of 256 pixels, so each im2col A tile is gathered once) with the Conv3A loader
        auto pp = [&](auto rl) -> int {
          Conv3A<128, decltype(rl)::value> la{};
          la.x = (const bf16*)x; la.B = g.B; la.H = g.SH; la.W = g.SW; la.SC = g.SC; la.M = M;
          la.lgc = __builtin_ctz((unsigned)(g.SC / 64));
          DenseKC<bf16, 128> lb{(const bf16*)wp, (long)K, N, K, 0};
          EpiStd<bf16, bf16> e{(bf16*)out, (long)Cout, 0, bias, scale, shift, (const bf16*)res1, (long)Cout, (const bf16*)res2,
                               (long)Cout, (bf16*)pre, (long)Cout, stats, act, M, N, dense_rm(), colsum};
          return launch_igemm<bf16, 256, 256, decltype(la), decltype(lb), decltype(e)>(la, lb, e, M, N, KTILES, 1, 1, st);
        };
        return relu_in ? pp(std::true_type{}) : pp(std::false_type{});
      }
    }
    // 128-output-channel 3x3 convs over >= 2M pixels (output_conv1 at 512^2): 256x128 tiles, 3 stages (one workgroup
    // per CU) -- 2630 vs 2765 us at bs 16 (tools/lin_sweep.py, S3OD_GEMM_CFG 0 vs 1); S3OD_CONV_N128_CFG picks another
    const int def = Cout <= 64 ? 3 : (g.KH == 3 && Cout < 256 && M >= (1 << 21)) ? S3OD_KNOB("S3OD_CONV_N128_CFG", 0) : 1;
    auto go = [&](auto bn, auto rl) -> int {
      return with_cfg<T>(def, [&](auto C0) -> int {
        typedef ConvCfg<decltype(C0), decltype(bn)::value> CC;
        constexpr int BM = CC::BM, NST = CC::NST;
        constexpr int BN = decltype(bn)::value < CC::BN ? decltype(bn)::value : CC::BN;
        constexpr int LN = CC::PP ? CC::LN : BN;
        CC C{};
        ConvFwdA<T, CC::LM, decltype(rl)::value, CC::W> la{}; la.x = (const T*)x; la.g = g; la.M = M; la.relu = relu_in;
        DenseKC<T, LN, CC::W> lb{(const T*)wp, (long)K, N, K, 0};
        EpiStd<T, T> e{(T*)out, (long)Cout, 0, bias, scale, shift, (const T*)res1, (long)Cout, (const T*)res2, (long)Cout,
                       (T*)pre, (long)Cout, stats, act, M, N, dense_rm(), colsum};
        return launch_igemm<T, BM, BN, decltype(la), decltype(lb), decltype(e), NST, decltype(C)::WM>(la, lb, e, M, N, KTILES, 1, 1, st);
      });
    };
    if (relu_in) {
      if (Cout <= 64) return go(std::integral_constant<int, 64>{}, std::true_type{});
      if (Cout < 256) return go(std::integral_constant<int, 128>{}, std::true_type{});
      return go(std::integral_constant<int, 256>{}, std::true_type{});
    }
    if (Cout <= 64) return go(std::integral_constant<int, 64>{}, std::false_type{});
    if (Cout < 256) return go(std::integral_constant<int, 128>{}, std::false_type{});
    return go(std::integral_constant<int, 256>{}, std::false_type{});
  });
  return 0;
}

// ---------------------------------------------------------------------------------- convs
// NHWC activations, weights repacked [Cout][KH][KW][Cin].
// pre = conv(relu?(x)) + bias[n]; out[b,oy,ox,n] = act(pre*scale[n] + shift[n]) (+res1 +res2);
// stats: BN batch sums of pre, fp64 [S3OD_NREP = 32][sum | sum of squares][Cout] replicas, all zero on entry
// (s3od_bn_finalize folds and clears them).
int s3od_conv_fwd(int dtype, int B, int H, int W, int Cin, int OH, int OW, int Cout, int KH, int KW,
                  int stride, int pad, const void* x, int relu_in, const void* wp,
                  const float* bias, const float* scale, const float* shift, int act, const void* res1, const void* res2,
                  void* out, void* pre, double* stats, float* colsum, void* stream) {
  S3OD_REQUIRE(Cin % 8 == 0 && Cout % 8 == 0, "conv_fwd: channels %% 8 (Cin=%d Cout=%d)", Cin, Cout);
  ConvGeo g{}; g.B = B; g.SH = H; g.SW = W; g.SC = Cin; g.RH = OH; g.RW = OW; g.KH = KH; g.KW = KW; g.s = stride; g.p = pad;
  const int M = B * OH * OW, N = Cout, K = KH * KW * Cin;
  hipStream_t st = (hipStream_t)stream;
  if (KH == 4 && KW == 4 && stride == 2 && pad == 1 && H == 2 * OH && W == 2 * OW && Cin == 64 && Cout == 128 && !relu_in &&
      !bias && !scale && !shift && !res1 && !res2 && !pre && !stats && act == ACT_NONE && convt_rw_ok(dtype, B, OH, OW))
    // the data gradient of upsample_2x.0 (ConvTranspose2d(128, 64, 4, 2, 1)): register-weight strided conv
    return launch_conv4s2_rw((const bf16*)x, (const bf16*)wp, colsum, (bf16*)out, B, OH, OW, st);
  if (KH == 3 && KW == 3 && stride == 1 && pad == 1 && OH == H && OW == W && Cin == 64 && Cout == 64 && !relu_in && !stats &&
      !scale && !shift && !res1 && !res2 && !pre && !colsum && (act == ACT_NONE || act == ACT_RELU) && rw_ok(dtype, B, H, W))
    return act == ACT_RELU ? launch_rw<2, 64>((const bf16*)x, (const bf16*)wp, bias, nullptr, nullptr, (bf16*)out, B, H, W, st)
                           : launch_rw<0, 64>((const bf16*)x, (const bf16*)wp, bias, nullptr, nullptr, (bf16*)out, B, H, W, st);
  return conv_fwd_igemm(dtype, g, M, N, K, Cin, Cout, x, relu_in, wp, bias, scale, shift, act, res1, res2, out, pre, stats,
                        colsum, st);
}

// conv dgrad == ConvTranspose2d forward.  dy: [B,OH,OW,Cout] (conv output grid); w: [Cout][KH][KW][Cin];
// dx: [B,H,W,Cin] (conv input grid).  One launch per output parity class.  wT (nullable, bf16): [Cin][KH][KW][Cout],
// taps reversed for 3x3 s1 (the data gradient as a forward conv of dy), as-is for the 4x4 s2 sub-pixel kernel.
int s3od_conv_dgrad(int dtype, int B, int H, int W, int Cin, int OH, int OW, int Cout, int KH, int KW,
                    int stride, int pad, const void* dy, const void* wp,
                    const float* bias, const float* scale, const float* shift, int act, const void* res1,
                    const void* res2, void* dx, void* pre, double* stats, float* colsum, const void* wT, void* stream) {
  S3OD_REQUIRE(Cin % 8 == 0 && Cout % 8 == 0, "conv_dgrad: channels %% 8");
  if (wT && KH == 4 && KW == 4 && stride == 2 && pad == 1 && H == 2 * OH && W == 2 * OW && Cout == 128 && Cin == 64 && !scale &&
      !shift && !res1 && !res2 && !pre && !stats && !colsum && (act == ACT_NONE || act == ACT_RELU) && convt_rw_ok(dtype, B, OH, OW))
    // ConvTranspose2d(128, 64, 4, 2, 1) forward (upsample_2x.0): the register-weight sub-pixel kernel; wT =
    // [Cin = 64][4][4][Cout = 128], the conv-view weight transposed WITHOUT tap reversal (s3od_repack_multi mode 2)
    return launch_convt_rw((const bf16*)dy, (const bf16*)wT, bias, act == ACT_RELU, (bf16*)dx, B, OH, OW, (hipStream_t)stream);
  if (wT && KH == 3 && KW == 3 && stride == 1 && pad == 1 && OH == H && OW == W && Cin == 64 && (Cout == 64 || Cout == 96) &&
      !bias && !scale && !shift && !res2 && !pre && !stats && act == ACT_RELU_BWD && res1 && rw_ok(dtype, B, H, W))
    // stride-1 3x3 data gradient = forward conv of dy with the transposed, tap-reversed weight wT ([Cin][3][3][Cout])
    return Cout == 64 ? launch_rw<1, 64>((const bf16*)dy, (const bf16*)wT, nullptr, (const bf16*)res1, colsum, (bf16*)dx, B, H,
                                         W, (hipStream_t)stream)
                      : launch_rw<1, 96>((const bf16*)dy, (const bf16*)wT, nullptr, (const bf16*)res1, colsum, (bf16*)dx, B, H,
                                         W, (hipStream_t)stream);
  if (wT && KH == 3 && KW == 3 && stride == 1 && pad == 1 && OH == H && OW == W && (Cin != 64 || Cout > 96) && !pre &&
      !stats && !S3OD_OFF("S3OD_DGRAD_WT")) {
    // stride-1 3x3 data gradient = forward conv of dy (Cout channels) with wT [Cin][3][3][Cout]: the forward
    // gather (ConvFwdA) instead of the transposed-conv gather (measured faster on the 256-channel RCU convs)
    ConvGeo gf{}; gf.B = B; gf.SH = H; gf.SW = W; gf.SC = Cout; gf.RH = H; gf.RW = W; gf.KH = 3; gf.KW = 3; gf.s = 1; gf.p = 1;
    return conv_fwd_igemm(dtype, gf, B * H * W, Cin, 9 * Cout, Cout, Cin, dy, 0, wT, bias, scale, shift, act, res1, res2, dx,
                          nullptr, nullptr, colsum, (hipStream_t)stream);
  }
  ConvGeo g0{}; g0.B = B; g0.SH = OH; g0.SW = OW; g0.SC = Cout; g0.KH = KH; g0.KW = KW; g0.s = stride; g0.p = pad;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    for (int py = 0; py < stride; py++)
      for (int px = 0; px < stride; px++) {
        ConvGeo g = make_class(g0, H, W, py, px);
        const int M = B * g.RH * g.RW, N = Cin, K = g.nth * g.ntw * Cout;
        if (M == 0) continue;
        RowMap rm{}; rm.mode = 2; rm.RH = g.RH; rm.RW = g.RW; rm.OH = H; rm.OW = W; rm.s = stride; rm.py = py; rm.px = px;
        auto go = [&](auto bn) -> int {
          return with_cfg<T>(Cin <= 64 ? 3 : 1, [&](auto C0) -> int {
            typedef ConvCfg<decltype(C0), decltype(bn)::value> CC;
            constexpr int BM = CC::BM, NST = CC::NST;
            constexpr int BN = decltype(bn)::value < CC::BN ? decltype(bn)::value : CC::BN;
            constexpr int LN = CC::PP ? CC::LN : BN;
            CC C{};
            ConvDgradA<T, CC::LM, CC::W> la{}; la.dy = (const T*)dy; la.g = g; la.M = M;
            ConvDgradB<T, LN, CC::W> lb{}; lb.w = (const T*)wp; lb.g = g; lb.NC = Cin;
            EpiStd<T, T> e{(T*)dx, (long)Cin, 0, bias, scale, shift, (const T*)res1, (long)Cin, (const T*)res2, (long)Cin,
                           (T*)pre, (long)Cin, stats, act, M, N, rm, colsum};
            return launch_igemm<T, BM, BN, decltype(la), decltype(lb), decltype(e), NST, decltype(C)::WM>(la, lb, e, M, N, cdiv(K, KT<T>::BK), 1, 1, st);
          });
        };
        int rc = Cin <= 64 ? go(std::integral_constant<int, 64>{})
                           : (Cin < 256 ? go(std::integral_constant<int, 128>{}) : go(std::integral_constant<int, 256>{}));
        if (rc) return rc;
      }
  });
  return 0;
}

// the 256-channel 3x3 s1 weight gradients on the ping-pong kernel (Wgrad3B): the split-K factor, 0 when the
// call does not take that path
static int conv_wgrad_pp_split(int dtype, int B, int H, int W, int Cin, int OH, int OW, int Cout, int KH, int KW, int stride,
                               int pad, int split) {
  if (!(dtype == S3OD_BF16 && KH == 3 && KW == 3 && stride == 1 && pad == 1 && OH == H && OW == W && W % 64 == 0 &&
        Cin % 256 == 0 && Cout % 256 == 0 && ((long)H * W >= 128L * 128 || Cin >= 512) && tl_cfg < 0 && gemm_cfg() < 0 &&
        !S3OD_OFF("S3OD_WGRAD_PP")))
    return 0;
  const int KTILES = B * OH * OW / 64, tiles = (Cout / 256) * (9 * Cin / 256);
  return split > 0 ? split : std::max(1, std::min(256 / tiles, KTILES / 8));
}

// bytes of the slab workspace s3od_conv_wgrad uses for these arguments (0 = none needed)
// The LDS-DMA 3x3 weight gradient (wgrad_dma.hip) takes every 3x3 s1 p1 bf16 conv whose tiles are whole (H % 8,
// W % 32), input channels a multiple of 64 and output channels a multiple of 64 (or the 96 of the mask heads, Cin 64).
// Measured at bs 16 against the ping-pong Wgrad3B kernel (tools/wgrad_bench.py big, same box): 256^2 256->256
// 1523-1571 vs 822-834 us, 128^2 256->256 401 vs 215, 128^2 512->256 755 vs 394, 64^2 1024->256 425 vs 220,
// 64^2 256->256 128 vs 84.  S3OD_WGRAD_DMA=0 restores the earlier routing.
static bool wgrad_dma_ok(int dtype, int H, int W, int Cin, int OH, int OW, int Cout, int KH, int KW, int stride, int pad) {
  return dtype == S3OD_BF16 && KH == 3 && KW == 3 && stride == 1 && pad == 1 && OH == H && OW == W && Cin % 64 == 0 &&
         (Cout % 64 == 0 || (Cout == 96 && Cin == 64)) && H % HT_TH == 0 && W % HT_TW == 0 &&
         (long)H * W * (Cin > Cout ? Cin : Cout) * 2 < (1L << 31) && !S3OD_OFF("S3OD_WGRAD_DMA");
}

// the routing decision shared by the slab query and the call (the query ignored S3OD_WGRAD_HALO, so with
// the knob off the call took the ping-pong path without the slab it needed)
static bool wgrad_takes_dma(int dtype, int H, int W, int Cin, int OH, int OW, int Cout, int KH, int KW, int stride, int pad) {
  return S3OD_KNOB("S3OD_WGRAD_HALO", 1) && wgrad_dma_ok(dtype, H, W, Cin, OH, OW, Cout, KH, KW, stride, pad);
}

int s3od_conv_wgrad_ws(int dtype, int B, int H, int W, int Cin, int OH, int OW, int Cout, int KH, int KW, int stride,
                       int pad, int split, long* bytes) {
  S3OD_REQUIRE(bytes != nullptr, "conv_wgrad_ws: null output");
  const int sp = slab_ok() && !wgrad_takes_dma(dtype, H, W, Cin, OH, OW, Cout, KH, KW, stride, pad)
                     ? conv_wgrad_pp_split(dtype, B, H, W, Cin, OH, OW, Cout, KH, KW, stride, pad, split) : 0;
  *bytes = sp > 1 ? 4L * sp * Cout * KH * KW * Cin : 0;
  return 0;
}

// conv wgrad: dw[Cout][Cin][KH][KW] (PyTorch layout, fp32) += sum_pix dy[pix][co] * x[src(pix,tap)][ci]
// dy: [B,OH,OW,Cout]; x: [B,H,W,Cin].  Also serves ConvTranspose2d weights (conv view).
// ws (nullable): Cout*KH*KW*Cin floats, all zero on entry and left all zero (split-K partials in the GEMM layout)
// slab (nullable): caller-owned scratch of slab_bytes (>= s3od_conv_wgrad_ws) for the ping-pong kernel's split-K slabs;
// without it that path adds its partials into ws by fp32 atomics.  The library never allocates.
int s3od_conv_wgrad(int dtype, int B, int H, int W, int Cin, int OH, int OW, int Cout, int KH, int KW,
                    int stride, int pad, const void* dy, const void* x, int relu_x, float* dw, float* ws, int split,
                    float* slab, long slab_bytes, void* stream) {
  S3OD_REQUIRE(Cin % 8 == 0 && Cout % 8 == 0, "conv_wgrad: channels %% 8");
  ConvGeo g{}; g.B = B; g.SH = H; g.SW = W; g.SC = Cin; g.RH = OH; g.RW = OW; g.KH = KH; g.KW = KW; g.s = stride; g.p = pad;
  const int NPIX = B * OH * OW, M = Cout, N = KH * KW * Cin;
  hipStream_t st = (hipStream_t)stream;
  const int wg_knob = S3OD_KNOB("S3OD_WGRAD_HALO", 1);
  // halo-tile kernel: 3x3 s1 p1, Cin a multiple of 64, Cout a multiple of 64 (or 96 for the mask heads).
  // Measured at bs 16 (tools/lin_sweep.py SWEEP=conv64): 2.4x / 1.75x on the 1024^2 64 -> 64 / 96 convs,
  // 1.2x on 512^2 256 -> 128, equal at 256^2 / 128^2 and 8 % slower at 64^2 -> used for Cin 64 or >= 512^2 maps
  if (dtype == S3OD_BF16 && ws && KH == 4 && KW == 4 && stride == 2 && pad == 1 && H == 2 * OH && W == 2 * OW && Cin % 64 == 0 &&
      Cout % 64 == 0 && !relu_x && (long)H * W * Cin * 2 < (1L << 31) && (long)OH * OW * Cout * 2 < (1L << 31) &&
      !S3OD_OFF("S3OD_WGRAD_DMA")) {
    // the ConvTranspose2d(128, 64, 4, 2, 1) weight (upsample_2x.0) in its conv view
    int rc = launch_wgrad4s2((const bf16*)dy, (const bf16*)x, ws, B, OH, OW, Cin, Cout, st);
    if (rc) return rc;
    hipLaunchKernelGGL(wgrad_permute_add_kernel, dim3(cdiv((long)M * N, 256)), dim3(256), 0, st, ws, dw, M, Cin, KH * KW);
    return s3od_check_launch("conv_wgrad permute");
  }
  const int coblk = Cout % 64 == 0 ? 64 : (Cout == 96 ? 96 : 0);
  // the LDS-DMA kernel works on 64 x 64 channel blocks; the 96-output-channel mask heads (Cin 64) run as two output
  // blocks, the second reading 32 channels past each pixel's 96 (finite data of the next pixel, zeros past the image)
  // whose products are never flushed
  const bool dma = ws && wgrad_takes_dma(dtype, H, W, Cin, OH, OW, Cout, KH, KW, stride, pad);
  if (dma || (wg_knob && dtype == S3OD_BF16 && ws && KH == 3 && KW == 3 && stride == 1 && pad == 1 && OH == H && OW == W &&
              Cin % 64 == 0 && coblk && (Cin == 64 || (long)H * W >= 512L * 512))) {
    int rc = dma ? wgrad3x3_dma_launch(relu_x, (const bf16*)dy, (const bf16*)x, ws, B, H, W, Cin, Cout, st) :
             coblk == 64 ? (relu_x ? launch_wgrad_halo<64, true>((const bf16*)dy, (const bf16*)x, ws, B, H, W, Cin, Cout, st)
                                   : launch_wgrad_halo<64, false>((const bf16*)dy, (const bf16*)x, ws, B, H, W, Cin, Cout, st))
                         : (relu_x ? launch_wgrad_halo<96, true>((const bf16*)dy, (const bf16*)x, ws, B, H, W, Cin, Cout, st)
                                   : launch_wgrad_halo<96, false>((const bf16*)dy, (const bf16*)x, ws, B, H, W, Cin, Cout, st));
    if (rc) return rc;
    hipLaunchKernelGGL(wgrad_permute_add_kernel, dim3(cdiv((long)M * N, 256)), dim3(256), 0, st, ws, dw, M, Cin, KH * KW);
    return s3od_check_launch("conv_wgrad permute");
  }
  if (ws && conv_wgrad_pp_split(dtype, B, H, W, Cin, OH, OW, Cout, KH, KW, stride, pad, split) > 0) {
    // the 256-channel RCU / layerK_rn weight gradients on the ping-pong kernel: one 256 x 256 tile = 256 output
    // channels x one tap's 256 input channels, K = pixels split over ~one round of workgroups (fp32 atomics into the
    // GEMM-layout workspace, then the permute into dW).  Measured vs the 128x128 implicit GEMM (tools/conv_cfg_bench.py
    // WG=1, bs 16): 256^2 1.47 vs 1.63-1.66 ms (ReLU'd input 1.52 vs 1.77-1.97), 128^2 0.39 vs 0.42, 128^2 512 -> 256
    // 0.76 vs 0.85, 64^2 1024 -> 256 0.38 vs 0.44; the 64^2 256 -> 256 one (0.14 vs 0.13 ms) stays on 128x128
    const int KTILES = NPIX / 64;
    const int sp = conv_wgrad_pp_split(dtype, B, H, W, Cin, OH, OW, Cout, KH, KW, stride, pad, split);
    DenseMC<bf16, 128> la{(const bf16*)dy, (long)Cout, NPIX, Cout};
    if (!(slab_ok() && sp > 1 && slab_bytes >= 4L * sp * M * N)) slab = nullptr;
    auto pp = [&](auto rl, auto e) -> int {
      Wgrad3B<128, decltype(rl)::value> lb{}; lb.x = (const bf16*)x; lb.B = B; lb.H = H; lb.W = W; lb.Cin = Cin;
      return launch_igemm<bf16, 256, 256, decltype(la), decltype(lb), decltype(e)>(la, lb, e, M, N, KTILES, sp, 1, st);
    };
    if (slab) {       // split-K slabs, summed straight into dW's PyTorch layout (the atomic workspace stays untouched)
      EpiWgradPart e{slab, M, N};
      int rc = relu_x ? pp(std::true_type{}, e) : pp(std::false_type{}, e);
      if (rc) return rc;
      hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(cdiv((long)M * N / 4, 256)), dim3(256), 0, st, slab, sp, M, N, dw, Cin, KH * KW);
      return s3od_check_launch("conv_wgrad reduce");
    }
    EpiWgrad e{ws, M, N, N, 1};
    int rc = relu_x ? pp(std::true_type{}, e) : pp(std::false_type{}, e);
    if (rc) return rc;
    hipLaunchKernelGGL(wgrad_permute_add_kernel, dim3(cdiv((long)M * N, 256)), dim3(256), 0, st, ws, dw, M, Cin, KH * KW);
    return s3od_check_launch("conv_wgrad permute");
  }
  DISPATCH_T(dtype, {
    const int KTILES = cdiv(NPIX, KT<T>::BK);
    auto go = [&](auto bm, auto rl) -> int {
      constexpr int BM = decltype(bm)::value, BN = 128, NST = 2;
      int sp = split > 0 ? split : wgrad_split<T, BM, BN, NST>(cdiv(M, BM) * cdiv(N, BN), KTILES);
      DenseMC<T, BM> la{(const T*)dy, (long)Cout, NPIX, Cout};
      WgradB<T, BN, decltype(rl)::value> lb{}; lb.x = (const T*)x; lb.g = g; lb.NPIX = NPIX; lb.relu = relu_x;
      // taps > 1: the split-K atomics go to a workspace in the GEMM's own [Cout][tap][Cin] layout
      // (a wave's adds hit contiguous addresses), then one pass permutes into the PyTorch layout
      const bool viaws = ws != nullptr && KH * KW > 1;
      EpiWgrad e = viaws ? EpiWgrad{ws, M, N, N, 1} : EpiWgrad{dw, M, N, Cin, KH * KW};
      int rc = launch_igemm<T, BM, BN, decltype(la), decltype(lb), decltype(e), NST>(la, lb, e, M, N, KTILES, sp, 1, st);
      if (rc || !viaws) return rc;
      hipLaunchKernelGGL(wgrad_permute_add_kernel, dim3(cdiv((long)M * N, 256)), dim3(256), 0, st, ws, dw, M, Cin, KH * KW);
      return s3od_check_launch("conv_wgrad permute");
    };
    if (relu_x) {
      if (Cout <= 64) return go(std::integral_constant<int, 64>{}, std::true_type{});
      return go(std::integral_constant<int, 128>{}, std::true_type{});
    }
    if (Cout <= 64) return go(std::integral_constant<int, 64>{}, std::false_type{});
    return go(std::integral_constant<int, 128>{}, std::false_type{});
  });
  return 0;
}

// NM (3 for dinob, 1 for dinol) 3x3 64->32 + ReLU + 1x1 32->1 mask heads as one GEMM (N=32NM) with
// a fused epilogue.  feat: [B,H,W,64] T ; w1p: [32NM][3][3][64] T ; b1: [32NM]; w2: [NM][32]; b2: [NM]
// logits: [B,NM,H,W] fp32 (NCHW, the reference output layout); hsave: optional [B*H*W, 32NM] T
int s3od_mask_heads_fwd(int dtype, int B, int H, int W, int NM, const void* feat, const void* w1p, const float* b1,
                        const float* w2, const float* b2, float* logits, void* hsave, void* stream) {
  S3OD_REQUIRE(NM == 1 || NM == 3, "mask_heads_fwd: %d heads not built (1 or 3)", NM);
  ConvGeo g{}; g.B = B; g.SH = H; g.SW = W; g.SC = 64; g.RH = H; g.RW = W; g.KH = 3; g.KW = 3; g.s = 1; g.p = 1;
  const int M = B * H * W, N = 32 * NM, K = 9 * 64;
  hipStream_t st = (hipStream_t)stream;
  if (N == 96 && rw_ok(dtype, B, H, W) && (long)3 * H * W * 4 < (1L << 31))
    return launch_rw<3, 64>((const bf16*)feat, (const bf16*)w1p, b1, nullptr, nullptr, (bf16*)hsave, B, H, W, st, w2, b2, logits);
  DISPATCH_T(dtype, {
    constexpr int BM = 128;
    ConvFwdA<T, BM> la{}; la.x = (const T*)feat; la.g = g; la.M = M; la.relu = 0;
    EpiHeads<T> e{logits, (T*)hsave, b1, w2, b2, M, H * W, NM};
    // 2 K stages -> 2 workgroups per CU, so one's epilogue overlaps the other's K loop
    if (NM == 3) {
      DenseKC<T, 128> lb{(const T*)w1p, (long)K, N, K, 0};
      return launch_igemm<T, BM, 128, decltype(la), decltype(lb), decltype(e), 2>(la, lb, e, M, 128, cdiv(K, KT<T>::BK), 1, 1, st);
    }
    DenseKC<T, 64> lb{(const T*)w1p, (long)K, N, K, 0};
    return launch_igemm<T, BM, 64, decltype(la), decltype(lb), decltype(e), 2>(la, lb, e, M, 64, cdiv(K, KT<T>::BK), 1, 1, st);
  });
  return 0;
}

}  // extern "C"
