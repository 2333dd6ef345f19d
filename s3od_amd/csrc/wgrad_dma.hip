// LDS-DMA 3x3 / stride-1 weight gradient for 64 x 64 channel blocks (the DPT RefineNet / ResidualConvUnit convs,
// reference src/s3od/model.py:223-226, 334-345): dW[co][tap][ci] += sum_p dy[p][co] x[p + tap - (1, 1)][ci].
// Its own translation unit: built WITHOUT -amdgpu-mfma-vgpr-form=1 (Makefile), so the 144 accumulators live in
// AGPRs and the 256 VGPRs hold the fragment bases, the DMA offsets and the operand fragments -- in the VGPR form
// the same loop spilled 44 VGPRs and ran ~140 VALU (AGPR copies) per 576 MFMAs, ~50 without.
#include "gemm.hpp"
#include <type_traits>
#include <utility>

// LDS-DMA form of the 64-channel-block halo wgrad (Cout block 64): the dy tile (256 px x 64) and the x halo
// (10 x 34 px x 64) of the NEXT tile land by buffer_load ... lds into the other half of a 2-deep ring while this
// tile's MFMAs run, so there is no register staging (PT x 4 VGPRs), no ds_write and one barrier per tile.  The
// DMA lanes pick the global 16-B chunk that the XOR swizzle (dy_at / hx_at) puts at their LDS position.
namespace wgd {
constexpr int DYB = 256 * 128, HXB = HT_PX * 128, PIECES = 76, PPW = PIECES / 4, BUF = PIECES * 1024, LDS = 2 * BUF;
static_assert(DYB % 1024 == 0 && DYB + HXB <= BUF && LDS <= 160 * 1024, "wgrad dma layout");
}  // namespace wgd
// Transposed 16 x 32 fragment (rows = K) at a precomputed per-lane LDS address (lo rows) + 2048 (hi rows, 16 rows on)
typedef __attribute__((address_space(3))) char lds_char;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
DEV bf16x8 trf_at(const lds_char* a) {
  typedef __attribute__((address_space(3))) s16x4 lds4;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)a);
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(a + 2048));
  bf16x4 x = __builtin_bit_cast(bf16x4, lo), y = __builtin_bit_cast(bf16x4, hi);
  return bf16x8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
}
// One 32-pixel row (K step TY) of a tile.  Wave w owns ci-block w and all 9 taps x 4 co-blocks, so the taps are
// compile-time constants and every fragment address is a per-lane base + an immediate: the dy fragment of co-block
// cb at fa[cb] + 4096 TY, the x-halo fragment of tap (dy, dx) at hb[r & 7] + 128 r with r = (TY + dy) 34 + dx
// (the XOR swizzle depends on the row only through r & 7).  (The runtime (tap, ci-block) split of the earlier version
// spent ~85 VALU on swizzled addresses per 36 MFMAs, at one wave per SIMD.)
template <bool RELU, int TY>
DEV void wgd_row(const lds_char* sb, const unsigned (&fa_b)[4], const unsigned (&hb)[8], f32x4 (&acc)[9][4]) {
  bf16x8 fa[4];
#pragma unroll
  for (int cb = 0; cb < 4; cb++) fa[cb] = trf_at(sb + fa_b[cb] + TY * HT_TW * 128);
#pragma unroll
  for (int tap = 0; tap < 9; tap++) {
    const int r = (TY + tap / 3) * HT_HC + tap % 3;
    bf16x8 fb = trf_at(sb + hb[r & 7] + r * 128);
    if constexpr (RELU) fb = __builtin_bit_cast(bf16x8, relu16<bf16>(__builtin_bit_cast(uint4, fb)));
#pragma unroll
    for (int cb = 0; cb < 4; cb++) acc[tap][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[cb], fb, acc[tap][cb], 0, 0, 0);
  }
}
static_assert(HT_TH == 8, "wgd rows");

template <bool RELU>
__global__ void __launch_bounds__(256, 1)
conv3x3_wgrad_dma_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x, float* __restrict__ ws, int H, int W,
                         int tiles_x, int tiles_y, int ntiles, int CinT, int CoT, int nci, int wpc) {
  using namespace wgd;
  constexpr int NCO = 4, NP = 9;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  // channel block of this workgroup and its contiguous tile range (as in the register-staged kernel; an XCD-grouped
  // order that runs the channel blocks of one tile behind one L2 measured the same)
  const int combo = blockIdx.x / wpc, wi = blockIdx.x - combo * wpc;
  const int t_beg = (int)((long)ntiles * wi / wpc), t_end = (int)((long)ntiles * (wi + 1) / wpc);
  const int co0 = (combo / nci) * 64, ci0 = (combo % nci) * 64;
  f32x4 acc[NP][NCO];                                    // [tap][co-block] of this wave's ci-block
#pragma unroll
  for (int i = 0; i < NP; i++)
#pragma unroll
    for (int j = 0; j < NCO; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // A ring slot = dy image [256 px][128 B] (pieces 0..31 of 1024 B) + halo image [340 px][128 B] (pieces 32..75, the
  // tail dummy).  Wave w DMAs dy pieces 8w .. 8w+7 and halo pieces 11w .. 11w+10.  A lane's 16-B slot (pixel row
  // 8 piece + l / 8, position l % 8) holds logical chunk (l % 8) ^ (l / 8) of its pixel (the XOR swizzle of
  // dy_at / hx_at; the row's low 3 bits are l / 8).  The launcher only takes this kernel when H % 8 == 0 and
  // W % 32 == 0, so dy pixels are always in the image: a dy piece's offset from the tile's dy origin is a per-lane
  // part (row l / 8, chunk) + a scalar part (tile row p / 4, column 8 (p % 4)).  Halo pieces keep one per-lane
  // offset each (halo rows are 34 pixels, not a multiple of 8) from the halo origin (row - 1, column - 1); halo pixels
  // outside the image (border tiles only) are masked to the out-of-range offset by a 4-bit per-piece code (row 0,
  // row 9, column 0, column 33), so the origin may lie before the image (the descriptor base moves with it; only
  // in-image lanes are ever in range).
  constexpr int DPW = DYB / 1024 / 4, HPW = PPW - DPW;   // 8 dy + 11 halo pieces per wave
  static_assert(DPW * 4 * 1024 == DYB && HPW * 4 * 8 >= HT_PX, "wgrad dma pieces");
  const int l8 = lane >> 3, ch = (lane & 7) ^ l8;
  const unsigned dlo = (unsigned)(l8 * CoT * 2 + ch * 16);
  unsigned hlo[HPW], hcode[2] = {0u, 0u};
#pragma unroll
  for (int j = 0; j < HPW; j++) {
    const int row = (wave * HPW + j) * 8 + l8, hy = row / HT_HC, hx = row - hy * HT_HC;
    hlo[j] = row < HT_PX ? (unsigned)(((hy * W + hx) * CinT) * 2 + ch * 16) : BUF_OOB;
    const unsigned code = (hy == 0 ? 1u : 0u) | (hy == HT_HR - 1 ? 2u : 0u) | (hx == 0 ? 4u : 0u) | (hx == HT_HC - 1 ? 8u : 0u);
    hcode[j / 8] |= code << (4 * (j % 8));
  }
  auto issue = [&](int tile, int slot) __attribute__((always_inline)) {
    const int txi = tile % tiles_x, t2 = tile / tiles_x, tyi = t2 % tiles_y, b = t2 / tiles_y;
    const int ty0 = tyi * HT_TH, tx0 = txi * HT_TW;
    const long img_d = (long)H * W * CoT, img_x = (long)H * W * CinT;
    const long od = ((long)ty0 * W + tx0) * CoT + co0, ox = ((long)(ty0 - 1) * W + tx0 - 1) * CinT + ci0;
    const auto rd = make_rsrc(dy + b * img_d + od, (unsigned long)(img_d - od) * 2);
    const auto rx = make_rsrc(x + b * img_x + ox, (unsigned long)(img_x - ox) * 2);
    char* dd = smem + slot * BUF + wave * DPW * 1024;
    char* hd = smem + slot * BUF + DYB + wave * HPW * 1024;
#pragma unroll
    for (int i = 0; i < DPW; i++) {
      const int p = wave * DPW + i;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rd, (lds_void*)(dd + i * 1024), 16, dlo, ((p >> 2) * W + 8 * (p & 3)) * CoT * 2, 0, 0);
    }
    const unsigned m = (ty0 == 0 ? 1u : 0u) | (ty0 + HT_TH == H ? 2u : 0u) | (tx0 == 0 ? 4u : 0u) | (tx0 + HT_TW == W ? 8u : 0u);
    if (m == 0) {                                        // interior tile (wave-uniform)
#pragma unroll
      for (int j = 0; j < HPW; j++) blds16(rx, hlo[j], hd + j * 1024);
    } else {
#pragma unroll
      for (int j = 0; j < HPW; j++)
        blds16(rx, ((hcode[j / 8] >> (4 * (j % 8))) & m) ? BUF_OOB : hlo[j], hd + j * 1024);
    }
  };
  // per-lane fragment bases (lane (g, l): u = 4 g + l / 4 its first K row, p = l % 4 its 4-column group), per ring slot
  const int u = 4 * (lane >> 4) + ((lane & 15) >> 2), pq = lane & 3;
  const lds_char* sb = (const lds_char*)smem;           // 32-bit LDS addresses (byte offsets from the ring base)
  unsigned fab[2][4], hxb[2][8];
#pragma unroll
  for (int sl = 0; sl < 2; sl++) {
#pragma unroll
    for (int cb = 0; cb < 4; cb++)
      fab[sl][cb] = sl * BUF + u * 128 + 16 * ((2 * cb + (pq >> 1)) ^ (u & 7)) + 8 * (pq & 1);
#pragma unroll
    for (int k = 0; k < 8; k++)
      hxb[sl][k] = sl * BUF + DYB + u * 128 + 16 * ((2 * wave + (pq >> 1)) ^ ((k + u) & 7)) + 8 * (pq & 1);
  }
  // the tile loop unrolled by the ring depth (2), so the slot is a compile-time index into the bases
  auto tile_step = [&](int tile, auto SLOT) __attribute__((always_inline)) {
    constexpr int slot = decltype(SLOT)::value;
    wait_vmcnt<0>();                                     // this tile's pieces (the only vector-memory ops in flight)
    __builtin_amdgcn_s_barrier();                        // ... of every wave; every wave done with the other slot
    asm volatile("" ::: "memory");
    if (tile + 1 < t_end) issue(tile + 1, slot ^ 1);
    wgd_row<RELU, 0>(sb, fab[slot], hxb[slot], acc); wgd_row<RELU, 1>(sb, fab[slot], hxb[slot], acc);
    wgd_row<RELU, 2>(sb, fab[slot], hxb[slot], acc); wgd_row<RELU, 3>(sb, fab[slot], hxb[slot], acc);
    wgd_row<RELU, 4>(sb, fab[slot], hxb[slot], acc); wgd_row<RELU, 5>(sb, fab[slot], hxb[slot], acc);
    wgd_row<RELU, 6>(sb, fab[slot], hxb[slot], acc); wgd_row<RELU, 7>(sb, fab[slot], hxb[slot], acc);
  };
  int tile = t_beg;
  if (tile < t_end) issue(tile, 0);
  for (; tile + 1 < t_end; tile += 2) {
    tile_step(tile, std::integral_constant<int, 0>{});
    tile_step(tile + 1, std::integral_constant<int, 1>{});
  }
  if (tile < t_end) tile_step(tile, std::integral_constant<int, 0>{});
  // flush: lane holds D[co = cb*16 + 4g + r][ci = 16 wave + li] of tap t -> ws[co][tap*Cin + ci]
  const int g = lane >> 4, li = lane & 15;
#pragma unroll
  for (int t = 0; t < NP; t++)
#pragma unroll
    for (int cb = 0; cb < NCO; cb++)
#pragma unroll
      for (int r = 0; r < 4; r++)
        if (co0 + cb * 16 + 4 * g + r < CoT)               // (CoT = 96: the second block's top half is padding)
          atomicAdd(ws + (long)(co0 + cb * 16 + 4 * g + r) * (9 * CinT) + t * CinT + ci0 + wave * 16 + li, acc[t][cb][r]);
}

// Producer-wave form: waves 0..3 compute exactly as above and never touch vector memory; NPROD more waves issue the
// 76 DMA pieces of the next tile (piece j by producer j % NPROD).  In the 4-wave kernel every compute wave issues
// 19 pieces at the top of each tile and stalls at issue once the memory queue is full (1.4 us of a 5.5 us tile at
// 1024^2, measured with wall_clock64 stamps), and compute alone (800 us) + DMA alone (786 us) ran in 1215 us together.
// The producers absorb the issue stalls; the compute waves only meet them at the one barrier per tile.  A second
// wave on a SIMD caps every wave at 256 registers (144 AGPR accumulators + <= 112 VGPRs).
template <bool RELU, int NPROD>
__global__ void __launch_bounds__(64 * (4 + NPROD), 1)
conv3x3_wgrad_dmap_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x, float* __restrict__ ws, int H, int W,
                          int tiles_x, int tiles_y, int ntiles, int CinT, int CoT, int nci, int wpc, int ymaj) {
  using namespace wgd;
  constexpr int NCO = 4, NP = 9, DP = DYB / 1024, HP = PIECES - DP;    // 32 dy + 44 halo pieces
  constexpr int DPP = DP / NPROD, HPP = HP / NPROD;                    // per producer
  static_assert(HP * 8 >= HT_PX && DP % NPROD == 0 && HP % NPROD == 0, "wgrad dma pieces");
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int combo = blockIdx.x / wpc, wi = blockIdx.x - combo * wpc;
  const int t_beg = (int)((long)ntiles * wi / wpc), t_end = (int)((long)ntiles * (wi + 1) / wpc);
  const int co0 = (combo / nci) * 64, ci0 = (combo % nci) * 64;
  if (wave >= 4) {
    // the piece layout of the 4-wave kernel; producer pw takes dy pieces pw + NPROD i and halo pieces pw + NPROD j
    const int pw = wave - 4;
    const int l8 = lane >> 3, ch = (lane & 7) ^ l8;
    const unsigned dlo = (unsigned)(l8 * CoT * 2 + ch * 16);
    unsigned hlo[HPP], hcode[(HPP + 7) / 8];
#pragma unroll
    for (int j = 0; j < (HPP + 7) / 8; j++) hcode[j] = 0u;
#pragma unroll
    for (int j = 0; j < HPP; j++) {
      const int row = (pw + NPROD * j) * 8 + l8, hy = row / HT_HC, hx = row - hy * HT_HC;
      hlo[j] = row < HT_PX ? (unsigned)(((hy * W + hx) * CinT) * 2 + ch * 16) : BUF_OOB;
      const unsigned code = (hy == 0 ? 1u : 0u) | (hy == HT_HR - 1 ? 2u : 0u) | (hx == 0 ? 4u : 0u) | (hx == HT_HC - 1 ? 8u : 0u);
      hcode[j / 8] |= code << (4 * (j % 8));
    }
    auto issue = [&](int tile, int slot) __attribute__((always_inline)) {
      // ymaj: a workgroup's consecutive tiles walk DOWN a column of tiles, so each halo shares its top 2 rows with the
      // previous tile's (read moments ago: L2) -- 8 of 10 halo rows per tile from HBM instead of 10
      int txi, tyi, b;
      if (ymaj) { tyi = tile % tiles_y; const int t2 = tile / tiles_y; txi = t2 % tiles_x; b = t2 / tiles_x; }
      else { txi = tile % tiles_x; const int t2 = tile / tiles_x; tyi = t2 % tiles_y; b = t2 / tiles_y; }
      const int ty0 = tyi * HT_TH, tx0 = txi * HT_TW;
      const long img_d = (long)H * W * CoT, img_x = (long)H * W * CinT;
      const long od = ((long)ty0 * W + tx0) * CoT + co0, ox = ((long)(ty0 - 1) * W + tx0 - 1) * CinT + ci0;
      const auto rd = make_rsrc(dy + b * img_d + od, (unsigned long)(img_d - od) * 2);
      const auto rx = make_rsrc(x + b * img_x + ox, (unsigned long)(img_x - ox) * 2);
      char* dd = smem + slot * BUF;
      char* hd = smem + slot * BUF + DYB;
      const unsigned m = (ty0 == 0 ? 1u : 0u) | (ty0 + HT_TH == H ? 2u : 0u) | (tx0 == 0 ? 4u : 0u) | (tx0 + HT_TW == W ? 8u : 0u);
      // halo pieces first: under a ReLU'd input the producers rectify the halo while the dy pieces still land
#pragma unroll
      for (int j = 0; j < HPP; j++)
        blds16(rx, ((hcode[j / 8] >> (4 * (j % 8))) & m) ? BUF_OOB : hlo[j], hd + (pw + NPROD * j) * 1024);
#pragma unroll
      for (int j = 0; j < DPP; j++) {
        const int p = pw + NPROD * j;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rd, (lds_void*)(dd + p * 1024), 16, dlo, ((p >> 2) * W + 8 * (p & 3)) * CoT * 2, 0, 0);
      }
    };
    if (t_beg < t_end) issue(t_beg, 0);
    for (int tile = t_beg, k = 0; tile < t_end; tile++, k++) {
      if (RELU) {
        wait_vmcnt<DPP>();                               // the halo pieces landed (the dy pieces are the younger DPP)
        // ReLU'd input: the producers rectify the landed halo in place (the compute waves read it unchanged; a
        // v_pk_max per fragment read there cost 384 VALU per 576 MFMAs and spilled)
        // every 16-B chunk of the slot's halo region, dummy tail included (HP KiB = NPROD x 64 lanes x NIT chunks),
        // in inline asm: compiled LDS accesses here get a conservative vmcnt(0) in front (the dy DMA still in flight
        // may alias for the compiler) and an lgkmcnt(0) each, which serialised the pass
        constexpr int STEP = 64 * NPROD, NIT = HP * 64 / STEP;
        static_assert(NIT * STEP == HP * 64 && NIT * STEP * 16 <= 65536, "relu pass layout");
        const unsigned a0 = (unsigned)(size_t)(const lds_char*)(smem + (k & 1) * BUF + DYB) + (pw * 64 + lane) * 16;
        u32x4 v[NIT];
#pragma unroll
        for (int i = 0; i < NIT; i++) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v[i]) : "v"(a0), "n"(i * STEP * 16));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < NIT; i++)
#pragma unroll
          for (int e = 0; e < 4; e++) asm volatile("v_pk_max_i16 %0, %0, 0" : "+v"(v[i][e]));
#pragma unroll
        for (int i = 0; i < NIT; i++) asm volatile("ds_write_b128 %0, %1 offset:%2" :: "v"(a0), "v"(v[i]), "n"(i * STEP * 16) : "memory");
        wait_lgkm0();                                    // the stores are in LDS before the barrier
      }
      wait_vmcnt<0>();                                   // tile's pieces landed
      __builtin_amdgcn_s_barrier();                      // pairs with the compute waves' barrier of this tile
      asm volatile("" ::: "memory");
      if (tile + 1 < t_end) issue(tile + 1, (k + 1) & 1);
    }
    return;
  }
  f32x4 acc[NP][NCO];
#pragma unroll
  for (int i = 0; i < NP; i++)
#pragma unroll
    for (int j = 0; j < NCO; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int u = 4 * (lane >> 4) + ((lane & 15) >> 2), pq = lane & 3;
  const lds_char* sb = (const lds_char*)smem;
  unsigned fab[2][4], hxb[2][8];
#pragma unroll
  for (int sl = 0; sl < 2; sl++) {
#pragma unroll
    for (int cb = 0; cb < 4; cb++)
      fab[sl][cb] = sl * BUF + u * 128 + 16 * ((2 * cb + (pq >> 1)) ^ (u & 7)) + 8 * (pq & 1);
#pragma unroll
    for (int k = 0; k < 8; k++)
      hxb[sl][k] = sl * BUF + DYB + u * 128 + 16 * ((2 * wave + (pq >> 1)) ^ ((k + u) & 7)) + 8 * (pq & 1);
  }
  // A compiler memory clobber every second row: the two rows of a pair share their halo reads, but fragments are not
  // kept live across pairs (all-rows reuse needs ~30 live halo fragments: > 112 VGPRs; per-row clobbers: 1062 vs 1000 us
  // for pairs, opaque per-row bases 1108 us -- v_mov / v_add per fragment -- at 1024^2, same process)
  auto tile_step = [&](auto SLOT) __attribute__((always_inline)) {
    constexpr int slot = decltype(SLOT)::value;
    __syncthreads();                                     // LDS reads of the previous tile done; this tile's data landed
    asm volatile("" ::: "memory");
    wgd_row<false, 0>(sb, fab[slot], hxb[slot], acc); wgd_row<false, 1>(sb, fab[slot], hxb[slot], acc);
    asm volatile("" ::: "memory");
    wgd_row<false, 2>(sb, fab[slot], hxb[slot], acc); wgd_row<false, 3>(sb, fab[slot], hxb[slot], acc);
    asm volatile("" ::: "memory");
    wgd_row<false, 4>(sb, fab[slot], hxb[slot], acc); wgd_row<false, 5>(sb, fab[slot], hxb[slot], acc);
    asm volatile("" ::: "memory");
    wgd_row<false, 6>(sb, fab[slot], hxb[slot], acc); wgd_row<false, 7>(sb, fab[slot], hxb[slot], acc);
  };
  int tile = t_beg;
  for (; tile + 1 < t_end; tile += 2) {
    tile_step(std::integral_constant<int, 0>{});
    tile_step(std::integral_constant<int, 1>{});
  }
  if (tile < t_end) tile_step(std::integral_constant<int, 0>{});
  const int g = lane >> 4, li = lane & 15;
#pragma unroll
  for (int t = 0; t < NP; t++)
#pragma unroll
    for (int cb = 0; cb < NCO; cb++)
#pragma unroll
      for (int r = 0; r < 4; r++)
        if (co0 + cb * 16 + 4 * g + r < CoT)               // (CoT = 96: the second block's top half is padding)
          atomicAdd(ws + (long)(co0 + cb * 16 + 4 * g + r) * (9 * CinT) + t * CinT + ci0 + wave * 16 + li, acc[t][cb][r]);
}

// S3OD_WGD_PROD=0 (under S3OD_AB=1: per call) keeps the 4-wave kernel
template <bool RELU>
static int launch_wgrad_dma(const bf16* dy, const bf16* x, float* ws, int B, int H, int W, int CinT, int CoT, hipStream_t st) {
  const bool prod = S3OD_KNOB("S3OD_WGD_PROD", 1) != 0;
  const int np = S3OD_KNOB("S3OD_WGD_NPROD", 2);
  auto kp = np == 4 ? conv3x3_wgrad_dmap_kernel<RELU, 4> : np == 2 ? conv3x3_wgrad_dmap_kernel<RELU, 2> : conv3x3_wgrad_dmap_kernel<RELU, 1>;
  static const bool attr = ((void)hipFuncSetAttribute((const void*)conv3x3_wgrad_dma_kernel<RELU>, hipFuncAttributeMaxDynamicSharedMemorySize, wgd::LDS),
                            (void)hipFuncSetAttribute((const void*)conv3x3_wgrad_dmap_kernel<RELU, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, wgd::LDS),
                            (void)hipFuncSetAttribute((const void*)conv3x3_wgrad_dmap_kernel<RELU, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, wgd::LDS),
                            (void)hipFuncSetAttribute((const void*)conv3x3_wgrad_dmap_kernel<RELU, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, wgd::LDS),
                            true);   // once per process (thread-safe static init)
  (void)attr;
  const int tx = cdiv(W, HT_TW), ty = cdiv(H, HT_TH);
  const long tiles = (long)B * tx * ty;
  const int nci = CinT / 64, nblk = cdiv(CoT, 64) * nci;
  const int wpc = (int)std::max<long>(1, std::min<long>(tiles, std::max(1, s3od_cu_count() / nblk)));
  if (prod)
    hipLaunchKernelGGL(kp, dim3(nblk * wpc), dim3(64 * (4 + (np == 4 || np == 2 ? np : 1))), wgd::LDS, st, dy, x, ws, H, W, tx, ty, (int)tiles,
                       CinT, CoT, nci, wpc, S3OD_KNOB("S3OD_WGD_YMAJ", 1));
  else
    hipLaunchKernelGGL(conv3x3_wgrad_dma_kernel<RELU>, dim3(nblk * wpc), dim3(256), wgd::LDS, st, dy, x, ws, H, W, tx, ty, (int)tiles, CinT, CoT, nci, wpc);
  return s3od_check_launch("conv3x3_wgrad_dma");
}

int wgrad3x3_dma_launch(bool relu_x, const bf16* dy, const bf16* x, float* ws, int B, int H, int W, int CinT, int CoT,
                        hipStream_t st) {
  return relu_x ? launch_wgrad_dma<true>(dy, x, ws, B, H, W, CinT, CoT, st) : launch_wgrad_dma<false>(dy, x, ws, B, H, W, CinT, CoT, st);
}
