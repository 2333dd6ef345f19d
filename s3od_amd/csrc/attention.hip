// Flash attention for DINOv3 ViT-B/16 (12 heads x d=64, non-causal, no mask), gfx950.
// Reference semantics: SDPA softmax(q k^T / 8) v (tf:integrations/sdpa_attention.py:79-166,
// tf:models/dinov3_vit/modeling_dinov3_vit.py:294-334).
// Conventions (base-2 domain): q arrives pre-scaled by log2(e)/8 (S3OD_QSCALE, applied in the QKV
// epilogue), so q.k is the score in log2 units; LSE is stored in log2 units (lse2 = m + log2 l).
//
// Forward: one workgroup = 4 waves = 128 query rows of one (b, h); each wave owns 32 queries.
// "Swapped" products keep the softmax row lane-local:
//   S^T[key][q] = K . Q^T       (A = K tile from LDS, B = Q fragments held in registers)
//   O^T[d][q]  += V^T . P^T     (A = V^T via ds_read_b64_tr_b16, B = P^T straight from the
//                                S^T accumulator registers; the K-order of the MFMA is permuted
//                                identically on both operands, so no shuffles / LDS round trip)
// The loop is VALU-issue bound on CDNA4 (an MFMA 16x16x32 leaves room for ~2 VALU ops), so the
// bf16 path spends as little VALU per score as possible:
//   * the running row max m is folded into the S accumulator's C operand (C = -m), so
//     P = exp2(acc) is ONE v_exp per score;
//   * lazy rescaling: m only moves when some score exceeds it by > 2^8 (wave-uniform branch);
//   * the row sum l comes out of the matrix core: l += 1^T P^T (one extra MFMA per 32 keys).
// K/V tiles of 64 keys are register-staged into double-buffered LDS (one barrier per tile).
// T=float runs the exact online softmax on v_mfma_f32_16x16x4_f32 (strict-parity path).
#include "common.hpp"
#include <type_traits>

#define DISPATCH_T(dtype, ...)                                                  \
  do {                                                                          \
    if ((dtype) == S3OD_BF16) { typedef bf16 T; __VA_ARGS__ }                   \
    else if ((dtype) == S3OD_F32) { typedef float T; __VA_ARGS__ }              \
    else { s3od_set_error("bad dtype %d", (int)(dtype)); return 22; }           \
  } while (0)

namespace {
constexpr float LN2 = 0.6931471805599453f;
constexpr float RESCALE_TH = 8.f;       // lazy-rescale threshold (log2 units): P <= 2^8 between rescales

DEV float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }   // bare v_exp_f32 (no denormal fix-up)

// LDS images of a 64-key x 64-d tile.  bf16: 128-B rows, 32-B slots XOR (key>>1)&3 (tr reads),
// 16-B slots XOR ((key>>1)&7) for row (ds_read_b128) reads.  f32: 256-B rows + 16-B pad.
template <typename T> struct TileL;
template <> struct TileL<bf16> {
  static constexpr int BYTES = 64 * 128;
  DEV static int krow(int key, int byte) { return key * 128 + ((((byte >> 4) ^ ((key >> 1) & 7)) << 4) | (byte & 15)); }
  DEV static int vrow(int key, int byte) { return key * 128 + ((((byte >> 5) ^ ((key >> 1) & 3)) << 5) | (byte & 31)); }
};
template <> struct TileL<float> {
  static constexpr int BYTES = 64 * 272;
  DEV static int krow(int key, int byte) { return key * 272 + byte; }
  DEV static int vrow(int key, int byte) { return key * 272 + byte; }
};

typedef __attribute__((address_space(3))) void lds_void;
DEV __amdgpu_buffer_rsrc_t attn_rsrc(const void* p, unsigned long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(unsigned)bytes, 0x00020000);
}

template <typename T> struct Stage {
  static constexpr int CH = 64 * 64 * sizeof(T) / 16 / 256;   // 16-B chunks per thread per tile
  uint4 k[CH], v[CH];
  DEV void load(const T* K, const T* V, int key0, int N, int tid) {
    constexpr int CPR = 64 * sizeof(T) / 16;
    if (key0 + 64 <= N) {             // whole tile in range (uniform): no per-key selects
#pragma unroll
      for (int i = 0; i < CH; i++) {
        const int c = tid + 256 * i;
        const long o = (long)(key0 + c / CPR) * 64 + (c % CPR) * (16 / sizeof(T));
        k[i] = *(const uint4*)(K + o);
        v[i] = *(const uint4*)(V + o);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < CH; i++) {
      int c = tid + 256 * i;
      int key = key0 + c / CPR, col = (c % CPR) * (16 / sizeof(T));
      bool ok = key < N;
      k[i] = ok ? *(const uint4*)(K + (long)key * 64 + col) : make_uint4(0, 0, 0, 0);
      v[i] = ok ? *(const uint4*)(V + (long)key * 64 + col) : make_uint4(0, 0, 0, 0);
    }
  }
  // bf16: the same chunks by buffer loads -- per-thread byte offsets fixed, the tile's key offset on the scalar unit,
  // keys >= N read zeros by the range check: no per-tile address or select VALU (the global-pointer form spent ~80
  // VALU per tile on 64-bit addresses and tail selects beside 36 MFMAs)
  DEV void load_buf(__amdgpu_buffer_rsrc_t rk, __amdgpu_buffer_rsrc_t rv, const unsigned (&vo)[CH], int key0) {
    const int so = key0 * 64 * (int)sizeof(T);
#pragma unroll
    for (int i = 0; i < CH; i++) {
      k[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rk, vo[i], so, 0));
      v[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rv, vo[i], so, 0));
    }
  }
  DEV static unsigned chunk_off(int tid, int i) {
    constexpr int CPR = 64 * sizeof(T) / 16;
    const int c = tid + 256 * i;
    return (unsigned)((c / CPR) * 64 * sizeof(T) + (c % CPR) * 16);
  }
  DEV void store(char* ks, char* vs, int tid) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      int c = tid + 256 * i;
      constexpr int CPR = 64 * sizeof(T) / 16;
      int key = c / CPR, byte = (c % CPR) * 16;
      *(uint4*)(ks + TileL<T>::krow(key, byte)) = k[i];
      *(uint4*)(vs + TileL<T>::vrow(key, byte)) = v[i];
    }
  }
};

DEV float max16(const f32x4* s) {   // max over 4 accumulators (16 values)
  float a = fmaxf(fmaxf(s[0][0], s[0][1]), s[0][2]);
  a = fmaxf(fmaxf(a, s[0][3]), s[1][0]); a = fmaxf(fmaxf(a, s[1][1]), s[1][2]);
  a = fmaxf(fmaxf(a, s[1][3]), s[2][0]); a = fmaxf(fmaxf(a, s[2][1]), s[2][2]);
  a = fmaxf(fmaxf(a, s[2][3]), s[3][0]); a = fmaxf(fmaxf(a, s[3][1]), s[3][2]);
  return fmaxf(a, s[3][3]);
}
DEV float xmax4(float v) { v = fmaxf(v, __shfl_xor(v, 16)); return fmaxf(v, __shfl_xor(v, 32)); }
DEV float xsum4(float v) { v += __shfl_xor(v, 16); return v + __shfl_xor(v, 32); }
}  // namespace

// DMA (bf16): K / V tiles by LDS-DMA (buffer_load ... lds, 4 x 1 KiB pieces per wave and tile, the image swizzle
// applied to each lane's source chunk) instead of buffer loads into registers + ds_write: no staging registers and no
// LDS store instructions in the loop; the next tile's pieces land during the current tile (vmcnt(0) + the barrier)
template <typename T, bool DMA = false>
__global__ void __launch_bounds__(256, 3) attn_fwd_kernel(const T* __restrict__ Q, const T* __restrict__ K, const T* __restrict__ V,
                                                        T* __restrict__ O, float* __restrict__ LSE, int N, int H, int fast) {
  constexpr bool F32 = std::is_same<T, float>::value;
  static_assert(!DMA || !F32, "attn_fwd: LDS-DMA staging is the bf16 path");
  typedef TileL<T> L;
  // DMA: the second K / V stage is its own array -- a distinct object, so alias analysis can tell this tile's LDS
  // reads from the next tile's DMA without relying on offsets (with one array it waited vmcnt(0) before the V^T reads
  // of every other tile)
  __shared__ __attribute__((aligned(DMA ? 1024 : 16))) char smem[(DMA ? 2 : 4) * L::BYTES];
  __shared__ __attribute__((aligned(DMA ? 1024 : 16))) char smem1[DMA ? 2 * L::BYTES : 16];
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, li = lane & 15;
  const T* Qp = Q + (long)bh * N * 64;
  const T* Kp = K + (long)bh * N * 64;
  const T* Vp = V + (long)bh * N * 64;
  const int q0 = blockIdx.x * 128 + wave * 32;
  const bool active = q0 < N;        // wave-uniform

  // Q fragments (B operand of S^T = K Q^T): lane holds Q[q0 + qs*16 + li][d-slice of group g]
  constexpr int QK = F32 ? 16 : 2;     // k-steps over d=64
  typedef typename std::conditional<F32, float, bf16x8>::type qfrag;
  qfrag qf[2][QK];
#pragma unroll
  for (int qs = 0; qs < 2; qs++) {
    int q = q0 + qs * 16 + li;
#pragma unroll
    for (int kk = 0; kk < QK; kk++) {
      if constexpr (F32) qf[qs][kk] = q < N ? Qp[(long)q * 64 + kk * 4 + g] : 0.f;
      else {
        if (q < N) qf[qs][kk] = *(const bf16x8*)(Qp + (long)q * 64 + kk * 32 + 8 * g);
        else { bf16x8 z; for (int e = 0; e < 8; e++) z[e] = (bf16)0.f; qf[qs][kk] = z; }
      }
    }
  }
  f32x4 o[4][2];
  // running max m (log2 units); bf16: C operand -m of the S MFMA, row sums in lacc (MFMA)
  float mrow[2], lrow[2];
  f32x4 negm[2], lacc[2];
  // FAST (bf16): the max is taken over the first key tile only and never moved again -- P = exp2(s - m0) has the
  // floating-point range of bf16 / fp32, so no per-tile max / threshold VALU is needed (one v_exp + the packing per
  // score).  A score more than ~120 log2 units above m0 would overflow: the row sum then comes out non-finite and the
  // workgroup reruns its block with the lazy-rescale loop (FAST = false) before the epilogue.  l >= 1 always (the
  // maximum of tile 0 contributes exp2(0)), so nothing underflows.
  auto run = [&](auto FASTc) {
  constexpr bool FAST = decltype(FASTc)::value;
#pragma unroll
  for (int i = 0; i < 4; i++) { o[i][0] = f32x4{0, 0, 0, 0}; o[i][1] = f32x4{0, 0, 0, 0}; }
  mrow[0] = mrow[1] = -INFINITY; lrow[0] = lrow[1] = 0.f;
  negm[0] = negm[1] = f32x4{0, 0, 0, 0};
  lacc[0] = lacc[1] = f32x4{0, 0, 0, 0};

  if constexpr (DMA) {
  const int nkt = (N + 63) / 64;
  // the per-tile work on the staged K / V images ks, vs (both staging forms)
  auto tile_compute = [&](int kt, const char* ks, const char* vs) {
    // a wave whose 32 queries are all >= N (the partial last block: N = 4096 + 5 prefix tokens) only helps stage K / V
    if (active) {
    // ---- S^T = K Q^T (- m) : acc[kb][qs], element i: key = kb*16 + 4g + i, query = qs*16 + li
    f32x4 s[4][2];
#pragma unroll
    for (int kb = 0; kb < 4; kb++) {
      if constexpr (F32) {
        s[kb][0] = f32x4{0, 0, 0, 0}; s[kb][1] = f32x4{0, 0, 0, 0};
#pragma unroll
        for (int kk = 0; kk < QK; kk++) {
          float a = *(const float*)(ks + L::krow(kb * 16 + li, (kk * 4 + g) * 4));
          s[kb][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, qf[0][kk], s[kb][0], 0, 0, 0);
          s[kb][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, qf[1][kk], s[kb][1], 0, 0, 0);
        }
      } else {
        bf16x8 a0 = *(const bf16x8*)(ks + L::krow(kb * 16 + li, g * 16));
        bf16x8 a1 = *(const bf16x8*)(ks + L::krow(kb * 16 + li, 64 + g * 16));
        s[kb][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, qf[0][0], negm[0], 0, 0, 0);
        s[kb][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, qf[1][0], negm[1], 0, 0, 0);
        s[kb][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, qf[0][1], s[kb][0], 0, 0, 0);
        s[kb][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, qf[1][1], s[kb][1], 0, 0, 0);
      }
    }
    // ---- mask keys >= N (last tile only)
    if (kt * 64 + 64 > N) {
#pragma unroll
      for (int kb = 0; kb < 4; kb++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
          int key = kt * 64 + kb * 16 + 4 * g + i;
          if (key >= N) { s[kb][0][i] = -INFINITY; s[kb][1][i] = -INFINITY; }
        }
    }
    if constexpr (F32) {
      // ---- exact online softmax per query column
#pragma unroll
      for (int qs = 0; qs < 2; qs++) {
        f32x4 col[4] = {s[0][qs], s[1][qs], s[2][qs], s[3][qs]};
        float mx = xmax4(max16(col));
        float mnew = fmaxf(mrow[qs], mx);
        float alpha = fexp2(mrow[qs] - mnew);
        float sum = 0.f;
#pragma unroll
        for (int kb = 0; kb < 4; kb++)
#pragma unroll
          for (int i = 0; i < 4; i++) { float p = fexp2(s[kb][qs][i] - mnew); s[kb][qs][i] = p; sum += p; }
        lrow[qs] = lrow[qs] * alpha + xsum4(sum);
        mrow[qs] = mnew;
#pragma unroll
        for (int ds = 0; ds < 4; ds++) o[ds][qs] *= alpha;
      }
#pragma unroll
      for (int kb = 0; kb < 4; kb++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
          int key = kb * 16 + 4 * g + i;
#pragma unroll
          for (int ds = 0; ds < 4; ds++) {
            float a = *(const float*)(vs + L::vrow(key, (ds * 16 + li) * 4));
            o[ds][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, s[kb][0][i], o[ds][0], 0, 0, 0);
            o[ds][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, s[kb][1][i], o[ds][1], 0, 0, 0);
          }
        }
    } else {
      // ---- lazy max: s already holds score - m.  The first tile sets m exactly; later tiles only
      // rescale when a score exceeds m by more than RESCALE_TH (wave-uniform branch).
      float lm0 = 0.f, lm1 = 0.f;
      if (!FAST || kt == 0) {
        f32x4 c0[4] = {s[0][0], s[1][0], s[2][0], s[3][0]}, c1[4] = {s[0][1], s[1][1], s[2][1], s[3][1]};
        lm0 = max16(c0); lm1 = max16(c1);
      }
      if (kt == 0 || (!FAST && __any(fmaxf(lm0, lm1) > RESCALE_TH))) {
        float lmq[2] = {lm0, lm1};
#pragma unroll
        for (int qs = 0; qs < 2; qs++) {
          float d = xmax4(lmq[qs]);
          d = kt == 0 ? d : fmaxf(d, 0.f);
          mrow[qs] = kt == 0 ? d : mrow[qs] + d;
          float alpha = kt == 0 ? 1.f : fexp2(-d);
#pragma unroll
          for (int kb = 0; kb < 4; kb++) s[kb][qs] -= d;
#pragma unroll
          for (int ds = 0; ds < 4; ds++) o[ds][qs] *= alpha;
          lacc[qs] *= alpha;
          negm[qs] = f32x4{-mrow[qs], -mrow[qs], -mrow[qs], -mrow[qs]};
        }
      }
      // ---- P = exp2(s); O^T += V^T P^T ; l += 1^T P^T
      typedef __attribute__((address_space(3))) s16x4 lds_s4;
      bf16x8 ones;
#pragma unroll
      for (int e = 0; e < 8; e++) ones[e] = (bf16)1.f;
#pragma unroll
      for (int kst = 0; kst < 2; kst++) {
        bf16x8 pb[2];
#pragma unroll
        for (int qs = 0; qs < 2; qs++)
#pragma unroll
          for (int i = 0; i < 4; i++) {
            pb[qs][i] = (bf16)fexp2(s[2 * kst][qs][i]);
            pb[qs][4 + i] = (bf16)fexp2(s[2 * kst + 1][qs][i]);
          }
        const int q = li >> 2, p = li & 3;
#pragma unroll
        for (int ds = 0; ds < 4; ds++) {
          int byte = (ds * 16 + 4 * p) * 2;
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(vs + L::vrow(32 * kst + 4 * g + q, byte)));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(vs + L::vrow(32 * kst + 16 + 4 * g + q, byte)));
          bf16x4 a0 = __builtin_bit_cast(bf16x4, lo), a1 = __builtin_bit_cast(bf16x4, hi);
          bf16x8 a = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
          o[ds][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pb[0], o[ds][0], 0, 0, 0);
          o[ds][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pb[1], o[ds][1], 0, 0, 0);
        }
        lacc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pb[0], lacc[0], 0, 0, 0);
        lacc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pb[1], lacc[1], 0, 0, 0);
      }
    }
    }
  };
    // piece p = 4 wave + i of a tile: K pieces 0..7 (waves 0, 1), V pieces 8..15 (waves 2, 3); piece p & 7 holds keys
    // 8 (p & 7) .. +7, lane l writes physical 16-B chunk l & 7 of key 8 (p & 7) + (l >> 3), i.e. the logical chunk the
    // TileL swizzle puts there (K: 16-B chunks XOR (key >> 1) & 7; V: 32-B slots XOR (key >> 1) & 3)
    const int wv = __builtin_amdgcn_readfirstlane(wave);     // wave-uniform: the descriptor and M0 stay scalar
    unsigned dvo[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int pp = (wv & 1) * 4 + i, key = 8 * pp + (lane >> 3), c = lane & 7;
      const int lc = wv < 2 ? (c ^ ((key >> 1) & 7)) : ((((c >> 1) ^ ((key >> 1) & 3)) << 1) | (c & 1));
      dvo[i] = (unsigned)(key * 128 + lc * 16);
    }
    const char* src = (const char*)(wv < 2 ? Kp : Vp);
    const int dsto = (wv < 2 ? 0 : L::BYTES) + (wv & 1) * 4096;
    auto dma = [&](int kt, char* stage) {
      // the descriptor rebased on the tile's first key (scalar work): keys >= N read zeros by the range check
      const long off = (long)kt * 64 * 128;
      const auto r = attn_rsrc(src + off, (unsigned long)N * 128 - off);
#pragma unroll
      for (int i = 0; i < 4; i++)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)(stage + dsto + i * 1024), 16, dvo[i], 0, 0, 0);
    };
    dma(0, smem);
    vm_drain();
    __syncthreads();
    // unrolled by two so the stages are compile-time offsets; __restrict__ stage pointers let the wait-count pass see
    // that this tile's LDS reads cannot alias the next tile's DMA (as in the backward kernels)
    auto tile = [&](int kt, char* __restrict__ nxt, const char* __restrict__ cs) {
      if (kt + 1 < nkt) dma(kt + 1, nxt);
      tile_compute(kt, cs, cs + L::BYTES);
      vm_drain();           // this wave's pieces of the next tile landed ...
      __syncthreads();      // ... and every wave's; every wave done with this stage
    };
    int kt = 0;
    for (; kt + 1 < nkt; kt += 2) { tile(kt, smem1, smem); tile(kt + 1, smem, smem1); }
    if (kt < nkt) tile(kt, smem1, smem);
  } else {
  Stage<T> stg;
  const int nkt = (N + 63) / 64;
  const auto rk = attn_rsrc(Kp, (unsigned long)N * 64 * sizeof(T)), rv = attn_rsrc(Vp, (unsigned long)N * 64 * sizeof(T));
  unsigned vo[Stage<T>::CH];
#pragma unroll
  for (int i = 0; i < Stage<T>::CH; i++) vo[i] = Stage<T>::chunk_off(tid, i);
  auto stage_load = [&](int key0) {
    if constexpr (F32) stg.load(Kp, Vp, key0, N, tid);
    else stg.load_buf(rk, rv, vo, key0);
  };
  stage_load(0);
  stg.store(smem, smem + L::BYTES, tid);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nkt; kt++) {
    const bool more = kt + 1 < nkt;
    if (more) stage_load((kt + 1) * 64);
    const char* ks = smem + cur * 2 * L::BYTES;
    const char* vs = ks + L::BYTES;
    // a wave whose 32 queries are all >= N (the partial last block: N = 4096 + 5 prefix tokens) only helps stage K / V
    if (active) {
    // ---- S^T = K Q^T (- m) : acc[kb][qs], element i: key = kb*16 + 4g + i, query = qs*16 + li
    f32x4 s[4][2];
#pragma unroll
    for (int kb = 0; kb < 4; kb++) {
      if constexpr (F32) {
        s[kb][0] = f32x4{0, 0, 0, 0}; s[kb][1] = f32x4{0, 0, 0, 0};
#pragma unroll
        for (int kk = 0; kk < QK; kk++) {
          float a = *(const float*)(ks + L::krow(kb * 16 + li, (kk * 4 + g) * 4));
          s[kb][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, qf[0][kk], s[kb][0], 0, 0, 0);
          s[kb][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, qf[1][kk], s[kb][1], 0, 0, 0);
        }
      } else {
        bf16x8 a0 = *(const bf16x8*)(ks + L::krow(kb * 16 + li, g * 16));
        bf16x8 a1 = *(const bf16x8*)(ks + L::krow(kb * 16 + li, 64 + g * 16));
        s[kb][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, qf[0][0], negm[0], 0, 0, 0);
        s[kb][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, qf[1][0], negm[1], 0, 0, 0);
        s[kb][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, qf[0][1], s[kb][0], 0, 0, 0);
        s[kb][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, qf[1][1], s[kb][1], 0, 0, 0);
      }
    }
    // ---- mask keys >= N (last tile only)
    if (kt * 64 + 64 > N) {
#pragma unroll
      for (int kb = 0; kb < 4; kb++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
          int key = kt * 64 + kb * 16 + 4 * g + i;
          if (key >= N) { s[kb][0][i] = -INFINITY; s[kb][1][i] = -INFINITY; }
        }
    }
    if constexpr (F32) {
      // ---- exact online softmax per query column
#pragma unroll
      for (int qs = 0; qs < 2; qs++) {
        f32x4 col[4] = {s[0][qs], s[1][qs], s[2][qs], s[3][qs]};
        float mx = xmax4(max16(col));
        float mnew = fmaxf(mrow[qs], mx);
        float alpha = fexp2(mrow[qs] - mnew);
        float sum = 0.f;
#pragma unroll
        for (int kb = 0; kb < 4; kb++)
#pragma unroll
          for (int i = 0; i < 4; i++) { float p = fexp2(s[kb][qs][i] - mnew); s[kb][qs][i] = p; sum += p; }
        lrow[qs] = lrow[qs] * alpha + xsum4(sum);
        mrow[qs] = mnew;
#pragma unroll
        for (int ds = 0; ds < 4; ds++) o[ds][qs] *= alpha;
      }
#pragma unroll
      for (int kb = 0; kb < 4; kb++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
          int key = kb * 16 + 4 * g + i;
#pragma unroll
          for (int ds = 0; ds < 4; ds++) {
            float a = *(const float*)(vs + L::vrow(key, (ds * 16 + li) * 4));
            o[ds][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, s[kb][0][i], o[ds][0], 0, 0, 0);
            o[ds][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, s[kb][1][i], o[ds][1], 0, 0, 0);
          }
        }
    } else {
      // ---- lazy max: s already holds score - m.  The first tile sets m exactly; later tiles only
      // rescale when a score exceeds m by more than RESCALE_TH (wave-uniform branch).
      float lm0 = 0.f, lm1 = 0.f;
      if (!FAST || kt == 0) {
        f32x4 c0[4] = {s[0][0], s[1][0], s[2][0], s[3][0]}, c1[4] = {s[0][1], s[1][1], s[2][1], s[3][1]};
        lm0 = max16(c0); lm1 = max16(c1);
      }
      if (kt == 0 || (!FAST && __any(fmaxf(lm0, lm1) > RESCALE_TH))) {
        float lmq[2] = {lm0, lm1};
#pragma unroll
        for (int qs = 0; qs < 2; qs++) {
          float d = xmax4(lmq[qs]);
          d = kt == 0 ? d : fmaxf(d, 0.f);
          mrow[qs] = kt == 0 ? d : mrow[qs] + d;
          float alpha = kt == 0 ? 1.f : fexp2(-d);
#pragma unroll
          for (int kb = 0; kb < 4; kb++) s[kb][qs] -= d;
#pragma unroll
          for (int ds = 0; ds < 4; ds++) o[ds][qs] *= alpha;
          lacc[qs] *= alpha;
          negm[qs] = f32x4{-mrow[qs], -mrow[qs], -mrow[qs], -mrow[qs]};
        }
      }
      // ---- P = exp2(s); O^T += V^T P^T ; l += 1^T P^T
      typedef __attribute__((address_space(3))) s16x4 lds_s4;
      bf16x8 ones;
#pragma unroll
      for (int e = 0; e < 8; e++) ones[e] = (bf16)1.f;
#pragma unroll
      for (int kst = 0; kst < 2; kst++) {
        bf16x8 pb[2];
#pragma unroll
        for (int qs = 0; qs < 2; qs++)
#pragma unroll
          for (int i = 0; i < 4; i++) {
            pb[qs][i] = (bf16)fexp2(s[2 * kst][qs][i]);
            pb[qs][4 + i] = (bf16)fexp2(s[2 * kst + 1][qs][i]);
          }
        const int q = li >> 2, p = li & 3;
#pragma unroll
        for (int ds = 0; ds < 4; ds++) {
          int byte = (ds * 16 + 4 * p) * 2;
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(vs + L::vrow(32 * kst + 4 * g + q, byte)));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(vs + L::vrow(32 * kst + 16 + 4 * g + q, byte)));
          bf16x4 a0 = __builtin_bit_cast(bf16x4, lo), a1 = __builtin_bit_cast(bf16x4, hi);
          bf16x8 a = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
          o[ds][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pb[0], o[ds][0], 0, 0, 0);
          o[ds][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pb[1], o[ds][1], 0, 0, 0);
        }
        lacc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pb[0], lacc[0], 0, 0, 0);
        lacc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pb[1], lacc[1], 0, 0, 0);
      }
    }
    }
    if (more) stg.store(smem + (cur ^ 1) * 2 * L::BYTES, smem + (cur ^ 1) * 2 * L::BYTES + L::BYTES, tid);
    __syncthreads();
    cur ^= 1;
  }
  }
  };
  if constexpr (!F32) {
    if (fast) {
      run(std::true_type{});
      // the rare overflow of the fixed-max path: rerun the block with the lazy rescale.  O overflows first when
      // |V| > 1 (l just under FLT_MAX times |v| > FLT_MAX), so the accumulators are checked too (once per block).
      bool bad = !(lacc[0][0] < 3.0e38f) || !(lacc[1][0] < 3.0e38f);
#pragma unroll
      for (int ds = 0; ds < 4; ds++)
#pragma unroll
        for (int qs = 0; qs < 2; qs++)
#pragma unroll
          for (int i = 0; i < 4; i++) bad |= !(fabsf(o[ds][qs][i]) < 3.0e38f);
      if (__syncthreads_or(bad)) run(std::false_type{});
    } else {
      run(std::false_type{});
    }
  } else {
    run(std::false_type{});
  }
  if constexpr (!F32) { lrow[0] = lacc[0][0]; lrow[1] = lacc[1][0]; }
  // ---- epilogue: O[b][t][h*64 + d], d = ds*16 + 4g + i ; LSE (log2 units) = m + log2(l)
#pragma unroll
  for (int qs = 0; qs < 2; qs++) {
    int q = q0 + qs * 16 + li;
    if (q >= N) continue;
    float inv = 1.0f / lrow[qs];
    T* orow = O + ((long)b * N + q) * (H * 64) + h * 64;
#pragma unroll
    for (int ds = 0; ds < 4; ds++) {
      int d = ds * 16 + 4 * g;
      if constexpr (F32) *(float4*)(orow + d) = make_float4(o[ds][qs][0] * inv, o[ds][qs][1] * inv, o[ds][qs][2] * inv, o[ds][qs][3] * inv);
      else { bf16x4 v = {(bf16)(o[ds][qs][0] * inv), (bf16)(o[ds][qs][1] * inv), (bf16)(o[ds][qs][2] * inv), (bf16)(o[ds][qs][3] * inv)}; *(bf16x4*)(orow + d) = v; }
    }
    if (g == 0 && LSE) LSE[(long)bh * N + q] = mrow[qs] + __log2f(lrow[qs]);
  }
}


// ===================================================================================== backward
// delta[bh][q] = sum_d dO[b][q][h*64+d] * O[b][q][h*64+d]
// one thread per 8 consecutive d of one (token, head): 16-B loads over the contiguous token rows,
// the 8 partial dots of a head reduced with 3 lane shuffles (consecutive lanes)
template <typename T>
__global__ void attn_delta_kernel(const T* __restrict__ O, const T* __restrict__ dO, float* __restrict__ delta, int N, int H, int BH) {
  const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;          // chunk over [B*N][H][8]
  const long total = (long)BH * N * 8;
  float v = 0.f;
  const bool live = c < total;
  long tok = 0; int h = 0;
  if (live) {
    tok = c / (H * 8);
    const int rem = (int)(c - tok * (H * 8));
    h = rem >> 3;
    float a[8], d[8];
    load8<T>(O + c * 8, a);
    load8<T>(dO + c * 8, d);
#pragma unroll
    for (int e = 0; e < 8; e++) v += a[e] * d[e];
  }
  v += __shfl_xor(v, 1); v += __shfl_xor(v, 2); v += __shfl_xor(v, 4);
  if (live && (c & 7) == 0) {
    const long b = tok / N, q = tok - b * N;
    delta[(b * H + h) * N + q] = v;
  }
}

namespace {
// 64-row x 64-d tile image used for both row reads (ds_read_b128 / scalar) and transposed reads
template <typename T> struct Img;
template <> struct Img<bf16> {
  // 16-B slot XOR f((row >> 1) & 7) with f = (0,2,4,6,5,7,1,3): conflict-free for BOTH the
  // row-fragment ds_read_b128 and the transposed ds_read_b64_tr_b16 patterns (exhaustive search
  // over the 8! slot permutations against the gfx950 lane groups; the plain (row>>1)&7 XOR left
  // the transposed reads 2-way conflicted)
  static constexpr int BYTES = 64 * 128;
  DEV static int swz(int row) { return (0x31756420u >> (((row >> 1) & 7) * 4)) & 7; }
  DEV static int at(int row, int byte) { return row * 128 + ((((byte >> 4) ^ swz(row)) << 4) | (byte & 15)); }
};
template <> struct Img<float> {
  static constexpr int BYTES = 64 * 272;
  DEV static int at(int row, int byte) { return row * 272 + byte; }
};

// stage a [64 rows][64] tile of a strided tensor (row stride ld elements) into registers / LDS
template <typename T> struct RowTile {
  static constexpr int CH = 64 * 64 * sizeof(T) / 16 / 256;
  uint4 r[CH];
  DEV void load(const T* base, long ld, int row0, int N, int tid) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      int c = tid + 256 * i;
      constexpr int CPR = 64 * sizeof(T) / 16;
      int row = row0 + c / CPR, col = (c % CPR) * (16 / sizeof(T));
      r[i] = row < N ? *(const uint4*)(base + (long)row * ld + col) : make_uint4(0, 0, 0, 0);
    }
  }
  DEV void store(char* lds, int tid) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      int c = tid + 256 * i;
      constexpr int CPR = 64 * sizeof(T) / 16;
      *(uint4*)(lds + Img<T>::at(c / CPR, (c % CPR) * 16)) = r[i];
    }
  }
};

typedef __attribute__((address_space(3))) s16x4 lds_s4;
// bf16 A/B fragment of a 16x32 block read TRANSPOSED from an Img<bf16>:
// lane (g, i) gets X[row(g,j)][col0 + i] for j = 0..7 with row(g,j) = r0 + 4g + j (j<4), r0 + 16 + 4g + j-4 (j>=4)
DEV bf16x8 tr_frag(const char* img, int r0, int col0, int lane) {
  int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  int byte = (col0 + 4 * p) * 2;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + Img<bf16>::at(r0 + 4 * g + q, byte)));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + Img<bf16>::at(r0 + 16 + 4 * g + q, byte)));
  bf16x4 a = __builtin_bit_cast(bf16x4, lo), b = __builtin_bit_cast(bf16x4, hi);
  return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
// row fragment: lane (g, i) gets X[r0 + i][kk*32 + 8g .. +7]
DEV bf16x8 row_frag(const char* img, int r0, int kk, int lane) {
  return *(const bf16x8*)(img + Img<bf16>::at(r0 + (lane & 15), kk * 64 + (lane >> 4) * 16));
}
DEV bf16x8 pack8(f32x4 a, f32x4 b) {
  return bf16x8{(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3], (bf16)b[0], (bf16)b[1], (bf16)b[2], (bf16)b[3]};
}
DEV f32x4 mma_bf(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
DEV f32x4 mma_f(float a, float b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
DEV float ldsf(const char* img, int row, int col) { return *(const float*)(img + Img<float>::at(row, col * 4)); }
}  // namespace

// Fused backward epilogue (s3od_attn_bwd_qkv): instead of dQ / dK / dV in [B*H, N, 64], write the
// gradient of the QKV projection's output directly: d_qkv [B*N][3*H*64] (q | k | v column blocks,
// the layout s3od_qkv_rope_fwd reads), with the inverse RoPE applied to the patch tokens of q and k
// (tf:modeling_dinov3_vit.py:238-268: y = x cos + R(x) sin -> dx = cos dy + R^T(sin dy)), the 1/8 of
// the pre-scaled q, and the q / v bias gradients as replicated column sums (k_proj has no bias).
// Lane layout of the accumulators: token = lane's row, d = ds*16 + 4g + i, so the RoPE partner
// d +- 32 is ds ^ 2 in the same lane.
struct QkvSink {
  void* dqkv; const float* cs; const float* sn; float* ws; int P;
};
template <typename T>
DEV void qkv_sink_row(const QkvSink& o, int which, int b, int h, int H, int tok, int N, int g, const f32x4 (&val)[4], float scale,
                      f32x4 (&csum)[4]) {
  float out[4][4];
  const bool rope = which < 2 && tok >= N - o.P;
  if (rope) {
    const int tp = tok - (N - o.P);
#pragma unroll
    for (int ds = 0; ds < 4; ds++) {
      const float4 c = *(const float4*)(o.cs + (long)tp * 64 + ds * 16 + 4 * g);
      const float4 sn = *(const float4*)(o.sn + (long)tp * 64 + (ds ^ 2) * 16 + 4 * g);
      const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {sn.x, sn.y, sn.z, sn.w};
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const float rt = ss[i] * val[ds ^ 2][i];
        out[ds][i] = (cc[i] * val[ds][i] + (ds < 2 ? rt : -rt)) * scale;
      }
    }
  } else {
#pragma unroll
    for (int ds = 0; ds < 4; ds++)
#pragma unroll
      for (int i = 0; i < 4; i++) out[ds][i] = val[ds][i] * scale;
  }
  T* row = (T*)o.dqkv + ((long)b * N + tok) * (3L * H * 64) + (long)which * H * 64 + h * 64;
#pragma unroll
  for (int ds = 0; ds < 4; ds++) {
    T* dst = row + ds * 16 + 4 * g;
    if constexpr (std::is_same<T, float>::value) *(float4*)dst = make_float4(out[ds][0], out[ds][1], out[ds][2], out[ds][3]);
    else *(bf16x4*)dst = bf16x4{(bf16)out[ds][0], (bf16)out[ds][1], (bf16)out[ds][2], (bf16)out[ds][3]};
#pragma unroll
    for (int i = 0; i < 4; i++) csum[ds][i] += out[ds][i];
  }
}
// sum the 16 row-lanes of each column group and add into replica `rep` of ws [q D | v D]
DEV void qkv_sink_colsum(const QkvSink& o, int which, int h, int H, int rep, int lane, f32x4 (&csum)[4]) {
#pragma unroll
  for (int ds = 0; ds < 4; ds++)
#pragma unroll
    for (int i = 0; i < 4; i++) {
      float v = csum[ds][i];
      v += __shfl_xor(v, 1); v += __shfl_xor(v, 2); v += __shfl_xor(v, 4); v += __shfl_xor(v, 8);
      csum[ds][i] = v;
    }
  if ((lane & 15) == 0) {
    const int D = H * 64, g = lane >> 4;
    float* dst = o.ws + (long)rep * 2 * D + (which == 0 ? 0 : D) + h * 64 + 4 * g;
#pragma unroll
    for (int ds = 0; ds < 4; ds++)
#pragma unroll
      for (int i = 0; i < 4; i++) atomicAdd(dst + ds * 16 + i, csum[ds][i]);
  }
}

// dK, dV.  Workgroup = 4 waves x 16*KS keys of one (b,h); loop over 64-query tiles.
//   S  = Q K^T     (A = Q rows from LDS, B = K fragments in registers)   -> lane = key, regs = q
//   dP = dO V^T    (A = dO rows from LDS, B = V fragments in registers)
//   dV^T += dO^T P (A = dO^T via transposed LDS reads, B = P from the accumulators)
//   dK^T += Q^T dS (A = Q^T via transposed LDS reads, B = dS from the accumulators)
template <typename T, int KS>
__global__ void __launch_bounds__(256) attn_bwd_dkdv_kernel(const T* __restrict__ Q, const T* __restrict__ K, const T* __restrict__ V,
                                                             const T* __restrict__ dO, const float* __restrict__ LSE,
                                                             const float* __restrict__ Dl, T* __restrict__ dK, T* __restrict__ dV,
                                                             int N, int H, QkvSink sink) {
  constexpr bool F32 = std::is_same<T, float>::value;
  typedef Img<T> I;
  __shared__ __attribute__((aligned(16))) char smem[2 * (2 * I::BYTES + 512)];
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, li = lane & 15;
  const T* Qp = Q + (long)bh * N * 64;
  const T* Kp = K + (long)bh * N * 64;
  const T* Vp = V + (long)bh * N * 64;
  const T* dOp = dO + (long)b * N * (H * 64) + h * 64;
  const long ldo = (long)H * 64;
  const float* Lp = LSE + (long)bh * N;
  const float* Dp = Dl + (long)bh * N;
  const int k0 = blockIdx.x * (64 * KS) + wave * (16 * KS);

  constexpr int KK = F32 ? 16 : 2;
  typedef typename std::conditional<F32, float, bf16x8>::type frag;
  frag kf[KS][KK], vf[KS][KK];
#pragma unroll
  for (int ks = 0; ks < KS; ks++) {
    int key = k0 + ks * 16 + li;
#pragma unroll
    for (int kk = 0; kk < KK; kk++) {
      if constexpr (F32) {
        kf[ks][kk] = key < N ? Kp[(long)key * 64 + kk * 4 + g] : 0.f;
        vf[ks][kk] = key < N ? Vp[(long)key * 64 + kk * 4 + g] : 0.f;
      } else {
        bf16x8 z; for (int e = 0; e < 8; e++) z[e] = (bf16)0.f;
        kf[ks][kk] = key < N ? *(const bf16x8*)(Kp + (long)key * 64 + kk * 32 + 8 * g) : z;
        vf[ks][kk] = key < N ? *(const bf16x8*)(Vp + (long)key * 64 + kk * 32 + 8 * g) : z;
      }
    }
  }
  f32x4 dk[4][KS], dv[4][KS];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < KS; j++) { dk[i][j] = f32x4{0, 0, 0, 0}; dv[i][j] = f32x4{0, 0, 0, 0}; }

  RowTile<T> tq, tdo;
  float lse_r = 0.f, dl_r = 0.f;
  const int nqt = (N + 63) / 64;
  auto stage_load = [&](int qt) {
    tq.load(Qp, 64, qt * 64, N, tid);
    tdo.load(dOp, ldo, qt * 64, N, tid);
    if (tid < 64) { int q = qt * 64 + tid; lse_r = q < N ? -Lp[q] : -INFINITY; dl_r = q < N ? -Dp[q] : 0.f; }   // negated
  };
  auto stage_store = [&](char* base) {
    tq.store(base, tid); tdo.store(base + I::BYTES, tid);
    if (tid < 64) { ((float*)(base + 2 * I::BYTES))[tid] = lse_r; ((float*)(base + 2 * I::BYTES))[64 + tid] = dl_r; }
  };
  stage_load(0);
  stage_store(smem);
  __syncthreads();
  int cur = 0;
  constexpr int SB = 2 * I::BYTES + 512;
  for (int qt = 0; qt < nqt; qt++) {
    const bool more = qt + 1 < nqt;
    if (more) stage_load(qt + 1);
    const char* qs_ = smem + cur * SB;
    const char* dos = qs_ + I::BYTES;
    const float* lsel = (const float*)(qs_ + 2 * I::BYTES);
    const float* dll = lsel + 64;
    // accumulators start at -LSE[q] / -delta[q] (q = qb*16 + 4g + i), so after the MFMAs
    // s = score - lse (log2 units) and dp = dO.v - delta
    f32x4 s[4][KS], dp[4][KS];
#pragma unroll
    for (int qb = 0; qb < 4; qb++) {
      f32x4 nl = *(const f32x4*)(lsel + qb * 16 + 4 * g), nd = *(const f32x4*)(dll + qb * 16 + 4 * g);
#pragma unroll
      for (int ks = 0; ks < KS; ks++) { s[qb][ks] = nl; dp[qb][ks] = nd; }
    }
#pragma unroll
    for (int qb = 0; qb < 4; qb++) {
#pragma unroll
      for (int kk = 0; kk < KK; kk++) {
        if constexpr (F32) {
          float a = ldsf(qs_, qb * 16 + li, kk * 4 + g), c = ldsf(dos, qb * 16 + li, kk * 4 + g);
#pragma unroll
          for (int ks = 0; ks < KS; ks++) { s[qb][ks] = mma_f(a, kf[ks][kk], s[qb][ks]); dp[qb][ks] = mma_f(c, vf[ks][kk], dp[qb][ks]); }
        } else {
          bf16x8 a = row_frag(qs_, qb * 16, kk, lane), c = row_frag(dos, qb * 16, kk, lane);
#pragma unroll
          for (int ks = 0; ks < KS; ks++) { s[qb][ks] = mma_bf(a, kf[ks][kk], s[qb][ks]); dp[qb][ks] = mma_bf(c, vf[ks][kk], dp[qb][ks]); }
        }
      }
    }
    // P = exp2(S - LSE[q]), dS = P*(dP - delta[q])   (invalid q: LSE = +inf -> P = 0)
#pragma unroll
    for (int qb = 0; qb < 4; qb++)
#pragma unroll
      for (int ks = 0; ks < KS; ks++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
          float p = fexp2(s[qb][ks][i]);
          s[qb][ks][i] = p;
          dp[qb][ks][i] = p * dp[qb][ks][i];
        }
    // dV^T += dO^T P ; dK^T += Q^T dS
    if constexpr (F32) {
#pragma unroll
      for (int qb = 0; qb < 4; qb++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
          int qq = qb * 16 + 4 * g + i;
#pragma unroll
          for (int ds = 0; ds < 4; ds++) {
            float ao = ldsf(dos, qq, ds * 16 + li), aq = ldsf(qs_, qq, ds * 16 + li);
#pragma unroll
            for (int ks = 0; ks < KS; ks++) { dv[ds][ks] = mma_f(ao, s[qb][ks][i], dv[ds][ks]); dk[ds][ks] = mma_f(aq, dp[qb][ks][i], dk[ds][ks]); }
          }
        }
    } else {
#pragma unroll
      for (int qst = 0; qst < 2; qst++) {
        bf16x8 pb[KS], sb[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ks++) { pb[ks] = pack8(s[2 * qst][ks], s[2 * qst + 1][ks]); sb[ks] = pack8(dp[2 * qst][ks], dp[2 * qst + 1][ks]); }
#pragma unroll
        for (int ds = 0; ds < 4; ds++) {
          bf16x8 ao = tr_frag(dos, 32 * qst, ds * 16, lane), aq = tr_frag(qs_, 32 * qst, ds * 16, lane);
#pragma unroll
          for (int ks = 0; ks < KS; ks++) { dv[ds][ks] = mma_bf(ao, pb[ks], dv[ds][ks]); dk[ds][ks] = mma_bf(aq, sb[ks], dk[ds][ks]); }
        }
      }
    }
    if (more) stage_store(smem + (cur ^ 1) * SB);
    __syncthreads();
    cur ^= 1;
  }
  if (sink.dqkv) {   // fused: dK (inverse RoPE) and dV straight into d_qkv + the v-bias column sums
    f32x4 csk[4] = {f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}};
    f32x4 csv[4] = {f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}};
#pragma unroll
    for (int ks = 0; ks < KS; ks++) {
      const int key = k0 + ks * 16 + li;
      if (key >= N) continue;
      const f32x4 kv[4] = {dk[0][ks], dk[1][ks], dk[2][ks], dk[3][ks]};
      const f32x4 vv[4] = {dv[0][ks], dv[1][ks], dv[2][ks], dv[3][ks]};
      qkv_sink_row<T>(sink, 1, b, h, H, key, N, g, kv, LN2, csk);
      qkv_sink_row<T>(sink, 2, b, h, H, key, N, g, vv, 1.f, csv);
    }
    if (sink.ws) qkv_sink_colsum(sink, 2, h, H, (blockIdx.y * gridDim.x + blockIdx.x) % S3OD_NREP, lane, csv);
    return;
  }
  // store: lane = key (li), rows d = ds*16 + 4g + i
#pragma unroll
  for (int ks = 0; ks < KS; ks++) {
    int key = k0 + ks * 16 + li;
    if (key >= N) continue;
    T* dkr = dK + ((long)bh * N + key) * 64;
    T* dvr = dV + ((long)bh * N + key) * 64;
#pragma unroll
    for (int ds = 0; ds < 4; ds++) {
      int d = ds * 16 + 4 * g;
      dk[ds][ks] *= LN2;   // d(q.k*ln2)/dk with q in log2 scaling
      if constexpr (F32) {
        *(float4*)(dkr + d) = make_float4(dk[ds][ks][0], dk[ds][ks][1], dk[ds][ks][2], dk[ds][ks][3]);
        *(float4*)(dvr + d) = make_float4(dv[ds][ks][0], dv[ds][ks][1], dv[ds][ks][2], dv[ds][ks][3]);
      } else {
        *(bf16x4*)(dkr + d) = bf16x4{(bf16)dk[ds][ks][0], (bf16)dk[ds][ks][1], (bf16)dk[ds][ks][2], (bf16)dk[ds][ks][3]};
        *(bf16x4*)(dvr + d) = bf16x4{(bf16)dv[ds][ks][0], (bf16)dv[ds][ks][1], (bf16)dv[ds][ks][2], (bf16)dv[ds][ks][3]};
      }
    }
  }
}

// dQ (w.r.t. the pre-scaled q).  Workgroup = 4 waves x 16*QS queries; loop over 64-key tiles.
//   S^T = K Q^T, dP^T = V dO^T (B operands Q, dO in registers)  -> lane = q, regs = keys
//   dQ^T += K^T dS^T            (A = K^T via transposed LDS reads, B = dS^T from accumulators)
template <typename T, int QS>
__global__ void __launch_bounds__(256) attn_bwd_dq_kernel(const T* __restrict__ Q, const T* __restrict__ K, const T* __restrict__ V,
                                                           const T* __restrict__ dO, const float* __restrict__ LSE,
                                                           const float* __restrict__ Dl, T* __restrict__ dQ, int N, int H,
                                                           QkvSink sink) {
  constexpr bool F32 = std::is_same<T, float>::value;
  typedef Img<T> I;
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * I::BYTES];
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, li = lane & 15;
  const T* Qp = Q + (long)bh * N * 64;
  const T* Kp = K + (long)bh * N * 64;
  const T* Vp = V + (long)bh * N * 64;
  const T* dOp = dO + (long)b * N * (H * 64) + h * 64;
  const long ldo = (long)H * 64;
  const int q0 = blockIdx.x * (64 * QS) + wave * (16 * QS);
  constexpr int KK = F32 ? 16 : 2;
  typedef typename std::conditional<F32, float, bf16x8>::type frag;
  frag qf[QS][KK], of[QS][KK];
  float Lq[QS], Dq[QS];
#pragma unroll
  for (int qs = 0; qs < QS; qs++) {
    int q = q0 + qs * 16 + li;
    Lq[qs] = q < N ? LSE[(long)bh * N + q] : INFINITY;
    Dq[qs] = q < N ? Dl[(long)bh * N + q] : 0.f;
#pragma unroll
    for (int kk = 0; kk < KK; kk++) {
      if constexpr (F32) {
        qf[qs][kk] = q < N ? Qp[(long)q * 64 + kk * 4 + g] : 0.f;
        of[qs][kk] = q < N ? dOp[(long)q * ldo + kk * 4 + g] : 0.f;
      } else {
        bf16x8 z; for (int e = 0; e < 8; e++) z[e] = (bf16)0.f;
        qf[qs][kk] = q < N ? *(const bf16x8*)(Qp + (long)q * 64 + kk * 32 + 8 * g) : z;
        of[qs][kk] = q < N ? *(const bf16x8*)(dOp + (long)q * ldo + kk * 32 + 8 * g) : z;
      }
    }
  }
  f32x4 dq[4][QS];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int qs = 0; qs < QS; qs++) dq[i][qs] = f32x4{0, 0, 0, 0};
  f32x4 nl[QS], nd[QS];   // C operands: -lse (log2 units), -delta of the lane's query column
#pragma unroll
  for (int qs = 0; qs < QS; qs++) { nl[qs] = f32x4{-Lq[qs], -Lq[qs], -Lq[qs], -Lq[qs]}; nd[qs] = f32x4{-Dq[qs], -Dq[qs], -Dq[qs], -Dq[qs]}; }
  RowTile<T> tk, tv;
  const int nkt = (N + 63) / 64;
  tk.load(Kp, 64, 0, N, tid); tv.load(Vp, 64, 0, N, tid);
  tk.store(smem, tid); tv.store(smem + I::BYTES, tid);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nkt; kt++) {
    const bool more = kt + 1 < nkt;
    if (more) { tk.load(Kp, 64, (kt + 1) * 64, N, tid); tv.load(Vp, 64, (kt + 1) * 64, N, tid); }
    const char* ks_ = smem + cur * 2 * I::BYTES;
    const char* vs_ = ks_ + I::BYTES;
    f32x4 s[4][QS], dp[4][QS];
#pragma unroll
    for (int kb = 0; kb < 4; kb++) {
#pragma unroll
      for (int qs = 0; qs < QS; qs++) { s[kb][qs] = nl[qs]; dp[kb][qs] = nd[qs]; }
#pragma unroll
      for (int kk = 0; kk < KK; kk++) {
        if constexpr (F32) {
          float a = ldsf(ks_, kb * 16 + li, kk * 4 + g), c = ldsf(vs_, kb * 16 + li, kk * 4 + g);
#pragma unroll
          for (int qs = 0; qs < QS; qs++) { s[kb][qs] = mma_f(a, qf[qs][kk], s[kb][qs]); dp[kb][qs] = mma_f(c, of[qs][kk], dp[kb][qs]); }
        } else {
          bf16x8 a = row_frag(ks_, kb * 16, kk, lane), c = row_frag(vs_, kb * 16, kk, lane);
#pragma unroll
          for (int qs = 0; qs < QS; qs++) { s[kb][qs] = mma_bf(a, qf[qs][kk], s[kb][qs]); dp[kb][qs] = mma_bf(c, of[qs][kk], dp[kb][qs]); }
        }
      }
    }
    // dS^T = exp2(s - lse) * (dp - delta)
#pragma unroll
    for (int kb = 0; kb < 4; kb++)
#pragma unroll
      for (int qs = 0; qs < QS; qs++)
#pragma unroll
        for (int i = 0; i < 4; i++) dp[kb][qs][i] *= fexp2(s[kb][qs][i]);
    if (kt * 64 + 64 > N) {   // last tile: zero dS of keys >= N (exp2(-lse) may overflow)
#pragma unroll
      for (int kb = 0; kb < 4; kb++)
#pragma unroll
        for (int i = 0; i < 4; i++)
          if (kt * 64 + kb * 16 + 4 * g + i >= N) {
#pragma unroll
            for (int qs = 0; qs < QS; qs++) dp[kb][qs][i] = 0.f;
          }
    }
    if constexpr (F32) {
#pragma unroll
      for (int kb = 0; kb < 4; kb++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
          int key = kb * 16 + 4 * g + i;
#pragma unroll
          for (int ds = 0; ds < 4; ds++) {
            float a = ldsf(ks_, key, ds * 16 + li);
#pragma unroll
            for (int qs = 0; qs < QS; qs++) dq[ds][qs] = mma_f(a, dp[kb][qs][i], dq[ds][qs]);
          }
        }
    } else {
#pragma unroll
      for (int kst = 0; kst < 2; kst++) {
        bf16x8 sb[QS];
#pragma unroll
        for (int qs = 0; qs < QS; qs++) sb[qs] = pack8(dp[2 * kst][qs], dp[2 * kst + 1][qs]);
#pragma unroll
        for (int ds = 0; ds < 4; ds++) {
          bf16x8 a = tr_frag(ks_, 32 * kst, ds * 16, lane);
#pragma unroll
          for (int qs = 0; qs < QS; qs++) dq[ds][qs] = mma_bf(a, sb[qs], dq[ds][qs]);
        }
      }
    }
    if (more) { tk.store(smem + (cur ^ 1) * 2 * I::BYTES, tid); tv.store(smem + (cur ^ 1) * 2 * I::BYTES + I::BYTES, tid); }
    __syncthreads();
    cur ^= 1;
  }
  if (sink.dqkv) {   // fused: dQ (inverse RoPE, x 1/8 for the raw q) into d_qkv + the q-bias column sums
    f32x4 csq[4] = {f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}};
#pragma unroll
    for (int qs = 0; qs < QS; qs++) {
      const int q = q0 + qs * 16 + li;
      if (q >= N) continue;
      const f32x4 qv[4] = {dq[0][qs], dq[1][qs], dq[2][qs], dq[3][qs]};
      qkv_sink_row<T>(sink, 0, b, h, H, q, N, g, qv, 0.125f, csq);
    }
    if (sink.ws) qkv_sink_colsum(sink, 0, h, H, (blockIdx.y * gridDim.x + blockIdx.x) % S3OD_NREP, lane, csq);
    return;
  }
#pragma unroll
  for (int qs = 0; qs < QS; qs++) {
    int q = q0 + qs * 16 + li;
    if (q >= N) continue;
    T* r = dQ + ((long)bh * N + q) * 64;
#pragma unroll
    for (int ds = 0; ds < 4; ds++) {
      int d = ds * 16 + 4 * g;
      if constexpr (F32) *(float4*)(r + d) = make_float4(dq[ds][qs][0], dq[ds][qs][1], dq[ds][qs][2], dq[ds][qs][3]);
      else *(bf16x4*)(r + d) = bf16x4{(bf16)dq[ds][qs][0], (bf16)dq[ds][qs][1], (bf16)dq[ds][qs][2], (bf16)dq[ds][qs][3]};
    }
  }
}

// ===================================================================================== backward, bf16, 32x32x16
// The bf16 backward on v_mfma_f32_32x32x16_bf16: an MFMA of this shape holds the SIMD's vector issue for 8 of
// its 32 cycles (16x16x32: 8 of 16), so per multiply-add it leaves 1.5x the VALU issue room for the softmax
// recompute (exp2, P*(dP - delta), two bf16 packs per score), which is what bounds the 16x16x32 kernels above
// (PMC: ~2.7 VALU per MFMA, 22 % MFMA-busy).  Same algorithm and register-operand tricks:
//   dK/dV pass (one wave = 32 keys):  S = Q K^T, dP = dO V^T with the key on the lane (B = K / V fragments in
//     registers, A = Q / dO rows from LDS, C = -LSE / -delta rows); P and dS are then, as they stand in the
//     accumulators, the A operands of dV = P^T dO and dK = dS^T Q, whose B operands (dO, Q with the query on
//     the k index) come from transposed LDS reads of the same images.
//   dQ pass (one wave = 32 queries): S^T = K Q^T, dP^T = V dO^T with the query on the lane (C = -LSE / -delta
//     of the lane's query: constant register blocks, no per-tile init), dQ = dS K (A = dS^T accumulators,
//     B = K by transposed reads).
typedef float f32x16 __attribute__((ext_vector_type(16)));
namespace {
DEV f32x16 mma32(bf16x8 a, bf16x8 b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0); }

// 64-row x 64-col bf16 image, 128-B rows; 16-B chunk ch of row r at r*128 + 16*(ch ^ sw(r)) with
// sw(r) = ((r>>1)&1)<<2 | ((r>>2)&3): conflict-free for the 32x32x16 A-operand row reads (ds_read_b128, rows
// r0 + lane&31 in the b128 lane groups) AND the transposed B-operand reads (ds_read_b64_tr_b16: per 32-lane
// half 4 rows x 32 columns; rows 4m and 4m+2 land in chunk sets that differ in bit 2)
struct Img32 {
  static constexpr int BYTES = 64 * 128;
  DEV static int sw(int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); }
  DEV static int at(int row, int byte) { return row * 128 + ((((byte >> 4) ^ sw(row)) << 4) | (byte & 15)); }
};
// A fragment of rows r0..r0+31, k-step ks (16 columns): lane (r = lane&31, h = lane>>5) gets X[r0+r][16ks+8h .. +7]
DEV bf16x8 row32(const char* img, int r0, int ks, int lane) {
  return *(const bf16x8*)(img + Img32::at(r0 + (lane & 31), ks * 32 + (lane >> 5) * 16));
}
// B fragment (k = rows, column on the lane) of rows r0..r0+15 in the 32x32x16 accumulator k order:
// element j of lane half h = row r0 + 8(j>>2) + 4h + (j&3), column c0 + (lane&31)
DEV bf16x8 tr32(const char* img, int r0, int c0, int lane) {
  const int h = lane >> 5, g16 = (lane >> 4) & 1, li = lane & 15, q = li >> 2, p = li & 3;
  const int byte = (c0 + 16 * g16 + 4 * p) * 2;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + Img32::at(r0 + 4 * h + q, byte)));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + Img32::at(r0 + 8 + 4 * h + q, byte)));
  bf16x4 a = __builtin_bit_cast(bf16x4, lo), b = __builtin_bit_cast(bf16x4, hi);
  return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
// accumulator registers 8s .. 8s+7 as a bf16 operand fragment (k-step s of the row index)
DEV bf16x8 pack_acc(const f32x16& x, int s) {
  return bf16x8{(bf16)x[8 * s + 0], (bf16)x[8 * s + 1], (bf16)x[8 * s + 2], (bf16)x[8 * s + 3],
                (bf16)x[8 * s + 4], (bf16)x[8 * s + 5], (bf16)x[8 * s + 6], (bf16)x[8 * s + 7]};
}
// row of accumulator register i of lane half h (32x32 C/D layout)
DEV int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// stage a [64 rows][64] bf16 tile (row stride ld) through registers into an Img32, NT threads
template <int NT> struct RowTile32 {
  static constexpr int CH = 512 / NT;     // 16-B chunks per thread
  uint4 r[CH];
  DEV void load(const bf16* base, long ld, int row0, int N, int tid) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      const int c = tid + NT * i, row = row0 + (c >> 3), col = (c & 7) * 8;
      r[i] = row < N ? *(const uint4*)(base + (long)row * ld + col) : make_uint4(0, 0, 0, 0);
    }
  }
  DEV void store(char* lds, int tid) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      const int c = tid + NT * i;
      *(uint4*)(lds + Img32::at(c >> 3, (c & 7) * 16)) = r[i];
    }
  }
};

// fused epilogue of one wave's 32-row x 64-d result (rows tok0 + acc_row, column d = 32 db + lane&31) into
// d_qkv (inverse RoPE on the patch tokens of q / k, `scale`), with the column sums for the q / v bias
template <typename T>
DEV void qkv_sink32(const QkvSink& o, int which, int b, int hh, int H, int tok0, int N, int lane, const f32x16 (&val)[2],
                    float scale, float (&csum)[2]) {
  const int h = lane >> 5, c = lane & 31;
  T* base = (T*)o.dqkv + (long)which * H * 64 + hh * 64;
  // the RoPE table entries of all 16 rows are loaded before the first store (identity for prefix tokens, v and rows
  // past N): read row by row, every row's loads waited behind the previous row's stores (one vmcnt counts both), 16
  // serialized round trips at the end of every wave
  // (unconditional loads from a clamped row, then selects: a conditional load became a branchy loop and the
  // wait-count pass put a vmcnt(0) before every row's stores again)
  float c0[16], c1[16], s0[16], s1[16];
  const bool rq = which < 2 && o.P > 0;      // wave-uniform
  if (rq) {
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const int tok = tok0 + acc_row(i, h);
      const bool rope = tok < N && tok >= N - o.P;
      const long tp = rope ? (long)(tok - (N - o.P)) * 64 : 0;
      const float a = o.cs[tp + c], bb = o.cs[tp + c + 32], d = o.sn[tp + c], e = o.sn[tp + c + 32];
      c0[i] = rope ? a : 1.f;
      c1[i] = rope ? bb : 1.f;
      s0[i] = rope ? d : 0.f;
      s1[i] = rope ? e : 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const int tok = tok0 + acc_row(i, h);
    if (tok >= N) continue;
    float out[2] = {val[0][i] * scale, val[1][i] * scale};
    if (rq) {
      out[0] = (c0[i] * val[0][i] + s1[i] * val[1][i]) * scale;
      out[1] = (c1[i] * val[1][i] - s0[i] * val[0][i]) * scale;
    }
    T* row = base + ((long)b * N + tok) * (3L * H * 64);
#pragma unroll
    for (int db = 0; db < 2; db++) {
      row[32 * db + c] = from_f<T>(out[db]);
      csum[db] += out[db];
    }
  }
}
DEV void qkv_colsum32(const QkvSink& o, int which, int hh, int H, int rep, int lane, float (&csum)[2]) {
  const int D = H * 64;
#pragma unroll
  for (int db = 0; db < 2; db++) {
    const float v = csum[db] + __shfl_xor(csum[db], 32);
    if (lane < 32) atomicAdd(o.ws + (long)rep * 2 * D + (which == 0 ? 0 : D) + hh * 64 + 32 * db + lane, v);
  }
}
}  // namespace

// LDS-DMA of a 64-row x 128-B tile into an Img32 (buffer_load_dwordx4 ... lds: one wave instruction fills 1 KiB
// of LDS lane-linearly, so the image's XOR swizzle is applied to each lane's SOURCE chunk), W waves.  Rows past
// the buffer's end read zeros (hardware range check), so tile tails need no masking.
// Stage rows row0 .. row0+63 (row stride ldb bytes) into the image, the descriptor rebased on the tile's first row
// (scalar work only): the per-lane source offsets are loop-invariant registers, so a tile's DMA issue costs no
// vector ALU.  `total` = the buffer's byte size from `base`;
// rows past its end still read zeros (range check against the rebased size).
template <int W> struct Dma64R {
  static constexpr int NIW = 8 / W;
  unsigned vo[NIW];
  DEV void init(long ldb, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < NIW; i++) {
      const int o = (wave * NIW + i) * 1024 + lane * 16, row = o >> 7, lc = ((o >> 4) & 7) ^ Img32::sw(row);
      vo[i] = (unsigned)(row * ldb + lc * 16);
    }
  }
  DEV void issue(const char* base, unsigned long total, long row0, long ldb, char* img, int wave) const {
    const long off = row0 * ldb;
    const auto r = attn_rsrc(base + off, total - off);
#pragma unroll
    for (int i = 0; i < NIW; i++)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)(img + (wave * NIW + i) * 1024), 16, vo[i], 0, 0, 0);
  }
};
// 64 fp32 row constants (LSE or delta of one 64-query tile) by one wave's LDS-DMA (lanes 0..15 carry data)
DEV void dma_row64r(const float* base, int N, int q0, unsigned vo, char* dst) {   // vo = lane < 16 ? 16 lane : OOB
  __builtin_amdgcn_raw_ptr_buffer_load_lds(attn_rsrc(base + q0, (unsigned long)(N - q0) * 4), (lds_void*)dst, 16, vo, 0, 0, 0);
}
DEV f32x16 ld16(const float* p) {      // 4 consecutive-row groups of the 32x32 C layout (rows 8m + 0..3)
  const f32x4 a = *(const f32x4*)(p), b = *(const f32x4*)(p + 8), c = *(const f32x4*)(p + 16), d = *(const f32x4*)(p + 24);
  return f32x16{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3], c[0], c[1], c[2], c[3], d[0], d[1], d[2], d[3]};
}
DEV bf16x8 neg8(bf16x8 v) {
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 8; e++) r[e] = (bf16)(-(float)v[e]);
  return r;
}

// dK, dV.  Workgroup = W waves x 32 keys of one (b,h); loop over 64-query tiles.  Q, dO, LSE and delta of the
// next tile arrive by LDS-DMA during the current one (two LDS stages, one barrier per tile).  Signs: the key
// and value fragments are held negated, so the accumulators start at +LSE / +delta straight from LDS and hold
// LSE - S and delta - dP (exp2 takes the negation for free as an input modifier); dS is carried negated and
// flipped at the store.
// (s_setprio halves and sched_group_barrier-interleaved softmax variants were measured slower and removed: DESIGN §6)
template <int W>
__global__ void __launch_bounds__(64 * W) attn_bwd_dkdv32_kernel(const bf16* __restrict__ Q, const bf16* __restrict__ K,
                                                                   const bf16* __restrict__ V, const bf16* __restrict__ dO,
                                                                   const float* __restrict__ LSE, const float* __restrict__ Dl,
                                                                   bf16* __restrict__ dK, bf16* __restrict__ dV, int N, int H,
                                                                   QkvSink sink) {
  constexpr int SB = 2 * Img32::BYTES + 2048;
  __shared__ __attribute__((aligned(1024))) char smem[2 * SB];
  const int bh = blockIdx.y, b = bh / H, hh = bh - b * H;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5;
  const long ldo = (long)H * 64;
  Dma64R<W> dq_, ddo;
  dq_.init(128, wave, lane);
  ddo.init(ldo * 2, wave, lane);
  const unsigned vrow = lane < 16 ? 16u * lane : 0x80000000u;
  const int k0 = blockIdx.x * (32 * W) + wave * 32;
  const bool active = k0 < N;        // wave-uniform
  bf16x8 kf[4], vf[4];
  {
    const int key = k0 + (lane & 31);
    const bf16* kr = K + ((long)bh * N + key) * 64 + 8 * h;
    const bf16* vr = V + ((long)bh * N + key) * 64 + 8 * h;
    bf16x8 z; for (int e = 0; e < 8; e++) z[e] = (bf16)0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ks++) {
      kf[ks] = key < N ? neg8(*(const bf16x8*)(kr + 16 * ks)) : z;
      vf[ks] = key < N ? neg8(*(const bf16x8*)(vr + 16 * ks)) : z;
    }
  }
  f32x16 dk[2], dv[2];
#pragma unroll
  for (int db = 0; db < 2; db++) for (int i = 0; i < 16; i++) { dk[db][i] = 0.f; dv[db][i] = 0.f; }
  const int nqt = (N + 63) / 64;
  auto stage = [&](int qt, char* base) {
    dq_.issue((const char*)(Q + (long)bh * N * 64), (unsigned long)N * 128, (long)qt * 64, 128, base, wave);
    ddo.issue((const char*)(dO + (long)b * N * ldo + hh * 64), ((unsigned long)(N - 1) * ldo + 64) * 2, (long)qt * 64, ldo * 2,
              base + Img32::BYTES, wave);
    if (wave == 0) dma_row64r(LSE + (long)bh * N, N, qt * 64, vrow, base + 2 * Img32::BYTES);
    if (wave == W - 1) dma_row64r(Dl + (long)bh * N, N, qt * 64, vrow, base + 2 * Img32::BYTES + 1024);
  };
  stage(0, smem);
  __syncthreads();
  // the tile loop is unrolled by two so the LDS stage is a compile-time constant (every fragment address
  // becomes a per-lane base + immediate instead of being recomputed from the stage index each tile)
  // the stage pointers are __restrict__ parameters: the noalias scopes they carry after inlining let the
  // compiler's wait-count pass see that this tile's LDS reads cannot alias the next tile's LDS-DMA (without
  // them it put a vmcnt(0) before the first transposed read of every tile, waiting out the prefetch)
  auto tile = [&](int qt, char* __restrict__ nxt, const char* __restrict__ qs_) {
    if (qt + 1 < nqt) stage(qt + 1, nxt);
    const char* dos = qs_ + Img32::BYTES;
    const float* lsel = (const float*)(qs_ + 2 * Img32::BYTES);
    const float* dll = (const float*)(qs_ + 2 * Img32::BYTES + 1024);
    // software-pipelined over the two 32-query halves: the softmax VALU of one half is scheduled between the
    // MFMAs of the other (sched_group_barrier), so the matrix pipe does not idle through the exp / pack work
    f32x16 s[2], dp[2];
    bf16x8 pa[2][2], da[2][2];
    auto sdp = [&](int qb) {
      bf16x8 a[4], c[4];
#pragma unroll
      for (int ks = 0; ks < 4; ks++) { a[ks] = row32(qs_, 32 * qb, ks, lane); c[ks] = row32(dos, 32 * qb, ks, lane); }
      s[qb] = mma32(a[0], kf[0], ld16(lsel + 32 * qb + 4 * h));
      dp[qb] = mma32(c[0], vf[0], ld16(dll + 32 * qb + 4 * h));
#pragma unroll
      for (int ks = 1; ks < 4; ks++) { s[qb] = mma32(a[ks], kf[ks], s[qb]); dp[qb] = mma32(c[ks], vf[ks], dp[qb]); }
    };
    // s = LSE - S, dp = delta - dP:  P = exp2(-s);  -dS = P * dp ; packed as the A operands of dV / dK
    auto softmax = [&](int qb) {
#pragma unroll
      for (int i = 0; i < 16; i++) {
        const float p = fexp2(-s[qb][i]);
        s[qb][i] = p;
        dp[qb][i] *= p;
      }
#pragma unroll
      for (int st = 0; st < 2; st++) { pa[qb][st] = pack_acc(s[qb], st); da[qb][st] = pack_acc(dp[qb], st); }
    };
    auto dvdk = [&](int qb) {
#pragma unroll
      for (int st = 0; st < 2; st++) {
        bf16x8 bo[2], bq[2];
#pragma unroll
        for (int db = 0; db < 2; db++) { bo[db] = tr32(dos, 32 * qb + 16 * st, 32 * db, lane); bq[db] = tr32(qs_, 32 * qb + 16 * st, 32 * db, lane); }
#pragma unroll
        for (int db = 0; db < 2; db++) { dv[db] = mma32(pa[qb][st], bo[db], dv[db]); dk[db] = mma32(da[qb][st], bq[db], dk[db]); }
      }
    };
    if (active) {      // a wave past the partial last block only stages tiles
      sdp(0);
      __builtin_amdgcn_sched_barrier(0);
      sdp(1);
      softmax(0);
      __builtin_amdgcn_sched_barrier(0);
      dvdk(0);
      softmax(1);
      __builtin_amdgcn_sched_barrier(0);
      dvdk(1);
    }
    __syncthreads();      // drains this tile's reads and the next tile's LDS-DMA (vmcnt(0)) before the flip
  };
  int qt = 0;
  for (; qt + 1 < nqt; qt += 2) { tile(qt, smem + SB, smem); tile(qt + 1, smem, smem + SB); }
  if (qt < nqt) tile(qt, smem + SB, smem);
  if (sink.dqkv) {
    float csk[2] = {0.f, 0.f}, csv[2] = {0.f, 0.f};
    qkv_sink32<bf16>(sink, 1, b, hh, H, k0, N, lane, dk, -LN2, csk);
    qkv_sink32<bf16>(sink, 2, b, hh, H, k0, N, lane, dv, 1.f, csv);
    if (sink.ws) qkv_colsum32(sink, 2, hh, H, (blockIdx.y * gridDim.x + blockIdx.x) % S3OD_NREP, lane, csv);
    return;
  }
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const int key = k0 + acc_row(i, h);
    if (key >= N) continue;
    bf16* dkr = dK + ((long)bh * N + key) * 64;
    bf16* dvr = dV + ((long)bh * N + key) * 64;
#pragma unroll
    for (int db = 0; db < 2; db++) {
      dkr[32 * db + (lane & 31)] = (bf16)(dk[db][i] * -LN2);
      dvr[32 * db + (lane & 31)] = (bf16)dv[db][i];
    }
  }
}

// dQ (w.r.t. the pre-scaled q).  Workgroup = W waves x 32 queries; loop over 64-key tiles (K, V by LDS-DMA).
// Same sign convention: Q and dO fragments negated, C = +LSE / +delta of the lane's query (constant blocks).
template <int W>
__global__ void __launch_bounds__(64 * W) attn_bwd_dq32_kernel(const bf16* __restrict__ Q, const bf16* __restrict__ K,
                                                                 const bf16* __restrict__ V, const bf16* __restrict__ dO,
                                                                 const float* __restrict__ LSE, const float* __restrict__ Dl,
                                                                 bf16* __restrict__ dQ, int N, int H, QkvSink sink) {
  constexpr int SB = 2 * Img32::BYTES;
  __shared__ __attribute__((aligned(1024))) char smem[2 * SB];
  const int bh = blockIdx.y, b = bh / H, hh = bh - b * H;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5;
  Dma64R<W> dkv;
  dkv.init(128, wave, lane);
  const int q0 = blockIdx.x * (32 * W) + wave * 32;
  const bool active = q0 < N;        // wave-uniform
  bf16x8 qf[4], of[4];
  f32x16 cl, cd;     // C operands: LSE (log2 units) / delta of the lane's query, all 16 rows
  {
    const int q = q0 + (lane & 31);
    const bf16* qr = Q + ((long)bh * N + q) * 64 + 8 * h;
    const bf16* orow = dO + ((long)b * N + q) * (H * 64) + hh * 64 + 8 * h;
    bf16x8 z; for (int e = 0; e < 8; e++) z[e] = (bf16)0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ks++) {
      qf[ks] = q < N ? neg8(*(const bf16x8*)(qr + 16 * ks)) : z;
      of[ks] = q < N ? neg8(*(const bf16x8*)(orow + 16 * ks)) : z;
    }
    const float l = q < N ? LSE[(long)bh * N + q] : INFINITY, d = q < N ? Dl[(long)bh * N + q] : 0.f;
#pragma unroll
    for (int i = 0; i < 16; i++) { cl[i] = l; cd[i] = d; }
  }
  f32x16 dq[2];
#pragma unroll
  for (int db = 0; db < 2; db++) for (int i = 0; i < 16; i++) dq[db][i] = 0.f;
  const int nkt = (N + 63) / 64;
  auto stage = [&](int kt, char* base) {
    dkv.issue((const char*)(K + (long)bh * N * 64), (unsigned long)N * 128, (long)kt * 64, 128, base, wave);
    dkv.issue((const char*)(V + (long)bh * N * 64), (unsigned long)N * 128, (long)kt * 64, 128, base + Img32::BYTES, wave);
  };
  stage(0, smem);
  __syncthreads();
  auto tile = [&](int kt, char* __restrict__ nxt, const char* __restrict__ ks_) {   // unrolled by two, as in the dK/dV pass
    if (kt + 1 < nkt) stage(kt + 1, nxt);
    const char* vs_ = ks_ + Img32::BYTES;
    f32x16 s[2], dp[2];
    bf16x8 da[2][2];
    auto sdp = [&](int kb) {
      bf16x8 a[4], c[4];
#pragma unroll
      for (int ks = 0; ks < 4; ks++) { a[ks] = row32(ks_, 32 * kb, ks, lane); c[ks] = row32(vs_, 32 * kb, ks, lane); }
      s[kb] = mma32(a[0], qf[0], cl);
      dp[kb] = mma32(c[0], of[0], cd);
#pragma unroll
      for (int ks = 1; ks < 4; ks++) { s[kb] = mma32(a[ks], qf[ks], s[kb]); dp[kb] = mma32(c[ks], of[ks], dp[kb]); }
    };
    // s = LSE - S^T, dp = delta - dP^T:  -dS^T = exp2(-s) * dp, packed as the A operand of dQ
    auto softmax = [&](int kb) {
#pragma unroll
      for (int i = 0; i < 16; i++) dp[kb][i] *= fexp2(-s[kb][i]);
      if (kt * 64 + 64 > N) {   // last tile: zero dS of keys >= N (exp2(-lse) may overflow)
#pragma unroll
        for (int i = 0; i < 16; i++)
          if (kt * 64 + 32 * kb + acc_row(i, h) >= N) dp[kb][i] = 0.f;
      }
#pragma unroll
      for (int st = 0; st < 2; st++) da[kb][st] = pack_acc(dp[kb], st);
    };
    auto dqk = [&](int kb) {
#pragma unroll
      for (int st = 0; st < 2; st++) {
        bf16x8 bk[2];
#pragma unroll
        for (int db = 0; db < 2; db++) bk[db] = tr32(ks_, 32 * kb + 16 * st, 32 * db, lane);
#pragma unroll
        for (int db = 0; db < 2; db++) dq[db] = mma32(da[kb][st], bk[db], dq[db]);
      }
    };
    if (active) {      // a wave past the partial last block only stages tiles
      sdp(0);
      __builtin_amdgcn_sched_barrier(0);
      sdp(1);
      softmax(0);
      __builtin_amdgcn_sched_barrier(0);
      dqk(0);
      softmax(1);
      __builtin_amdgcn_sched_barrier(0);
      dqk(1);
    }
    __syncthreads();
  };
  int kt = 0;
  for (; kt + 1 < nkt; kt += 2) { tile(kt, smem + SB, smem); tile(kt + 1, smem, smem + SB); }
  if (kt < nkt) tile(kt, smem + SB, smem);
  if (sink.dqkv) {
    float csq[2] = {0.f, 0.f};
    qkv_sink32<bf16>(sink, 0, b, hh, H, q0, N, lane, dq, -0.125f, csq);
    if (sink.ws) qkv_colsum32(sink, 0, hh, H, (blockIdx.y * gridDim.x + blockIdx.x) % S3OD_NREP, lane, csq);
    return;
  }
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const int q = q0 + acc_row(i, h);
    if (q >= N) continue;
    bf16* r = dQ + ((long)bh * N + q) * 64;
#pragma unroll
    for (int db = 0; db < 2; db++) r[32 * db + (lane & 31)] = (bf16)(-dq[db][i]);
  }
}

// (hipcc 7.2 left the host stubs of these instances undefined when they were only named in the launcher below)
template __global__ void attn_fwd_kernel<bf16, true>(const bf16*, const bf16*, const bf16*, bf16*, float*, int, int, int);
template __global__ void attn_bwd_dq32_kernel<4>(const bf16*, const bf16*, const bf16*, const bf16*, const float*, const float*, bf16*,
                                                 int, int, QkvSink);
template __global__ void attn_bwd_dkdv32_kernel<4>(const bf16*, const bf16*, const bf16*, const bf16*, const float*, const float*, bf16*,
                                                   bf16*, int, int, QkvSink);

extern "C" {

// q,k,v: [B*H, N, 64] (q pre-scaled by log2(e)/8); o: [B, N, H*64]; lse: [B*H, N] fp32, log2 units (optional)
int s3od_attn_fwd(int dtype, const void* q, const void* k, const void* v, void* o, float* lse, int B, int H, int N, void* stream) {
  dim3 grid(cdiv(N, 128), B * H);
  // bf16 and f32: the 16x16 kernel (a 32x32x16 bf16 variant measured 6-8 % slower: 1083 -> 1150 us at bs 16, N 4101;
  // 3532 -> 3817 us at bs 4, N 16389, same box -- its extra row-sum MFMAs cost 2x the cycles; removed)
  // bf16: K / V by LDS-DMA -- same box, one process, alternating: 902 -> 739 us at bs 16 N 4101, 3374 -> 2805 us at
  // bs 4 N 16389, outputs bit-identical (profiles/r06k_attn_fwd_dma_ab.txt); S3OD_ATTN_DMA=0: the register-staged form
  if (dtype == S3OD_BF16 && S3OD_KNOB("S3OD_ATTN_DMA", 1)) {
    hipLaunchKernelGGL((attn_fwd_kernel<bf16, true>), grid, dim3(256), 0, (hipStream_t)stream, (const bf16*)q, (const bf16*)k,
                       (const bf16*)v, (bf16*)o, lse, N, H, S3OD_KNOB("S3OD_ATTN_FAST", 1));
    return s3od_check_launch("attn_fwd");
  }
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL(attn_fwd_kernel<T>, grid, dim3(256), 0, (hipStream_t)stream, (const T*)q, (const T*)k, (const T*)v, (T*)o, lse, N, H,
                       S3OD_KNOB("S3OD_ATTN_FAST", 1));   // 0: the lazy-rescale loop throughout (A/B)
  });
  return s3od_check_launch("attn_fwd");
}
}  // extern "C"

namespace {
__global__ void qkv_fold_kernel(float* __restrict__ ws, float* __restrict__ a, float* __restrict__ b, int D) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * D) return;
  float s = 0.f;
  for (int r = 0; r < S3OD_NREP; r++) { s += ws[(long)r * 2 * D + i]; ws[(long)r * 2 * D + i] = 0.f; }
  if (i < D) { if (a) a[i] += s; }
  else if (b) b[i - D] += s;
}

template <typename T>
void launch_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout, const float* lse, float* delta,
                void* dq, void* dk, void* dv, QkvSink sink, int B, int H, int N, hipStream_t st) {
  // 32 keys (dK/dV pass) / 32 queries (dQ pass) per wave: 64 per wave halves the LDS bytes per MFMA but
  // needs > 256 registers -> one wave per SIMD: the whole backward measured 19 % (dK/dV) / 11 % (dQ) slower at N=4101
  hipLaunchKernelGGL(attn_delta_kernel<T>, dim3(cdiv((long)B * H * N * 8, 256)), dim3(256), 0, st, (const T*)o, (const T*)dout, delta, N, H, B * H);
  if constexpr (std::is_same<T, bf16>::value) {
    // bf16: the 32x32x16 kernels, 4 waves per workgroup, tile loops unrolled by two (the 16x16x32 bf16 bodies,
    // 8-wave workgroups, s_setprio and interleaved variants were measured slower and removed: DESIGN §6)
    hipLaunchKernelGGL((attn_bwd_dkdv32_kernel<4>), dim3(cdiv(N, 128), B * H), dim3(256), 0, st,
                       (const bf16*)q, (const bf16*)k, (const bf16*)v, (const bf16*)dout, lse, delta, (bf16*)dk, (bf16*)dv, N, H,
                       sink);
    hipLaunchKernelGGL((attn_bwd_dq32_kernel<4>), dim3(cdiv(N, 128), B * H), dim3(256), 0, st,
                       (const bf16*)q, (const bf16*)k, (const bf16*)v, (const bf16*)dout, lse, delta, (bf16*)dq, N, H, sink);
    return;
  } else {
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<T, 2>), dim3(cdiv(N, 128), B * H), dim3(256), 0, st, (const T*)q, (const T*)k, (const T*)v,
                       (const T*)dout, lse, delta, (T*)dk, (T*)dv, N, H, sink);
    hipLaunchKernelGGL((attn_bwd_dq_kernel<T, 2>), dim3(cdiv(N, 128), B * H), dim3(256), 0, st, (const T*)q, (const T*)k, (const T*)v,
                       (const T*)dout, lse, delta, (T*)dq, N, H, sink);
  }
}
}  // namespace

extern "C" {

// backward: o, do: [B, N, H*64]; q,k,v: [B*H, N, 64]; lse, delta(workspace): [B*H, N] fp32
// outputs dq = dS.K (dS in natural units; the caller scales by 1/8 for d(rope(q))), dk, dv: [B*H, N, 64]
int s3od_attn_bwd(int dtype, const void* q, const void* k, const void* v, const void* o, const void* dout, const float* lse,
                  float* delta, void* dq, void* dk, void* dv, int B, int H, int N, void* stream) {
  QkvSink none{};
  DISPATCH_T(dtype, { launch_bwd<T>(q, k, v, o, dout, lse, delta, dq, dk, dv, none, B, H, N, (hipStream_t)stream); });
  return s3od_check_launch("attn_bwd");
}

// backward fused with the QKV+RoPE projection's output gradient: d_qkv [B*N][3*H*64] (T) with the
// inverse RoPE on the last P tokens (cos_t / sin_t: [P][64] fp32, the forward's tables), q x 1/8,
// and dbq / dbv (fp32 [H*64], nullable) += column sums; ws: S3OD_NREP * 2 * H*64 floats, all zero on entry
// and left all zero (nullable when both bias gradients are null).  Replaces s3od_attn_bwd + s3od_qkv_unrope.
int s3od_attn_bwd_qkv(int dtype, const void* q, const void* k, const void* v, const void* o, const void* dout, const float* lse,
                      float* delta, const float* cos_t, const float* sin_t, int P, void* dqkv, float* dbq, float* dbv,
                      float* ws, int B, int H, int N, void* stream) {
  S3OD_REQUIRE(dqkv && cos_t && sin_t && P >= 0 && P <= N, "attn_bwd_qkv: bad arguments");
  S3OD_REQUIRE(ws || (!dbq && !dbv), "attn_bwd_qkv: bias gradients need the workspace");
  hipStream_t st = (hipStream_t)stream;
  const int D = 64 * H;
  QkvSink sink{dqkv, cos_t, sin_t, ws, P};
  DISPATCH_T(dtype, { launch_bwd<T>(q, k, v, o, dout, lse, delta, nullptr, nullptr, nullptr, sink, B, H, N, st); });
  if (ws) hipLaunchKernelGGL(qkv_fold_kernel, dim3(cdiv(2 * D, 256)), dim3(256), 0, st, ws, dbq, dbv, D);
  return s3od_check_launch("attn_bwd_qkv");
}
}  // extern "C"
