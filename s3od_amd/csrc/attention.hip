// Flash attention for DINOv3 ViT-B/16 (12 heads x d=64, non-causal, no mask), gfx950.
// Reference semantics: SDPA softmax(q k^T / 8) v (tf:integrations/sdpa_attention.py:79-166,
// tf:models/dinov3_vit/modeling_dinov3_vit.py:294-334).  q arrives pre-scaled by 1/8.
//
// Forward: one workgroup = 4 waves = 128 query rows of one (b, h); each wave owns 32 queries.
// "Swapped" products keep the softmax row lane-local:
//   S^T[key][q] = K . Q^T       (A = K tile from LDS, B = Q fragments held in registers)
//   O^T[d][q]  += V^T . P^T     (A = V^T via ds_read_b64_tr_b16, B = P^T straight from the
//                                S^T accumulator registers; the K-order of the MFMA is permuted
//                                identically on both operands, so no shuffles / LDS round trip)
// K/V tiles of 64 keys are register-staged into double-buffered LDS (one barrier per tile).
// T=float runs the same dataflow on v_mfma_f32_16x16x4_f32 (strict-parity path).
#include "common.hpp"
#include <type_traits>

#define DISPATCH_T(dtype, ...)                                                  \
  do {                                                                          \
    if ((dtype) == S3OD_BF16) { typedef bf16 T; __VA_ARGS__ }                   \
    else if ((dtype) == S3OD_F32) { typedef float T; __VA_ARGS__ }              \
    else { s3od_set_error("bad dtype %d", (int)(dtype)); return 22; }           \
  } while (0)

namespace {
constexpr float LOG2E = 1.4426950408889634f;

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

template <typename T> struct Stage {
  static constexpr int CH = 64 * 64 * sizeof(T) / 16 / 256;   // 16-B chunks per thread per tile
  uint4 k[CH], v[CH];
  DEV void load(const T* K, const T* V, int key0, int N, int tid) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      int c = tid + 256 * i;
      constexpr int CPR = 64 * sizeof(T) / 16;
      int key = key0 + c / CPR, col = (c % CPR) * (16 / sizeof(T));
      bool ok = key < N;
      k[i] = ok ? *(const uint4*)(K + (long)key * 64 + col) : make_uint4(0, 0, 0, 0);
      v[i] = ok ? *(const uint4*)(V + (long)key * 64 + col) : make_uint4(0, 0, 0, 0);
    }
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
}  // namespace

template <typename T>
__global__ void __launch_bounds__(256) attn_fwd_kernel(const T* __restrict__ Q, const T* __restrict__ K, const T* __restrict__ V,
                                                        T* __restrict__ O, float* __restrict__ LSE, int N, int H) {
  constexpr bool F32 = std::is_same<T, float>::value;
  typedef TileL<T> L;
  __shared__ __attribute__((aligned(16))) char smem[4 * L::BYTES];
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, li = lane & 15;
  const T* Qp = Q + (long)bh * N * 64;
  const T* Kp = K + (long)bh * N * 64;
  const T* Vp = V + (long)bh * N * 64;
  const int q0 = blockIdx.x * 128 + wave * 32;

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
#pragma unroll
  for (int i = 0; i < 4; i++) { o[i][0] = f32x4{0, 0, 0, 0}; o[i][1] = f32x4{0, 0, 0, 0}; }
  float mrow[2] = {-INFINITY, -INFINITY}, lrow[2] = {0.f, 0.f};

  Stage<T> stg;
  const int nkt = (N + 63) / 64;
  stg.load(Kp, Vp, 0, N, tid);
  stg.store(smem, smem + L::BYTES, tid);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nkt; kt++) {
    const bool more = kt + 1 < nkt;
    if (more) stg.load(Kp, Vp, (kt + 1) * 64, N, tid);
    const char* ks = smem + cur * 2 * L::BYTES;
    const char* vs = ks + L::BYTES;
    // ---- S^T = K Q^T : acc[ks][qs], element i: key = ks*16 + 4g + i, query = qs*16 + li
    f32x4 s[4][2];
#pragma unroll
    for (int kb = 0; kb < 4; kb++) {
      s[kb][0] = f32x4{0, 0, 0, 0}; s[kb][1] = f32x4{0, 0, 0, 0};
#pragma unroll
      for (int kk = 0; kk < QK; kk++) {
        if constexpr (F32) {
          float a = *(const float*)(ks + L::krow(kb * 16 + li, (kk * 4 + g) * 4));
          s[kb][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, qf[0][kk], s[kb][0], 0, 0, 0);
          s[kb][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, qf[1][kk], s[kb][1], 0, 0, 0);
        } else {
          bf16x8 a = *(const bf16x8*)(ks + L::krow(kb * 16 + li, kk * 64 + g * 16));
          s[kb][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[0][kk], s[kb][0], 0, 0, 0);
          s[kb][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[1][kk], s[kb][1], 0, 0, 0);
        }
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
    // ---- online softmax per query column
#pragma unroll
    for (int qs = 0; qs < 2; qs++) {
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 4; kb++)
#pragma unroll
        for (int i = 0; i < 4; i++) mx = fmaxf(mx, s[kb][qs][i]);
      mx = fmaxf(mx, __shfl_xor(mx, 16));
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      float mnew = fmaxf(mrow[qs], mx);
      float alpha = exp2f((mrow[qs] - mnew) * LOG2E);
      float nb = mnew * LOG2E;
      float sum = 0.f;
#pragma unroll
      for (int kb = 0; kb < 4; kb++)
#pragma unroll
        for (int i = 0; i < 4; i++) { float p = exp2f(s[kb][qs][i] * LOG2E - nb); s[kb][qs][i] = p; sum += p; }
      sum += __shfl_xor(sum, 16);
      sum += __shfl_xor(sum, 32);
      lrow[qs] = lrow[qs] * alpha + sum;
      mrow[qs] = mnew;
#pragma unroll
      for (int ds = 0; ds < 4; ds++) o[ds][qs] *= alpha;
    }
    // ---- O^T += V^T P^T
    if constexpr (F32) {
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
      typedef __attribute__((address_space(3))) s16x4 lds_s4;
#pragma unroll
      for (int kst = 0; kst < 2; kst++) {
        bf16x8 pb[2];
#pragma unroll
        for (int qs = 0; qs < 2; qs++)
#pragma unroll
          for (int i = 0; i < 4; i++) { pb[qs][i] = (bf16)s[2 * kst][qs][i]; pb[qs][4 + i] = (bf16)s[2 * kst + 1][qs][i]; }
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
      }
    }
    if (more) stg.store(smem + (cur ^ 1) * 2 * L::BYTES, smem + (cur ^ 1) * 2 * L::BYTES + L::BYTES, tid);
    __syncthreads();
    cur ^= 1;
  }
  // ---- epilogue: O[b][t][h*64 + d], d = ds*16 + 4g + i ; LSE = m + ln(l)
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
    if (g == 0 && LSE) LSE[(long)bh * N + q] = mrow[qs] + logf(lrow[qs]);
  }
}

extern "C" {

// q,k,v: [B*H, N, 64] (q pre-scaled by 1/8); o: [B, N, H*64]; lse: [B*H, N] fp32 (optional)
int s3od_attn_fwd(int dtype, const void* q, const void* k, const void* v, void* o, float* lse, int B, int H, int N, void* stream) {
  dim3 grid(cdiv(N, 128), B * H);
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL(attn_fwd_kernel<T>, grid, dim3(256), 0, (hipStream_t)stream, (const T*)q, (const T*)k, (const T*)v, (T*)o, lse, N, H);
  });
  return s3od_check_launch("attn_fwd");
}

}  // extern "C"
