// C-ABI entry points built on the implicit-GEMM engine (gemm.hpp).
#include "gemm.hpp"
#include <type_traits>

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
static int gemm_cfg() {
  static int c = -2;
  if (c == -2) { const char* e = getenv("S3OD_GEMM_CFG"); c = e ? atoi(e) : -1; }
  return c;
}
// W = waves that issue the operand loads (the loaders are built for that many waves)
template <int BM_, int BN_, int NST_, int W_ = GEMM_WAVES, int WM_ = 0> struct TileCfg {
  static constexpr int BM = BM_, BN = BN_, NST = NST_, W = W_, WM = WM_;
};
// call f(TileCfg) for the selected config; `def` = per-op default config index
template <typename T, class F> static int with_cfg(int def, F f) {
  int c = gemm_cfg(); if (c < 0) c = def;
  switch (c) {
    case 1: return f(TileCfg<128, 128, 2>{});
    case 2: return f(TileCfg<128, 128, 3>{});
    case 3: return f(TileCfg<256, 128, 2>{});
    case 4: return f(TileCfg<256, 256, 2>{});
    default: return f(TileCfg<256, 128, 3>{});
  }
}

// ------------------------------------------------------------------ QKV + RoPE epilogue
// n in [0,2304): q | k | v ; RoPE on patch tokens for q,k (tf:…/modeling_dinov3_vit.py:238-268);
// q pre-multiplied by the softmax scale 1/8 (exact in any binary float format).
template <typename T> struct EpiQKV {
  T* q; T* k; T* v; const float* bias; const float* cs; const float* sn;
  int M, Ntok, P, H;
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
      int b = m / Ntok, t = m - b * Ntok;
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
  DEV void prepare(int) {}
  DEV void operator()(const float* ct, int LDT, int m0, int n0, int tid, int BM, int BN, int NT) const {
    const int C = 32 * NM, SPR = 4 * NM;                      // channels / 8-channel segments per row
    // h = relu(acc + b1) is formed on the fly from the staged fp32 tile (no in-place pass)
    if (hsave) {
      const int segs = BM * SPR;
      for (int s = tid; s < segs; s += NT) {
        int r = s / SPR, c = (s - r * SPR) * 8, m = m0 + r;
        if (m >= M) continue;
        const float4* src = (const float4*)(ct + r * LDT + c);
        float4 x0 = src[0], x1 = src[1];
        float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
        for (int e = 0; e < 8; e++) v[e] = fmaxf(v[e] + b1[c + e], 0.f);
        store8<T>(hsave + (long)m * C + c, v);
      }
    }
    // logit_k = b2[k] + sum_j relu(acc[32k + j] + b1[32k + j]) * w2[32k + j]; k is wave-uniform
    for (int s = tid; s < NM * BM; s += NT) {
      int k = s / BM, r = s - k * BM;
      int m = m0 + r;
      if (m >= M) continue;
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
      int b = m / HW, pix = m - b * HW;
      logits[((long)b * NM + k) * HW + pix] = acc;
    }
  }
};

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

// dw[(co*Cin + ci)*taps + tap] += ws[(co*taps + tap)*Cin + ci]   (one thread per dw element)
__global__ void wgrad_permute_add_kernel(const float* __restrict__ ws, float* __restrict__ dw, int Cout, int Cin, int taps) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)Cout * Cin * taps) return;
  int tap = i % taps; long r = i / taps;
  int ci = r % Cin; int co = r / Cin;
  dw[i] += ws[((long)co * taps + tap) * Cin + ci];
}

extern "C" {

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
  RowMap rm = dense_rm(); rm.mode = row_mode; rm.P = P; rm.prefix = prefix;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    const int KTILES = cdiv(K, KT<T>::BK);
    auto go = [&](auto tile, auto tout, auto tres) -> int {
      typedef decltype(tout) TO; typedef decltype(tres) TR;
      // measured (tools/lin_sweep.py): 256x128 x 3 stages for K >= 2048; the GELU(+pre) up-projection
      // runs best on 256x256 tiles (574 vs 621 us at M=65616 N=3072 K=768); 128x128 otherwise
      const int def = K >= 2048 ? 0 : (act == ACT_GELU && N >= 2048 ? 4 : 1);
      return with_cfg<T>(def, [&](auto C) -> int {
        constexpr int BM = decltype(C)::BM, BN = decltype(C)::BN, NST = decltype(C)::NST;
        DenseKC<T, BM, decltype(C)::W> la{(const T*)x, ldx, M, K, 0};
        DenseKC<T, BN, decltype(C)::W> lb{(const T*)w, (long)K, N, K, 0};
        EpiStd<TO, TR, T> e{(TO*)out, ldo, 0, bias, scale, shift, (const TR*)res1, ldr1, (const TR*)res2, ldr2,
                            (T*)pre, ldp, nullptr, act, M, N, rm};
        static const int epi_probe = dev_knob("S3OD_EPI_PROBE", 0);   // dev: 1 = skip the epilogue's stores
        if (epi_probe == 1) e.M = 0;
        return launch_igemm<T, BM, BN, decltype(la), decltype(lb), decltype(e), NST, decltype(C)::WM>(la, lb, e, M, N, KTILES, 1, 1, st);
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
  RowMap rm = dense_rm(); rm.mode = row_mode; rm.P = P; rm.prefix = prefix;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    const int KTILES = cdiv(K, KT<T>::BK);
    return with_cfg<T>(1, [&](auto C) -> int {
      constexpr int BM = decltype(C)::BM, BN = decltype(C)::BN, NST = decltype(C)::NST;
      DenseKC<T, BM, decltype(C)::W> la{(const T*)dy, lddy, M, K, 0};
      DenseMC<T, BN, decltype(C)::W> lb{(const T*)w, (long)N, K, N};
      if (out_f32) {
        // f32 output: aux is an f32 tensor to add (e.g. the residual-stream gradient, in place)
        EpiStd<float, float> e{(float*)dx, lddx, 0, nullptr, nullptr, nullptr, (const float*)aux, ldaux, nullptr, 0, nullptr, 0, nullptr, act, M, N, rm, colsum};
        return launch_igemm<T, BM, BN, decltype(la), decltype(lb), decltype(e), NST, decltype(C)::WM>(la, lb, e, M, N, KTILES, 1, 1, st);
      }
      EpiStd<T, T> e{(T*)dx, lddx, 0, nullptr, nullptr, nullptr, (const T*)aux, ldaux, nullptr, 0, nullptr, 0, nullptr, act, M, N, rm, colsum};
      return launch_igemm<T, BM, BN, decltype(la), decltype(lb), decltype(e), NST, decltype(C)::WM>(la, lb, e, M, N, KTILES, 1, 1, st);
    });
  });
  return 0;
}

// dw[n_out, k_in] += sum_rows dy[row, n_out] x[row, k_in]   (fp32 atomics, split over rows)
int s3od_linear_wgrad(int dtype, int Nout, int Kin, int rows, const void* dy, long lddy,
                      const void* x, long ldx, float* dw, int split, void* stream) {
  S3OD_REQUIRE(Nout % 8 == 0 && Kin % 8 == 0, "linear_wgrad: dims %% 8");
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    const int KTILES = cdiv(rows, KT<T>::BK);
    // measured (tools/lin_sweep.py, bs16 1024^2 ViT shapes): 128x128 tiles for the large outputs
    // (3072x768, 2304x768, 768x3072: 7-12 % faster than 256x256), 256x128 for 768x768
    const int def = (long)Nout * Kin <= 1024L * 1024 ? 0 : 1;
    return with_cfg<T>(def, [&](auto C) -> int {
      constexpr int BM = decltype(C)::BM, BN = decltype(C)::BN, NST = decltype(C)::NST;
      int sp = split > 0 ? split : wgrad_split<T, BM, BN, NST>(cdiv(Nout, BM) * cdiv(Kin, BN), KTILES);
      DenseMC<T, BM, decltype(C)::W> la{(const T*)dy, lddy, rows, Nout};
      DenseMC<T, BN, decltype(C)::W> lb{(const T*)x, ldx, rows, Kin};
      EpiWgrad e{dw, Nout, Kin, Kin, 1};
      return launch_igemm<T, BM, BN, decltype(la), decltype(lb), decltype(e), NST, decltype(C)::WM>(la, lb, e, Nout, Kin, KTILES, sp, 1, st);
    });
  });
  return 0;
}

// fused QKV projection + bias + RoPE + head split. x: [B*Ntok, D] T ; w: [3D, D] T ; D = 64 H
int s3od_qkv_rope_fwd(int dtype, int B, int Ntok, int P, int H, const void* x, const void* w, const float* bias,
                      const float* cos_t, const float* sin_t, void* q, void* k, void* v, void* stream) {
  const int D = 64 * H, N = 3 * D, M = B * Ntok;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    return with_cfg<T>(4, [&](auto C) -> int {
      constexpr int BM = decltype(C)::BM, BN = decltype(C)::BN, NST = decltype(C)::NST;
      DenseKC<T, BM, decltype(C)::W> la{(const T*)x, (long)D, M, D, 0};
      DenseKC<T, BN, decltype(C)::W> lb{(const T*)w, (long)D, N, D, 0};
      EpiQKV<T> e{(T*)q, (T*)k, (T*)v, bias, cos_t, sin_t, M, Ntok, P, H};
      return launch_igemm<T, BM, BN, decltype(la), decltype(lb), decltype(e), NST, decltype(C)::WM>(la, lb, e, M, N, cdiv(D, KT<T>::BK), 1, 1, st);
    });
  });
  return 0;
}

// ---------------------------------------------------------------------------------- convs
// NHWC activations, weights repacked [Cout][KH][KW][Cin].
// pre = conv(relu?(x)) + bias[n]; out[b,oy,ox,n] = act(pre*scale[n] + shift[n]) (+res1 +res2);
// stats: BN batch sums of pre.
int s3od_conv_fwd(int dtype, int B, int H, int W, int Cin, int OH, int OW, int Cout, int KH, int KW,
                  int stride, int pad, const void* x, int relu_in, const void* wp,
                  const float* bias, const float* scale, const float* shift, int act, const void* res1, const void* res2,
                  void* out, void* pre, double* stats, float* colsum, void* stream) {
  S3OD_REQUIRE(Cin % 8 == 0 && Cout % 8 == 0, "conv_fwd: channels %% 8 (Cin=%d Cout=%d)", Cin, Cout);
  ConvGeo g{}; g.B = B; g.SH = H; g.SW = W; g.SC = Cin; g.RH = OH; g.RW = OW; g.KH = KH; g.KW = KW; g.s = stride; g.p = pad;
  const int M = B * OH * OW, N = Cout, K = KH * KW * Cin;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    const int KTILES = cdiv(K, KT<T>::BK);
    auto go = [&](auto bn, auto rl) -> int {
      return with_cfg<T>(Cout <= 64 ? 3 : 1, [&](auto C) -> int {
        constexpr int BM = decltype(C)::BM, NST = decltype(C)::NST;
        constexpr int BN = decltype(bn)::value < decltype(C)::BN ? decltype(bn)::value : decltype(C)::BN;
        ConvFwdA<T, BM, decltype(rl)::value, decltype(C)::W> la{}; la.x = (const T*)x; la.g = g; la.M = M; la.relu = relu_in;
        DenseKC<T, BN, decltype(C)::W> lb{(const T*)wp, (long)K, N, K, 0};
        EpiStd<T, T> e{(T*)out, (long)Cout, 0, bias, scale, shift, (const T*)res1, (long)Cout, (const T*)res2, (long)Cout,
                       (T*)pre, (long)Cout, stats, act, M, N, dense_rm(), colsum};
        return launch_igemm<T, BM, BN, decltype(la), decltype(lb), decltype(e), NST, decltype(C)::WM>(la, lb, e, M, N, KTILES, 1, 1, st);
      });
    };
    if (relu_in) {
      if (Cout <= 64) return go(std::integral_constant<int, 64>{}, std::true_type{});
      return go(std::integral_constant<int, 128>{}, std::true_type{});
    }
    if (Cout <= 64) return go(std::integral_constant<int, 64>{}, std::false_type{});
    return go(std::integral_constant<int, 128>{}, std::false_type{});
  });
  return 0;
}

// conv dgrad == ConvTranspose2d forward.  dy: [B,OH,OW,Cout] (conv output grid); w: [Cout][KH][KW][Cin];
// dx: [B,H,W,Cin] (conv input grid).  One launch per output parity class.
int s3od_conv_dgrad(int dtype, int B, int H, int W, int Cin, int OH, int OW, int Cout, int KH, int KW,
                    int stride, int pad, const void* dy, const void* wp,
                    const float* bias, const float* scale, const float* shift, int act, const void* res1,
                    const void* res2, void* dx, void* pre, double* stats, float* colsum, void* stream) {
  S3OD_REQUIRE(Cin % 8 == 0 && Cout % 8 == 0, "conv_dgrad: channels %% 8");
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
          return with_cfg<T>(Cin <= 64 ? 3 : 1, [&](auto C) -> int {
            constexpr int BM = decltype(C)::BM, NST = decltype(C)::NST;
            constexpr int BN = decltype(bn)::value < decltype(C)::BN ? decltype(bn)::value : decltype(C)::BN;
            ConvDgradA<T, BM, decltype(C)::W> la{}; la.dy = (const T*)dy; la.g = g; la.M = M;
            ConvDgradB<T, BN, decltype(C)::W> lb{}; lb.w = (const T*)wp; lb.g = g; lb.NC = Cin;
            EpiStd<T, T> e{(T*)dx, (long)Cin, 0, bias, scale, shift, (const T*)res1, (long)Cin, (const T*)res2, (long)Cin,
                           (T*)pre, (long)Cin, stats, act, M, N, rm, colsum};
            return launch_igemm<T, BM, BN, decltype(la), decltype(lb), decltype(e), NST, decltype(C)::WM>(la, lb, e, M, N, cdiv(K, KT<T>::BK), 1, 1, st);
          });
        };
        int rc = Cin <= 64 ? go(std::integral_constant<int, 64>{}) : go(std::integral_constant<int, 128>{});
        if (rc) return rc;
      }
  });
  return 0;
}

// conv wgrad: dw[Cout][Cin][KH][KW] (PyTorch layout, fp32) += sum_pix dy[pix][co] * x[src(pix,tap)][ci]
// dy: [B,OH,OW,Cout]; x: [B,H,W,Cin].  Also serves ConvTranspose2d weights (conv view).
int s3od_conv_wgrad(int dtype, int B, int H, int W, int Cin, int OH, int OW, int Cout, int KH, int KW,
                    int stride, int pad, const void* dy, const void* x, int relu_x, float* dw, float* ws, int split,
                    void* stream) {
  S3OD_REQUIRE(Cin % 8 == 0 && Cout % 8 == 0, "conv_wgrad: channels %% 8");
  ConvGeo g{}; g.B = B; g.SH = H; g.SW = W; g.SC = Cin; g.RH = OH; g.RW = OW; g.KH = KH; g.KW = KW; g.s = stride; g.p = pad;
  const int NPIX = B * OH * OW, M = Cout, N = KH * KW * Cin;
  hipStream_t st = (hipStream_t)stream;
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
      if (viaws) (void)hipMemsetAsync(ws, 0, sizeof(float) * (size_t)M * N, st);
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
