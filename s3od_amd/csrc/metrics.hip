// SOD evaluation metrics on device: synth_sod/src/synth_sod/model_training/metrics.py:213-424
// (EvaluationMetrics.step: MAE, MaxF/AvgF over 255 thresholds, S-measure) with :14-137 (EMeasure,
// changeable E-measure over 256 uint8 thresholds) and :140-210 (WeightedFMeasure, exact Euclidean
// distance transform with nearest-feature indices + 7x7 sigma-5 Gaussian).
//
// One image per call (the reference steps image by image at the image's own size).  HBM-bound
// byte/float work: every pass is a coalesced grid-stride sweep over the H*W plane with block-level
// LDS reductions and one global (vector) atomic per block and accumulator; the only serial work is
// the distance transform's 1D lower envelopes (one thread per column / per row).
//
// Pass order on `stream`:
//   stats   : MAE, sum gt, binarised-mask moments (S_object), centroid moments, PR histogram
//             (bin = last threshold <= p), uint8 E-measure histograms, EDT-free
//   region  : centroid -> quadrant moments (S_region); optional in-place binarisation of gt
//   edt_col : nearest foreground row per column (ties -> lower row)
//   edt_row : Maurer lower envelope per row (strict remove / strict advance: ties -> lower column),
//             which reproduces scipy.ndimage.distance_transform_edt(return_indices=True)'s choice
//   wf_et   : E = |p - g|, Et = E at the nearest foreground pixel
//   wf_sum  : EA = f32(7x7 Gaussian of Et, zero border), Ew sums
//   final   : one block: E-measure curve, F curve, S-measure, weighted F -> out[6]
#include "common.hpp"

namespace {

constexpr int NT = 255;          // PR thresholds (metrics.py:251)
constexpr int TB = 256;          // threads per block for the sweeps
constexpr double EPS = 2.220446049250313e-16;   // np.spacing(1)

// accumulator slots (double) at the start of the workspace
enum {
  A_MAE = 0, A_YSUM, A_N1, A_FG1, A_FG2, A_BG1, A_BG2, A_CX, A_CY, A_PSUM,
  A_EWFG, A_EWBG, A_NSCAL
};
// quadrant moments: [4][6] = n, sp, sm, spp, smm, spm
constexpr int Q_OFF = 16;
constexpr int H_CNT = Q_OFF + 24;            // u64 [256] pixels per PR bin
constexpr int H_TP = H_CNT + 256;            // double [256] gt mass per PR bin
constexpr int H_FG = H_TP + 256;             // u64 [256] uint8 histogram of pred on gt
constexpr int H_BG = H_FG + 256;             // u64 [256] uint8 histogram of pred off gt
constexpr int ACC_WORDS = H_BG + 256;        // 8-byte words

struct Tables {
  float thr[NT];     // torch.linspace(0, 1 - 1e-10, 255) float32
  double k7[49];     // matlab_style_gauss2D((7,7), 5)
};

DEV double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// block-wide sum of NV doubles, thread 0 adds them to dst[slot[i]]
template <int NV>
DEV void block_add(double (&v)[NV], double* acc, const int (&slot)[NV]) {
  __shared__ double red[TB / 64][NV];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; i++) {
    double s = wave_sum(v[i]);
    if (lane == 0) red[w][i] = s;
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    double s = 0.0;
    for (int j = 0; j < TB / 64; j++) s += red[j][threadIdx.x];
    // NV <= 64: one lane per accumulator
    int i = threadIdx.x;
    atomicAdd(acc + slot[i], s);
  }
}

DEV int pr_bin(const float* thr, float p) {     // largest i with thr[i] <= p, -1 if none
  int lo = 0, hi = NT;                            // invariant: thr[<lo] <= p, thr[>=hi] > p
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (thr[mid] <= p) lo = mid + 1; else hi = mid;
  }
  return lo - 1;
}

__global__ void __launch_bounds__(TB) stats_kernel(const float* __restrict__ pred, const float* __restrict__ gt, long N, int W,
                                                   Tables T, int sm_only, double* __restrict__ acc) {
  __shared__ float thr[NT];
  __shared__ unsigned long long hc[256], hf[256], hb[256];
  __shared__ double ht[256];
  for (int i = threadIdx.x; i < NT; i += TB) thr[i] = T.thr[i];
  hc[threadIdx.x] = hf[threadIdx.x] = hb[threadIdx.x] = 0ull;
  ht[threadIdx.x] = 0.0;
  __syncthreads();
  double v[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (long i = blockIdx.x * (long)TB + threadIdx.x; i < N; i += (long)gridDim.x * TB) {
    const float p = pred[i], m = gt[i];
    const double pd = p, md = m;
    v[0] += fabs(pd - md);                       // |pred - mask| in float64 (pred f32, mask f64)
    v[1] += md;
    v[9] += pd;
    if (m >= 0.5f) {                             // binarised mask (metrics.py:239-240)
      const long y = i / W, x = i - y * W;
      v[2] += 1.0; v[3] += pd; v[4] += pd * pd; v[7] += (double)x; v[8] += (double)y;
    } else {                                     // bg = 1 - pred (float32 in the reference)
      const double q = (double)(1.f - p);
      v[5] += q; v[6] += q * q;
    }
    if (!sm_only) {
      const int b = pr_bin(thr, p);
      if (b >= 0) {
        atomicAdd(&hc[b], 1ull);
        atomicAdd(&ht[b], md);
      }
      float s = p * 255.f;                       // (pred * 255).astype(np.uint8): truncation
      s = fminf(fmaxf(s, 0.f), 255.f);
      const int u = (int)s;
      if (m >= 0.5f) atomicAdd(&hf[u], 1ull); else atomicAdd(&hb[u], 1ull);
    }
  }
  const int slot[10] = {A_MAE, A_YSUM, A_N1, A_FG1, A_FG2, A_BG1, A_BG2, A_CX, A_CY, A_PSUM};
  block_add<10>(v, acc, slot);
  if (!sm_only) {
    __syncthreads();
    const int t = threadIdx.x;
    unsigned long long* acc_u = (unsigned long long*)acc;
    if (hc[t]) atomicAdd(acc_u + H_CNT + t, hc[t]);
    if (ht[t] != 0.0) atomicAdd(acc + H_TP + t, ht[t]);
    if (hf[t]) atomicAdd(acc_u + H_FG + t, hf[t]);
    if (hb[t]) atomicAdd(acc_u + H_BG + t, hb[t]);
  }
}

// centroid (metrics.py:358-378): round-half-even of the exact mean coordinate; empty mask -> round(dim/2)
DEV void centroid(const double* acc, int H, int W, long& X, long& Y) {
  const double n1 = acc[A_N1];
  if (n1 == 0.0) {
    X = (long)rint(W / 2.0); Y = (long)rint(H / 2.0);
  } else {
    X = (long)rint(acc[A_CX] / n1); Y = (long)rint(acc[A_CY] / n1);
  }
}

__global__ void __launch_bounds__(TB) region_kernel(const float* __restrict__ pred, float* __restrict__ gt, int H, int W,
                                                    int binarize, double* __restrict__ acc) {
  long X, Y;
  centroid(acc, H, W, X, Y);
  const long N = (long)H * W;
  const double ysum = acc[A_YSUM];
  const bool special = ysum == 0.0 || ysum == (double)N;   // y == 0 / y == 1: no binarisation
  double v[24];
#pragma unroll
  for (int j = 0; j < 24; j++) v[j] = 0.0;
  for (long i = blockIdx.x * (long)TB + threadIdx.x; i < N; i += (long)gridDim.x * TB) {
    const long y = i / W, x = i - y * W;
    const float m = gt[i];
    const double p = pred[i], mb = m >= 0.5f ? 1.0 : 0.0;
    const int q = (y < Y ? 0 : 2) + (x < X ? 0 : 1);     // LT, RT, LB, RB
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (k == q) {
        v[6 * k + 0] += 1.0; v[6 * k + 1] += p; v[6 * k + 2] += mb;
        v[6 * k + 3] += p * p; v[6 * k + 4] += mb * mb; v[6 * k + 5] += p * mb;
      }
    }
    if (binarize && !special) gt[i] = m >= 0.5f ? 1.f : 0.f;
  }
  int slot[24];
#pragma unroll
  for (int j = 0; j < 24; j++) slot[j] = Q_OFF + j;
  block_add<24>(v, acc, slot);
}

// nearest foreground row in each column (scipy's first-axis pass; ties -> lower row).  One thread
// per column; rows are read 16 at a time so each thread keeps 16 independent loads in flight.
__global__ void edt_col_kernel(const float* __restrict__ gt, int H, int W, int* __restrict__ feat) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= W) return;
  constexpr int R = 16;
  int last = -1;
  for (int y0 = 0; y0 < H; y0 += R) {            // nearest foreground at or above
    float g[R];
#pragma unroll
    for (int r = 0; r < R; r++) g[r] = y0 + r < H ? gt[(long)(y0 + r) * W + x] : 0.f;
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (y0 + r < H) {
        if (g[r] >= 0.5f) last = y0 + r;
        feat[(long)(y0 + r) * W + x] = last;
      }
    }
  }
  int next = -1;
  for (int y1 = H - 1; y1 >= 0; y1 -= R) {       // nearest foreground at or below; the upper one wins ties
    float g[R];
    int up[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int y = y1 - r;
      g[r] = y >= 0 ? gt[(long)y * W + x] : 0.f;
      up[r] = y >= 0 ? feat[(long)y * W + x] : -1;
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int y = y1 - r;
      if (y >= 0) {
        if (g[r] >= 0.5f) next = y;
        int best = up[r];
        if (next >= 0 && (best < 0 || (next - y) < (y - best))) best = next;
        feat[(long)y * W + x] = best;
      }
    }
  }
}

// per row: Maurer's lower envelope of the column features (remove when c*dv - b*du - a*dw - a*b*c > 0,
// advance while d(l) > d(l+1)); frow/gx/gd live in LDS when the row fits, else in global scratch
DEV void envelope_row(const int* frow, int y, int W, int* gx, int* gd, int* __restrict__ idx_row, int* __restrict__ d2_row) {
  int n = 0;
  for (int x = 0; x < W; x++) {
    const int fy = frow[x];
    if (fy < 0) continue;
    const int dw = (fy - y) * (fy - y);
    while (n >= 2) {
      const long long u = gx[n - 2], v = gx[n - 1], du = gd[n - 2], dv = gd[n - 1];
      const long long a = v - u, b = x - v, c = x - u;
      if (c * dv - b * du - a * (long long)dw - a * b * c > 0) n--;
      else break;
    }
    gx[n] = x; gd[n] = dw; n++;
  }
  if (n == 0) {                                  // no foreground anywhere in the image
    for (int x = 0; x < W; x++) { idx_row[x] = -1; d2_row[x] = 0; }
    return;
  }
  int l = 0;
  for (int x = 0; x < W; x++) {
    while (l < n - 1) {
      const long long d1 = gd[l] + (long long)(gx[l] - x) * (gx[l] - x);
      const long long d2 = gd[l + 1] + (long long)(gx[l + 1] - x) * (gx[l + 1] - x);
      if (d1 > d2) l++; else break;
    }
    const int fx = gx[l], fy = frow[fx];
    idx_row[x] = fy * W + fx;
    d2_row[x] = gd[l] + (fx - x) * (fx - x);
  }
}

constexpr int EDT_LDS_W = 4096;

__global__ void __launch_bounds__(64) edt_row_kernel(const int* __restrict__ feat, int H, int W, int* __restrict__ idx,
                                                     int* __restrict__ d2, int* __restrict__ sx, int* __restrict__ sd) {
  __shared__ int fr[EDT_LDS_W], gx[EDT_LDS_W], gd[EDT_LDS_W];
  const int y = blockIdx.x;
  const long o = (long)y * W;
  if (W <= EDT_LDS_W) {
    for (int x = threadIdx.x; x < W; x += 64) fr[x] = feat[o + x];     // coalesced row copy
    __syncthreads();
    if (threadIdx.x == 0) envelope_row(fr, y, W, gx, gd, idx + o, d2 + o);
  } else if (threadIdx.x == 0) {
    envelope_row(feat + o, y, W, sx + o, sd + o, idx + o, d2 + o);
  }
}

__global__ void __launch_bounds__(TB) wf_et_kernel(const float* __restrict__ pred, const float* __restrict__ gt, long N,
                                                   const int* __restrict__ idx, float* __restrict__ et) {
  for (long i = blockIdx.x * (long)TB + threadIdx.x; i < N; i += (long)gridDim.x * TB) {
    const bool g = gt[i] >= 0.5f;
    float e;
    if (g) {
      e = fabsf(pred[i] - 1.f);
    } else {
      const int j = idx[i];
      e = j >= 0 ? fabsf(pred[j] - 1.f) : fabsf(pred[i]);   // Et = E at the nearest foreground pixel
    }
    et[i] = e;
  }
}

__global__ void __launch_bounds__(TB) wf_sum_kernel(const float* __restrict__ pred, const float* __restrict__ gt, int H, int W,
                                                    const float* __restrict__ et, const int* __restrict__ d2, Tables T,
                                                    double* __restrict__ acc) {
  __shared__ double k7[49];
  if (threadIdx.x < 49) k7[threadIdx.x] = T.k7[threadIdx.x];
  __syncthreads();
  const long N = (long)H * W;
  const double c5 = log(0.5) / 5.0;
  double v[2] = {0.0, 0.0};
  for (long i = blockIdx.x * (long)TB + threadIdx.x; i < N; i += (long)gridDim.x * TB) {
    const long y = i / W, x = i - y * W;
    double s = 0.0;                                // scipy.ndimage.convolve(mode="constant", cval=0)
    for (int dy = -3; dy <= 3; dy++) {
      const long yy = y + dy;
      if (yy < 0 || yy >= H) continue;
      for (int dx = -3; dx <= 3; dx++) {
        const long xx = x + dx;
        if (xx < 0 || xx >= W) continue;
        s += k7[(3 - dy) * 7 + (3 - dx)] * (double)et[yy * W + xx];
      }
    }
    const float ea = (float)s;                     // output keeps the input dtype (float32)
    const bool g = gt[i] >= 0.5f;
    const float e = g ? fabsf(pred[i] - 1.f) : fabsf(pred[i]);
    const float mn = (g && ea < e) ? ea : e;
    if (g) v[0] += (double)mn;
    else v[1] += (double)mn * (2.0 - exp(c5 * sqrt((double)d2[i])));
  }
  const int slot[2] = {A_EWFG, A_EWBG};
  block_add<2>(v, acc, slot);
}

DEV float fsc(float prec, float rec) {            // (1 + 0.3) * prec * recall / (0.3 * prec + recall), f32 ops
  const float num = (1.3f * prec) * rec;
  const float den = 0.3f * prec + rec;
  const float f = num / den;
  return f != f ? 0.f : f;
}

// S-measure SSIM of one quadrant (metrics.py:405-424) from its moments
DEV double q_ssim(const double* q) {
  const double n = q[0];
  const double x = q[1] / n, y = q[2] / n;
  const double sx2 = (q[3] - n * x * x) / (n - 1 + 1e-20);
  const double sy2 = (q[4] - n * y * y) / (n - 1 + 1e-20);
  const double sxy = (q[5] - n * x * y) / (n - 1 + 1e-20);
  const double al = 4 * x * y * sxy, be = (x * x + y * y) * (sx2 + sy2);
  if (al != 0.0) return al / (be + 1e-20);       // NaN (empty quadrant) lands here, as in the reference
  if (be == 0.0) return 1.0;
  return 0.0;
}

DEV double o_score(double n, double s1, double s2) {   // _object: 2x / (x^2 + 1 + std + 1e-20), unbiased std
  const double x = s1 / n;
  const double var = (s2 - n * x * x) / (n - 1);
  const double sd = sqrt(var < 0.0 ? 0.0 : var);           // n == 1 -> 0/0 = NaN, as torch.std
  return 2.0 * x / (x * x + 1.0 + sd + 1e-20);
}

__global__ void __launch_bounds__(256) final_kernel(const double* __restrict__ acc, int H, int W, int sm_only,
                                                    double* __restrict__ out) {
  __shared__ double red[256];
  __shared__ float fs[256];
  const int t = threadIdx.x;
  const long N = (long)H * W;
  const double Nd = (double)N;
  const unsigned long long* acc_u = (const unsigned long long*)acc;
  // ---- S-measure (every thread computes it; thread 0 writes)
  double S;
  {
    const double y = acc[A_YSUM] / Nd, xm = acc[A_PSUM] / Nd;
    if (y == 0.0) S = 1.0 - xm;
    else if (y == 1.0) S = xm;
    else {
      const double n1 = acc[A_N1], n0 = Nd - n1, u = n1 / Nd;
      const double ofg = o_score(n1, acc[A_FG1], acc[A_FG2]);
      const double obg = o_score(n0, acc[A_BG1], acc[A_BG2]);
      const double so = u * ofg + (1 - u) * obg;
      long X, Y;
      centroid(acc, H, W, X, Y);
      const double area = Nd;
      const double w1 = (double)X * Y / area, w2 = (double)(W - X) * Y / area, w3 = (double)X * (H - Y) / area;
      const double w4 = 1 - w1 - w2 - w3;
      const double* q = acc + Q_OFF;
      const double sr = w1 * q_ssim(q) + w2 * q_ssim(q + 6) + w3 * q_ssim(q + 12) + w4 * q_ssim(q + 18);
      S = 0.5 * so + 0.5 * sr;
      if (S < 0) S = 0.0;
    }
  }
  if (sm_only) {
    if (t == 0) { out[0] = 0; out[1] = 0; out[2] = 0; out[3] = S; out[4] = 0; out[5] = 0; }
    return;
  }
  // ---- PR curve: counts of p >= thr[i] are suffix sums over the bins
  __shared__ double cnt_s[256], tp_s[256];
  cnt_s[t] = t < NT ? (double)acc_u[H_CNT + t] : 0.0;
  tp_s[t] = t < NT ? acc[H_TP + t] : 0.0;
  __syncthreads();
  if (t == 0) {                                   // 255-long suffix scan: trivial, serial
    double c = 0, p = 0;
    for (int i = NT - 1; i >= 0; i--) { c += cnt_s[i]; p += tp_s[i]; cnt_s[i] = c; tp_s[i] = p; }
  }
  __syncthreads();
  const double ysum = acc[A_YSUM];
  if (t < NT) {
    const float cnt = (float)cnt_s[t];            // y_temp.sum() in float32 (+1e-20 is absorbed unless 0)
    const double den = cnt == 0.f ? (double)1e-20f : (double)cnt;
    const float prec = (float)(tp_s[t] / den);
    const float rec = (float)(tp_s[t] / (ysum + 1e-20));
    fs[t] = fsc(prec, rec);
  }
  __syncthreads();
  // ---- E-measure over the 256 uint8 thresholds (metrics.py:80-110, 112-132)
  {
    // thresholds k = 0..255 count pred values >= 255 - k (cumsum of the flipped histogram)
    __shared__ double ff[256], fb[256];
    ff[t] = (double)acc_u[H_FG + 255 - t];
    fb[t] = (double)acc_u[H_BG + 255 - t];
    __syncthreads();
    if (t == 0) {
      double a = 0, b = 0;
      for (int i = 0; i < 256; i++) { a += ff[i]; b += fb[i]; ff[i] = a; fb[i] = b; }
    }
    __syncthreads();
    const double gfg = acc[A_N1], gsz = Nd;
    const double fgfg = ff[t], fgbg = fb[t], predfg = fgfg + fgbg, predbg = gsz - predfg;
    double em_sum;
    if (gfg == 0.0) em_sum = predbg;
    else if (gfg == gsz) em_sum = predfg;
    else {
      const double bgfg = gfg - fgfg, bgbg = predbg - bgfg;
      const double mp = predfg / gsz, mg = gfg / gsz;
      const double parts[4] = {fgfg, fgbg, bgfg, bgbg};
      const double cp[4] = {1 - mp, 1 - mp, 0 - mp, 0 - mp}, cg[4] = {1 - mg, 0 - mg, 1 - mg, 0 - mg};
      em_sum = 0.0;
      for (int i = 0; i < 4; i++) {
        const double al = 2 * (cp[i] * cg[i]) / (cp[i] * cp[i] + cg[i] * cg[i] + EPS);
        const double en = (al + 1) * (al + 1) / 4;
        em_sum += en * parts[i];
      }
    }
    red[t] = em_sum / (gsz - 1 + EPS);
  }
  __syncthreads();
  if (t == 0) {
    double em = 0.0;
    for (int i = 0; i < 256; i++) em += red[i];
    float mx = fs[0];
    double fsum = 0.0;
    for (int i = 0; i < NT; i++) { mx = fmaxf(mx, fs[i]); fsum += fs[i]; }
    // weighted F (metrics.py:147-191): 0 when the mask has no foreground
    double wf = 0.0;
    const double ng = acc[A_N1];
    if (ng > 0) {
      const double tpw = ng - acc[A_EWFG], fpw = acc[A_EWBG];
      const double R = 1 - acc[A_EWFG] / ng, P = tpw / (tpw + fpw + EPS);
      wf = (1 + 1.0) * R * P / (R + 1.0 * P + EPS);
    }
    out[0] = acc[A_MAE] / Nd;
    out[1] = (double)mx;
    out[2] = (double)(float)(fsum / NT);
    out[3] = S;
    out[4] = em / 256.0;
    out[5] = wf;
  }
}

inline int sweep_grid(long N) { return (int)std::min<long>(2048, std::max<long>(1, (N + TB - 1) / TB)); }

}  // namespace

extern "C" {

static long ws_bytes_for(int H, int W) {
  const long N = (long)H * W;
  return (long)ACC_WORDS * 8 + N * 4 /*feat*/ + N * 4 /*idx*/ + N * 4 /*d2*/ + N * 4 /*et*/ +
         (W > EDT_LDS_W ? N * 8 : 0) /*envelope scratch*/;
}

// *bytes (host) = scratch s3od_eval_metrics needs for an H x W image
int s3od_eval_metrics_ws(int H, int W, long* bytes) {
  S3OD_REQUIRE(bytes && H > 0 && W > 0, "eval_metrics_ws: bad arguments");
  *bytes = ws_bytes_for(H, W);
  return 0;
}

// pred: fp32 [H][W] soft mask in [0,1]; gt: fp32 [H][W] in [0,1] (binarised in place at 0.5 when
// `binarize` and the mask is neither all-0 nor all-1, as metrics.py:239-240 does to the caller's
// tensor); thr: host float[255] = torch.linspace(0, 1 - 1e-10, 255); k7: host double[49] =
// matlab_style_gauss2D((7, 7), 5); ws: device scratch of s3od_eval_metrics_ws(H, W) bytes;
// out: device double[6] = MAE, MaxF, AvgF, S-measure, E-measure (mean of the 256-point curve), weighted F
// (sm_only: only out[3] is meaningful).
int s3od_eval_metrics(const float* pred, float* gt, int H, int W, const float* thr, const double* k7, void* ws, long ws_bytes,
                      int sm_only, int binarize, double* out, void* stream) {
  S3OD_REQUIRE(pred && gt && ws && out && thr && k7, "eval_metrics: null pointer");
  S3OD_REQUIRE(H >= 2 && W >= 2 && H <= 32768 && W <= 32768, "eval_metrics: image must be 2..32768 on each side");
  S3OD_REQUIRE(ws_bytes >= ws_bytes_for(H, W), "eval_metrics: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const long N = (long)H * W;
  Tables T;
  for (int i = 0; i < NT; i++) T.thr[i] = thr[i];
  for (int i = 0; i < 49; i++) T.k7[i] = k7[i];
  char* w = (char*)ws;
  double* acc = (double*)w;
  int* feat = (int*)(w + (long)ACC_WORDS * 8);
  int* idx = feat + N;
  int* d2 = idx + N;
  float* et = (float*)(d2 + N);
  int* sx = (int*)(et + N);
  int* sd = sx + (W > EDT_LDS_W ? N : 0);
  hipError_t e = hipMemsetAsync(acc, 0, (size_t)ACC_WORDS * 8, st);
  if (e != hipSuccess) return (int)e;
  const int g = sweep_grid(N);
  hipLaunchKernelGGL(stats_kernel, dim3(g), dim3(TB), 0, st, pred, (const float*)gt, N, W, T, sm_only, acc);
  if (!sm_only) {
    // the distance transform reads gt before region_kernel may binarise it (same foreground either way)
    hipLaunchKernelGGL(edt_col_kernel, dim3(cdiv(W, 64)), dim3(64), 0, st, (const float*)gt, H, W, feat);
    hipLaunchKernelGGL(edt_row_kernel, dim3(H), dim3(64), 0, st, (const int*)feat, H, W, idx, d2, sx, sd);
    hipLaunchKernelGGL(wf_et_kernel, dim3(g), dim3(TB), 0, st, pred, (const float*)gt, N, (const int*)idx, et);
    hipLaunchKernelGGL(wf_sum_kernel, dim3(g), dim3(TB), 0, st, pred, (const float*)gt, H, W, (const float*)et,
                       (const int*)d2, T, acc);
  }
  hipLaunchKernelGGL(region_kernel, dim3(g), dim3(TB), 0, st, pred, gt, H, W, binarize, acc);
  hipLaunchKernelGGL(final_kernel, dim3(1), dim3(256), 0, st, (const double*)acc, H, W, sm_only, out);
  return s3od_check_launch("eval_metrics");
}

}  // extern "C"
