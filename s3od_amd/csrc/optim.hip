// Fused multi-tensor AdamW (torch.optim.AdamW semantics, lightning_module.py:183-193:
// weight_decay 0.05, betas (0.9, 0.999), eps 1e-8; per-tensor lr for the 2 param groups).
// One launch updates every parameter: a chunk table maps blocks -> (tensor, offset).
#include "common.hpp"

struct AdamTab {
  const long* ptrs;     // [T][4] device pointers: param, grad, exp_avg, exp_avg_sq
  const long* sizes;    // [T]
  const float* coef;    // [T][2]: 1 - lr*wd, lr / (1 - beta1^step)   (host double -> f32, as torch)
  const int* chunk_t;   // [C] tensor index of chunk
  const long* chunk_o;  // [C] element offset of chunk
};

// torch.optim.AdamW single-tensor step (torch/optim/adamw.py -> adam.py _single_tensor_adam):
//   p *= 1 - lr*wd;  m.lerp_(g, 1-b1);  v = v*b2 + (1-b2)*g*g;  p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)
// with every scalar formed in double on the host (Python floats) and rounded to f32 once.
__global__ void __launch_bounds__(256) adamw_kernel(AdamTab tab, int chunk, float beta2, float omb1, float omb2, float eps,
                                                    float bc2_sqrt) {
  const int c = blockIdx.x;
  const int t = tab.chunk_t[c];
  const long o0 = tab.chunk_o[c];
  const long n = tab.sizes[t];
  float* p = (float*)tab.ptrs[4 * t + 0];
  const float* g = (const float*)tab.ptrs[4 * t + 1];
  float* m = (float*)tab.ptrs[4 * t + 2];
  float* v = (float*)tab.ptrs[4 * t + 3];
  if (g == nullptr) return;
  const float decay = tab.coef[2 * t], step = tab.coef[2 * t + 1];
  const long o1 = min(n, o0 + chunk);
  for (long i = o0 + threadIdx.x; i < o1; i += blockDim.x) {
    float pi = p[i] * decay;
    float gi = g[i], mo = m[i];
    float mi = omb1 < 0.5f ? mo + omb1 * (gi - mo) : gi - (gi - mo) * (1.f - omb1);   // at::lerp
    float vi = v[i] * beta2 + gi * gi * omb2;
    m[i] = mi; v[i] = vi;
    float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = pi + (-step) * (mi / denom);
  }
}

extern "C" {

// ptrs: device int64 [ntensors][4]; sizes: device int64 [ntensors]; coef: device f32 [ntensors][2]
// (1 - lr*wd, lr / (1 - beta1^step), formed in double by the caller); chunk_t / chunk_o: device chunk
// table of nchunks entries (chunk elements each).  step >= 1.
int s3od_adamw_step(const long* ptrs, const long* sizes, const float* coef, const int* chunk_t, const long* chunk_o,
                    int nchunks, int chunk, int step, double beta1, double beta2, double eps, void* stream) {
  AdamTab tab{ptrs, sizes, coef, chunk_t, chunk_o};
  double bc2 = 1.0 - pow(beta2, (double)step);
  hipLaunchKernelGGL(adamw_kernel, dim3(nchunks), dim3(256), 0, (hipStream_t)stream, tab, chunk, (float)beta2, (float)(1.0 - beta1),
                     (float)(1.0 - beta2), (float)eps, (float)sqrt(bc2));
  return s3od_check_launch("adamw_step");
}

}  // extern "C"
