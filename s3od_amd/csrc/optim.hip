// Fused multi-tensor AdamW (torch.optim.AdamW semantics, lightning_module.py:183-193:
// weight_decay 0.05, betas (0.9, 0.999), eps 1e-8; per-tensor lr for the 2 param groups).
// One launch updates every parameter: a chunk table maps blocks -> (tensor, offset).
#include "common.hpp"

struct AdamTab {
  const long* ptrs;     // [T][4] device pointers: param, grad, exp_avg, exp_avg_sq
  const long* sizes;    // [T]
  const float* lrs;     // [T]
  const int* chunk_t;   // [C] tensor index of chunk
  const long* chunk_o;  // [C] element offset of chunk
};

__global__ void __launch_bounds__(256) adamw_kernel(AdamTab tab, int chunk, float beta1, float beta2, float eps, float wd,
                                                    float bc1, float bc2_sqrt) {
  const int c = blockIdx.x;
  const int t = tab.chunk_t[c];
  const long o0 = tab.chunk_o[c];
  const long n = tab.sizes[t];
  float* p = (float*)tab.ptrs[4 * t + 0];
  const float* g = (const float*)tab.ptrs[4 * t + 1];
  float* m = (float*)tab.ptrs[4 * t + 2];
  float* v = (float*)tab.ptrs[4 * t + 3];
  if (g == nullptr) return;
  const float lr = tab.lrs[t];
  const float step = lr / bc1;
  const long o1 = min(n, o0 + chunk);
  for (long i = o0 + threadIdx.x; i < o1; i += blockDim.x) {
    float pi = p[i] * (1.f - lr * wd);
    float gi = g[i];
    float mi = beta1 * m[i] + (1.f - beta1) * gi;
    float vi = beta2 * v[i] + (1.f - beta2) * gi * gi;
    m[i] = mi; v[i] = vi;
    float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = pi - step * mi / denom;
  }
}

extern "C" {

// ptrs: device int64 [ntensors][4]; sizes: device int64 [ntensors]; lrs: device f32 [ntensors];
// chunk_t / chunk_o: device chunk table of nchunks entries (chunk elements each).  step >= 1.
int s3od_adamw_step(const long* ptrs, const long* sizes, const float* lrs, const int* chunk_t, const long* chunk_o,
                    int nchunks, int chunk, int step, float beta1, float beta2, float eps, float wd, void* stream) {
  AdamTab tab{ptrs, sizes, lrs, chunk_t, chunk_o};
  double bc1 = 1.0 - pow((double)beta1, (double)step);
  double bc2 = 1.0 - pow((double)beta2, (double)step);
  hipLaunchKernelGGL(adamw_kernel, dim3(nchunks), dim3(256), 0, (hipStream_t)stream, tab, chunk, beta1, beta2, eps, wd, (float)bc1,
                     (float)sqrt(bc2));
  return s3od_check_launch("adamw_step");
}

}  // extern "C"
