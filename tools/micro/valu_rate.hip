// VALU issue-rate microbenchmark (dev tool, GPU box): cycles per wave64 instruction for v_exp_f32 (transcendental),
// v_fma_f32, v_pk_fma_f32 and a mix, 1 .. 4 waves per SIMD.   hipcc --offload-arch=gfx950 -O3 valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ void k(float* out, int iters, float seed) {
  float a0 = seed + threadIdx.x, a1 = a0 * 1.1f, a2 = a0 * 1.2f, a3 = a0 * 1.3f, a4 = a0 * 1.4f, a5 = a0 * 1.5f, a6 = a0 * 1.6f, a7 = a0 * 1.7f;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
      if (OP == 0) {   // 8 independent v_exp_f32
        asm volatile("v_exp_f32 %0, %0\n v_exp_f32 %1, %1\n v_exp_f32 %2, %2\n v_exp_f32 %3, %3\n v_exp_f32 %4, %4\n v_exp_f32 %5, %5\n v_exp_f32 %6, %6\n v_exp_f32 %7, %7"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
      } else if (OP == 1) {   // 8 independent v_fma_f32
        asm volatile("v_fma_f32 %0, %0, %0, %1\n v_fma_f32 %1, %1, %1, %2\n v_fma_f32 %2, %2, %2, %3\n v_fma_f32 %3, %3, %3, %4\n v_fma_f32 %4, %4, %4, %5\n v_fma_f32 %5, %5, %5, %6\n v_fma_f32 %6, %6, %6, %7\n v_fma_f32 %7, %7, %7, %0"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
      } else if (OP == 2) {   // 4 independent v_pk_fma_f32 (8 fp32 FMAs)
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7};
        asm volatile("v_pk_fma_f32 %0, %0, %0, %1\n v_pk_fma_f32 %1, %1, %1, %2\n v_pk_fma_f32 %2, %2, %2, %3\n v_pk_fma_f32 %3, %3, %3, %0\n"
                     "v_pk_fma_f32 %0, %0, %0, %1\n v_pk_fma_f32 %1, %1, %1, %2\n v_pk_fma_f32 %2, %2, %2, %3\n v_pk_fma_f32 %3, %3, %3, %0"
                     : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3));
        a0 = p0.x; a1 = p0.y; a2 = p1.x; a3 = p1.y; a4 = p2.x; a5 = p2.y; a6 = p3.x; a7 = p3.y;
      } else {   // 4 exp + 4 fma interleaved
        asm volatile("v_exp_f32 %0, %0\n v_fma_f32 %1, %1, %1, %2\n v_exp_f32 %2, %2\n v_fma_f32 %3, %3, %3, %4\n v_exp_f32 %4, %4\n v_fma_f32 %5, %5, %5, %6\n v_exp_f32 %6, %6\n v_fma_f32 %7, %7, %7, %0"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

template <int OP> void run(const char* name, float* out, int wps) {
  const int iters = 4096, blocks = 256, threads = 256 * wps;   // one block per CU, wps waves per SIMD
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(threads), 0, 0, out, 16, 1.0f);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  // instructions per wave: iters * 8 unroll * 8 (OP 2: 8 pk instructions too)
  const double inst = (double)iters * 8 * 8 * wps;           // per SIMD
  const double ns_per = ms * 1e6 / inst;
  printf("%-34s waves/SIMD %d: %.3f ns per wave-instruction per SIMD (%.2f cycles at 2.4 GHz)\n", name, wps, ns_per, ns_per * 2.4);
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 1024 * sizeof(float));
  for (int w : {1, 2, 4}) {
    run<0>("v_exp_f32", out, w);
    run<1>("v_fma_f32", out, w);
    run<2>("v_pk_fma_f32", out, w);
    run<3>("exp/fma interleaved", out, w);
  }
  return 0;
}
