// Store-path microbenchmark (dev tool, GPU box): the ping-pong GEMM's epilogue write pattern in isolation.
// 3072 blocks of 512 threads write a 256 x 256 bf16 tile each into a 65536 x 3072 bf16 matrix (the up-projection
// output), tiles assigned like the GEMM (XCD-contiguous, row-major over 256 x 12 tiles):
//   mode 0: straight from registers, 16 B per thread per row segment (the for_segments mapping)
//   mode 1: through LDS -- fp32 128 x 260 staging per half, barrier, read back, convert, store (the pp epilogue)
//   mode 2: mode 0 preceded by a dummy 30 us spin, so blocks desynchronise like the GEMM's rounds
// Build + run: hipcc --offload-arch=gfx950 -O3 tools/micro/store_bench.hip -o /tmp/store_bench && /tmp/store_bench
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <cstdio>

typedef __hip_bfloat16 bf16;

__device__ __forceinline__ void tile_of_block(int& mt, int& nt) {
  const int nN = gridDim.x, nwg = gridDim.x * gridDim.y;
  const int L = blockIdx.y * nN + blockIdx.x;
  const int q = nwg >> 3, r = nwg & 7, xcd = L & 7, idx = L >> 3;
  const int W = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  mt = W / nN; nt = W % nN;
}

template <int MODE>
__global__ void __launch_bounds__(512) store_kernel(bf16* out, int N, float seed) {
  __shared__ float ct[128 * 260];
  int mt, nt;
  tile_of_block(mt, nt);
  const int tid = threadIdx.x, cs = tid % 32, r0 = tid / 32;
  if (MODE == 2) {
    long long t0 = clock64();
    while (clock64() - t0 < 60000) { }
  }
  for (int h = 0; h < 2; h++) {
    if (MODE == 1) {
      __syncthreads();
      for (int i = tid; i < 128 * 64; i += 512) {
        const int r = i / 64, c = (i % 64) * 4;
        *(float4*)(ct + r * 260 + c) = make_float4(seed + i, seed - i, seed * i, seed + 2 * i);
      }
      __syncthreads();
    }
#pragma unroll
    for (int it = 0; it < 8; it++) {
      const int r = r0 + it * 16;
      float v[8];
      if (MODE == 1) {
        const float4* src = (const float4*)(ct + r * 260 + cs * 8);
        float4 a = src[0], b = src[1];
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      } else {
#pragma unroll
        for (int e = 0; e < 8; e++) v[e] = seed * (r + e) + cs;
      }
      const long row = (long)mt * 256 + h * 128 + r;
      uint4 u;
      unsigned* pu = (unsigned*)&u;
#pragma unroll
      for (int e = 0; e < 4; e++) {
        bf16 lo = __float2bfloat16(v[2 * e]), hi = __float2bfloat16(v[2 * e + 1]);
        pu[e] = (unsigned)__bfloat16_as_ushort(lo) | ((unsigned)__bfloat16_as_ushort(hi) << 16);
      }
      *(uint4*)(out + row * N + nt * 256 + cs * 8) = u;
    }
  }
}

template <int MODE> float run(bf16* out, int reps, int rows = 256) {
  dim3 grid(12, rows);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  store_kernel<MODE><<<grid, 512>>>(out, 3072, 1.0f);
  hipEventRecord(e0);
  for (int i = 0; i < reps; i++) store_kernel<MODE><<<grid, 512>>>(out, 3072, 1.0f + i);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.f / reps;
}

int main() {
  bf16* out;
  const size_t bytes = 65536ull * 3072 * 2;
  if (hipMalloc(&out, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipMemset(out, 0, bytes);
  hipEventRecord(e0);
  for (int i = 0; i < 10; i++) hipMemsetAsync(out, i, bytes);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("hipMemset 403 MB: %.1f us (%.2f TB/s)\n", ms * 100.f, bytes / (ms / 10 * 1e-3) / 1e12);
  float t0 = run<0>(out, 10), t1 = run<1>(out, 10), t2 = run<2>(out, 10);
  printf("mode 0 (registers):       %.1f us  %.2f TB/s  %.2f us per round of 256 blocks\n", t0, bytes / (t0 * 1e-6) / 1e12, t0 / 12);
  printf("mode 1 (LDS staged):      %.1f us  %.2f TB/s  %.2f us per round\n", t1, bytes / (t1 * 1e-6) / 1e12, t1 / 12);
  printf("mode 2 (30 us spin + 0):  %.1f us  (spin-only would be ~%.0f us)\n", t2, 12 * 60000 / 2100.0);
  // fewer blocks than CUs: per-block store time with most of the chip idle (per-CU store path vs HBM)
  for (int rows : {1, 2, 5, 10, 21}) {
    const float t = run<0>(out, 10, rows), tl = run<1>(out, 10, rows);
    printf("%4d blocks: registers %.2f us, LDS staged %.2f us per block-tile (128 KB)\n", 12 * rows, t, tl);
  }
  hipFree(out);
  return 0;
}
