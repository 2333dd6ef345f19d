// hipBLASLt for the PLAIN linear data gradients (no epilogue beyond an optional in-place accumulate): the task's
// rule -- hand-written kernels for the fused hot ops, the library for plain GEMMs -- and measured: on the ViT
// backward's up-projection / QKV data gradients (dx[65616, 768] = dy[., 3072 | 2304] . w) hipBLASLt runs 1.24-1.35x
// faster than the ping-pong kernel, whose advantage is its fused epilogues (profiles/r06h_dgrad_vs_hipblaslt.txt).
//
// Row-major D[M][N] = A[M][K] . B[K][N] (+ C[M][N]) is column-major D^T = B^T . A^T: hipBLASLt's "A" is the row-major
// B viewed column-major (N x K, ld = ldb), its "B" the row-major A (K x M, ld = lda), D / C column-major N x M with
// their row strides as ld.  bf16 in / out, fp32 compute and scale; no workspace (the C ABI allocates nothing).
// Descriptors and the heuristic's algorithm are cached per shape; a shape the heuristic returns nothing for (or any
// hipBLASLt error) makes blaslt_gemm_rm return nonzero and the caller runs its own kernel.
#include "common.hpp"
#include <hipblaslt/hipblaslt.h>
#include <map>
#include <mutex>
#include <tuple>

namespace {
struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo;
  bool ok = false;
};
typedef std::tuple<int, int, int, long, long, long, long, int, int> Key;   // M N K lda ldb ldc ldd beta device

std::mutex mu;
std::map<int, hipblasLtHandle_t> handles;
std::map<Key, Plan> plans;

hipblasLtHandle_t handle_for(int dev) {
  auto it = handles.find(dev);
  if (it != handles.end()) return it->second;
  hipblasLtHandle_t h = nullptr;
  if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) h = nullptr;
  handles[dev] = h;
  return h;
}

Plan make_plan(hipblasLtHandle_t h, int M, int N, int K, long lda, long ldb, long ldc, long ldd, bool beta) {
  Plan p;
  bool good = hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) == HIPBLAS_STATUS_SUCCESS;
  const hipblasOperation_t nt = HIPBLAS_OP_N;
  good = good && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &nt, sizeof(nt)) == HIPBLAS_STATUS_SUCCESS;
  good = good && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &nt, sizeof(nt)) == HIPBLAS_STATUS_SUCCESS;
  good = good && hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, N, K, ldb) == HIPBLAS_STATUS_SUCCESS;
  good = good && hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, K, M, lda) == HIPBLAS_STATUS_SUCCESS;
  good = good && hipblasLtMatrixLayoutCreate(&p.c, HIP_R_16BF, N, M, beta ? ldc : ldd) == HIPBLAS_STATUS_SUCCESS;
  good = good && hipblasLtMatrixLayoutCreate(&p.d, HIP_R_16BF, N, M, ldd) == HIPBLAS_STATUS_SUCCESS;
  if (good) {
    hipblasLtMatmulPreference_t pref = nullptr;
    if (hipblasLtMatmulPreferenceCreate(&pref) == HIPBLAS_STATUS_SUCCESS) {
      const uint64_t ws = 0;
      hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
      hipblasLtMatmulHeuristicResult_t res[1];
      int n = 0;
      if (hipblasLtMatmulAlgoGetHeuristic(h, p.desc, p.a, p.b, p.c, p.d, pref, 1, res, &n) == HIPBLAS_STATUS_SUCCESS && n > 0 &&
          res[0].state == HIPBLAS_STATUS_SUCCESS && res[0].workspaceSize == 0) {
        p.algo = res[0].algo;
        p.ok = true;
      }
      hipblasLtMatmulPreferenceDestroy(pref);
    }
  }
  return p;
}
}  // namespace

// D[M][N] = A[M][K] . B[K][N] (+ C when C != nullptr), all bf16 row-major with the given row strides.  0 = done.
int blaslt_gemm_rm(const void* A, long lda, const void* B, long ldb, const void* C, long ldc, void* D, long ldd, int M,
                   int N, int K, hipStream_t st) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 1;
  const Key key{M, N, K, lda, ldb, C ? ldc : 0, ldd, C ? 1 : 0, dev};
  Plan p;
  hipblasLtHandle_t h;
  {
    std::lock_guard<std::mutex> g(mu);
    h = handle_for(dev);
    if (!h) return 1;
    auto it = plans.find(key);
    if (it == plans.end()) it = plans.emplace(key, make_plan(h, M, N, K, lda, ldb, ldc, ldd, C != nullptr)).first;
    p = it->second;
  }
  if (!p.ok) return 1;
  const float alpha = 1.f, beta = C ? 1.f : 0.f;
  const hipblasStatus_t s = hipblasLtMatmul(h, p.desc, &alpha, B, p.a, A, p.b, &beta, C ? C : D, p.c, D, p.d, &p.algo,
                                            nullptr, 0, st);
  return s == HIPBLAS_STATUS_SUCCESS ? 0 : 1;
}
