// 256x256 GEMM on FOUR waves, one per SIMD, each owning a 128x128 sub-tile (8 x 8 blocks of 16x16: 256 fp32
// accumulators per lane, in AGPRs -- this translation unit is built WITHOUT the VGPR MFMA form, see the Makefile).
//
// Why: the 8-wave ping-pong kernel (gemm.hpp igemm_pp_kernel, two 128x64 waves per SIMD) reads 0.38 LDS instructions
// and issues 1.1 SALU + 0.5 VALU per MFMA and spends 37 % of its wave-cycles in s_waitcnt / barrier waits: 8192^3 bf16
// on random data 1040 TF/s at 58 % MFMA-busy, where hipBLASLt's 256x256x64 kernel -- four waves, one per SIMD --
// reaches 1450-1470 TF/s at 87 % MFMA-busy with 0.25 LDS instructions per MFMA (profiles/r06d_gemm_pmc.txt).
// A 128x128 wave tile halves the fragment reads per MFMA (each A / B fragment feeds 8 MFMAs instead of 4).
//
// K loop (BK = 64 = two 32-deep k-steps, 64 MFMAs each per wave), two LDS stages of 64 KB (A 256 x 64 | B 256 x 64):
//   k-step 0 of tile t:  read tile t's k-step-1 fragments (16 x ds_read_b128 / tr pairs) | 64 MFMAs
//   k-step 1 of tile t:  vmcnt(0) (tile t+1 landed) + barrier  ->  LDS-DMA of tile t+2 into tile t's stage (its last
//                        reads were the k-step-1 fragments, read before the barrier) | read tile t+1's k-step-0
//                        fragments | 64 MFMAs
// so a tile's DMA is issued two k-steps (128 MFMAs) before its wait, and the MFMAs of each k-step find their
// fragments in registers (double-buffered by k-step).  One barrier per K tile.
// Epilogue: the fp32 C tile is staged through the (free) K-stage LDS in two 128-row halves and handed to the same
// block-level epilogue functors as the other kernels (NT = 256 threads).
#include "gemm.hpp"

namespace {
constexpr int Q_THREADS = 256, Q_BM = 256, Q_BN = 256, Q_STAGE = (Q_BM + Q_BN) * 128, Q_LDT = Q_BN + 4;
constexpr int Q_LDS = (2 * Q_STAGE > 128 * Q_LDT * 4) ? 2 * Q_STAGE : 128 * Q_LDT * 4;
static_assert(Q_LDS <= 160 * 1024, "q kernel LDS budget");
}

// lgkmcnt(0) as the builtin (vmcnt 63, expcnt 7 = no wait): unlike the inline-asm wait_lgkm0(), the waitcnt pass sees
// it and clears its scoreboard, so it does not add its own lgkmcnt(0) behind the next fragment reads
DEV void q_wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }

template <class LA, class LB, class EPI>
__global__ void __launch_bounds__(Q_THREADS, 1) igemm_q_kernel(LA la, LB lb, EPI epi, int KTILES, int split, int group) {
  typedef bf16 T;
  static_assert(LA::ROWS == 256 && LB::ROWS == 256 && LA::NIW == 8 && LB::NIW == 8, "q kernel: 256-row loaders on 4 waves");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int wm = wave >> 1, wn = wave & 1;
  int m0, n0;
  {
    int mt, nt_;
    tile_of_block(group, mt, nt_);
    m0 = mt * Q_BM; n0 = nt_ * Q_BN;
  }
  const int per = (KTILES + split - 1) / split;
  const int kt0 = blockIdx.z * per, kt1 = min(KTILES, kt0 + per);
  const int nt = kt1 - kt0;
  epi.prepare(blockIdx.z);
  la.setup(m0, tid);
  lb.setup(n0, tid);
  constexpr int NL = LA::NIW + LB::NIW;        // LDS-DMA instructions per wave per K tile
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; i++)
#pragma unroll
    for (int j = 0; j < 8; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[2][8], fb[2][8];
  auto read_frags = [&](int buf, const char* stage, int kk) {
#pragma unroll
    for (int i = 0; i < 8; i++) fa[buf][i] = Frag<T, LA::KCL, Q_BM>::read(stage, wm * 128 + i * 16, kk, lane);
#pragma unroll
    for (int j = 0; j < 8; j++) fb[buf][j] = Frag<T, LB::KCL, Q_BN>::read(stage + Q_BM * 128, wn * 128 + j * 16, kk, lane);
  };
  // The MFMAs are inline asm with tied "+a" accumulators: with the builtin, the register allocator rotates the 64
  // accumulator tuples through VGPRs at the loop back-edge (180 v_accvgpr moves per K tile).  Inline asm is outside
  // the hazard recogniser, so the block covers its own hazards: s_nop 1 ahead of it (VALU write -> XDL SrcA/B read),
  // every fragment kept live to its end (no register of a fragment an in-flight MFMA still reads is reallocated
  // inside the block) and s_nop 7 x 2 behind it (XDL SrcA/B/C read -> VALU / DS write of the same register).
  auto mfmas = [&](int buf) {
    if constexpr (LA::RELU) {
#pragma unroll
      for (int i = 0; i < 8; i++) fa[buf][i] = relu_frag(fa[buf][i]);
    }
    if constexpr (LB::RELU) {
#pragma unroll
      for (int j = 0; j < 8; j++) fb[buf][j] = relu_frag(fb[buf][j]);
    }
    asm volatile("s_nop 1");
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
      for (int j = 0; j < 8; j++)
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(fb[buf][j]), "v"(fa[buf][i]));
    asm volatile("s_nop 7\n\ts_nop 7" :: "v"(fa[buf][0]), "v"(fa[buf][1]), "v"(fa[buf][2]), "v"(fa[buf][3]),
                 "v"(fa[buf][4]), "v"(fa[buf][5]), "v"(fa[buf][6]), "v"(fa[buf][7]), "v"(fb[buf][0]), "v"(fb[buf][1]),
                 "v"(fb[buf][2]), "v"(fb[buf][3]), "v"(fb[buf][4]), "v"(fb[buf][5]), "v"(fb[buf][6]), "v"(fb[buf][7]));
  };
  auto issue = [&](int kt, char* stage) {
    la.issue(kt, stage);
    lb.issue(kt, stage + Q_BM * 128);
  };
  if (nt > 0) {
    issue(kt0, smem);
    if (nt > 1) { issue(kt0 + 1, smem + Q_STAGE); wait_vmcnt<NL>(); }
    else wait_vmcnt<0>();
    raw_barrier();
    read_frags(0, smem, 0);
    // the last tile is peeled: a loop body whose second k-step may or may not issue fragment reads makes the
    // waitcnt pass merge both paths and wait (lgkmcnt 7..0) on the NEXT tile's fragment reads inside the MFMAs
    for (int t = 0; t + 1 < nt; ++t) {
      char* cur = smem + (t & 1) * Q_STAGE;
      char* nxt = smem + ((t + 1) & 1) * Q_STAGE;
      // k-step 0: tile t's k-step-1 fragments are read behind its 64 MFMAs (lgkmcnt(0) first: the k-step-0
      // fragments, read 64 MFMAs ago, are in -- the counter cannot tell them from the 16 reads issued after them)
      q_wait_lgkm0();
      read_frags(1, cur, 1);
      mfmas(0);
      // k-step 1: tile t+1 landed (the only DMA in flight) -> barrier -> tile t+2 into this tile's stage
      wait_vmcnt<0>();
      q_wait_lgkm0();
      raw_barrier();
      if (t + 2 < nt) issue(kt0 + t + 2, cur);
      read_frags(0, nxt, 0);
      mfmas(1);
    }
    q_wait_lgkm0();
    read_frags(1, smem + ((nt - 1) & 1) * Q_STAGE, 1);
    mfmas(0);
    mfmas(1);
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");   // XDL write -> accumulator read (epilogue)
  vm_drain();
  // stage the C tile (fp32) through LDS in two 128-row halves: waves wm = h write half h
  float* ct = (float*)smem;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    lds_barrier();
    if (wm == h) {
#pragma unroll
      for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 8; j++) {
          const int r = i * 16 + (lane & 15), c = wn * 128 + j * 16 + (lane >> 4) * 4;
          *(f32x4*)(ct + r * Q_LDT + c) = acc[i][j];
        }
    }
    lds_barrier();
    epi(ct, Q_LDT, m0 + h * 128, n0, tid, 128, Q_BN, Q_THREADS);
  }
}

template <class LA, class LB, class EPI>
int launch_igemm_q(LA la, LB lb, EPI epi, int M, int N, int KTILES, int split, int zdim_extra, hipStream_t st) {
  if (!la.buf_ok() || !lb.buf_ok()) {
    s3od_set_error("igemm_q: operand window too large for a buffer descriptor");
    return 22;
  }
  auto kfn = igemm_q_kernel<LA, LB, EPI>;
  static const bool attr = ((void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, Q_LDS), true);
  (void)attr;
  dim3 grid(cdiv(N, Q_BN), cdiv(M, Q_BM), split * zdim_extra);
  const int group = S3OD_KNOB("S3OD_GEMM_GROUP", 0);
  hipLaunchKernelGGL(kfn, grid, dim3(Q_THREADS), Q_LDS, st, la, lb, epi, KTILES, split, group);
  return s3od_check_launch("igemm_q");
}

// the (loader, epilogue) combinations the linears use (gemm_ops.hip: s3od_linear_fwd / _dgrad / _wgrad)
typedef DenseKC<bf16, 256, 4> QKC;
typedef DenseMC<bf16, 256, 4> QMC;
template int launch_igemm_q<QKC, QKC, EpiStd<bf16, bf16, bf16>>(QKC, QKC, EpiStd<bf16, bf16, bf16>, int, int, int, int, int, hipStream_t);
template int launch_igemm_q<QKC, QKC, EpiStd<float, float, bf16>>(QKC, QKC, EpiStd<float, float, bf16>, int, int, int, int, int, hipStream_t);
template int launch_igemm_q<QKC, QKC, EpiStd<float, bf16, bf16>>(QKC, QKC, EpiStd<float, bf16, bf16>, int, int, int, int, int, hipStream_t);
template int launch_igemm_q<QKC, QKC, EpiStd<bf16, float, bf16>>(QKC, QKC, EpiStd<bf16, float, bf16>, int, int, int, int, int, hipStream_t);
template int launch_igemm_q<QKC, QMC, EpiStd<bf16, bf16, bf16>>(QKC, QMC, EpiStd<bf16, bf16, bf16>, int, int, int, int, int, hipStream_t);
template int launch_igemm_q<QKC, QMC, EpiStd<float, float, float>>(QKC, QMC, EpiStd<float, float, float>, int, int, int, int, int, hipStream_t);
template int launch_igemm_q<QMC, QMC, EpiWgradPart>(QMC, QMC, EpiWgradPart, int, int, int, int, int, hipStream_t);
template int launch_igemm_q<QMC, QMC, EpiWgrad>(QMC, QMC, EpiWgrad, int, int, int, int, int, hipStream_t);
