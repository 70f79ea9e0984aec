// Weight-gradient GEMM for CDNA4 (gfx950): C[P][Q] (+)= A^T · B with A = [T][P], B = [T][Q]
// (both row-major, the reduction index T is the OUTER dimension of both operands), bf16 in, fp32
// accumulate, bf16 out.  This is dW = dY^T · X of every linear layer (T = tokens, dY = [T][out],
// X = [T][in]), the layout hipBLASLt is weakest at on gfx950 ("NT", 1.1-1.35 PF/s on the Llama
// shapes vs 1.6-1.9 PF/s for the forward "TN" GEMMs, see dstack_amd/ops/tuned/*.csv).
//
// Design (one workgroup = 256x256 output tile, 8 waves, 2 waves/SIMD):
//  * Each 64-deep slice of A and B is two [64][128] LDS images per operand (256-byte rows, the
//    XOR swizzle of mfma_tiles.h), filled by LDS-DMA (global_load_lds, 16 B/lane, no staging
//    VGPRs) into a 2-deep ring: 4 x 16 KiB per stage, 128 KiB total -> one workgroup per CU.
//  * Both MFMA operands have the reduction index on the LDS row, so both are read with
//    ds_read_b64_tr_b16 (lds_tr); A and B fragments use the same k permutation, so the 32x32x16
//    MFMA reduces matching k pairs.
//  * Wave (wp, wq) owns C rows 128*wp.. (4 MFMA row tiles) and columns 64*wq.. (2 column tiles):
//    per 16-deep k step 4+2 transposed fragment reads feed 8 MFMAs (128 accumulator registers).
//  * XCD-aware tile order: workgroup ids are dealt round-robin to the 8 XCDs, so the logical tile
//    index is remapped to give each XCD a contiguous run of tiles, grouped 4 row-blocks wide, and
//    the 32 concurrently running workgroups of an XCD share A/B slices in that XCD's L2.
//
// Measured on MI355X (tools/bench_gemm.py, T = 8192, same box, profiles/gemm_wgrad_r1.txt): 0.87-1.12
// PF/s against hipBLASLt's 0.95-1.20 on the five Llama-3-8B weight-gradient shapes -- parity, not a
// win, so training keeps the library GEMM for dW.  Counters (o-proj shape): MFMA busy 51 %, LDS 19 %
// busy with no bank conflicts, L2 hit 80 % (the same traffic as hipBLASLt's kernel); the kernel
// runs at 1.41 PF/s when the HBM/L2 traffic after the first slice is removed, so the load path
// (one 64 KiB slice in flight per CU) is what bounds it.  Tried and measured slower: BK=32 rings
// with 3-4 slices in flight, a barrier-staggered two-group ping-pong schedule, fragment reads
// software-pipelined across the barrier, an L2 warm-up stream 1-3 slices ahead, and other tile
// orders (group 1/2/8/16 row blocks, no XCD remap: all within +-3 %).
#include "mfma_tiles.h"

using namespace dsa;

namespace {

constexpr int GT_BM = 256, GT_BN = 256, GT_BK = 64;  // GT_BK: T granularity accepted
constexpr int GT_GROUP = 4;  // row blocks per tile-order group

__device__ __forceinline__ int xcd_tile(int b, int n) {
  const int xcd = b & 7, idx = b >> 3, per = n >> 3, rem = n & 7;
  return xcd * per + (xcd < rem ? xcd : rem) + idx;
}

}  // namespace

// Stage the [BK][128] bf16 slice at g (row stride `stride` elements) into a swizzled LDS image:
// BK/4 pieces of 4 rows (1 KiB each) over 4 waves.  Each LDS-DMA is an inline-asm statement: hipcc
// does not track it, so it cannot drain it with a vmcnt(0) in front of the next ds_read of the same
// LDS array -- which it does for __builtin_amdgcn_global_load_lds, serialising every stage's DMA
// with its compute (measured: +10 % throughput from this alone).  Completion is counted by hand
// (wait_vmcnt).  `wave` must be wave-uniform.
template <int BK>
__device__ __forceinline__ void dma_slice_asm(const bf16_t* g, long stride, char* lds, int wave, int lane) {
  const unsigned base = (unsigned)(uintptr_t)LDS3(char, lds);
#pragma unroll
  for (int i = 0; i < BK / 16; ++i) {
    const int piece = wave * (BK / 16) + i;
    const int row = piece * 4 + (lane >> 4);
    const int pc = lane & 15;
    const int ch = pc ^ (((row & 3) << 2) | ((row >> 2) & 3));
    const bf16_t* src = g + (long)row * stride + ch * 8;
    const unsigned dst = __builtin_amdgcn_readfirstlane(base + piece * 1024);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(dst)
                 : "memory");
  }
}

__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int N>
__device__ __forceinline__ void wait_lgkmcnt() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

// BK = reduction depth per pipeline stage, NST = stages in the LDS ring (NST-1 in flight).
template <bool ACC, int BK, int NST>
__global__ __launch_bounds__(512, 2) void gemm_tn_kernel(const bf16_t* __restrict__ A,
                                                         const bf16_t* __restrict__ B,
                                                         bf16_t* __restrict__ C, int P, int Q, int T,
                                                         long lda, long ldb, long ldc, int group, int xcd) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int SUB = BK * 256;  // one [BK][128] image
  constexpr int STAGE = 4 * SUB;  // A[0:128) | A[128:256) | B[0:128) | B[128:256)
  constexpr int IPS = 2 * (BK / 16);  // DMA instructions per wave per stage
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hf = lane >> 5, l32 = lane & 31;
  const int wp = w >> 2, wq = w & 3, w4 = w & 3;
  const int tp = P / GT_BM, tq = Q / GT_BN;
  const int tile = xcd ? xcd_tile(blockIdx.x, tp * tq) : (int)blockIdx.x;
  const int in_group = group * tq;
  const int first_p = (tile / in_group) * group;
  const int gm = min(tp - first_p, group);
  const int pb = first_p + (tile % in_group) % gm;
  const int qb = (tile % in_group) / gm;
  const int p0 = pb * GT_BM, q0 = qb * GT_BN;
  const int nk = T / BK;

  // waves 0-3 stage the first 128 columns of A and B, waves 4-7 the second 128
  const int half = w >> 2;
  const bf16_t* asrc = A + p0 + 128 * half;
  const bf16_t* bsrc = B + q0 + 128 * half;
  const int w4u = __builtin_amdgcn_readfirstlane(w4);
  auto issue = [&](int kt) {
    char* st = smem + (kt % NST) * STAGE;
    dma_slice_asm<BK>(asrc + (long)kt * BK * lda, lda, st + half * SUB, w4u, lane);
    dma_slice_asm<BK>(bsrc + (long)kt * BK * ldb, ldb, st + (2 + half) * SUB, w4u, lane);
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nk) issue(s);
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt landed (later stages may still be in flight) and every wave is done with kt-1
    if (kt + NST - 2 < nk)
      wait_vmcnt<(NST - 2) * IPS>();
    else
      wait_vmcnt<0>();
    wait_lgkmcnt<0>();  // this wave's reads of the slot about to be refilled are done
    raw_barrier();
    if (kt + NST - 1 < nk) issue(kt + NST - 1);  // into the slot read at kt-1
    const char* st = smem + (kt % NST) * STAGE;
    const char* al = st + wp * SUB;
    const char* bl = st + (2 + (wq >> 1)) * SUB;
    const int qc = 64 * (wq & 1);
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 a[4], b[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = lds_tr(al, 16 * ks, 32 * i, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = lds_tr(bl, 16 * ks, qc + 32 * j, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma(a[i], b[j], acc[i][j]);
    }
  }

  // accumulator (i, j): column q = lane, rows p = 8*(r>>2) + 4*hf + (r&3) of the 32x32 tile
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int q = q0 + 64 * wq + 32 * j + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int p = p0 + 128 * wp + 32 * i + 8 * (r >> 2) + 4 * hf + (r & 3);
        bf16_t* c = C + (long)p * ldc + q;
        float v = acc[i][j][r];
        if (ACC) v += bf2f(*c);
        *c = f2bf(v);
      }
    }
}

extern "C" bool dsa_gemm_tn_supported(int P, int Q, int T) {
  return P > 0 && Q > 0 && T > 0 && P % GT_BM == 0 && Q % GT_BN == 0 && T % GT_BK == 0;
}

// C[P][Q] = A^T B (+ C when accumulate).  Leading dimensions in elements; every row must be
// 16-byte aligned (ld % 8 == 0) for the 16-byte LDS-DMA.
extern "C" hipError_t dsa_gemm_tn(const void* A, const void* B, void* C, int P, int Q, int T, long lda,
                                  long ldb, long ldc, int accumulate, hipStream_t st) {
  if (!dsa_gemm_tn_supported(P, Q, T) || lda % 8 || ldb % 8 || lda < P || ldb < Q || ldc < Q)
    return hipErrorInvalidValue;
  const int grid = (P / GT_BM) * (Q / GT_BN);
  const size_t lds = 2 * 4 * 64 * 256;
  if (accumulate)
    gemm_tn_kernel<true, 64, 2><<<grid, 512, lds, st>>>((const bf16_t*)A, (const bf16_t*)B, (bf16_t*)C, P, Q, T, lda,
                                                        ldb, ldc, GT_GROUP, 1);
  else
    gemm_tn_kernel<false, 64, 2><<<grid, 512, lds, st>>>((const bf16_t*)A, (const bf16_t*)B, (bf16_t*)C, P, Q, T, lda,
                                                         ldb, ldc, GT_GROUP, 1);
  return hipGetLastError();
}
