// Decode-batch fp8 GEMM for CDNA4 (gfx950): Y[m][n] = bf16( xs[m] * ws[n] * sum_k X[m][k] W[n][k] )
// for M <= 256 rows (a serving decode batch) against e4m3 weights with one fp32 scale per output
// row (the layout of serving/model.py Fp8Weight) and e4m3 activations with one scale per token.
//
// At M <= 256 the projection streams its weights once and is HBM-bound (512 flops per weight byte
// against ~770 at the fp8 MFMA rate), so the design is about keeping every CU's weight stream
// full with few bytes of anything else:
//  * One workgroup = 64 batch rows x 128 weight rows x all of K.  The batch is cut into 64-row
//    blocks rather than K into slices: a 256-row batch gives 4 x N/128 workgroups (256 for a
//    d=8192 projection, one per CU) with no split-K partials (at M = 256 an fp32 partial is 1 KiB
//    per weight row, 12-50 % of the weight bytes per extra slice).  The 4 batch blocks of one
//    column block are consecutive multiples of N/128 in the grid, i.e. on one XCD under
//    round-robin placement, so the weight rows come from HBM once and from that XCD's L2 after.
//  * 8 waves: wave (wr, wc) owns batch rows 32wr + [0,32) and weight rows 32wc + [0,32);
//    v_mfma_scale_f32_16x16x128_f8f6f4 with unit E8M0 scales (the fp8 rate; the unscaled fp8
//    MFMA runs at the bf16 rate), weights as the A operand so a lane's accumulator holds 4
//    consecutive output columns of one batch row (8-byte bf16 stores).
//  * K advances 128 bytes per step; a step's X tile (64 x 128 B) and W tile (128 x 128 B) are
//    LDS-DMA'd (global_load_lds_dwordx4, inline asm, hand-counted vmcnt) into a 3-slot ring, two
//    steps ahead (72 KiB: two workgroups per CU).  128-byte rows with chunk c of row r at slot
//    c ^ ((r>>1 & 1) | (r>>3 & 1) << 2): the two ds_read_b128 of a fragment (row r, 32-byte k chunk
//    g = lane >> 4) hit 16 different 16-byte bank windows in every ds_read_b128 lane group (searched
//    exhaustively over the XOR-linear swizzles of the row's low 4 bits).
#include <stdint.h>

#include "mfma_tiles.h"

using namespace dsa;

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int F8_MAXM = 256;           // batch rows
constexpr int F8_BM = 64;              // batch rows per workgroup
constexpr int F8_BN = 128;             // weight rows per workgroup
constexpr int F8_BK = 128;             // K bytes per step
constexpr int F8_XT = F8_BM * F8_BK;   // 8 KiB X tile
constexpr int F8_WT = F8_BN * F8_BK;   // 16 KiB W tile
constexpr int F8_STAGE = F8_XT + F8_WT;
constexpr int F8_NSTAGE = 3;
constexpr int F8_LDS = F8_NSTAGE * F8_STAGE;  // 72 KiB

struct F8Args {
  const uint8_t* X;
  const float* xs;
  const uint8_t* W;
  const float* ws;
  bf16_t* Y;
  long ldx, ldw, ldy;
  int M, N, K;
};

__device__ __forceinline__ int f8_swz(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 2); }

// one LDS-DMA instruction: 64 lanes x 16 B from SGPR base + per-lane offset into LDS `lds` (M0)
__device__ __forceinline__ void f8_dma(const uint8_t* sbase, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds)
      : "memory");
}

template <int N>
__device__ __forceinline__ void f8_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ i32x8 f8_frag(const char* p0, const char* p1) {
  const i32x4 a = *reinterpret_cast<const i32x4*>(p0);
  const i32x4 b = *reinterpret_cast<const i32x4*>(p1);
  return i32x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

}  // namespace

__global__ __launch_bounds__(512, 2) void fp8_rows_gemm_kernel(F8Args p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  // tile order: groups of 8 column blocks x all batch blocks; within a group the batch blocks of
  // one column block are 8 ids apart (one XCD under round-robin placement) and dispatched together,
  // so their shared weight rows come from HBM once and from that XCD's L2 after (a 1792-workgroup
  // gate/up projection read its weights ~4x from HBM with the batch blocks N/128 ids apart)
  const int nN = p.N / F8_BN, nM = gridDim.x / nN;
  int nb, mb;
  if (nN % 8 == 0) {
    const int grp = blockIdx.x / (8 * nM), in = blockIdx.x % (8 * nM);
    nb = grp * 8 + (in & 7);
    mb = in >> 3;
  } else {
    nb = blockIdx.x % nN;
    mb = blockIdx.x / nN;
  }
  const int n0 = nb * F8_BN, m0 = mb * F8_BM;
  const int nsteps = p.K / F8_BK;

  // --- DMA: this wave's 3 pieces of a stage (pieces w, w+8, w+16 of 24: 0-7 X, 8-23 W) ---------
  unsigned voff[3], ldsoff[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int piece = w + 8 * i;
    if (i == 0) {  // X rows 8w .. 8w+7
      const int row = 8 * piece + (lane >> 3);
      const int ch = (lane & 7) ^ f8_swz(row & 15);
      const int srow = m0 + row < p.M ? m0 + row : p.M - 1;  // padded rows re-read the last real row
      voff[i] = (unsigned)((long)srow * p.ldx + ch * 16);
      ldsoff[i] = (unsigned)(piece * 1024);
    } else {       // W rows 8(piece - 8) ..
      const int row = 8 * (piece - 8) + (lane >> 3);
      const int ch = (lane & 7) ^ f8_swz(row & 15);
      voff[i] = (unsigned)((long)row * p.ldw + ch * 16);
      ldsoff[i] = (unsigned)(F8_XT + (piece - 8) * 1024);
    }
  }
  const unsigned lds0 = (unsigned)(uintptr_t)LDS3(char, smem);
  const uint8_t* wbase = p.W + (long)n0 * p.ldw;
  auto issue = [&](int step) {
    const unsigned slot = lds0 + (unsigned)((step % F8_NSTAGE) * F8_STAGE);
    const long ko = (long)step * F8_BK;
    f8_dma(p.X + ko, voff[0], slot + ldsoff[0]);
    f8_dma(wbase + ko, voff[1], slot + ldsoff[1]);
    f8_dma(wbase + ko, voff[2], slot + ldsoff[2]);
  };

  // --- fragment read offsets: row (lane & 15) of a 16-row block, k chunk pair g = lane >> 4 ----
  const int r = lane & 15, g = lane >> 4, sw = f8_swz(r);
  const int c0 = ((2 * g) ^ sw) * 16, c1 = ((2 * g + 1) ^ sw) * 16;
  const int xrow = (32 * wr + r) * F8_BK, wrow = F8_XT + (32 * wc + r) * F8_BK;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(0);
  if (nsteps > 1) issue(1);
  for (int t = 0; t < nsteps; ++t) {
    if (t + 1 < nsteps) f8_vmcnt<3>(); else f8_vmcnt<0>();  // step t landed (this wave's pieces)
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();                                          // ... and every wave's
    if (t + 2 < nsteps) issue(t + 2);  // into the slot step t-1 read: every wave is past it
    const char* st = smem + (t % F8_NSTAGE) * F8_STAGE;
    i32x8 wf[2], xf[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      wf[j] = f8_frag(st + wrow + j * 2048 + c0, st + wrow + j * 2048 + c1);
      xf[j] = f8_frag(st + xrow + j * 2048 + c0, st + xrow + j * 2048 + c1);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wf[j], xf[i], acc[i][j], 0, 0, 0, 127, 0, 127);
  }

  // --- epilogue: lane holds C[n = 4(lane>>4) + e][m = lane & 15] of each 16x16 block ------------
  const int mrow = m0 + 32 * wr + r, ncol = n0 + 32 * wc + 4 * g;
  float wsc[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) wsc[j][e] = p.ws[ncol + 16 * j + e];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = mrow + 16 * i;
    if (m >= p.M) continue;
    const float xsc = p.xs[m];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      unsigned short o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = f2bf(acc[i][j][e] * xsc * wsc[j][e]);
      *reinterpret_cast<uint2*>(p.Y + (long)m * p.ldy + ncol + 16 * j) =
          uint2{(unsigned)o[0] | ((unsigned)o[1] << 16), (unsigned)o[2] | ((unsigned)o[3] << 16)};
    }
  }
}

extern "C" bool dsa_fp8_rows_gemm_supported(int M, int N, int K) {
  return M > 0 && M <= F8_MAXM && N > 0 && N % F8_BN == 0 && K > 0 && K % F8_BK == 0;
}

// Y[M][N] = bf16(xs[m] ws[n] X W^T); X [M][K] e4m3 (row stride ldx bytes), W [N][K] e4m3 (ldw
// bytes), Y bf16 (ldy elements).
extern "C" hipError_t dsa_fp8_rows_gemm(const void* X, const float* xs, const void* W, const float* ws, void* Y,
                                        int M, int N, int K, long ldx, long ldw, long ldy, hipStream_t st) {
  if (!dsa_fp8_rows_gemm_supported(M, N, K) || ldx % 16 || ldw % 16 || ldy % 4 || ldx < K || ldw < K || ldy < N)
    return hipErrorInvalidValue;
  if ((long)(F8_BN - 1) * ldw + K > 0xffffffffL || (long)(M - 1) * ldx + K > 0xffffffffL) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    DSA_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&fp8_rows_gemm_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, F8_LDS));
    attr = true;
  }
  F8Args a{(const uint8_t*)X, xs, (const uint8_t*)W, ws, (bf16_t*)Y, ldx, ldw, ldy, M, N, K};
  const int mblocks = (M + F8_BM - 1) / F8_BM;
  fp8_rows_gemm_kernel<<<(N / F8_BN) * mblocks, 512, F8_LDS, st>>>(a);
  return hipGetLastError();
}
