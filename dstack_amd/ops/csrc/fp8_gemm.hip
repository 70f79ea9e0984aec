// Decode-batch fp8 GEMM for CDNA4 (gfx950): Y[m][n] = bf16( xs[m] * ws[n] * sum_k X[m][k] W[n][k] )
// for M <= 256 rows (a serving decode batch) against e4m3 weights with one fp32 scale per output
// row (the layout of serving/model.py Fp8Weight) and e4m3 activations with one scale per token.
//
// At M = 256 the projection streams its weights once and is HBM-bound (512 flops per weight byte
// against ~770 at the fp8 MFMA rate), so the design is about keeping every CU's weight stream
// full:
//  * One workgroup = the whole (padded) batch x 128 weight rows x a K slice (split-K over
//    blockIdx.y so a short-N projection still fills the chip: 64 column blocks x 4 slices).
//  * 8 waves: wave (wr, wc) owns batch rows 128wr + [0,128) and weight rows 32wc + [0,32);
//    v_mfma_scale_f32_16x16x128_f8f6f4 with unit E8M0 scales (the fp8 rate; the unscaled fp8
//    MFMA runs at the bf16 rate), weights as the A operand so a lane's accumulator holds 4
//    consecutive output columns of one batch row (8-byte bf16 stores).
//  * K advances 128 bytes per step; a step's X tile (256 x 128 B) and W tile (128 x 128 B) are
//    LDS-DMA'd (global_load_lds_dwordx4, inline asm, hand-counted vmcnt) into a 3-slot ring, two
//    steps ahead.  128-byte rows with chunk c of row r at slot c ^ ((r>>1 & 1) | (r>>3 & 1) << 2):
//    the two ds_read_b128 of a fragment (rows r, 32-byte k chunk g = lane >> 4) hit 16 different
//    16-byte bank windows in every ds_read_b128 lane group (searched exhaustively over the XOR-linear
//    swizzles of the row's low 4 bits).
//  * Split-K partials: fp32 slabs [S][256][N]; every workgroup stores its slab, then (one lane,
//    after every storing wave drained and an agent-scope release) takes a ticket on its column
//    block's counter; the last arrival acquires, adds the other slabs to its accumulators, applies
//    the scales and writes bf16, and resets the counter for the next launch.
#include <stdint.h>

#include "mfma_tiles.h"

using namespace dsa;

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int F8_MP = 256;             // padded batch rows
constexpr int F8_BN = 128;             // weight rows per workgroup
constexpr int F8_BK = 128;             // K bytes per step
constexpr int F8_XT = F8_MP * F8_BK;   // 32 KiB X tile
constexpr int F8_WT = F8_BN * F8_BK;   // 16 KiB W tile
constexpr int F8_STAGE = F8_XT + F8_WT;
constexpr int F8_NSTAGE = 3;
constexpr int F8_LDS = F8_NSTAGE * F8_STAGE;  // 144 KiB

struct F8Args {
  const uint8_t* X;
  const float* xs;
  const uint8_t* W;
  const float* ws;
  bf16_t* Y;
  float* part;   // [S][256][N] fp32 (S > 1)
  int* cnt;      // [N / 128] tickets, zero between launches (S > 1)
  long ldx, ldw, ldy;
  int M, N, K, S;
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

__global__ __launch_bounds__(512) void fp8_rows_gemm_kernel(F8Args p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int nb = blockIdx.x, split = blockIdx.y;
  const int n0 = nb * F8_BN;
  const int ks = p.K / p.S, kbeg = split * ks, nsteps = ks / F8_BK;

  // --- DMA: this wave's 6 pieces of a stage (pieces w, w+8, ..., w+40; 0-31 X, 32-47 W) -------
  unsigned voff[6], ldsoff[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int piece = w + 8 * i;
    const int row = 8 * (piece & 31) + (lane >> 3);
    const int ch = (lane & 7) ^ f8_swz(row & 15);
    if (i >= 4) {
      voff[i] = (unsigned)((long)row * p.ldw + ch * 16);
      ldsoff[i] = (unsigned)(F8_XT + (piece - 32) * 1024);
    } else {
      const int srow = row < p.M ? row : p.M - 1;  // padded batch rows re-read the last real row
      voff[i] = (unsigned)((long)srow * p.ldx + ch * 16);
      ldsoff[i] = (unsigned)(piece * 1024);
    }
  }
  const unsigned lds0 = (unsigned)(uintptr_t)LDS3(char, smem);
  const uint8_t* xbase = p.X + kbeg;
  const uint8_t* wbase = p.W + (long)n0 * p.ldw + kbeg;
  auto issue = [&](int step) {
    const unsigned slot = lds0 + (unsigned)((step % F8_NSTAGE) * F8_STAGE);
    const long ko = (long)step * F8_BK;
#pragma unroll
    for (int i = 0; i < 6; ++i) f8_dma(i >= 4 ? wbase + ko : xbase + ko, voff[i], slot + ldsoff[i]);
  };

  // --- fragment read offsets: row (lane & 15) of a 16-row block, k chunk pair g = lane >> 4 ----
  const int r = lane & 15, g = lane >> 4, sw = f8_swz(r);
  const int c0 = ((2 * g) ^ sw) * 16, c1 = ((2 * g + 1) ^ sw) * 16;
  const int xrow = (128 * wr + r) * F8_BK, wrow = F8_XT + (32 * wc + r) * F8_BK;

  f32x4 acc[8][2];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(0);
  if (nsteps > 1) issue(1);
  for (int t = 0; t < nsteps; ++t) {
    if (t + 1 < nsteps) f8_vmcnt<6>(); else f8_vmcnt<0>();  // step t landed (this wave's pieces)
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();                                          // ... and every wave's
    if (t + 2 < nsteps) issue(t + 2);  // into the slot step t-1 read: every wave is past it
    const char* st = smem + (t % F8_NSTAGE) * F8_STAGE;
    i32x8 wf[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) wf[j] = f8_frag(st + wrow + j * 2048 + c0, st + wrow + j * 2048 + c1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const i32x8 xf = f8_frag(st + xrow + i * 2048 + c0, st + xrow + i * 2048 + c1);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wf[j], xf, acc[i][j], 0, 0, 0, 127, 0, 127);
    }
  }

  // --- epilogue: lane holds C[n = 4(lane>>4) + e][m = lane & 15] of each 16x16 block ------------
  // batch row m = 128wr + 16i + (lane & 15); weight row n = n0 + 32wc + 16j + 4(lane >> 4) + e
  const int mrow = 128 * wr + r, ncol = n0 + 32 * wc + 4 * g;
  if (p.S > 1) {
    int* ticket = reinterpret_cast<int*>(smem);  // the ring is free once every wave is past the loop
    float* mine = p.part + (long)split * F8_MP * p.N;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        *reinterpret_cast<f32x4*>(mine + (long)(mrow + 16 * i) * p.N + ncol + 16 * j) = acc[i][j];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      *ticket = __hip_atomic_fetch_add(p.cnt + nb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (*ticket == p.S - 1) {  // the last slice of this column block: acquire the others' slabs
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __syncthreads();
    if (*ticket != p.S - 1) return;
    for (int s = 0; s < p.S; ++s) {
      if (s == split) continue;
      const float* other = p.part + (long)s * F8_MP * p.N;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] += *reinterpret_cast<const f32x4*>(other + (long)(mrow + 16 * i) * p.N + ncol + 16 * j);
    }
    if (tid == 0) __hip_atomic_store(p.cnt + nb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  float wsc[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) wsc[j][e] = p.ws[ncol + 16 * j + e];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
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

extern "C" bool dsa_fp8_rows_gemm_supported(int M, int N, int K, int S) {
  return M > 0 && M <= F8_MP && N > 0 && N % F8_BN == 0 && S >= 1 && K > 0 && K % (F8_BK * S) == 0;
}

// Y[M][N] = bf16(xs[m] ws[n] X W^T); X [M][K] e4m3 (row stride ldx bytes), W [N][K] e4m3 (ldw
// bytes), Y bf16 (ldy elements).  S > 1: `part` holds S * 256 * N floats and `cnt` N / 128 ints,
// zero on the first call (each call leaves them zero).
extern "C" hipError_t dsa_fp8_rows_gemm(const void* X, const float* xs, const void* W, const float* ws, void* Y,
                                        float* part, int* cnt, int M, int N, int K, long ldx, long ldw, long ldy,
                                        int S, hipStream_t st) {
  if (!dsa_fp8_rows_gemm_supported(M, N, K, S) || ldx % 16 || ldw % 16 || ldy % 4 || ldx < K || ldw < K || ldy < N)
    return hipErrorInvalidValue;
  if (S > 1 && (!part || !cnt)) return hipErrorInvalidValue;
  if ((long)(F8_BN - 1) * ldw + K > 0xffffffffL || (long)(M - 1) * ldx + K > 0xffffffffL) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    DSA_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&fp8_rows_gemm_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, F8_LDS));
    attr = true;
  }
  F8Args a{(const uint8_t*)X, xs, (const uint8_t*)W, ws, (bf16_t*)Y, part, cnt, ldx, ldw, ldy, M, N, K, S};
  fp8_rows_gemm_kernel<<<dim3(N / F8_BN, S), 512, F8_LDS, st>>>(a);
  return hipGetLastError();
}
