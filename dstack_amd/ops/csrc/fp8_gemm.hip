// Decode-batch fp8 GEMM for CDNA4 (gfx950): Y[m][n] = bf16( xs[m] * ws[n] * sum_k X[m][k] W[n][k] )
// for M <= 256 rows (a serving decode batch) against e4m3 weights with one fp32 scale per output
// row (the layout of serving/model.py Fp8Weight) and e4m3 activations with one scale per token.
//
// At M <= 256 the projection streams its weights once and is HBM-bound (512 flops per weight byte
// against ~770 at the fp8 MFMA rate), so the design is about keeping every CU's weight stream
// full with few bytes of anything else:
//  * One workgroup = a 64- or 128-row batch block x 128 weight rows x all of K or a K slice.  The
//    batch is cut into blocks so a 256-row batch still gives enough workgroups (4 x N/128 at 64
//    rows: 256 for a d=8192 projection, one per CU) without split-K partials; the 4 (or 2) batch
//    blocks of one column block are consecutive multiples of 8 in the grid, i.e. on one XCD under
//    round-robin placement, so the weight rows come from HBM once and from that XCD's L2 after.
//    What bounds it is the bytes each CU pulls into LDS (~67 GB/s per CU measured, whatever the
//    ring depth): a 64-row block moves 24 KiB per 16 KiB of weights, so each weight byte crosses
//    6x at M = 256.  The 128-row blocks halve the X re-reads (4x) and, for long K, split K in two
//    (fp32 slabs, the last-arriving slice of a tile adds the others: agent-scope release / ticket /
//    acquire) to keep 256 workgroups.
//  * 8 waves: wave (wr, wc) owns 32 batch rows and 32 (BM 64) or 64 (BM 128) weight rows;
//    v_mfma_scale_f32_16x16x128_f8f6f4 with unit E8M0 scales (the fp8 rate; the unscaled fp8
//    MFMA runs at the bf16 rate), weights as the A operand so a lane's accumulator holds 4
//    consecutive output columns of one batch row (8-byte bf16 stores).
//  * K advances 128 bytes per step; a step's X tile (64 x 128 B) and W tile (128 x 128 B) are
//    LDS-DMA'd (global_load_lds_dwordx4, inline asm, hand-counted vmcnt) into a 3-slot ring, two
//    steps ahead (72 / 96 KiB).  128-byte rows with chunk c of row r at slot
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
constexpr int F8_BN = 128;             // weight rows per workgroup
constexpr int F8_BK = 128;             // K bytes per step
constexpr int F8_WT = F8_BN * F8_BK;   // 16 KiB W tile
constexpr int F8_NSTAGE = 3;
template <int BM>
constexpr int f8_stage() { return BM * F8_BK + F8_WT; }  // X tile + W tile

struct F8Args {
  const uint8_t* X;
  const float* xs;
  const uint8_t* W;
  const float* ws;
  bf16_t* Y;
  float* part;   // [S][256][N] fp32 split-K slabs (S > 1)
  int* cnt;      // one ticket per output tile, zero between launches (S > 1)
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

// BM = 64: waves (wr 0..1, wc 0..3) own 32 batch rows x 32 weight rows; BM = 128: waves (wr 0..3,
// wc 0..1) own 32 batch rows x 64 weight rows.  Per stage each wave issues BM/64 X pieces and 2 W
// pieces of 1 KiB.
template <int BM>
__global__ __launch_bounds__(512, 2) void fp8_rows_gemm_kernel(F8Args p) {
  constexpr int XT = BM * F8_BK, STAGE = f8_stage<BM>();
  constexpr int WR = BM / 32, WCN = 8 / WR;       // wave grid: WR batch x WCN weight slices
  constexpr int CB = F8_BN / WCN / 16;            // 16-column blocks per wave (2 or 4)
  constexpr int XP = BM / 64, NP = XP + 2;        // DMA pieces per wave per stage
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w / WCN, wc = w % WCN;
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
  const int n0 = nb * F8_BN, m0 = mb * BM, split = blockIdx.y;
  const int ks = p.K / p.S, nsteps = ks / F8_BK;

  // --- DMA pieces: X pieces w + 8i (rows 8 piece ..), W pieces 8 XP + w + 8i ------------------
  unsigned voff[NP], ldsoff[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    if (i < XP) {
      const int piece = w + 8 * i;
      const int row = 8 * piece + (lane >> 3);
      const int ch = (lane & 7) ^ f8_swz(row & 15);
      const int srow = m0 + row < p.M ? m0 + row : p.M - 1;  // padded rows re-read the last real row
      voff[i] = (unsigned)((long)srow * p.ldx + ch * 16);
      ldsoff[i] = (unsigned)(piece * 1024);
    } else {
      const int piece = w + 8 * (i - XP);
      const int row = 8 * piece + (lane >> 3);
      const int ch = (lane & 7) ^ f8_swz(row & 15);
      voff[i] = (unsigned)((long)row * p.ldw + ch * 16);
      ldsoff[i] = (unsigned)(XT + piece * 1024);
    }
  }
  const unsigned lds0 = (unsigned)(uintptr_t)LDS3(char, smem);
  const uint8_t* xbase = p.X + (long)split * ks;
  const uint8_t* wbase = p.W + (long)n0 * p.ldw + (long)split * ks;
  auto issue = [&](int step) {
    const unsigned slot = lds0 + (unsigned)((step % F8_NSTAGE) * STAGE);
    const long ko = (long)step * F8_BK;
#pragma unroll
    for (int i = 0; i < NP; ++i) f8_dma(i < XP ? xbase + ko : wbase + ko, voff[i], slot + ldsoff[i]);
  };

  // --- fragment read offsets: row (lane & 15) of a 16-row block, k chunk pair g = lane >> 4 ----
  const int r = lane & 15, g = lane >> 4, sw = f8_swz(r);
  const int c0 = ((2 * g) ^ sw) * 16, c1 = ((2 * g + 1) ^ sw) * 16;
  const int xrow = (32 * wr + r) * F8_BK, wrow = XT + (CB * 16 * wc + r) * F8_BK;

  f32x4 acc[2][CB];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < CB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(0);
  if (nsteps > 1) issue(1);
  for (int t = 0; t < nsteps; ++t) {
    if (t + 1 < nsteps) f8_vmcnt<NP>(); else f8_vmcnt<0>();  // step t landed (this wave's pieces)
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();                                           // ... and every wave's
    if (t + 2 < nsteps) issue(t + 2);  // into the slot step t-1 read: every wave is past it
    const char* st = smem + (t % F8_NSTAGE) * STAGE;
    i32x8 wf[CB], xf[2];
#pragma unroll
    for (int j = 0; j < CB; ++j) wf[j] = f8_frag(st + wrow + j * 2048 + c0, st + wrow + j * 2048 + c1);
#pragma unroll
    for (int i = 0; i < 2; ++i) xf[i] = f8_frag(st + xrow + i * 2048 + c0, st + xrow + i * 2048 + c1);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < CB; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wf[j], xf[i], acc[i][j], 0, 0, 0, 127, 0, 127);
  }

  // --- epilogue: lane holds C[n = 4(lane>>4) + e][m = lane & 15] of each 16x16 block ------------
  const int mrow = m0 + 32 * wr + r, ncol = n0 + CB * 16 * wc + 4 * g;
  if (p.S > 1) {
    // split-K: store the fp32 slab; the last slice of this output tile (ticket) adds the others
    float* mine = p.part + (long)split * F8_MAXM * p.N;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < CB; ++j)
        *reinterpret_cast<f32x4*>(mine + (long)(mrow + 16 * i) * p.N + ncol + 16 * j) = acc[i][j];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* ticket = reinterpret_cast<int*>(smem);  // the ring is free: every wave is past the loop
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int t = __hip_atomic_fetch_add(p.cnt + blockIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *ticket = t;
      if (t == p.S - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __syncthreads();
    if (*ticket != p.S - 1) return;
    for (int s2 = 0; s2 < p.S; ++s2) {
      if (s2 == split) continue;
      const float* other = p.part + (long)s2 * F8_MAXM * p.N;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < CB; ++j)
          acc[i][j] += *reinterpret_cast<const f32x4*>(other + (long)(mrow + 16 * i) * p.N + ncol + 16 * j);
    }
    if (tid == 0) __hip_atomic_store(p.cnt + blockIdx.x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  float wsc[CB][4];
#pragma unroll
  for (int j = 0; j < CB; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) wsc[j][e] = p.ws[ncol + 16 * j + e];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = mrow + 16 * i;
    if (m >= p.M) continue;
    const float xsc = p.xs[m];
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      unsigned short o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = f2bf(acc[i][j][e] * xsc * wsc[j][e]);
      *reinterpret_cast<uint2*>(p.Y + (long)m * p.ldy + ncol + 16 * j) =
          uint2{(unsigned)o[0] | ((unsigned)o[1] << 16), (unsigned)o[2] | ((unsigned)o[3] << 16)};
    }
  }
}

extern "C" bool dsa_fp8_rows_gemm_supported(int M, int N, int K, int bm, int S) {
  return M > 0 && M <= F8_MAXM && N > 0 && N % F8_BN == 0 && (bm == 64 || bm == 128) && S >= 1 && K > 0 &&
         K % (F8_BK * S) == 0;
}

// Y[M][N] = bf16(xs[m] ws[n] X W^T); X [M][K] e4m3 (row stride ldx bytes), W [N][K] e4m3 (ldw
// bytes), Y bf16 (ldy elements).  bm: batch rows per workgroup (64 or 128).  S > 1 splits K over
// S workgroups per output tile: `part` holds S * 256 * N floats and `cnt` one int per output tile
// ((N / 128) * ceil(M / bm)), zero on the first call (each call leaves them zero).
extern "C" hipError_t dsa_fp8_rows_gemm(const void* X, const float* xs, const void* W, const float* ws, void* Y,
                                        float* part, int* cnt, int M, int N, int K, long ldx, long ldw, long ldy,
                                        int bm, int S, hipStream_t st) {
  if (!dsa_fp8_rows_gemm_supported(M, N, K, bm, S) || ldx % 16 || ldw % 16 || ldy % 4 || ldx < K || ldw < K ||
      ldy < N)
    return hipErrorInvalidValue;
  if (S > 1 && (!part || !cnt)) return hipErrorInvalidValue;
  if ((long)(F8_BN - 1) * ldw + K > 0xffffffffL || (long)(M - 1) * ldx + K > 0xffffffffL) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    DSA_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&fp8_rows_gemm_kernel<64>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, F8_NSTAGE * f8_stage<64>()));
    DSA_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&fp8_rows_gemm_kernel<128>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, F8_NSTAGE * f8_stage<128>()));
    attr = true;
  }
  F8Args a{(const uint8_t*)X, xs, (const uint8_t*)W, ws, (bf16_t*)Y, part, cnt, ldx, ldw, ldy, M, N, K, S};
  const dim3 grid((N / F8_BN) * ((M + bm - 1) / bm), S);
  if (bm == 64)
    fp8_rows_gemm_kernel<64><<<grid, 512, F8_NSTAGE * f8_stage<64>(), st>>>(a);
  else
    fp8_rows_gemm_kernel<128><<<grid, 512, F8_NSTAGE * f8_stage<128>(), st>>>(a);
  return hipGetLastError();
}
