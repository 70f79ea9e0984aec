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

#include <type_traits>

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
  int wimg;      // W stored as LDS images (ops.serving.fp8_rows_shuffle): 16 KiB per 128-row tile and K-step
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
      : "v"(voff), "s"(sbase), "s"(__builtin_amdgcn_readfirstlane(lds))  // (uniform; kept in an SGPR)
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
      // LDS-image weights: the piece's 1 KiB is contiguous, already in the swizzled LDS order
      voff[i] = p.wimg ? (unsigned)(piece * 1024 + lane * 16) : (unsigned)((long)row * p.ldw + ch * 16);
      ldsoff[i] = (unsigned)(XT + piece * 1024);
    }
  }
  const unsigned lds0 = (unsigned)(uintptr_t)LDS3(char, smem);
  const uint8_t* xbase = p.X + (long)split * ks;
  const uint8_t* wbase = p.wimg ? p.W + ((long)nb * (p.K / F8_BK) + (long)split * nsteps) * (F8_BN * F8_BK)
                                : p.W + (long)n0 * p.ldw + (long)split * ks;
  const long wstep = p.wimg ? F8_BN * F8_BK : F8_BK;
  auto issue = [&](int step) {
    const unsigned slot = lds0 + (unsigned)((step % F8_NSTAGE) * STAGE);
    const long ko = (long)step * F8_BK, kw = (long)step * wstep;
#pragma unroll
    for (int i = 0; i < NP; ++i) f8_dma(i < XP ? xbase + ko : wbase + kw, voff[i], slot + ldsoff[i]);
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
    // ... and every wave's: a bare s_barrier (__syncthreads() is also a fence, for which the compiler
    // drained vmcnt to 0 here -- the ring then never had a step in flight across the barrier)
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
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
// ((N / 128) * ceil(M / bm)), zero on the first call (each call leaves them zero).  wimg: W holds
// ops.serving.fp8_rows_shuffle(w) (per 128-row tile and K-step the 16 KiB LDS image; ldw ignored).
extern "C" hipError_t dsa_fp8_rows_gemm(const void* X, const float* xs, const void* W, const float* ws, void* Y,
                                        float* part, int* cnt, int M, int N, int K, long ldx, long ldw, long ldy,
                                        int bm, int S, int wimg, hipStream_t st) {
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
  F8Args a{(const uint8_t*)X, xs, (const uint8_t*)W, ws, (bf16_t*)Y, part, cnt, ldx, ldw, ldy, M, N, K, S, wimg};
  const dim3 grid((N / F8_BN) * ((M + bm - 1) / bm), S);
  if (bm == 64)
    fp8_rows_gemm_kernel<64><<<grid, 512, F8_NSTAGE * f8_stage<64>(), st>>>(a);
  else
    fp8_rows_gemm_kernel<128><<<grid, 512, F8_NSTAGE * f8_stage<128>(), st>>>(a);
  return hipGetLastError();
}

// ================================================================================================
// Weight-streaming decode GEMM for 128 < M <= 256 token rows (fp8_stream_gemm): the weights never
// touch LDS.  fp8_rows_gemm above stages both operands through LDS, and each CU pulls 1.5-3x the
// weight bytes into it; the 256x256 e4m3 tile (gemm_nt_f8) keeps one 64 KiB K-step (activations +
// weights) in flight per CU and waits ~2 us for each, i.e. ~3.6 TB/s at gate/up.  Here:
//  * a workgroup = 4 waves (one per SIMD) x 64 weight rows x all 256 token rows x a K slice; the
//    256 x 64 fp32 accumulators of a wave fill its 256 accumulation registers;
//  * each wave loads ITS 64 weight rows straight from HBM into VGPRs (nontemporal: read once) as the
//    MFMA A operands, two K-steps ahead (3 live register sets, 96 VGPRs) -- no LDS, nothing shared;
//  * the activations (256 x 128 B per K-step, L2-resident: every workgroup reads them) are LDS-DMA'd
//    into a 4-slot ring (128 KiB) two steps ahead, one barrier per step; every wave reads all 16
//    token blocks of a step from LDS (the f8_swz swizzle: conflict-free fragment reads);
//  * v_mfma_scale_f32_16x16x128_f8f6f4 (unit E8M0 scales): a lane's accumulator holds 4 consecutive
//    output columns (weight rows) of one token row, so the epilogue stores 8-byte bf16 pieces;
//  * S > 1 splits K: fp32 partials [S][M][N] and fp8_stream_reduce_kernel adds them with the scales.
// In flight per CU: 2 K-steps x 4 waves x 64 rows x 128 B = 64 KiB of weights, against 32 KiB of
// weights (+ 32 KiB of activations) for the LDS-staged 256x256 tile -- the Little's-law term that
// bounds an HBM stream at this grid size.  LDS fragment reads: 4 bytes per weight byte (a 16-row
// wave, measured first, read 16 and was LDS-bound at 0.8x hipBLASLt).
// ================================================================================================
namespace {
constexpr int FS_NX = 4;                   // activation ring slots
constexpr int FS_XT = F8_MAXM * F8_BK;     // one slot: 256 token rows x 128 B = 32 KiB

struct FSArgs {
  const uint8_t* X;
  const float* xs;
  const uint8_t* W;
  const float* ws;
  bf16_t* Y;
  float* part;  // [S][M][N] fp32 (S > 1)
  long ldx, ldw, ldy;
  int M, N, K, S;
  int shuffled;  // W in ops.serving.fp8_stream_shuffle order: 0 row-major, 1 per 16-row block, 2 per 256 rows
};

template <int N>
__device__ __forceinline__ void fs_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// a bare workgroup barrier: __syncthreads() is a release/acquire fence as well, for which the compiler
// drains vmcnt to 0 before the s_barrier -- every prefetch in flight would be waited for each step
__device__ __forceinline__ void fs_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
}  // namespace

// (device functions rather than lambdas of the kernel template: a lambda using these builtins made
// the host pass drop the template's launch stub -- an undefined symbol at load time)
// (TAG: the calling kernel's prefetch depth -- one specialization per kernel; the host pass rejected a
// second kernel template calling an already-used specialization, "substitution failure")
template <int XP, int NWV, int TAG>
__device__ __forceinline__ void fs_issue_x(__amdgpu_buffer_rsrc_t xrs, const unsigned (&xoff)[XP], char* slot, int so,
                                           int w) {
#pragma unroll
  for (int i = 0; i < XP; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, LDS3(void, slot + (w + NWV * i) * 1024), 16, xoff[i], so, 0, 0);
}
// 7 waves (XP = 5 pieces, the last ones loaded twice -- identical bytes to one slot): the offsets are
// recomputed at every issue from the lane id behind an opaque move (kept live, 5 offsets spilled in
// the main loop)
template <int XP, int NWV>
__device__ __forceinline__ void fs_issue_x_rc(__amdgpu_buffer_rsrc_t xrs, char* slot, int so, int w, int M, long ldx) {
  int lane = __lane_id();
  asm volatile("" : "+v"(lane));
#pragma unroll
  for (int i = 0; i < XP; ++i) {
    const int piece = min(w + NWV * i, 31), row = 8 * piece + (lane >> 3);
    const int ch = (lane & 7) ^ f8_swz(row & 15);
    const int srow = row < M ? row : M - 1;  // rows past M re-read the last real row (not stored)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, LDS3(void, slot + piece * 1024), 16,
                                             (unsigned)((long)srow * ldx + ch * 16), so, 0, 0);
  }
}
// half: the byte distance of a fragment's two 16-byte pieces (16: adjacent in a row; 1 KiB: pre-shuffled),
// added to the uniform offset so that it costs no VGPRs
template <int NF>
__device__ __forceinline__ void fs_load_w(__amdgpu_buffer_rsrc_t wrs, const unsigned (&woff)[NF], int so, int half,
                                          i32x8 (&dst)[NF]) {
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const auto a = __builtin_amdgcn_raw_buffer_load_b128(wrs, (int)woff[f], so, 2);  // 2: nontemporal
    const auto b = __builtin_amdgcn_raw_buffer_load_b128(wrs, (int)woff[f], so + half, 2);
    dst[f] = i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
  }
}

// NWV waves x NF 16-row weight fragments per wave (a workgroup: 16 NWV NF weight rows); D: prefetch
// distance in K-steps for activations and weights.  p.shuffled: the weights are pre-shuffled
// (ops.serving.fp8_stream_shuffle: per 16-row block and K-step, the 2 KiB a wave's fragment reads, in lane
// order) -- every weight load is 1 KiB contiguous and each fragment's stream is sequential over K
template <int NWV, int NF, int D>
__global__ __launch_bounds__(64 * NWV, 1) void fp8_stream_gemm_kernel(FSArgs p) {
  constexpr int NSET = 4;               // weight register sets = the unroll factor (D + 1 live)
  constexpr int XP = (32 + NWV - 1) / NWV;  // X pieces (1 KiB) per wave per step
  constexpr int OPS = XP + 2 * NF;      // vector-memory ops per wave per step
  constexpr int WAIT = (D - 1) * OPS;   // issued after W(t): X(t+1), W(t+1), ..., X(t+D-1), W(t+D-1)
  static_assert(D >= 1 && D + 1 <= NSET, "D + 1 weight sets live");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int n0 = (blockIdx.x * NWV + w) * 16 * NF;  // this wave's first weight row
  const int ks = p.K / p.S, nsteps = ks / F8_BK;
  const long k0 = (long)blockIdx.y * ks;

  // --- activation DMA: 32 pieces of 1 KiB (8 token rows x 128 B) per step, XP per wave ------------
  const __amdgpu_buffer_rsrc_t xrs = make_rsrc(p.X, (unsigned)((long)(p.M - 1) * p.ldx + p.K));
  unsigned xoff[32 % NWV ? 1 : XP];
  if constexpr (32 % NWV == 0) {
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      const int piece = w + NWV * i, row = 8 * piece + (lane >> 3);
      const int ch = (lane & 7) ^ f8_swz(row & 15);
      const int srow = row < p.M ? row : p.M - 1;  // rows past M re-read the last real row (not stored)
      xoff[i] = (unsigned)((long)srow * p.ldx + ch * 16);
    }
  }
  auto issue_x = [&](int t) {
    const int so = __builtin_amdgcn_readfirstlane((int)(k0 + (long)t * F8_BK));
    if constexpr (32 % NWV == 0)
      fs_issue_x<XP, NWV, D>(xrs, xoff, smem + (t & (FS_NX - 1)) * FS_XT, so, w);
    else
      fs_issue_x_rc<XP, NWV>(xrs, smem + (t & (FS_NX - 1)) * FS_XT, so, w, p.M, p.ldx);
  };
  // --- weights: rows n0 + 16 f + r, bytes [32 g, 32 g + 32) of the K-step, through a buffer
  // descriptor (one 32-bit offset per fragment, the step in an SGPR: 64-bit row pointers spilled),
  // nontemporal (read once: the weights must not evict the activations from L2)
  // shuffled 1: a 16-row block's 2 KiB pieces consecutive over K; 2: the GB blocks of a workgroup's rows
  // side by side per K-step (GB x 2 KiB contiguous per workgroup and step)
  constexpr int GB = NWV * NF;
  const int sh = p.shuffled;
  const __amdgpu_buffer_rsrc_t wrs =
      make_rsrc(p.W, sh ? (unsigned)((long)p.N * p.K) : (unsigned)((long)(p.N - 1) * p.ldw + p.K));
  const int wstep = sh == 2 ? GB * 2048 : sh ? 2048 : F8_BK, whalf = sh ? 1024 : 16;
  const long ksteps = p.K / F8_BK;
  unsigned woff[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const int blk = (n0 >> 4) + f;  // 16-row block
    woff[f] = sh == 2 ? (unsigned)((((long)(blk / GB) * ksteps + k0 / F8_BK) * GB + blk % GB) * 2048 + lane * 16)
              : sh    ? (unsigned)(((long)blk * ksteps + k0 / F8_BK) * 2048 + lane * 16)
                      : (unsigned)((long)(n0 + 16 * f + r) * p.ldw + k0 + 32 * g);
  }
  auto load_w = [&](int t, i32x8 (&dst)[NF]) {
    fs_load_w<NF>(wrs, woff, __builtin_amdgcn_readfirstlane(t * wstep), whalf, dst);
  };

  f32x4 acc[16][NF];
#pragma unroll
  for (int tb = 0; tb < 16; ++tb)
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[tb][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int sw = f8_swz(r), c0 = ((2 * g) ^ sw) * 16, c1 = ((2 * g + 1) ^ sw) * 16;

  // prologue in the order the waits count: X(0) W(0) ... X(D-1) W(D-1)
  i32x8 wf[NSET][NF];
#pragma unroll
  for (int j = 0; j < D; ++j) {
    issue_x(j);
    load_w(j, wf[j]);
  }
  // one K-step on weight set J; ISSUE: it issues X(t+3), W(t+3); WN: the vmcnt it may leave
  // outstanding (all compile-time: no branch inside a step, where a branch made the compiler copy
  // the accumulators)
  auto step = [&](int t, auto J, auto ISSUE, auto WN) {
    constexpr int j = decltype(J)::value;
    fs_vmcnt<decltype(WN)::value>();  // this wave's X(t) and W(t) have landed
    fs_barrier();                      // every wave's X(t); every wave is past step t-1 (its X slot is free)
    if constexpr (decltype(ISSUE)::value) {
      issue_x(t + D);
      load_w(t + D, wf[(j + D) % NSET]);  // a set no live step uses (D + 1 of the 4 are live)
    }
    __builtin_amdgcn_sched_barrier(0);
    const char* st = smem + (t & (FS_NX - 1)) * FS_XT + r * F8_BK;
    // token-block fragments LA = 2 blocks ahead of their MFMAs (3 buffers), the interleave pinned
    constexpr int LA = 2;
    i32x8 xf[LA + 1];
#pragma unroll
    for (int i = 0; i < LA; ++i) xf[i] = f8_frag(st + i * 2048 + c0, st + i * 2048 + c1);
#pragma unroll
    for (int tb = 0; tb < 16; ++tb) {
      if (tb + LA < 16) xf[(tb + LA) % (LA + 1)] = f8_frag(st + (tb + LA) * 2048 + c0, st + (tb + LA) * 2048 + c1);
#pragma unroll
      for (int f = 0; f < NF; ++f)
        acc[tb][f] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wf[j][f], xf[tb % (LA + 1)], acc[tb][f], 0, 0, 0,
                                                                      127, 0, 127);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 2 * LA, 0);  // the first LA blocks: 2 ds_read_b128 each
#pragma unroll
    for (int tb = 0; tb < 16 - LA; ++tb) {
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // block tb + LA
      __builtin_amdgcn_sched_group_barrier(0x008, NF, 0);  // block tb's MFMAs
    }
    __builtin_amdgcn_sched_group_barrier(0x008, LA * NF, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
  using T = std::true_type;
  using F = std::false_type;
  using W0 = std::integral_constant<int, 0>;
  using WF = std::integral_constant<int, WAIT>;
  // every group but the last: full issue, WAIT outstanding
  const int last = nsteps - NSET;
  for (int t0 = 0; t0 < last; t0 += NSET) {
    step(t0 + 0, std::integral_constant<int, 0>{}, T{}, WF{});
    step(t0 + 1, std::integral_constant<int, 1>{}, T{}, WF{});
    step(t0 + 2, std::integral_constant<int, 2>{}, T{}, WF{});
    step(t0 + 3, std::integral_constant<int, 3>{}, T{}, WF{});
  }
  // the last group (t = nsteps - 4 + j): steps with j + D < 4 still issue (up to step nsteps - 1)
  // and wait as usual; the rest drain
  step(last + 0, std::integral_constant<int, 0>{}, std::bool_constant<(0 + D < NSET)>{},
       std::integral_constant<int, (0 + D < NSET) ? WAIT : 0>{});
  step(last + 1, std::integral_constant<int, 1>{}, std::bool_constant<(1 + D < NSET)>{},
       std::integral_constant<int, (1 + D < NSET) ? WAIT : 0>{});
  step(last + 2, std::integral_constant<int, 2>{}, std::bool_constant<(2 + D < NSET)>{},
       std::integral_constant<int, (2 + D < NSET) ? WAIT : 0>{});
  step(last + 3, std::integral_constant<int, 3>{}, F{}, W0{});

  // --- epilogue: lane holds C[n = 4 g + e][m = r] of each (token block, fragment) ------------------
  if (p.S > 1) {
    float* part = p.part + (long)blockIdx.y * p.M * p.N;
#pragma unroll
    for (int tb = 0; tb < 16; ++tb) {
      const int m = 16 * tb + r;
      if (m >= p.M) continue;
#pragma unroll
      for (int f = 0; f < NF; ++f)
        *reinterpret_cast<f32x4*>(part + (long)m * p.N + n0 + 16 * f + 4 * g) = acc[tb][f];
    }
    return;
  }
  f32x4 wsc[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) wsc[f] = *reinterpret_cast<const f32x4*>(p.ws + n0 + 16 * f + 4 * g);
#pragma unroll
  for (int tb = 0; tb < 16; ++tb) {
    const int m = 16 * tb + r;
    if (m >= p.M) continue;
    const float xsc = p.xs[m];
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      unsigned short o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = f2bf(acc[tb][f][e] * xsc * wsc[f][e]);
      *reinterpret_cast<uint2*>(p.Y + (long)m * p.ldy + n0 + 16 * f + 4 * g) =
          uint2{(unsigned)o[0] | ((unsigned)o[1] << 16), (unsigned)o[2] | ((unsigned)o[3] << 16)};
    }
  }
}

// y[m][n] = bf16(xs[m] ws[n] sum_s part[s][m][n]), 4 columns per thread
__global__ __launch_bounds__(256) void fp8_stream_reduce_kernel(const float* __restrict__ part,
                                                                const float* __restrict__ xs,
                                                                const float* __restrict__ ws, bf16_t* __restrict__ Y,
                                                                int M, int N, long ldy, int S) {
  const long n4 = N / 4, total = (long)M * n4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int m = (int)(i / n4), n = (int)(i % n4) * 4;
    f32x4 a = *reinterpret_cast<const f32x4*>(part + (long)m * N + n);
    for (int s2 = 1; s2 < S; ++s2) a += *reinterpret_cast<const f32x4*>(part + ((long)s2 * M + m) * N + n);
    const float xsc = xs[m];
    const f32x4 wsv = *reinterpret_cast<const f32x4*>(ws + n);
    unsigned short o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = f2bf(a[e] * xsc * wsv[e]);
    *reinterpret_cast<uint2*>(Y + (long)m * ldy + n) =
        uint2{(unsigned)o[0] | ((unsigned)o[1] << 16), (unsigned)o[2] | ((unsigned)o[3] << 16)};
  }
}

extern "C" bool dsa_fp8_stream_gemm_supported(int M, int N, int K, int rw, int S) {
  // rw weight rows per wave: 64 (4 waves: 256 per workgroup), 32 (8 waves: 256 per workgroup) or 28
  // (7 waves x 32 rows: 224 per workgroup, e.g. 256 workgroups for the 70B gate/up); each K slice whole
  // groups of 4 K-steps.  rw 64 without split only: its split-K epilogue (the accumulators spilled
  // around the last K-step's MFMAs) stored one wrong register per tile on gfx950
  // (profiles/fp8_stream_shuffle_r9u.txt), and rw 32 is the faster form there anyway
  const int wgr = rw == 28 ? 224 : 256;
  return M > 0 && M <= F8_MAXM && (rw == 32 || rw == 28 || (rw == 64 && S == 1)) && N > 0 && N % wgr == 0 &&
         S >= 1 && K > 0 && K % (4 * F8_BK * S) == 0;
}

// Y[M][N] = bf16(xs[m] ws[n] X W^T) with X [M][K] e4m3 (ldx bytes), W [N][K] e4m3 (ldw bytes); rw weight
// rows per wave (64 | 32 | 28: 7 waves); S > 1: `part` holds S * M * N floats; depth: weight / activation
// prefetch distance in K-steps for rw 32 (2, or 3: 4 weight register sets live; rw 64 runs 3, rw 28 2)
// shuffled: W is in the ops.serving.fp8_stream_shuffle order (ldw ignored; N * K bytes, < 4 GiB)
extern "C" hipError_t dsa_fp8_stream_gemm(const void* X, const float* xs, const void* W, const float* ws, void* Y,
                                          float* part, int M, int N, int K, long ldx, long ldw, long ldy, int rw,
                                          int S, int shuffled, int depth, hipStream_t st) {
  if (!dsa_fp8_stream_gemm_supported(M, N, K, rw, S) || ldx % 16 || ldw % 16 || ldy % 4 || ldx < K || ldw < K ||
      ldy < N)
    return hipErrorInvalidValue;
  if (S > 1 && part == nullptr) return hipErrorInvalidValue;
  if ((long)(M - 1) * ldx + K > 0xffffffffL) return hipErrorInvalidValue;  // X through a 32-bit buffer range
  if (shuffled && (long)N * K > 0xffffffffL) return hipErrorInvalidValue;
  if (depth != 2 && !(depth == 3 && rw == 32)) return hipErrorInvalidValue;  // weight prefetch distance in K-steps
  static bool attr = false;
  if (!attr) {
    DSA_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&fp8_stream_gemm_kernel<4, 4, 3>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, FS_NX * FS_XT));
    DSA_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&fp8_stream_gemm_kernel<8, 2, 2>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, FS_NX * FS_XT));
    DSA_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&fp8_stream_gemm_kernel<7, 2, 2>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, FS_NX * FS_XT));
    DSA_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&fp8_stream_gemm_kernel<8, 2, 3>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, FS_NX * FS_XT));
    attr = true;
  }
  FSArgs a{(const uint8_t*)X, xs, (const uint8_t*)W, ws, (bf16_t*)Y, part, ldx, ldw, ldy, M, N, K, S, shuffled};
  if (rw == 64)
    fp8_stream_gemm_kernel<4, 4, 3><<<dim3(N / 256, S), 256, FS_NX * FS_XT, st>>>(a);
  else if (rw == 28)
    fp8_stream_gemm_kernel<7, 2, 2><<<dim3(N / 224, S), 448, FS_NX * FS_XT, st>>>(a);
  else if (depth == 3)
    fp8_stream_gemm_kernel<8, 2, 3><<<dim3(N / 256, S), 512, FS_NX * FS_XT, st>>>(a);
  else
    fp8_stream_gemm_kernel<8, 2, 2><<<dim3(N / 256, S), 512, FS_NX * FS_XT, st>>>(a);
  DSA_CHECK(hipGetLastError());
  if (S > 1) {
    const long work = (long)M * (N / 4);
    const int g = (int)((work + 255) / 256 < 4096 ? (work + 255) / 256 : 4096);
    fp8_stream_reduce_kernel<<<g, 256, 0, st>>>(part, xs, ws, (bf16_t*)Y, M, N, ldy, S);
  }
  return hipGetLastError();
}
