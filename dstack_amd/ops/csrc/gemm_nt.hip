// Projection GEMM for CDNA4 (gfx950): C[M][N] (+)= A[M][K] · B[N][K]^T, bf16 in, fp32 accumulate,
// bf16 out -- the layout of every GEMM of the Llama training step once the weight-gradient and
// input-gradient operands are token-/reduction-contiguous (ops/functional.py): y = x W^T,
// dX = dY (W^T)^T, dW = (dY^T)(X^T)^T.  Epilogues fuse the SwiGLU forward into the gate/up GEMM
// and the SwiGLU backward into the down projection's input-gradient GEMM.
//
// Design (one workgroup = one 256x256 output tile, 8 waves = two groups of 4, one workgroup/CU):
//  * K advances in 64-deep tiles.  Each tile is four 16 KiB "units" in LDS -- A rows 0-127 (a0),
//    A rows 128-255 (a1), B rows 0-127 (b0), B rows 128-255 (b1) -- filled by LDS-DMA
//    (global_load_lds_dwordx4, 2 instructions per thread per unit) into a 2-tile ring (128 KiB).
//    Rows are 128 B; the 16-byte chunk c of row r sits at slot c ^ ((r >> 1) & 7), applied to the
//    per-lane DMA source address, so every ds_read_b128 fragment read is bank-conflict free.
//  * Wave (wr, wc) owns output rows {64wr + [0,64)} and {128 + 64wr + [0,64)} (m-subtiles 0/1,
//    from a0/a1) and columns {32wc + [0,32)} and {128 + 32wc + [0,32)} (n-subtiles 0/1, from
//    b0/b1): 128x64 per wave, 32 accumulators of mfma_f32_16x16x32_bf16.
//  * Eight phases per two K-tiles.  A phase = fragment reads + one unit of LDS-DMA, barrier, 16
//    MFMAs (one 64x32 quadrant x K 64), barrier.  Quadrant order per tile (m,n) = (0,0) (0,1)
//    (1,0) (1,1): reads 12 / 4 / 8 / 0 ds_read_b128.  Group 1 (waves 4-7) runs one barrier behind
//    group 0, so on every SIMD one wave issues MFMAs while its partner reads LDS and issues DMA.
//  * DMA schedule (unit issued per phase, tile t = this iteration's even tile):
//      P1 a1(t+1)  P2 b0(t+2)  P3 a0(t+2)  P4 b1(t+2) | P5 a1(t+2)  P6 b0(t+3)  P7 a0(t+3)  P8 b1(t+3)
//    Every unit is restaged only after its last read was retired before a barrier both groups
//    passed (b0: lgkmcnt(8) after the B reads that P1/P5 issue first).  vmcnt(6) at P4 / P8 leaves
//    three units in flight and retires exactly the tile read in the next four phases.
//  * XCD-aware tile order: workgroup ids are dealt round-robin to the 8 XCDs; the logical tile is
//    remapped so an XCD works on a contiguous, group-M ordered block of tiles that share A rows
//    and B rows in its L2.
//  * Operand roles in the MFMA are swapped (B fragment as the "A" operand), so each lane's
//    accumulator holds 4 consecutive output columns of one row: 8-byte row-contiguous pieces for
//    the LDS-staged epilogue.
//
// The SwiGLU tile maps its 256 columns to gate columns [f0, f0+128) (b0) and up columns
// [F+f0, F+f0+128) (b1): a lane holds g and u of the same (t, f) in accumulators n and n+2.
//
// KM form (weight gradients, C[M][N] (+)= A[K][M]^T B[K][N]: dW = dY^T X with both operands
// token-major, as the forward and the input gradient leave them -- no transposed copies): the same
// kernel with the units filled as 64 k-rows x 128 columns (256-byte rows, LDS-DMA from the
// [K][M] / [K][N] rows) and the fragments read with ds_read_b64_tr_b16 (gfx950's transposed LDS
// read): two reads of a 4-k x 16-column block give a lane 8 consecutive k of one column, the
// fragment the row read gives in the NT form.  Chunk c of k-row r sits at c ^ 2((r & 3) | (r & 8) >> 1):
// a 32-lane half reads 8 rows (4 per 16-lane group, the groups 8 rows apart) x 32 bytes, and the
// XOR puts them on 8 different 32-byte bank windows.  The XOR depends only on the lane, so the
// k-half and the 4-row step of a read are immediate offsets; each 16-column block has one address.
#include <stdlib.h>

#include <atomic>

#include "mfma_tiles.h"

using namespace dsa;

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short us4 __attribute__((ext_vector_type(4)));

constexpr int NT_BM = 256, NT_BN = 256, NT_BK = 64;
constexpr int UNIT = 16384;                // one 128 x 64 bf16 unit
constexpr int BUF = 4 * UNIT;              // a0 | a1 | b0 | b1
constexpr int EPI_LD = 520;                // epilogue LDS row stride (bytes): 256 bf16 + 8 B pad
constexpr int NT_LDS = 2 * BUF + 2 * 16384;  // 160 KiB: ring + room for the SwiGLU epilogue

// EPI_NONE: timing-only build (the accumulators are kept live, nothing is stored): what the
// epilogue's stores cost (tools/diag, accumulate = 2 in dsa_gemm_nt)
// EPI_SWIGLU_R / EPI_SWIGLU_BWD_R: the SwiGLU epilogues without the transposed copies (a^T, dgu^T),
// for a step whose weight gradients take the token-major operands (KM form): barrier-free, so the
// groups stay staggered as in the plain epilogue.
// EPI_STORE32 / EPI_ACC32: C is fp32 (an fp32 gradient accumulator: weight gradients summed over
// micro-batches without a bf16 rounding per micro-batch); EPI_ACC32_BF16: the last micro-batch --
// the fp32 accumulator F32 (ld ldc32) plus this tile, rounded once, written as bf16 to C.
// EPI_ROPE: the qkv projection with RoPE (rotate-half, head_dim 128) applied to the fp32
// accumulators of the first `rcols` columns (the q and k heads) before the one rounding to bf16.
// The tile's 256 columns are two heads; unit b0 takes dims 0-63 of both, b1 dims 64-127 (the B
// rows of the second 64 unit rows come from 64 rows further on), so a lane's accumulators n and
// n + 2 are the rotated pair (d, d + 64) of one row and head.
enum Epi { EPI_STORE = 0, EPI_ACC = 1, EPI_SWIGLU = 2, EPI_SWIGLU_BWD = 3, EPI_NONE = 4, EPI_SWIGLU_R = 5,
           EPI_SWIGLU_BWD_R = 6, EPI_STORE32 = 7, EPI_ACC32 = 8, EPI_ACC32_BF16 = 9, EPI_ROPE = 10,
           EPI_SWIGLU_F8 = 11 };
// EPI_SWIGLU_F8 (F8 only): the serving engine's fp8 gate/up projection -- the SwiGLU tile map of
// EPI_SWIGLU over raw e4m3 products, the row-wise scales srow[m] scol[n] applied in the epilogue,
// a = silu(g) u written as bf16 [M][F] (C2) and each wave's per-row max |a| over its 32 columns as
// pmax[m][F / 32] for the one-pass row quantizer that follows (no [M][2F] product in HBM).

struct NTArgs {
  const bf16_t* A;
  const bf16_t* B;
  bf16_t* C;      // output (STORE/ACC); gu (SWIGLU); dgu (SWIGLU_BWD)
  bf16_t* C2;     // a (SWIGLU)
  bf16_t* C3;     // a^T (SWIGLU); dgu^T (SWIGLU_BWD)
  const bf16_t* G;  // gu read by SWIGLU_BWD
  const float* F32;  // fp32 accumulator read by ACC32_BF16
  const float* rcos;  // ROPE: cos / sin tables [S][64] fp32
  const float* rsin;
  int rS;             // ROPE: sequence length (row % rS = position)
  int rcols;          // ROPE: columns [0, rcols) are rotated (multiple of 128)
  const float* srow;  // SWIGLU_F8: per-row (token) and per-output-channel scales, partial maxima
  const float* scol;
  float* pmax;
  long lda, ldb, ldc;
  long ldc32;
  int M, K;
  int ntn;        // tiles along N
  int nstride;    // column origin step per n tile (256 plain, 128 SwiGLU)
  int bsplit;     // offset of the second 128 columns (128 plain, F SwiGLU)
  int F;          // SwiGLU width (ld of a, columns of gu / 2)
  int group;      // tile-order group height (tile rows)
  int wg_per_xcd; // workgroups per XCD (gridDim / 8 when persistent)
  int* queue;     // dynamic tile order (persistent grids): [0..7] per-XCD tile counters, [8] exited
                  // workgroups (the last one re-zeroes the slot); null: the static order
  float* split_ws;  // split remainder (persistent grids): fp32 partial tiles [8 * wg_per_xcd / 2][2][65536]
  int* split_cnt;   // one ticket counter per split tile, zero between launches
  unsigned long long* trace;  // TRACE builds: per-phase s_memtime stamps of workgroup 0
};

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void nt_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int N>
__device__ __forceinline__ void nt_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int N>
__device__ __forceinline__ void nt_lgkmcnt() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// Two LDS-DMA instructions of one unit: this wave's 2 KiB piece (16 rows).  The global address is
// SGPR base + 32-bit per-lane offset (saddr form), the LDS address M0.  Inline asm: the compiler
// neither drains it (vmcnt(0)) in front of the next ds_read nor counts it; the loop counts by hand.
__device__ __forceinline__ void nt_dma(const bf16_t* sbase, unsigned v0, unsigned v1, unsigned lds) {
  unsigned keep;
  const unsigned lds1 = lds + 1024;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %4\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %3\n\t"
      "s_mov_b32 m0, %5\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %2, %3\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(v0), "v"(v1), "s"(sbase), "s"(lds), "s"(lds1)
      : "memory");
}

__device__ __forceinline__ int nt_xcd_tile(int b, int n) {
  const int xcd = b & 7, idx = b >> 3, per = n >> 3, rem = n & 7;
  return xcd * per + (xcd < rem ? xcd : rem) + idx;
}

__device__ __forceinline__ bf16x8 ldsr(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }

__device__ __forceinline__ float silu(float g) { return g / (1.f + __expf(-g)); }

// Row-contiguous 16-byte output pieces from two 16-column accumulator tiles x (columns c..c+15)
// and y (c+16..c+31): a lane of 16-lane row q holds columns 4q..4q+3 of each.  v_permlane16_swap
// (gfx950) swaps the odd rows of its first operand with the even rows of its second, after which
// rows 0/2 hold 8 consecutive columns of x, rows 1/3 8 of y: the lane's piece starts at column
// 16 * (q & 1) + 8 * (q >> 1) of the pair.  One dwordx4 store instead of two dwordx2: the store
// issue, not bandwidth, bounds an epilogue.
__device__ __forceinline__ unsigned nt_pk(unsigned short lo, unsigned short hi) {
  return (unsigned)lo | ((unsigned)hi << 16);
}

__device__ __forceinline__ us8 nt_pair8(const us4& x, const us4& y) {
  const auto r0 = __builtin_amdgcn_permlane16_swap(nt_pk(x[0], x[1]), nt_pk(y[0], y[1]), false, false);
  const auto r1 = __builtin_amdgcn_permlane16_swap(nt_pk(x[2], x[3]), nt_pk(y[2], y[3]), false, false);
  const unsigned d[4] = {r0[0], r1[0], r0[1], r1[1]};
  us8 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = (unsigned short)(d[i] & 0xffff);
    v[2 * i + 1] = (unsigned short)(d[i] >> 16);
  }
  return v;
}

// the same for fp32 accumulators (before rounding): 8 consecutive columns as floats
__device__ __forceinline__ void nt_pair8f(const f32x4& x, const f32x4& y, float (&o)[8]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x[j]), __float_as_uint(y[j]), false, false);
    o[j] = __uint_as_float(r[0]);
    o[4 + j] = __uint_as_float(r[1]);
  }
}

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

template <int MS, int NS>
__device__ __forceinline__ void nt_quadrant(f32x4 (&acc)[2][4][4], const bf16x8 (&af)[4][2],
                                            const bf16x8 (&bf)[2][2][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int n = 0; n < 2; ++n)
        acc[MS][mi][2 * NS + n] = mfma16(bf[NS][n][kk], af[mi][kk], acc[MS][mi][2 * NS + n]);
  __builtin_amdgcn_s_setprio(0);
}

// F8: one v_mfma_scale_f32_16x16x128_f8f6f4 (unit E8M0 scales: the fp8 rate) per accumulator, the
// two bf16 MFMAs' cycles for twice the k.  The fragments are read straight into 32-byte operands
// (nt_read_a8 / nt_read_b8: chunks g and g + 4 of the 128-byte row; A and B take the same chunk
// order, so the product runs over a permutation of k -- the same sum).
template <int MS, int NS>
__device__ __forceinline__ void nt_quadrant8(f32x4 (&acc)[2][4][4], const i32x8 (&af)[4], const i32x8 (&bf)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int n = 0; n < 2; ++n)
      acc[MS][mi][2 * NS + n] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bf[NS][n], af[mi], acc[MS][mi][2 * NS + n],
                                                                               0, 0, 0, 127, 0, 127);
  // pin the MFMAs into this phase: without the use, the compiler sinks them past the phase's
  // barrier into later phases, where their fragments stay live beside the next ones (spills)
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int n = 0; n < 2; ++n) asm volatile("" : "+v"(acc[MS][mi][2 * NS + n]));
  __builtin_amdgcn_s_setprio(0);
}

__device__ __forceinline__ i32x8 ldsr8(const char* p0, const char* p1) {
  const i32x4 a = *reinterpret_cast<const i32x4*>(p0), b = *reinterpret_cast<const i32x4*>(p1);
  return i32x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

template <int MS>
__device__ __forceinline__ void nt_read_a8(i32x8 (&af)[4], const char* buf, int ra0, int ra1) {
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) af[mi] = ldsr8(buf + MS * UNIT + mi * 2048 + ra0, buf + MS * UNIT + mi * 2048 + ra1);
}

template <int NS>
__device__ __forceinline__ void nt_read_b8(i32x8 (&bf)[2][2], const char* buf, int rb0, int rb1) {
#pragma unroll
  for (int n = 0; n < 2; ++n)
    bf[NS][n] = ldsr8(buf + (2 + NS) * UNIT + n * 2048 + rb0, buf + (2 + NS) * UNIT + n * 2048 + rb1);
}

// A fragments of m-subtile MS (unit a_MS of buffer `buf`): 4 row tiles x 2 k halves
template <int MS>
__device__ __forceinline__ void nt_read_a(bf16x8 (&af)[4][2], const char* buf, int ra0, int ra1) {
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    af[mi][0] = ldsr(buf + MS * UNIT + mi * 2048 + ra0);
    af[mi][1] = ldsr(buf + MS * UNIT + mi * 2048 + ra1);
  }
}

template <int NS>
__device__ __forceinline__ void nt_read_b(bf16x8 (&bf)[2][2][2], const char* buf, int rb0, int rb1) {
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    bf[NS][n][0] = ldsr(buf + (2 + NS) * UNIT + n * 2048 + rb0);
    bf[NS][n][1] = ldsr(buf + (2 + NS) * UNIT + n * 2048 + rb1);
  }
}

// KM form: the same fragments by transposed reads.  ka[mi] / kb[n]: the lane's byte offset of its
// 4-k x 16-column block for k-half 0, first 4 rows; +8192 selects k-half 1, +1024 the next 4 rows.
__device__ __forceinline__ bf16x8 km_frag(const char* p) {
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS3(bf16x4, p));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS3(bf16x4, p + 1024));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

template <int MS>
__device__ __forceinline__ void km_read_a(bf16x8 (&af)[4][2], const char* buf, const int (&ka)[4]) {
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    af[mi][0] = km_frag(buf + MS * UNIT + ka[mi]);
    af[mi][1] = km_frag(buf + MS * UNIT + ka[mi] + 8192);
  }
}

template <int NS>
__device__ __forceinline__ void km_read_b(bf16x8 (&bf)[2][2][2], const char* buf, const int (&kb)[2]) {
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    bf[NS][n][0] = km_frag(buf + (2 + NS) * UNIT + kb[n]);
    bf[NS][n][1] = km_frag(buf + (2 + NS) * UNIT + kb[n] + 8192);
  }
}

}  // namespace

// the epilogues the split-remainder path runs (the plain and fp32-accumulator ones)
template <int EPI>
constexpr bool nt_split_ok() {
  return EPI == EPI_STORE || EPI == EPI_ACC || EPI == EPI_STORE32 || EPI == EPI_ACC32 || EPI == EPI_ACC32_BF16;
}

// Tile origin (first row of A/C, first B row of the tile's first 128 columns) of logical tile t.
__device__ __forceinline__ void nt_tile_origin(const NTArgs& p, int t, int& m0, int& nb0) {
  const int ntm = p.M / NT_BM;
  const int in_group = p.group * p.ntn;
  const int first_m = (t / in_group) * p.group;
  const int gm = min(ntm - first_m, p.group);
  m0 = (first_m + (t % in_group) % gm) * NT_BM;
  nb0 = ((t % in_group) / gm) * p.nstride;
}

// F8: A and B are e4m3 bytes addressed as bf16 pairs (lda, ldb, K in 2-byte units): the K-tile
// of 64 "elements" is the same 128-byte row piece, so the DMA ring, the swizzle and the fragment
// reads are unchanged; only the MFMA differs (nt_quadrant).
template <int EPI, bool TRACE = false, bool KM = false, bool F8 = false>
__global__ __launch_bounds__(512) void gemm_nt_kernel(NTArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // the plain epilogues store straight from the accumulators while the next tile's prologue DMA
  // is in flight; the SwiGLU ones stage through LDS (transposed copies) and reload afterwards
  // the plain and SwiGLU-forward epilogues store straight from the accumulators (a^T through the
  // 32 KiB of LDS above the ring) while the next tile's first K-tiles stream into the ring; the
  // SwiGLU backward stages whole tiles through LDS and reloads afterwards
  constexpr bool OVERLAP = EPI != EPI_SWIGLU_BWD;
  // barrier-free epilogues keep the two wave groups staggered across tiles: group 0 stores its
  // half of the tile while group 1 issues its last MFMAs, group 1 stores while group 0 runs the
  // next tile's first MFMAs -- the stores take the place of a memory segment of the ping-pong
  constexpr bool STAGGERED = EPI != EPI_SWIGLU && EPI != EPI_SWIGLU_BWD;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  // TRACE: waves 0 and 4 of workgroup 0 stamp every phase boundary of K-iterations 8..11 into
  // the spare LDS above the ring (ds_write: no VMEM op disturbs the counted vmcnt), copied out at
  // the end -- where a phase's cycles go (reads, barrier waits, MFMAs)
  const bool tracer = TRACE && blockIdx.x == 0 && (w == 0 || w == 4);
  int tcount = 0;
  auto stamp = [&](int it) {
    if constexpr (TRACE) {
      if (tracer && it >= 8 && it < 12) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) reinterpret_cast<unsigned long long*>(smem + 2 * BUF)[(w >> 2) * 64 + tcount] = t;
        ++tcount;
      }
    }
  };

  // --- this workgroup's tiles: XCD x = blockIdx % 8 owns a contiguous slice of the logical tile
  // order; its workgroups take every (gridDim/8)-th tile of the slice (persistent when the grid is
  // smaller than the tile count)
  const int ntiles = (p.M / NT_BM) * p.ntn;
  const int xcd = blockIdx.x & 7, xj = blockIdx.x >> 3;
  const int per = ntiles >> 3, rem = ntiles & 7;
  const int cnt = per + (xcd < rem ? 1 : 0), start = xcd * per + (xcd < rem ? xcd : rem);
  const int stride = p.wg_per_xcd;
  const int nk = p.K / NT_BK;
  // Split remainder: a persistent grid runs ceil(cnt / stride) rounds per XCD; when the last round
  // holds r <= stride / 2 tiles, those tiles are split into two K halves (units), so the last round
  // takes half a tile's time on every workgroup instead of a whole one on half of them (the qkv
  // weight gradient: 384 tiles = 1.5 rounds; the down projection's: 3.5).  Unit u < full is tile u;
  // unit full + 2 s + h is half h of tile full + s (see the split-remainder block after the loop).
  const int rx = cnt % stride;
  const bool split = nt_split_ok<EPI>() && !TRACE && p.split_ws != nullptr && rx > 0 && 2 * rx <= stride &&
                     (nk & 3) == 0;
  const int full = cnt - (split ? rx : 0);
  const int ucnt = split ? full + 2 * rx : cnt;
  auto utile = [&](int u) { return u < full ? u : full + ((u - full) >> 1); };
  auto uhalf = [&](int u) { return u < full ? -1 : ((u - full) & 1); };
  auto ukb = [&](int u) { return uhalf(u) == 1 ? (nk >> 1) : 0; };
  auto uke = [&](int u) { return uhalf(u) == 0 ? (nk >> 1) : nk; };
  // Dynamic tile order (p.queue): instead of every (wg_per_xcd)-th tile of its XCD's slice, a
  // workgroup claims the slice's next tile from a per-XCD counter, one tile ahead (the claim for
  // tile i+2 is made at the top of tile i and read at its end, many barriers later, through two
  // LDS slots at the top of the 160 KiB that the plain / barrier-free epilogues never touch).
  // With some CUs held by a concurrent kernel -- RCCL's reduce-scatter / all-gather blocks beside
  // ZeRO-1's backward, the side-stream AdamW -- the static order waits for the late workgroups'
  // share; claimed tiles go to whoever is free (tools/diag/cu_hog.py).
  int* const q = p.queue;
  volatile int* qslot = reinterpret_cast<volatile int*>(smem + NT_LDS - 64);
  int local = xj, next = xj + stride, par = 0;
  if (q) {
    if (w == 0 && lane == 0) {
      const int a0 = atomicAdd(q + xcd, 1);
      qslot[0] = a0;
      qslot[1] = a0 < cnt ? atomicAdd(q + xcd, 1) : cnt;
    }
    __syncthreads();
    local = __builtin_amdgcn_readfirstlane(qslot[0]);  // (uniform: the DMA bases are SGPRs)
    next = __builtin_amdgcn_readfirstlane(qslot[1]);
    __syncthreads();
  }
  auto leave = [&]() {  // the last workgroup to leave re-zeroes the counters for the slot's next use
    if (q && w == 0 && lane == 0 && atomicAdd(q + 8, 1) == (int)gridDim.x - 1) {
#pragma unroll
      for (int i = 0; i < 9; ++i) q[i] = 0;
    }
  };
  if (local >= ucnt) {
    leave();
    return;
  }
  int m0, nb0;
  nt_tile_origin(p, start + utile(local), m0, nb0);

  // --- DMA: per-lane source offsets (bytes) of this wave's two 1 KiB pieces of a unit ----------
  // piece i covers unit rows 16w + 8i + (lane>>3); lane's 16 B slot (lane&7) holds the chunk
  // (lane&7) ^ (4i + (lane>>4)), the inverse of the read swizzle c ^ ((r>>1)&7).
  unsigned va[2], vb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if constexpr (KM) {
      // piece i = k-rows 8w + 4i + (lane >> 4), lane's 16 B slot (lane & 15) holds chunk
      // (lane & 15) ^ 2((r & 3) | (r & 8) >> 1)
      const int r = 8 * w + 4 * i + (lane >> 4);
      const int ch = (lane & 15) ^ (2 * ((r & 3) | ((r >> 1) & 4)));
      va[i] = (unsigned)((r * p.lda + ch * 8) * 2);
      vb[i] = (unsigned)((r * p.ldb + ch * 8) * 2);
    } else {
      const int r = 16 * w + 8 * i + (lane >> 3);
      const int ch = (lane & 7) ^ (4 * i + (lane >> 4));
      // ROPE: unit rows 64-127 are the B rows 128-191 past the unit's origin (the second head)
      const int rb = (EPI == EPI_ROPE && r >= 64) ? r + 64 : r;
      va[i] = (unsigned)((r * p.lda + ch * 8) * 2);
      vb[i] = (unsigned)((rb * p.ldb + ch * 8) * 2);
    }
  }
  const unsigned lds0 = (unsigned)(uintptr_t)LDS3(char, smem) + (unsigned)(w * 2048);
  const bf16_t *a_src0, *a_src1, *b_src0, *b_src1;
  auto set_src = [&](int tm0, int tnb0) {
    if constexpr (KM) {  // the tile's columns of the [K][M] / [K][N] rows
      a_src0 = p.A + tm0;
      a_src1 = p.A + tm0 + 128;
      b_src0 = p.B + tnb0;
      b_src1 = p.B + tnb0 + p.bsplit;
    } else {
      a_src0 = p.A + (long)tm0 * p.lda;
      a_src1 = p.A + (long)(tm0 + 128) * p.lda;
      b_src0 = p.B + (long)tnb0 * p.ldb;
      b_src1 = p.B + (long)(tnb0 + p.bsplit) * p.ldb;
    }
  };
  // units: 0 = a0, 1 = a1, 2 = b0, 3 = b1 of K-tile kt, into ring slot kt & 1
  auto dma = [&](int unit, int kt) {
    const unsigned dst = lds0 + (unsigned)((kt & 1) * BUF + unit * UNIT);
    const long ka = KM ? (long)kt * NT_BK * p.lda : (long)kt * NT_BK;
    const long kb = KM ? (long)kt * NT_BK * p.ldb : (long)kt * NT_BK;
    if (unit == 0) nt_dma(a_src0 + ka, va[0], va[1], dst);
    else if (unit == 1) nt_dma(a_src1 + ka, va[0], va[1], dst);
    else if (unit == 2) nt_dma(b_src0 + kb, vb[0], vb[1], dst);
    else nt_dma(b_src1 + kb, vb[0], vb[1], dst);
  };
  // K-tile 0 whole and K-tile 1's b0, b1 (its a0, a1 are the first phase's DMA): 12 instructions
  auto prologue = [&](int k0) {
    dma(0, k0);
    dma(1, k0);
    dma(2, k0);
    dma(3, k0);
    dma(2, k0 + 1);
    dma(3, k0 + 1);
  };

  // --- fragment read offsets: row (lane&15) of a 16-row tile, k chunk (lane>>4) (+4 for k 32..63)
  const int sw = (lane >> 1) & 7;
  const int c0 = (lane >> 4) ^ sw, c1 = ((lane >> 4) + 4) ^ sw;
  const int rrow = (lane & 15) * 128;
  const int ra0 = 64 * wr * 128 + rrow + 16 * c0, ra1 = 64 * wr * 128 + rrow + 16 * c1;
  const int rb0 = 32 * wc * 128 + rrow + 16 * c0, rb1 = 32 * wc * 128 + rrow + 16 * c1;
  const char* bufE = smem;
  const char* bufO = smem + BUF;
  f32x4 acc[2][4][4];
  bf16x8 af[4][2], bf[2][2][2];
  const int er = lane & 15, ec = 4 * (lane >> 4);
  // KM form: lane 4q + p of 16-lane group g addresses k-row 8g + q, columns 16j + 4p .. +3 of
  // block j (the chunk pair j ^ (q | (g & 1) << 2))
  int ka[4], kb[2];
  {
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3, x = q | ((g & 1) << 2);
    const int row = (8 * g + q) * 256 + 8 * pp;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) ka[mi] = row + 32 * ((4 * wr + mi) ^ x);
#pragma unroll
    for (int n = 0; n < 2; ++n) kb[n] = row + 32 * ((2 * wc + n) ^ x);
  }
  i32x8 af8[4], bf8[2][2];  // F8 fragments
  auto read_a0 = [&](const char* buf) {
    if constexpr (KM) km_read_a<0>(af, buf, ka);
    else if constexpr (F8) nt_read_a8<0>(af8, buf, ra0, ra1);
    else nt_read_a<0>(af, buf, ra0, ra1);
  };
  auto read_a1 = [&](const char* buf) {
    if constexpr (KM) km_read_a<1>(af, buf, ka);
    else if constexpr (F8) nt_read_a8<1>(af8, buf, ra0, ra1);
    else nt_read_a<1>(af, buf, ra0, ra1);
  };
  auto read_b = [&](const char* buf) {
    if constexpr (KM) {
      km_read_b<0>(bf, buf, kb);
      km_read_b<1>(bf, buf, kb);
    } else if constexpr (F8) {
      nt_read_b8<0>(bf8, buf, rb0, rb1);
      nt_read_b8<1>(bf8, buf, rb0, rb1);
    } else {
      nt_read_b<0>(bf, buf, rb0, rb1);
      nt_read_b<1>(bf, buf, rb0, rb1);
    }
  };

#define NT_QUAD(MS, NS)                                  \
  do {                                                   \
    if constexpr (F8) nt_quadrant8<MS, NS>(acc, af8, bf8); \
    else nt_quadrant<MS, NS>(acc, af, bf);               \
  } while (0)
  set_src(m0, nb0);
  prologue(ukb(local));
  nt_vmcnt<4>();
  nt_barrier();

  while (true) {
    if (!STAGGERED || local == xj) {
      if (wr == 1) nt_barrier();  // group 1 runs one barrier behind
    }
    const bool has_next = next < ucnt;
    if (q && w == 0 && lane == 0) qslot[par] = has_next ? atomicAdd(q + xcd, 1) : cnt;  // the tile after next
    int m1 = 0, nb1 = 0;
    if (has_next) nt_tile_origin(p, start + utile(next), m1, nb1);
    const int kbn = has_next ? ukb(next) : 0;  // the next unit's first K-tile
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[a][b][c] = f32x4{0.f, 0.f, 0.f, 0.f};

    // Four phases per two K-tiles t (ring slot E) and t+1 (slot O).  A phase: fragment reads and
    // two units of DMA, all reads retired (lgkmcnt(0)) before the first barrier, 32 MFMAs between
    // the barriers.  DMA: P1 a0,a1(t+1)->O  P2 b0,b1(t+2)->E  P3 a0,a1(t+2)->E  P4 b0,b1(t+3)->O;
    // each unit is restaged at least one phase after the phase whose barrier retired its reads.
    // vmcnt(4) at P2 / P4 keeps two units in flight and retires the tile the next phase reads.
    // With the plain epilogues the K-tile stream runs on across tiles: the last iteration loads
    // the next tile's K-tiles 0 and 1, so a tile starts with no prologue.
    const int kb0 = ukb(local);
    const int niter = (uke(local) - kb0) >> 1;
    for (int it = 0; it < niter; ++it) {
      const int t = kb0 + 2 * it;
      const bool more = it + 1 < niter;
      const bool go = more || (OVERLAP && has_next);
      const int t2 = more ? t + 2 : kbn, t3 = more ? t + 3 : kbn + 1;
      // P1: m-subtile 0 of tile t
      stamp(it);
      read_b(bufE);
      read_a0(bufE);
      dma(0, t + 1);
      dma(1, t + 1);
      if (!more && go) set_src(m1, nb1);
      nt_lgkmcnt<0>();
      stamp(it);
      nt_barrier();
      stamp(it);
      NT_QUAD(0, 0);
      NT_QUAD(0, 1);
      stamp(it);
      nt_barrier();
      // P2: m-subtile 1 of tile t; retire tile t+1
      stamp(it);
      read_a1(bufE);
      if (go) {
        dma(2, t2);
        dma(3, t2);
        nt_vmcnt<4>();
      } else {
        nt_vmcnt<0>();
      }
      nt_lgkmcnt<0>();
      stamp(it);
      nt_barrier();
      stamp(it);
      NT_QUAD(1, 0);
      NT_QUAD(1, 1);
      stamp(it);
      nt_barrier();
      // P3: m-subtile 0 of tile t+1
      stamp(it);
      read_b(bufO);
      read_a0(bufO);
      if (go) {
        dma(0, t2);
        dma(1, t2);
      }
      nt_lgkmcnt<0>();
      stamp(it);
      nt_barrier();
      stamp(it);
      NT_QUAD(0, 0);
      NT_QUAD(0, 1);
      stamp(it);
      nt_barrier();
      // P4: m-subtile 1 of tile t+1; retire tile t+2
      stamp(it);
      read_a1(bufO);
      if (go) {
        dma(2, t3);
        dma(3, t3);
        nt_vmcnt<4>();
      }
      nt_lgkmcnt<0>();
      stamp(it);
      nt_barrier();
      stamp(it);
      NT_QUAD(1, 0);
      NT_QUAD(1, 1);
      stamp(it);
      nt_barrier();
    }
    if constexpr (TRACE) {
      if (tracer && lane < 64 && tcount > 0)
        p.trace[(w >> 2) * 64 + lane] = reinterpret_cast<unsigned long long*>(smem + 2 * BUF)[(w >> 2) * 64 + lane];
    }
    if constexpr (!STAGGERED) {
      if (wr == 0) nt_barrier();  // re-align the groups
    }
    if constexpr (!OVERLAP) nt_barrier();  // every wave is past its last fragment read: LDS is free

    // --- epilogue (a lambda: the split-remainder path below runs it from its own branch) ---------
    auto run_epilogue = [&]() {
    // --- epilogue ---------------------------------------------------------------------------------
    // accumulator (ms, mi, n): tile row 128ms + 64wr + 16mi + (lane&15), tile columns
    // 128(n>>1) + 32wc + 16(n&1) + 4(lane>>4) + [0,4)
    if constexpr (EPI == EPI_NONE) {
#pragma unroll
      for (int ms = 0; ms < 2; ++ms)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int n = 0; n < 4; ++n) asm volatile("" ::"v"(acc[ms][mi][n]));
    } else if constexpr (EPI == EPI_STORE || EPI == EPI_ACC) {
      // 16-byte pieces: column pair p (n = 2p, 2p+1) of row (ms, mi) -> columns
      // 128p + 32wc + 16(q&1) + 8(q>>1) .. +8 of the lane's row (q = lane >> 4)
      const int q = lane >> 4;
      bf16_t* cbase = p.C + (long)(m0 + 64 * wr + er) * p.ldc + nb0 + 32 * wc + 16 * (q & 1) + 8 * (q >> 1);
      if constexpr (EPI == EPI_ACC) {
        us8 old[2][4][2];
#pragma unroll
        for (int ms = 0; ms < 2; ++ms)
#pragma unroll
          for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int pp = 0; pp < 2; ++pp)
              old[ms][mi][pp] = *reinterpret_cast<const us8*>(cbase + (long)(128 * ms + 16 * mi) * p.ldc + pp * p.bsplit);
#pragma unroll
        for (int ms = 0; ms < 2; ++ms)
#pragma unroll
          for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int pp = 0; pp < 2; ++pp) {
              float v[8];
              nt_pair8f(acc[ms][mi][2 * pp], acc[ms][mi][2 * pp + 1], v);
              us8 o;
#pragma unroll
              for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j] + bf2f(old[ms][mi][pp][j]));
              *reinterpret_cast<us8*>(cbase + (long)(128 * ms + 16 * mi) * p.ldc + pp * p.bsplit) = o;
            }
      } else {
#pragma unroll
        for (int ms = 0; ms < 2; ++ms)
#pragma unroll
          for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int pp = 0; pp < 2; ++pp) {
              us4 x, y;
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                x[j] = f2bf(acc[ms][mi][2 * pp][j]);
                y[j] = f2bf(acc[ms][mi][2 * pp + 1][j]);
              }
              *reinterpret_cast<us8*>(cbase + (long)(128 * ms + 16 * mi) * p.ldc + pp * p.bsplit) = nt_pair8(x, y);
            }
      }
    } else if constexpr (EPI == EPI_ROPE) {
      // unit column u = 32wc + 16(n&1) + 4q + j of b0 (b1) is dim 32(wc&1) + 16(n&1) + 4q + j (+64)
      // of head nb0/128 + (wc>>1); the 8-column pieces of EPI_STORE land at
      // nb0 + 128(wc>>1) + 32(wc&1) + 16(q&1) + 8(q>>1), the b1 piece 64 columns on
      const int q = lane >> 4;
      const int hcol = nb0 + 128 * (wc >> 1);
      if (hcol < p.rcols) {  // wave-uniform: q / k heads rotate, v heads pass through
        const int pos0 = m0 % p.rS + 64 * wr + er;
        const int d0 = 32 * (wc & 1) + 4 * q;
#pragma unroll
        for (int ms = 0; ms < 2; ++ms)
#pragma unroll
          for (int mi = 0; mi < 4; ++mi) {
            const long t = (long)(pos0 + 128 * ms + 16 * mi) * 64 + d0;
#pragma unroll
            for (int n = 0; n < 2; ++n) {
              const f4 c = *reinterpret_cast<const f4*>(p.rcos + t + 16 * n);
              const f4 sn = *reinterpret_cast<const f4*>(p.rsin + t + 16 * n);
              const f32x4 x1 = acc[ms][mi][n], x2 = acc[ms][mi][n + 2];
              acc[ms][mi][n] = x1 * c - x2 * sn;
              acc[ms][mi][n + 2] = x2 * c + x1 * sn;
            }
          }
      }
      bf16_t* cbase = p.C + (long)(m0 + 64 * wr + er) * p.ldc + hcol + 32 * (wc & 1) + 16 * (q & 1) + 8 * (q >> 1);
#pragma unroll
      for (int ms = 0; ms < 2; ++ms)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int pp = 0; pp < 2; ++pp) {
            us4 x, y;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              x[j] = f2bf(acc[ms][mi][2 * pp][j]);
              y[j] = f2bf(acc[ms][mi][2 * pp + 1][j]);
            }
            *reinterpret_cast<us8*>(cbase + (long)(128 * ms + 16 * mi) * p.ldc + 64 * pp) = nt_pair8(x, y);
          }
    } else if constexpr (EPI == EPI_STORE32 || EPI == EPI_ACC32 || EPI == EPI_ACC32_BF16) {
      // the same 8-column pieces as EPI_STORE, as 8 floats (two 16-byte accesses); old values are
      // loaded one 128-row half (ms) at a time: 64 VGPRs beside the 128 of the accumulators
      const int q = lane >> 4;
      const long col = nb0 + 32 * wc + 16 * (q & 1) + 8 * (q >> 1);
      const long row = m0 + 64 * wr + er;
      float* c32 = reinterpret_cast<float*>(p.C) + row * p.ldc + col;
      const float* o32 = (EPI == EPI_ACC32_BF16 ? p.F32 + row * p.ldc32 + col : c32);
      const long ldo = EPI == EPI_ACC32_BF16 ? p.ldc32 : p.ldc;
#pragma unroll
      for (int ms = 0; ms < 2; ++ms) {
        f4 old[4][2][2];
        if constexpr (EPI != EPI_STORE32) {
#pragma unroll
          for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int pp = 0; pp < 2; ++pp)
#pragma unroll
              for (int h = 0; h < 2; ++h)
                old[mi][pp][h] = *reinterpret_cast<const f4*>(o32 + (long)(128 * ms + 16 * mi) * ldo + pp * p.bsplit + 4 * h);
        }
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int pp = 0; pp < 2; ++pp) {
            float v[8];
            nt_pair8f(acc[ms][mi][2 * pp], acc[ms][mi][2 * pp + 1], v);
            if constexpr (EPI != EPI_STORE32) {
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] += old[mi][pp][j >> 2][j & 3];
            }
            if constexpr (EPI == EPI_ACC32_BF16) {
              us8 o;
#pragma unroll
              for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j]);
              *reinterpret_cast<us8*>(p.C + row * p.ldc + col + (long)(128 * ms + 16 * mi) * p.ldc + pp * p.bsplit) = o;
            } else {
              float* dst = c32 + (long)(128 * ms + 16 * mi) * p.ldc + pp * p.bsplit;
              *reinterpret_cast<f4*>(dst) = f4{v[0], v[1], v[2], v[3]};
              *reinterpret_cast<f4*>(dst + 4) = f4{v[4], v[5], v[6], v[7]};
            }
          }
      }
    } else if constexpr (EPI == EPI_SWIGLU_R) {
      // gu and a straight from the accumulators, no transposed copy
      const int q = lane >> 4;
      const int pc = 16 * (q & 1) + 8 * (q >> 1);
      bf16_t* gbase = p.C + (long)(m0 + 64 * wr + er) * p.ldc + nb0 + 32 * wc + pc;
      bf16_t* abase = p.C2 + (long)(m0 + 64 * wr + er) * p.F + nb0 + 32 * wc + pc;
#pragma unroll
      for (int ms = 0; ms < 2; ++ms)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          us4 g4[2], u4[2], o4[2];
#pragma unroll
          for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              g4[n][j] = f2bf(acc[ms][mi][n][j]);
              u4[n][j] = f2bf(acc[ms][mi][n + 2][j]);
              o4[n][j] = f2bf(silu(bf2f(g4[n][j])) * bf2f(u4[n][j]));
            }
          const long ro = (long)(128 * ms + 16 * mi);
          *reinterpret_cast<us8*>(gbase + ro * p.ldc) = nt_pair8(g4[0], g4[1]);
          *reinterpret_cast<us8*>(gbase + ro * p.ldc + p.bsplit) = nt_pair8(u4[0], u4[1]);
          *reinterpret_cast<us8*>(abase + ro * p.F) = nt_pair8(o4[0], o4[1]);
        }
    } else if constexpr (EPI == EPI_SWIGLU_F8) {
      // acc n / n + 2 = raw g / u of (row, f); the deferred-scale SwiGLU-quant's arithmetic
      // (swiglu_quant_rows_kernel<SCALED>): bf16(raw) * rs * cs -> bf16, a = bf16(silu(g) u)
      const int q = lane >> 4;
      const int f0 = nb0 + 32 * wc;  // this wave's 32 columns of the F outputs
      bf16_t* abase = p.C2 + (long)(m0 + 64 * wr + er) * p.F + f0 + 16 * (q & 1) + 8 * (q >> 1);
      f4 cg[2], cu[2];
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        cg[n] = *reinterpret_cast<const f4*>(p.scol + f0 + 16 * n + 4 * q);
        cu[n] = *reinterpret_cast<const f4*>(p.scol + p.F + f0 + 16 * n + 4 * q);
      }
      const int P = p.F / 32;
#pragma unroll
      for (int ms = 0; ms < 2; ++ms)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          const int row = m0 + 128 * ms + 64 * wr + 16 * mi + er;
          const float r = p.srow[row];
          us4 o4[2];
          float am = 0.f;
#pragma unroll
          for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float g = bf2f(f2bf(bf2f(f2bf(acc[ms][mi][n][j])) * r * cg[n][j]));
              const float u = bf2f(f2bf(bf2f(f2bf(acc[ms][mi][n + 2][j])) * r * cu[n][j]));
              o4[n][j] = f2bf(silu(g) * u);
              am = fmaxf(am, fabsf(bf2f(o4[n][j])));
            }
          *reinterpret_cast<us8*>(abase + (long)(128 * ms + 16 * mi) * p.F) = nt_pair8(o4[0], o4[1]);
          am = fmaxf(am, __shfl_xor(am, 16));
          am = fmaxf(am, __shfl_xor(am, 32));
          if (q == 0) p.pmax[(long)row * P + f0 / 32] = am;
        }
    } else if constexpr (EPI == EPI_SWIGLU_BWD_R) {
      // acc = da[t][f] (plain column map); 16-byte pieces of 8 consecutive f: g, u loaded, dg, du
      // stored -- dg = da * u * silu'(g), du = da * silu(g), da rounded to bf16 as the unfused path
      // g, u of row group i + 1 are loaded while group i is computed and stored (two register
      // sets of 16 VGPRs): each group's load latency was exposed, 8 times per tile
      const int q = lane >> 4;
      const int pc = 32 * wc + 16 * (q & 1) + 8 * (q >> 1);
      const long rbase = (long)(m0 + 64 * wr + er) * (2L * p.F) + nb0 + pc;
      us8 g8[2][2], u8[2][2];
      auto load_gu = [&](int i, int b) {
        const long ro = rbase + (long)(128 * (i >> 2) + 16 * (i & 3)) * (2L * p.F);
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          g8[b][pp] = *reinterpret_cast<const us8*>(p.G + ro + 128 * pp);
          u8[b][pp] = *reinterpret_cast<const us8*>(p.G + ro + 128 * pp + p.F);
        }
      };
      load_gu(0, 0);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int ms = i >> 2, mi = i & 3, b = i & 1;
        if (i + 1 < 8) load_gu(i + 1, b ^ 1);
        const long ro = rbase + (long)(128 * ms + 16 * mi) * (2L * p.F);
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          float v[8];
          nt_pair8f(acc[ms][mi][2 * pp], acc[ms][mi][2 * pp + 1], v);
          us8 dg, du;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float da = bf2f(f2bf(v[j]));
            const float g = bf2f(g8[b][pp][j]), u = bf2f(u8[b][pp][j]);
            const float sg = 1.f / (1.f + __expf(-g));
            const float sl = g * sg;
            dg[j] = f2bf(da * u * (sg + sl * (1.f - sg)));
            du[j] = f2bf(da * sl);
          }
          *reinterpret_cast<us8*>(p.C + ro + 128 * pp) = dg;
          *reinterpret_cast<us8*>(p.C + ro + 128 * pp + p.F) = du;
        }
      }
    } else if constexpr (EPI == EPI_SWIGLU) {
      // gu and a = silu(g) * u (from the bf16-rounded g, u: what the backward re-reads from gu)
      // straight from the accumulators; a^T through the spare LDS, one 128-token half at a time
      const int f0 = nb0;  // nstride 128: the tile's gate columns
      const int q = lane >> 4;
      const int pc = 16 * (q & 1) + 8 * (q >> 1);  // the lane's 16-byte piece of a 32-column pair
      bf16_t* gbase = p.C + (long)(m0 + 64 * wr + er) * p.ldc + f0 + 32 * wc + pc;
      bf16_t* abase = p.C2 + (long)(m0 + 64 * wr + er) * p.F + f0 + 32 * wc + pc;
      // a^T half: [128 f][128 t] bf16, 256-byte rows, 16-byte chunk c of row f at c ^ ((f >> 2) & 7)
      // (the 2-byte transposed writes of lanes 4 f-rows apart land in different banks)
      char* sat = smem + 2 * BUF;
#pragma unroll
      for (int ms = 0; ms < 2; ++ms) {
        us4 o[4][2];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          us4 g4[2], u4[2];
#pragma unroll
          for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              g4[n][j] = f2bf(acc[ms][mi][n][j]);
              u4[n][j] = f2bf(acc[ms][mi][n + 2][j]);
              o[mi][n][j] = f2bf(silu(bf2f(g4[n][j])) * bf2f(u4[n][j]));
            }
          const long ro = (long)(128 * ms + 16 * mi);
          *reinterpret_cast<us8*>(gbase + ro * p.ldc) = nt_pair8(g4[0], g4[1]);
          *reinterpret_cast<us8*>(gbase + ro * p.ldc + p.bsplit) = nt_pair8(u4[0], u4[1]);
          *reinterpret_cast<us8*>(abase + ro * p.F) = nt_pair8(o[mi][0], o[mi][1]);
        }
        nt_barrier();  // the previous half's a^T rows have been read
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int f = 32 * wc + 16 * n + ec + j, t = 64 * wr + 16 * mi + er;
              *reinterpret_cast<bf16_t*>(sat + f * 256 + ((2 * t) ^ (((f >> 2) & 7) << 4))) = o[mi][n][j];
            }
        nt_barrier();
        // 128 rows x 256 B: 16 B per lane, a wave writes 4 rows per instruction
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 32 * i + 4 * w + (lane >> 4), c = 8 * (lane & 15);
          *reinterpret_cast<us8*>(p.C3 + (long)(f0 + r) * p.M + m0 + 128 * ms + c) =
              *reinterpret_cast<const us8*>(sat + r * 256 + ((2 * c) ^ (((r >> 2) & 7) << 4)));
        }
      }
    } else {  // EPI_SWIGLU_BWD: acc = da[t][f] for the tile's 256 f columns (plain column map)
      // dg = da * u * silu'(g), du = da * silu(g); g, u from gu[t][f], gu[t][F + f]
      char* sdt = smem;  // dgu^T staging: [256 f][256 t] for gate, then up (two passes)
      us4 dgv[2][4][4], duv[2][4][4];
#pragma unroll
      for (int ms = 0; ms < 2; ++ms)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int n = 0; n < 4; ++n) {
            const int r = 128 * ms + 64 * wr + 16 * mi + er;
            const int c = 128 * (n >> 1) + 32 * wc + 16 * (n & 1) + ec;
            const bf16_t* gp = p.G + (long)(m0 + r) * (2L * p.F) + nb0 + c;
            const us4 g4 = *reinterpret_cast<const us4*>(gp);
            const us4 u4 = *reinterpret_cast<const us4*>(gp + p.F);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float da = bf2f(f2bf(acc[ms][mi][n][j]));
              const float g = bf2f(g4[j]), u = bf2f(u4[j]);
              const float sg = 1.f / (1.f + __expf(-g));
              const float s = g * sg;
              dgv[ms][mi][n][j] = f2bf(da * u * (sg + s * (1.f - sg)));
              duv[ms][mi][n][j] = f2bf(da * s);
            }
            bf16_t* dp = p.C + (long)(m0 + r) * (2L * p.F) + nb0 + c;
            *reinterpret_cast<us4*>(dp) = dgv[ms][mi][n];
            *reinterpret_cast<us4*>(dp + p.F) = duv[ms][mi][n];
          }
      // dgu^T [2F][T]: gate rows nb0 + c, up rows F + nb0 + c; staged transposed per half
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        if (half) nt_barrier();
#pragma unroll
        for (int ms = 0; ms < 2; ++ms)
#pragma unroll
          for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int n = 0; n < 4; ++n) {
              const int r = 128 * ms + 64 * wr + 16 * mi + er;
              const int c = 128 * (n >> 1) + 32 * wc + 16 * (n & 1) + ec;
#pragma unroll
              for (int j = 0; j < 4; ++j)
                *reinterpret_cast<bf16_t*>(sdt + (c + j) * EPI_LD + 2 * r) =
                    half ? duv[ms][mi][n][j] : dgv[ms][mi][n][j];
            }
        nt_barrier();
#pragma unroll 4
        for (int i = 0; i < 32; ++i) {
          const int r = 8 * i + w, c = 4 * lane;
          *reinterpret_cast<us4*>(p.C3 + (long)(half * p.F + nb0 + r) * p.M + m0 + c) =
              *reinterpret_cast<const us4*>(sdt + r * EPI_LD + 2 * c);
        }
      }
    }
    };  // run_epilogue
    // --- split remainder: both K halves of a last-round tile store their fp32 accumulators; the
    // half that takes the tile's ticket second adds the other's and runs the epilogue (no waiting
    // on a partner).  The epilogue is inlined once per branch: a single copy reached by both the
    // plain and the combined accumulators made the register allocator spill them on every tile.
    bool aligned = false;
    if constexpr (nt_split_ok<EPI>()) {
      const int khalf = split ? uhalf(local) : -1;
      if (khalf >= 0) {
        if constexpr (STAGGERED) {
          if (wr == 0) nt_barrier();  // group 1 has finished its last phase: both groups aligned
        }
        aligned = true;
        const int pair = xcd * (stride >> 1) + ((local - full) >> 1);
        float* mine = p.split_ws + (long)(2 * pair + khalf) * 65536 + w * 8192 + 4 * lane;
        const float* other = p.split_ws + (long)(2 * pair + (khalf ^ 1)) * 65536 + w * 8192 + 4 * lane;
#pragma unroll
        for (int ms = 0; ms < 2; ++ms)
#pragma unroll
          for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int n = 0; n < 4; ++n)
              *reinterpret_cast<f32x4*>(mine + ((ms * 4 + mi) * 4 + n) * 256) = acc[ms][mi][n];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        nt_barrier();  // every wave's partial is stored
        volatile int* tslot = reinterpret_cast<volatile int*>(smem + NT_LDS - 64);
        if (w == 0 && lane == 0) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          const int t = __hip_atomic_fetch_add(p.split_cnt + pair, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (t == 1) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(p.split_cnt + pair, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next launch
          }
          tslot[2] = t;
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the broadcast lands before the barrier
        }
        nt_barrier();
        if (tslot[2] == 1) {
          // 4 pieces at a time (the compiler would issue all 32 loads first: 128 more VGPRs)
#pragma unroll
          for (int ms = 0; ms < 2; ++ms)
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
#pragma unroll
              for (int n = 0; n < 4; ++n)
                acc[ms][mi][n] += *reinterpret_cast<const f32x4*>(other + ((ms * 4 + mi) * 4 + n) * 256);
#pragma unroll
              for (int n = 0; n < 4; ++n) asm volatile("" : "+v"(acc[ms][mi][n])::"memory");
            }
          run_epilogue();
        }
      } else {
        run_epilogue();
      }
    } else {
      run_epilogue();
    }
    if (!has_next) {
      if constexpr (STAGGERED) {
        if (wr == 0 && !aligned) nt_barrier();  // equal barrier counts for both groups at exit
      }
      leave();
      break;
    }
    if constexpr (!OVERLAP) {
      nt_barrier();  // every wave is done with the LDS staging
      set_src(m1, nb1);
      prologue(kbn);
      nt_vmcnt<4>();
      nt_barrier();
    }
    local = next;
    next = q ? __builtin_amdgcn_readfirstlane(qslot[par]) : next + stride;
    par ^= 1;
    m0 = m1;
    nb0 = nb1;
  }
}

#undef NT_QUAD

namespace {

bool nt_shape_ok(int M, int N, int K) {
  return M > 0 && N > 0 && K > 0 && M % NT_BM == 0 && N % NT_BN == 0 && K % (2 * NT_BK) == 0;
}

// tile-order group height: an XCD's 32 concurrent tiles are a group x (32 / group) block; taller
// blocks suit wide outputs, wider blocks tall ones (tools/diag/gemm_group_sweep.sh,
// profiles/gemm_nt_group_r7d.txt: group 8 for the 8192 x 28672 gate/up GEMM, 4 for the 28672 x 4096
// weight gradient)
int nt_group(int ntm, int ntn) {
  const int g = ntm > 2 * ntn ? 4 : 8;
  return ntm >= g ? g : ntm;
}

int nt_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cus[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

// One workgroup per CU (128 KiB ring): a grid of min(tiles, CUs rounded down to a multiple of 8)
// workgroups that loop over their XCD's tiles.
// Dynamic-order counter slots: one 64-byte slot per launch from a ring per device, zeroed once; a
// launch's last workgroup re-zeroes its slot, which is reused 1024 launches later.
constexpr int NT_QSLOTS = 1024;
int* nt_queue_slot(hipStream_t st) {
  static int* ring[64] = {nullptr};
  static std::atomic<unsigned> seq[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  if (!ring[dev]) {
    int* r = nullptr;
    if (hipMalloc(&r, NT_QSLOTS * 64) != hipSuccess) return nullptr;
    if (hipMemset(r, 0, NT_QSLOTS * 64) != hipSuccess) return nullptr;
    ring[dev] = r;
  }
  return ring[dev] + (seq[dev].fetch_add(1) % NT_QSLOTS) * 16;
}

// Split-remainder workspaces (see the kernel's `split`): a ring of NT_SPLIT_RING per device, one per
// launch in turn (the launches of one stream are ordered; concurrent launches on other streams take
// the other entry): fp32 partials and one ticket counter per split tile (zeroed once; the second
// arriver re-zeroes it).  Not under stream capture (no allocation there).
constexpr int NT_SPLIT_RING = 2;
bool nt_split_slot(hipStream_t st, int pairs, float** ws, int** cnt) {
  static float* wring[64][NT_SPLIT_RING] = {{nullptr}};
  static int* cring[64][NT_SPLIT_RING] = {{nullptr}};
  static int have[64][NT_SPLIT_RING] = {{0}};
  static std::atomic<unsigned> seq[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return false;
  const int i = (int)(seq[dev].fetch_add(1) % NT_SPLIT_RING);
  if (have[dev][i] < pairs) {
    float* w = nullptr;
    int* c = nullptr;
    if (hipMalloc(&w, (size_t)pairs * 2 * 65536 * sizeof(float)) != hipSuccess) return false;
    if (hipMalloc(&c, (size_t)pairs * sizeof(int)) != hipSuccess || hipMemset(c, 0, (size_t)pairs * sizeof(int)) != hipSuccess) {
      (void)hipFree(w);
      return false;
    }
    if (wring[dev][i]) (void)hipFree(wring[dev][i]);  // (hipFree synchronises the device)
    if (cring[dev][i]) (void)hipFree(cring[dev][i]);
    wring[dev][i] = w;
    cring[dev][i] = c;
    have[dev][i] = pairs;
  }
  *ws = wring[dev][i];
  *cnt = cring[dev][i];
  return true;
}

// EPIs whose epilogue stages through LDS (the SwiGLU forms with transposed copies) keep the
// static order: the dynamic order's broadcast slots sit at the top of the LDS they use.
template <int EPI>
constexpr bool nt_dynamic_ok() { return EPI != EPI_SWIGLU && EPI != EPI_SWIGLU_BWD; }


// Grid form chosen at run time (dsa_gemm_nt_set_grid): -1 = DSTACK_AMD_GEMM_NT_PERSISTENT (default
// persistent), 0 = one workgroup per tile, 1 = persistent.  The trainer picks the per-tile grid for
// the micro-batch whose backward runs beside RCCL's reduce-scatter / all-gather: a collective's
// workgroups hold CUs, and a persistent grid's workgroups on those CUs then start only when the
// collective ends (tools/diag/cu_hog.py, profiles/cu_hog_*_r9q.txt: 1.53 -> 2.31 ms for the
// gate/up GEMM beside 32 held CUs, 1.72 per tile).
std::atomic<int> g_nt_grid{-1};

template <int EPI, bool TRACE = false, bool KM = false, bool F8 = false>
hipError_t nt_launch(NTArgs a, int tiles, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    DSA_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt_kernel<EPI, TRACE, KM, F8>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, NT_LDS));
    attr = true;
  }
  const int cap = (nt_cus() / 8) * 8;
  int grid = tiles;
  a.wg_per_xcd = 1 << 30;  // one tile per workgroup
  // DSTACK_AMD_GEMM_NT_PERSISTENT=0: one workgroup per tile even when the tiles outnumber the CUs
  // (A/B against CUs held by a concurrent kernel, tools/diag/cu_hog.py)
  static const bool persistent = [] {
    const char* v = getenv("DSTACK_AMD_GEMM_NT_PERSISTENT");
    return !(v && atoi(v) == 0);
  }();
  // DSTACK_AMD_GEMM_NT_DYNAMIC=1: claimed (dynamic) tile order; 0 (default): the static order
  static const bool dynamic = [] {
    const char* v = getenv("DSTACK_AMD_GEMM_NT_DYNAMIC");
    return v && atoi(v) == 1;
  }();
  const int mode = g_nt_grid.load(std::memory_order_relaxed);
  if ((mode >= 0 ? mode == 1 : persistent) && tiles > cap && cap >= 8) {
    grid = cap;
    a.wg_per_xcd = cap / 8;
    if (dynamic && !TRACE && nt_dynamic_ok<EPI>()) a.queue = nt_queue_slot(st);
    // DSTACK_AMD_GEMM_NT_SPLIT=0: keep the last round's tiles whole
    static const bool split_env = [] {
      const char* v = getenv("DSTACK_AMD_GEMM_NT_SPLIT");
      return !(v && atoi(v) == 0);
    }();
    const int per_xcd = (tiles + 7) / 8, rx = per_xcd % a.wg_per_xcd;
    if (split_env && !a.queue && !TRACE && nt_split_ok<EPI>() && rx > 0 && 2 * rx <= a.wg_per_xcd &&
        (a.K / NT_BK) % 4 == 0)
      if (!nt_split_slot(st, 8 * (a.wg_per_xcd / 2), &a.split_ws, &a.split_cnt)) a.split_ws = nullptr;
  }
  if (const char* g = getenv("DSTACK_AMD_GEMM_NT_GROUP")) a.group = atoi(g) > 0 ? atoi(g) : a.group;
  gemm_nt_kernel<EPI, TRACE, KM, F8><<<grid, 512, NT_LDS, st>>>(a);
  return hipGetLastError();
}

}  // namespace

extern "C" bool dsa_gemm_nt_supported(int M, int N, int K) { return nt_shape_ok(M, N, K); }

// -1: the environment's default grid form, 0: one workgroup per tile, 1: persistent (see g_nt_grid)
extern "C" void dsa_gemm_nt_set_grid(int mode) { g_nt_grid.store(mode < 0 ? -1 : (mode ? 1 : 0)); }

// C[M][N] (+)= A[M][K] B[N][K]^T.  Leading dimensions in elements, multiples of 8 (16-byte rows);
// every operand must be < 4 GiB from its tile origin (32-bit DMA offsets).
extern "C" hipError_t dsa_gemm_nt(const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb,
                                  long ldc, int accumulate, hipStream_t st) {
  if (!nt_shape_ok(M, N, K) || lda % 8 || ldb % 8 || ldc % 4 || lda < K || ldb < K || ldc < N)
    return hipErrorInvalidValue;
  if (255L * lda * 2 + 2L * K > 0xffffffffL || 255L * ldb * 2 + 2L * K > 0xffffffffL) return hipErrorInvalidValue;
  NTArgs a{};
  a.A = (const bf16_t*)A;
  a.B = (const bf16_t*)B;
  a.C = (bf16_t*)C;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  a.M = M;
  a.K = K;
  a.ntn = N / NT_BN;
  a.nstride = NT_BN;
  a.bsplit = 128;
  a.group = nt_group(M / NT_BM, N / NT_BN);
  const int tiles = (M / NT_BM) * (N / NT_BN);
  if (accumulate == 2) return nt_launch<EPI_NONE>(a, tiles, st);  // timing-only diagnostic
  return accumulate ? nt_launch<EPI_ACC>(a, tiles, st) : nt_launch<EPI_STORE>(a, tiles, st);
}

// C[M][N] = bf16(A[M][K] B[N][K]^T) for e4m3 A and B (row strides lda / ldb in bytes, K in
// bytes): the raw product, no scales (the serving engine applies the row-wise scales in the
// consumer kernels, serving/model.py).  Same tiles and schedule as the bf16 GEMM.
extern "C" bool dsa_gemm_nt_f8_supported(int M, int N, int K) { return K % 2 == 0 && nt_shape_ok(M, N, K / 2); }

extern "C" hipError_t dsa_gemm_nt_f8(const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb,
                                     long ldc, hipStream_t st) {
  if (!dsa_gemm_nt_f8_supported(M, N, K) || lda % 16 || ldb % 16 || ldc % 8 || lda < K || ldb < K || ldc < N)
    return hipErrorInvalidValue;
  if (255L * lda + K > 0xffffffffL || 255L * ldb + K > 0xffffffffL) return hipErrorInvalidValue;
  NTArgs a{};
  a.A = (const bf16_t*)A;
  a.B = (const bf16_t*)B;
  a.C = (bf16_t*)C;
  a.lda = lda / 2;
  a.ldb = ldb / 2;
  a.ldc = ldc;
  a.M = M;
  a.K = K / 2;
  a.ntn = N / NT_BN;
  a.nstride = NT_BN;
  a.bsplit = 128;
  a.group = nt_group(M / NT_BM, N / NT_BN);
  return nt_launch<EPI_STORE, false, false, true>(a, (M / NT_BM) * (N / NT_BN), st);
}

// Serving fp8 gate/up with the SwiGLU in the epilogue: X [M][K] e4m3 (ldx bytes), W [2F][K] e4m3
// (gate rows, then up rows; ldw bytes), rs [M] / cs [2F] the row-wise scales; writes a [M][F] bf16
// and pmax [M][F / 32] (per-row partial max |a|, for quant_rows_pmax).
extern "C" bool dsa_gemm_nt_f8_swiglu_supported(int M, int F, int K) {
  return M > 0 && F > 0 && M % NT_BM == 0 && F % 128 == 0 && K % (4 * NT_BK) == 0;
}

extern "C" hipError_t dsa_gemm_nt_f8_swiglu(const void* X, const void* W, void* a_out, float* pmax, const float* rs,
                                            const float* cs, int M, int F, int K, long ldx, long ldw,
                                            hipStream_t st) {
  if (!dsa_gemm_nt_f8_swiglu_supported(M, F, K) || ldx % 16 || ldw % 16 || ldx < K || ldw < K)
    return hipErrorInvalidValue;
  if (255L * ldx + K > 0xffffffffL || 255L * ldw + K > 0xffffffffL) return hipErrorInvalidValue;
  NTArgs a{};
  a.A = (const bf16_t*)X;
  a.B = (const bf16_t*)W;
  a.C2 = (bf16_t*)a_out;
  a.srow = rs;
  a.scol = cs;
  a.pmax = pmax;
  a.lda = ldx / 2;
  a.ldb = ldw / 2;
  a.M = M;
  a.K = K / 2;
  a.F = F;
  a.ntn = F / 128;
  a.nstride = 128;
  a.bsplit = F;
  a.group = nt_group(M / NT_BM, F / 128);
  return nt_launch<EPI_SWIGLU_F8, false, false, true>(a, (M / NT_BM) * (F / 128), st);
}

// qkv = A[M][K] B[N][K]^T with RoPE on the columns [0, rot_cols) (head_dim 128, rotate-half, fp32
// tables cos / sin [>= S][64]), rounded once to bf16.  Row m is position m % S.
extern "C" bool dsa_gemm_nt_rope_supported(int M, int N, int K, int S, int rot_cols) {
  return nt_shape_ok(M, N, K) && S > 0 && S % NT_BM == 0 && M % S == 0 && rot_cols % 128 == 0 &&
         rot_cols <= N;
}

extern "C" hipError_t dsa_gemm_nt_rope(const void* A, const void* B, void* C, const float* cosT, const float* sinT,
                                       int M, int N, int K, long lda, long ldb, long ldc, int S, int rot_cols,
                                       hipStream_t st) {
  if (!dsa_gemm_nt_rope_supported(M, N, K, S, rot_cols) || lda % 8 || ldb % 8 || ldc % 8 || lda < K || ldb < K ||
      ldc < N)
    return hipErrorInvalidValue;
  if (255L * lda * 2 + 2L * K > 0xffffffffL || 255L * ldb * 2 + 2L * K > 0xffffffffL) return hipErrorInvalidValue;
  NTArgs a{};
  a.A = (const bf16_t*)A;
  a.B = (const bf16_t*)B;
  a.C = (bf16_t*)C;
  a.rcos = cosT;
  a.rsin = sinT;
  a.rS = S;
  a.rcols = rot_cols;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  a.M = M;
  a.K = K;
  a.ntn = N / NT_BN;
  a.nstride = NT_BN;
  a.bsplit = 64;  // b1 = dims 64-127 of the tile's two heads
  a.group = nt_group(M / NT_BM, N / NT_BN);
  return nt_launch<EPI_ROPE>(a, (M / NT_BM) * (N / NT_BN), st);
}

// Diagnostic: one plain GEMM with waves 0 and 4 of workgroup 0 stamping every phase boundary of
// K-iterations 8..11 (s_memtime, 4 per phase) into trace[2][64] (tools/diag/gemm_nt_phases.py).
extern "C" hipError_t dsa_gemm_nt_trace(const void* A, const void* B, void* C, int M, int N, int K,
                                        unsigned long long* trace, hipStream_t st) {
  if (!nt_shape_ok(M, N, K) || K < 24 * NT_BK) return hipErrorInvalidValue;
  NTArgs a{};
  a.A = (const bf16_t*)A;
  a.B = (const bf16_t*)B;
  a.C = (bf16_t*)C;
  a.lda = K;
  a.ldb = K;
  a.ldc = N;
  a.M = M;
  a.K = K;
  a.ntn = N / NT_BN;
  a.nstride = NT_BN;
  a.bsplit = 128;
  a.group = nt_group(M / NT_BM, N / NT_BN);
  a.trace = trace;
  return nt_launch<EPI_STORE, true>(a, (M / NT_BM) * (N / NT_BN), st);
}

extern "C" bool dsa_gemm_nt_swiglu_supported(int T, int F, int K) {
  return T % NT_BM == 0 && F % 128 == 0 && K % (2 * NT_BK) == 0 && F > 0 && T > 0;
}

// gu[T][2F] = X[T][K] Wgu[2F][K]^T (gate rows 0..F-1, up rows F..2F-1), a = silu(g) * u [T][F] and
// a^T [F][T] from the same tile.
extern "C" hipError_t dsa_gemm_nt_swiglu(const void* X, const void* W, void* gu, void* a_out, void* aT, int T, int F,
                                         int K, long ldx, long ldw, hipStream_t st) {
  if (!dsa_gemm_nt_swiglu_supported(T, F, K) || ldx % 8 || ldw % 8 || ldx < K || ldw < K) return hipErrorInvalidValue;
  NTArgs a{};
  a.A = (const bf16_t*)X;
  a.B = (const bf16_t*)W;
  a.C = (bf16_t*)gu;
  a.C2 = (bf16_t*)a_out;
  a.C3 = (bf16_t*)aT;  // null: no a^T (EPI_SWIGLU_R)
  a.lda = ldx;
  a.ldb = ldw;
  a.ldc = 2L * F;
  a.M = T;
  a.K = K;
  a.F = F;
  a.ntn = F / 128;
  a.nstride = 128;
  a.bsplit = F;
  a.group = nt_group(T / NT_BM, F / 128);
  if (!aT) return nt_launch<EPI_SWIGLU_R>(a, (T / NT_BM) * (F / 128), st);
  return nt_launch<EPI_SWIGLU>(a, (T / NT_BM) * (F / 128), st);
}

extern "C" bool dsa_gemm_nt_swiglu_bwd_supported(int T, int F, int K) {
  return T % NT_BM == 0 && F % NT_BN == 0 && K % (2 * NT_BK) == 0 && F > 0 && T > 0;
}

// da = dY[T][K] WdT[F][K]^T (WdT = W_down^T), fused with the SwiGLU backward against gu [T][2F]:
// dgu [T][2F] and dgu^T [2F][T].
extern "C" hipError_t dsa_gemm_nt_swiglu_bwd(const void* dY, const void* WdT, const void* gu, void* dgu, void* dguT,
                                             int T, int F, int K, long ldy, long ldw, hipStream_t st) {
  if (!dsa_gemm_nt_swiglu_bwd_supported(T, F, K) || ldy % 8 || ldw % 8 || ldy < K || ldw < K)
    return hipErrorInvalidValue;
  NTArgs a{};
  a.A = (const bf16_t*)dY;
  a.B = (const bf16_t*)WdT;
  a.C = (bf16_t*)dgu;
  a.C3 = (bf16_t*)dguT;
  a.G = (const bf16_t*)gu;
  a.lda = ldy;
  a.ldb = ldw;
  a.ldc = 2L * F;
  a.M = T;
  a.K = K;
  a.F = F;
  a.ntn = F / NT_BN;
  a.nstride = NT_BN;
  a.bsplit = 128;
  a.group = nt_group(T / NT_BM, F / NT_BN);
  if (!dguT) return nt_launch<EPI_SWIGLU_BWD_R>(a, (T / NT_BM) * (F / NT_BN), st);
  return nt_launch<EPI_SWIGLU_BWD>(a, (T / NT_BM) * (F / NT_BN), st);
}

extern "C" bool dsa_gemm_km_supported(int M, int N, int K) { return nt_shape_ok(M, N, K); }

// KM form with an fp32 gradient accumulator (weight gradients summed over micro-batches in fp32):
// mode 0: C32 = A^T B (first micro-batch), 1: C32 += A^T B, 2: C (bf16) = bf16(C32 + A^T B) (last
// micro-batch: one rounding).  C32 [M][ldc32] fp32, C [M][ldc] bf16 (mode 2 only).
extern "C" hipError_t dsa_gemm_km_f32(const void* A, const void* B, void* C, float* C32, int M, int N, int K, long lda,
                                      long ldb, long ldc, long ldc32, int mode, hipStream_t st) {
  if (!nt_shape_ok(M, N, K) || lda % 8 || ldb % 8 || ldc32 % 4 || lda < M || ldb < N || ldc32 < N || mode < 0 ||
      mode > 2 || (mode == 2 && (!C || ldc % 8 || ldc < N)))
    return hipErrorInvalidValue;
  if (63L * lda * 2 + 512 > 0xffffffffL || 63L * ldb * 2 + 512 > 0xffffffffL) return hipErrorInvalidValue;
  NTArgs a{};
  a.A = (const bf16_t*)A;
  a.B = (const bf16_t*)B;
  a.lda = lda;
  a.ldb = ldb;
  a.M = M;
  a.K = K;
  a.ntn = N / NT_BN;
  a.nstride = NT_BN;
  a.bsplit = 128;
  a.group = nt_group(M / NT_BM, N / NT_BN);
  const int tiles = (M / NT_BM) * (N / NT_BN);
  if (mode == 2) {
    a.C = (bf16_t*)C;
    a.ldc = ldc;
    a.F32 = C32;
    a.ldc32 = ldc32;
    return nt_launch<EPI_ACC32_BF16, false, true>(a, tiles, st);
  }
  a.C = reinterpret_cast<bf16_t*>(C32);
  a.ldc = ldc32;
  return mode ? nt_launch<EPI_ACC32, false, true>(a, tiles, st) : nt_launch<EPI_STORE32, false, true>(a, tiles, st);
}

// KM form: C[M][N] (+)= A[K][M]^T B[K][N] (weight gradient dW = dY^T X of token-major dY, X).
// Leading dimensions (row strides of A, B, C) in elements, multiples of 8.
extern "C" hipError_t dsa_gemm_km(const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb,
                                  long ldc, int accumulate, hipStream_t st) {
  if (!nt_shape_ok(M, N, K) || lda % 8 || ldb % 8 || ldc % 4 || lda < M || ldb < N || ldc < N)
    return hipErrorInvalidValue;
  if (63L * lda * 2 + 512 > 0xffffffffL || 63L * ldb * 2 + 512 > 0xffffffffL) return hipErrorInvalidValue;
  NTArgs a{};
  a.A = (const bf16_t*)A;
  a.B = (const bf16_t*)B;
  a.C = (bf16_t*)C;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  a.M = M;
  a.K = K;
  a.ntn = N / NT_BN;
  a.nstride = NT_BN;
  a.bsplit = 128;
  a.group = nt_group(M / NT_BM, N / NT_BN);
  const int tiles = (M / NT_BM) * (N / NT_BN);
  if (accumulate == 2) return nt_launch<EPI_NONE, false, true>(a, tiles, st);
  return accumulate ? nt_launch<EPI_ACC, false, true>(a, tiles, st) : nt_launch<EPI_STORE, false, true>(a, tiles, st);
}
