// MFMA / LDS tile helpers shared by the CDNA4 (gfx950) matrix kernels (flash_attn.hip, gemm.hip).
//
// Tiles are [rows][128] bf16 images in LDS (256-byte rows) with a 16-byte-chunk XOR swizzle
//   ch ^ (((row&3)<<2) | ((row>>2)&3))
// that is conflict-free both for ds_read_b128 row reads (operands whose reduction index is
// contiguous) and for ds_read_b64_tr_b16 transposed reads (operands whose reduction index is the
// row).  Tiles are filled by LDS-DMA (global_load_lds, 16 B/lane) with the swizzle applied to the
// per-lane source address, so no staging VGPRs are used.
#pragma once
#include "common.h"

namespace dsa {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define LDS3(T, p) ((__attribute__((address_space(3))) T*)(p))
#define GLB1(T, p) ((__attribute__((address_space(1))) T*)(p))


constexpr int TILE_BYTES = 64 * 256;  // 64 rows x 128 bf16

__device__ __forceinline__ int swz(int row, int ch) {
  return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

// v_exp_f32 directly: exp2f() adds a denormal range-reduction (cmp/cndmask/add/ldexp) around it;
// softmax probabilities below 2^-126 are irrelevant, so the bare instruction is exact enough
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ f32x16 mfma(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 lds_row(const char* base, int row, int ch) {
  return *reinterpret_cast<const bf16x8*>(base + swz(row, ch));
}

// A-operand fragment of X^T where X is a [rows][128] tile in LDS read by columns:
// element j of lane-half h = X[16*ks + 8*(j>>2) + 4*h + (j&3)][col0 + (lane&31)]  (the k order of
// an MFMA accumulator used as the other operand).  Two ds_read_b64_tr_b16 per fragment.
__device__ __forceinline__ bf16x8 lds_tr(const char* base, int row_base, int col0, int lane) {
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int r0 = row_base + 4 * (g >> 1) + q4;
  const int c0 = (col0 >> 3) + 2 * (g & 1) + (p4 >> 1);
  const int sub = 8 * (p4 & 1);
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS3(bf16x4, base + swz(r0, c0) + sub));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS3(bf16x4, base + swz(r0 + 8, c0) + sub));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// Issue LDS-DMA of a [64 x 128] bf16 tile (rows row0.., row stride `stride` elements) into the
// swizzled LDS image at `lds`.  4 waves x 4 wave-instructions of 1 KiB (4 rows each).
__device__ __forceinline__ void dma_tile64(const bf16_t* g, long stride, char* lds, int wave,
                                           int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = wave * 4 + i;
    const int row = piece * 4 + (lane >> 4);
    const int pc = lane & 15;
    const int ch = pc ^ (((row & 3) << 2) | ((row >> 2) & 3));
    const bf16_t* src = g + (long)row * stride + ch * 8;
    __builtin_amdgcn_global_load_lds(GLB1(void, src), LDS3(void, lds + piece * 1024), 16, 0, 0);
  }
}

// Same tile, issued by NW waves (16 / NW wave-instructions each).
template <int NW>
__device__ __forceinline__ void dma_tile64_n(const bf16_t* g, long stride, char* lds, int wave, int lane) {
  static_assert(16 % NW == 0, "16 pieces split over NW waves");
#pragma unroll
  for (int i = 0; i < 16 / NW; ++i) {
    const int piece = wave * (16 / NW) + i;
    const int row = piece * 4 + (lane >> 4);
    const int pc = lane & 15;
    const int ch = pc ^ (((row & 3) << 2) | ((row >> 2) & 3));
    const bf16_t* src = g + (long)row * stride + ch * 8;
    __builtin_amdgcn_global_load_lds(GLB1(void, src), LDS3(void, lds + piece * 1024), 16, 0, 0);
  }
}

// Buffer descriptor over `bytes` of a wave-uniform base (readfirstlane'd so the compiler can prove
// uniformity and keeps it in SGPRs), for LDS-DMA whose per-iteration offset is an SGPR (soffset)
// and whose per-lane part is one 32-bit voffset: no 64-bit VGPR address pair stays live across a
// loop (under 256-VGPR pressure such a pair gets spilled, and its reload drains vmcnt).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(base);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  void* p = reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// The same tile through a buffer descriptor: the per-lane source offsets (32-bit, swizzle included)
// are computed once per kernel by dma_tile64_offsets, the tile's row offset is an SGPR byte offset.
// Besides dropping the per-tile 64-bit address arithmetic, this keeps LDS-read waits counted: the
// compiler's waitcnt pass counts a FLAT-encoded global_load_lds in lgkmcnt as well as vmcnt, so with
// one in flight every ds_read consumer gets lgkmcnt(0); a buffer load counts in vmcnt only.
template <int NW>
__device__ __forceinline__ void dma_tile64_offsets(long stride, int wave, int lane, unsigned (&off)[16 / NW]) {
#pragma unroll
  for (int i = 0; i < 16 / NW; ++i) {
    const int row = (wave * (16 / NW) + i) * 4 + (lane >> 4);
    const int ch = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
    off[i] = (unsigned)(((long)row * stride + ch * 8) * 2);
  }
}

template <int NW>
__device__ __forceinline__ void dma_tile64_buf(__amdgpu_buffer_rsrc_t r, const unsigned* off, int soff,
                                               char* lds, int wave) {
  const int so = __builtin_amdgcn_readfirstlane(soff);
#pragma unroll
  for (int i = 0; i < 16 / NW; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, LDS3(void, lds + (wave * (16 / NW) + i) * 1024), 16, off[i], so, 0,
                                             0);
}

// 64 contiguous floats -> LDS (one wave-instruction, 4 B/lane)
__device__ __forceinline__ void dma_f32x64(const float* g, char* lds, int lane) {
  __builtin_amdgcn_global_load_lds(GLB1(void, g + lane), LDS3(void, lds), 4, 0, 0);
}

// 64 contiguous floats at element `elem0` of the buffer -> LDS (one wave-instruction, 4 B/lane)
__device__ __forceinline__ void dma_f32x64_buf(__amdgpu_buffer_rsrc_t r, int elem0, char* lds, int lane) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, LDS3(void, lds), 4, lane * 4, elem0 * 4, 0, 0);
}

__device__ __forceinline__ void wait_dma_and_barrier() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

__device__ __forceinline__ bf16x8 to_bf16x8(const f32x16& acc, int base) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = static_cast<__bf16>(acc[base + j]);
  return r;
}


}  // namespace dsa
