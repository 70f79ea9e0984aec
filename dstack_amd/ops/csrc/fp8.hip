// FP8 (OCP e4m3, the gfx950 v_cvt_pk_fp8_f32 / v_cvt_pk_f32_fp8 format) serving kernels.
//
// Weight-only bytes dominate a decode step (a 70B model streams 140 GB of bf16 weights per step):
// e4m3 weights with one fp32 scale per output row halve that and let hipBLASLt run the larger
// batches on the fp8 MFMA rate.  Two kernels:
//  * quant_rows: x [M][K] bf16 -> q [M][K] e4m3 + s [M] fp32 with s = max|x_row| / 448 (dynamic
//    per-token activation scales; also used once per weight at load time, per output row).
//  * gemv_fp8: y[m][n] = s_w[n] * sum_k x[m][k] * q[n][k] for M <= 4 rows — the batch-1 decode
//    weight stream at half the bytes of csrc/gemv.hip.  One wave per 1, 2 or 4 output rows (the
//    x slice loaded once per step serves all of them), 16 weights (16 B) per lane per load,
//    XCD-banded rows, fp32 accumulation.
#include "common.h"

#include <cstdlib>

using namespace dsa;

namespace {

typedef unsigned int u4 __attribute__((ext_vector_type(4)));
constexpr float E4M3_MAX = 448.f;

// 4 fp8 (one dword) -> 4 floats
__device__ __forceinline__ void fp8x4_to_f32(unsigned int v, float* o) {
  auto lo = __builtin_amdgcn_cvt_pk_f32_fp8(v, false);  // bytes 0, 1
  auto hi = __builtin_amdgcn_cvt_pk_f32_fp8(v, true);   // bytes 2, 3
  o[0] = lo[0];
  o[1] = lo[1];
  o[2] = hi[0];
  o[3] = hi[1];
}

// 4 floats (already scaled into range) -> one dword of fp8, saturating at +-448
__device__ __forceinline__ unsigned int f32x4_to_fp8(float a, float b, float c, float d) {
  a = __builtin_amdgcn_fmed3f(a, E4M3_MAX, -E4M3_MAX);
  b = __builtin_amdgcn_fmed3f(b, E4M3_MAX, -E4M3_MAX);
  c = __builtin_amdgcn_fmed3f(c, E4M3_MAX, -E4M3_MAX);
  d = __builtin_amdgcn_fmed3f(d, E4M3_MAX, -E4M3_MAX);
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (unsigned int)w;
}

// one 256-thread workgroup per row; K % 8 == 0
// NIT > 0: the row stays in registers between the absmax and quantization passes (x read once),
// K <= 2048 * NIT; NIT = 0: two passes over x (any K)
template <int NIT = 0>
__global__ __launch_bounds__(256) void quant_rows_kernel(const bf16_t* __restrict__ x, long ldx,
                                                         unsigned char* __restrict__ q, long ldq,
                                                         float* __restrict__ s, int K) {
  __shared__ float red[4];
  const int row = blockIdx.x, tid = threadIdx.x;
  const bf16_t* xr = x + (long)row * ldx;
  float amax = 0.f;
  us8 pk[NIT > 0 ? NIT : 1];
  if constexpr (NIT > 0) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int k = (tid + it * 256) * 8;
      if (k < K) {
        pk[it] = *reinterpret_cast<const us8*>(xr + k);
        float v[8];
        unpack8(pk[it], v);
#pragma unroll
        for (int i = 0; i < 8; ++i) amax = fmaxf(amax, fabsf(v[i]));
      }
    }
  } else {
    for (int k = tid * 8; k < K; k += 256 * 8) {
      float v[8];
      unpack8(*reinterpret_cast<const us8*>(xr + k), v);
#pragma unroll
      for (int i = 0; i < 8; ++i) amax = fmaxf(amax, fabsf(v[i]));
    }
  }
  amax = wave_max(amax);
  if ((tid & 63) == 0) red[tid >> 6] = amax;
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float scale = fmaxf(amax, 1e-12f) / E4M3_MAX;
  const float inv = 1.f / scale;
  if (tid == 0) s[row] = scale;
  unsigned char* qr = q + (long)row * ldq;
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
  if constexpr (NIT > 0) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int k = (tid + it * 256) * 8;
      if (k < K) {
        float v[8];
        unpack8(pk[it], v);
        const unsigned int w0 = f32x4_to_fp8(v[0] * inv, v[1] * inv, v[2] * inv, v[3] * inv);
        const unsigned int w1 = f32x4_to_fp8(v[4] * inv, v[5] * inv, v[6] * inv, v[7] * inv);
        *reinterpret_cast<u2*>(qr + k) = u2{w0, w1};
      }
    }
  } else {
    for (int k = tid * 8; k < K; k += 256 * 8) {
      float v[8];
      unpack8(*reinterpret_cast<const us8*>(xr + k), v);
      const unsigned int w0 = f32x4_to_fp8(v[0] * inv, v[1] * inv, v[2] * inv, v[3] * inv);
      const unsigned int w1 = f32x4_to_fp8(v[4] * inv, v[5] * inv, v[6] * inv, v[7] * inv);
      *reinterpret_cast<u2*>(qr + k) = u2{w0, w1};
    }
  }
}

// SwiGLU + per-row quantization for the fp8 down projection of a decode step: gu [M][2F] bf16
// (gate | up) -> q [M][F] e4m3 + s [M], q * s ~= bf16(silu(g) * u) -- the separate swiglu_fwd and
// quant_rows kernels wrote and re-read the bf16 product.  One workgroup per row: pass 1 takes the
// row max of the bf16-rounded product, pass 2 writes e4m3 from the products it kept in registers
// (F up to 32768; wider rows recompute them from gu).
__device__ __forceinline__ float silu_q(float g) { return g / (1.f + __expf(-g)); }

// SCALED: gu is the raw e4m3 x e4m3 product of a tensor-wise-scaled fp8 GEMM (hipBLASLt runs the
// Llama-3-70B prefill shapes 12-25 % faster with scalar scales than with row-wise ones,
// profiles/fp8_scaling_modes_r8z.txt); the per-token scale rs[row] and the per-output-channel scale
// cs[c] of the row-wise form are applied here, on the fp32 values, before the SwiGLU.
// NIT > 0: the row's products stay in registers (packed bf16, exact: they are bf16-rounded) between
// the absmax pass and the quantization pass, so gu (and cs) are read once instead of twice; NIT is
// the number of 2048-column steps, F <= 2048 * NIT.  NIT = 0: two passes over gu (any F).
// BS: threads per row (256, or 1024 for decode-sized M: one workgroup per row leaves a 256-row batch
// with 4 waves per CU, too few loads in flight to stream the row at HBM rate)
template <bool SCALED, int NIT = 0, int BS = 256>
__global__ __launch_bounds__(BS) void swiglu_quant_rows_kernel(const bf16_t* __restrict__ gu, long ldg,
                                                                unsigned char* __restrict__ q, long ldq,
                                                                float* __restrict__ s, int F,
                                                                const float* __restrict__ rs,
                                                                const float* __restrict__ cs) {
  __shared__ float red[BS / 64];
  const int row = blockIdx.x, tid = threadIdx.x;
  const bf16_t* gr = gu + (long)row * ldg;
  const float r = SCALED ? rs[row] : 1.f;
  auto prod8 = [&](int k, float* a) {
    float g[8], u[8];
    unpack8(*reinterpret_cast<const us8*>(gr + k), g);
    unpack8(*reinterpret_cast<const us8*>(gr + F + k), u);
    if constexpr (SCALED) {
      const f4 cg0 = *reinterpret_cast<const f4*>(cs + k), cg1 = *reinterpret_cast<const f4*>(cs + k + 4);
      const f4 cu0 = *reinterpret_cast<const f4*>(cs + F + k), cu1 = *reinterpret_cast<const f4*>(cs + F + k + 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        g[i] = bf2f(f2bf(g[i] * r * cg0[i]));
        g[4 + i] = bf2f(f2bf(g[4 + i] * r * cg1[i]));
        u[i] = bf2f(f2bf(u[i] * r * cu0[i]));
        u[4 + i] = bf2f(f2bf(u[4 + i] * r * cu1[i]));
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = bf2f(f2bf(silu_q(g[i]) * u[i]));
  };
  float amax = 0.f;
  us8 pk[NIT > 0 ? NIT : 1];
  if constexpr (NIT > 0) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int k = (tid + it * BS) * 8;
      if (k < F) {
        float a[8];
        prod8(k, a);
#pragma unroll
        for (int i = 0; i < 8; ++i) amax = fmaxf(amax, fabsf(a[i]));
        pk[it] = pack8(a);
      }
    }
  } else {
    for (int k = tid * 8; k < F; k += BS * 8) {
      float a[8];
      prod8(k, a);
#pragma unroll
      for (int i = 0; i < 8; ++i) amax = fmaxf(amax, fabsf(a[i]));
    }
  }
  amax = wave_max(amax);
  if ((tid & 63) == 0) red[tid >> 6] = amax;
  __syncthreads();
  amax = red[0];
#pragma unroll
  for (int i = 1; i < BS / 64; ++i) amax = fmaxf(amax, red[i]);
  const float scale = fmaxf(amax, 1e-12f) / E4M3_MAX;
  const float inv = 1.f / scale;
  if (tid == 0) s[row] = scale;
  unsigned char* qr = q + (long)row * ldq;
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
  if constexpr (NIT > 0) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int k = (tid + it * BS) * 8;
      if (k < F) {
        float a[8];
        unpack8(pk[it], a);
        const unsigned int w0 = f32x4_to_fp8(a[0] * inv, a[1] * inv, a[2] * inv, a[3] * inv);
        const unsigned int w1 = f32x4_to_fp8(a[4] * inv, a[5] * inv, a[6] * inv, a[7] * inv);
        *reinterpret_cast<u2*>(qr + k) = u2{w0, w1};
      }
    }
  } else {
    for (int k = tid * 8; k < F; k += BS * 8) {
      float a[8];
      prod8(k, a);
      const unsigned int w0 = f32x4_to_fp8(a[0] * inv, a[1] * inv, a[2] * inv, a[3] * inv);
      const unsigned int w1 = f32x4_to_fp8(a[4] * inv, a[5] * inv, a[6] * inv, a[7] * inv);
      *reinterpret_cast<u2*>(qr + k) = u2{w0, w1};
    }
  }
}

template <int M, int U>
__global__ __launch_bounds__(256) void gemv_fp8_kernel(const bf16_t* __restrict__ x, long ldx,
                                                       const unsigned char* __restrict__ W,
                                                       const float* __restrict__ sw, bf16_t* __restrict__ y,
                                                       long ldy, int N, int K) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwg = gridDim.x, b = blockIdx.x;
  const int per = nwg >> 3, rem = nwg & 7, xcd = b & 7, idx = b >> 3;
  const int wg = (nwg >= 8) ? xcd * per + (xcd < rem ? xcd : rem) + idx : b;
  const int row = wg * 4 + wave;
  if (row >= N) return;  // wave-uniform
  const unsigned char* wr = W + (long)row * K;
  float acc[M];
#pragma unroll
  for (int m = 0; m < M; ++m) acc[m] = 0.f;
  // lane l covers columns 16 l .. 16 l + 15 of every 1024-column step
  for (int k0 = lane * 16; k0 < K; k0 += 1024 * U) {
    u4 wv[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (k0 + 1024 * u < K) wv[u] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(wr + k0 + 1024 * u));
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + 1024 * u;
      if (k >= K) break;
      float w16[16];
#pragma unroll
      for (int j = 0; j < 4; ++j) fp8x4_to_f32(wv[u][j], w16 + 4 * j);
#pragma unroll
      for (int m = 0; m < M; ++m) {
        float x8[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          unpack8(*reinterpret_cast<const us8*>(x + m * ldx + k + 8 * h), x8);
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[m] = fmaf(w16[8 * h + i], x8[i], acc[m]);
        }
      }
    }
  }
  const float scale = sw[row];
#pragma unroll
  for (int m = 0; m < M; ++m) acc[m] = wave_sum(acc[m]);
  if (lane < M) {
    float v = acc[0];
#pragma unroll
    for (int m = 1; m < M; ++m)
      if (lane == m) v = acc[m];
    y[lane * ldy + row] = f2bf(v * scale);
  }
}

// R output rows per wave: the x slice a lane loads (16 bf16 = 32 B) is reused for R rows of
// weights (R x 16 B), so a step issues 2 + R loads for 16 R weight bytes instead of 3 loads for
// 16 (the one-row form loads twice as many x bytes as weight bytes).
template <int M, int R, int U>
__global__ __launch_bounds__(256) void gemv_fp8_rows_kernel(const bf16_t* __restrict__ x, long ldx,
                                                            const unsigned char* __restrict__ W,
                                                            const float* __restrict__ sw, bf16_t* __restrict__ y,
                                                            long ldy, int N, int K) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwg = gridDim.x, b = blockIdx.x;
  const int per = nwg >> 3, rem = nwg & 7, xcd = b & 7, idx = b >> 3;
  const int wg = (nwg >= 8) ? xcd * per + (xcd < rem ? xcd : rem) + idx : b;
  const int row0 = (wg * 4 + wave) * R;
  if (row0 >= N) return;  // wave-uniform
  const int nr = min(R, N - row0);
  float acc[R][M];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < M; ++m) acc[r][m] = 0.f;
  for (int k0 = lane * 16; k0 < K; k0 += 1024 * U) {
    u4 wv[U][R];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (k0 + 1024 * u < K && r < nr)
          wv[u][r] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(W + (long)(row0 + r) * K + k0 + 1024 * u));
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + 1024 * u;
      if (k >= K) break;
      float xs[M][16];
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const us8 a = *reinterpret_cast<const us8*>(x + m * ldx + k);
        const us8 c = *reinterpret_cast<const us8*>(x + m * ldx + k + 8);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          xs[m][i] = bf2f(a[i]);
          xs[m][8 + i] = bf2f(c[i]);
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r >= nr) break;
        float w16[16];
#pragma unroll
        for (int j = 0; j < 4; ++j) fp8x4_to_f32(wv[u][r][j], w16 + 4 * j);
#pragma unroll
        for (int m = 0; m < M; ++m)
#pragma unroll
          for (int i = 0; i < 16; ++i) acc[r][m] = fmaf(w16[i], xs[m][i], acc[r][m]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (r >= nr) break;
    const float scale = sw[row0 + r];
#pragma unroll
    for (int m = 0; m < M; ++m) acc[r][m] = wave_sum(acc[r][m]);
    if (lane < M) {
      float v = acc[r][0];
#pragma unroll
      for (int m = 1; m < M; ++m)
        if (lane == m) v = acc[r][m];
      y[lane * ldy + row0 + r] = f2bf(v * scale);
    }
  }
}

}  // namespace

// Row quantizer whose row max comes precomputed as P partial maxima per row (pmax [M][P], written by
// the fp8 gate/up GEMM's SwiGLU epilogue): one pass over x instead of two (or a register-held row).
// Same scale and rounding as quant_rows_kernel.
__global__ __launch_bounds__(256) void quant_rows_pmax_kernel(const bf16_t* __restrict__ x, long ldx,
                                                              const float* __restrict__ pmax, int P,
                                                              unsigned char* __restrict__ q, long ldq,
                                                              float* __restrict__ s, int K) {
  __shared__ float red[4];
  const int row = blockIdx.x, tid = threadIdx.x;
  float amax = 0.f;
  for (int i = tid; i < P; i += 256) amax = fmaxf(amax, pmax[(long)row * P + i]);
  amax = wave_max(amax);
  if ((tid & 63) == 0) red[tid >> 6] = amax;
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float scale = fmaxf(amax, 1e-12f) / E4M3_MAX;
  const float inv = 1.f / scale;
  if (tid == 0) s[row] = scale;
  const bf16_t* xr = x + (long)row * ldx;
  unsigned char* qr = q + (long)row * ldq;
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
  for (int k = tid * 8; k < K; k += 256 * 8) {
    float v[8];
    unpack8(*reinterpret_cast<const us8*>(xr + k), v);
    const unsigned int w0 = f32x4_to_fp8(v[0] * inv, v[1] * inv, v[2] * inv, v[3] * inv);
    const unsigned int w1 = f32x4_to_fp8(v[4] * inv, v[5] * inv, v[6] * inv, v[7] * inv);
    *reinterpret_cast<u2*>(qr + k) = u2{w0, w1};
  }
}

extern "C" bool dsa_quant_fp8_supported(int K) { return K > 0 && K % 8 == 0; }

extern "C" hipError_t dsa_quant_fp8_rows_pmax(const void* x, long ldx, const float* pmax, int P, void* q, long ldq,
                                              float* s, int M, int K, hipStream_t st) {
  if (!dsa_quant_fp8_supported(K) || M <= 0 || P <= 0) return hipErrorInvalidValue;
  quant_rows_pmax_kernel<<<M, 256, 0, st>>>((const bf16_t*)x, ldx, pmax, P, (unsigned char*)q, ldq, s, K);
  return hipGetLastError();
}

extern "C" hipError_t dsa_quant_fp8_rows(const void* x, long ldx, void* q, long ldq, float* s, int M, int K,
                                         hipStream_t st) {
  if (!dsa_quant_fp8_supported(K) || M <= 0) return hipErrorInvalidValue;
  const int nit = (K + 2047) / 2048;
#define DSA_QR(N) quant_rows_kernel<N><<<M, 256, 0, st>>>((const bf16_t*)x, ldx, (unsigned char*)q, ldq, s, K)
  if (nit <= 2) DSA_QR(2);
  else if (nit <= 4) DSA_QR(4);
  else if (nit <= 8) DSA_QR(8);
  else if (nit <= 16) DSA_QR(16);
  else DSA_QR(0);
#undef DSA_QR
  return hipGetLastError();
}

extern "C" hipError_t dsa_swiglu_quant_fp8_rows(const void* gu, long ldg, void* q, long ldq, float* s, int M, int F,
                                                const float* rs, const float* cs, hipStream_t st) {
  if (F <= 0 || F % 8 || M <= 0 || ((rs == nullptr) != (cs == nullptr))) return hipErrorInvalidValue;
  // products held in registers for F <= 32768 (Llama-3-70B: F = 28672 -> 14 steps of 2048 columns);
  // decode-sized batches (M <= 512) run 1024 threads per row (4 steps of 8192 columns)
  const int nit = (F + 2047) / 2048, nit4 = (F + 8191) / 8192;
#define DSA_SWQ(SC, N, BS)                                                                        \
  swiglu_quant_rows_kernel<SC, N, BS><<<M, BS, 0, st>>>((const bf16_t*)gu, ldg, (unsigned char*)q, ldq, s, F, \
                                                        SC ? rs : nullptr, SC ? cs : nullptr)
#define DSA_SWQ_N(SC)                                  \
  if (M <= 512 && nit4 <= 2) DSA_SWQ(SC, 2, 1024);     \
  else if (M <= 512 && nit4 <= 4) DSA_SWQ(SC, 4, 1024); \
  else if (nit <= 2) DSA_SWQ(SC, 2, 256);              \
  else if (nit <= 4) DSA_SWQ(SC, 4, 256);              \
  else if (nit <= 8) DSA_SWQ(SC, 8, 256);              \
  else if (nit <= 16) DSA_SWQ(SC, 16, 256);            \
  else DSA_SWQ(SC, 0, 256);
  if (rs) {
    DSA_SWQ_N(true)
  } else {
    DSA_SWQ_N(false)
  }
#undef DSA_SWQ_N
#undef DSA_SWQ
  return hipGetLastError();
}

// y[r][c] = bf16(y[r][c] * rs[r] * cs[c]) in place: the row-wise scales of a tensor-wise-scaled fp8
// GEMM's raw product (see swiglu_quant_rows_kernel).  One workgroup per row, 8 columns per lane.
__global__ __launch_bounds__(256) void scale_rows_cols_kernel(bf16_t* __restrict__ y, long ldy, int N,
                                                              const float* __restrict__ rs,
                                                              const float* __restrict__ cs) {
  const int row = blockIdx.x;
  bf16_t* yr = y + (long)row * ldy;
  const float r = rs[row];
  for (int c = threadIdx.x * 8; c < N; c += 256 * 8) {
    float v[8];
    unpack8(*reinterpret_cast<const us8*>(yr + c), v);
    const f4 c0 = *reinterpret_cast<const f4*>(cs + c), c1 = *reinterpret_cast<const f4*>(cs + c + 4);
    us8 o;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[i] = f2bf(v[i] * r * c0[i]);
      o[4 + i] = f2bf(v[4 + i] * r * c1[i]);
    }
    *reinterpret_cast<us8*>(yr + c) = o;
  }
}

extern "C" hipError_t dsa_scale_rows_cols(void* y, long ldy, int M, int N, const float* rs, const float* cs,
                                          hipStream_t st) {
  if (M <= 0 || N <= 0 || N % 8) return hipErrorInvalidValue;
  scale_rows_cols_kernel<<<M, 256, 0, st>>>((bf16_t*)y, ldy, N, rs, cs);
  return hipGetLastError();
}

extern "C" bool dsa_gemv_fp8_supported(int M, int K) { return M >= 1 && M <= 4 && K % 1024 == 0 && K > 0; }

extern "C" hipError_t dsa_gemv_fp8(const void* x, long ldx, const void* W, const float* sw, void* y, long ldy,
                                   int M, int N, int K, hipStream_t st) {
  if (!dsa_gemv_fp8_supported(M, K) || N <= 0) return hipErrorInvalidValue;
  // rows per wave (x reuse): the most of 4 / 2 / 1 that still leaves >= 1024 workgroups (4 per CU).
  // Per Llama-3-70B layer at batch 1: 159 us with one row per wave, 143 us with 4 everywhere,
  // 142.5 us with this choice (profiles/bench_gemv_fp8_rows_r3f.txt).  DSTACK_AMD_GEMV_FP8_R forces 1 / 2 / 4.
  static const int forced = [] {
    const char* v = getenv("DSTACK_AMD_GEMV_FP8_R");
    return v ? atoi(v) : 0;
  }();
  int rows = forced;
  if (rows != 1 && rows != 2 && rows != 4) rows = N / 16 >= 1024 ? 4 : (N / 8 >= 1024 ? 2 : 1);
  if (rows == 4 || rows == 2) {
    const int R = rows, grid = (N + 4 * R - 1) / (4 * R);
#define DSA_GEMV8R(MM, RR)                                                                                   \
  gemv_fp8_rows_kernel<MM, RR, 2><<<grid, 256, 0, st>>>((const bf16_t*)x, ldx, (const unsigned char*)W, sw, \
                                                        (bf16_t*)y, ldy, N, K)
#define DSA_GEMV8R_M(RR)                \
  switch (M) {                          \
    case 1: DSA_GEMV8R(1, RR); break;   \
    case 2: DSA_GEMV8R(2, RR); break;   \
    case 3: DSA_GEMV8R(3, RR); break;   \
    default: DSA_GEMV8R(4, RR); break;  \
  }
    if (R == 4) {
      DSA_GEMV8R_M(4)
    } else {
      DSA_GEMV8R_M(2)
    }
#undef DSA_GEMV8R_M
#undef DSA_GEMV8R
    return hipGetLastError();
  }
  const int grid = (N + 3) / 4;
#define DSA_GEMV8(MM)                                                                                 \
  gemv_fp8_kernel<MM, 4><<<grid, 256, 0, st>>>((const bf16_t*)x, ldx, (const unsigned char*)W, sw,   \
                                               (bf16_t*)y, ldy, N, K)
  switch (M) {
    case 1: DSA_GEMV8(1); break;
    case 2: DSA_GEMV8(2); break;
    case 3: DSA_GEMV8(3); break;
    default: DSA_GEMV8(4); break;
  }
#undef DSA_GEMV8
  return hipGetLastError();
}
