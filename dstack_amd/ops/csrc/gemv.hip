// Small-batch decode projections for CDNA4 (gfx950): y[m][n] = sum_k x[m][k] * W[n][k] for M <= 4
// rows (batch-1..4 decode: every weight byte is read once per token, so the op is a pure HBM
// stream of W).  hipBLASLt's solutions at M = 1 stream Llama-3-70B's weights at ~4 TB/s
// (34.8 ms/token, profiles/serve_70b_latency32k_r2n.log); this is the guide's "GEMV / M <= 16
// decode weights" form: W straight to VGPRs with 16-byte loads, U loads per lane in flight, no
// LDS round trip, late waits.
//
// Layout: W [N][K] row-major (the nn.Linear weight, K contiguous), x [M][ldx], y [M][ldy], bf16;
// fp32 accumulation.  One wave per output row (4 rows per 256-thread workgroup): lane l covers
// columns 8l .. 8l+7 of every 512-column step; x is re-read per row from L1/L2 (M x 16 KB at K =
// 8192 is cache resident).  Rows are dealt so that each XCD streams a contiguous band of W.
#include "common.h"

using namespace dsa;

namespace {

template <int M, int U>
__global__ __launch_bounds__(256) void gemv_kernel(const bf16_t* __restrict__ x, long ldx, const bf16_t* __restrict__ W,
                                                   bf16_t* __restrict__ y, long ldy, int N, int K) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // XCD-aware row band: workgroup b runs on XCD b % 8; give each XCD a contiguous range of rows
  const int nwg = gridDim.x, b = blockIdx.x;
  const int per = nwg >> 3, rem = nwg & 7, xcd = b & 7, idx = b >> 3;
  const int wg = (nwg >= 8) ? xcd * per + (xcd < rem ? xcd : rem) + idx : b;
  const int row = wg * 4 + wave;
  if (row >= N) return;  // wave-uniform
  const bf16_t* wr = W + (long)row * K;
  float acc[M];
#pragma unroll
  for (int m = 0; m < M; ++m) acc[m] = 0.f;
  const int step = 512 * U;
  int k0 = lane * 8;
  for (; k0 + 512 * (U - 1) < K; k0 += step) {
    us8 wv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) wv[u] = __builtin_nontemporal_load(reinterpret_cast<const us8*>(wr + k0 + 512 * u));
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float w8[8];
      unpack8(wv[u], w8);
#pragma unroll
      for (int m = 0; m < M; ++m) {
        float x8[8];
        unpack8(*reinterpret_cast<const us8*>(x + m * ldx + k0 + 512 * u), x8);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[m] = fmaf(w8[i], x8[i], acc[m]);
      }
    }
  }
  for (; k0 < K; k0 += 512) {  // K % (512 U) tail, one 512-column step at a time
    float w8[8];
    unpack8(*reinterpret_cast<const us8*>(wr + k0), w8);
#pragma unroll
    for (int m = 0; m < M; ++m) {
      float x8[8];
      unpack8(*reinterpret_cast<const us8*>(x + m * ldx + k0), x8);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[m] = fmaf(w8[i], x8[i], acc[m]);
    }
  }
#pragma unroll
  for (int m = 0; m < M; ++m) acc[m] = wave_sum(acc[m]);
  if (lane < M) {
    float v = acc[0];
#pragma unroll
    for (int m = 1; m < M; ++m)
      if (lane == m) v = acc[m];
    y[lane * ldy + row] = f2bf(v);
  }
}

}  // namespace

extern "C" bool dsa_gemv_supported(int M, int K) { return M >= 1 && M <= 4 && K % 512 == 0 && K > 0; }

extern "C" hipError_t dsa_gemv(const void* x, long ldx, const void* W, void* y, long ldy, int M, int N, int K,
                               hipStream_t st) {
  if (!dsa_gemv_supported(M, K) || N <= 0) return hipErrorInvalidValue;
  const int grid = (N + 3) / 4;
#define DSA_GEMV(MM)                                                                                  \
  gemv_kernel<MM, 4><<<grid, 256, 0, st>>>((const bf16_t*)x, ldx, (const bf16_t*)W, (bf16_t*)y, ldy, N, K)
  switch (M) {
    case 1: DSA_GEMV(1); break;
    case 2: DSA_GEMV(2); break;
    case 3: DSA_GEMV(3); break;
    default: DSA_GEMV(4); break;
  }
#undef DSA_GEMV
  return hipGetLastError();
}
