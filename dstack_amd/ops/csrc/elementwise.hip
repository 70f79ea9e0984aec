// Memory-bound fused ops for the Llama training step on MI355X (gfx950).
//
// Every kernel moves bf16 as 16-byte vectors (8 x bf16 per lane, one dwordx4 per lane per access,
// 1 KiB per wave-instruction) and reduces rows inside ONE 64-lane wave with __shfl_xor, so no LDS
// and no __syncthreads sit on the critical path. Grids are sized to keep >=4 waves per SIMD
// resident across all 256 CUs.
#include "mfma_tiles.h"

using namespace dsa;

// ------------------------------------------------------------------------------------------------
// RMSNorm forward (optionally fused with the residual add h = x + delta).
// One wave per row; the row stays in registers between the reduction and the normalisation.
// ------------------------------------------------------------------------------------------------
template <int NCH, bool ADD>
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(const bf16_t* __restrict__ x,
                                                          const bf16_t* __restrict__ delta,
                                                          const bf16_t* __restrict__ w,
                                                          bf16_t* __restrict__ h_out,
                                                          bf16_t* __restrict__ y,
                                                          float* __restrict__ rstd_out, int rows,
                                                          int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nch = D >> 3;
  const size_t base = (size_t)row * D;
  float v[NCH][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      us8 a = *reinterpret_cast<const us8*>(x + base + ch * 8);
      unpack8(a, v[c]);
      if constexpr (ADD) {
        float d[8];
        unpack8(*reinterpret_cast<const us8*>(delta + base + ch * 8), d);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[c][i] = bf2f(f2bf(v[c][i] + d[i]));  // h is stored in bf16
        *reinterpret_cast<us8*>(h_out + base + ch * 8) = pack8(v[c]);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += v[c][i] * v[c][i];
    }
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)D + eps);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      float wv[8], o[8];
      unpack8(*reinterpret_cast<const us8*>(w + ch * 8), wv);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = v[c][i] * r * wv[i];
      *reinterpret_cast<us8*>(y + base + ch * 8) = pack8(o);
    }
  }
  if (lane == 0) rstd_out[row] = r;
}

// Block-per-row variant for few rows (serving decode: rows = batch <= 256): one wave per row left
// 1 wave per CU at batch 256 (latency-bound: 17 us for 256 x 8192, 1 TB/s); a 256-thread block per
// row gives every lane 1-4 chunks, issues the weight loads before the reduction, and combines the
// 4 wave sums through LDS.
// Q (fp8 serving): instead of the bf16 y, write y as e4m3 bytes with one per-row scale
// (max|y| / 448) to q_out / qs_out — the activation quantization of the next fp8 GEMM fused in.
// SC (with ADD): delta is the raw product of a tensor-wise-scaled fp8 GEMM whose row-wise scales
// dr[row] (per token) and dc[col] (per output channel) are applied here -- rounded to bf16 as the
// GEMM's own output would be -- before the residual add (fp8 serving prefill, model.py RawScaled)
template <int NCH, bool ADD, bool Q = false, bool SC = false>
__global__ __launch_bounds__(256) void rmsnorm_fwd_rowblock_kernel(const bf16_t* __restrict__ x,
                                                                   const bf16_t* __restrict__ delta,
                                                                   const bf16_t* __restrict__ w,
                                                                   bf16_t* __restrict__ h_out,
                                                                   bf16_t* __restrict__ y,
                                                                   float* __restrict__ rstd_out,
                                                                   int D, float eps,
                                                                   unsigned char* __restrict__ q_out = nullptr,
                                                                   float* __restrict__ qs_out = nullptr,
                                                                   const float* __restrict__ dr = nullptr,
                                                                   const float* __restrict__ dc = nullptr) {
  __shared__ float part[4];
  __shared__ float pmax[4];
  const int tid = threadIdx.x, row = blockIdx.x;
  const int nch = D >> 3;
  const size_t base = (size_t)row * D;
  float v[NCH][8], wv[NCH][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int ch = tid + c * 256;
    if (ch < nch) {
      unpack8(*reinterpret_cast<const us8*>(x + base + ch * 8), v[c]);
      unpack8(*reinterpret_cast<const us8*>(w + ch * 8), wv[c]);
      if constexpr (ADD) {
        float d[8];
        unpack8(*reinterpret_cast<const us8*>(delta + base + ch * 8), d);
        if constexpr (SC) {
          const float rr = dr[row];
          const f4 c0 = *reinterpret_cast<const f4*>(dc + ch * 8), c1 = *reinterpret_cast<const f4*>(dc + ch * 8 + 4);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            d[i] = bf2f(f2bf(d[i] * rr * c0[i]));
            d[4 + i] = bf2f(f2bf(d[4 + i] * rr * c1[i]));
          }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) v[c][i] = bf2f(f2bf(v[c][i] + d[i]));  // h is stored in bf16
        *reinterpret_cast<us8*>(h_out + base + ch * 8) = pack8(v[c]);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += v[c][i] * v[c][i];
    }
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) part[tid >> 6] = ss;
  __syncthreads();
  ss = part[0] + part[1] + part[2] + part[3];
  const float r = rsqrtf(ss / (float)D + eps);
  if constexpr (Q) {
    // y in registers, the row's absmax across the block, then e4m3 bytes (8 per chunk)
    float amax = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int ch = tid + c * 256;
      if (ch < nch) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          v[c][i] = bf2f(f2bf(v[c][i] * r * wv[c][i]));  // the bf16 value the unfused path quantizes
          amax = fmaxf(amax, fabsf(v[c][i]));
        }
      }
    }
    amax = wave_max(amax);
    if ((tid & 63) == 0) pmax[tid >> 6] = amax;
    __syncthreads();
    amax = fmaxf(fmaxf(pmax[0], pmax[1]), fmaxf(pmax[2], pmax[3]));
    const float scale = fmaxf(amax, 1e-12f) / 448.f, inv = 1.f / scale;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int ch = tid + c * 256;
      if (ch < nch) {
        typedef unsigned int u2 __attribute__((ext_vector_type(2)));
        u2 wq;
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const float* o = v[c] + 4 * h2;
          int wd = __builtin_amdgcn_cvt_pk_fp8_f32(__builtin_amdgcn_fmed3f(o[0] * inv, 448.f, -448.f),
                                                   __builtin_amdgcn_fmed3f(o[1] * inv, 448.f, -448.f), 0, false);
          wq[h2] = __builtin_amdgcn_cvt_pk_fp8_f32(__builtin_amdgcn_fmed3f(o[2] * inv, 448.f, -448.f),
                                                   __builtin_amdgcn_fmed3f(o[3] * inv, 448.f, -448.f), wd, true);
        }
        *reinterpret_cast<u2*>(q_out + base + ch * 8) = wq;
      }
    }
    if (tid == 0) qs_out[row] = scale;
  } else {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int ch = tid + c * 256;
      if (ch < nch) {
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = v[c][i] * r * wv[c][i];
        *reinterpret_cast<us8*>(y + base + ch * 8) = pack8(o);
      }
    }
  }
  if (tid == 0) rstd_out[row] = r;
}

// ------------------------------------------------------------------------------------------------
// RMSNorm backward: dx = r*g - h*r^3*mean(g*h) (+ dres), g = dy*w ;  dw partials per block.
// One 256-thread block per row (grid-strided over rows): each thread owns NCH chunks of 8
// columns, so its dw contribution stays in NCH*8 registers for the whole launch; the row dot is a
// wave shuffle + a 4-entry LDS combine.  Each block writes one fp32 dw partial row; colsum (two passes)
// reduces the [grid, D] partials.
// ------------------------------------------------------------------------------------------------
template <int NCH, bool RES>
__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(const bf16_t* __restrict__ dy,
                                                          const bf16_t* __restrict__ h,
                                                          const bf16_t* __restrict__ w,
                                                          const float* __restrict__ rstd,
                                                          const bf16_t* __restrict__ dres,
                                                          bf16_t* __restrict__ dx,
                                                          float* __restrict__ dw_part, int rows,
                                                          int D) {
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nch = D >> 3;
  float wv[NCH][8];
  float dwa[NCH][8];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int ch = threadIdx.x + c * 256;
#pragma unroll
    for (int i = 0; i < 8; ++i) dwa[c][i] = 0.f;
    if (ch < nch) unpack8(*reinterpret_cast<const us8*>(w + ch * 8), wv[c]);
  }
  int parity = 0;
  for (int row = blockIdx.x; row < rows; row += gridDim.x, parity ^= 1) {
    const size_t base = (size_t)row * D;
    const float r = rstd[row];
    float hv[NCH][8], g[NCH][8];
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int ch = threadIdx.x + c * 256;
      if (ch < nch) {
        float d[8];
        unpack8(*reinterpret_cast<const us8*>(dy + base + ch * 8), d);
        unpack8(*reinterpret_cast<const us8*>(h + base + ch * 8), hv[c]);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          g[c][i] = d[i] * wv[c][i];
          dot += g[c][i] * hv[c][i];
          dwa[c][i] += d[i] * hv[c][i] * r;
        }
      }
    }
    dot = wave_sum(dot);
    if (lane == 0) red[parity][wid] = dot;  // double-buffered: one barrier per row
    __syncthreads();
    dot = red[parity][0] + red[parity][1] + red[parity][2] + red[parity][3];
    const float k = dot * r * r * r / (float)D;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int ch = threadIdx.x + c * 256;
      if (ch < nch) {
        float o[8];
        if constexpr (RES) {
          unpack8(*reinterpret_cast<const us8*>(dres + base + ch * 8), o);
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] = 0.f;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] += r * g[c][i] - hv[c][i] * k;
        *reinterpret_cast<us8*>(dx + base + ch * 8) = pack8(o);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int ch = threadIdx.x + c * 256;
    if (ch < nch) {
      f4* dst = reinterpret_cast<f4*>(dw_part + (size_t)blockIdx.x * D + ch * 8);
      dst[0] = f4{dwa[c][0], dwa[c][1], dwa[c][2], dwa[c][3]};
      dst[1] = f4{dwa[c][4], dwa[c][5], dwa[c][6], dwa[c][7]};
    }
  }
}

// column sums of a [P, D] fp32 matrix -> out[D], two deterministic passes that fill the chip
// (the old single pass ran D/64 = 64 workgroups for D=4096: 69 us for 16 MB, r1f profile).
//  pass 1: grid (D/256) x RS; a wave reads 256 columns as float4, the 4 waves of a block split
//          the block's row range, LDS combine, and the block's partial overwrites the FIRST row
//          of its own range (only this block reads that range, and it has finished reading).
//  pass 2: one wave per 256 columns sums the RS partial rows.
constexpr int COLSUM_RS = 16;
__global__ __launch_bounds__(256) void colsum_pass1_kernel(float* __restrict__ part, int P, int D,
                                                           int rpb) {
  __shared__ float4 red[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int col = (blockIdx.x * 64 + lane) * 4;
  const int r0 = blockIdx.y * rpb, r1 = min(P, r0 + rpb);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col < D)
    for (int r = r0 + wv; r < r1; r += 4) {
      const float4 v = *reinterpret_cast<const float4*>(part + (size_t)r * D + col);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  red[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && col < D && r0 < r1) {
    float4 a = red[0][lane];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const float4 b = red[k][lane];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    *reinterpret_cast<float4*>(part + (size_t)r0 * D + col) = a;
  }
}

// out (fp32) = column sums, or -- when out_bf16 is given -- out_bf16 = (accumulate ? out_bf16 : 0)
// + column sums: the norm weight's gradient lands directly in the optimizer's flat bf16 buffer
// (no fp32 -> bf16 copy kernel and no AccumulateGrad add kernel per norm per micro-batch)
__global__ __launch_bounds__(64) void colsum_pass2_kernel(const float* __restrict__ part,
                                                          float* __restrict__ out,
                                                          bf16_t* __restrict__ out_bf16, int accumulate,
                                                          int P, int D, int rpb) {
  const int col = (blockIdx.x * 64 + threadIdx.x) * 4;
  if (col >= D) return;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
  for (int r = 0; r < P; r += rpb) {
    const float4 v = *reinterpret_cast<const float4*>(part + (size_t)r * D + col);
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  if (out_bf16 == nullptr) {
    *reinterpret_cast<float4*>(out + col) = a;
    return;
  }
  bf16_t* o = out_bf16 + col;
  if (accumulate) {
    a.x += bf2f(o[0]); a.y += bf2f(o[1]); a.z += bf2f(o[2]); a.w += bf2f(o[3]);
  }
  o[0] = f2bf(a.x); o[1] = f2bf(a.y); o[2] = f2bf(a.z); o[3] = f2bf(a.w);
}

static hipError_t colsum(float* part, float* out, bf16_t* out_bf16, int accumulate, int P, int D,
                         hipStream_t st) {
  const int rpb = (P + COLSUM_RS - 1) / COLSUM_RS;
  const int cb = (D + 255) / 256;
  colsum_pass1_kernel<<<dim3(cb, COLSUM_RS), 256, 0, st>>>(part, P, D, rpb);
  DSA_CHECK(hipGetLastError());
  colsum_pass2_kernel<<<cb, 64, 0, st>>>(part, out, out_bf16, accumulate, P, D, rpb);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// SwiGLU on [T, 2F] = [gate | up]  ->  [T, F]
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float silu_f(float g) { return g / (1.f + __expf(-g)); }

__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const bf16_t* __restrict__ gu,
                                                         bf16_t* __restrict__ out, int rows,
                                                         int F) {
  const int nch = F >> 3;
  const size_t total = (size_t)rows * nch;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t row = i / nch, ch = i % nch;
    float g[8], u[8], o[8];
    unpack8(*reinterpret_cast<const us8*>(gu + row * 2 * F + ch * 8), g);
    unpack8(*reinterpret_cast<const us8*>(gu + row * 2 * F + F + ch * 8), u);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = silu_f(g[k]) * u[k];
    *reinterpret_cast<us8*>(out + row * F + ch * 8) = pack8(o);
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const bf16_t* __restrict__ da,
                                                         const bf16_t* __restrict__ gu,
                                                         bf16_t* __restrict__ dgu, int rows,
                                                         int F) {
  const int nch = F >> 3;
  const size_t total = (size_t)rows * nch;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t row = i / nch, ch = i % nch;
    float g[8], u[8], d[8], dg[8], du[8];
    unpack8(*reinterpret_cast<const us8*>(gu + row * 2 * F + ch * 8), g);
    unpack8(*reinterpret_cast<const us8*>(gu + row * 2 * F + F + ch * 8), u);
    unpack8(*reinterpret_cast<const us8*>(da + row * F + ch * 8), d);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float s = 1.f / (1.f + __expf(-g[k]));
      du[k] = d[k] * g[k] * s;
      dg[k] = d[k] * u[k] * s * (1.f + g[k] * (1.f - s));
    }
    *reinterpret_cast<us8*>(dgu + row * 2 * F + ch * 8) = pack8(dg);
    *reinterpret_cast<us8*>(dgu + row * 2 * F + F + ch * 8) = pack8(du);
  }
}

// ------------------------------------------------------------------------------------------------
// RoPE (rotate-half) over the first n_rot heads of a fused qkv row [NH*D]; other heads copied.
// cos/sin tables [S, D/2] fp32 are precomputed on the host (no on-device trig).
// Each lane owns 8 consecutive pairs (i, i + D/2) of one head.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rope_qkv_kernel(const bf16_t* __restrict__ in,
                                                       bf16_t* __restrict__ out,
                                                       const float* __restrict__ cosT,
                                                       const float* __restrict__ sinT, int rows,
                                                       int S, int NH, int n_rot, int D,
                                                       float sign) {
  const int half = D >> 1;
  const int cph = half >> 3;  // 8-pair chunks per head
  const size_t per_row = (size_t)NH * cph;
  const size_t total = (size_t)rows * per_row;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t row = i / per_row;
    const int rem = (int)(i % per_row);
    const int head = rem / cph, c = rem % cph;
    const size_t off = row * (size_t)NH * D + (size_t)head * D + c * 8;
    us8 a = *reinterpret_cast<const us8*>(in + off);
    us8 b = *reinterpret_cast<const us8*>(in + off + half);
    if (head < n_rot) {
      const int pos = (int)(row % S);
      const f4* cp = reinterpret_cast<const f4*>(cosT + (size_t)pos * half + c * 8);
      const f4* sp = reinterpret_cast<const f4*>(sinT + (size_t)pos * half + c * 8);
      const f4 c0 = cp[0], c1 = cp[1], s0 = sp[0], s1 = sp[1];
      const float cs[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
      const float sn[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
      float x1[8], x2[8], o1[8], o2[8];
      unpack8(a, x1);
      unpack8(b, x2);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float s = sign * sn[k];
        o1[k] = x1[k] * cs[k] - x2[k] * s;
        o2[k] = x2[k] * cs[k] + x1[k] * s;
      }
      a = pack8(o1);
      b = pack8(o2);
    }
    *reinterpret_cast<us8*>(out + off) = a;
    *reinterpret_cast<us8*>(out + off + half) = b;
  }
}

// ------------------------------------------------------------------------------------------------
// Softmax cross-entropy over a [T, V] bf16 logits matrix. One 256-thread block per row.
// fwd: online (max, sum-exp) per lane -> block combine -> lse, loss = lse - logit[target].
// bwd: dlogit = scale * (exp(logit - lse) - onehot), written in place over the logits.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mn));
  m = mn;
}

__global__ __launch_bounds__(256) void ce_fwd_kernel(const bf16_t* __restrict__ logits,
                                                     const int64_t* __restrict__ target,
                                                     float* __restrict__ loss,
                                                     float* __restrict__ lse_out, int V) {
  __shared__ float sm[8], ss[8];
  const size_t row = blockIdx.x;
  const bf16_t* L = logits + row * (size_t)V;
  float m = -INFINITY, s = 0.f;
  const int nch = V >> 3;
  for (int ch = threadIdx.x; ch < nch; ch += blockDim.x) {
    float v[8];
    unpack8(*reinterpret_cast<const us8*>(L + ch * 8), v);
    float lm = v[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) lm = fmaxf(lm, v[k]);
    float ls = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) ls += __expf(v[k] - lm);
    online_merge(m, s, lm, ls);
  }
  for (int i = (nch << 3) + threadIdx.x; i < V; i += blockDim.x) online_merge(m, s, bf2f(L[i]), 1.f);
  // wave combine
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    online_merge(m, s, m2, s2);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    sm[wid] = m;
    ss[wid] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) online_merge(m, s, sm[w], ss[w]);
    const float lse = m + __logf(s);
    lse_out[row] = lse;
    const int64_t t = target[row];
    loss[row] = (t >= 0 && t < V) ? lse - bf2f(L[t]) : 0.f;
  }
}

__global__ __launch_bounds__(256) void ce_bwd_kernel(const bf16_t* __restrict__ logits,
                                                     const int64_t* __restrict__ target,
                                                     const float* __restrict__ lse,
                                                     const float* __restrict__ scale_ptr,
                                                     bf16_t* __restrict__ dlogits, int V) {
  const size_t row = blockIdx.x;
  const float l = lse[row];
  const float scale = scale_ptr[0];
  const int64_t t = target[row];
  const bf16_t* L = logits + row * (size_t)V;
  bf16_t* G = dlogits + row * (size_t)V;
  const int nch = V >> 3;
  for (int ch = threadIdx.x; ch < nch; ch += blockDim.x) {
    float v[8];
    unpack8(*reinterpret_cast<const us8*>(L + ch * 8), v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      v[k] = __expf(v[k] - l);
      if (ch * 8 + k == t) v[k] -= 1.f;
      v[k] *= scale;
    }
    *reinterpret_cast<us8*>(G + ch * 8) = pack8(v);
  }
  for (int i = (nch << 3) + threadIdx.x; i < V; i += blockDim.x) {
    float p = __expf(bf2f(L[i]) - l);
    if (i == t) p -= 1.f;
    G[i] = f2bf(p * scale);
  }
}

// ------------------------------------------------------------------------------------------------
// Fused AdamW over flat shards: bf16 param/grad, fp32 master/m/v (decoupled weight decay).
// 8 elements per lane per iteration: one dwordx4 for param/grad, two for each fp32 stream.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void adamw_kernel(bf16_t* __restrict__ param,
                                                    const bf16_t* __restrict__ grad,
                                                    float* __restrict__ master,
                                                    float* __restrict__ mom,
                                                    float* __restrict__ var, size_t n, float lr,
                                                    float b1, float b2, float eps, float wd,
                                                    float bc1, float bc2, float gscale) {
  const size_t nv = n >> 3;
  const float step_size = lr / bc1;
  const float inv_bc2_sqrt = rsqrtf(bc2);
  const float decay = 1.f - lr * wd;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nv;
       i += (size_t)gridDim.x * blockDim.x) {
    float g[8];
    unpack8(*reinterpret_cast<const us8*>(grad + i * 8), g);
    f4* mp = reinterpret_cast<f4*>(master + i * 8);
    f4* m1 = reinterpret_cast<f4*>(mom + i * 8);
    f4* m2 = reinterpret_cast<f4*>(var + i * 8);
    f4 p0 = mp[0], p1 = mp[1], a0 = m1[0], a1 = m1[1], v0 = m2[0], v1 = m2[1];
    float p[8] = {p0[0], p0[1], p0[2], p0[3], p1[0], p1[1], p1[2], p1[3]};
    float a[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
    float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float gg = g[k] * gscale;
      a[k] = b1 * a[k] + (1.f - b1) * gg;
      v[k] = b2 * v[k] + (1.f - b2) * gg * gg;
      const float denom = sqrtf(v[k]) * inv_bc2_sqrt + eps;
      p[k] = p[k] * decay - step_size * a[k] / denom;
    }
    mp[0] = f4{p[0], p[1], p[2], p[3]};
    mp[1] = f4{p[4], p[5], p[6], p[7]};
    m1[0] = f4{a[0], a[1], a[2], a[3]};
    m1[1] = f4{a[4], a[5], a[6], a[7]};
    m2[0] = f4{v[0], v[1], v[2], v[3]};
    m2[1] = f4{v[4], v[5], v[6], v[7]};
    *reinterpret_cast<us8*>(param + i * 8) = pack8(p);
  }
  // scalar tail (n % 8)
  for (size_t i = (nv << 3) + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const float gg = bf2f(grad[i]) * gscale;
    const float a = b1 * mom[i] + (1.f - b1) * gg;
    const float v = b2 * var[i] + (1.f - b2) * gg * gg;
    const float p = master[i] * decay - step_size * a / (sqrtf(v) * inv_bc2_sqrt + eps);
    mom[i] = a;
    var[i] = v;
    master[i] = p;
    param[i] = f2bf(p);
  }
}

// ================================================================================================
// host launchers (raw pointers + stream; the torch binding lives in bindings.cpp)
// ================================================================================================
// Grid for a grid-stride elementwise kernel: uncapped by default, i.e. one work item per thread:
// blocks are then dispatched in address order and the chip streams memory front to back (a plain
// copy measured 6.18 TB/s that way vs 4.2-4.8 TB/s with 8-32 resident blocks per CU striding
// across the buffer, tools/diag/hbm_variants.hip; same box: SwiGLU fwd 139 -> 123 us, bwd 225 ->
// 209 us, AdamW 6.22 -> 6.49 TB/s, profiles/grid_cap_r1q.txt).  DSTACK_AMD_GRID_CAP=N caps it.
static inline int grid_for(size_t work, int block, int cap = 0x7fffffff) {
  static const long env_cap = [] {
    const char* v = getenv("DSTACK_AMD_GRID_CAP");
    return v ? atol(v) : -1L;
  }();
  if (env_cap >= 0) cap = env_cap == 0 ? 0x7fffffff : (int)env_cap;
  size_t g = (work + block - 1) / block;
  if (g > (size_t)cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

#define NCH_DISPATCH(D, ...)                       \
  do {                                             \
    const int _n = ((D) / 8 + 63) / 64;            \
    if (_n <= 1) { constexpr int NCH = 1; __VA_ARGS__; }        \
    else if (_n <= 2) { constexpr int NCH = 2; __VA_ARGS__; }   \
    else if (_n <= 4) { constexpr int NCH = 4; __VA_ARGS__; }   \
    else if (_n <= 8) { constexpr int NCH = 8; __VA_ARGS__; }   \
    else if (_n <= 16) { constexpr int NCH = 16; __VA_ARGS__; } \
    else return hipErrorInvalidValue;              \
  } while (0)

// chunks-per-thread dispatch for block-per-row kernels (256 threads x 8 columns per chunk)
#define NCH_DISPATCH_BLK(D, ...)                   \
  do {                                             \
    const int _n = ((D) / 8 + 255) / 256;          \
    if (_n <= 1) { constexpr int NCH = 1; __VA_ARGS__; }      \
    else if (_n <= 2) { constexpr int NCH = 2; __VA_ARGS__; } \
    else if (_n <= 4) { constexpr int NCH = 4; __VA_ARGS__; } \
    else return hipErrorInvalidValue;              \
  } while (0)

// ------------------------------------------------------------------------------------------------
// 2-D bf16 transpose out[C, R] = in[R, C]^T (reduction-contiguous operands for the weight-gradient
// GEMMs: hipBLASLt runs dW = g^T x at ~1.1 PFLOP/s when both operands are token-major and at
// 1.35-1.56 PFLOP/s when they are token-contiguous, tools/bench_wgrad_layouts.py).
// Tile 128 rows x 64 columns per 256-thread workgroup: 16-byte coalesced row loads into LDS, then
// ds_read_b64_tr_b16 (gfx950's transposed LDS read: a 16-lane group gets a 4-row x 16-column block
// column-major, lane i = column i) twice per lane gives 8 consecutive rows of one column = one
// 16-byte store into an output row.
//  * Store coalescing: wave w owns output rows c0+16w .. +15 (column block w of the tile) and its 4
//    lane groups take 4 consecutive 8-row chunks, so one store instruction writes 16 output rows x
//    64 contiguous bytes (the first version spread an instruction over 64 rows x 16 B).
//  * LDS banks: row pitch 96 elements (48 dwords: rows 0-3 of a block start on banks 0/48/32/16) and
//    the two 32-byte halves of a row's 64-byte column span swapped on rows with bit 3 set, so a
//    32-lane half (two groups = rows 8 apart, same columns) covers all 64 banks once.
// (2-byte LDS gathers: 45-49 us per 64 MB = 2.7 TB/s, r1j profile; 64-row stores: 3.7 TB/s, r1k.)
// ------------------------------------------------------------------------------------------------
constexpr int TR_R = 128, TR_C = 64, TR_P = 96;

// element offset in the LDS tile of (row r, column c); c's 16-column block is swizzled by row bit 3
__device__ __forceinline__ int tr_off(int r, int c) { return r * TR_P + (c ^ (((r >> 3) & 1) << 4)); }

// write the [TR_R][TR_C] LDS tile transposed: out[(c0 + c) * ld + r0 + r]
__device__ __forceinline__ void tr_store_tile(const bf16_t* tile, bf16_t* out, size_t ld, int c0, int r0,
                                              int t) {
  const int w = t >> 6, j = (t >> 4) & 3, lane16 = t & 15, q = (t >> 2) & 3, p = t & 3;
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    const int rk = pass * 4 + j;  // 8-row chunk
    const int row = rk * 8 + q;
    const bf16_t* lo_p = tile + tr_off(row, w * 16 + 4 * p);
    const bf16_t* hi_p = tile + tr_off(row + 4, w * 16 + 4 * p);
    const dsa::bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS3(dsa::bf16x4, lo_p));
    const dsa::bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS3(dsa::bf16x4, hi_p));
    const dsa::bf16x8 o = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    *reinterpret_cast<dsa::bf16x8*>(out + (size_t)(c0 + w * 16 + lane16) * ld + r0 + rk * 8) = o;
  }
}

__global__ __launch_bounds__(256) void transpose2d_kernel(const bf16_t* __restrict__ in,
                                                          bf16_t* __restrict__ out, int R, int C) {
  __shared__ __attribute__((aligned(16))) bf16_t tile[TR_R * TR_P];
  const int c0 = blockIdx.x * TR_C, r0 = blockIdx.y * TR_R;
  const int t = threadIdx.x;
  us8 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // 128 rows x 8 chunks of 8 columns = 1024 chunks / 256 threads
    const int idx = i * 256 + t, r = idx >> 3, ch = idx & 7;
    v[i] = *reinterpret_cast<const us8*>(in + (size_t)(r0 + r) * C + c0 + ch * 8);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = i * 256 + t, r = idx >> 3, ch = idx & 7;
    *reinterpret_cast<us8*>(tile + tr_off(r, ch * 8)) = v[i];
  }
  __syncthreads();
  tr_store_tile(tile, out, (size_t)R, c0, r0, t);
}

// SwiGLU forward that also writes the transposed output aT[F, T] (the down projection's
// token-contiguous weight-gradient operand, so backward needs no separate transpose of a: the
// extra 2 B/element write replaces a 4 B/element transpose pass).  Same 128 x 64 tiling and
// transposed store as transpose2d_kernel.
__global__ __launch_bounds__(256) void swiglu_fwd_t_kernel(const bf16_t* __restrict__ gu,
                                                           bf16_t* __restrict__ out,
                                                           bf16_t* __restrict__ outT, int T, int F) {
  __shared__ __attribute__((aligned(16))) bf16_t tile[TR_R * TR_P];
  const int c0 = blockIdx.x * TR_C, r0 = blockIdx.y * TR_R;
  const int t = threadIdx.x;
  us8 gv[4], uv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = i * 256 + t, r = idx >> 3, ch = idx & 7;
    const bf16_t* src = gu + (size_t)(r0 + r) * 2 * F + c0 + ch * 8;
    gv[i] = *reinterpret_cast<const us8*>(src);
    uv[i] = *reinterpret_cast<const us8*>(src + F);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = i * 256 + t, r = idx >> 3, ch = idx & 7;
    float g[8], u[8], o[8];
    unpack8(gv[i], g);
    unpack8(uv[i], u);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = silu_f(g[k]) * u[k];
    const us8 a = pack8(o);
    *reinterpret_cast<us8*>(out + (size_t)(r0 + r) * F + c0 + ch * 8) = a;
    *reinterpret_cast<us8*>(tile + tr_off(r, ch * 8)) = a;
  }
  __syncthreads();
  tr_store_tile(tile, outT, (size_t)T, c0, r0, t);
}

// SwiGLU backward that also writes dgu^T [2F, T]: the gate/up projection's weight gradient
// dW = dgu^T h then runs with both operands token-contiguous (TN) instead of token-major (TT),
// for one extra 2 B/element write of the [T, 2F] gradient.  Same 128 x 64 tiling and transposed
// store as transpose2d_kernel; the gate and up halves go through two LDS tiles.
__global__ __launch_bounds__(256) void swiglu_bwd_t_kernel(const bf16_t* __restrict__ da,
                                                           const bf16_t* __restrict__ gu,
                                                           bf16_t* __restrict__ dgu,
                                                           bf16_t* __restrict__ dguT, int T, int F) {
  __shared__ __attribute__((aligned(16))) bf16_t tile_g[TR_R * TR_P];
  __shared__ __attribute__((aligned(16))) bf16_t tile_u[TR_R * TR_P];
  const int c0 = blockIdx.x * TR_C, r0 = blockIdx.y * TR_R;
  const int t = threadIdx.x;
  us8 gv[4], uv[4], dv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = i * 256 + t, r = idx >> 3, ch = idx & 7;
    const bf16_t* src = gu + (size_t)(r0 + r) * 2 * F + c0 + ch * 8;
    gv[i] = *reinterpret_cast<const us8*>(src);
    uv[i] = *reinterpret_cast<const us8*>(src + F);
    dv[i] = *reinterpret_cast<const us8*>(da + (size_t)(r0 + r) * F + c0 + ch * 8);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = i * 256 + t, r = idx >> 3, ch = idx & 7;
    float g[8], u[8], d[8], dg[8], du[8];
    unpack8(gv[i], g);
    unpack8(uv[i], u);
    unpack8(dv[i], d);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float s = 1.f / (1.f + __expf(-g[k]));
      du[k] = d[k] * g[k] * s;
      dg[k] = d[k] * u[k] * s * (1.f + g[k] * (1.f - s));
    }
    const us8 a = pack8(dg), b = pack8(du);
    bf16_t* dst = dgu + (size_t)(r0 + r) * 2 * F + c0 + ch * 8;
    *reinterpret_cast<us8*>(dst) = a;
    *reinterpret_cast<us8*>(dst + F) = b;
    *reinterpret_cast<us8*>(tile_g + tr_off(r, ch * 8)) = a;
    *reinterpret_cast<us8*>(tile_u + tr_off(r, ch * 8)) = b;
  }
  __syncthreads();
  tr_store_tile(tile_g, dguT, (size_t)T, c0, r0, t);
  tr_store_tile(tile_u, dguT, (size_t)T, F + c0, r0, t);
}

extern "C" hipError_t dsa_swiglu_bwd_t(const void* da, const void* gu, void* dgu, void* dguT, int T, int F,
                                       hipStream_t st) {
  if (T % TR_R || F % TR_C) return hipErrorInvalidValue;
  swiglu_bwd_t_kernel<<<dim3(F / TR_C, T / TR_R), 256, 0, st>>>((const bf16_t*)da, (const bf16_t*)gu,
                                                                (bf16_t*)dgu, (bf16_t*)dguT, T, F);
  return hipGetLastError();
}

extern "C" hipError_t dsa_swiglu_fwd_t(const void* gu, void* out, void* outT, int T, int F, hipStream_t st) {
  if (T % TR_R || F % TR_C) return hipErrorInvalidValue;
  swiglu_fwd_t_kernel<<<dim3(F / TR_C, T / TR_R), 256, 0, st>>>((const bf16_t*)gu, (bf16_t*)out,
                                                                (bf16_t*)outT, T, F);
  return hipGetLastError();
}

extern "C" bool dsa_transpose2d_supported(int R, int C) { return R % TR_R == 0 && C % TR_C == 0; }

extern "C" hipError_t dsa_transpose2d(const void* in, void* out, int R, int C, hipStream_t st) {
  if (!dsa_transpose2d_supported(R, C)) return hipErrorInvalidValue;
  transpose2d_kernel<<<dim3(C / TR_C, R / TR_R), 256, 0, st>>>((const bf16_t*)in, (bf16_t*)out, R, C);
  return hipGetLastError();
}

extern "C" hipError_t dsa_rmsnorm_fwd(const void* x, const void* delta, const void* w, void* h_out,
                                      void* y, float* rstd, int rows, int D, float eps,
                                      hipStream_t st) {
  if (D % 8) return hipErrorInvalidValue;
  const int block = 256, rpb = block / 64;
  const int grid = (rows + rpb - 1) / rpb;
  if (rows <= 1024 && D <= 8192) {  // few rows: a block per row (decode)
    if (delta) {
      NCH_DISPATCH_BLK(D, rmsnorm_fwd_rowblock_kernel<NCH, true><<<rows, 256, 0, st>>>(
          (const bf16_t*)x, (const bf16_t*)delta, (const bf16_t*)w, (bf16_t*)h_out, (bf16_t*)y, rstd, D, eps));
    } else {
      NCH_DISPATCH_BLK(D, rmsnorm_fwd_rowblock_kernel<NCH, false><<<rows, 256, 0, st>>>(
          (const bf16_t*)x, nullptr, (const bf16_t*)w, nullptr, (bf16_t*)y, rstd, D, eps));
    }
    return hipGetLastError();
  }
  if (delta) {
    NCH_DISPATCH(D, rmsnorm_fwd_kernel<NCH, true><<<grid, block, 0, st>>>(
        (const bf16_t*)x, (const bf16_t*)delta, (const bf16_t*)w, (bf16_t*)h_out, (bf16_t*)y, rstd,
        rows, D, eps));
  } else {
    NCH_DISPATCH(D, rmsnorm_fwd_kernel<NCH, false><<<grid, block, 0, st>>>(
        (const bf16_t*)x, nullptr, (const bf16_t*)w, nullptr, (bf16_t*)y, rstd, rows, D, eps));
  }
  return hipGetLastError();
}

// (add +) RMSNorm whose output goes straight to e4m3 with per-row scales (fp8 serving: decode
// batches and prefill, one workgroup per row); dr / dc: row-wise scales of a raw fp8 GEMM delta
extern "C" bool dsa_rmsnorm_fwd_fp8_supported(int rows, int D) { return rows > 0 && D % 8 == 0 && D <= 8192; }

extern "C" hipError_t dsa_rmsnorm_fwd_fp8(const void* x, const void* delta, const void* w, void* h_out, void* q,
                                          float* qs, float* rstd, int rows, int D, float eps, const float* dr,
                                          const float* dc, hipStream_t st) {
  if (!dsa_rmsnorm_fwd_fp8_supported(rows, D) || ((dr == nullptr) != (dc == nullptr)) || (dr && !delta))
    return hipErrorInvalidValue;
  if (dr) {
    NCH_DISPATCH_BLK(D, rmsnorm_fwd_rowblock_kernel<NCH, true, true, true><<<rows, 256, 0, st>>>(
        (const bf16_t*)x, (const bf16_t*)delta, (const bf16_t*)w, (bf16_t*)h_out, nullptr, rstd, D, eps,
        (unsigned char*)q, qs, dr, dc));
  } else if (delta) {
    NCH_DISPATCH_BLK(D, rmsnorm_fwd_rowblock_kernel<NCH, true, true><<<rows, 256, 0, st>>>(
        (const bf16_t*)x, (const bf16_t*)delta, (const bf16_t*)w, (bf16_t*)h_out, nullptr, rstd, D, eps,
        (unsigned char*)q, qs));
  } else {
    NCH_DISPATCH_BLK(D, rmsnorm_fwd_rowblock_kernel<NCH, false, true><<<rows, 256, 0, st>>>(
        (const bf16_t*)x, nullptr, (const bf16_t*)w, nullptr, nullptr, rstd, D, eps, (unsigned char*)q, qs));
  }
  return hipGetLastError();
}

// dw_part must hold grid*D floats where grid = dsa_rmsnorm_bwd_grid(rows)
extern "C" int dsa_rmsnorm_bwd_grid(int rows) {
  int g = rows;
  return g > 1024 ? 1024 : (g < 1 ? 1 : g);
}

// dw_bf16 != null: the weight gradient goes to dw_bf16 (bf16, accumulated into when `accumulate`)
// instead of the fp32 dw
extern "C" hipError_t dsa_rmsnorm_bwd(const void* dy, const void* h, const void* w, const float* rstd,
                                      const void* dres, void* dx, float* dw_part, float* dw,
                                      void* dw_bf16, int accumulate, int rows, int D, hipStream_t st) {
  if (D % 8) return hipErrorInvalidValue;
  const int block = 256;
  const int grid = dsa_rmsnorm_bwd_grid(rows);
  const size_t lds = 0;
  if (dres) {
    NCH_DISPATCH_BLK(D, rmsnorm_bwd_kernel<NCH, true><<<grid, block, lds, st>>>(
        (const bf16_t*)dy, (const bf16_t*)h, (const bf16_t*)w, rstd, (const bf16_t*)dres,
        (bf16_t*)dx, dw_part, rows, D));
  } else {
    NCH_DISPATCH_BLK(D, rmsnorm_bwd_kernel<NCH, false><<<grid, block, lds, st>>>(
        (const bf16_t*)dy, (const bf16_t*)h, (const bf16_t*)w, rstd, nullptr, (bf16_t*)dx, dw_part,
        rows, D));
  }
  DSA_CHECK(hipGetLastError());
  return colsum(dw_part, dw, (bf16_t*)dw_bf16, accumulate, grid, D, st);
}

extern "C" hipError_t dsa_swiglu_fwd(const void* gu, void* out, int rows, int F, hipStream_t st) {
  if (F % 8) return hipErrorInvalidValue;
  const size_t work = (size_t)rows * (F / 8);
  swiglu_fwd_kernel<<<grid_for(work, 256), 256, 0, st>>>((const bf16_t*)gu, (bf16_t*)out, rows, F);
  return hipGetLastError();
}

extern "C" hipError_t dsa_swiglu_bwd(const void* da, const void* gu, void* dgu, int rows, int F,
                                     hipStream_t st) {
  if (F % 8) return hipErrorInvalidValue;
  const size_t work = (size_t)rows * (F / 8);
  swiglu_bwd_kernel<<<grid_for(work, 256), 256, 0, st>>>((const bf16_t*)da, (const bf16_t*)gu,
                                                         (bf16_t*)dgu, rows, F);
  return hipGetLastError();
}

extern "C" hipError_t dsa_rope_qkv(const void* in, void* out, const float* cosT, const float* sinT,
                                   int rows, int S, int NH, int n_rot, int D, int inverse,
                                   hipStream_t st) {
  if (D % 16) return hipErrorInvalidValue;
  const size_t work = (size_t)rows * NH * (D / 16);
  rope_qkv_kernel<<<grid_for(work, 256), 256, 0, st>>>((const bf16_t*)in, (bf16_t*)out, cosT, sinT,
                                                       rows, S, NH, n_rot, D,
                                                       inverse ? -1.f : 1.f);
  return hipGetLastError();
}

extern "C" hipError_t dsa_ce_fwd(const void* logits, const int64_t* target, float* loss, float* lse,
                                 int rows, int V, hipStream_t st) {
  ce_fwd_kernel<<<rows, 256, 0, st>>>((const bf16_t*)logits, target, loss, lse, V);
  return hipGetLastError();
}

extern "C" hipError_t dsa_ce_bwd(const void* logits, const int64_t* target, const float* lse,
                                 const float* scale, void* dlogits, int rows, int V,
                                 hipStream_t st) {
  ce_bwd_kernel<<<rows, 256, 0, st>>>((const bf16_t*)logits, target, lse, scale, (bf16_t*)dlogits,
                                      V);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Embedding backward, deterministic with fp32 sums: the token ids are stably sorted on the host side
// (sorted_tok, order).  Workgroup j looks at sorted position j; only the first position of a run
// of equal ids does work: it sums the run's dy rows in fp32 (in stable order) and writes the bf16
// gradient row (or adds it to the row already there).  Only the touched rows are read/written,
// ~T*D*6 bytes, instead of PyTorch's dense [V, D] zero-fill + scatter + add per micro-batch
// (~1.9 ms per 8192-token micro-batch of Llama-3-8B, r2g trace).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void embed_bwd_kernel(const bf16_t* __restrict__ dy,
                                                        const int64_t* __restrict__ sorted_tok,
                                                        const int64_t* __restrict__ order,
                                                        bf16_t* __restrict__ grad, int T, int D,
                                                        int accumulate) {
  const int j = blockIdx.x;
  const int64_t tok = sorted_tok[j];
  if (j > 0 && sorted_tok[j - 1] == tok) return;  // not the first of its run (workgroup-uniform)
  int end = j + 1;
  while (end < T && sorted_tok[end] == tok) ++end;
  bf16_t* g = grad + tok * (int64_t)D;
  for (int c = threadIdx.x * 8; c < D; c += 256 * 8) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = j; k < end; ++k) {
      float v[8];
      unpack8(*reinterpret_cast<const us8*>(dy + order[k] * (int64_t)D + c), v);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += v[i];
    }
    if (accumulate) {
      float o[8];
      unpack8(*reinterpret_cast<const us8*>(g + c), o);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += o[i];
    }
    *reinterpret_cast<us8*>(g + c) = pack8(acc);
  }
}

extern "C" hipError_t dsa_embedding_bwd(const void* dy, const int64_t* sorted_tok, const int64_t* order,
                                        void* grad, int T, int D, int accumulate, hipStream_t st) {
  if (D % 8 || T <= 0) return hipErrorInvalidValue;
  embed_bwd_kernel<<<T, 256, 0, st>>>((const bf16_t*)dy, sorted_tok, order, (bf16_t*)grad, T, D, accumulate);
  return hipGetLastError();
}

extern "C" hipError_t dsa_adamw(void* param, const void* grad, float* master, float* m, float* v,
                                size_t n, float lr, float b1, float b2, float eps, float wd,
                                float bc1, float bc2, float gscale, int max_blocks, hipStream_t st) {
  // max_blocks > 0 caps the grid (persistent grid-stride): the optimizer-in-backward path runs
  // AdamW on a side stream beside MFMA-bound kernels, where a full-chip grid takes every CU's
  // slots and just serialises the two (r1g trace: dK/dV 1.13 -> 2.3 ms while AdamW ran).  Measured
  // same box (tools/gpu_sessions/run_r1l.sh, ms/step): full grid 799, 64 blocks 807, 32 843, 16 956, no
  // overlap 802 -- per-CU HBM bandwidth is too low for a small persistent grid, so 0 stays default
  const int cap = max_blocks > 0 ? max_blocks : 0x7fffffff;  // (DSTACK_AMD_GRID_CAP overrides)
  adamw_kernel<<<grid_for(n / 8 + 1, 256, cap), 256, 0, st>>>(
      (bf16_t*)param, (const bf16_t*)grad, master, m, v, n, lr, b1, b2, eps, wd, bc1, bc2, gscale);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Diagnostic: occupy `blocks` workgroup slots (threads x LDS bytes each) for `us` microseconds of
// wall clock (s_memrealtime, 100 MHz), the way a collective's kernel holds CUs beside compute
// (tools/diag/cu_hog.py: what a persistent GEMM pays when some CUs are taken).  Every wave exits
// when the time is up.
// ------------------------------------------------------------------------------------------------
__global__ void cu_hog_kernel(unsigned long long ticks, int* sink) {
  extern __shared__ int hog_lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  int acc = threadIdx.x;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    hog_lds[threadIdx.x & 255] = acc;
    acc += hog_lds[(threadIdx.x + 1) & 255];
    __builtin_amdgcn_s_sleep(2);
  }
  if (acc == 0x7fffffff) sink[0] = acc;  // keep the loop; practically never true
}

extern "C" hipError_t dsa_cu_hog(int blocks, int threads, int lds_bytes, double us, int* sink, hipStream_t st) {
  if (blocks <= 0 || threads <= 0 || threads > 1024 || lds_bytes < 1024 || lds_bytes > 160 * 1024 || us <= 0 ||
      us > 1e6)
    return hipErrorInvalidValue;
  if (lds_bytes > 64 * 1024)
    DSA_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&cu_hog_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes));
  cu_hog_kernel<<<blocks, threads, lds_bytes, st>>>((unsigned long long)(us * 100.0), sink);
  return hipGetLastError();
}
