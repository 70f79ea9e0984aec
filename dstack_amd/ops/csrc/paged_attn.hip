// Serving kernels for CDNA4 / gfx950: paged KV cache writes, paged decode attention (GQA,
// split-KV "flash decoding") and fused sampling.  Used by dstack_amd.serving (the MI355X-native
// inference engine behind `type: service` runs); the reference orchestrator ships no model code
// and delegates serving to vLLM/TGI containers (reference examples/deployment/vllm, tgi).
//
// KV cache layout, one pair of tensors per layer (PAGE = 64 tokens, head_dim 128):
//   k_cache [num_pages][KVH][PAGE][128]   token-major: one 256-B row per key
//   v_cache [num_pages][KVH][128][PAGE]   dim-major:   each V column is a 128-B run of 64 keys
// so every MFMA operand of the decode kernel is one 16-byte load straight from HBM (no LDS):
//
//  * S^T = K · Q^T with v_mfma_f32_16x16x32_bf16: A = 16 keys x 32 dims (lane = key row, 16 B of
//    its 256-B row), B = Q^T (lane = query column: the <=16 query heads that share one KV head,
//    GQA), so one lane holds 4 keys' scores of ONE query -> the softmax max/sum are 16 in-register
//    ops plus two xor-shuffles (lanes q, q+16, q+32, q+48).
//  * The 4 key tiles of a page are ordered so that the S^T accumulators, packed to bf16, are
//    directly the B operand of O^T += V^T · P^T with the keys in natural order (element j of lane
//    group g = key 32m + 8g + j), and the V^T operand is one 16-B load of the dim-major V page.
//  * O^T's layout puts the query on the lane, so the online-softmax rescale is lane-local.
//  * Split-KV: grid = (splits, KVH, batch); each one-wave workgroup walks `pages_per_split` pages,
//    writes a normalised partial O and its log2-sum-exp, and a combine kernel merges the splits
//    (skipped when there is one split).  The grid is a function of the batch size and the
//    maximum context only, so the decode step can be captured once per batch bucket in a
//    hipGraph.
#include "common.h"

#include <type_traits>

using namespace dsa;

namespace {

constexpr int PAGE = 64;
constexpr int HDIM = 128;

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4_t mfma16(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ bf16x8_t ld8(const bf16_t* p) { return *reinterpret_cast<const bf16x8_t*>(p); }

typedef unsigned int u2_t __attribute__((ext_vector_type(2)));

// 8 e4m3 cache bytes (held raw while in flight: half the registers of bf16) -> the same bf16x8
// MFMA operand the bf16 cache gives, converted right before the MFMA that reads it
__device__ __forceinline__ bf16x8_t fp8x8_to_bf16(const u2_t w) {
  bf16x8_t r;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const auto lo = __builtin_amdgcn_cvt_pk_f32_fp8(w[h], false);
    const auto hi = __builtin_amdgcn_cvt_pk_f32_fp8(w[h], true);
    r[4 * h + 0] = (__bf16)lo[0];
    r[4 * h + 1] = (__bf16)lo[1];
    r[4 * h + 2] = (__bf16)hi[0];
    r[4 * h + 3] = (__bf16)hi[1];
  }
  return r;
}

// one float -> one e4m3 byte (saturating at +-448)
__device__ __forceinline__ unsigned char to_fp8(float x) {
  x = __builtin_amdgcn_fmed3f(x, 448.f, -448.f);
  return (unsigned char)(__builtin_amdgcn_cvt_pk_fp8_f32(x, x, 0, false) & 0xff);
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// RoPE on q and k of the fused projection output (in place) + K/V scatter into the paged cache.
// qkv [T][(H + 2*KVH) * 128]; token t sits at position positions[t] and cache slot slots[t]
// (= page * PAGE + offset; < 0: padding token, not cached).  One thread = 8 rotation pairs.
// ------------------------------------------------------------------------------------------------
// FP8: the cache holds e4m3 bytes of k / k_scale and v / v_scale (same layout, 1 byte per value).
// SC: qkv is the raw product of a tensor-wise-scaled fp8 GEMM (serving prefill, model.py RawScaled);
// the per-token scale rs[t] and per-column scale cs[col] are applied first (rounded to bf16 as the
// row-wise GEMM's output would be), and the v heads are written back scaled as well.
template <bool FP8, bool SC = false>
__global__ __launch_bounds__(256) void rope_cache_write_kernel(bf16_t* __restrict__ qkv,
                                                               const int* __restrict__ positions,
                                                               const int* __restrict__ slots,
                                                               const float* __restrict__ cosT,
                                                               const float* __restrict__ sinT,
                                                               void* __restrict__ k_cache,
                                                               void* __restrict__ v_cache, int T,
                                                               int H, int KVH, float inv_ks, float inv_vs,
                                                               const float* __restrict__ rs = nullptr,
                                                               const float* __restrict__ cs = nullptr) {
  constexpr int half = HDIM / 2, cph = half / 8;  // 8 chunks of 8 pairs per head
  const int NH = H + 2 * KVH;
  const size_t total = (size_t)T * NH * cph;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int t = (int)(i / ((size_t)NH * cph));
    const int rem = (int)(i % ((size_t)NH * cph));
    const int head = rem / cph, c = rem % cph;
    bf16_t* row = qkv + (size_t)t * NH * HDIM + (size_t)head * HDIM;
    us8 a = *reinterpret_cast<const us8*>(row + c * 8);
    us8 b = *reinterpret_cast<const us8*>(row + half + c * 8);
    if constexpr (SC) {
      const float r = rs[t];
      const float* cc = cs + (size_t)head * HDIM + c * 8;
      const f4 ca0 = *reinterpret_cast<const f4*>(cc), ca1 = *reinterpret_cast<const f4*>(cc + 4);
      const f4 cb0 = *reinterpret_cast<const f4*>(cc + half), cb1 = *reinterpret_cast<const f4*>(cc + half + 4);
      float xa[8], xb[8];
      unpack8(a, xa);
      unpack8(b, xb);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        xa[k] = bf2f(f2bf(xa[k] * r * ca0[k]));
        xa[4 + k] = bf2f(f2bf(xa[4 + k] * r * ca1[k]));
        xb[k] = bf2f(f2bf(xb[k] * r * cb0[k]));
        xb[4 + k] = bf2f(f2bf(xb[4 + k] * r * cb1[k]));
      }
      a = pack8(xa);
      b = pack8(xb);
      if (head >= H + KVH) {  // v heads: the scaled values back in place (q / k: after the rotation)
        *reinterpret_cast<us8*>(row + c * 8) = a;
        *reinterpret_cast<us8*>(row + half + c * 8) = b;
      }
    }
    if (head < H + KVH) {  // q and k heads rotate
      const int pos = positions[t];
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
        o1[k] = x1[k] * cs[k] - x2[k] * sn[k];
        o2[k] = x2[k] * cs[k] + x1[k] * sn[k];
      }
      a = pack8(o1);
      b = pack8(o2);
      *reinterpret_cast<us8*>(row + c * 8) = a;
      *reinterpret_cast<us8*>(row + half + c * 8) = b;
    }
    const int slot = slots[t];
    if (head < H || slot < 0) continue;
    const int page = slot / PAGE, off = slot % PAGE;
    if constexpr (FP8) {
      typedef unsigned int u2 __attribute__((ext_vector_type(2)));
      if (head < H + KVH) {
        unsigned char* dst = (unsigned char*)k_cache + (((size_t)page * KVH + (head - H)) * PAGE + off) * HDIM;
        float x[8], y[8];
        unpack8(a, x);
        unpack8(b, y);
        u2 wa, wb;
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          int w = __builtin_amdgcn_cvt_pk_fp8_f32(__builtin_amdgcn_fmed3f(x[4 * h2] * inv_ks, 448.f, -448.f),
                                                  __builtin_amdgcn_fmed3f(x[4 * h2 + 1] * inv_ks, 448.f, -448.f), 0,
                                                  false);
          wa[h2] = __builtin_amdgcn_cvt_pk_fp8_f32(__builtin_amdgcn_fmed3f(x[4 * h2 + 2] * inv_ks, 448.f, -448.f),
                                                   __builtin_amdgcn_fmed3f(x[4 * h2 + 3] * inv_ks, 448.f, -448.f), w,
                                                   true);
          w = __builtin_amdgcn_cvt_pk_fp8_f32(__builtin_amdgcn_fmed3f(y[4 * h2] * inv_ks, 448.f, -448.f),
                                              __builtin_amdgcn_fmed3f(y[4 * h2 + 1] * inv_ks, 448.f, -448.f), 0,
                                              false);
          wb[h2] = __builtin_amdgcn_cvt_pk_fp8_f32(__builtin_amdgcn_fmed3f(y[4 * h2 + 2] * inv_ks, 448.f, -448.f),
                                                   __builtin_amdgcn_fmed3f(y[4 * h2 + 3] * inv_ks, 448.f, -448.f), w,
                                                   true);
        }
        *reinterpret_cast<u2*>(dst + c * 8) = wa;
        *reinterpret_cast<u2*>(dst + half + c * 8) = wb;
      } else {
        unsigned char* dst =
            (unsigned char*)v_cache + ((size_t)page * KVH + (head - H - KVH)) * HDIM * PAGE + off;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          dst[(size_t)(c * 8 + k) * PAGE] = to_fp8(bf2f(a[k]) * inv_vs);
          dst[(size_t)(half + c * 8 + k) * PAGE] = to_fp8(bf2f(b[k]) * inv_vs);
        }
      }
    } else if (head < H + KVH) {
      bf16_t* dst = (bf16_t*)k_cache + (((size_t)page * KVH + (head - H)) * PAGE + off) * HDIM;
      *reinterpret_cast<us8*>(dst + c * 8) = a;
      *reinterpret_cast<us8*>(dst + half + c * 8) = b;
    } else {
      bf16_t* dst = (bf16_t*)v_cache + ((size_t)page * KVH + (head - H - KVH)) * HDIM * PAGE + off;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        dst[(size_t)(c * 8 + k) * PAGE] = a[k];
        dst[(size_t)(half + c * 8 + k) * PAGE] = b[k];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Paged decode attention.  One wave = (batch row b, kv head, split).  q row b is at q + b*q_stride
// with its H heads contiguous (128 elements each): the fused qkv output is read in place.
// G = query heads per KV head (1..16).  Output: DIRECT -> out[b][h*128 + d] bf16 (one split);
// otherwise o_part[b][h][split][128] fp32 (normalised) + lse_part[b][h][split] (log2 domain).
// ------------------------------------------------------------------------------------------------
// FP8: e4m3 cache (half the bytes of the HBM-bound page stream), converted to the same bf16
// operands in registers; k_scale is folded into scale_log2 by the host, v_scale into the output.
template <bool DIRECT, bool FP8>
__global__ __launch_bounds__(64) void paged_decode_kernel(
    const bf16_t* __restrict__ q, long q_stride, const void* __restrict__ k_cache,
    const void* __restrict__ v_cache, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ ctx_lens, bf16_t* __restrict__ out, float* __restrict__ o_part,
    float* __restrict__ lse_part, int H, int KVH, int G, int nsplit, int pages_per_split,
    float scale_log2, float v_scale) {
  // grid (B * KVH, nsplit): consecutive workgroups are different (sequence, KV head) pairs of the
  // SAME split, so the populated splits are dealt round-robin over all 8 XCDs.  (With the split
  // as the fastest index, split s landed on XCD s % 8: at 8 splits and short contexts every
  // populated wave ran on one XCD, 5.5x slower, tools/bench_paged_decode.py.)
  const int kvh = blockIdx.x % KVH, b = blockIdx.x / KVH, split = blockIdx.y;
  const int lane = threadIdx.x, qc = lane & 15, g = lane >> 4;
  const int ctx = ctx_lens[b];
  const int n_pages = (ctx + PAGE - 1) / PAGE;
  const int p0 = split * pages_per_split;
  const int p1 = min(p0 + pages_per_split, n_pages);
  const int h = kvh * G + qc;
  const bool qvalid = qc < G;

  float m = -INFINITY, l = 0.f;
  f32x4_t acc[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) acc[n] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  if (p0 < p1) {
    // Q^T operand: lane (qc, g) holds q[h][32kk + 8g .. +8] for k-step kk
    bf16x8_t qf[4];
    const bf16_t* qrow = q + (long)b * q_stride + (long)(qvalid ? h : kvh * G) * HDIM;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      qf[kk] = ld8(qrow + 32 * kk + 8 * g);
      if (!qvalid) qf[kk] = bf16x8_t{};
    }
    const int* bt = block_tables + (long)b * bt_stride;
    const int r = lane & 15;
    // K row offsets of the 4 S^T tiles (key 32(t>>1) + 8(r>>2) + 4(t&1) + (r&3)) and the V^T
    // fragment offset are lane constants; one page = 16 K + 16 V 16-byte loads per lane.
    // Two-stage software pipeline, pinned with sched_barrier (left alone, hipcc interleaved
    // load -> wait -> MFMA with <= 3 loads in flight, which made the kernel latency-bound at
    // ~1.8 TB/s): V(p) is in flight during S(p) = K(p) Q^T, and K(p+1) during softmax + P V(p).
    int koff[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) koff[t] = (32 * (t >> 1) + 8 * (r >> 2) + 4 * (t & 1) + (r & 3)) * HDIM + 8 * g;
    const int voff = r * PAGE + 8 * g;
    // operands in flight: bf16x8 (16 B) per lane, or the raw 8 e4m3 bytes of an fp8 cache
    using OpT = typename std::conditional<FP8, u2_t, bf16x8_t>::type;
    OpT kf[4][4], vf[2][8];
    auto op = [](const OpT& v) -> bf16x8_t {
      if constexpr (FP8)
        return fp8x8_to_bf16(v);
      else
        return v;
    };
    auto load_k = [&](long page) {
      if constexpr (FP8) {
        const unsigned char* kb = (const unsigned char*)k_cache + (page * KVH + kvh) * (long)(PAGE * HDIM);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) kf[t][kk] = *reinterpret_cast<const u2_t*>(kb + koff[t] + 32 * kk);
      } else {
        const bf16_t* kb = (const bf16_t*)k_cache + (page * KVH + kvh) * (long)(PAGE * HDIM);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) kf[t][kk] = ld8(kb + koff[t] + 32 * kk);
      }
    };
    auto load_v = [&](long page) {
      if constexpr (FP8) {
        const unsigned char* vb = (const unsigned char*)v_cache + (page * KVH + kvh) * (long)(PAGE * HDIM);
#pragma unroll
        for (int mm = 0; mm < 2; ++mm)
#pragma unroll
          for (int n = 0; n < 8; ++n) vf[mm][n] = *reinterpret_cast<const u2_t*>(vb + voff + 16 * n * PAGE + 32 * mm);
      } else {
        const bf16_t* vb = (const bf16_t*)v_cache + (page * KVH + kvh) * (long)(PAGE * HDIM);
#pragma unroll
        for (int mm = 0; mm < 2; ++mm)
#pragma unroll
          for (int n = 0; n < 8; ++n) vf[mm][n] = ld8(vb + voff + 16 * n * PAGE + 32 * mm);
      }
    };
    long page = bt[p0];
    load_k(page);
    for (int p = p0; p < p1; ++p) {
      const long next = p + 1 < p1 ? bt[p + 1] : page;
      load_v(page);
      __builtin_amdgcn_sched_barrier(0);
      // S^T tiles: lane holds keys 32(t>>1) + 8g + 4(t&1) + i, i = 0..3, of query qc
      f32x4_t s[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        s[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) s[t] = mfma16(op(kf[t][kk]), qf[kk], s[t]);
      }
      __builtin_amdgcn_sched_barrier(0);
      load_k(next);  // unconditional (last page: a redundant reload) so vmcnt counting stays static
      __builtin_amdgcn_sched_barrier(0);
      page = next;
      const int base = p * PAGE;
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = base + 32 * (t >> 1) + 8 * g + 4 * (t & 1) + i;
          const float v = key < ctx ? s[t][i] * scale_log2 : -INFINITY;
          s[t][i] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m, mx);
      const float alpha = fexp2(m - mn);
      m = mn;
      float ls = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float e = fexp2(s[t][i] - mn);
          s[t][i] = e;
          ls += e;
        }
      l = l * alpha + ls;
#pragma unroll
      for (int n = 0; n < 8; ++n) acc[n] *= alpha;
      // P^T operand of PV step mm: element j of lane group g = key 32mm + 8g + j
#pragma unroll
      for (int mm = 0; mm < 2; ++mm) {
        bf16x8_t pf;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          pf[i] = (__bf16)s[2 * mm][i];
          pf[4 + i] = (__bf16)s[2 * mm + 1][i];
        }
#pragma unroll
        for (int n = 0; n < 8; ++n) acc[n] = mfma16(op(vf[mm][n]), pf, acc[n]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // O^T accumulator: lane (qc, g) holds O[h][16n + 4g + i]
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  if (!qvalid) return;
  const float inv = l > 0.f ? v_scale / l : 0.f;
  if (DIRECT) {
    bf16_t* o = out + (long)b * H * HDIM + (long)h * HDIM;
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      typedef unsigned short us4 __attribute__((ext_vector_type(4)));
      us4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = f2bf(acc[n][i] * inv);
      *reinterpret_cast<us4*>(o + 16 * n + 4 * g) = v;
    }
  } else {
    const long idx = ((long)b * H + h) * nsplit + split;
    if (g == 0) lse_part[idx] = l > 0.f ? m + __log2f(l) : -INFINITY;
    if (l > 0.f) {  // an empty split writes only its -inf lse; the combine never reads its o
      float* o = o_part + idx * HDIM;
#pragma unroll
      for (int n = 0; n < 8; ++n) *reinterpret_cast<f32x4_t*>(o + 16 * n + 4 * g) = acc[n] * inv;
    }
  }
}

// merge the split partials: out[b][h*128 + d] = sum_s 2^(lse_s - M) o_s / sum_s 2^(lse_s - M)
// One 256-thread workgroup per (b, h): 8 groups of 32 lanes take every 8th split, a lane owns 4
// d values (one 16-byte load of a 512-byte partial row per split), and the groups meet in LDS.
// (The first form walked all splits serially with one thread per d: at batch 1 and 32k context,
// ~256 splits, it was latency-bound at 85 us per layer -- 6.8 ms of a 33 ms 70B decode step,
// profiles/decode_batch1_32k_r2p.txt.)
__global__ __launch_bounds__(256) void paged_combine_kernel(const float* __restrict__ o_part,
                                                            const float* __restrict__ lse_part,
                                                            bf16_t* __restrict__ out, int H,
                                                            int nsplit) {
  __shared__ float red_max[4];
  __shared__ float red_den[8];
  __shared__ f4 red_num[8][32];
  const long bh = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = tid >> 5, l32 = tid & 31;
  const float* lse = lse_part + bh * nsplit;
  float M = -INFINITY;
  for (int s = tid; s < nsplit; s += 256) M = fmaxf(M, lse[s]);
  M = wave_max(M);
  if (lane == 0) red_max[wave] = M;
  __syncthreads();
  M = fmaxf(fmaxf(red_max[0], red_max[1]), fmaxf(red_max[2], red_max[3]));
  f4 num = {0.f, 0.f, 0.f, 0.f};
  float den = 0.f;
  if (M > -INFINITY) {
    const f4* op = reinterpret_cast<const f4*>(o_part + bh * (long)nsplit * HDIM) + l32;
#pragma unroll 4
    for (int s = g; s < nsplit; s += 8) {
      const float ls = lse[s];
      if (ls == -INFINITY) continue;  // empty split: its o row was never written (0 * garbage = NaN)
      const float w = fexp2(ls - M);
      const f4 o = op[(long)s * (HDIM / 4)];
      num += w * o;
      den += w;
    }
  }
  red_num[g][l32] = num;
  if (l32 == 0) red_den[g] = den;
  __syncthreads();
  if (tid < 32) {
    f4 n = red_num[0][tid];
    float dsum = red_den[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) {
      n += red_num[k][tid];
      dsum += red_den[k];
    }
    const float inv = dsum > 0.f ? 1.f / dsum : 0.f;
    typedef unsigned short us4 __attribute__((ext_vector_type(4)));
    us4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = f2bf(n[i] * inv);
    *reinterpret_cast<us4*>(out + bh * HDIM + 4 * tid) = v;
  }
}

// ------------------------------------------------------------------------------------------------
// Sampling: one workgroup per row of logits [rows][V] (bf16, row stride `stride`).
// temperature <= 0 -> greedy argmax; otherwise Gumbel-max over logits / T (exactly a draw from
// softmax(logits / T)) with a counter-based hash of (seed, step, index).  Also returns the chosen
// token's log-probability under softmax(logits / T) (greedy: T = 1), from an online max/sum in the
// same pass.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void sample_kernel(const bf16_t* __restrict__ logits, long stride,
                                                     int V, const float* __restrict__ temps,
                                                     const int64_t* __restrict__ seeds,
                                                     const int* __restrict__ steps,
                                                     int* __restrict__ tokens,
                                                     float* __restrict__ logprobs) {
  const int row = blockIdx.x, tid = threadIdx.x;
  const bf16_t* x = logits + (long)row * stride;
  const float T = temps[row];
  const bool greedy = !(T > 0.f);
  const float invT = greedy ? 1.f : 1.f / T;
  const uint64_t key = mix64((uint64_t)seeds[row] * 0x9e3779b97f4a7c15ULL + (uint64_t)steps[row]);
  float best = -INFINITY, mx = -INFINITY, sum = 0.f, bestx = -INFINITY;
  int bi = 0x7fffffff;
  for (int i0 = tid * 8; i0 < V; i0 += 256 * 8) {
    float v[8];
    if (i0 + 8 <= V && (stride % 8) == 0) {
      unpack8(*reinterpret_cast<const us8*>(x + i0), v);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = i0 + k < V ? bf2f(x[i0 + k]) : -INFINITY;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = i0 + k;
      if (i >= V) break;
      const float z = v[k] * invT;
      if (z == -INFINITY) continue;  // masked logit (e.g. a banned token)
      // online log-sum-exp of z
      if (z > mx) {
        sum = sum * __expf(mx - z) + 1.f;
        mx = z;
      } else {
        sum += __expf(z - mx);
      }
      float score = z;
      if (!greedy) {
        const uint64_t hsh = mix64(key ^ ((uint64_t)i * 0xd1b54a32d192ed03ULL));
        const float u = ((float)(hsh >> 40) + 0.5f) * (1.0f / 16777216.0f);
        score = z - __logf(-__logf(u));
      }
      if (score > best || (score == best && i < bi)) {
        best = score;
        bi = i;
        bestx = z;
      }
    }
  }
  // wave reduction of (best, bi, bestx) and (mx, sum)
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    const float ox = __shfl_xor(bestx, o, 64);
    if (ob > best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
      bestx = ox;
    }
    const float om = __shfl_xor(mx, o, 64), os = __shfl_xor(sum, o, 64);
    const float nm = fmaxf(mx, om);
    sum = (mx > -INFINITY ? sum * __expf(mx - nm) : 0.f) + (om > -INFINITY ? os * __expf(om - nm) : 0.f);
    mx = nm;
  }
  __shared__ float sb[4], sx[4], sm[4], ss[4];
  __shared__ int si[4];
  const int w = tid >> 6;
  if ((tid & 63) == 0) {
    sb[w] = best;
    si[w] = bi;
    sx[w] = bestx;
    sm[w] = mx;
    ss[w] = sum;
  }
  __syncthreads();
  if (tid == 0) {
    for (int k = 1; k < 4; ++k) {
      if (sb[k] > best || (sb[k] == best && si[k] < bi)) {
        best = sb[k];
        bi = si[k];
        bestx = sx[k];
      }
      const float nm = fmaxf(mx, sm[k]);
      sum = (mx > -INFINITY ? sum * __expf(mx - nm) : 0.f) + (sm[k] > -INFINITY ? ss[k] * __expf(sm[k] - nm) : 0.f);
      mx = nm;
    }
    tokens[row] = bi;
    if (logprobs) logprobs[row] = bestx - (mx + __logf(sum));
  }
}

// ------------------------------------------------------------------------------------------------
extern "C" int dsa_paged_page_size() { return PAGE; }

extern "C" hipError_t dsa_rope_cache_write(void* qkv, const int* positions, const int* slots,
                                           const float* cosT, const float* sinT, void* k_cache,
                                           void* v_cache, int T, int H, int KVH, int fp8, float k_scale,
                                           float v_scale, const float* rs, const float* cs, hipStream_t st) {
  if (T <= 0) return hipSuccess;
  if ((rs == nullptr) != (cs == nullptr)) return hipErrorInvalidValue;
  const size_t work = (size_t)T * (H + 2 * KVH) * (HDIM / 16);
  size_t grid = (work + 255) / 256;
  if (grid > 65535 * 4) grid = 65535 * 4;
  if (rs && fp8)
    rope_cache_write_kernel<true, true><<<(unsigned)grid, 256, 0, st>>>(
        (bf16_t*)qkv, positions, slots, cosT, sinT, k_cache, v_cache, T, H, KVH, 1.f / k_scale, 1.f / v_scale, rs, cs);
  else if (rs)
    rope_cache_write_kernel<false, true><<<(unsigned)grid, 256, 0, st>>>(
        (bf16_t*)qkv, positions, slots, cosT, sinT, k_cache, v_cache, T, H, KVH, 1.f, 1.f, rs, cs);
  else if (fp8)
    rope_cache_write_kernel<true><<<(unsigned)grid, 256, 0, st>>>((bf16_t*)qkv, positions, slots, cosT, sinT,
                                                                  k_cache, v_cache, T, H, KVH, 1.f / k_scale,
                                                                  1.f / v_scale);
  else
    rope_cache_write_kernel<false><<<(unsigned)grid, 256, 0, st>>>((bf16_t*)qkv, positions, slots, cosT, sinT,
                                                                   k_cache, v_cache, T, H, KVH, 1.f, 1.f);
  return hipGetLastError();
}

extern "C" hipError_t dsa_paged_decode(const void* q, long q_stride, const void* k_cache,
                                       const void* v_cache, const int* block_tables, int bt_stride,
                                       const int* ctx_lens, void* out, float* o_part,
                                       float* lse_part, int B, int H, int KVH, int nsplit,
                                       int pages_per_split, float scale, int fp8, float k_scale,
                                       float v_scale, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (KVH <= 0 || H % KVH || H / KVH > 16 || nsplit < 1 || pages_per_split < 1) return hipErrorInvalidValue;
  const int G = H / KVH;
  const float sl2 = scale * 1.4426950408889634f * (fp8 ? k_scale : 1.f);
  const float vs = fp8 ? v_scale : 1.f;
  const dim3 grid(B * KVH, nsplit);
#define DSA_PAGED(D, F8)                                                                               \
  paged_decode_kernel<D, F8><<<grid, 64, 0, st>>>((const bf16_t*)q, q_stride, k_cache, v_cache, block_tables, \
                                                  bt_stride, ctx_lens, D ? (bf16_t*)out : nullptr,             \
                                                  D ? nullptr : o_part, D ? nullptr : lse_part, H, KVH, G,     \
                                                  nsplit, pages_per_split, sl2, vs)
  if (nsplit == 1) {
    if (fp8) DSA_PAGED(true, true); else DSA_PAGED(true, false);
    return hipGetLastError();
  }
  if (fp8) DSA_PAGED(false, true); else DSA_PAGED(false, false);
#undef DSA_PAGED
  DSA_CHECK(hipGetLastError());
  paged_combine_kernel<<<B * H, 256, 0, st>>>(o_part, lse_part, (bf16_t*)out, H, nsplit);
  return hipGetLastError();
}

extern "C" hipError_t dsa_sample(const void* logits, long stride, int rows, int V, const float* temps,
                                 const int64_t* seeds, const int* steps, int* tokens, float* logprobs,
                                 hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  sample_kernel<<<rows, 256, 0, st>>>((const bf16_t*)logits, stride, V, temps, seeds, steps, tokens,
                                      logprobs);
  return hipGetLastError();
}
