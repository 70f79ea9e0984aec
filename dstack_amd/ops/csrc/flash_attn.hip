// Causal GQA flash attention (forward + backward) for CDNA4 / gfx950, head_dim 128, bf16.
//
// Layout: the kernels read q, k and v straight out of the fused projection output
// qkv[B, S, (H + 2*KVH) * 128] (row stride = (H + 2*KVH)*128 elements), so the model never
// transposes or splits qkv.  Output o is [B, S, H*128]; lse/delta are fp32 [B, H, S] in the log2
// domain of the scaled scores.
//
// Structure (one workgroup = 4 waves, each wave owns 32 rows of the 32x32x16 bf16 MFMA):
//  * K/V (and Q/dO in the dK/dV pass) tiles are staged HBM -> LDS by global_load_lds (LDS-DMA,
//    16 B/lane, no staging VGPRs) into a 2-deep ring; the next tile's DMA is in flight while the
//    current tile computes, one barrier per tile.
//  * LDS image: 256-byte rows with a 16-byte-chunk XOR  ch ^ (((row&3)<<2)|((row>>2)&3)) — conflict-
//    free both for ds_read_b128 row reads (MFMA operands with d contiguous) and for
//    ds_read_b64_tr_b16 transposed reads (operands with the key/query index contiguous).  LDS-DMA
//    writes lane-linearly, so the swizzle is applied to the per-lane SOURCE address.
//  * "key on the row" orientation: forward computes S^T = K·Q^T so a lane owns one query and the
//    softmax row max / sum are in-register (+1 xor-32 shuffle); the S^T accumulator is directly the
//    B operand of O^T += V^T·P^T (no LDS round trip for P).  The backward dK/dV pass uses
//    "key on the lane" (S = Q·K^T) so P and dS feed dV^T/dK^T directly; the dQ pass uses the
//    forward orientation and feeds dS^T as the A operand of dQ = dS·K.  dQ is computed by its own
//    q-major pass instead of cross-workgroup atomics (deterministic, no atomic-rate floor).
#include "mfma_tiles.h"
typedef unsigned short us4 __attribute__((ext_vector_type(4)));

#include <cstdlib>
#include <mutex>
#include <string>

using namespace dsa;

namespace {

constexpr int HD = 128;          // head dim
#ifndef DKDV_WAVES_PER_SIMD
#define DKDV_WAVES_PER_SIMD 1  // dK/dV + K/V fragments need ~300 registers: 1 wave/SIMD, no spills
#endif

}  // namespace

// ================================================================================================
// Forward
// ================================================================================================
// NW waves per workgroup, 32 query rows each (QB = 32 * NW rows per workgroup); every wave of the
// workgroup shares the K/V tiles.  NW = 4 (2 workgroups per CU) or 8 (1 per CU: half the K/V
// LDS-DMA traffic per query row; the default when S % 256 == 0).
// PF: the S^T = K·Q^T phase keeps 4 K-fragment reads in flight and alternates the two accumulator
// chains, instead of one read -> lgkmcnt(0) -> MFMA per step (which exposes the LDS latency on
// every MFMA of the phase): 0.702 vs 0.713 ms at S=8192 over three interleaved same-box runs
// (tools/gpu_sessions/run_r1ze.sh); DSTACK_AMD_FA_FWD_PF=0 selects the old form.
// PRIO (A/B, DSTACK_AMD_FA_PRIO): 0 = no priority games; 1 = a wave raises its issue priority
// (s_setprio) for its MFMA phases, so of the two waves on a SIMD the one with matrix work queues
// it first and the other's softmax VALU fills the gaps; 2 = the softmax phase gets the priority.
// Measured (3 interleaved runs, S=8192, profiles/fa_prio_ab_r4r.txt): 0 = 0.641-0.650 ms,
// 1 = 0.659-0.665, 2 = 0.657-0.658 -- both slower, kept opt-in only.
// STAG (A/B, DSTACK_AMD_FA_FWD_STAG=1; NW = 8): the two waves sharing a SIMD (w and w + 4) run the
// same per-tile program in lockstep -- both in S = K·Q^T, then both in the softmax VALU while the
// matrix pipe idles, then both in P·V.  With STAG the second half (w >= 4) defers each tile's P·V
// into the next iteration, ahead of its own S: one wave's softmax then runs beside the other's
// MFMAs.  V of the previous tile must outlive one more iteration, so the K/V ring is 3 deep
// (96 KiB of LDS); the deferred P (4 x bf16x8) is carried in registers across the barrier.
// Measured (3 interleaved runs, S=8192, profiles/fa_stag_ab_r4x.txt): 0.750-0.757 ms vs 0.664-0.673
// for the lockstep default, identical outputs -- slower, kept opt-in only.  With one barrier per
// tile the two halves still meet every tile, so the deferred P·V lands on the partner's S phase
// (matrix beside matrix on one SIMD) instead of beside its softmax.
// PRIO 3 (DSTACK_AMD_FA_HALF_PRIO=1, also for the 8-wave dK/dV and dQ passes): one s_setprio 1 for
// waves 4-7 at kernel start, no per-phase flips.  Measured (4 interleaved runs, S=8192,
// profiles/fa_hprio_ab_r4y.txt): forward 0.656-0.670 vs 0.657-0.668 ms, backward 2.018-2.036 vs
// 2.009-2.053 ms -- within noise, kept opt-in.
// BUF (default; DSTACK_AMD_FA_FWD_BUF=0 turns it off): K/V tiles through buffer descriptors (dma_tile64_buf), which keeps
// the S phase's LDS-read waits counted instead of lgkmcnt(0).
template <bool CAUSAL, int NW = 4, bool PF = true, int PRIO = 0, bool STAG = false, bool BUF = false, int FPD = 4>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void fa_fwd_kernel(const bf16_t* __restrict__ qkv,
                                                        bf16_t* __restrict__ out,
                                                        float* __restrict__ lse, int B, int S,
                                                        int H, int KVH, float scale_log2, float thr) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int QB = 32 * NW;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hf = lane >> 5, l32 = lane & 31;
  const int NH = H + 2 * KVH;
  const long rs = (long)NH * HD;  // row stride
  const int nqb = S / QB;
  const int bid = blockIdx.x;
  const int qb = CAUSAL ? nqb - 1 - bid / (B * H) : bid / (B * H);  // heaviest blocks first
  const int bh = bid % (B * H);
  const int b = bh / H, hh = bh % H, kvh = hh / (H / KVH);
  const bf16_t* base = qkv + (long)b * S * rs;
  const bf16_t* qp = base + hh * HD;
  const bf16_t* kp = base + (H + kvh) * HD;
  const bf16_t* vp = base + (H + KVH + kvh) * HD;
  const int q0 = qb * QB, qw0 = q0 + 32 * w, myq = qw0 + l32;
  // PRIO 3: static priority for the second-dispatched half (the arbitration loser of each SIMD pair)
  if constexpr (PRIO == 3) {
    if (w >= NW / 2) __builtin_amdgcn_s_setprio(1);
  }

  bf16x8 qf[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
    qf[ks] = *reinterpret_cast<const bf16x8*>(qp + (long)myq * rs + 16 * ks + 8 * hf);

  f32x16 o[4];
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  float m = -INFINITY, lsum = 0.f;
  const int nkv = CAUSAL ? (q0 + QB) / 64 : S / 64;
  constexpr int NST = STAG ? 3 : 2;          // K/V ring depth
  const bool late = STAG && w >= NW / 2;     // wave-uniform: this wave defers its P·V by one tile
  bf16x8 pbp[4];                             // the deferred P of the previous tile (late waves)
  bool pend = false;

  const unsigned kvbytes = (unsigned)(((long)(S - 1) * rs + HD) * 2);
  const __amdgpu_buffer_rsrc_t krs = make_rsrc(kp, kvbytes), vrs = make_rsrc(vp, kvbytes);
  unsigned kvoff[16 / NW];
  dma_tile64_offsets<NW>(rs, w, lane, kvoff);
  auto issue = [&](int t, char* nk) {
    if constexpr (BUF) {
      dma_tile64_buf<NW>(krs, kvoff, (int)((long)t * 64 * rs * 2), nk, w);
      dma_tile64_buf<NW>(vrs, kvoff, (int)((long)t * 64 * rs * 2), nk + TILE_BYTES, w);
    } else {
      dma_tile64_n<NW>(kp + (long)t * 64 * rs, rs, nk, w, lane);
      dma_tile64_n<NW>(vp + (long)t * 64 * rs, rs, nk + TILE_BYTES, w, lane);
    }
  };
  issue(0, smem);
  wait_dma_and_barrier();

  int stg = 0;  // ring slot of tile it
  for (int it = 0; it < nkv; ++it) {
    const char* kl = smem + stg * 2 * TILE_BYTES;
    const char* vl = kl + TILE_BYTES;
    const int nstg = stg + 1 == NST ? 0 : stg + 1;
    if (it + 1 < nkv) issue(it + 1, smem + nstg * 2 * TILE_BYTES);
    if constexpr (STAG) {
      if (late && pend) {  // P·V of the previous tile, whose V is still in its ring slot
        const char* pv = smem + (stg == 0 ? NST - 1 : stg - 1) * 2 * TILE_BYTES + TILE_BYTES;
#pragma unroll
        for (int d = 0; d < 4; ++d)
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) o[d] = mfma(lds_tr(pv, 16 * s4, 32 * d, lane), pbp[s4], o[d]);
        pend = false;
      }
    }
    stg = nstg;
    const int kv0 = it * 64;
    if (!CAUSAL || kv0 <= qw0 + 31) {
      f32x16 st[2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) st[t][r] = 0.f;
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(3);
      if constexpr (PF) {
        // step i: key tile t = i & 1, k-slice ks = i >> 1; fragment i + 4 is read while i computes
        constexpr int PD = BUF ? FPD : 4;  // reads in flight
        bf16x8 kf[PD];
#pragma unroll
        for (int i = 0; i < PD; ++i) kf[i] = lds_row(kl, 32 * (i & 1) + l32, 2 * (i >> 1) + hf);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const bf16x8 a = kf[i % PD];
          if (i + PD < 16) kf[i % PD] = lds_row(kl, 32 * ((i + PD) & 1) + l32, 2 * ((i + PD) >> 1) + hf);
          st[i & 1] = mfma(a, qf[i >> 1], st[i & 1]);
        }
        // pin the interleave (the scheduler otherwise sinks each read below the MFMAs that free
        // its register, leaving one read pair in flight): PD reads, then (MFMA, read) x (16 - PD),
        // PD MFMAs
        __builtin_amdgcn_sched_group_barrier(0x100, PD, 0);
#pragma unroll
        for (int i = 0; i < 16 - PD; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, PD, 0);
      } else {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int ks = 0; ks < 8; ++ks) st[t] = mfma(lds_row(kl, 32 * t + l32, 2 * ks + hf), qf[ks], st[t]);
      }
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(0);
      if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(3);
      // only the tile(s) crossing this wave's diagonal need the causal mask (wave-uniform test)
      if (CAUSAL && kv0 + 63 > qw0) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = kv0 + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hf;
            if (key > myq) st[t][r] = -INFINITY;
          }
      }
      // max on the raw scores (scale > 0 commutes with max); p = 2^(s*scale - m) as one fma + exp
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, st[t][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * scale_log2;
      // deferred max: keep the running max until a tile exceeds it by more than thr (log2 units),
      // so P stays <= 2^thr and O / lsum are rescaled only on those tiles (thr = 0: exact max)
      const float mn = (mx > m + thr) ? mx : m;
      const float alpha = fexp2(m - mn);
      m = mn;
      float ps = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fexp2(fmaf(st[t][r], scale_log2, -mn));
          st[t][r] = p;
          ps += p;
        }
      lsum = lsum * alpha + ps;
      // rescale O only when some lane's running max moved (after the first tiles it rarely does)
      if (__any(alpha != 1.f)) {
#pragma unroll
        for (int d = 0; d < 4; ++d)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[d][r] *= alpha;
      }
      bf16x8 pb[4];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) pb[s4] = to_bf16x8(st[s4 >> 1], 8 * (s4 & 1));
      if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(0);
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(3);
      if (late) {
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) pbp[s4] = pb[s4];
        pend = true;
      } else {
#pragma unroll
        for (int d = 0; d < 4; ++d)
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) o[d] = mfma(lds_tr(vl, 16 * s4, 32 * d, lane), pb[s4], o[d]);
      }
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(0);
    }
    wait_dma_and_barrier();
  }
  if constexpr (STAG) {
    if (late && pend) {  // the last tile's deferred P·V (its V was the last DMA: complete, not overwritten)
      const char* pv = smem + (stg == 0 ? NST - 1 : stg - 1) * 2 * TILE_BYTES + TILE_BYTES;
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) o[d] = mfma(lds_tr(pv, 16 * s4, 32 * d, lane), pbp[s4], o[d]);
    }
  }

  lsum += __shfl_xor(lsum, 32, 64);
  const float inv = 1.f / lsum;
  bf16_t* op = out + ((long)b * S + myq) * H * HD + hh * HD;
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int dd = 32 * d + 8 * rr + 4 * hf;
      typedef unsigned short us4 __attribute__((ext_vector_type(4)));
      us4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = f2bf(o[d][4 * rr + i] * inv);
      *reinterpret_cast<us4*>(op + dd) = v;
    }
  if (hf == 0) lse[((long)b * H + hh) * S + myq] = m + log2f(lsum);
}

// ================================================================================================
// Backward preprocess: delta = rowsum(dO * O) (fp32, [B, H, S]); 16 lanes per (b, s, h) row.
// ================================================================================================
__global__ __launch_bounds__(256) void fa_bwd_delta_kernel(const bf16_t* __restrict__ o,
                                                           const bf16_t* __restrict__ dout,
                                                           float* __restrict__ delta, int B, int S,
                                                           int H) {
  const long row = (long)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int sub = threadIdx.x & 15;
  const long rows = (long)B * S * H;
  float acc = 0.f;
  if (row < rows) {
    float a[8], g[8];
    unpack8(*reinterpret_cast<const us8*>(o + row * HD + sub * 8), a);
    unpack8(*reinterpret_cast<const us8*>(dout + row * HD + sub * 8), g);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += a[i] * g[i];
  }
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (row < rows && sub == 0) {
    const long bs = row / H;
    const int hh = (int)(row % H);
    const long b = bs / S, s = bs % S;
    delta[(b * H + hh) * S + s] = acc;
  }
}

// Tiled delta: workgroup = 32 consecutive positions x 8 heads of one batch row.  Reads are 2 KiB
// contiguous per position (8 heads x 128 d); the [B, H, S] result is staged in LDS and written
// as full 128-byte lines per head.  The row-per-16-lanes kernel above scatters 4-byte stores
// with stride S, and adjacent positions land on different XCDs' L2s: partial-line write-backs
// made it 558 us at S=8192 (measured, r1f profile) for 134 MB of reads.
__global__ __launch_bounds__(256) void fa_bwd_delta_tiled_kernel(const bf16_t* __restrict__ o,
                                                                 const bf16_t* __restrict__ dout,
                                                                 float* __restrict__ delta, int B,
                                                                 int S, int H) {
  constexpr int ST = 32, HT = 8;
  __shared__ float red[HT][ST + 1];
  const int nht = H / HT, nst = S / ST;
  int bid = blockIdx.x;
  const int ht = bid % nht;
  bid /= nht;
  const int st = bid % nst, b = bid / nst;
  const int sub = threadIdx.x & 15, r = threadIdx.x >> 4;
  const long base = ((long)b * S + (long)st * ST) * H + ht * HT;
#pragma unroll 4
  for (int it = 0; it < ST * HT / 16; ++it) {
    const int idx = it * 16 + r;
    const int s = idx / HT, h = idx % HT;
    const long row = base + (long)s * H + h;
    float a[8], g[8];
    unpack8(*reinterpret_cast<const us8*>(o + row * HD + sub * 8), a);
    unpack8(*reinterpret_cast<const us8*>(dout + row * HD + sub * 8), g);
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += a[i] * g[i];
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (sub == 0) red[h][s] = acc;
  }
  __syncthreads();
  const int h = threadIdx.x / ST, s = threadIdx.x % ST;  // 256 threads = HT x ST outputs
  delta[((long)b * H + ht * HT + h) * S + (long)st * ST + s] = red[h][s];
}

// ================================================================================================
// Backward dK/dV pass: workgroup = 128 keys of one (b, q-head); wave w owns keys kb0 + 32w.
// Loops over 64-row q tiles from the diagonal to S; writes fp32 per-q-head partials
// dkp/dvp [B, S, H, 128] that fa_bwd_reduce_kv sums over the GQA group.
// ================================================================================================
template <bool CAUSAL, int NQS>
__global__ __launch_bounds__(256, DKDV_WAVES_PER_SIMD) void fa_bwd_dkdv_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, float* __restrict__ dkp, float* __restrict__ dvp, int B, int S,
    int H, int KVH, float scale_log2) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // a stage holds QT = 32*NQS query rows: Q (QT x 256 B) | dO (QT x 256 B) | lse (QT x 4) | delta
  constexpr int QT = 32 * NQS;
  constexpr int QB = QT * 256;
  constexpr int STAGE = 2 * QB + 8 * QT;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hf = lane >> 5, l32 = lane & 31;
  const int NH = H + 2 * KVH;
  const long rs = (long)NH * HD;
  const long ors = (long)H * HD;
  const int bid = blockIdx.x;
  const int kb = bid / (B * H);  // small kb = most q tiles: heaviest first
  const int bh = bid % (B * H);
  const int b = bh / H, hh = bh % H, kvh = hh / (H / KVH);
  const bf16_t* base = qkv + (long)b * S * rs;
  const bf16_t* qp = base + hh * HD;
  const bf16_t* kp = base + (H + kvh) * HD;
  const bf16_t* vp = base + (H + KVH + kvh) * HD;
  const bf16_t* dop = dout + (long)b * S * ors + hh * HD;
  const float* lp = lse + ((long)b * H + hh) * S;
  const float* dp = delta + ((long)b * H + hh) * S;
  const int kb0 = kb * 128, kw0 = kb0 + 32 * w, mykey = kw0 + l32;

  bf16x8 kf[8], vf[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
    kf[ks] = *reinterpret_cast<const bf16x8*>(kp + (long)mykey * rs + 16 * ks + 8 * hf);
    vf[ks] = *reinterpret_cast<const bf16x8*>(vp + (long)mykey * rs + 16 * ks + 8 * hf);
  }
  f32x16 dk[4], dv[4];
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dk[d][r] = 0.f;
      dv[d][r] = 0.f;
    }

  const int qt_begin = CAUSAL ? kb0 / QT : 0;
  const int nqt = S / QT;
  auto issue = [&](int qt, char* st) {
#pragma unroll
    for (int h64 = 0; h64 < QT / 64; ++h64) {
      dma_tile64(qp + ((long)qt * QT + 64 * h64) * rs, rs, st + h64 * TILE_BYTES, w, lane);
      dma_tile64(dop + ((long)qt * QT + 64 * h64) * ors, ors, st + QB + h64 * TILE_BYTES, w, lane);
      if (w == 0) dma_f32x64(lp + qt * QT + 64 * h64, st + 2 * QB + 256 * h64, lane);
      if (w == 1) dma_f32x64(dp + qt * QT + 64 * h64, st + 2 * QB + 4 * QT + 256 * h64, lane);
    }
  };
  issue(qt_begin, smem);
  wait_dma_and_barrier();

  for (int qt = qt_begin; qt < nqt; ++qt) {
    const int stage = (qt - qt_begin) & 1;
    const char* ql = smem + stage * STAGE;
    const char* dol = ql + QB;
    const float* ll = reinterpret_cast<const float*>(ql + 2 * QB);
    const float* dl = ll + QT;
    if (qt + 1 < nqt) issue(qt + 1, smem + (stage ^ 1) * STAGE);
    // One 32-query sub-tile at a time: S/dP MFMAs, exp + dS on the VALU, then dV/dK MFMAs.
    // (Straight-line pairs of sub-tiles were measured 10 % slower: at 256 VGPRs the longer live
    // ranges cost more LDS-latency hiding than the extra MFMA/VALU overlap gained.)
#pragma unroll
    for (int qs = 0; qs < NQS; ++qs) {
      const int qlo = qt * QT + 32 * qs;
      if (CAUSAL && qlo + 31 < kw0) continue;  // every query of this sub-tile precedes my keys
      f32x16 sc, dpv;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sc[r] = 0.f;
        dpv[r] = 0.f;
      }
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        sc = mfma(lds_row(ql, 32 * qs + l32, 2 * ks + hf), kf[ks], sc);
        dpv = mfma(lds_row(dol, 32 * qs + l32, 2 * ks + hf), vf[ks], dpv);
      }
      // rows of sc/dpv: q = qlo + (r&3) + 8*(r>>2) + 4*hf ; column (lane) = mykey
      const bool diag = CAUSAL && qlo < kw0 + 31;  // sub-tile straddles this wave's keys
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int qi = 32 * qs + 8 * rr + 4 * hf;
        const f4 L = *reinterpret_cast<const f4*>(ll + qi);
        const f4 Dl = *reinterpret_cast<const f4*>(dl + qi);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * rr + i;
          float pv = fexp2(fmaf(sc[r], scale_log2, -L[i]));
          if (diag && mykey > qt * QT + qi + i) pv = 0.f;
          sc[r] = pv;
          dpv[r] = pv * (dpv[r] - Dl[i]);
        }
      }
      bf16x8 pb[2], dsb[2];
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        pb[k2] = to_bf16x8(sc, 8 * k2);
        dsb[k2] = to_bf16x8(dpv, 8 * k2);
      }
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int k2 = 0; k2 < 2; ++k2) {
          dv[d] = mfma(lds_tr(dol, 32 * qs + 16 * k2, 32 * d, lane), pb[k2], dv[d]);
          dk[d] = mfma(lds_tr(ql, 32 * qs + 16 * k2, 32 * d, lane), dsb[k2], dk[d]);
        }
    }
    wait_dma_and_barrier();
  }
  // dk^T/dv^T accumulators: column (lane) = key, rows = d
  const float sm = scale_log2 * 0.6931471805599453f;  // softmax scale = scale_log2 * ln2
  float* dkr = dkp + (((long)b * S + mykey) * H + hh) * HD;
  float* dvr = dvp + (((long)b * S + mykey) * H + hh) * HD;
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int dd = 32 * d + 8 * rr + 4 * hf;
      *reinterpret_cast<f4*>(dkr + dd) =
          f4{dk[d][4 * rr] * sm, dk[d][4 * rr + 1] * sm, dk[d][4 * rr + 2] * sm, dk[d][4 * rr + 3] * sm};
      *reinterpret_cast<f4*>(dvr + dd) = f4{dv[d][4 * rr], dv[d][4 * rr + 1], dv[d][4 * rr + 2], dv[d][4 * rr + 3]};
    }
}

// ================================================================================================
// Backward dK/dV pass, 8-wave variant: workgroup = 128 keys of one (b, q-head), 512 threads.
// Wave w owns keys kb0 + 32*(w&3) and the (w>>2)-th 32-query half of every 64-query tile, so a
// key group's dK/dV is accumulated by two waves that are reduced through LDS at the end.  K and V
// of the block stay resident in LDS (B operands re-read per MFMA instead of living in 64 VGPRs),
// which brings a wave under 256 registers: 2 waves per SIMD hide each other's LDS/exp latency.
// LDS: K|V (64 KiB) + 2-stage Q/dO/lse/delta ring (65 KiB) = 129 KiB -> one workgroup per CU.
// ================================================================================================
// SPILL: also write dS^T (bf16, the same values that feed dK) to dsg = [B*H][S keys][S queries]
// for the recompute-free dQ pass below: a lane owns one key and 4 consecutive queries per register
// group, so it stores 8 bytes at a time (the [q][key] forms measured 1.40-1.53 ms for this pass
// with 2-byte stores), and the dQ pass DMAs row-major 64-key tiles and reads them transposed.
// GQA: one workgroup owns a key block of one KV head and walks the q tiles of every query head of
// its group (H / KVH heads) in turn, so dK/dV are summed over the group in the accumulators and
// written once as bf16 straight into dqkv -- no fp32 per-q-head partials in HBM (2 x B*S*H*128*4
// bytes written and read back) and no reduce kernel.  Grid: B * KVH * S/128 workgroups, each G
// times longer; K/V are staged into LDS once per block instead of once per query head.
// TR (diagnostic, DSTACK_AMD_FA_TRACE=1 through dsa_fa_dkdv_trace): waves 0 and 4 of workgroup 0
// stamp s_memtime at 5 points of q-tiles 8..11 (tile top, after S/dP, after the softmax / dS math,
// after dV/dK, after the tile barrier) into the buffer passed as `dsg` -- where a tile's cycles go
// PF (DSTACK_AMD_FA_DKDV_PF=1): the S/dP phase keeps the next step's two fragment reads in flight
// while the current MFMA runs (S and dP alternate, so consecutive MFMAs never share an accumulator),
// pinned with sched_group_barrier; without it the compiler serialises read -> lgkmcnt(0) -> MFMA
// for most of the 16 steps.
// P16 (DSTACK_AMD_FA_DKDV_BF16, default on): the per-query-head dK/dV partials go to HBM as bf16 (the
// layout flash-attention 2 uses for its GQA expansion: per-head bf16 partials, summed in fp32 by the
// group reduction), halving the 2 x B*S*H*128 partial bytes written here and read back by the reduce.
template <bool CAUSAL, bool SEED = false, bool HP = false, bool SPILL = false, bool GQA = false, bool TR = false,
          int PF = 0, bool P16 = false>
__global__ __launch_bounds__(512, 2) void fa_bwd_dkdv8_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, float* __restrict__ dkp, float* __restrict__ dvp, int B, int S,
    int H, int KVH, float scale_log2, bf16_t* __restrict__ dsg, bf16_t* __restrict__ dqkv = nullptr) {
  static_assert(!(GQA && SPILL), "the dS spill is per query head");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KV_BYTES = 2 * 128 * 256;            // K (128 rows) | V (128 rows)
  constexpr int STAGE = 2 * TILE_BYTES + 512;        // Q (64) | dO (64) | lse | delta
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hf = lane >> 5, l32 = lane & 31;
  const int g = w & 3, qh = w >> 2, w4 = w & 3;
  if constexpr (HP) {
    if (w >= 4) __builtin_amdgcn_s_setprio(1);
  }
  const int NH = H + 2 * KVH;
  const long rs = (long)NH * HD;
  const long ors = (long)H * HD;
  const int bid = blockIdx.x;
  const int G = H / KVH;
  const int nbh = GQA ? B * KVH : B * H;
  const int kb = bid / nbh;  // small kb = most q tiles: heaviest first
  const int bh = bid % nbh;  // (b, q head), or (b, kv head) with GQA
  const int b = bh / (GQA ? KVH : H);
  const int kvh = GQA ? bh % KVH : (bh % H) / G;
  const int h_first = GQA ? kvh * G : bh % H;  // the query head(s) this workgroup walks
  const int n_heads = GQA ? G : 1;
  int hh = h_first;
  const bf16_t* base = qkv + (long)b * S * rs;
  const bf16_t* kp = base + (H + kvh) * HD;
  const bf16_t* vp = base + (H + KVH + kvh) * HD;
  const int kb0 = kb * 128, kw0 = kb0 + 32 * g, mykey = kw0 + l32;
  char* kl = smem;
  char* vl = smem + 128 * 256;
  char* ring = smem + KV_BYTES;

  // K/V of the block: waves 0-3 stage K, waves 4-7 stage V (two 64-row halves each)
  {
    const bf16_t* src = qh == 0 ? kp : vp;
    char* dst = qh == 0 ? kl : vl;
    dma_tile64(src + (long)kb0 * rs, rs, dst, w4, lane);
    dma_tile64(src + (long)(kb0 + 64) * rs, rs, dst + TILE_BYTES, w4, lane);
  }
  f32x16 dk[4], dv[4];
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dk[d][r] = 0.f;
      dv[d][r] = 0.f;
    }
  const int qt_begin = CAUSAL ? kb0 / 64 : 0;
  const int nqt = S / 64;
  // GQA walks (query head of the group, q tile) pairs: the next head's first tile is prefetched
  // under the previous head's last one.  Without GQA this is the plain q-tile loop.
  const __amdgpu_buffer_rsrc_t lrs0 = make_rsrc(lse + ((long)b * H + h_first) * S, (unsigned)S * 4);
  const __amdgpu_buffer_rsrc_t drs0 = make_rsrc(delta + ((long)b * H + h_first) * S, (unsigned)S * 4);
  // PF: the Q / dO tiles come through one buffer descriptor per wave (Q for waves 0-3, dO for 4-7)
  // with 4 loop-invariant 32-bit per-lane offsets and the tile's row offset in an SGPR, instead of
  // 4 rematerialised 64-bit address pairs per tile (frees ~20 VGPRs for the read pipeline)
  const long tstride = qh == 0 ? rs : ors;
  const __amdgpu_buffer_rsrc_t trs =
      make_rsrc(qh == 0 ? base + h_first * HD : dout + (long)b * S * ors + h_first * HD,
                (unsigned)(((long)(S - 1) * tstride + HD) * 2));
  unsigned toff[4];
  dma_tile64_offsets<4>(tstride, w4, lane, toff);
  auto issue = [&](int h, int qt, char* st) {
    if constexpr (PF && !GQA)
      dma_tile64_buf<4>(trs, toff, (int)((long)qt * 64 * tstride * 2), st + qh * TILE_BYTES, w4);
    else if (qh == 0)
      dma_tile64(base + h * HD + (long)qt * 64 * rs, rs, st, w4, lane);
    else
      dma_tile64(dout + (long)b * S * ors + h * HD + (long)qt * 64 * ors, ors, st + TILE_BYTES, w4, lane);
    if constexpr (GQA) {
      if (w == 0)
        dma_f32x64_buf(make_rsrc(lse + ((long)b * H + h) * S, (unsigned)S * 4), qt * 64, st + 2 * TILE_BYTES, lane);
      if (w == 4)
        dma_f32x64_buf(make_rsrc(delta + ((long)b * H + h) * S, (unsigned)S * 4), qt * 64,
                       st + 2 * TILE_BYTES + 256, lane);
    } else {
      if (w == 0) dma_f32x64_buf(lrs0, qt * 64, st + 2 * TILE_BYTES, lane);
      if (w == 4) dma_f32x64_buf(drs0, qt * 64, st + 2 * TILE_BYTES + 256, lane);
    }
  };
  issue(h_first, qt_begin, ring);
  wait_dma_and_barrier();

  const int h_end = h_first + n_heads;
  int qt = qt_begin, stage = 0, tnum = 0;
  const bool tracer = TR && blockIdx.x == 0 && (w == 0 || w == 4);
  auto stamp = [&](int k) {
    if constexpr (TR) {
      if (tracer && tnum >= 8 && tnum < 12) {
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0)
          reinterpret_cast<unsigned long long*>(dsg)[(w >> 2) * 64 + (tnum - 8) * 5 + k] = t;
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  for (;;) {
    stamp(0);
    const char* ql = ring + stage * STAGE;
    const char* dol = ql + TILE_BYTES;
    const float* ll = reinterpret_cast<const float*>(ql + 2 * TILE_BYTES);
    const float* dl = ll + 64;
    int nqt_next = qt + 1, nh = hh;
    if (GQA && nqt_next == nqt) {
      nqt_next = qt_begin;
      ++nh;
    }
    const bool more = GQA ? nh < h_end : nqt_next < nqt;
    if (more) issue(nh, nqt_next, ring + (stage ^ 1) * STAGE);
    const int qlo = qt * 64 + 32 * qh;
    if (!CAUSAL || qlo + 31 >= kw0) {  // some query of my half-tile sees my keys
      f32x16 sc, dpv;
      // SEED: the row constants start the accumulators (S' = Q.K^T - lse/scale, dP' = dO.V^T -
      // delta), so p = exp2(scale * S') and dS = p * dP' need no per-element subtractions
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int qi = 32 * qh + 8 * rr + 4 * hf;
        f4 L = {0.f, 0.f, 0.f, 0.f}, Dl = {0.f, 0.f, 0.f, 0.f};
        if constexpr (SEED) {
          L = *reinterpret_cast<const f4*>(ll + qi);
          Dl = *reinterpret_cast<const f4*>(dl + qi);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          sc[4 * rr + i] = SEED ? -L[i] / scale_log2 : 0.f;
          dpv[4 * rr + i] = SEED ? -Dl[i] : 0.f;
        }
      }
      if constexpr (PF) {
        // step i: chain i & 1 (0 = S from Q.K^T, 1 = dP from dO.V^T), k-slice i >> 1
        auto rd_a = [&](int i) { return lds_row((i & 1) ? dol : ql, 32 * qh + l32, 2 * (i >> 1) + hf); };
        auto rd_b = [&](int i) { return lds_row((i & 1) ? vl : kl, 32 * g + l32, 2 * (i >> 1) + hf); };
        constexpr int NB = PF + 1;  // fragment buffers: PF steps in flight + the one computing
        bf16x8 fa[NB], fb[NB];
#pragma unroll
        for (int j = 0; j < PF; ++j) {
          fa[j] = rd_a(j);
          fb[j] = rd_b(j);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const bf16x8 a = fa[i % NB], bb = fb[i % NB];
          if (i + PF < 16) {
            fa[(i + PF) % NB] = rd_a(i + PF);
            fb[(i + PF) % NB] = rd_b(i + PF);
          }
          if (i & 1)
            dpv = mfma(a, bb, dpv);
          else
            sc = mfma(a, bb, sc);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * PF, 0);
#pragma unroll
        for (int i = 0; i < 16 - PF; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, PF, 0);
      } else {
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
          sc = mfma(lds_row(ql, 32 * qh + l32, 2 * ks + hf), lds_row(kl, 32 * g + l32, 2 * ks + hf), sc);
          dpv = mfma(lds_row(dol, 32 * qh + l32, 2 * ks + hf), lds_row(vl, 32 * g + l32, 2 * ks + hf), dpv);
        }
      }
      stamp(1);
      const bool diag = CAUSAL && qlo < kw0 + 31;
      // P, then (diagonal tiles only, a wave-uniform branch: 2 of ~64 tiles) the causal mask, then
      // dS.  Folding the mask into the P loop as a select costs every tile 16 v_cmp + 16 v_cndmask
      // + 16 s_and; the branch costs the other tiles nothing.
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        f4 L = {0.f, 0.f, 0.f, 0.f};
        if constexpr (!SEED) L = *reinterpret_cast<const f4*>(ll + 32 * qh + 8 * rr + 4 * hf);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          sc[4 * rr + i] = SEED ? fexp2(sc[4 * rr + i] * scale_log2) : fexp2(fmaf(sc[4 * rr + i], scale_log2, -L[i]));
      }
      if (__builtin_expect(diag, 0)) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (mykey > qt * 64 + 32 * qh + 8 * (r >> 2) + 4 * hf + (r & 3)) sc[r] = 0.f;
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        f4 Dl = {0.f, 0.f, 0.f, 0.f};
        if constexpr (!SEED) Dl = *reinterpret_cast<const f4*>(dl + 32 * qh + 8 * rr + 4 * hf);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * rr + i;
          dpv[r] = SEED ? sc[r] * dpv[r] : sc[r] * (dpv[r] - Dl[i]);
        }
      }
      bf16x8 pb[2], dsb[2];
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        pb[k2] = to_bf16x8(sc, 8 * k2);
        dsb[k2] = to_bf16x8(dpv, 8 * k2);
      }
      stamp(2);
      if constexpr (SPILL) {  // lane = key mykey, registers 4*rr+i = queries qlo + 8*rr + 4*hf + i
        bf16_t* dt = dsg + (((long)b * H + hh) * S + mykey) * S + qlo + 4 * hf;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          *reinterpret_cast<us4*>(dt + 8 * rr) =
              us4{f2bf(dpv[4 * rr]), f2bf(dpv[4 * rr + 1]), f2bf(dpv[4 * rr + 2]), f2bf(dpv[4 * rr + 3])};
      }
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int k2 = 0; k2 < 2; ++k2) {
          dv[d] = mfma(lds_tr(dol, 32 * qh + 16 * k2, 32 * d, lane), pb[k2], dv[d]);
          dk[d] = mfma(lds_tr(ql, 32 * qh + 16 * k2, 32 * d, lane), dsb[k2], dk[d]);
        }
    }
    stamp(3);
    wait_dma_and_barrier();
    stamp(4);
    ++tnum;
    if (!more) break;
    qt = nqt_next;
    hh = nh;
    stage ^= 1;
  }
  // reduce the two q-halves of every key group through LDS (the K/V + ring space is free now):
  // layout [g][dk|dv][d][r][lane] floats -> lane-contiguous, conflict-free
  float* red = reinterpret_cast<float*>(smem);
  if (qh == 1) {
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        red[(((g * 2 + 0) * 4 + d) * 16 + r) * 64 + lane] = dk[d][r];
        red[(((g * 2 + 1) * 4 + d) * 16 + r) * 64 + lane] = dv[d][r];
      }
  }
  __syncthreads();
  if (GQA && qh == 0) {  // the group's sum, bf16, straight into dqkv's K and V slots
    const float sm = scale_log2 * 0.6931471805599453f;
    bf16_t* dkr = dqkv + ((long)b * S + mykey) * NH * HD + (H + kvh) * HD;
    bf16_t* dvr = dkr + KVH * HD;
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int dd = 32 * d + 8 * rr + 4 * hf;
        float ok[4], ov[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * rr + i;
          ok[i] = (dk[d][r] + red[(((g * 2 + 0) * 4 + d) * 16 + r) * 64 + lane]) * sm;
          ov[i] = dv[d][r] + red[(((g * 2 + 1) * 4 + d) * 16 + r) * 64 + lane];
        }
        *reinterpret_cast<us4*>(dkr + dd) = us4{f2bf(ok[0]), f2bf(ok[1]), f2bf(ok[2]), f2bf(ok[3])};
        *reinterpret_cast<us4*>(dvr + dd) = us4{f2bf(ov[0]), f2bf(ov[1]), f2bf(ov[2]), f2bf(ov[3])};
      }
  } else if (qh == 0) {
    const float sm = scale_log2 * 0.6931471805599453f;  // softmax scale = scale_log2 * ln2
    const long row = (((long)b * S + mykey) * H + hh) * HD;
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int dd = 32 * d + 8 * rr + 4 * hf;
        f4 ok, ov;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * rr + i;
          ok[i] = (dk[d][r] + red[(((g * 2 + 0) * 4 + d) * 16 + r) * 64 + lane]) * sm;
          ov[i] = dv[d][r] + red[(((g * 2 + 1) * 4 + d) * 16 + r) * 64 + lane];
        }
        if constexpr (P16) {
          *reinterpret_cast<us4*>(reinterpret_cast<bf16_t*>(dkp) + row + dd) =
              us4{f2bf(ok[0]), f2bf(ok[1]), f2bf(ok[2]), f2bf(ok[3])};
          *reinterpret_cast<us4*>(reinterpret_cast<bf16_t*>(dvp) + row + dd) =
              us4{f2bf(ov[0]), f2bf(ov[1]), f2bf(ov[2]), f2bf(ov[3])};
        } else {
          *reinterpret_cast<f4*>(dkp + row + dd) = ok;
          *reinterpret_cast<f4*>(dvp + row + dd) = ov;
        }
      }
  }
}

// ================================================================================================
// Backward dK/dV pass, 8 waves with DECOUPLED halves (DSTACK_AMD_FA_DKDV_DEC=1).
// Same work split as fa_bwd_dkdv8_kernel (128 keys of one (b, q-head); wave w: keys kb0 + 32*(w&3),
// query half w>>2 of every 64-query tile), but the two 4-wave halves no longer meet at a workgroup
// barrier every tile.  A half reads only its own 32 query rows of Q / dO (and K / V, which are
// resident and read-only after the prologue), so each half now stages its own rows in a ring of its
// own (2 x [Q 32 rows | dO 32 rows | lse 64 | delta 64] per half) and closes a tile with a 4-wave
// rendezvous on an LDS counter (each wave: its DMA for the next tile landed and its reads of this
// one returned -> one lane's ds_add; then it polls until all four have added).  The phase trace of the
// barrier form (profiles/fa_dkdv_phases_r8s.txt) had both halves in the same phase at once -- the
// LDS-heavy S/dP reads together, the VALU-only softmax together (matrix pipe idle), and waves 0-3
// idle ~1,150 ticks per tile at the barrier waiting for waves 4-7.  Decoupled, a half that is ahead
// keeps going, and `stag` (s_sleep units of 64 clocks, DSTACK_AMD_FA_DKDV_STAG) starts waves 4-7
// that much later so the halves settle out of phase: one half's softmax beside the other's MFMAs.
// LDS: K|V 64 KiB + 4 x 16.5 KiB of rings + 2 counters = 130 KiB.  TR: the phase trace (see above).
// ================================================================================================
template <bool CAUSAL, bool TR = false, bool EARLY = false>
__global__ __launch_bounds__(512, 2) void fa_bwd_dkdv8d_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, float* __restrict__ dkp, float* __restrict__ dvp, int B, int S, int H,
    int KVH, float scale_log2, int stag, unsigned long long* __restrict__ trace) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KV_BYTES = 2 * 128 * 256;  // K (128 rows) | V (128 rows)
  constexpr int HT = 32 * 256;             // one half tile: 32 rows x 128 bf16
  constexpr int HSTAGE = 2 * HT + 512;     // Q half | dO half | lse (64) | delta (64)
  constexpr int PF = 2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hf = lane >> 5, l32 = lane & 31;
  const int g = w & 3, qh = w >> 2;
  const int NH = H + 2 * KVH;
  const long rs = (long)NH * HD;
  const long ors = (long)H * HD;
  const int bid = blockIdx.x;
  const int kb = bid / (B * H);  // small kb = most q tiles: heaviest first
  const int bh = bid % (B * H);
  const int b = bh / H, hh = bh % H, kvh = hh / (H / KVH);
  const bf16_t* base = qkv + (long)b * S * rs;
  const bf16_t* kp = base + (H + kvh) * HD;
  const bf16_t* vp = base + (H + KVH + kvh) * HD;
  const int kb0 = kb * 128, kw0 = kb0 + 32 * g, mykey = kw0 + l32;
  char* kl = smem;
  char* vl = smem + 128 * 256;
  char* ring = smem + KV_BYTES;  // [stage][half] HSTAGE each
  unsigned* cnt = reinterpret_cast<unsigned*>(ring + 4 * HSTAGE);
  {  // K/V of the block: waves 0-3 stage K, waves 4-7 stage V (two 64-row halves each)
    const bf16_t* src = qh == 0 ? kp : vp;
    char* dst = qh == 0 ? kl : vl;
    dma_tile64(src + (long)kb0 * rs, rs, dst, g, lane);
    dma_tile64(src + (long)(kb0 + 64) * rs, rs, dst + TILE_BYTES, g, lane);
  }
  if (tid < 2) cnt[tid] = 0u;
  f32x16 dk[4], dv[4];
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dk[d][r] = 0.f;
      dv[d][r] = 0.f;
    }
  const int qt_begin = CAUSAL ? kb0 / 64 : 0;
  const int nqt = S / 64;
  // this half's 32 rows of Q and dO through buffer descriptors: wave g DMAs rows 8g..8g+7 of each
  // (two 1 KiB pieces), per-lane offsets loop-invariant, the tile's row offset an SGPR
  const __amdgpu_buffer_rsrc_t qr = make_rsrc(base + hh * HD, (unsigned)(((long)(S - 1) * rs + HD) * 2));
  const __amdgpu_buffer_rsrc_t dr =
      make_rsrc(dout + (long)b * S * ors + hh * HD, (unsigned)(((long)(S - 1) * ors + HD) * 2));
  const __amdgpu_buffer_rsrc_t lr = make_rsrc(lse + (long)bh * S, (unsigned)S * 4);
  const __amdgpu_buffer_rsrc_t er = make_rsrc(delta + (long)bh * S, (unsigned)S * 4);
  unsigned qoff[2], doff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (2 * g + i) * 4 + (lane >> 4);
    const int ch = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
    qoff[i] = (unsigned)(((long)row * rs + ch * 8) * 2);
    doff[i] = (unsigned)(((long)row * ors + ch * 8) * 2);
  }
  auto issue = [&](int qt, char* st) {  // this half's rows of q tile qt -> its stage `st`
    const int r0 = qt * 64 + 32 * qh;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(qr, LDS3(void, st + (2 * g + i) * 1024), 16, qoff[i],
                                               __builtin_amdgcn_readfirstlane((int)((long)r0 * rs * 2)), 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(dr, LDS3(void, st + HT + (2 * g + i) * 1024), 16, doff[i],
                                               __builtin_amdgcn_readfirstlane((int)((long)r0 * ors * 2)), 0, 0);
    }
    if (g == 0) dma_f32x64_buf(lr, qt * 64, st + 2 * HT, lane);        // lse of the whole 64-row tile
    if (g == 1) dma_f32x64_buf(er, qt * 64, st + 2 * HT + 256, lane);  // delta
  };
  issue(qt_begin, ring + qh * HSTAGE);
  wait_dma_and_barrier();  // K/V, both halves' first tiles and the counters: the one full barrier
  if (qh == 1)
    for (int i = 0; i < stag; ++i) __builtin_amdgcn_s_sleep(1);
  const bool tracer = TR && blockIdx.x == 0 && (w == 0 || w == 4);
  int qt = qt_begin, stage = 0, tnum = 0;
  unsigned gen = 0;
  auto stamp = [&](int k) {
    if constexpr (TR) {
      if (tracer && tnum >= 8 && tnum < 12) {
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) trace[qh * 64 + (tnum - 8) * 5 + k] = t;
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  for (;;) {
    stamp(0);
    const char* ql = ring + (stage * 2 + qh) * HSTAGE;
    const char* dol = ql + HT;
    const float* ll = reinterpret_cast<const float*>(ql + 2 * HT) + 32 * qh;
    const float* dl = ll + 64;
    const bool more = qt + 1 < nqt;
    if (more) issue(qt + 1, ring + ((stage ^ 1) * 2 + qh) * HSTAGE);
    const int qlo = qt * 64 + 32 * qh;
    if (!CAUSAL || qlo + 31 >= kw0) {  // some query of my half-tile sees my keys
      f32x16 sc, dpv;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sc[r] = 0.f;
        dpv[r] = 0.f;
      }
      // step i: chain i & 1 (0 = S from Q.K^T, 1 = dP from dO.V^T), k-slice i >> 1; the reads of
      // step i + PF are issued before the MFMA of step i
      auto rd_a = [&](int i) { return lds_row((i & 1) ? dol : ql, l32, 2 * (i >> 1) + hf); };
      auto rd_b = [&](int i) { return lds_row((i & 1) ? vl : kl, 32 * g + l32, 2 * (i >> 1) + hf); };
      constexpr int NB = PF + 1;
      bf16x8 fa[NB], fb[NB];
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        fa[j] = rd_a(j);
        fb[j] = rd_b(j);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const bf16x8 a = fa[i % NB], bb = fb[i % NB];
        if (i + PF < 16) {
          fa[(i + PF) % NB] = rd_a(i + PF);
          fb[(i + PF) % NB] = rd_b(i + PF);
        }
        if (i & 1)
          dpv = mfma(a, bb, dpv);
        else
          sc = mfma(a, bb, sc);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * PF, 0);
#pragma unroll
      for (int i = 0; i < 16 - PF; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, PF, 0);
      stamp(1);
      // the dV/dK operands (transposed dO / Q fragments) do not depend on P or dS: with EARLY the
      // first d-group is read here and lands under the softmax math, and every later group is read
      // one group ahead of its MFMAs (without it: 8 reads -> lgkmcnt(0) -> 4 MFMAs per group)
      bf16x8 gf[2][4];
      auto rd_g = [&](int d, bf16x8(&f)[4]) {
        f[0] = lds_tr(dol, 0, 32 * d, lane);
        f[1] = lds_tr(dol, 16, 32 * d, lane);
        f[2] = lds_tr(ql, 0, 32 * d, lane);
        f[3] = lds_tr(ql, 16, 32 * d, lane);
      };
      if constexpr (EARLY) rd_g(0, gf[0]);
      const bool diag = CAUSAL && qlo < kw0 + 31;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const f4 L = *reinterpret_cast<const f4*>(ll + 8 * rr + 4 * hf);
#pragma unroll
        for (int i = 0; i < 4; ++i) sc[4 * rr + i] = fexp2(fmaf(sc[4 * rr + i], scale_log2, -L[i]));
      }
      if (__builtin_expect(diag, 0)) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (mykey > qlo + 8 * (r >> 2) + 4 * hf + (r & 3)) sc[r] = 0.f;
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const f4 Dl = *reinterpret_cast<const f4*>(dl + 8 * rr + 4 * hf);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * rr + i;
          dpv[r] = sc[r] * (dpv[r] - Dl[i]);
        }
      }
      bf16x8 pb[2], dsb[2];
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        pb[k2] = to_bf16x8(sc, 8 * k2);
        dsb[k2] = to_bf16x8(dpv, 8 * k2);
      }
      stamp(2);
      if constexpr (EARLY) {
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          if (d + 1 < 4) rd_g(d + 1, gf[(d + 1) & 1]);
          const bf16x8(&f)[4] = gf[d & 1];
          dv[d] = mfma(f[0], pb[0], dv[d]);
          dk[d] = mfma(f[2], dsb[0], dk[d]);
          dv[d] = mfma(f[1], pb[1], dv[d]);
          dk[d] = mfma(f[3], dsb[1], dk[d]);
        }
      } else {
#pragma unroll
        for (int d = 0; d < 4; ++d)
#pragma unroll
          for (int k2 = 0; k2 < 2; ++k2) {
            dv[d] = mfma(lds_tr(dol, 16 * k2, 32 * d, lane), pb[k2], dv[d]);
            dk[d] = mfma(lds_tr(ql, 16 * k2, 32 * d, lane), dsb[k2], dk[d]);
          }
      }
    }
    stamp(3);
    if (!more) break;
    // the half's rendezvous: my DMA of the next tile has landed and my reads of this one returned
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    gen += 4;
    if (lane == 0) __hip_atomic_fetch_add(&cnt[qh], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(&cnt[qh], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < gen)
      __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
    stamp(4);
    ++tnum;
    ++qt;
    stage ^= 1;
  }
  __syncthreads();  // both halves are done with K/V and their rings: the LDS is reused below
  // reduce the two q-halves of every key group through LDS: [g][dk|dv][d][r][lane] floats
  float* red = reinterpret_cast<float*>(smem);
  if (qh == 1) {
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        red[(((g * 2 + 0) * 4 + d) * 16 + r) * 64 + lane] = dk[d][r];
        red[(((g * 2 + 1) * 4 + d) * 16 + r) * 64 + lane] = dv[d][r];
      }
  }
  __syncthreads();
  if (qh == 0) {
    const float sm = scale_log2 * 0.6931471805599453f;  // softmax scale = scale_log2 * ln2
    const long row = (((long)b * S + mykey) * H + hh) * HD;
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int dd = 32 * d + 8 * rr + 4 * hf;
        f4 ok, ov;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * rr + i;
          ok[i] = (dk[d][r] + red[(((g * 2 + 0) * 4 + d) * 16 + r) * 64 + lane]) * sm;
          ov[i] = dv[d][r] + red[(((g * 2 + 1) * 4 + d) * 16 + r) * 64 + lane];
        }
        *reinterpret_cast<f4*>(dkp + row + dd) = ok;
        *reinterpret_cast<f4*>(dvp + row + dd) = ov;
      }
  }
}

// ================================================================================================
// Backward dK/dV pass, 64 keys per wave: workgroup = 4 waves = 256 keys of one (b, q-head), one
// wave per SIMD.  Each wave keeps K (and, with VREG, V) of its 64 keys in registers and dK^T / dV^T
// of those keys in 256 accumulator registers, and sweeps 32-query slices of Q/dO staged in LDS:
// every Q / dO fragment read from LDS (rows for S and dP, transposed for dV^T and dK^T) feeds the
// MFMAs of TWO 32-key tiles, so a slice costs 32 KiB of LDS reads for 64 MFMAs per wave (the 8-wave
// kernel above: 48 KiB for 32) -- MFMA-bound instead of LDS-bound.  With VREG = false, V of the
// block sits in LDS (64 KiB) and is read as the dP B operand, which frees 64 VGPRs.  Same fp32
// per-q-head partial output as fa_bwd_dkdv_kernel.
// ================================================================================================
template <bool CAUSAL, bool VREG>
__global__ __launch_bounds__(256, 1) void fa_bwd_dkdv64_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, float* __restrict__ dkp, float* __restrict__ dvp, int B, int S,
    int H, int KVH, float scale_log2) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int STAGE = 2 * TILE_BYTES + 512;         // Q (64 rows) | dO (64 rows) | lse | delta
  constexpr int V_BYTES = VREG ? 0 : 4 * TILE_BYTES;  // V of the 256 keys (four 64-row tiles)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hf = lane >> 5, l32 = lane & 31;
  const int NH = H + 2 * KVH;
  const long rs = (long)NH * HD;
  const long ors = (long)H * HD;
  const int bid = blockIdx.x;
  const int kb = bid / (B * H);  // small kb = most q tiles: heaviest first
  const int bh = bid % (B * H);
  const int b = bh / H, hh = bh % H, kvh = hh / (H / KVH);
  const bf16_t* base = qkv + (long)b * S * rs;
  const bf16_t* qp = base + hh * HD;
  const bf16_t* kp = base + (H + kvh) * HD;
  const bf16_t* vp = base + (H + KVH + kvh) * HD;
  const bf16_t* dop = dout + (long)b * S * ors + hh * HD;
  const float* lp = lse + ((long)b * H + hh) * S;
  const float* dp = delta + ((long)b * H + hh) * S;
  const int kb0 = kb * 256, kw0 = kb0 + 64 * w;
  char* vl = smem;  // (VREG = false) V rows of the block, 4 x 64-row tiles
  char* ring = smem + V_BYTES;

  bf16x8 kf[2][8];
  bf16x8 vf[2][VREG ? 8 : 1];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      kf[t][ks] = *reinterpret_cast<const bf16x8*>(kp + (long)(kw0 + 32 * t + l32) * rs + 16 * ks + 8 * hf);
      if constexpr (VREG)
        vf[t][ks] = *reinterpret_cast<const bf16x8*>(vp + (long)(kw0 + 32 * t + l32) * rs + 16 * ks + 8 * hf);
    }
  if constexpr (!VREG) {
#pragma unroll
    for (int h64 = 0; h64 < 4; ++h64)
      dma_tile64(vp + (long)(kb0 + 64 * h64) * rs, rs, vl + h64 * TILE_BYTES, w, lane);
  }
  f32x16 dk[2][4], dv[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        dk[t][d][r] = 0.f;
        dv[t][d][r] = 0.f;
      }
  const int qt_begin = CAUSAL ? kb0 / 64 : 0;
  const int nqt = S / 64;
  auto issue = [&](int qt, char* st) {
    dma_tile64(qp + (long)qt * 64 * rs, rs, st, w, lane);
    dma_tile64(dop + (long)qt * 64 * ors, ors, st + TILE_BYTES, w, lane);
    if (w == 0) dma_f32x64(lp + qt * 64, st + 2 * TILE_BYTES, lane);
    if (w == 1) dma_f32x64(dp + qt * 64, st + 2 * TILE_BYTES + 256, lane);
  };
  issue(qt_begin, ring);
  wait_dma_and_barrier();

  for (int qt = qt_begin; qt < nqt; ++qt) {
    const int stage = (qt - qt_begin) & 1;
    const char* ql = ring + stage * STAGE;
    const char* dol = ql + TILE_BYTES;
    const float* ll = reinterpret_cast<const float*>(ql + 2 * TILE_BYTES);
    const float* dl = ll + 64;
    if (qt + 1 < nqt) issue(qt + 1, ring + (stage ^ 1) * STAGE);
#pragma unroll 1  // one slice's temporaries live at a time (256 AGPR accumulators + K/V)
    for (int qs = 0; qs < 2; ++qs) {
      const int qlo = qt * 64 + 32 * qs;
      if (CAUSAL && qlo + 31 < kw0) continue;  // every query of the slice precedes my keys
      f32x16 sc[2], dpv[2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          sc[t][r] = 0.f;
          dpv[t][r] = 0.f;
        }
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const bf16x8 aq = lds_row(ql, 32 * qs + l32, 2 * ks + hf);
        const bf16x8 ad = lds_row(dol, 32 * qs + l32, 2 * ks + hf);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          sc[t] = mfma(aq, kf[t][ks], sc[t]);
          if constexpr (VREG)
            dpv[t] = mfma(ad, vf[t][ks], dpv[t]);
          else
            dpv[t] = mfma(ad, lds_row(vl, 64 * w + 32 * t + l32, 2 * ks + hf), dpv[t]);
        }
      }
      // rows of sc/dpv: q = qlo + (r&3) + 8*(r>>2) + 4*hf ; column (lane) = key kw0 + 32t + l32
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int qi = 32 * qs + 8 * rr + 4 * hf;
        const f4 L = *reinterpret_cast<const f4*>(ll + qi);
        const f4 Dl = *reinterpret_cast<const f4*>(dl + qi);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * rr + i;
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            float pv = fexp2(fmaf(sc[t][r], scale_log2, -L[i]));
            if (CAUSAL && qlo < kw0 + 32 * t + 31 && kw0 + 32 * t + l32 > qt * 64 + qi + i) pv = 0.f;
            sc[t][r] = pv;
            dpv[t][r] = pv * (dpv[t][r] - Dl[i]);
          }
        }
      }
      bf16x8 pb[2][2], dsb[2][2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int k2 = 0; k2 < 2; ++k2) {
          pb[t][k2] = to_bf16x8(sc[t], 8 * k2);
          dsb[t][k2] = to_bf16x8(dpv[t], 8 * k2);
        }
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int k2 = 0; k2 < 2; ++k2) {
          const bf16x8 at = lds_tr(dol, 32 * qs + 16 * k2, 32 * d, lane);
          const bf16x8 qtr = lds_tr(ql, 32 * qs + 16 * k2, 32 * d, lane);
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            dv[t][d] = mfma(at, pb[t][k2], dv[t][d]);
            dk[t][d] = mfma(qtr, dsb[t][k2], dk[t][d]);
          }
        }
    }
    wait_dma_and_barrier();
  }
  const float sm = scale_log2 * 0.6931471805599453f;  // softmax scale = scale_log2 * ln2
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int key = kw0 + 32 * t + l32;
    float* dkr = dkp + (((long)b * S + key) * H + hh) * HD;
    float* dvr = dvp + (((long)b * S + key) * H + hh) * HD;
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int dd = 32 * d + 8 * rr + 4 * hf;
        *reinterpret_cast<f4*>(dkr + dd) = f4{dk[t][d][4 * rr] * sm, dk[t][d][4 * rr + 1] * sm,
                                              dk[t][d][4 * rr + 2] * sm, dk[t][d][4 * rr + 3] * sm};
        *reinterpret_cast<f4*>(dvr + dd) = f4{dv[t][d][4 * rr], dv[t][d][4 * rr + 1], dv[t][d][4 * rr + 2],
                                              dv[t][d][4 * rr + 3]};
      }
  }
}

// sum the per-q-head fp32 (P16: bf16) partials over each GQA group -> bf16 dk/dv inside dqkv
template <bool P16 = false>
__global__ __launch_bounds__(256) void fa_bwd_reduce_kv_kernel(const float* __restrict__ dkp,
                                                               const float* __restrict__ dvp,
                                                               bf16_t* __restrict__ dqkv, int B,
                                                               int S, int H, int KVH) {
  const int G = H / KVH;
  const long total = (long)B * S * KVH * (HD / 8);
  const long NHD = (long)(H + 2 * KVH) * HD;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % (HD / 8));
    const long r = i / (HD / 8);
    const int kvh = (int)(r % KVH);
    const long bs = r / KVH;
    float ak[8] = {0, 0, 0, 0, 0, 0, 0, 0}, av[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int g = 0; g < G; ++g) {
      const long src = (bs * H + kvh * G + g) * HD + c * 8;
      if constexpr (P16) {
        float k8[8], v8[8];
        unpack8(*reinterpret_cast<const us8*>(reinterpret_cast<const bf16_t*>(dkp) + src), k8);
        unpack8(*reinterpret_cast<const us8*>(reinterpret_cast<const bf16_t*>(dvp) + src), v8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          ak[j] += k8[j];
          av[j] += v8[j];
        }
      } else {
        const f4* pk = reinterpret_cast<const f4*>(dkp + src);
        const f4* pv = reinterpret_cast<const f4*>(dvp + src);
        const f4 k0 = pk[0], k1 = pk[1], v0 = pv[0], v1 = pv[1];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          ak[j] += k0[j];
          ak[4 + j] += k1[j];
          av[j] += v0[j];
          av[4 + j] += v1[j];
        }
      }
    }
    bf16_t* row = dqkv + bs * NHD;
    *reinterpret_cast<us8*>(row + (H + kvh) * HD + c * 8) = pack8(ak);
    *reinterpret_cast<us8*>(row + (H + KVH + kvh) * HD + c * 8) = pack8(av);
  }
}

// the same with the RoPE backward fused into dk: a thread sums 8 dims d and their partners d + 64
// of one (b, s, kv-head) and writes the gradient w.r.t. the unrotated k (cos / sin [S][64])
template <bool P16 = false>  // P16: the partials are bf16 (fa_bwd_dkdv8_kernel<..., P16>)
__global__ __launch_bounds__(256) void fa_bwd_reduce_kv_rope_kernel(const float* __restrict__ dkp,
                                                                    const float* __restrict__ dvp,
                                                                    bf16_t* __restrict__ dqkv, int B, int S,
                                                                    int H, int KVH,
                                                                    const float* __restrict__ rcos,
                                                                    const float* __restrict__ rsin) {
  const int G = H / KVH;
  const long total = (long)B * S * KVH * (HD / 16);
  const long NHD = (long)(H + 2 * KVH) * HD;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % (HD / 16));
    const long r = i / (HD / 16);
    const int kvh = (int)(r % KVH);
    const long bs = r / KVH;
    float ak[2][8], av[2][8];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 8; ++j) ak[h][j] = av[h][j] = 0.f;
    for (int g = 0; g < G; ++g) {
      const long src = (bs * H + kvh * G + g) * HD + c * 8;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if constexpr (P16) {
          float k8[8], v8[8];
          unpack8(*reinterpret_cast<const us8*>(reinterpret_cast<const bf16_t*>(dkp) + src + 64 * h), k8);
          unpack8(*reinterpret_cast<const us8*>(reinterpret_cast<const bf16_t*>(dvp) + src + 64 * h), v8);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            ak[h][j] += k8[j];
            av[h][j] += v8[j];
          }
        } else {
          const f4* pk = reinterpret_cast<const f4*>(dkp + src + 64 * h);
          const f4* pv = reinterpret_cast<const f4*>(dvp + src + 64 * h);
          const f4 k0 = pk[0], k1 = pk[1], v0 = pv[0], v1 = pv[1];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            ak[h][j] += k0[j];
            ak[h][4 + j] += k1[j];
            av[h][j] += v0[j];
            av[h][4 + j] += v1[j];
          }
        }
      }
    }
    const long t = (bs % S) * (HD / 2) + c * 8;
    const f4 c0 = *reinterpret_cast<const f4*>(rcos + t), c1 = *reinterpret_cast<const f4*>(rcos + t + 4);
    const f4 s0 = *reinterpret_cast<const f4*>(rsin + t), s1 = *reinterpret_cast<const f4*>(rsin + t + 4);
    const float cs[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
    const float sn[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
    float o1[8], o2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o1[j] = ak[0][j] * cs[j] + ak[1][j] * sn[j];
      o2[j] = ak[1][j] * cs[j] - ak[0][j] * sn[j];
    }
    bf16_t* row = dqkv + bs * NHD;
    *reinterpret_cast<us8*>(row + (H + kvh) * HD + c * 8) = pack8(o1);
    *reinterpret_cast<us8*>(row + (H + kvh) * HD + 64 + c * 8) = pack8(o2);
    *reinterpret_cast<us8*>(row + (H + KVH + kvh) * HD + c * 8) = pack8(av[0]);
    *reinterpret_cast<us8*>(row + (H + KVH + kvh) * HD + 64 + c * 8) = pack8(av[1]);
  }
}

// ================================================================================================
// Backward dQ pass: workgroup = 128 queries of one (b, q-head); loops over 64-key K/V tiles.
// ================================================================================================
// PF > 0 (DSTACK_AMD_FA_DQ_PF, default 1): K/V tiles through a buffer descriptor (counted LDS waits, see
// dma_tile64_buf) and the 32 S/dP fragment reads of a tile kept PF steps ahead of their MFMAs;
// the default form reads -> lgkmcnt(0) -> MFMA on every step.
template <bool CAUSAL, int NW = 4, bool HP = false, int PF = 0>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void fa_bwd_dq_kernel(const bf16_t* __restrict__ qkv,
                                                           const bf16_t* __restrict__ dout,
                                                           const float* __restrict__ lse,
                                                           const float* __restrict__ delta,
                                                           bf16_t* __restrict__ dqkv, int B, int S,
                                                           int H, int KVH, float scale_log2,
                                                           const float* __restrict__ rcos,
                                                           const float* __restrict__ rsin) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hf = lane >> 5, l32 = lane & 31;
  const int NH = H + 2 * KVH;
  const long rs = (long)NH * HD;
  const long ors = (long)H * HD;
  constexpr int QB = 32 * NW;
  if constexpr (HP) {
    if (w >= NW / 2) __builtin_amdgcn_s_setprio(1);
  }
  const int nqb = S / QB;
  const int bid = blockIdx.x;
  const int qb = CAUSAL ? nqb - 1 - bid / (B * H) : bid / (B * H);
  const int bh = bid % (B * H);
  const int b = bh / H, hh = bh % H, kvh = hh / (H / KVH);
  const bf16_t* base = qkv + (long)b * S * rs;
  const bf16_t* qp = base + hh * HD;
  const bf16_t* kp = base + (H + kvh) * HD;
  const bf16_t* vp = base + (H + KVH + kvh) * HD;
  const bf16_t* dop = dout + (long)b * S * ors + hh * HD;
  const int q0 = qb * QB, qw0 = q0 + 32 * w, myq = qw0 + l32;

  bf16x8 qf[8], df[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
    qf[ks] = *reinterpret_cast<const bf16x8*>(qp + (long)myq * rs + 16 * ks + 8 * hf);
    df[ks] = *reinterpret_cast<const bf16x8*>(dop + (long)myq * ors + 16 * ks + 8 * hf);
  }
  const float L = lse[((long)b * H + hh) * S + myq];
  const float Dl = delta[((long)b * H + hh) * S + myq];
  f32x16 dq[4];
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[d][r] = 0.f;
  const int nkv = CAUSAL ? (q0 + QB) / 64 : S / 64;

  const unsigned kvbytes = (unsigned)(((long)(S - 1) * rs + HD) * 2);
  const __amdgpu_buffer_rsrc_t krs = make_rsrc(kp, kvbytes), vrs = make_rsrc(vp, kvbytes);
  unsigned kvoff[16 / NW];
  dma_tile64_offsets<NW>(rs, w, lane, kvoff);
  auto issue = [&](int t, char* nk) {
    if constexpr (PF > 0) {
      dma_tile64_buf<NW>(krs, kvoff, (int)((long)t * 64 * rs * 2), nk, w);
      dma_tile64_buf<NW>(vrs, kvoff, (int)((long)t * 64 * rs * 2), nk + TILE_BYTES, w);
    } else {
      dma_tile64_n<NW>(kp + (long)t * 64 * rs, rs, nk, w, lane);
      dma_tile64_n<NW>(vp + (long)t * 64 * rs, rs, nk + TILE_BYTES, w, lane);
    }
  };
  issue(0, smem);
  wait_dma_and_barrier();
  for (int it = 0; it < nkv; ++it) {
    const char* kl = smem + (it & 1) * 2 * TILE_BYTES;
    const char* vl = kl + TILE_BYTES;
    if (it + 1 < nkv) issue(it + 1, smem + ((it + 1) & 1) * 2 * TILE_BYTES);
    const int kv0 = it * 64;
    if (!CAUSAL || kv0 <= qw0 + 31) {
      f32x16 st[2], dpt[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          st[t][r] = 0.f;
          dpt[t][r] = NW == 8 ? -Dl : 0.f;  // 8 waves: -delta seeds dP (see the launch note)
        }
      }
      if constexpr (PF > 0) {
        // step i: key sub-tile i >> 4, k-slice (i >> 1) & 7, chain i & 1 (0 = S from K, 1 = dP from V)
        auto rd = [&](int i) { return lds_row((i & 1) ? vl : kl, 32 * (i >> 4) + l32, 2 * ((i >> 1) & 7) + hf); };
        constexpr int NB = PF + 1;
        bf16x8 fr[NB];
#pragma unroll
        for (int j = 0; j < PF; ++j) fr[j] = rd(j);
#pragma unroll
        for (int i = 0; i < 32; ++i) {
          const bf16x8 a = fr[i % NB];
          if (i + PF < 32) fr[(i + PF) % NB] = rd(i + PF);
          const int t = i >> 4, ks = (i >> 1) & 7;
          if (i & 1)
            dpt[t] = mfma(a, df[ks], dpt[t]);
          else
            st[t] = mfma(a, qf[ks], st[t]);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, PF, 0);
#pragma unroll
        for (int i = 0; i < 32 - PF; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, PF, 0);
      } else {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int ks = 0; ks < 8; ++ks) {
            st[t] = mfma(lds_row(kl, 32 * t + l32, 2 * ks + hf), qf[ks], st[t]);
            dpt[t] = mfma(lds_row(vl, 32 * t + l32, 2 * ks + hf), df[ks], dpt[t]);
          }
      }
      const bool diag = CAUSAL && kv0 + 63 > qw0;
      // P, the causal mask on diagonal tiles only (a wave-uniform branch, not a per-element select
      // in every tile: 32 v_cmp + 32 v_cndmask + 31 s_and + the key arithmetic per tile), then dS
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) st[t][r] = fexp2(fmaf(st[t][r], scale_log2, -L));
      if (__builtin_expect(diag, 0)) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (kv0 + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hf > myq) st[t][r] = 0.f;
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          dpt[t][r] = NW == 8 ? st[t][r] * dpt[t][r] : st[t][r] * (dpt[t][r] - Dl);
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const bf16x8 a = to_bf16x8(dpt[s4 >> 1], 8 * (s4 & 1));
#pragma unroll
        for (int d = 0; d < 4; ++d) dq[d] = mfma(a, lds_tr(kl, 16 * s4, 32 * d, lane), dq[d]);
      }
    }
    wait_dma_and_barrier();
  }
  // dq accumulator: column (lane) = d within block, rows q = (r&3) + 8*(r>>2) + 4*hf (wave-local)
  const float sm = scale_log2 * 0.6931471805599453f;
  bf16_t* dqb = dqkv + ((long)b * S + qw0) * rs + hh * HD;
  if (rcos != nullptr) {
    // RoPE backward fused (the forward rotated q in the qkv GEMM's epilogue): the gradient w.r.t.
    // the unrotated q, g1 c + g2 s / g2 c - g1 s for the pair (d, d + 64) = accumulators d, d + 2
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qq = (r & 3) + 8 * (r >> 2) + 4 * hf;
        const long t = (long)(qw0 + qq) * (HD / 2) + 32 * d + l32;
        const float c = rcos[t], sn = rsin[t];
        const float g1 = dq[d][r] * sm, g2 = dq[d + 2][r] * sm;
        dqb[(long)qq * rs + 32 * d + l32] = f2bf(g1 * c + g2 * sn);
        dqb[(long)qq * rs + 64 + 32 * d + l32] = f2bf(g2 * c - g1 * sn);
      }
    return;
  }
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qq = (r & 3) + 8 * (r >> 2) + 4 * hf;
      dqb[(long)qq * rs + 32 * d + l32] = f2bf(dq[d][r] * sm);
    }
}

// ================================================================================================
// Backward dQ pass without recompute: dQ = dS . K over the dS^T spilled by the dK/dV pass
// (fa_bwd_dkdv8_kernel<..., SPILL>): one GEMM per tile instead of three (S, dP, dQ), no Q/dO/lse/
// delta.  Per 64-key step a stage holds the K tile and the dS^T tiles (64 keys x 128 queries) of
// the workgroup's queries, all DMA'd row-major into the swizzled LDS image; the A operand is the
// transposed read of dS^T, the B operand the transposed read of K.  Causal: keys > query are
// zeroed after the read (the dK/dV pass never writes fully masked 32x32 sub-tiles).
// ================================================================================================
template <bool CAUSAL, int NW>
__global__ __launch_bounds__(64 * NW) void fa_bwd_dq_ds_kernel(const bf16_t* __restrict__ qkv,
                                                               const bf16_t* __restrict__ dsg,
                                                               bf16_t* __restrict__ dqkv, int B, int S, int H,
                                                               int KVH, float scale_log2) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hf = lane >> 5, l32 = lane & 31;
  const int NH = H + 2 * KVH;
  const long rs = (long)NH * HD;
  constexpr int QB = 32 * NW, NT = NW / 4, STG = (1 + NT) * TILE_BYTES;
  const int nqb = S / QB;
  const int bid = blockIdx.x;
  const int qb = CAUSAL ? nqb - 1 - bid / (B * H) : bid / (B * H);
  const int bh = bid % (B * H);
  const int b = bh / H, hh = bh % H, kvh = hh / (H / KVH);
  const bf16_t* kp = qkv + (long)b * S * rs + (H + kvh) * HD;
  const int q0 = qb * QB, qw0 = q0 + 32 * w, myq = qw0 + l32;
  const bf16_t* dst = dsg + (long)bh * S * S + q0;  // dS^T rows (keys) of this workgroup's queries
  f32x16 dq[4];
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[d][r] = 0.f;
  const int nkv = CAUSAL ? (q0 + QB) / 64 : S / 64;
  const int nmine = CAUSAL ? (qw0 + 31) / 64 + 1 : nkv;  // tiles with kv0 <= qw0 + 31
  auto issue = [&](int it, char* st) {
    dma_tile64_n<NW>(kp + (long)it * 64 * rs, rs, st, w, lane);
#pragma unroll
    for (int t = 0; t < NT; ++t)
      dma_tile64_n<NW>(dst + (long)it * 64 * S + 128 * t, S, st + (1 + t) * TILE_BYTES, w, lane);
  };
  issue(0, smem);
  wait_dma_and_barrier();
  for (int it = 0; it < nkv; ++it) {
    const char* kl = smem + (it & 1) * STG;
    if (it + 1 < nkv) issue(it + 1, smem + ((it + 1) & 1) * STG);
    const int kv0 = it * 64;
    if (it < nmine) {
      const char* dl = kl + (1 + (w >> 2)) * TILE_BYTES;
      const bool diag = CAUSAL && kv0 + 63 > qw0;
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        us8 a = __builtin_bit_cast(us8, lds_tr(dl, 16 * s4, 32 * (w & 3), lane));
        if (diag) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int key = kv0 + 16 * s4 + 4 * hf + (j & 3) + 8 * (j >> 2);
            if (key > myq) a[j] = 0;
          }
        }
        const bf16x8 av = __builtin_bit_cast(bf16x8, a);
#pragma unroll
        for (int d = 0; d < 4; ++d) dq[d] = mfma(av, lds_tr(kl, 16 * s4, 32 * d, lane), dq[d]);
      }
    }
    wait_dma_and_barrier();
  }
  const float sm = scale_log2 * 0.6931471805599453f;
  bf16_t* dqb = dqkv + ((long)b * S + qw0) * rs + hh * HD;
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qq = (r & 3) + 8 * (r >> 2) + 4 * hf;
      dqb[(long)qq * rs + 32 * d + l32] = f2bf(dq[d][r] * sm);
    }
}

// ================================================================================================
// launchers
// ================================================================================================
static inline bool fa_shape_ok(int S, int H, int KVH, int D) {
  return D == HD && S % 128 == 0 && S > 0 && KVH > 0 && H % KVH == 0;
}

extern "C" hipError_t dsa_fa_fwd(const void* qkv, void* out, float* lse, int B, int S, int H, int KVH,
                                 int D, float scale, int causal, hipStream_t st) {
  if (!fa_shape_ok(S, H, KVH, D)) return hipErrorInvalidValue;
  const float sl2 = scale * 1.4426950408889634f;
  const size_t lds = 4 * TILE_BYTES;
  // deferred-max threshold (log2 units; 0 = rescale on every new max): 8 takes the S=8192 causal
  // forward from 0.700 to 0.660 ms, same fp32-reference error (tools/gpu_sessions/run_r2r.sh)
  static const float thr = [] {
    const char* v = getenv("DSTACK_AMD_FA_RESCALE_THR");
    return v ? (float)atof(v) : 8.f;
  }();
  // 8 waves (one 256-row workgroup per CU) by default: 0.710 vs 0.720 ms at S=8192, three
  // interleaved same-box runs (tools/gpu_sessions/run_r1s.sh); DSTACK_AMD_FA_FWD_WAVES=4 selects the 4-wave form
  static const int waves = [] {
    const char* v = getenv("DSTACK_AMD_FA_FWD_WAVES");
    return (v && atoi(v) == 4) ? 4 : 8;
  }();
  static const bool pf = [] {
    const char* v = getenv("DSTACK_AMD_FA_FWD_PF");
    return !(v && atoi(v) == 0);
  }();
  static const int prio = [] {
    const char* v = getenv("DSTACK_AMD_FA_PRIO");
    return v ? atoi(v) : 0;
  }();
  static const bool stag = [] {
    const char* v = getenv("DSTACK_AMD_FA_FWD_STAG");
    return v && atoi(v) == 1;
  }();
  static const bool half_prio = [] {
    const char* v = getenv("DSTACK_AMD_FA_HALF_PRIO");
    return v && atoi(v) == 1;
  }();
  // K/V through buffer descriptors (DSTACK_AMD_FA_FWD_BUF=0 selects global_load_lds): forward
  // 0.647-0.663 vs 0.660-0.679 ms, S=8192, 3 interleaved runs (profiles/fa_dq_fwd_ab_r8w.txt)
  static const bool fwd_buf_env = [] {
    const char* v = getenv("DSTACK_AMD_FA_FWD_BUF");
    return !(v && atoi(v) == 0);
  }();
  const bool fwd_buf = fwd_buf_env && (long)S * (H + 2 * KVH) * HD * 2 < (1L << 31);
  static const int fwd_pfd = [] {  // S-phase K reads in flight (buffer-DMA form): 4 or 8 (A/B)
    const char* v = getenv("DSTACK_AMD_FA_FWD_PFD");
    return (v && atoi(v) == 8) ? 8 : 4;
  }();
  if (waves == 8 && S % 256 == 0) {
    const int grid = B * H * (S / 256);
    if (causal && pf && half_prio)
      fa_fwd_kernel<true, 8, true, 3><<<grid, 512, lds, st>>>((const bf16_t*)qkv, (bf16_t*)out, lse, B, S, H, KVH, sl2,
                                                            thr);
    else if (causal && pf && stag)
      fa_fwd_kernel<true, 8, true, 0, true><<<grid, 512, 6 * TILE_BYTES, st>>>((const bf16_t*)qkv, (bf16_t*)out, lse, B, S,
                                                                            H, KVH, sl2, thr);
    else if (causal && pf && prio == 1)
      fa_fwd_kernel<true, 8, true, 1><<<grid, 512, lds, st>>>((const bf16_t*)qkv, (bf16_t*)out, lse, B, S, H, KVH, sl2,
                                                            thr);
    else if (causal && pf && prio == 2)
      fa_fwd_kernel<true, 8, true, 2><<<grid, 512, lds, st>>>((const bf16_t*)qkv, (bf16_t*)out, lse, B, S, H, KVH, sl2,
                                                            thr);
    else if (causal && pf && fwd_buf && fwd_pfd == 8)
      fa_fwd_kernel<true, 8, true, 0, false, true, 8><<<grid, 512, lds, st>>>((const bf16_t*)qkv, (bf16_t*)out, lse, B,
                                                                            S, H, KVH, sl2, thr);
    else if (causal && pf && fwd_buf)
      fa_fwd_kernel<true, 8, true, 0, false, true><<<grid, 512, lds, st>>>((const bf16_t*)qkv, (bf16_t*)out, lse, B, S,
                                                                         H, KVH, sl2, thr);
    else if (causal && pf)
      fa_fwd_kernel<true, 8><<<grid, 512, lds, st>>>((const bf16_t*)qkv, (bf16_t*)out, lse, B, S, H, KVH, sl2, thr);
    else if (causal)
      fa_fwd_kernel<true, 8, false><<<grid, 512, lds, st>>>((const bf16_t*)qkv, (bf16_t*)out, lse, B, S, H, KVH, sl2, thr);
    else
      fa_fwd_kernel<false, 8><<<grid, 512, lds, st>>>((const bf16_t*)qkv, (bf16_t*)out, lse, B, S, H, KVH, sl2, thr);
    return hipGetLastError();
  }
  const int grid = B * H * (S / 128);
  if (causal)
    fa_fwd_kernel<true><<<grid, 256, lds, st>>>((const bf16_t*)qkv, (bf16_t*)out, lse, B, S, H, KVH, sl2, thr);
  else
    fa_fwd_kernel<false><<<grid, 256, lds, st>>>((const bf16_t*)qkv, (bf16_t*)out, lse, B, S, H, KVH, sl2, thr);
  return hipGetLastError();
}

// dS spill for the recompute-free dQ pass (DSTACK_AMD_FA_DQ=ds|recompute): B*H*S*S bf16 of
// workspace, used while it stays under DSTACK_AMD_FA_DS_MAX_GB (default 16)
static bool fa_ds_spill(int B, int S, int H) {
  static const int mode = [] {
    const char* v = getenv("DSTACK_AMD_FA_DQ");
    return (v && std::string(v) == "ds") ? 1 : 0;
  }();
  static const double max_gb = [] {
    const char* v = getenv("DSTACK_AMD_FA_DS_MAX_GB");
    return v ? atof(v) : 16.0;
  }();
  return mode == 1 && (double)B * H * S * S * 2 <= max_gb * 1e9;
}

// workspace: delta (B*H*S fp32) + dkp + dvp (2 * B*S*H*128 fp32) [+ dS spill (B*H*S*S bf16)]
extern "C" size_t dsa_fa_bwd_workspace(int B, int S, int H) {
  return (size_t)B * H * S * 4 + 2 * (size_t)B * S * H * HD * 4 +
         (fa_ds_spill(B, S, H) ? (size_t)B * H * S * S * 2 : 0);
}

extern "C" hipError_t dsa_rope_qkv(const void* in, void* out, const float* cosT, const float* sinT, int rows, int S,
                                   int NH, int n_rot, int D, int inverse, hipStream_t st);

// rcos / rsin (nullable, [S][64] fp32): q and k were rotated by RoPE after the projection (the qkv
// GEMM's epilogue); dqkv is then the gradient w.r.t. the unrotated projection -- fused into the dQ
// epilogue and the dK reduction on the default path, an in-place pass on the others.
// The dQ pass on a second stream of the same device (DSTACK_AMD_FA_DQ_STREAM=1): it depends only on
// the delta pass, like the dK/dV pass, so the two can share the CUs -- the workgroups of one fill
// what the other's causal tail leaves idle.  The side stream is non-blocking (no implicit sync with
// the legacy default stream); the caller's stream waits for it before anything reads dqkv.
namespace {
struct FaSide {
  hipStream_t s = nullptr;
  hipEvent_t ready = nullptr, done = nullptr;
};
FaSide* fa_side() {
  static std::mutex mu;
  static FaSide sides[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> g(mu);
  FaSide& f = sides[dev];
  if (f.s == nullptr) {
    if (hipStreamCreateWithFlags(&f.s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    if (hipEventCreateWithFlags(&f.ready, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&f.done, hipEventDisableTiming) != hipSuccess)
      return nullptr;
  }
  return &f;
}
}  // namespace

extern "C" hipError_t dsa_fa_bwd(const void* qkv, const void* out, const void* dout, const float* lse,
                                 void* dqkv, void* workspace, int B, int S, int H, int KVH, int D,
                                 float scale, int causal, const float* rcos, const float* rsin,
                                 hipStream_t st) {
  if (!fa_shape_ok(S, H, KVH, D)) return hipErrorInvalidValue;
  const float sl2 = scale * 1.4426950408889634f;
  float* delta = (float*)workspace;
  float* dkp = delta + (size_t)B * H * S;
  float* dvp = dkp + (size_t)B * S * H * HD;
  const long rows = (long)B * S * H;
  if (H % 8 == 0 && S % 32 == 0)
    fa_bwd_delta_tiled_kernel<<<B * (S / 32) * (H / 8), 256, 0, st>>>(
        (const bf16_t*)out, (const bf16_t*)dout, delta, B, S, H);
  else
    fa_bwd_delta_kernel<<<(int)((rows + 15) / 16), 256, 0, st>>>((const bf16_t*)out,
                                                                 (const bf16_t*)dout, delta, B, S, H);
  DSA_CHECK(hipGetLastError());
  const int grid = B * H * (S / 128);
  // dK/dV q-tile per pipeline stage: 64 rows (default) or 128 (DSTACK_AMD_FA_DKDV_QT=128: half
  // the barriers, 130 KiB of LDS)
  static const int dkdv_qt = [] {
    const char* v = getenv("DSTACK_AMD_FA_DKDV_QT");
    return (v && atoi(v) == 128) ? 128 : 64;
  }();
  const size_t lds_kv = 2 * (2 * (size_t)dkdv_qt * 256 + 8 * (size_t)dkdv_qt);
  const size_t lds_q = 4 * TILE_BYTES;
  // dK/dV kernel: the 8-wave K/V-resident variant is the default (2.10 vs 2.53 ms for the whole
  // backward at S=8192, same box); DSTACK_AMD_FA_DKDV=4w selects the 4-wave register-resident one.
  // Opt-in variants measured slower and kept for A/B only (profiles/fa_dkdv_seed_ab_r4h.txt, 3
  // interleaved runs, whole backward S=8192): default 675-684 TFLOP/s, 'seed' (row-constant seeded
  // dK/dV accumulators) 583-592, '64kv' (64 keys per wave, V in registers) 576-581.
  static const int dkdv_kind = [] {  // 8 = 8-wave (default), 4 = 4-wave, 64 / 65 = 64 keys per wave
    const char* v = getenv("DSTACK_AMD_FA_DKDV");
    if (!v) return 8;
    const std::string s(v);
    return s == "4w" ? 4 : (s == "64k" ? 64 : (s == "64kv" ? 65 : (s == "seed" ? 9 : 8)));
  }();
  const bool dkdv8 = dkdv_kind == 8 || dkdv_kind == 9;
  // dQ pass: 8 waves / 256 query rows per workgroup when S % 256 == 0 (DSTACK_AMD_FA_DQ_WAVES=4|8).
  // Whole backward at S=8192, same box, 3 interleaved runs each (tools/gpu_sessions/run_r1t.sh): 4 waves 2.06-2.08
  // ms; 8 waves 2.04-2.07; 8 waves with the dP accumulator seeded with -delta ('row constant')
  // 2.00-2.05 -- the seeding is kept for 8 waves only: with 4 waves it measured 2.14-2.17 ms.
  static const int dq_waves_env = [] {
    const char* v = getenv("DSTACK_AMD_FA_DQ_WAVES");
    return (v && atoi(v) == 4) ? 4 : 8;
  }();
  const int dq_waves = (dq_waves_env == 8 && S % 256 == 0) ? 8 : 4;
  static const bool half_prio = [] {  // static priority for waves 4-7 (see the forward's PRIO 3)
    const char* v = getenv("DSTACK_AMD_FA_HALF_PRIO");
    return v && atoi(v) == 1;
  }();
  // GQA-summed dK/dV (one workgroup per KV head and key block, bf16 written directly, no reduce
  // kernel): DSTACK_AMD_FA_DKDV_GQA=1
  static const bool dkdv_gqa_env = [] {
    const char* v = getenv("DSTACK_AMD_FA_DKDV_GQA");
    return v && atoi(v) == 1;
  }();
  const bool dkdv_gqa = dkdv_gqa_env && dkdv_kind == 8 && !half_prio && !fa_ds_spill(B, S, H);
  const bool rope_fused = rcos != nullptr && !dkdv_gqa && !fa_ds_spill(B, S, H);
  const float* rq = rope_fused ? rcos : nullptr;
  const float* rsq = rope_fused ? rsin : nullptr;
  auto rope_after = [&]() -> hipError_t {  // the paths without the fused RoPE backward
    if (rcos == nullptr || rope_fused) return hipSuccess;
    return dsa_rope_qkv(dqkv, dqkv, rcos, rsin, B * S, S, H + 2 * KVH, H + KVH, HD, 1, st);
  };
  // S/dP read pipeline of the 8-wave dK/dV pass (DSTACK_AMD_FA_DKDV_PF=0|1|2, default 2).  Whole
  // backward at S=8192, 3 interleaved runs (profiles/fa_bwd_pf_ab_r8t.txt): PF 0 2.031-2.045 ms,
  // PF 2 1.959-1.963 ms.  The dQ pass's counterpart (DSTACK_AMD_FA_DQ_PF=1|2) measured no gain.
  static const int dkdv_pf_env = [] {
    const char* v = getenv("DSTACK_AMD_FA_DKDV_PF");
    return v ? atoi(v) : 2;
  }();
  // the PF form addresses a Q / dO tile through a buffer descriptor with 32-bit offsets
  const int dkdv_pf = ((long)S * (H + 2 * KVH) * HD * 2 < (1L << 31)) ? dkdv_pf_env : 0;
  // dQ pass: DSTACK_AMD_FA_DQ_PF=0|1|2, default 1 (whole backward 1.924-1.946 vs 1.945-1.964 ms;
  // 2 spills and measured 1.976-2.000, profiles/fa_dq_fwd_ab_r8w.txt)
  static const int dq_pf_env = [] {
    const char* v = getenv("DSTACK_AMD_FA_DQ_PF");
    return v ? atoi(v) : 1;
  }();
  const int dq_pf = ((long)S * (H + 2 * KVH) * HD * 2 < (1L << 31)) ? dq_pf_env : 0;
  // decoupled halves (fa_bwd_dkdv8d_kernel): DSTACK_AMD_FA_DKDV_DEC=1, waves 4-7 started
  // DSTACK_AMD_FA_DKDV_STAG x 64 clocks late
  static const int dkdv_dec_env = [] {
    const char* v = getenv("DSTACK_AMD_FA_DKDV_DEC");
    return v ? atoi(v) : 0;
  }();
  static const int dkdv_stag = [] {
    const char* v = getenv("DSTACK_AMD_FA_DKDV_STAG");
    return v ? atoi(v) : 0;
  }();
  const bool dkdv_dec = dkdv_dec_env >= 1 && dkdv_kind == 8 && !half_prio && !dkdv_gqa && dkdv_pf >= 2;
  // bf16 per-query-head dK/dV partials (DSTACK_AMD_FA_DKDV_BF16=1|0): the default 8-wave PF-2 pass only
  static const bool dkdv_bf16_env = [] {
    const char* v = getenv("DSTACK_AMD_FA_DKDV_BF16");
    return v ? atoi(v) == 1 : true;
  }();
  const bool p16 = dkdv_bf16_env && dkdv_kind == 8 && dkdv_pf == 2 && !dkdv_dec && !half_prio && !dkdv_gqa &&
                   !fa_ds_spill(B, S, H);
  const size_t lds_dec = 2 * 128 * 256 + 4 * (2 * 32 * 256 + 512) + 16;
#define DSA_DKDV(C, N)                                                                                 \
  do {                                                                                                 \
    if (dkdv_dec && dkdv_dec_env == 2) {                                                               \
      fa_bwd_dkdv8d_kernel<C, false, true><<<grid, 512, lds_dec, st>>>(                                  \
          (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, dkp, dvp, B, S, H, KVH, sl2, dkdv_stag, nullptr); \
    } else if (dkdv_dec) {                                                                             \
      fa_bwd_dkdv8d_kernel<C><<<grid, 512, lds_dec, st>>>((const bf16_t*)qkv, (const bf16_t*)dout, lse,  \
                                                          delta, dkp, dvp, B, S, H, KVH, sl2, dkdv_stag,  \
                                                          nullptr);                                      \
    } else if (dkdv_kind >= 64 && S % 256 == 0) {                                                      \
      if (dkdv_kind == 64)                                                                             \
        fa_bwd_dkdv64_kernel<C, true><<<B * H * (S / 256), 256, 2 * (2 * TILE_BYTES + 512), st>>>(     \
            (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, dkp, dvp, B, S, H, KVH, sl2);         \
      else                                                                                             \
        fa_bwd_dkdv64_kernel<C, false><<<B * H * (S / 256), 256, 4 * TILE_BYTES + 2 * (2 * TILE_BYTES + 512), \
                                         st>>>((const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, dkp, dvp, \
                                               B, S, H, KVH, sl2);                                     \
    } else if (dkdv_kind == 9) {                                                                      \
      fa_bwd_dkdv8_kernel<C, true><<<grid, 512, 2 * 128 * 256 + 2 * (2 * TILE_BYTES + 512), st>>>(     \
          (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, dkp, dvp, B, S, H, KVH, sl2, nullptr);  \
    } else if ((dkdv8 || dkdv_kind >= 64) && half_prio && dkdv_pf >= 2) {                              \
      fa_bwd_dkdv8_kernel<C, false, true, false, false, false, 2>                                      \
          <<<grid, 512, 2 * 128 * 256 + 2 * (2 * TILE_BYTES + 512), st>>>(                             \
              (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, dkp, dvp, B, S, H, KVH, sl2, nullptr); \
    } else if ((dkdv8 || dkdv_kind >= 64) && half_prio) {                                              \
      fa_bwd_dkdv8_kernel<C, false, true><<<grid, 512, 2 * 128 * 256 + 2 * (2 * TILE_BYTES + 512), st>>>( \
          (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, dkp, dvp, B, S, H, KVH, sl2, nullptr);  \
    } else if (dkdv_gqa) {                                                                             \
      fa_bwd_dkdv8_kernel<C, false, false, false, true>                                                \
          <<<B * KVH * (S / 128), 512, 2 * 128 * 256 + 2 * (2 * TILE_BYTES + 512), st>>>(              \
              (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, dkp, dvp, B, S, H, KVH, sl2, nullptr, \
              (bf16_t*)dqkv);                                                                          \
    } else if (dkdv_pf == 1 && dkdv_kind == 8) {                                                       \
      fa_bwd_dkdv8_kernel<C, false, false, false, false, false, 1>                                     \
          <<<grid, 512, 2 * 128 * 256 + 2 * (2 * TILE_BYTES + 512), st>>>(                             \
              (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, dkp, dvp, B, S, H, KVH, sl2, nullptr); \
    } else if (dkdv_pf >= 3 && dkdv_kind == 8) {                                                       \
      fa_bwd_dkdv8_kernel<C, false, false, false, false, false, 3>                                     \
          <<<grid, 512, 2 * 128 * 256 + 2 * (2 * TILE_BYTES + 512), st>>>(                             \
              (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, dkp, dvp, B, S, H, KVH, sl2, nullptr); \
    } else if (p16) {                                                                                  \
      fa_bwd_dkdv8_kernel<C, false, false, false, false, false, 2, true>                               \
          <<<grid, 512, 2 * 128 * 256 + 2 * (2 * TILE_BYTES + 512), st>>>(                             \
              (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, dkp, dvp, B, S, H, KVH, sl2, nullptr); \
    } else if (dkdv_pf == 2 && dkdv_kind == 8) {                                                       \
      fa_bwd_dkdv8_kernel<C, false, false, false, false, false, 2>                                     \
          <<<grid, 512, 2 * 128 * 256 + 2 * (2 * TILE_BYTES + 512), st>>>(                             \
              (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, dkp, dvp, B, S, H, KVH, sl2, nullptr); \
    } else if (dkdv8 || dkdv_kind >= 64) {                                                             \
      fa_bwd_dkdv8_kernel<C><<<grid, 512, 2 * 128 * 256 + 2 * (2 * TILE_BYTES + 512), st>>>(          \
          (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, dkp, dvp, B, S, H, KVH, sl2, nullptr);  \
    } else                                                                                             \
      fa_bwd_dkdv_kernel<C, N><<<grid, 256, lds_kv, st>>>((const bf16_t*)qkv, (const bf16_t*)dout, lse, \
                                                          delta, dkp, dvp, B, S, H, KVH, sl2);         \
  } while (0)
  static const bool dq_stream_env = [] {
    const char* v = getenv("DSTACK_AMD_FA_DQ_STREAM");
    return v && atoi(v) == 1;
  }();
  FaSide* side = nullptr;  // set when the causal dQ pass runs on the side stream
  // the caller's stream waits for the side stream's dQ pass before anything after this call
  auto join = [&]() -> hipError_t { return side ? hipStreamWaitEvent(st, side->done, 0) : hipSuccess; };
  if (fa_ds_spill(B, S, H)) {  // dK/dV pass writes dS; dQ is one GEMM over the spilled dS
    bf16_t* dsg = (bf16_t*)(dvp + (size_t)B * S * H * HD);
    const size_t lds8 = 2 * 128 * 256 + 2 * (2 * TILE_BYTES + 512);
    if (causal)
      fa_bwd_dkdv8_kernel<true, false, false, true><<<grid, 512, lds8, st>>>(
          (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, dkp, dvp, B, S, H, KVH, sl2, dsg);
    else
      fa_bwd_dkdv8_kernel<false, false, false, true><<<grid, 512, lds8, st>>>(
          (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, dkp, dvp, B, S, H, KVH, sl2, dsg);
    DSA_CHECK(hipGetLastError());
    const size_t lds_ds8 = 2 * 3 * TILE_BYTES, lds_ds4 = 2 * 2 * TILE_BYTES;
    if (S % 256 == 0) {
      if (causal)
        fa_bwd_dq_ds_kernel<true, 8><<<B * H * (S / 256), 512, lds_ds8, st>>>((const bf16_t*)qkv, dsg, (bf16_t*)dqkv,
                                                                             B, S, H, KVH, sl2);
      else
        fa_bwd_dq_ds_kernel<false, 8><<<B * H * (S / 256), 512, lds_ds8, st>>>((const bf16_t*)qkv, dsg,
                                                                              (bf16_t*)dqkv, B, S, H, KVH, sl2);
    } else {
      if (causal)
        fa_bwd_dq_ds_kernel<true, 4><<<grid, 256, lds_ds4, st>>>((const bf16_t*)qkv, dsg, (bf16_t*)dqkv, B, S, H,
                                                                KVH, sl2);
      else
        fa_bwd_dq_ds_kernel<false, 4><<<grid, 256, lds_ds4, st>>>((const bf16_t*)qkv, dsg, (bf16_t*)dqkv, B, S, H,
                                                                 KVH, sl2);
    }
  } else if (causal) {
    hipStream_t qs = st;  // the dQ pass's stream
    if (dq_stream_env && (side = fa_side()) != nullptr) {
      DSA_CHECK(hipEventRecord(side->ready, st));  // after the delta pass
      DSA_CHECK(hipStreamWaitEvent(side->s, side->ready, 0));
      qs = side->s;
    }
    if (dkdv_qt == 128) DSA_DKDV(true, 4); else DSA_DKDV(true, 2);
    DSA_CHECK(hipGetLastError());
    if (dq_waves == 8 && half_prio)
      fa_bwd_dq_kernel<true, 8, true><<<B * H * (S / 256), 512, lds_q, qs>>>(
          (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv, B, S, H, KVH, sl2, rq, rsq);
    else if (dq_waves == 8 && dq_pf == 1)
      fa_bwd_dq_kernel<true, 8, false, 1><<<B * H * (S / 256), 512, lds_q, qs>>>(
          (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv, B, S, H, KVH, sl2, rq, rsq);
    else if (dq_waves == 8 && dq_pf >= 2)
      fa_bwd_dq_kernel<true, 8, false, 2><<<B * H * (S / 256), 512, lds_q, qs>>>(
          (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv, B, S, H, KVH, sl2, rq, rsq);
    else if (dq_waves == 8)
      fa_bwd_dq_kernel<true, 8><<<B * H * (S / 256), 512, lds_q, qs>>>(
          (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv, B, S, H, KVH, sl2, rq, rsq);
    else
      fa_bwd_dq_kernel<true><<<grid, 256, lds_q, qs>>>((const bf16_t*)qkv, (const bf16_t*)dout, lse, delta,
                                                       (bf16_t*)dqkv, B, S, H, KVH, sl2, rq, rsq);
    if (side != nullptr) DSA_CHECK(hipEventRecord(side->done, qs));
  } else {
    if (dkdv_qt == 128) DSA_DKDV(false, 4); else DSA_DKDV(false, 2);
    DSA_CHECK(hipGetLastError());
    if (dq_waves == 8)
      fa_bwd_dq_kernel<false, 8><<<B * H * (S / 256), 512, lds_q, st>>>(
          (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv, B, S, H, KVH, sl2, rq, rsq);
    else
      fa_bwd_dq_kernel<false><<<grid, 256, lds_q, st>>>((const bf16_t*)qkv, (const bf16_t*)dout, lse,
                                                        delta, (bf16_t*)dqkv, B, S, H, KVH, sl2, rq, rsq);
  }
#undef DSA_DKDV
  DSA_CHECK(hipGetLastError());
  if (dkdv_gqa) {  // dK/dV already summed over the group, in dqkv
    DSA_CHECK(join());
    return rope_after();
  }
  if (rope_fused) {
    const long work = (long)B * S * KVH * (HD / 16);
    int g = (int)((work + 255) / 256);
    if (g > 4096) g = 4096;
    if (p16)
      fa_bwd_reduce_kv_rope_kernel<true><<<g, 256, 0, st>>>(dkp, dvp, (bf16_t*)dqkv, B, S, H, KVH, rcos, rsin);
    else
      fa_bwd_reduce_kv_rope_kernel<false><<<g, 256, 0, st>>>(dkp, dvp, (bf16_t*)dqkv, B, S, H, KVH, rcos, rsin);
    DSA_CHECK(hipGetLastError());
    return join();
  }
  const long work = (long)B * S * KVH * (HD / 8);
  int g = (int)((work + 255) / 256);
  if (g > 4096) g = 4096;
  if (p16)
    fa_bwd_reduce_kv_kernel<true><<<g, 256, 0, st>>>(dkp, dvp, (bf16_t*)dqkv, B, S, H, KVH);
  else
    fa_bwd_reduce_kv_kernel<false><<<g, 256, 0, st>>>(dkp, dvp, (bf16_t*)dqkv, B, S, H, KVH);
  DSA_CHECK(hipGetLastError());
  DSA_CHECK(join());
  return rope_after();
}

// Diagnostic: one causal dK/dV pass (8-wave kernel) with waves 0 and 4 of workgroup 0 stamping 5
// points of q-tiles 8..11 (trace [2][64] int64; index (tile - 8) * 5 + point).
extern "C" hipError_t dsa_fa_dkdv_trace(const void* qkv, const void* dout, const float* lse, const float* delta,
                                        float* dkp, float* dvp, unsigned long long* trace, int B, int S, int H,
                                        int KVH, float sl2, hipStream_t st) {
  if (S % 128) return hipErrorInvalidValue;
  const char* dec = getenv("DSTACK_AMD_FA_DKDV_DEC");
  if (dec && atoi(dec) >= 1) {  // the decoupled-halves form: stamp 4 is after the half's rendezvous
    const char* sg = getenv("DSTACK_AMD_FA_DKDV_STAG");
    const size_t lds_dec = 2 * 128 * 256 + 4 * (2 * 32 * 256 + 512) + 16;
    if (atoi(dec) == 2)
      fa_bwd_dkdv8d_kernel<true, true, true><<<B * H * (S / 128), 512, lds_dec, st>>>(
          (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, dkp, dvp, B, S, H, KVH, sl2, sg ? atoi(sg) : 0, trace);
    else
      fa_bwd_dkdv8d_kernel<true, true><<<B * H * (S / 128), 512, lds_dec, st>>>(
          (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, dkp, dvp, B, S, H, KVH, sl2, sg ? atoi(sg) : 0, trace);
    return hipGetLastError();
  }
  const size_t lds8 = 2 * 128 * 256 + 2 * (2 * TILE_BYTES + 512);
  fa_bwd_dkdv8_kernel<true, false, false, false, false, true, 2><<<B * H * (S / 128), 512, lds8, st>>>(
      (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, dkp, dvp, B, S, H, KVH, sl2, (bf16_t*)trace);
  return hipGetLastError();
}
