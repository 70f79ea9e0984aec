// The bench's synthetic token stream (workloads/data.py SyntheticLM) as one HIP kernel.
//
// Why a kernel of its own: generated with PyTorch ops, the stream's first batch in a fresh process
// paid 15-130 ms per op for the first use of PyTorch's elementwise kernels (their code objects are
// loaded from libtorch_hip on first launch; tools/diag/data_first_use.py, profiles/
// data_first_use_r9l.txt): 0.36-0.39 s of the applied task's first optimizer step
// (profiles/first_step_split_r9j.json), which is half of the headline metric's cold start.  This
// kernel lives in the extension the task has already loaded.
//
// The stream, per position i of the micro-batch's mb x (S + 1) tokens (key = the batch's
// (seed, index) key):
//   x0 = splitmix64(key ^ splitmix64(2i)), x1 = splitmix64(key ^ splitmix64(2i + 1))
//   u = (x0 >> 11) * 2^-53             -> z_i = perm[min(lower_bound(cdf, u), V - 1)]  (Zipf unigram)
//   copy_i = (x1 >> 40) * 2^-24 < p and i % (S + 1) != 0
//   last_i = max_{j <= i} (copy_j ? 0 : j)                       (the run's fresh sample)
//   x_i = (A^k z_last + B (1 + A + ... + A^(k-1))) mod V, k = i - last_i  (bigram chains)
// with A^k and the geometric sums precomputed mod V (pow_a, geo_b).  workloads/data.py holds the
// same definition in torch ops for CPU tensors; the GPU test checks the two agree bit for bit.
//
// One workgroup of 1024 threads: n = mb * (S + 1) is a few thousand to a few tens of thousands,
// the whole batch costs tens of microseconds, and the run-start prefix max is one block scan
// (pass 1 keeps (fresh index, z) per position in a workspace, pass 2 scans and writes x).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

constexpr int SYN_THREADS = 1024;
constexpr int SYN_MAX_N = 1 << 20;

__device__ __forceinline__ int64_t zipf_token(const double* __restrict__ cdf, const int64_t* __restrict__ perm,
                                              uint64_t key, int i, int V) {
  const uint64_t x0 = splitmix64(key ^ splitmix64(2ull * (uint64_t)i));
  const double u = (double)(x0 >> 11) * (1.0 / 9007199254740992.0);
  int lo = 0, hi = V;  // lower_bound: the first c with cdf[c] >= u
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cdf[mid] < u) lo = mid + 1;
    else hi = mid;
  }
  return perm[min(lo, V - 1)];
}

// ws [n] int64: pass 1 stores (fresh index or 0) << 32 | z_i; pass 2 scans the fresh indices (a
// contiguous chunk per thread, then a block scan of the chunk maxima) and writes the chain values.
__global__ __launch_bounds__(SYN_THREADS) void synthetic_tokens_kernel(
    const double* __restrict__ cdf, const int64_t* __restrict__ perm, const int64_t* __restrict__ pow_a,
    const int64_t* __restrict__ geo_b, int64_t* __restrict__ out, int64_t* __restrict__ ws, uint64_t key,
    float copy_p, int n, int row_len, int V) {
  __shared__ int wave_max[SYN_THREADS / 64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int i = tid; i < n; i += SYN_THREADS) {
    const uint64_t x1 = splitmix64(key ^ splitmix64(2ull * (uint64_t)i + 1ull));
    const float c = (float)(x1 >> 40) * (1.0f / 16777216.0f);
    const bool copy = c < copy_p && (i % row_len) != 0;
    ws[i] = ((int64_t)(copy ? 0 : i) << 32) | zipf_token(cdf, perm, key, i, V);
  }
  __syncthreads();
  const int per = (n + SYN_THREADS - 1) / SYN_THREADS;
  const int i0 = min(n, tid * per), i1 = min(n, i0 + per);
  int run = 0;
  for (int i = i0; i < i1; ++i) run = max(run, (int)(ws[i] >> 32));
  int incl = run;  // inclusive wave scan (max) of the chunk maxima
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o, 64);
    if (lane >= o) incl = max(incl, y);
  }
  if (lane == 63) wave_max[wv] = incl;
  __syncthreads();
  int before = 0;  // max over the chunks of every earlier thread
  for (int k = 0; k < wv; ++k) before = max(before, wave_max[k]);
  const int prev = __shfl_up(incl, 1, 64);
  if (lane > 0) before = max(before, prev);
  run = before;
  for (int i = i0; i < i1; ++i) {
    run = max(run, (int)(ws[i] >> 32));
    const int k = i - run;
    const int64_t zl = ws[run] & 0xffffffffll;
    out[i] = (pow_a[k] * zl + geo_b[k]) % V;
  }
}

}  // namespace

extern "C" hipError_t dsa_synthetic_tokens(const double* cdf, const int64_t* perm, const int64_t* pow_a,
                                           const int64_t* geo_b, int64_t* out, int64_t* ws, uint64_t key,
                                           float copy_p, int n, int row_len, int V, hipStream_t st) {
  if (n <= 0 || n > SYN_MAX_N || row_len <= 0 || V <= 0) return hipErrorInvalidValue;
  synthetic_tokens_kernel<<<1, SYN_THREADS, 0, st>>>(cdf, perm, pow_a, geo_b, out, ws, key, copy_p, n, row_len, V);
  return hipGetLastError();
}
