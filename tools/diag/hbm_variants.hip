// HBM copy variants (1 GiB -> 1 GiB) to pick the health probe's streaming kernel.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f4 __attribute__((ext_vector_type(4)));
#define CK(x) do { if ((x) != hipSuccess) { printf("err %d\n", __LINE__); return 1; } } while (0)
template <int MODE>
__global__ __launch_bounds__(256) void copy(const f4* __restrict__ s, f4* __restrict__ d, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  if (MODE == 0) {  // plain grid-stride, 1 per iter
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride) d[i] = s[i];
  } else if (MODE == 1) {  // nt load, plain store
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride) d[i] = __builtin_nontemporal_load(s + i);
  } else if (MODE == 2) {  // one element per thread, full grid
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < n) d[i] = s[i];
  } else if (MODE == 3) {  // block-contiguous chunks: each block copies a contiguous 64 KiB span
    const size_t per = 4096;  // f4 per block
    size_t base = (size_t)blockIdx.x * per;
    for (size_t k = threadIdx.x; k < per && base + k < n; k += 256) d[base + k] = s[base + k];
  } else {  // 4 plain loads in flight
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
      f4 a = s[i], b = s[i + stride], c = s[i + 2 * stride], e = s[i + 3 * stride];
      d[i] = a; d[i + stride] = b; d[i + 2 * stride] = c; d[i + 3 * stride] = e;
    }
    for (; i < n; i += stride) d[i] = s[i];
  }
}
template <int MODE>
float run(const f4* a, f4* b, size_t n, int grid) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  copy<MODE><<<grid, 256>>>(a, b, n);
  hipEventRecord(e0);
  for (int r = 0; r < 20; ++r) copy<MODE><<<grid, 256>>>(a, b, n);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return 2.0 * n * 16 * 20 / (ms * 1e-3) / 1e12;
}
int main() {
  size_t bytes = 1ull << 30, n = bytes / 16;
  f4 *a, *b; CK(hipMalloc(&a, bytes)); CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 1, bytes));
  int cus = 256;
  printf("plain gs 8/CU  %.2f TB/s\n", run<0>(a, b, n, cus * 8));
  printf("plain gs 32/CU %.2f TB/s\n", run<0>(a, b, n, cus * 32));
  printf("nt-load gs 8/CU %.2f TB/s\n", run<1>(a, b, n, cus * 8));
  printf("1/thread full  %.2f TB/s\n", run<2>(a, b, n, (int)(n / 256)));
  printf("64KiB chunks   %.2f TB/s\n", run<3>(a, b, n, (int)(n / 4096)));
  printf("4x unroll 8/CU %.2f TB/s\n", run<4>(a, b, n, cus * 8));
  printf("4x unroll 4/CU %.2f TB/s\n", run<4>(a, b, n, cus * 4));
  return 0;
}
