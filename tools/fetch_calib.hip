// fetch_calib.hip -- what FETCH_SIZE reports for the transfer path's access
// widths (GPU box tool, not part of the product).  Run under
//   rocprofv3 --pmc FETCH_SIZE -- /tmp/fetch_calib
// Each k_calib<B> launch reads B bytes at the start of every 128-B line of a
// 4 GiB table exactly once (line = t * odd mod 2^25, a bijection, so no line
// is read twice and neighbouring lanes read far-apart lines); a 1 GiB
// stream in between evicts the Infinity Cache.  Expected fabric bytes if
// whole lines move: 2^25 * 128 B = 4.29 GB per launch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int B>
__global__ __launch_bounds__(256) void k_calib(const uint8_t *__restrict__ a, unsigned *sink) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t line = (t * 0x9E3779B1u) & ((1u << 25) - 1);
  const uint8_t *p = a + (uint64_t)line * 128;
  uint32_t acc = 0;
  if constexpr (B == 8) { uint2 v = *(const uint2 *)p; acc = v.x ^ v.y; }
  else if constexpr (B == 16) { uint4 v = *(const uint4 *)p; acc = v.x ^ v.w; }
  else if constexpr (B == 24) { uint4 v = *(const uint4 *)p; uint2 w = *(const uint2 *)(p + 16); acc = v.x ^ w.y; }
  else if constexpr (B == 32) { uint4 v = *(const uint4 *)p, w = *(const uint4 *)(p + 16); acc = v.x ^ w.w; }
  else if constexpr (B == 64) {
#pragma unroll
    for (int k = 0; k < 4; k++) { uint4 v = *(const uint4 *)(p + 16 * k); acc ^= v.x ^ v.w; }
  } else {
#pragma unroll
    for (int k = 0; k < 8; k++) { uint4 v = *(const uint4 *)(p + 16 * k); acc ^= v.x ^ v.w; }
  }
  if (acc == 0x12345678u) *sink = acc;
}

__global__ void k_flush(const uint4 *__restrict__ a, int64_t n, unsigned *sink) {
  uint32_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    acc ^= a[i].x;
  if (acc == 0x12345678u) *sink = acc;
}

int main() {
  const uint64_t big = 4ull << 30, fl = 1ull << 30;
  uint8_t *a, *f;
  unsigned *sink;
  if (hipMalloc(&a, big) != hipSuccess || hipMalloc(&f, fl) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
  hipMemset(a, 1, big);
  hipMemset(f, 2, fl);
  const unsigned nb = (1u << 25) / 256;
  auto flush = [&] { hipLaunchKernelGGL(k_flush, dim3(8192), dim3(256), 0, 0, (const uint4 *)f, (int64_t)(fl / 16), sink); };
#define CAL(B) flush(); hipLaunchKernelGGL((k_calib<B>), dim3(nb), dim3(256), 0, 0, a, sink); hipDeviceSynchronize();
  for (int rep = 0; rep < 2; rep++) { CAL(8) CAL(16) CAL(24) CAL(32) CAL(64) CAL(128) }
  printf("fetch_calib done: %u lines per launch\n", 1u << 25);
  return 0;
}
