// lane_bench.hip -- what bounds a divergent gather: bytes, lines or lane
// addresses?  (GPU box tool, not part of the product.)
//
//   hipcc -O3 --offload-arch=gfx950 tools/lane_bench.hip -o /tmp/lane_bench
//   /tmp/lane_bench
//
// Every lane issues LOADS dependent-free loads per iteration from a table of
// T bytes at pseudo-random positions.  Patterns (per wave instruction):
//   w<B>      : each lane B bytes (4/8/16) from its own random line
//   w16p<G>   : G consecutive lanes read consecutive 16-B pieces of one line
//   w32       : each lane a 32-B record as two 16-B loads (the walk's TetRec)
//   w24       : each lane a 24-B row (16 + 8, the walk's vertex)
// Reported: lane-accesses/s (one lane, one load instruction), requested GB/s,
// and lane-accesses per CU-cycle at 2.4 GHz.  Table sizes: 2 MiB (L2),
// 128 MiB (Infinity Cache), 4 GiB (HBM).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

__device__ __forceinline__ uint32_t hsh(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

#define ITERS 64

// B bytes per lane, G lanes share a line (G = 1: own line)
template <int B, int G>
__global__ __launch_bounds__(256) void k_gather(const uint8_t *__restrict__ a, uint32_t nlines,
                                                unsigned *sink) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  uint32_t s = hsh(t / G);
#pragma unroll 8
  for (int it = 0; it < ITERS; it++) {
    s = hsh(s + it);
    const uint32_t line = s % nlines;
    const uint8_t *p = a + (uint64_t)line * 128 + (uint64_t)((t % G) * B) % 128;
    if constexpr (B == 4) acc ^= *(const uint32_t *)p;
    else if constexpr (B == 8) { uint2 v = *(const uint2 *)p; acc ^= v.x ^ v.y; }
    else if constexpr (B == 16) { uint4 v = *(const uint4 *)p; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    else if constexpr (B == 32) {
      const uint4 *q = (const uint4 *)(a + (uint64_t)line * 128 + (uint64_t)((t % G) * 32) % 128);
      uint4 v = q[0], w = q[1];
      acc ^= v.x ^ v.y ^ v.z ^ v.w ^ w.x ^ w.y ^ w.z ^ w.w;
    } else if constexpr (B == 24) {
      // 24-B rows packed: row r at 24 r (may straddle a line)
      const uint64_t row = (uint64_t)s % ((uint64_t)nlines * 128 / 24 - 1);
      const uint8_t *r = a + row * 24;
      uint4 v = *(const uint4 *)r;   // unaligned 16 B: legal on gfx950
      uint2 w = *(const uint2 *)(r + 16);
      acc ^= v.x ^ v.y ^ v.z ^ v.w ^ w.x ^ w.y;
    }
  }
  if (acc == 0x12345678u) *sink = acc;
}

int main() {
  const uint64_t big = 4ull << 30;
  uint8_t *a;
  unsigned *sink;
  if (hipMalloc(&a, big) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
  hipMemset(a, 1, big);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int nb = 256 * 64, bs = 256;            // 16 waves per CU
  const double lanes = (double)nb * bs * ITERS;
  auto run = [&](const char *name, int loads_per_iter, int bytes_per_lane, uint64_t table, auto launch) {
    launch();
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      best = ms < best ? ms : best;
    }
    const double acc = lanes * loads_per_iter / (best * 1e-3);
    printf("{\"pattern\": \"%s\", \"table_MiB\": %llu, \"ms\": %.4f, \"Glane_acc_s\": %.1f, "
           "\"lane_acc_per_CU_clk\": %.3f, \"req_GBs\": %.1f}\n",
           name, (unsigned long long)(table >> 20), best, acc / 1e9, acc / 256 / 2.4e9,
           lanes * bytes_per_lane / (best * 1e-3) / 1e9);
    fflush(stdout);
  };
  const uint64_t tables[3] = {2ull << 20, 128ull << 20, big};
  for (uint64_t T : tables) {
    const uint32_t nl = (uint32_t)(T / 128);
#define RUN(NAME, B, G, L) \
    run(NAME, L, B, T, [&] { hipLaunchKernelGGL((k_gather<B, G>), dim3(nb), dim3(bs), 0, 0, a, nl, sink); })
    RUN("w4", 4, 1, 1);
    RUN("w8", 8, 1, 1);
    RUN("w16", 16, 1, 1);
    RUN("w16p2", 16, 2, 1);
    RUN("w16p4", 16, 4, 1);
    RUN("w16p8", 16, 8, 1);
    RUN("w32", 32, 1, 2);
    RUN("w32p4", 32, 4, 2);
    RUN("w24", 24, 1, 2);
  }
  hipFree(a);
  return 0;
}
