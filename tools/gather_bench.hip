// gather_bench.hip -- practical HBM ceilings for the access patterns of the
// transfer path (run on the GPU box; not part of the product).
//
//   hipcc -O3 --offload-arch=gfx950 tools/gather_bench.hip -o /tmp/gather_bench
//   /tmp/gather_bench [GiB]
//
// stream   : coalesced 16 B/lane reads of the whole array
// line     : 8 lanes read one random 128-B line (16 B each): random full lines
// rec32    : each lane reads one random 32-B record (2 x 16 B): a walk gather
// rec32x4  : 4 consecutive lanes read 4 consecutive 32-B records of a random
//            128-B line (a spatially local gather)
// Bytes are counted as requested bytes; one JSON line per pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}

__global__ void k_stream(const uint4 *a, int64_t n, unsigned *sink) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint4 v = a[i];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) *sink = 1;
}

// PER lanes share one random line; each lane reads 16 B
template <int PER>
__global__ void k_line(const uint4 *a, int64_t nlines, int64_t reqs, unsigned *sink) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < reqs; r += (int64_t)gridDim.x * blockDim.x) {
    int64_t g = r / PER;
    int64_t line = (int64_t)(mix((uint64_t)g) % (uint64_t)nlines);
    uint4 v = a[line * 8 + (r % PER)];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) *sink = 1;
}

// each lane reads one 32-B record; GROUP consecutive lanes take consecutive
// records of one random line (GROUP = 1: independent random records)
template <int GROUP>
__global__ void k_rec32(const uint4 *a, int64_t nrec, int64_t reqs, unsigned *sink) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < reqs; r += (int64_t)gridDim.x * blockDim.x) {
    int64_t g = r / GROUP;
    int64_t base = (int64_t)(mix((uint64_t)g) % (uint64_t)(nrec / 4)) * 4;
    int64_t rec = GROUP == 1 ? (int64_t)(mix((uint64_t)r * 7 + 1) % (uint64_t)nrec) : base + (r % GROUP);
    uint4 v0 = a[rec * 2], v1 = a[rec * 2 + 1];
    acc.x ^= v0.x ^ v1.x; acc.y ^= v0.y ^ v1.y; acc.z ^= v0.z ^ v1.z; acc.w ^= v0.w ^ v1.w;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) *sink = 1;
}

int main(int argc, char **argv) {
  double gib = argc > 1 ? atof(argv[1]) : 4.0;
  int64_t bytes = (int64_t)(gib * (1LL << 30));
  int64_t n16 = bytes / 16;
  uint4 *a;
  unsigned *sink;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
  hipMemset(a, 1, bytes);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int nb = 256 * 32, bs = 256;
  auto run = [&](const char *name, auto launch, double moved) {
    launch();
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int it = 0; it < 5; it++) {
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    printf("{\"pattern\": \"%s\", \"GiB\": %.1f, \"ms\": %.4f, \"GBs\": %.1f}\n", name, gib, best,
           moved / (best * 1e-3) / 1e9);
    fflush(stdout);
  };
  run("stream", [&] { hipLaunchKernelGGL(k_stream, dim3(nb), dim3(bs), 0, 0, a, n16, sink); },
      (double)bytes);
  const int64_t nlines = bytes / 128;
  const int64_t reqs = n16 / 2;   // half the array's bytes per pattern
  run("line", [&] { hipLaunchKernelGGL(k_line<8>, dim3(nb), dim3(bs), 0, 0, a, nlines, reqs, sink); },
      (double)reqs * 16);
  run("rec32", [&] { hipLaunchKernelGGL(k_rec32<1>, dim3(nb), dim3(bs), 0, 0, a, bytes / 32, reqs / 2, sink); },
      (double)reqs * 16);
  run("rec32x4", [&] { hipLaunchKernelGGL(k_rec32<4>, dim3(nb), dim3(bs), 0, 0, a, bytes / 32, reqs / 2, sink); },
      (double)reqs * 16);
  hipFree(a);
  return 0;
}
