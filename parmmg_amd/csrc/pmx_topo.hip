// pmx_topo.hip -- background-mesh topology on gfx950.
//
// pmx_build_adja  <- MMG3D_hashTetra's face adjacency (Mmg; called by ParMmg
//                    at src/libparmmg1.c:272, src/distributemesh_pmmg.c:1185,
//                    src/metis_pmmg.c:756, ...): adja[4*(k-1)+1+f] = 4*k'+f'
// pmx_build_bdry  <- MMG5_chkBdryTria + MMG3D_hashTria on the old-group
//                    snapshot (src/grpsplit_pmmg.c:400-414): boundary trias
//                    of the faces without a neighbour, in (tet, face) order,
//                    vertices in MMG5_idir order, and their edge adjacency
//                    adjt[3*(k-1)+1+e] = 3*k'+e'
//
// Hash-free face matching: every face (edge) record goes to the bucket of its
// smallest vertex (count, exclusive scan, scatter); a face's partner is the
// record of the same bucket with the same two other vertices.  Buckets hold
// ~4 ne / np ~ 24 faces, the threads of one bucket are adjacent and read its
// records together.  The result does not depend on the order inside a bucket:
// an interior face of a valid mesh has exactly one partner (a face with more
// than one is non-manifold: reported, left 0, like the CPU builders of
// parmmg_amd/csrc/meshgen.c that the tests compare against).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>
#include "pmx_internal.h"

static unsigned nblk_(int64_t n) { return (unsigned)std::max<int64_t>((n + 255) / 256, 1); }

// MMG5_idir: local vertices of face f (opposite vertex f), outward order
__constant__ int TOPO_IDIR[4][3] = {{1, 2, 3}, {0, 3, 2}, {0, 1, 3}, {0, 2, 1}};

__device__ __forceinline__ void sort3i(int &a, int &b, int &c) {
  int t;
  if (a > b) { t = a; a = b; b = t; }
  if (b > c) { t = b; b = c; c = t; }
  if (a > b) { t = a; a = b; b = t; }
}

// ---- tet faces -------------------------------------------------------------------

// One thread per tet (its 4 faces), the faces of a workgroup aggregated per
// bucket (smallest vertex) in an LDS hash table: one global atomic per
// distinct bucket and workgroup instead of one per face (the neighbouring
// tets of a workgroup share most of their vertices; per-face atomics cost
// 3.7 ms of 4.4 at 10M tets).
#define FACE_HT 2048
__device__ __forceinline__ void face_key(const int4 t, int f, int &a, int &b, int &c) {
  const int v[4] = {t.x, t.y, t.z, t.w};
  a = v[TOPO_IDIR[f][0]];
  b = v[TOPO_IDIR[f][1]];
  c = v[TOPO_IDIR[f][2]];
  sort3i(a, b, c);
}
// slot of key a (inserted if absent); the table holds < FACE_HT / 2 keys
__device__ __forceinline__ int ht_slot(int *keys, int a) {
  unsigned h = ((unsigned)a * 2654435761u) >> (32 - 11);
  for (;;) {
    const int old = atomicCAS(&keys[h], -1, a);
    if (old == -1 || old == a) return (int)h;
    h = (h + 1) & (FACE_HT - 1);
  }
}

__global__ __launch_bounds__(256) void k_face_count(const int4 *__restrict__ tv, int64_t ne,
                                                    unsigned *__restrict__ cnt) {
  __shared__ int keys[FACE_HT];
  __shared__ unsigned cnts[FACE_HT];
  for (int i = threadIdx.x; i < FACE_HT; i += blockDim.x) { keys[i] = -1; cnts[i] = 0u; }
  __syncthreads();
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + 1;
  if (k <= ne) {
    const int4 t = tv[k];
    if (t.x > 0) {                               // !MG_EOK: no faces
      for (int f = 0; f < 4; f++) {
        int a, b, c;
        face_key(t, f, a, b, c);
        atomicAdd(&cnts[ht_slot(keys, a)], 1u);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < FACE_HT; i += blockDim.x)
    if (keys[i] >= 0) atomicAdd(cnt + keys[i], cnts[i]);
}

__global__ __launch_bounds__(256) void k_face_scatter(const int4 *__restrict__ tv, int64_t ne,
                                                      unsigned *__restrict__ cursor,
                                                      int4 *__restrict__ rec) {
  __shared__ int keys[FACE_HT];
  __shared__ unsigned cnts[FACE_HT];
  for (int i = threadIdx.x; i < FACE_HT; i += blockDim.x) { keys[i] = -1; cnts[i] = 0u; }
  __syncthreads();
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + 1;
  int4 t = make_int4(0, 0, 0, 0);
  int slot[4] = {0, 0, 0, 0};
  unsigned rank[4] = {0u, 0u, 0u, 0u};
  if (k <= ne) {
    t = tv[k];
    if (t.x > 0) {
      for (int f = 0; f < 4; f++) {
        int a, b, c;
        face_key(t, f, a, b, c);
        slot[f] = ht_slot(keys, a);
        rank[f] = atomicAdd(&cnts[slot[f]], 1u);   // place inside the workgroup's run
      }
    }
  }
  __syncthreads();
  // one reservation per bucket: the workgroup's run starts there
  for (int i = threadIdx.x; i < FACE_HT; i += blockDim.x)
    if (keys[i] >= 0) cnts[i] = atomicAdd(cursor + keys[i], cnts[i]);
  __syncthreads();
  if (k <= ne && t.x > 0) {
    for (int f = 0; f < 4; f++) {
      int a, b, c;
      face_key(t, f, a, b, c);
      rec[cnts[slot[f]] + rank[f]] = make_int4(a, b, c, (int)(4 * k + f));
    }
  }
}

// one thread per record: its partner in the bucket of its smallest vertex
__global__ __launch_bounds__(256) void k_face_match(const int4 *__restrict__ rec, int64_t nb,
                                                    const unsigned *__restrict__ off,
                                                    int *__restrict__ adja,
                                                    unsigned *__restrict__ nbad) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= (int64_t)off[nb]) return;                // records of valid tets only
  const int4 me = rec[s];
  const unsigned lo = off[me.x], hi = off[me.x + 1];
  int partner = 0, n = 0;
  for (unsigned r = lo; r < hi; r++) {
    const int4 o = rec[r];
    if (r != (unsigned)s && o.y == me.y && o.z == me.z) { partner = o.w; n++; }
  }
  adja[me.w - 3] = (n == 1) ? partner : 0;       // 4*(k-1)+1+f = owner - 3
  if (n > 1) atomicAdd(nbad, 1u);
}

// The same matching with the records staged in LDS: a workgroup owns
// MATCH_R consecutive records and loads them with MATCH_PAD records on either
// side (coalesced, 16 KB); a record whose bucket lies inside that window is
// compared against the LDS copy, any other (a bucket longer than the pads)
// against global memory.  One global read per record and window instead of
// one per (record, bucket member): the global-scan variant re-reads every
// bucket once per member (~24 x 16 B per record).
#define MATCH_R 512
#define MATCH_PAD 256
__global__ __launch_bounds__(256) void k_face_match_lds(const int4 *__restrict__ rec, int64_t nb,
                                                        const unsigned *__restrict__ off,
                                                        int *__restrict__ adja,
                                                        unsigned *__restrict__ nbad) {
  __shared__ int4 win[MATCH_R + 2 * MATCH_PAD];
  const int64_t nrec = (int64_t)off[nb];
  const int64_t s0 = (int64_t)blockIdx.x * MATCH_R;
  const int64_t w0 = s0 - MATCH_PAD;              // window start (may be negative)
  for (int i = threadIdx.x; i < MATCH_R + 2 * MATCH_PAD; i += blockDim.x) {
    const int64_t r = w0 + i;
    win[i] = (r >= 0 && r < nrec) ? rec[r] : make_int4(-1, -1, -1, 0);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < MATCH_R; j += blockDim.x) {
    const int64_t s = s0 + j;
    if (s >= nrec) break;
    const int4 me = win[MATCH_PAD + j];
    const int64_t lo = off[me.x], hi = off[me.x + 1];
    int partner = 0, n = 0;
    if (lo >= w0 && hi <= w0 + MATCH_R + 2 * MATCH_PAD) {
      for (int64_t r = lo; r < hi; r++) {
        const int4 o = win[r - w0];
        if (r != s && o.y == me.y && o.z == me.z) { partner = o.w; n++; }
      }
    } else {
      for (int64_t r = lo; r < hi; r++) {
        const int4 o = rec[r];
        if (r != s && o.y == me.y && o.z == me.z) { partner = o.w; n++; }
      }
    }
    adja[me.w - 3] = (n == 1) ? partner : 0;
    if (n > 1) atomicAdd(nbad, 1u);
  }
}

// PMX_TOPO_MATCH=global: the global-scan matching, for the A/B
static bool topo_match_global() {
  static const bool g = [] {
    const char *e = getenv("PMX_TOPO_MATCH");
    return e && std::string(e) == "global";
  }();
  return g;
}
static void launch_face_match(const int4 *rec, int64_t ne, int64_t np, const unsigned *off, int *dadja,
                              unsigned *nbad, hipStream_t s) {
  if (topo_match_global())
    hipLaunchKernelGGL(k_face_match, dim3(nblk_(4 * ne)), dim3(256), 0, s, rec, np + 1, off, dadja, nbad);
  else
    hipLaunchKernelGGL(k_face_match_lds, dim3((unsigned)std::max<int64_t>((4 * ne + MATCH_R - 1) / MATCH_R, 1)),
                       dim3(256), 0, s, rec, np + 1, off, dadja, nbad);
}

// ---- boundary trias and their edge adjacency -------------------------------------

__global__ __launch_bounds__(256) void k_bdry_count(const int4 *__restrict__ tv,
                                                    const int *__restrict__ adja, int64_t ne,
                                                    unsigned *__restrict__ cnt) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + 1;
  if (k > ne) return;
  unsigned c = 0;
  if (tv[k].x > 0) {                              // !MG_EOK tets have no faces
#pragma unroll
    for (int f = 0; f < 4; f++) c += adja[4 * (k - 1) + 1 + f] == 0 ? 1u : 0u;
  }
  cnt[k - 1] = c;
}

__global__ __launch_bounds__(256) void k_bdry_write(const int4 *__restrict__ tv,
                                                    const int *__restrict__ adja, int64_t ne,
                                                    const unsigned *__restrict__ pos,
                                                    int *__restrict__ tria) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + 1;
  if (k > ne) return;
  const int4 t = tv[k];
  if (t.x <= 0) return;
  const int v[4] = {t.x, t.y, t.z, t.w};
  int64_t p = pos[k - 1] + 1;                    // 1-based tria index, (k, f) order
  for (int f = 0; f < 4; f++) {
    if (adja[4 * (k - 1) + 1 + f]) continue;
    tria[3 * p + 0] = v[TOPO_IDIR[f][0]];
    tria[3 * p + 1] = v[TOPO_IDIR[f][1]];
    tria[3 * p + 2] = v[TOPO_IDIR[f][2]];
    p++;
  }
}

// edge e of tria k joins its vertices (e+1)%3 and (e+2)%3
__global__ __launch_bounds__(256) void k_edge_count(const int *__restrict__ tria, int64_t nt,
                                                    unsigned *__restrict__ cnt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // 3(k-1)+e
  if (i >= 3 * nt) return;
  const int64_t k = i / 3 + 1;
  const int e = (int)(i % 3);
  const int a = tria[3 * k + (e + 1) % 3], b = tria[3 * k + (e + 2) % 3];
  atomicAdd(cnt + min(a, b), 1u);
}

__global__ __launch_bounds__(256) void k_edge_scatter(const int *__restrict__ tria, int64_t nt,
                                                      unsigned *__restrict__ cursor,
                                                      int2 *__restrict__ rec) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 3 * nt) return;
  const int64_t k = i / 3 + 1;
  const int e = (int)(i % 3);
  const int a = tria[3 * k + (e + 1) % 3], b = tria[3 * k + (e + 2) % 3];
  const unsigned s = atomicAdd(cursor + min(a, b), 1u);
  rec[s] = make_int2(max(a, b), (int)(3 * k + e));
}

__global__ __launch_bounds__(256) void k_edge_match(const int2 *__restrict__ rec, int64_t nrec,
                                                    const unsigned *__restrict__ off,
                                                    const int *__restrict__ bucket_of,
                                                    int *__restrict__ adjt) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nrec) return;
  const int2 me = rec[s];
  const int a = bucket_of[s];
  const unsigned lo = off[a], hi = off[a + 1];
  int partner = 0, n = 0;
  for (unsigned r = lo; r < hi; r++) {
    const int2 o = rec[r];
    if (r != (unsigned)s && o.x == me.x) { partner = o.y; n++; }
  }
  adjt[me.y - 2] = (n == 1) ? partner : 0;       // 3*(k-1)+1+e = owner - 2
}

// bucket index of every record (the records of bucket a fill [off[a], off[a+1]))
__global__ __launch_bounds__(256) void k_bucket_of(const unsigned *__restrict__ off, int64_t nb,
                                                   int *__restrict__ bucket_of) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= nb) return;
  for (unsigned r = off[a]; r < off[a + 1]; r++) bucket_of[r] = (int)a;
}

// ---- host side ---------------------------------------------------------------------

namespace {

struct Scratch {
  std::vector<void *> p;
  ~Scratch() {
    for (void *q : p) hipFree(q);
  }
  template <class T> T *get(size_t n) {
    void *q = nullptr;
    if (hipMalloc(&q, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) return nullptr;
    p.push_back(q);
    return (T *)q;
  }
};

unsigned nblk(int64_t n) { return (unsigned)std::max<int64_t>((n + 255) / 256, 1); }

// exclusive scan of n counts into off[0..n] (off[n] = total)
bool scan_counts(const unsigned *cnt, unsigned *off, int64_t n, hipStream_t s, Scratch &sc) {
  size_t bytes = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, cnt, off, (int)(n + 1), s);
  void *tmp = sc.get<char>(bytes);
  if (!tmp) return false;
  return hipcub::DeviceScan::ExclusiveSum(tmp, bytes, cnt, off, (int)(n + 1), s) == hipSuccess;
}

// strided host connectivity -> device int4 stream (1-based, slot 0 zero)
int4 *upload_tets(pmx_ctx *ctx, int64_t ne, int64_t np, const int *tetra_v, int64_t stride,
                  Scratch &sc) {
  std::vector<int4> h((size_t)(ne + 1));
  h[0] = make_int4(0, 0, 0, 0);
  const char *tc = (const char *)tetra_v;
  for (int64_t k = 1; k <= ne; k++) {
    const int *v = (const int *)(tc + k * stride);
    if (v[0] <= 0) { h[(size_t)k] = make_int4(0, 0, 0, 0); continue; }   // !MG_EOK
    for (int l = 0; l < 4; l++)
      if (v[l] < 1 || v[l] > np) {
        ctx->err = "topology: tet vertex index out of range";
        return nullptr;
      }
    h[(size_t)k] = make_int4(v[0], v[1], v[2], v[3]);
  }
  int4 *d = sc.get<int4>(h.size());
  if (!d) return nullptr;
  if (hipMemcpyAsync(d, h.data(), h.size() * sizeof(int4), hipMemcpyHostToDevice, ctx->stream) !=
      hipSuccess)
    return nullptr;
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) return nullptr;
  return d;
}

bool topo_fail(pmx_ctx *ctx, const char *what) {
  ctx->err = what;
  return false;
}

// device adjacency from the device connectivity stream
bool build_adja_dev(pmx_ctx *ctx, const int4 *tv, int64_t ne, int64_t np, int *dadja, Scratch &sc,
                    unsigned *nbad_out) {
  hipStream_t s = ctx->stream;
  unsigned *cnt = sc.get<unsigned>((size_t)(np + 2));
  unsigned *off = sc.get<unsigned>((size_t)(np + 2));
  int4 *rec = sc.get<int4>((size_t)(4 * ne));
  unsigned *nbad = sc.get<unsigned>(1);
  if (!cnt || !off || !rec || !nbad) return topo_fail(ctx, "pmx_build_adja: hipMalloc");
  hipMemsetAsync(cnt, 0, sizeof(unsigned) * (size_t)(np + 2), s);
  hipMemsetAsync(nbad, 0, sizeof(unsigned), s);
  hipMemsetAsync(dadja, 0, sizeof(int) * (size_t)(4 * ne + 5), s);
  hipLaunchKernelGGL(k_face_count, dim3(nblk(ne)), dim3(256), 0, s, tv, ne, cnt);
  if (!scan_counts(cnt, off, np + 1, s, sc)) return topo_fail(ctx, "pmx_build_adja: scan");
  hipMemcpyAsync(cnt, off, sizeof(unsigned) * (size_t)(np + 2), hipMemcpyDeviceToDevice, s);
  hipLaunchKernelGGL(k_face_scatter, dim3(nblk(ne)), dim3(256), 0, s, tv, ne, cnt, rec);
  launch_face_match(rec, ne, np, off, dadja, nbad, s);
  if (hipMemcpyAsync(nbad_out, nbad, sizeof(unsigned), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return topo_fail(ctx, "pmx_build_adja: launch");
  return true;
}

}  // namespace



// face adjacency of a device connectivity stream with the context's buffers
// (promoted backgrounds: the new tets are already on the device)
bool pmx_ctx_build_adja_device(pmx_ctx *ctx, const int4 *tv, int64_t ne, int64_t np, int *dadja,
                               hipStream_t s, unsigned *h_nbad) {
  size_t bytes = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const unsigned *)nullptr, (unsigned *)nullptr,
                                   (int)(np + 2), s);
  if (!pmx_dgrow(ctx, ctx->d_tcnt, (size_t)(np + 2)) || !pmx_dgrow(ctx, ctx->d_toff, (size_t)(np + 2)) ||
      !pmx_dgrow(ctx, ctx->d_trec, (size_t)(4 * ne)) || !pmx_dgrow(ctx, ctx->d_tbad, 1) ||
      !pmx_dgrow(ctx, ctx->d_ttmp, bytes))
    return false;
  unsigned *cnt = ctx->d_tcnt.p, *off = ctx->d_toff.p, *nbad = ctx->d_tbad.p;
  bool okk = hipMemsetAsync(cnt, 0, sizeof(unsigned) * (size_t)(np + 2), s) == hipSuccess &&
             hipMemsetAsync(nbad, 0, sizeof(unsigned), s) == hipSuccess &&
             hipMemsetAsync(dadja, 0, sizeof(int) * (size_t)(4 * ne + 5), s) == hipSuccess;
  if (!okk) return topo_fail(ctx, "device adjacency: memset");
  hipLaunchKernelGGL(k_face_count, dim3(nblk(ne)), dim3(256), 0, s, tv, ne, cnt);
  if (hipcub::DeviceScan::ExclusiveSum(ctx->d_ttmp.p, bytes, cnt, off, (int)(np + 2), s) != hipSuccess)
    return topo_fail(ctx, "device adjacency: scan");
  hipMemcpyAsync(cnt, off, sizeof(unsigned) * (size_t)(np + 2), hipMemcpyDeviceToDevice, s);
  hipLaunchKernelGGL(k_face_scatter, dim3(nblk(ne)), dim3(256), 0, s, tv, ne, cnt, ctx->d_trec.p);
  launch_face_match(ctx->d_trec.p, ne, np, off, dadja, nbad, s);
  if (h_nbad) {
    if (hipMemcpyAsync(h_nbad, nbad, sizeof(unsigned), hipMemcpyDeviceToHost, s) != hipSuccess)
      return topo_fail(ctx, "device adjacency: launch");
    return true;
  }
  unsigned hb = 0;
  if (hipMemcpyAsync(&hb, nbad, sizeof(unsigned), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return topo_fail(ctx, "device adjacency: launch");
  if (hb) return topo_fail(ctx, "device adjacency: non-manifold tet faces");
  return true;
}

extern "C" {

int pmx_build_adja(pmx_ctx *ctx, int64_t ne, int64_t np, const int *tetra_v, int64_t tetra_stride,
                   int *adja) {
  if (!ctx || !tetra_v || !adja || ne < 1 || np < 1 || 4 * ne >= (1LL << 31)) {
    if (ctx) ctx->err = "pmx_build_adja: bad arguments";
    return 0;
  }
  hipSetDevice(ctx->device);
  Scratch sc;
  int4 *tv = upload_tets(ctx, ne, np, tetra_v, tetra_stride, sc);
  if (!tv) return 0;                             // pmx_last_error says why
  int *dadja = sc.get<int>((size_t)(4 * ne + 5));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, ctx->stream);
  unsigned nbad = 0;
  const bool ok = dadja && build_adja_dev(ctx, tv, ne, np, dadja, sc, &nbad);
  hipEventRecord(e1, ctx->stream);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  ctx->topo_ms = ms;
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  if (!ok) return 0;
  if (hipMemcpy(adja, dadja, sizeof(int) * (size_t)(4 * ne + 5), hipMemcpyDeviceToHost) != hipSuccess)
    return topo_fail(ctx, "pmx_build_adja: download"), 0;
  if (nbad) return topo_fail(ctx, "pmx_build_adja: non-manifold tet faces (left 0)"), 0;
  return 1;
}

int64_t pmx_build_bdry(pmx_ctx *ctx, int64_t ne, int64_t np, const int *tetra_v,
                       int64_t tetra_stride, const int *adja, int *tria, int64_t maxnt, int *adjt) {
  if (!ctx || !tetra_v || !adja || !tria || ne < 1 || np < 1) {
    if (ctx) ctx->err = "pmx_build_bdry: bad arguments";
    return -1;
  }
  hipSetDevice(ctx->device);
  hipStream_t s = ctx->stream;
  Scratch sc;
  int4 *tv = upload_tets(ctx, ne, np, tetra_v, tetra_stride, sc);
  int *dadja = sc.get<int>((size_t)(4 * ne + 5));
  unsigned *tcnt = sc.get<unsigned>((size_t)(ne + 1));
  unsigned *tpos = sc.get<unsigned>((size_t)(ne + 1));
  if (!tv || !dadja || !tcnt || !tpos) return topo_fail(ctx, "pmx_build_bdry: hipMalloc"), -1;
  hipMemcpyAsync(dadja, adja, sizeof(int) * (size_t)(4 * ne + 5), hipMemcpyHostToDevice, s);
  hipMemsetAsync(tcnt, 0, sizeof(unsigned) * (size_t)(ne + 1), s);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, s);
  hipLaunchKernelGGL(k_bdry_count, dim3(nblk(ne)), dim3(256), 0, s, tv, dadja, ne, tcnt);
  if (!scan_counts(tcnt, tpos, ne, s, sc)) return topo_fail(ctx, "pmx_build_bdry: scan"), -1;
  unsigned nt_u = 0;
  hipMemcpyAsync(&nt_u, tpos + ne, sizeof(unsigned), hipMemcpyDeviceToHost, s);
  hipStreamSynchronize(s);
  const int64_t nt = nt_u;
  if (nt > maxnt) return topo_fail(ctx, "pmx_build_bdry: more boundary faces than maxnt"), -1;
  int *dtria = sc.get<int>((size_t)(3 * (nt + 1)));
  if (!dtria) return topo_fail(ctx, "pmx_build_bdry: hipMalloc"), -1;
  hipMemsetAsync(dtria, 0, sizeof(int) * 3, s);
  hipLaunchKernelGGL(k_bdry_write, dim3(nblk(ne)), dim3(256), 0, s, tv, dadja, ne, tpos, dtria);
  int *dadjt = nullptr;
  if (adjt && nt > 0) {
    unsigned *cnt = sc.get<unsigned>((size_t)(np + 2));
    unsigned *off = sc.get<unsigned>((size_t)(np + 2));
    int2 *rec = sc.get<int2>((size_t)(3 * nt));
    int *bof = sc.get<int>((size_t)(3 * nt));
    dadjt = sc.get<int>((size_t)(3 * nt + 4));
    if (!cnt || !off || !rec || !bof || !dadjt) return topo_fail(ctx, "pmx_build_bdry: hipMalloc"), -1;
    hipMemsetAsync(cnt, 0, sizeof(unsigned) * (size_t)(np + 2), s);
    hipMemsetAsync(dadjt, 0, sizeof(int) * (size_t)(3 * nt + 4), s);
    hipLaunchKernelGGL(k_edge_count, dim3(nblk(3 * nt)), dim3(256), 0, s, dtria, nt, cnt);
    if (!scan_counts(cnt, off, np + 1, s, sc)) return topo_fail(ctx, "pmx_build_bdry: scan"), -1;
    hipMemcpyAsync(cnt, off, sizeof(unsigned) * (size_t)(np + 2), hipMemcpyDeviceToDevice, s);
    hipLaunchKernelGGL(k_edge_scatter, dim3(nblk(3 * nt)), dim3(256), 0, s, dtria, nt, cnt, rec);
    hipLaunchKernelGGL(k_bucket_of, dim3(nblk(np + 1)), dim3(256), 0, s, off, np + 1, bof);
    hipLaunchKernelGGL(k_edge_match, dim3(nblk(3 * nt)), dim3(256), 0, s, rec, 3 * nt, off, bof,
                       dadjt);
  }
  hipEventRecord(e1, s);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  ctx->topo_ms = ms;
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  if (hipGetLastError() != hipSuccess) return topo_fail(ctx, "pmx_build_bdry: launch"), -1;
  if (hipMemcpy(tria, dtria, sizeof(int) * (size_t)(3 * (nt + 1)), hipMemcpyDeviceToHost) != hipSuccess)
    return topo_fail(ctx, "pmx_build_bdry: download"), -1;
  if (dadjt &&
      hipMemcpy(adjt, dadjt, sizeof(int) * (size_t)(3 * nt + 4), hipMemcpyDeviceToHost) != hipSuccess)
    return topo_fail(ctx, "pmx_build_bdry: download"), -1;
  return nt;
}

double pmx_topo_ms(pmx_ctx *ctx) { return ctx ? ctx->topo_ms : -1.0; }

}  // extern "C"
