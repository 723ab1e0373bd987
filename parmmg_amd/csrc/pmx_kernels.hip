// pmx_kernels.hip -- gfx950 kernels of the transfer path (volume part).
//
// k_bg_derive        per-background derived data, one launch: fixed-point grid
//                    coordinates of the old vertices (hint centroids) and the
//                    unit normals of the boundary trias
//                    (PMMG_precompute_triaNormals, src/locate_pmmg.c:68-90)
// k_hint_build       uniform grid over the background bbox, cell -> a sampled
//                    tet whose centroid falls in it (the walk start)
// k_ties             near-face ties: canonical (smallest-index) containing tet
// k_fallback         LDS-staged exhaustive scan (smallest containing tet
//                    index == the reference's first hit in index order,
//                    src/locate_pmmg.c:737-770), closest tet (argmin of
//                    |lambda_min|*vol, src/barycoord_pmmg.c:371-404) and the
//                    interpolation of the scanned points, phases separated by
//                    a grid barrier that reports a timeout instead of hiding it
// The production walk itself is pmx_walk.hip.
#include <algorithm>
#include <hipcub/hipcub.hpp>
#include "pmx_device.h"
#include "pmx_kernels.h"
#include "pmx_transfer.h"

__device__ __forceinline__ int clampi(double t, int n) {
  if (!(t > 0.0)) return 0;                 // also catches NaN
  if (t >= (double)(n - 1)) return n - 1;
  return (int)t;
}

// ---- per-background derived data -----------------------------------------------

// grid coordinates of the vertices in fixed point (k_hint_build's centroids,
// the fixed-point walk of k_walkq): q = (x - lo) * inv * 2^qf, clamped to
// [0, dim * 2^qf - 1] (21 bits per axis), packed x | y << 21 | z << 42; and
// the tria normals + areas
// a vertex's grid coordinates in fixed point, packed x | y << 21 | z << 42
__device__ __forceinline__ unsigned long long quant_xyz(const double *c, const GridDesc &g) {
  unsigned long long r = 0;
#pragma unroll
  for (int a = 0; a < 3; a++) {
    const double t = (c[a] - g.lo[a]) * g.inv[a] * (double)(1 << g.qf[a]);
    const long long hi = ((long long)g.dim[a] << g.qf[a]) - 1;
    const long long u = !(t > 0.0) ? 0 : (t >= (double)hi ? hi : (long long)t);
    r |= (unsigned long long)u << (21 * a);
  }
  return r;
}

// Blocks [0, nbv) quantise the vertices, 256 pairs of rows (12 KB) per
// block iteration: three fully coalesced 16-B loads per thread into LDS, each
// thread then takes its two rows from LDS (r05: two rows per thread straight
// from HBM -- three 16-B loads at a 48-B lane stride -- ran at 4.2 TB/s,
// 0.128 ms at C3).  Blocks [nbv, nbv + nbt) form the tria normals.
__global__ __launch_bounds__(256) void k_bg_derive(const double *__restrict__ xyz, int64_t np, GridDesc g,
                                                   unsigned long long *__restrict__ q,
                                                   const TriRec *__restrict__ tris, int64_t nt,
                                                   Pt4 *__restrict__ trn, int nbv) {
  __shared__ double2 sh[3 * 256];
  auto quant = [&](const double *c) { return quant_xyz(c, g); };
  if ((int)blockIdx.x < nbv) {
    const int64_t npair = (np + 2) / 2;         // rows 0 .. np, two per pair
    const int64_t nfull = (np + 1) / 2;         // pairs with both rows
    for (int64_t b0 = (int64_t)blockIdx.x * 256; b0 < npair; b0 += (int64_t)nbv * 256) {
      const int64_t m = b0 + threadIdx.x;
      if (b0 + 256 <= nfull) {                  // block-uniform: a whole chunk
        const double2 *p = reinterpret_cast<const double2 *>(xyz + 6 * b0);
        sh[threadIdx.x] = p[threadIdx.x];
        sh[threadIdx.x + 256] = p[threadIdx.x + 256];
        sh[threadIdx.x + 512] = p[threadIdx.x + 512];
        __syncthreads();
        const double2 a = sh[3 * threadIdx.x], b = sh[3 * threadIdx.x + 1], c = sh[3 * threadIdx.x + 2];
        __syncthreads();
        const double c0[3] = {a.x, a.y, b.x}, c1[3] = {b.y, c.x, c.y};
        reinterpret_cast<ulonglong2 *>(q)[m] = make_ulonglong2(quant(c0), quant(c1));
      } else if (m < npair) {                   // the tail
        if (2 * m + 1 <= np) {
          const double2 *p = reinterpret_cast<const double2 *>(xyz + 6 * m);
          const double2 a = p[0], b = p[1], c = p[2];
          const double c0[3] = {a.x, a.y, b.x}, c1[3] = {b.y, c.x, c.y};
          reinterpret_cast<ulonglong2 *>(q)[m] = make_ulonglong2(quant(c0), quant(c1));
        } else {
          const double c0[3] = {xyz[6 * m], xyz[6 * m + 1], xyz[6 * m + 2]};
          q[2 * m] = quant(c0);
        }
      }
    }
    return;
  }
  const int64_t st = (int64_t)(gridDim.x - nbv) * blockDim.x;
  for (int64_t k = 1 + (int64_t)(blockIdx.x - nbv) * blockDim.x + threadIdx.x; k <= nt; k += st) {
    const TriRec t = tris[k];
    if (t.v[0] <= 0) { trn[k] = Pt4{0, 0, 0, 0}; continue; }
    const D3 n = nonunit_normal(ld3(xyz, t.v[0]), ld3(xyz, t.v[1]), ld3(xyz, t.v[2]));
    const double a = sqrt(n.x * n.x + n.y * n.y + n.z * n.z);
    const double dd = 1.0 / a;
    trn[k] = Pt4{n.x * dd, n.y * dd, n.z * dd, a};
  }
}
// PMX_DERIVE_BLOCKS (A/B): the vertex pass's block cap
static int64_t derive_blocks() {
  const char *e = getenv("PMX_DERIVE_BLOCKS");
  return e ? std::max<int64_t>(1, atoll(e)) : 8192;
}
void launch_bg_derive(const double *xyz, int64_t np, GridDesc g, unsigned long long *xyzq,
                      const TriRec *tris, int64_t nt, Pt4 *trn, hipStream_t s) {
  const int64_t npair = np > 0 ? (np + 2) / 2 : 0;
  const int nbv = (int)std::min<int64_t>((npair + 255) / 256, derive_blocks());
  const int nbt = (int)std::min<int64_t>((nt + 255) / 256, 4096);
  if (nbv + nbt < 1) return;
  hipLaunchKernelGGL(k_bg_derive, dim3((unsigned)(nbv + nbt)), dim3(256), 0, s, xyz, np, g, xyzq, tris, nt, trn,
                     nbv);
}

// ---- hint grid ---------------------------------------------------------------------

// One sample per thread; XCD-aware block order: each XCD's L2 serves a
// contiguous range of samples, i.e. neighbouring tets sharing vertices.  The
// centroid's cell comes from the vertices' fixed-point grid coordinates (one
// 8-B gather per vertex, integer sums and a shift, no FP; r01 same-box A/B on
// C3: 0.197 ms against 0.295 ms from the double coordinates).  Plain store:
// any sampled tet of the cell is a valid start, the located tet does not
// depend on the start (unique containing tet, or the canonical min-index tet
// of a tie, see canonical_tet).
// FROM_XYZ (run flag exp 15, A/B of the r04 verdict's "derive fused into
// the hint build"): the four vertices' fixed-point coordinates computed here
// from their double rows (the same quant_xyz, so the same cells) instead of
// gathered from the derived xyzq array -- no separate pass over the vertices
// V0 (run flag exp 16, A/B): the cell of the sample's first vertex instead
// of its centroid -- one 8-B gather per sample instead of four; any tet of
// the neighbourhood is a valid start (a longer walk at most)
// the cell of a tet's centroid from its vertices' fixed-point coordinates
__device__ __forceinline__ int64_t hint_cell(unsigned long long a, unsigned long long b, unsigned long long c,
                                             unsigned long long d, const GridDesc &g) {
  const unsigned long long M = (1ull << 21) - 1;
  int cq[3];
#pragma unroll
  for (int ax = 0; ax < 3; ax++) {
    const int sh = 21 * ax;
    const unsigned s4 = (unsigned)((a >> sh) & M) + (unsigned)((b >> sh) & M) +
                        (unsigned)((c >> sh) & M) + (unsigned)((d >> sh) & M);
    cq[ax] = min((int)(s4 >> (g.qf[ax] + 2)), g.dim[ax] - 1);
  }
  return gcell(g, cq[0], cq[1], cq[2]);
}

template <bool PACKED, bool FROM_XYZ = false, bool V0 = false, int BS = 256>
__global__ __launch_bounds__(BS) void k_hint_build(const int4 *__restrict__ packed, const int *__restrict__ kidx,
                                                    const TetRec *__restrict__ tets, int64_t n,
                                                    int stride, int *__restrict__ grid, GridDesc g,
                                                    const unsigned long long *__restrict__ xyzq,
                                                    const double *__restrict__ xyz) {
  const int64_t t = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (t >= n) return;
  // the packed sample in cell order carries its tet indices (kidx)
  const int64_t k = (PACKED && kidx) ? (int64_t)kidx[t] : 1 + t * stride;
  const int4 v = PACKED ? packed[t] : *reinterpret_cast<const int4 *>(tets + k);
  if (v.x <= 0) return;
  if constexpr (V0) {
    const unsigned long long a = xyzq[v.x];
    const unsigned long long M = (1ull << 21) - 1;
    int cq[3];
#pragma unroll
    for (int ax = 0; ax < 3; ax++) cq[ax] = min((int)(((a >> (21 * ax)) & M) >> g.qf[ax]), g.dim[ax] - 1);
    grid[gcell(g, cq[0], cq[1], cq[2])] = (int)k;
    return;
  }
  unsigned long long a, b, c, d;
  if constexpr (FROM_XYZ) {
    a = quant_xyz(xyz + 3 * (int64_t)v.x, g);
    b = quant_xyz(xyz + 3 * (int64_t)v.y, g);
    c = quant_xyz(xyz + 3 * (int64_t)v.z, g);
    d = quant_xyz(xyz + 3 * (int64_t)v.w, g);
  } else {
    a = xyzq[v.x]; b = xyzq[v.y]; c = xyzq[v.z]; d = xyzq[v.w];
  }
  grid[hint_cell(a, b, c, d, g)] = (int)k;
}
// PMX_HINT_FILT=1 (A/B, late r06): the same build with one grid store per
// run of samples in one cell -- a lane whose left neighbour's sample falls in
// its cell leaves the store to it (consecutive samples of a coherent
// numbering share cells; any sample of the cell is a valid start, and the
// left one is as good as the racy last writer)
__global__ __launch_bounds__(256) void k_hint_build_filt(const int4 *__restrict__ packed, int64_t n, int stride,
                                                         int *__restrict__ grid, GridDesc g,
                                                         const unsigned long long *__restrict__ xyzq) {
  const int64_t t = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  const int64_t k = 1 + t * stride;
  const int4 v = packed[t < n ? t : n - 1];
  int64_t c = -1;
  if (t < n && v.x > 0) c = hint_cell(xyzq[v.x], xyzq[v.y], xyzq[v.z], xyzq[v.w], g);
  const long long cl = __shfl_up((long long)c, 1, 64);
  if (c >= 0 && ((threadIdx.x & 63) == 0 || cl != (long long)c)) grid[c] = (int)k;
}
void launch_hint_build(const int4 *packed, const int *kidx, const TetRec *tets, int64_t ne, int stride, int *grid,
                       GridDesc g, const unsigned long long *xyzq, const double *xyz, hipStream_t s,
                       bool v0, int bs, int64_t nsamp) {
  const int64_t n = nsamp >= 0 ? nsamp : (ne + stride - 1) / stride;   // nsamp < 0: every stride-th tet
  if (n < 1) return;
  const int64_t nb = (n + 255) / 256;
  static const bool filt = [] {
    const char *e = getenv("PMX_HINT_FILT");
    return e && e[0] == '1';
  }();
  if (filt && packed && !kidx && xyzq && !v0 && bs == 256 && nsamp < 0 && n < INT32_MAX) {
    hipLaunchKernelGGL(k_hint_build_filt, dim3((unsigned)nb), dim3(256), 0, s, packed, n, stride, grid, g, xyzq);
    return;
  }
  if (v0 && xyzq && packed)
    hipLaunchKernelGGL((k_hint_build<true, false, true>), dim3((unsigned)nb), dim3(256), 0, s, packed, kidx, tets, n,
                       stride, grid, g, xyzq, xyz);
  else if (v0 && xyzq)
    hipLaunchKernelGGL((k_hint_build<false, false, true>), dim3((unsigned)nb), dim3(256), 0, s, packed, kidx, tets, n,
                       stride, grid, g, xyzq, xyz);
  else if (packed && !xyzq)
    hipLaunchKernelGGL((k_hint_build<true, true>), dim3((unsigned)nb), dim3(256), 0, s, packed, kidx, tets, n, stride,
                       grid, g, xyzq, xyz);
  else if (packed && bs == 1024)
    hipLaunchKernelGGL((k_hint_build<true, false, false, 1024>), dim3((unsigned)((n + 1023) / 1024)), dim3(1024), 0,
                       s, packed, kidx, tets, n, stride, grid, g, xyzq, xyz);
  else if (packed && bs == 64)
    hipLaunchKernelGGL((k_hint_build<true, false, false, 64>), dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s,
                       packed, kidx, tets, n, stride, grid, g, xyzq, xyz);
  else if (packed)
    hipLaunchKernelGGL((k_hint_build<true, false>), dim3((unsigned)nb), dim3(256), 0, s, packed, kidx, tets, n, stride,
                       grid, g, xyzq, xyz);
  else
    hipLaunchKernelGGL((k_hint_build<false, false>), dim3((unsigned)nb), dim3(256), 0, s, packed, kidx, tets, n, stride,
                       grid, g, xyzq, xyz);
}

// The vertex-owner sample (r05): one tet per vertex -- the smallest tet
// among those whose smallest vertex it is -- in vertex order.  Like the
// every-4th-tet sample it is connectivity only, but it covers space whatever
// the tet numbering (a random numbering's every-4th-tet sample leaves a
// Poisson share of the cells empty), and it has one entry per vertex instead
// of ne / 4.
// (a lane whose left neighbour -- the previous tet -- has the same smallest
// vertex skips its atomic: a coherent numbering puts a vertex's tets next to
// each other, and same-address atomics serialise; r05: 3.6 -> see DESIGN)
__global__ __launch_bounds__(256) void k_vmin_owner(const TetRec *__restrict__ tets, int64_t ne,
                                                    unsigned *__restrict__ owner) {
  const int64_t st = (int64_t)gridDim.x * blockDim.x;
  const int64_t nit = (ne + st - 1) / st;           // uniform trip count (the shuffle below)
  for (int64_t it = 0; it < nit; it++) {
    const int64_t k = 1 + it * st + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int m = -1;
    if (k <= ne) {
      const int4 v = *reinterpret_cast<const int4 *>(tets + k);
      if (v.x > 0) m = min(min(v.x, v.y), min(v.z, v.w));
    }
    const int ml = __shfl_up(m, 1, 64);
    const bool first = (threadIdx.x & 63) == 0 || ml != m;
    if (m > 0 && first) atomicMin(owner + m, (unsigned)k);
  }
}
__global__ __launch_bounds__(256) void k_owner_flags(const unsigned *__restrict__ owner, int64_t np,
                                                     int *__restrict__ flag) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v <= np; v += (int64_t)gridDim.x * blockDim.x)
    flag[v] = (v >= 1 && owner[v] != 0xffffffffu) ? 1 : 0;
}
__global__ __launch_bounds__(256) void k_owner_gather(const unsigned *__restrict__ owner, const int *__restrict__ flag,
                                                      const int *__restrict__ pos, int64_t np,
                                                      const TetRec *__restrict__ tets, int4 *__restrict__ out,
                                                      int *__restrict__ kidx, unsigned *__restrict__ count) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v <= np; v += (int64_t)gridDim.x * blockDim.x) {
    if (flag[v]) {
      const int k = (int)owner[v];
      out[pos[v]] = *reinterpret_cast<const int4 *>(tets + k);
      kidx[pos[v]] = k;
    }
    if (v == np) *count = (unsigned)(pos[v] + flag[v]);
  }
}
size_t owner_scan_temp_bytes(int64_t np) {
  size_t bytes = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const int *)nullptr, (int *)nullptr, (int)(np + 1));
  return bytes;
}
bool launch_owner_sample(const TetRec *tets, int64_t ne, int64_t np, unsigned *owner, int *flag, int *pos,
                         int4 *out, int *kidx, unsigned *d_count, unsigned *h_count, void *tmp, size_t tmp_bytes,
                         hipStream_t s) {
  if (hipMemsetAsync(owner, 0xff, (size_t)(np + 1) * sizeof(unsigned), s) != hipSuccess) return false;
  const int64_t nbt = std::max<int64_t>(1, std::min<int64_t>((ne + 255) / 256, 65536));
  const int64_t nbv = std::max<int64_t>(1, std::min<int64_t>((np + 256) / 256, 65536));
  hipLaunchKernelGGL(k_vmin_owner, dim3((unsigned)nbt), dim3(256), 0, s, tets, ne, owner);
  hipLaunchKernelGGL(k_owner_flags, dim3((unsigned)nbv), dim3(256), 0, s, (const unsigned *)owner, np, flag);
  if (hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, (const int *)flag, pos, (int)(np + 1), s) != hipSuccess)
    return false;
  hipLaunchKernelGGL(k_owner_gather, dim3((unsigned)nbv), dim3(256), 0, s, (const unsigned *)owner,
                     (const int *)flag, (const int *)pos, np, tets, out, kidx, d_count);
  if (hipMemcpyAsync(h_count, d_count, sizeof(unsigned), hipMemcpyDeviceToHost, s) != hipSuccess) return false;
  return hipGetLastError() == hipSuccess;
}

// the hint cells with their start tet's compact record inline (run flag exp
// 13, A/B of the r04 verdict's item 2a): cell c -> {k, w0, w1, w2},
// {w3, w4, w5, 0}; the walk's first record comes with the cell (a read of
// neighbouring cells) instead of a dependent gather of a random tet line
__global__ __launch_bounds__(256) void k_hint_inline(const int *__restrict__ grid, int64_t cells,
                                                     const WRec *__restrict__ wr, uint4 *__restrict__ hrec) {
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < cells;
       c += (int64_t)gridDim.x * blockDim.x) {
    const int k = grid[c];
    uint4 a = make_uint4(0u, 0u, 0u, 0u), b = make_uint4(0u, 0u, 0u, 0u);
    if (k) {
      const WRec r = wr[k];
      a = make_uint4((unsigned)k, r.w[0], r.w[1], r.w[2]);
      b = make_uint4(r.w[3], r.w[4], r.w[5], 0u);
    }
    hrec[2 * c] = a;
    hrec[2 * c + 1] = b;
  }
}
void launch_hint_inline(const int *grid, int64_t cells, const WRec *wr, uint4 *hrec, hipStream_t s) {
  const int64_t nb = std::min<int64_t>(std::max<int64_t>((cells + 255) / 256, 1), 65536);
  hipLaunchKernelGGL(k_hint_inline, dim3((unsigned)nb), dim3(256), 0, s, grid, cells, wr, hrec);
}

// the walk's compact records (WRec, pmx_device.h) from the tet records, built
// with them at every upload / promotion (a re-layout of the connectivity, like
// the records themselves)
__global__ __launch_bounds__(256) void k_build_wrec(const TetRec *__restrict__ tets, int64_t ne,
                                                    WRec *__restrict__ wr, unsigned *__restrict__ nfar) {
  unsigned cnt = 0;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k <= ne;
       k += (int64_t)gridDim.x * blockDim.x) {
    WRec r;
    wrec_encode(tets[k], k, r);
    wr[k] = r;
    const TetRec d = wrec_decode(r, tets, (int)k);
    cnt += (d.nb[0] | d.nb[1] | d.nb[2] | d.nb[3]) < 0 ? 1u : 0u;
  }
  // tets with a far neighbour field, one atomic per wave
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(nfar, cnt);
}
void launch_build_wrec(const TetRec *tets, int64_t ne, WRec *wr, unsigned *d_nfar, unsigned *h_nfar,
                       hipStream_t s) {
  const int64_t nb = std::min<int64_t>(std::max<int64_t>((ne + 256) / 256, 1), 16384);
  hipMemsetAsync(d_nfar, 0, sizeof(unsigned), s);
  hipLaunchKernelGGL(k_build_wrec, dim3((unsigned)nb), dim3(256), 0, s, tets, ne, wr, d_nfar);
  hipMemcpyAsync(h_nfar, d_nfar, sizeof(unsigned), hipMemcpyDeviceToHost, s);
}

// connectivity stream out of the tet records (statistics pass, built on demand)
__global__ __launch_bounds__(256) void k_tet_conn(const TetRec *__restrict__ src, int64_t n,
                                                  int4 *__restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = *reinterpret_cast<const int4 *>(src + i);
}
void launch_tet_conn(const TetRec *src, int64_t n, int4 *dst, hipStream_t s) {
  int64_t nb = std::min<int64_t>(std::max<int64_t>((n + 255) / 256, 1), 16384);
  hipLaunchKernelGGL(k_tet_conn, dim3((unsigned)nb), dim3(256), 0, s, src, n, dst);
}

// ---- ties -----------------------------------------------------------------------

// A point with some lambda_f < TIE_NEAR in its tet may also satisfy the
// reference's inside test (lambda_min > -1e-6, src/barycoord_pmmg.c:102-107)
// in the neighbours across those faces (face / edge / vertex ties).  The
// reference returns whichever its path reaches first; the device returns the
// smallest index of the connected set of containing tets, so the answer is
// independent of the start tet (and equals the exhaustive scan's first hit).
// lambda_f < 10*EPS admits neighbours up to 10x larger across face f: a tie
// across a sharper size jump is still a containing tet, only not canonical
#define TIE_NEAR 1.e-5
#define TIE_CAP 48
__device__ __noinline__ int canonical_tet(const TetRec *tets, const double *xyz, int k0, D3 p) {
  int vis[TIE_CAP], inq[TIE_CAP];
  int nv = 0, nq = 0, head = 0, best = k0;
  vis[nv++] = k0;
  inq[nq++] = k0;
  while (head < nq) {
    int k = inq[head++];
    TetRec t = tets[k];
    D3 P[4] = {ld3(xyz, t.v[0]), ld3(xyz, t.v[1]), ld3(xyz, t.v[2]), ld3(xyz, t.v[3])};
    double lam[4], vol;
    tet_lambda(P, p, lam, &vol);
    for (int f = 0; f < 4; f++) {
      int nb = t.nb[f];
      if (!nb || !(lam[f] < TIE_NEAR)) continue;
      bool seen = false;
      for (int q = 0; q < nv; q++) seen |= (vis[q] == nb);
      if (seen) continue;
      if (nv == TIE_CAP) return -1;
      vis[nv++] = nb;
      TetRec u = tets[nb];
      if (u.v[0] <= 0) continue;
      D3 Q[4] = {ld3(xyz, u.v[0]), ld3(xyz, u.v[1]), ld3(xyz, u.v[2]), ld3(xyz, u.v[3])};
      double mu[4], vu;
      tet_lambda(Q, p, mu, &vu);
      if (fmin(fmin(mu[0], mu[1]), fmin(mu[2], mu[3])) > -PMX_EPS) {
        if (nq == TIE_CAP) return -1;
        inq[nq++] = nb;
        best = nb < best ? nb : best;
      }
    }
  }
  return best;
}

__device__ void d_ties(const VolArgs &A, unsigned bid, unsigned nblk) {
  const unsigned n = *A.tie_count;
  for (unsigned j = bid * blockDim.x + threadIdx.x; j < n; j += nblk * blockDim.x) {
    int2 e = A.tie_list[j];
    const int64_t i = e.x;
    const D3 p = ld3(A.q, (int)i);
    int kc = canonical_tet(A.tets, A.xyz, e.y, p);
    if (kc < 0) {                                   // tie set too large: scan
      unsigned slot = atomicAdd(A.stuck_count, 1u);
      A.stuck_list[slot] = (int)i;
      A.found[slot] = 0x7fffffff;
      A.bestk[slot] = 0x7fffffff;
      A.best[slot] = ~0ull;
      A.steps[i] = -A.steps[i];
      continue;
    }
    TetRec t = A.tets[kc];
    int v[4] = {t.v[0], t.v[1], t.v[2], t.v[3]};
    D3 P[4] = {ld3(A.xyz, v[0]), ld3(A.xyz, v[1]), ld3(A.xyz, v[2]), ld3(A.xyz, v[3])};
    double lam[4], vol;
    tet_lambda(P, p, lam, &vol);
    A.elem[i] = kc;
    A.status[i] = 1;
    unsigned wm = interp_bar<4>(A.sol, A.sd, v, lam, A.out + i * A.sd.S);
    A.wmask[i] = (uint8_t)(wm | A.const_bit);
  }
}

// ---- exhaustive fallback ---------------------------------------------------

#define EXH_CHUNK 256

// smallest tet index containing each stuck point (bbox prefilter, exact test)
__device__ void d_exh_find(const ExhArgs &A, unsigned bid, unsigned nblk) {
  __shared__ D3 sp[EXH_CHUNK];
  const unsigned n = *A.count;
  for (unsigned c0 = 0; c0 < n; c0 += EXH_CHUNK) {
    unsigned m = min((unsigned)EXH_CHUNK, n - c0);
    __syncthreads();
    for (unsigned j = threadIdx.x; j < m; j += blockDim.x) sp[j] = ld3(A.q, A.list[c0 + j]);
    __syncthreads();
    for (int64_t k = 1 + (int64_t)bid * blockDim.x + threadIdx.x; k <= A.ne;
         k += (int64_t)nblk * blockDim.x) {
      TetRec t = A.tets[k];
      if (t.v[0] <= 0) continue;
      D3 P[4] = {ld3(A.xyz, t.v[0]), ld3(A.xyz, t.v[1]), ld3(A.xyz, t.v[2]), ld3(A.xyz, t.v[3])};
      double lo[3] = {P[0].x, P[0].y, P[0].z}, hi[3] = {P[0].x, P[0].y, P[0].z};
#pragma unroll
      for (int l = 1; l < 4; l++) {
        lo[0] = fmin(lo[0], P[l].x); hi[0] = fmax(hi[0], P[l].x);
        lo[1] = fmin(lo[1], P[l].y); hi[1] = fmax(hi[1], P[l].y);
        lo[2] = fmin(lo[2], P[l].z); hi[2] = fmax(hi[2], P[l].z);
      }
      // lambda_i >= -1e-6 for all i keeps the point within 3e-6 * extent of
      // the bbox; 1e-5 * max extent is a safe margin
      double ext = fmax(hi[0] - lo[0], fmax(hi[1] - lo[1], hi[2] - lo[2]));
      double mg = 1.e-5 * ext;
      for (unsigned j = 0; j < m; j++) {
        D3 p = sp[j];
        if (p.x < lo[0] - mg || p.x > hi[0] + mg || p.y < lo[1] - mg || p.y > hi[1] + mg ||
            p.z < lo[2] - mg || p.z > hi[2] + mg)
          continue;
        double lam[4], vol;
        tet_lambda(P, p, lam, &vol);
        double mn = fmin(fmin(lam[0], lam[1]), fmin(lam[2], lam[3]));
        if (mn > -PMX_EPS) atomicMin(&A.found[c0 + j], (int)k);
      }
    }
  }
}

// argmin over all tets of |lambda_min| * vol for points found nowhere
__device__ void d_exh_closest(const ExhArgs &A, int pass, unsigned bid, unsigned nblk) {
  __shared__ D3 sp[EXH_CHUNK];
  __shared__ int act[EXH_CHUNK];
  const unsigned n = *A.count;
  for (unsigned c0 = 0; c0 < n; c0 += EXH_CHUNK) {
    unsigned m = min((unsigned)EXH_CHUNK, n - c0);
    __syncthreads();
    for (unsigned j = threadIdx.x; j < m; j += blockDim.x) {
      sp[j] = ld3(A.q, A.list[c0 + j]);
      act[j] = (A.found[c0 + j] == 0x7fffffff);
    }
    __syncthreads();
    for (int64_t k = 1 + (int64_t)bid * blockDim.x + threadIdx.x; k <= A.ne;
         k += (int64_t)nblk * blockDim.x) {
      TetRec t = A.tets[k];
      if (t.v[0] <= 0) continue;
      D3 P[4] = {ld3(A.xyz, t.v[0]), ld3(A.xyz, t.v[1]), ld3(A.xyz, t.v[2]), ld3(A.xyz, t.v[3])};
      for (unsigned j = 0; j < m; j++) {
        if (!act[j]) continue;
        double lam[4], vol;
        tet_lambda(P, sp[j], lam, &vol);
        double mn = fmin(fmin(lam[0], lam[1]), fmin(lam[2], lam[3]));
        double d = fabs(mn) * vol;                 // src/locate_pmmg.c:455-458
        unsigned long long bits = (unsigned long long)__double_as_longlong(d);
        if (pass == 0) atomicMin(&A.best[c0 + j], bits);
        else if (bits == A.best[c0 + j]) atomicMin(&A.bestk[c0 + j], (int)k);
      }
    }
  }
}

__device__ void d_exh_finish(const ExhArgs &A, const VolArgs &V, unsigned bid, unsigned nblk) {
  const unsigned n = *A.count;
  for (unsigned j = bid * blockDim.x + threadIdx.x; j < n; j += nblk * blockDim.x) {
    int64_t i = A.list[j];
    const D3 p = ld3(A.q, (int)i);
    int k = A.found[j];
    int st = 1;
    double phi[4];
    if (k == 0x7fffffff) {
      k = A.bestk[j];
      st = 0;
    }
    if (k == 0x7fffffff) {                          // no valid tet at all: left untouched
      V.elem[i] = 0;
      V.status[i] = 0;
      continue;
    }
    TetRec t = A.tets[k];
    int v[4] = {t.v[0], t.v[1], t.v[2], t.v[3]};
    D3 P[4] = {ld3(A.xyz, v[0]), ld3(A.xyz, v[1]), ld3(A.xyz, v[2]), ld3(A.xyz, v[3])};
    if (st) {
      double vol;
      tet_lambda(P, p, phi, &vol);
    } else {
      // PMMG_barycoord3d_getClosest: nearest vertex, first on ties
      double best = 0.0;
      int it = 0;
#pragma unroll
      for (int l = 0; l < 4; l++) {
        double d0 = p.x - P[l].x, d1 = p.y - P[l].y, d2 = p.z - P[l].z;
        double d = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
        if (l == 0 || d < best) { best = d; it = l; }
      }
#pragma unroll
      for (int l = 0; l < 4; l++) phi[l] = (l == it) ? 1.0 : 0.0;
    }
    V.elem[i] = k;
    V.status[i] = st ? -1 : 0;
    V.steps[i] = V.steps[i] - 1;
    unsigned wm = interp_bar<4>(V.sol, V.sd, v, phi, V.out + i * V.sd.S);
    V.wmask[i] = (uint8_t)(V.wmask[i] | wm);
  }
}

// ---- fused fallback -------------------------------------------------------------
//
// Exhaustive scan (find, closest value, closest index) and the final
// interpolation of the scanned points in ONE launch (four launches that almost
// always found nothing to do cost ~4.5 us each).  The launch reads the
// counters and leaves, or runs the phases separated by a grid barrier
// (MI355X_MICROARCH.md "barrier-counter": release fence + waitcnt before the
// arrive, relaxed agent-scope poll, acquire fence after).  Its grid is sized
// on the host from the occupancy query so that every workgroup is co-resident
// even beside another context's fallback (fallback_coresident_blocks); should
// a barrier still time out, the workgroup records PMX_DERR_BARRIER in the
// step's error word and every later phase is skipped, and the host turns that
// into a failed call (pmx_synchronize / pmx_download) -- never a silent result.

__device__ __forceinline__ unsigned ld_agent(const unsigned *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// false when the wait gave up (the error word is set then)
__device__ bool grid_barrier(unsigned *bar, unsigned target, unsigned *err, long spin_limit) {
  __shared__ int s_ok;
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    atomicAdd(bar, 1u);
    long it = 0;
    while (ld_agent(bar) < target && ld_agent(err) == 0u && it < spin_limit) {
      __builtin_amdgcn_s_sleep(2);
      it++;
    }
    const bool ok = ld_agent(bar) >= target && ld_agent(err) == 0u;
    if (!ok) atomicOr(err, PMX_DERR_BARRIER);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s_ok = ok ? 1 : 0;
  }
  __syncthreads();
  return s_ok != 0;
}

// The ties (canonical tet BFS, independent per point) are a launch of their
// own: a step with ties but no stuck point (the common case: 71 ties at C3)
// then needs no grid barrier, so its fallback never waits for co-residency
// behind another context's walk (C4: two groups per GPU).  The tie launch may
// append points to the stuck list; the kernel boundary orders that.
__global__ __launch_bounds__(256) void k_ties(VolArgs V) {
  if (ld_agent(V.tie_count) == 0) return;
  d_ties(V, blockIdx.x, gridDim.x);
}

__global__ __launch_bounds__(256) void k_fallback(ExhArgs E, VolArgs V) {
  const unsigned nb = gridDim.x, b = blockIdx.x;
  unsigned *bar = V.stuck_count + 4;           // counts[4], zeroed by the prologue
  unsigned *err = V.stuck_count + PMX_CNT_ERR;
  if (ld_agent(V.stuck_count) == 0) return;
  d_exh_find(E, b, nb);
  if (!grid_barrier(bar, nb, err, E.spin_limit)) return;
  d_exh_closest(E, 0, b, nb);
  if (!grid_barrier(bar, 2 * nb, err, E.spin_limit)) return;
  d_exh_closest(E, 1, b, nb);
  if (!grid_barrier(bar, 3 * nb, err, E.spin_limit)) return;
  d_exh_finish(E, V, b, nb);
}

int fallback_coresident_blocks(int device, int share) {
  int cus = 0, per_cu = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(k_fallback),
                                                   256, 0) != hipSuccess)
    return 0;
  const long cap = (long)cus * per_cu / std::max(1, share);
  return (int)std::min<long>(256, cap);
}

void launch_exhaustive(const ExhArgs &e, const VolArgs &v, int blocks, hipStream_t s) {
  hipLaunchKernelGGL(k_ties, dim3(64), dim3(256), 0, s, v);
  hipLaunchKernelGGL(k_fallback, dim3((unsigned)std::max(1, blocks)), dim3(256), 0, s, e, v);
}

// constant-size metric (MMG3D_Set_constantSize restated): all valid points
__global__ __launch_bounds__(256) void k_const_metric(const int8_t *__restrict__ kind, int64_t nq,
                                                      double *__restrict__ out, int S, int off,
                                                      int size, double hsiz,
                                                      uint8_t *__restrict__ wmask, int imet) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nq;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (kind[i] == KIND_NUL) continue;
    double *o = out + i * S + off;
    if (size == 1) {
      o[0] = hsiz;
    } else {
      double v = 1.0 / (hsiz * hsiz);
      o[0] = v; o[1] = 0.0; o[2] = 0.0; o[3] = v; o[4] = 0.0; o[5] = v;
    }
    wmask[i] |= (uint8_t)(1u << imet);
  }
}
void launch_const_metric(const int8_t *kind, int64_t nq, double *out, int S, int off, int size,
                         double hsiz, uint8_t *wmask, int imet, hipStream_t s) {
  int64_t nb = (nq + 255) / 256;
  if (nb > 8192) nb = 8192;
  if (nb < 1) return;
  hipLaunchKernelGGL(k_const_metric, dim3((unsigned)nb), dim3(256), 0, s, kind, nq, out, S, off,
                     size, hsiz, wmask, imet);
}

// the step's first launch: zero the ranges pmx_run adds -- the write masks,
// the step's counters and the volume hint grid (the orphan marks come from
// the host, the node -> trias counts are zeroed by their own builder)
__global__ __launch_bounds__(256) void k_prologue(ZeroRanges z) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
  for (int r = 0; r < z.n; r++) {
    // hipMalloc'd ranges: 256-B aligned starts
    const int64_t n16 = z.bytes[r] / 16;
    uint4 *q = reinterpret_cast<uint4 *>(z.p[r]);
    for (int64_t i = t; i < n16; i += st) q[i] = make_uint4(0, 0, 0, 0);
    char *c = reinterpret_cast<char *>(z.p[r]);
    for (int64_t i = n16 * 16 + t; i < z.bytes[r]; i += st) c[i] = 0;
  }
}
void launch_prologue(const ZeroRanges &z, hipStream_t s) {
  int64_t work = 1;
  for (int r = 0; r < z.n; r++) work = std::max<int64_t>(work, z.bytes[r] / 16);
  const int64_t nb = std::min<int64_t>(std::max<int64_t>((work + 255) / 256, 1), 4096);
  hipLaunchKernelGGL(k_prologue, dim3((unsigned)nb), dim3(256), 0, s, z);
}

// the rows of points in no valid new tet, after a step that located them:
// back to untouched (the constant-size bit kept), element / status / steps /
// start 0, edge / vertex unset (-1), and their kind KIND_ORPH, so that the
// locate statistics count only the points the reference visits (a NUL or
// frozen point keeps its kind: the step never located it)
__global__ __launch_bounds__(256) void k_orphans(const uint8_t *__restrict__ mk, int64_t n, uint8_t keep,
                                                 OrphanRows r) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    if (mk[j]) continue;
    r.wmask[j] &= keep;
    r.elem[j] = 0;
    r.status[j] = 0;
    r.steps[j] = 0;
    r.start[j] = 0;
    r.edge[j] = -1;
    r.vertex[j] = -1;
    const int8_t k = r.kind[j];
    if (k == KIND_VOL || k == KIND_BDY) r.kind[j] = KIND_ORPH;
  }
}
void launch_orphans(const uint8_t *mk, int64_t n, uint8_t keep, const OrphanRows &r, hipStream_t s) {
  if (n < 1) return;
  const int64_t nb = std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_orphans, dim3((unsigned)nb), dim3(256), 0, s, mk, n, keep, r);
}

// the orphan marks from the new tets on the device: point j (0-based) is
// marked when a valid new tet (1-based vertex j + 1) holds it -- the
// reference's vertex loop over the new tets (src/interpmesh_pmmg.c:535-541).
// HBM-bound on the 16-B tet reads; the byte stores are what costs beyond
// them (r06: 0.50 ms at C3 with four stores per tet), so a lane skips the
// vertices its left neighbour -- the previous tet, which in any coherent
// numbering shares most of them -- also holds (that lane stores them), and
// each lane takes two tets per round (two loads in flight).
// H tets per thread and iteration (loads in flight); PMX_MARK_TPT=4 (A/B)
template <int H>
__global__ __launch_bounds__(256) void k_mark_new_tets(const int4 *__restrict__ tv, int64_t ne,
                                                       uint8_t *__restrict__ mk) {
  // (r06: an XCD-aware split -- each XCD one contiguous eighth of the tets,
  // so its byte stores stay in its own L2 -- measured 0.565 vs 0.549 ms
  // beside the step's prefix: not kept)
  const int64_t st = (int64_t)gridDim.x * blockDim.x;
  const int64_t nit = (ne + H * st - 1) / (H * st);    // uniform trip count (the shuffles below)
  const bool lane0 = (threadIdx.x & 63) == 0;
  for (int64_t it = 0; it < nit; it++) {
    const int64_t k0 = 1 + H * (it * st + (int64_t)blockIdx.x * blockDim.x) + threadIdx.x;
    int4 v[H];
#pragma unroll
    for (int h = 0; h < H; h++) {
      const int64_t k = k0 + h * blockDim.x;
      v[h] = k <= ne ? tv[k] : make_int4(0, 0, 0, 0);
    }
#pragma unroll
    for (int h = 0; h < H; h++) {
      const int4 a = v[h];
      int4 u;
      u.x = __shfl_up(a.x, 1, 64); u.y = __shfl_up(a.y, 1, 64);
      u.z = __shfl_up(a.z, 1, 64); u.w = __shfl_up(a.w, 1, 64);
      if (lane0 || u.x <= 0) u = make_int4(0, 0, 0, 0);   // no valid left neighbour: store all
      if (a.x <= 0) continue;                             // !MG_EOK
      const int w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
      for (int l = 0; l < 4; l++) {
        const int q = w[l];
        if (q != u.x && q != u.y && q != u.z && q != u.w) mk[q - 1] = 1;
      }
    }
  }
}
// r06 (late): the same marks with the next round's tets loaded BEFORE this
// round's byte stores, and every store issued (a buffer store whose offset is
// out of the descriptor's range when it is filtered out: the hardware drops
// it, no branch).  vmcnt counts loads and stores in one in-order counter on
// gfx950, so k_mark_new_tets' loads, issued after the previous round's
// stores, waited for those stores too (`s_waitcnt vmcnt(0)` at the loop
// head); here the head waits vmcnt(4H): the stores stay in flight.
template <int H>
__global__ __launch_bounds__(256) void k_mark_new_tets_pipe(const int4 *__restrict__ tv, int64_t ne,
                                                            uint8_t *__restrict__ mk, int nmk) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(mk, (short)0, nmk, 0x00020000);
  const int64_t st = (int64_t)gridDim.x * blockDim.x;
  const int64_t nit = (ne + H * st - 1) / (H * st);    // uniform trip count (the shuffles below)
  const bool lane0 = (threadIdx.x & 63) == 0;
  const int64_t kb = 1 + H * (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int4 v[H];
#pragma unroll
  for (int h = 0; h < H; h++) v[h] = tv[min(kb + h * (int64_t)blockDim.x, ne)];
  // 4H dropped stores (offset out of range): the loop is entered with the
  // same VMEM pattern as its back edge (loads, then 4H stores), so the
  // compiler's wait at the loop head is vmcnt(4H) on both paths, not 0
#pragma unroll
  for (int l = 0; l < 4 * H; l++) __builtin_amdgcn_raw_buffer_store_b8((unsigned char)1, rs, nmk + l * 64, 0, 0);
  for (int64_t it = 0; it < nit; it++) {
    const int64_t k0 = kb + H * it * st;
    int4 a[H];
#pragma unroll
    for (int h = 0; h < H; h++) {
      a[h] = v[h];
      if (!(k0 + h * (int64_t)blockDim.x <= ne && a[h].x > 0)) a[h] = make_int4(0, 0, 0, 0);   // !MG_EOK / tail
    }
    // the next round's tets (clamped: the last round reloads row ne, unused)
#pragma unroll
    for (int h = 0; h < H; h++) v[h] = tv[min(k0 + H * st + h * (int64_t)blockDim.x, ne)];
#pragma unroll
    for (int h = 0; h < H; h++) {
      const int4 q4 = a[h];
      int4 u;
      u.x = __shfl_up(q4.x, 1, 64); u.y = __shfl_up(q4.y, 1, 64);
      u.z = __shfl_up(q4.z, 1, 64); u.w = __shfl_up(q4.w, 1, 64);
      if (lane0) u = make_int4(0, 0, 0, 0);             // no left neighbour: store all
      const int w[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
      for (int l = 0; l < 4; l++) {
        const int q = w[l];
        const bool keep = q > 0 && q != u.x && q != u.y && q != u.z && q != u.w;
        __builtin_amdgcn_raw_buffer_store_b8((unsigned char)1, rs, keep ? q - 1 : nmk, 0, 0);
      }
    }
  }
}

// r06 (late): the marks deduplicated in LDS.  What bounds k_mark_new_tets is
// not its 16-B tet stream but its byte stores: one L2 write request per lane
// and vertex (≈ 1.5-2 per tet after the left-neighbour filter, a vertex is in
// ≈ 24 tets).  Here a workgroup takes 256 H consecutive tets at a time and
// marks their vertices in an LDS byte window [wb, wb + MW_WIN) anchored at
// the chunk's first valid tet (a coherent numbering -- Morton or Scotch --
// keeps a chunk's vertices together); the window is flushed as 32-bit words,
// one global atomicOr per word that holds a mark (the bytes of the marks
// array ORed: marks are only ever set, so concurrent chunks and the plain
// byte stores of out-of-window vertices compose).  Any numbering stays
// correct: a vertex outside the window is stored directly, as before.
#define MW_WIN 16384
template <int H>
__global__ __launch_bounds__(256) void k_mark_new_tets_win(const int4 *__restrict__ tv, int64_t ne,
                                                           uint8_t *__restrict__ mk, int64_t nmk) {
  __shared__ unsigned win[MW_WIN / 4];
  __shared__ int s_base;
  unsigned *mk32 = reinterpret_cast<unsigned *>(mk);
  uint8_t *wb8 = reinterpret_cast<uint8_t *>(win);
  for (int i = threadIdx.x; i < MW_WIN / 4; i += 256) win[i] = 0u;
  const int64_t C = 256 * H;
  const int64_t nch = (ne + C - 1) / C;
  const bool lane0 = (threadIdx.x & 63) == 0;
  for (int64_t c = blockIdx.x; c < nch; c += gridDim.x) {        // uniform over the workgroup
    const int64_t k0 = 1 + c * C + threadIdx.x;
    int4 v[H];
#pragma unroll
    for (int h = 0; h < H; h++) {
      const int64_t k = k0 + h * 256;
      v[h] = k <= ne ? tv[k] : make_int4(0, 0, 0, 0);
    }
    // window anchor: the first valid tet's smallest vertex, less a quarter
    // window (vertices of a chunk's later cells may precede it), 4-aligned
    if (threadIdx.x == 0) {
      const int4 a = v[0];
      const int m = a.x > 0 ? min(min(a.x, a.y), min(a.z, a.w)) - 1 : 0;
      s_base = max(0, m - MW_WIN / 4) & ~3;
    }
    __syncthreads();
    const int wb = s_base;
#pragma unroll
    for (int h = 0; h < H; h++) {
      const int4 a = v[h];
      int4 u;
      u.x = __shfl_up(a.x, 1, 64); u.y = __shfl_up(a.y, 1, 64);
      u.z = __shfl_up(a.z, 1, 64); u.w = __shfl_up(a.w, 1, 64);
      if (lane0 || u.x <= 0) u = make_int4(0, 0, 0, 0);
      if (a.x <= 0) continue;                             // !MG_EOK
      const int w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
      for (int l = 0; l < 4; l++) {
        const int q = w[l];
        if (q == u.x || q == u.y || q == u.z || q == u.w) continue;
        const unsigned off = (unsigned)(q - 1 - wb);
        if (off < (unsigned)MW_WIN) wb8[off] = 1;
        else mk[q - 1] = 1;
      }
    }
    __syncthreads();
    // flush: one atomicOr per word holding a mark, then clear it
    const int64_t w0 = wb >> 2;
    for (int i = threadIdx.x; i < MW_WIN / 4; i += 256) {
      const unsigned x = win[i];
      if (x) {
        if (w0 + i < (nmk + 3) / 4) atomicOr(mk32 + w0 + i, x);
        win[i] = 0u;
      }
    }
    __syncthreads();
  }
}

void launch_mark_new_tets(const int4 *tv, int64_t ne, uint8_t *mk, int64_t nmk, hipStream_t s) {
  // PMX_MARK_WIN=0 (A/B): the marks without the LDS window
  static const bool winm = [] {
    const char *e = getenv("PMX_MARK_WIN");
    return !(e && e[0] == '0');
  }();
  // PMX_MARK_H=8 (A/B): 2048 tets per chunk instead of 1024
  static const int wh = [] {
    const char *e = getenv("PMX_MARK_H");
    return e && e[0] == '8' ? 8 : 4;
  }();
  if (winm && ne >= 1 && nmk > 0 && nmk < INT32_MAX - MW_WIN) {
    const int64_t nb = std::min<int64_t>((ne + 256 * wh - 1) / (256 * wh), 4096);
    if (wh == 8)
      hipLaunchKernelGGL(k_mark_new_tets_win<8>, dim3((unsigned)nb), dim3(256), 0, s, tv, ne, mk, nmk);
    else
      hipLaunchKernelGGL(k_mark_new_tets_win<4>, dim3((unsigned)nb), dim3(256), 0, s, tv, ne, mk, nmk);
    return;
  }
  if (ne < 1) return;
  static const int tpt = [] {
    const char *e = getenv("PMX_MARK_TPT");
    return e && e[0] == '4' ? 4 : 2;
  }();
  // PMX_MARK_PIPE=1 (A/B): k_mark_new_tets_pipe (beside the derived data it
  // takes memory bandwidth from them: C3 step 2.481-2.500 vs 2.470-2.488 ms)
  static const bool pipe = [] {
    const char *e = getenv("PMX_MARK_PIPE");
    return e && e[0] == '1';
  }();
  // PMX_MARK_BLOCKS (A/B): the block cap -- the marks run beside the derived
  // data and the hint build, which they slow by sharing the memory system
  static const int64_t cap = [] {
    const char *e = getenv("PMX_MARK_BLOCKS");
    return e ? std::max<int64_t>(1, atoll(e)) : (int64_t)8192;
  }();
  const int64_t nb = std::min<int64_t>((ne + 256 * tpt - 1) / (256 * tpt), cap);
  if (pipe && nmk > 0 && nmk < INT32_MAX - 4096) {
    if (tpt == 4)
      hipLaunchKernelGGL(k_mark_new_tets_pipe<4>, dim3((unsigned)nb), dim3(256), 0, s, tv, ne, mk, (int)nmk);
    else
      hipLaunchKernelGGL(k_mark_new_tets_pipe<2>, dim3((unsigned)nb), dim3(256), 0, s, tv, ne, mk, (int)nmk);
    return;
  }
  if (tpt == 4)
    hipLaunchKernelGGL(k_mark_new_tets<4>, dim3((unsigned)nb), dim3(256), 0, s, tv, ne, mk);
  else
    hipLaunchKernelGGL(k_mark_new_tets<2>, dim3((unsigned)nb), dim3(256), 0, s, tv, ne, mk);
}

// ---- device residency across iterations (pmx_promote_background) ----------------

// the last step's new points and results become the background: vertex ip
// (1..n) = new point ip-1, its solution row = the step's output row ip-1
__global__ __launch_bounds__(256) void k_promote(const double *__restrict__ q, const double *__restrict__ out,
                                                 const uint16_t *__restrict__ qtag, int64_t n, int S,
                                                 double *__restrict__ xyz, double *__restrict__ sol,
                                                 uint16_t *__restrict__ ptag) {
  for (int64_t ip = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; ip <= n;
       ip += (int64_t)gridDim.x * blockDim.x) {
    if (ip == 0) {
      xyz[0] = xyz[1] = xyz[2] = 0.0;
      for (int j = 0; j < S; j++) sol[j] = 0.0;
      if (ptag) ptag[0] = 0;
      continue;
    }
    xyz[3 * ip] = q[3 * (ip - 1)];
    xyz[3 * ip + 1] = q[3 * (ip - 1) + 1];
    xyz[3 * ip + 2] = q[3 * (ip - 1) + 2];
    for (int j = 0; j < S; j++) sol[ip * S + j] = out[(ip - 1) * S + j];
    if (ptag) ptag[ip] = qtag[ip - 1];
  }
}
// rows the step did not write (not located, frozen, failed): the caller's
// values, uploaded as (row, offset, size) + 6 doubles
__global__ __launch_bounds__(256) void k_patch_rows(const int4 *__restrict__ ent, const double *__restrict__ vals,
                                                    int64_t n, int S, double *__restrict__ sol) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int4 e = ent[i];                       // x: vertex, y: offset, z: size
    for (int j = 0; j < e.z; j++) sol[(int64_t)e.x * S + e.y + j] = vals[6 * i + j];
  }
}
// tet records from the new tets and their Mmg face adjacency
// (adja[4*(k-1)+1+f] = 4*k'+f'), and the packed hint sample
__global__ __launch_bounds__(256) void k_build_tetrec(const int4 *__restrict__ tv, const int *__restrict__ adja,
                                                      int64_t ne, int stride, TetRec *__restrict__ tets,
                                                      int4 *__restrict__ sample) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k <= ne;
       k += (int64_t)gridDim.x * blockDim.x) {
    TetRec r;
    const int4 v = tv[k];
    r.v[0] = v.x; r.v[1] = v.y; r.v[2] = v.z; r.v[3] = v.w;
    for (int f = 0; f < 4; f++) r.nb[f] = k ? adja[4 * (k - 1) + 1 + f] / 4 : 0;
    tets[k] = r;
    if (k >= 1 && (k - 1) % stride == 0) sample[(k - 1) / stride] = v;
  }
}
void launch_promote(const double *q, const double *out, const uint16_t *qtag, int64_t n, int S, double *xyz,
                    double *sol, uint16_t *ptag, hipStream_t s) {
  const int64_t nb = std::min<int64_t>(std::max<int64_t>((n + 256) / 256, 1), 16384);
  hipLaunchKernelGGL(k_promote, dim3((unsigned)nb), dim3(256), 0, s, q, out, qtag, n, S, xyz, sol, ptag);
}
void launch_patch_rows(const int4 *ent, const double *vals, int64_t n, int S, double *sol, hipStream_t s) {
  if (n < 1) return;
  const int64_t nb = std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_patch_rows, dim3((unsigned)nb), dim3(256), 0, s, ent, vals, n, S, sol);
}
void launch_build_tetrec(const int4 *tv, const int *adja, int64_t ne, int stride, TetRec *tets, int4 *sample,
                         hipStream_t s) {
  const int64_t nb = std::min<int64_t>(std::max<int64_t>((ne + 256) / 256, 1), 16384);
  hipLaunchKernelGGL(k_build_tetrec, dim3((unsigned)nb), dim3(256), 0, s, tv, adja, ne, stride, tets, sample);
}

// ---- new points: classification on the device (pmx_upload_points) ---------------

// sum over the 256-thread block, in every thread (red: 4 LDS slots)
__device__ __forceinline__ int2 block_sum2(int2 v, int2 *red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    v.x += __shfl_xor(v.x, o, 64);
    v.y += __shfl_xor(v.y, o, 64);
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  int2 r = red[0];
#pragma unroll
  for (int w = 1; w < 4; w++) { r.x += red[w].x; r.y += red[w].y; }
  return r;
}

// The kinds of the 16 points j0 .. j0+15 of one thread (j0 % 16 == 0): two
// 16-B tag loads and one 16-B mark load instead of 16 narrow loads per lane
// (r03: the one-point-per-lane rounds were latency-bound, 0.12 ms at C3 for
// 17 M points); points at or past n get 0xff.  kw: the kinds, 4 per word.
__device__ __forceinline__ void kinds16(const uint16_t *__restrict__ tag, const uint8_t *__restrict__ mark,
                                        int64_t j0, int64_t n, unsigned kw[4], int &cv, int &cb) {
  unsigned tw[8], mw[4];
  if (j0 + 16 <= n) {
    if (tag) {
      const uint4 a = reinterpret_cast<const uint4 *>(tag + j0)[0];
      const uint4 b = reinterpret_cast<const uint4 *>(tag + j0)[1];
      tw[0] = a.x; tw[1] = a.y; tw[2] = a.z; tw[3] = a.w;
      tw[4] = b.x; tw[5] = b.y; tw[6] = b.z; tw[7] = b.w;
    } else {
#pragma unroll
      for (int i = 0; i < 8; i++) tw[i] = 0u;
    }
    if (mark) {
      const uint4 c = *reinterpret_cast<const uint4 *>(mark + j0);
      mw[0] = c.x; mw[1] = c.y; mw[2] = c.z; mw[3] = c.w;
    }
  } else {                                    // the last, partial chunk
#pragma unroll
    for (int i = 0; i < 8; i++) tw[i] = 0u;
#pragma unroll
    for (int i = 0; i < 4; i++) mw[i] = 0u;
    for (int i = 0; i < 16 && j0 + i < n; i++) {
      if (tag) tw[i >> 1] |= (unsigned)tag[j0 + i] << (16 * (i & 1));
      if (mark) mw[i >> 2] |= (unsigned)mark[j0 + i] << (8 * (i & 3));
    }
  }
#pragma unroll
  for (int w = 0; w < 4; w++) kw[w] = 0u;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const unsigned t = (tw[i >> 1] >> (16 * (i & 1))) & 0xffffu;
    const bool in = j0 + i < n;
    // kind of a new point: PMMG_interpMetricsAndFields_mesh's dispatch
    // (src/interpmesh_pmmg.c:541-560): !MG_VOK, MG_REQ (copied by
    // PMMG_copyMetricsAndFields_point over every point, :311-446, whatever
    // the tets), in no valid new tet (never visited), MG_BDY, volume
    unsigned k = (t >= PMX_TAG_NUL) ? KIND_NUL
                 : (t & PMX_TAG_REQ) ? KIND_SKIP
                 : (mark && !((mw[i >> 2] >> (8 * (i & 3))) & 0xffu)) ? KIND_ORPH
                 : (t & PMX_TAG_BDY) ? KIND_BDY : KIND_VOL;
    k = in ? k : 0xffu;
    cv += k == KIND_VOL;
    cb += k == KIND_BDY;
    kw[i >> 2] |= k << (8 * (i & 3));
  }
}

// per tile of CLS_TILE points: how many volume / surface points
__global__ __launch_bounds__(256) void k_cls_count(const uint16_t *__restrict__ tag, const uint8_t *__restrict__ mark,
                                                   int64_t n, int2 *__restrict__ tcnt) {
  __shared__ int2 red[4];
  const int64_t t0 = (int64_t)blockIdx.x * CLS_TILE;
  int cv = 0, cb = 0;
#pragma unroll
  for (int r = 0; r < CLS_TILE / 4096; r++) {
    const int64_t j0 = t0 + r * 4096 + 16 * (int64_t)threadIdx.x;
    unsigned kw[4];
    if (j0 < n) kinds16(tag, mark, j0, n, kw, cv, cb);
  }
  const int2 c = block_sum2(make_int2(cv, cb), red);
  if (threadIdx.x == 0) tcnt[blockIdx.x] = c;
}

// kinds + the two lists in input order.  Per round of 4096 points: every
// thread classifies 16 consecutive points (vector loads, one 16-B kind
// store) into LDS; wave w owns points 1024 w .. 1024 w + 1023 of the round
// (its own threads' chunks), so the wave totals give each wave its base, and
// the wave then writes its list entries in 16 coalesced ballot sub-rounds.
// Tile base = sum of the previous tiles' counts, summed again by every
// workgroup (a few KB of L2 reads instead of a third launch).
__global__ __launch_bounds__(256) void k_cls_write(const uint16_t *__restrict__ tag,
                                                   const uint8_t *__restrict__ mark, int64_t n,
                                                   const int2 *__restrict__ tcnt, int8_t *__restrict__ kind,
                                                   int *__restrict__ vlist, int *__restrict__ blist,
                                                   int *__restrict__ nsel) {
  __shared__ int2 red[4];
  __shared__ int2 wc[4];
  __shared__ uint4 lk[256];                   // the round's 4096 kinds
  int pv = 0, pb = 0;
  for (unsigned t = threadIdx.x; t < blockIdx.x; t += 256) {
    const int2 c = tcnt[t];
    pv += c.x;
    pb += c.y;
  }
  int2 base = block_sum2(make_int2(pv, pb), red);
  const int64_t t0 = (int64_t)blockIdx.x * CLS_TILE;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long below = (1ull << lane) - 1ull;
  const uint8_t *lkb = reinterpret_cast<const uint8_t *>(lk);
  for (int r = 0; r < CLS_TILE / 4096; r++) {
    const int64_t r0 = t0 + r * 4096;
    if (r0 >= n) break;                                   // uniform: the tile's end
    const int64_t j0 = r0 + 16 * (int64_t)threadIdx.x;
    unsigned kw[4] = {~0u, ~0u, ~0u, ~0u};
    int cv = 0, cb = 0;
    if (j0 < n) {
      kinds16(tag, mark, j0, n, kw, cv, cb);
      if (j0 + 16 <= n) *reinterpret_cast<uint4 *>(kind + j0) = make_uint4(kw[0], kw[1], kw[2], kw[3]);
      else
        for (int i = 0; j0 + i < n; i++) kind[j0 + i] = (int8_t)((kw[i >> 2] >> (8 * (i & 3))) & 0xffu);
    }
    lk[threadIdx.x] = make_uint4(kw[0], kw[1], kw[2], kw[3]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      cv += __shfl_xor(cv, o, 64);
      cb += __shfl_xor(cb, o, 64);
    }
    if (lane == 0) wc[w] = make_int2(cv, cb);
    __syncthreads();
    int ov = base.x, ob = base.y;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int2 c = wc[q];
      ov += q < w ? c.x : 0;
      ob += q < w ? c.y : 0;
      base.x += c.x;
      base.y += c.y;
    }
    // the wave's 1024 points in input order, 64 per sub-round
#pragma unroll 4
    for (int s = 0; s < 16; s++) {
      const int p = 1024 * w + 64 * s + lane;
      const int k = lkb[p];
      const unsigned long long bv = __ballot(k == KIND_VOL), bb = __ballot(k == KIND_BDY);
      if (k == KIND_VOL) vlist[ov + __popcll(bv & below)] = (int)(r0 + p);
      else if (k == KIND_BDY) blist[ob + __popcll(bb & below)] = (int)(r0 + p);
      ov += __popcll(bv);
      ob += __popcll(bb);
    }
    __syncthreads();                                      // lk and wc rewritten next round
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
    nsel[0] = base.x;
    nsel[1] = base.y;
  }
}

void launch_classify(const uint16_t *tag, const uint8_t *mk, int64_t n, int2 *tcnt, int8_t *kind, int *vlist,
                     int *blist, int *nsel, hipStream_t s) {
  if (n < 1) return;
  const unsigned nt = (unsigned)cls_tiles(n);
  hipLaunchKernelGGL(k_cls_count, dim3(nt), dim3(256), 0, s, tag, mk, n, tcnt);
  hipLaunchKernelGGL(k_cls_write, dim3(nt), dim3(256), 0, s, tag, mk, n, (const int2 *)tcnt, kind, vlist,
                     blist, nsel);
}
