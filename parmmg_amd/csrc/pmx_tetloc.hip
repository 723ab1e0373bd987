// pmx_tetloc.hip -- tet-centric volume location + interpolation (gfx950).
//
// Same answer as the reference's adjacency walk (PMMG_locatePointVol,
// reference src/locate_pmmg.c:786-883) -- the unique tet whose barycentrics
// pass the inside test lambda_min > -1e-6 (src/barycoord_pmmg.c:102-107), the
// smallest index among several (documented ties), the closest tet otherwise --
// computed the way HBM likes it when new vertices are about as many as old
// ones (ParMmg's r ~ 1 remesh iterations):
//
//   1. bin:     the new volume vertices are bucketed by cell of a uniform grid
//               over the background bbox (one atomic per vertex + a scan);
//   2. stream:  one thread per OLD tet reads its 16-B connectivity once
//               (coalesced), gathers its 4 vertices, builds its 4 face normals
//               in registers, and tests the bucketed vertices of the cells
//               overlapping its bbox.  A vertex deep inside (lambda_min >=
//               TIE_NEAR) is interpolated right there from the tet's 4 vertex
//               rows (PMMG_interp4bar_{iso,ani}, src/interpmesh_pmmg.c:206-270);
//               a vertex within TIE_NEAR of a face records the tet with
//               atomicMin;
//   3. finish:  per vertex, the smallest containing tet wins (rare re-do),
//               vertices found nowhere go to the exhaustive closest scan.
//
// Every old tet is read once and no walk/hint pass re-reads the mesh: the
// connectivity traffic is ne*16 B instead of hint (ne*16..32 B) + walk
// (~ne*32 B).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <cmath>
#include "pmx_internal.h"

#define TIE_NEAR_T 1.e-5

__device__ __forceinline__ int cellc(double t, int n) {
  if (!(t > 0.0)) return 0;
  if (t >= (double)(n - 1)) return n - 1;
  return (int)t;
}

// 1a. cell of every volume vertex + its slot in the cell
__global__ __launch_bounds__(256) void k_qbin(const Pt4 *__restrict__ q, const int *__restrict__ list,
                                              int64_t n, GridDesc g, unsigned *__restrict__ cnt,
                                              int *__restrict__ qcell, int *__restrict__ qslot) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x) {
    Pt4 p = q[list[j]];
    int cx = cellc((p.x - g.lo[0]) * g.inv[0], g.dim[0]);
    int cy = cellc((p.y - g.lo[1]) * g.inv[1], g.dim[1]);
    int cz = cellc((p.z - g.lo[2]) * g.inv[2], g.dim[2]);
    int c = cx + g.dim[0] * (cy + g.dim[1] * cz);
    qcell[j] = c;
    qslot[j] = (int)atomicAdd(&cnt[c], 1u);
  }
}

// 1c. scatter into cell order: coordinates + point index packed in .w
__global__ __launch_bounds__(256) void k_qscatter(const Pt4 *__restrict__ q, const int *__restrict__ list,
                                                  int64_t n, const int *__restrict__ qcell,
                                                  const int *__restrict__ qslot,
                                                  const unsigned *__restrict__ start,
                                                  Pt4 *__restrict__ qs) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int i = list[j];
    Pt4 p = q[i];
    p.w = __longlong_as_double((long long)i);
    qs[start[qcell[j]] + qslot[j]] = p;
  }
}

struct TetLocArgs {
  const int4 *tetv;
  const Pt4 *pts;
  const double *sol;
  SolDesc sd;
  int64_t ne;
  GridDesc g;
  const unsigned *start;      // cells+1 exclusive offsets
  const Pt4 *qs;              // bucketed vertices
  double *out;
  uint8_t *wmask;
  int *elem, *status;
  int *best;                  // atomicMin of tets containing a near-face vertex
  unsigned const_bit;
  unsigned long long *tests;  // per-block partial: bbox-passing tests
};

template <int OCC>
__global__ __launch_bounds__(256, OCC) void k_tet_locate(TetLocArgs A) {
  unsigned long long ntest = 0;
  for (int64_t k = 1 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k <= A.ne;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int4 vv = A.tetv[k];
    if (vv.x <= 0) continue;
    const int v[4] = {vv.x, vv.y, vv.z, vv.w};
    D3 P[4] = {ld3(A.pts, v[0]), ld3(A.pts, v[1]), ld3(A.pts, v[2]), ld3(A.pts, v[3])};
    double lo[3] = {P[0].x, P[0].y, P[0].z}, hi[3] = {P[0].x, P[0].y, P[0].z};
#pragma unroll
    for (int l = 1; l < 4; l++) {
      lo[0] = fmin(lo[0], P[l].x); hi[0] = fmax(hi[0], P[l].x);
      lo[1] = fmin(lo[1], P[l].y); hi[1] = fmax(hi[1], P[l].y);
      lo[2] = fmin(lo[2], P[l].z); hi[2] = fmax(hi[2], P[l].z);
    }
    // lambda_i >= -1e-6 keeps a point within 3e-6 * extent of the bbox
    const double mg = 1.e-5 * fmax(hi[0] - lo[0], fmax(hi[1] - lo[1], hi[2] - lo[2]));
#pragma unroll
    for (int a = 0; a < 3; a++) { lo[a] -= mg; hi[a] += mg; }
    const int c0x = cellc((lo[0] - A.g.lo[0]) * A.g.inv[0], A.g.dim[0]);
    const int c1x = cellc((hi[0] - A.g.lo[0]) * A.g.inv[0], A.g.dim[0]);
    const int c0y = cellc((lo[1] - A.g.lo[1]) * A.g.inv[1], A.g.dim[1]);
    const int c1y = cellc((hi[1] - A.g.lo[1]) * A.g.inv[1], A.g.dim[1]);
    const int c0z = cellc((lo[2] - A.g.lo[2]) * A.g.inv[2], A.g.dim[2]);
    const int c1z = cellc((hi[2] - A.g.lo[2]) * A.g.inv[2], A.g.dim[2]);
    // face normals and 6*volume exactly as tet_lambda (bit-identical lambda)
    const double vol = orvol(P[0], P[1], P[2], P[3]);
    const D3 n0 = nonunit_normal(P[1], P[2], P[3]);
    const D3 n1 = nonunit_normal(P[0], P[3], P[2]);
    const D3 n2 = nonunit_normal(P[0], P[1], P[3]);
    const D3 n3 = nonunit_normal(P[0], P[2], P[1]);
    // division-free rejection: lambda_f = -dot_f/vol > -EPS needs
    // dot_f < EPS*vol (vol > 0); the margin covers the rounding of both sides
    const double dlim = PMX_EPS * vol * (1.0 + 1.e-6);
    for (int cz = c0z; cz <= c1z; cz++)
      for (int cy = c0y; cy <= c1y; cy++) {
        const int64_t row = (int64_t)A.g.dim[0] * (cy + (int64_t)A.g.dim[1] * cz);
        const unsigned s = A.start[row + c0x], e = A.start[row + c1x + 1];
        for (unsigned j = s; j < e; j++) {
          const Pt4 qq = A.qs[j];
          if (qq.x < lo[0] || qq.x > hi[0] || qq.y < lo[1] || qq.y > hi[1] || qq.z < lo[2] ||
              qq.z > hi[2])
            continue;
          ntest++;
          const D3 p{qq.x, qq.y, qq.z};
          const double d0 = (p.x - P[1].x) * n0.x + (p.y - P[1].y) * n0.y + (p.z - P[1].z) * n0.z;
          const double d1 = (p.x - P[0].x) * n1.x + (p.y - P[0].y) * n1.y + (p.z - P[0].z) * n1.z;
          const double d2 = (p.x - P[0].x) * n2.x + (p.y - P[0].y) * n2.y + (p.z - P[0].z) * n2.z;
          const double d3 = (p.x - P[0].x) * n3.x + (p.y - P[0].y) * n3.y + (p.z - P[0].z) * n3.z;
          if (!(vol > 0.0) || d0 > dlim || d1 > dlim || d2 > dlim || d3 > dlim) {
            if (vol > 0.0) continue;                 // rejected without a division
          }
          double lam[4] = {-d0 / vol, -d1 / vol, -d2 / vol, -d3 / vol};
          const double lmn = fmin(fmin(lam[0], lam[1]), fmin(lam[2], lam[3]));
          if (!(lmn > -PMX_EPS)) continue;
          const int i = (int)__double_as_longlong(qq.w);
          if (lmn >= TIE_NEAR_T) {
            // deep inside: the only containing tet of a valid mesh
            A.elem[i] = (int)k;
            A.status[i] = 1;
            unsigned wm = interp_bar<4>(A.sol, A.sd, v, lam, A.out + (int64_t)i * A.sd.S);
            A.wmask[i] = (uint8_t)(wm | A.const_bit);
          } else {
            atomicMin(&A.best[i], (int)k);
          }
        }
      }
  }
  // per-block test count (diagnostic, no same-address atomics)
  __shared__ unsigned long long sh[4];
  for (int o = 32; o > 0; o >>= 1) ntest += __shfl_xor(ntest, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = ntest;
  __syncthreads();
  if (threadIdx.x == 0 && A.tests) A.tests[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

// 3. per volume vertex: smallest containing tet, or hand over to the scan
__global__ __launch_bounds__(256) void k_tet_finish(TetLocArgs T, VolArgs V) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < V.nlist;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int i = V.list[j];
    const int b = T.best[i];
    const bool deep = T.status[i] == 1;
    if (deep && (b == 0x7f7f7f7f || b >= T.elem[i])) continue;
    if (b != 0x7f7f7f7f) {
      // near-face vertex (or a smaller tet also contains a deep one)
      int4 vv = T.tetv[b];
      int v[4] = {vv.x, vv.y, vv.z, vv.w};
      D3 P[4] = {ld3(T.pts, v[0]), ld3(T.pts, v[1]), ld3(T.pts, v[2]), ld3(T.pts, v[3])};
      Pt4 qq = V.q[i];
      double lam[4], vol;
      tet_lambda(P, D3{qq.x, qq.y, qq.z}, lam, &vol);
      T.elem[i] = b;
      T.status[i] = 1;
      unsigned wm = interp_bar<4>(T.sol, T.sd, v, lam, T.out + (int64_t)i * T.sd.S);
      T.wmask[i] = (uint8_t)(wm | T.const_bit);
      continue;
    }
    unsigned slot = atomicAdd(V.stuck_count, 1u);
    V.stuck_list[slot] = i;
    V.found[slot] = 0x7fffffff;
    V.bestk[slot] = 0x7fffffff;
    V.best[slot] = ~0ull;
    V.steps[i] = 0;
  }
}

// host side -------------------------------------------------------------------

bool pmx_ctx::launch_tet_locate(const VolArgs &A, const pmx_run_opts &o, hipStream_t s) {
  const int64_t nv = nq_vol;
  // vertex grid over the background bbox, about one volume vertex per cell
  GridDesc g;
  double ext[3], vol = 1.0;
  for (int a = 0; a < 3; a++) {
    ext[a] = std::max(bbhi[a] - bblo[a], 1e-300);
    vol *= ext[a];
  }
  // cell edge = f * (volume per vertex)^(1/3); the origin is shifted by an
  // irrational fraction of a cell so that lattice-aligned tet bboxes (Kuhn
  // cells, Cartesian-like meshes) do not straddle cell faces by the margin
  static const double fac[4] = {1.0, 0.5, 0.7, 1.4};
  const double h = fac[(o.tune >> 10) & 3] * std::cbrt(vol / std::max(1.0, (double)nv));
  const double shift = 0.3819660113 * h;
  int64_t cells = 1;
  for (int a = 0; a < 3; a++) {
    int d = (int)std::ceil((ext[a] + shift) / h * (1.0 - 1e-9));
    d = std::max(1, std::min(d, 2048));
    g.dim[a] = d;
    g.lo[a] = bblo[a] - shift;
    g.inv[a] = (double)d / (ext[a] + shift);
    cells *= d;
  }
  auto grow = [&](auto &b, size_t n) {
    using T = std::remove_pointer_t<decltype(b.p)>;
    if (b.p && b.cap >= n) return true;
    if (b.p) hipFree(b.p);
    b.p = nullptr;
    if (hipMalloc((void **)&b.p, sizeof(T) * std::max<size_t>(n, 1)) != hipSuccess) return false;
    b.cap = n;
    return true;
  };
  if (!grow(d_qcnt, (size_t)cells + 1) || !grow(d_qstart, (size_t)cells + 1) ||
      !grow(d_qcell, (size_t)nv) || !grow(d_qslot, (size_t)nv) || !grow(d_qs, (size_t)nv) ||
      !grow(d_tbest, (size_t)nq) || !grow(d_tests, 8192)) {
    err = "hipMalloc (tet-centric buffers)";
    return false;
  }
  size_t tmp_bytes = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, d_qcnt.p, d_qstart.p, (int)(cells + 1), s);
  if (!grow(d_scan_tmp, tmp_bytes)) { err = "hipMalloc scan"; return false; }

  hipMemsetAsync(d_qcnt.p, 0, sizeof(unsigned) * (size_t)(cells + 1), s);
  hipMemsetAsync(d_tbest.p, 0x7f, sizeof(int) * (size_t)nq, s);
  hipMemsetAsync(d_status.p, 0, sizeof(int) * (size_t)nq, s);
  int64_t nb = std::min<int64_t>((nv + 255) / 256, 16384);
  hipLaunchKernelGGL(k_qbin, dim3((unsigned)std::max<int64_t>(nb, 1)), dim3(256), 0, s, d_q.p,
                     d_vollist.p, nv, g, d_qcnt.p, d_qcell.p, d_qslot.p);
  hipcub::DeviceScan::ExclusiveSum(d_scan_tmp.p, tmp_bytes, d_qcnt.p, d_qstart.p, (int)(cells + 1), s);
  hipLaunchKernelGGL(k_qscatter, dim3((unsigned)std::max<int64_t>(nb, 1)), dim3(256), 0, s, d_q.p,
                     d_vollist.p, nv, d_qcell.p, d_qslot.p, d_qstart.p, d_qs.p);
  TetLocArgs T{};
  T.tetv = d_tetv.p; T.pts = d_pts.p; T.sol = d_sol.p; T.sd = A.sd; T.ne = ne; T.g = g;
  T.start = d_qstart.p; T.qs = d_qs.p; T.out = d_out.p; T.wmask = d_wmask.p;
  T.elem = d_elem.p; T.status = d_status.p; T.best = d_tbest.p; T.const_bit = A.const_bit;
  T.tests = d_tests.p;
  const int64_t tb = std::min<int64_t>((ne + 255) / 256, 8192);
  tests_blocks = (int)tb;
  const int occ = (o.tune >> 4) & 0xF;
  if (occ == 2)
    hipLaunchKernelGGL(k_tet_locate<2>, dim3((unsigned)tb), dim3(256), 0, s, T);
  else if (occ == 4)
    hipLaunchKernelGGL(k_tet_locate<4>, dim3((unsigned)tb), dim3(256), 0, s, T);
  else
    hipLaunchKernelGGL(k_tet_locate<1>, dim3((unsigned)tb), dim3(256), 0, s, T);
  hipLaunchKernelGGL(k_tet_finish, dim3((unsigned)std::max<int64_t>(nb, 1)), dim3(256), 0, s, T, A);
  return hipGetLastError() == hipSuccess;
}
