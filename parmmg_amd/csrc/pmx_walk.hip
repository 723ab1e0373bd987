// pmx_walk.hip -- the production volume kernel: k_walk (locate + interpolate).
//
// Same contract as k_locate_vol (pmx_kernels.hip): one thread per new volume
// vertex, adjacency walk from the hint grid (PMMG_locatePointVol, reference
// src/locate_pmmg.c:786-883), fused PMMG_interp4bar_{iso,ani}
// (src/interpmesh_pmmg.c:206-270), stuck lanes and near-face ties compacted
// into lists for k_fallback.  The located tet, its barycentrics and the fields
// are bit-identical to k_locate_vol's; what changes is the cost of a step:
//
//  * direction without divisions: a walk step only needs the ORDER of the
//    barycentrics and the sign test lambda_min > -1e-6.  lambda_f = -num_f/vol
//    (src/barycoord_pmmg.c:238-257) is ranked through -num_f * (1/vol) (one
//    division instead of four, <= 2 ulp from the quotient); when that
//    estimate comes within 1e-13 of the threshold the four exact quotients
//    are formed and decide, so "found" and the barycentrics used for the
//    interpolation are exactly the reference's.  The path may differ from a
//    walk ranked on exact quotients only where two barycentrics are within
//    2 ulp of each other; the answer does not depend on the path (unique
//    containing tet, or the canonical min-index tet of a tie -- k_ties).
//  * vertex reuse: the next tet shares a face (3 vertices) with the current
//    one; only its opposite vertex is gathered (1 instead of 4 32-B gathers
//    per step after the first), the shared coordinates are permuted in VGPRs.
//  * layout specialisation: the interpolation is compiled for the solution
//    layout (one anisotropic metric; S isotropic/vector components; generic)
//    so the register allocation is not the maximum over every layout.
#include <algorithm>
#include "pmx_device.h"
#include "pmx_kernels.h"

#define WALK_RING 4
#define TIE_NEAR 1.e-5
#define APPROX_GUARD 1.e-13

__device__ __forceinline__ int64_t walk_xcd_remap(int64_t b, int64_t nb) {
  // blocks b and b+8 share an XCD (round-robin dispatch): each XCD gets a
  // contiguous range of the Morton-ordered queries so its L2 sees neighbours
  int64_t xcd = b & 7, r = b >> 3, q = nb >> 3, rem = nb & 7;
  return (xcd < rem) ? xcd * (q + 1) + r : rem * (q + 1) + (xcd - rem) * q + r;
}

__device__ __forceinline__ int wclamp(double t, int n) {
  if (!(t > 0.0)) return 0;                 // also catches NaN
  if (t >= (double)(n - 1)) return n - 1;
  return (int)t;
}

// empty hint cell: nearest non-empty cell in growing shells (rare; kept out of
// line so that its loops do not inflate the walk's register allocation)
__device__ __noinline__ int hint_search(const int *grid, int gx, int gy, int gz, int cx, int cy,
                                        int cz) {
  for (int r = 1; r <= 3; r++) {
    for (int dz = -r; dz <= r; dz++)
      for (int dy = -r; dy <= r; dy++)
        for (int dx = -r; dx <= r; dx++) {
          if (max(abs(dx), max(abs(dy), abs(dz))) != r) continue;
          int x = cx + dx, y = cy + dy, z = cz + dz;
          if (x < 0 || y < 0 || z < 0 || x >= gx || y >= gy || z >= gz) continue;
          int kk = grid[(int64_t)x + (int64_t)gx * ((int64_t)y + (int64_t)gy * z)];
          if (kk) return kk;
        }
  }
  return 1;
}

// central-hint grid: empty cells hold ~0 (no sample)
__device__ __noinline__ int hint_search64(const unsigned long long *grid, int gx, int gy, int gz,
                                          int cx, int cy, int cz) {
  for (int r = 1; r <= 3; r++) {
    for (int dz = -r; dz <= r; dz++)
      for (int dy = -r; dy <= r; dy++)
        for (int dx = -r; dx <= r; dx++) {
          if (max(abs(dx), max(abs(dy), abs(dz))) != r) continue;
          int x = cx + dx, y = cy + dy, z = cz + dz;
          if (x < 0 || y < 0 || z < 0 || x >= gx || y >= gy || z >= gz) continue;
          unsigned long long kk = grid[(int64_t)x + (int64_t)gx * ((int64_t)y + (int64_t)gy * z)];
          if (kk != ~0ull) return (int)(unsigned)(kk & 0xffffffffu);
        }
  }
  return 1;
}

__device__ __forceinline__ int walk_hint(const int *grid, const GridDesc &g, D3 p,
                                         const unsigned long long *grid64 = nullptr) {
  int cx = wclamp((p.x - g.lo[0]) * g.inv[0], g.dim[0]);
  int cy = wclamp((p.y - g.lo[1]) * g.inv[1], g.dim[1]);
  int cz = wclamp((p.z - g.lo[2]) * g.inv[2], g.dim[2]);
  const int64_t c = (int64_t)cx + (int64_t)g.dim[0] * ((int64_t)cy + (int64_t)g.dim[1] * cz);
  if (grid64) {
    const unsigned long long kk = grid64[c];
    return kk != ~0ull ? (int)(unsigned)(kk & 0xffffffffu)
                       : hint_search64(grid64, g.dim[0], g.dim[1], g.dim[2], cx, cy, cz);
  }
  int k = grid[c];
  return k ? k : hint_search(grid, g.dim[0], g.dim[1], g.dim[2], cx, cy, cz);
}

// numerators of the barycentrics: lambda_f = -num_f / vol, with exactly the
// operations of tet_lambda (pmx_device.h) before its division
__device__ __forceinline__ void face_nums(const D3 P[4], D3 p, double num[4], double *volp) {
  double vol = orvol(P[0], P[1], P[2], P[3]);
  D3 n0 = nonunit_normal(P[1], P[2], P[3]);
  D3 n1 = nonunit_normal(P[0], P[3], P[2]);
  D3 n2 = nonunit_normal(P[0], P[1], P[3]);
  D3 n3 = nonunit_normal(P[0], P[2], P[1]);
  num[0] = (p.x - P[1].x) * n0.x + (p.y - P[1].y) * n0.y + (p.z - P[1].z) * n0.z;
  num[1] = (p.x - P[0].x) * n1.x + (p.y - P[0].y) * n1.y + (p.z - P[0].z) * n1.z;
  num[2] = (p.x - P[0].x) * n2.x + (p.y - P[0].y) * n2.y + (p.z - P[0].z) * n2.z;
  num[3] = (p.x - P[0].x) * n3.x + (p.y - P[0].y) * n3.y + (p.z - P[0].z) * n3.z;
  *volp = vol;
}

__device__ __forceinline__ void wranks(const double l[4], int rk[4]) {
  rk[0] = rk[1] = rk[2] = rk[3] = 0;
#pragma unroll
  for (int a = 0; a < 4; a++)
#pragma unroll
    for (int b = a + 1; b < 4; b++) {
      bool bfirst = l[b] < l[a];          // stable: b after a unless strictly smaller
      rk[a] += bfirst ? 1 : 0;
      rk[b] += bfirst ? 0 : 1;
    }
}

__device__ __forceinline__ void wave_stats_w(uint4 *rec, unsigned cnt, unsigned sum, unsigned mx,
                                             unsigned mn) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_xor(cnt, o, 64);
    sum += __shfl_xor(sum, o, 64);
    unsigned a = __shfl_xor(mx, o, 64), b = __shfl_xor(mn, o, 64);
    mx = a > mx ? a : mx;
    mn = b < mn ? b : mn;
  }
  if ((threadIdx.x & 63) == 0) *rec = make_uint4(cnt, sum, mx, mn);
}

// a[i] for a 4-array held in registers: masked OR (a select chain is turned
// back into an indexed private-array load, i.e. scratch, by the compiler)
__device__ __forceinline__ int pick4(const int a[4], int i) {
  return (a[0] & -(int)(i == 0)) | (a[1] & -(int)(i == 1)) | (a[2] & -(int)(i == 2)) |
         (a[3] & -(int)(i == 3));
}

__device__ __forceinline__ D3 dsel(bool c, D3 a, D3 b) {
  return D3{c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z};
}

// ---- layout-specialised interpolation --------------------------------------
//
// LAYOUT_ANI: one solution, the 6-component metric (C2): interp4bar_ani.
// LAYOUT_ISO: every solution of size 1 or 3 and no constant metric: a row of
//             S doubles per vertex, out_j = ((0 + phi0 a0j) + phi1 a1j) ...
//             (interp4bar_iso, src/interpmesh_pmmg.c:206-230, order kept).
// LAYOUT_GEN: interp_bar<4> of pmx_device.h.
enum { LAYOUT_GEN = 0, LAYOUT_ANI = 1, LAYOUT_ISO = 2 };

// dense coordinates for the slot walk (VolArgs::xyz): x, y, z of every old
// vertex, 24 B apart.  Built once per background upload, a second layout of
// the uploaded vertices (the walk's vertex gathers then touch 5.3 vertices per
// 128-B line instead of 4; measured r01: k_walks 2.6 % faster on C3).
__global__ __launch_bounds__(256) void k_build_xyz(const Pt4 *__restrict__ pts, int64_t n,
                                                   double *__restrict__ out,
                                                   float *__restrict__ outf) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const Pt4 p = pts[i];
    out[3 * i] = p.x;
    out[3 * i + 1] = p.y;
    out[3 * i + 2] = p.z;
    // single-precision copy for the hint build's centroids (k_hint_build FX)
    outf[3 * i] = (float)p.x;
    outf[3 * i + 1] = (float)p.y;
    outf[3 * i + 2] = (float)p.z;
  }
}
void launch_build_xyz(const Pt4 *pts, int64_t n, double *out, float *outf, hipStream_t s) {
  const int64_t nb = std::min<int64_t>(std::max<int64_t>((n + 255) / 256, 1), 65536);
  hipLaunchKernelGGL(k_build_xyz, dim3((unsigned)nb), dim3(256), 0, s, pts, n, out, outf);
}

// tet record load; NT: non-temporal (streaming) hint, the record is rarely
// re-read while the vertex and solution rows around it are
typedef int v4i_t __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ TetRec ldtet(const TetRec *__restrict__ tets, int k) {
  if constexpr (NT) {
    const v4i_t *r = reinterpret_cast<const v4i_t *>(tets + k);
    const v4i_t a = __builtin_nontemporal_load(r), b = __builtin_nontemporal_load(r + 1);
    TetRec t;
    t.v[0] = a.x; t.v[1] = a.y; t.v[2] = a.z; t.v[3] = a.w;
    t.nb[0] = b.x; t.nb[1] = b.y; t.nb[2] = b.z; t.nb[3] = b.w;
    return t;
  } else {
    return tets[k];
  }
}
template <bool NT, class T>
__device__ __forceinline__ void stw(T *p, T v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// layout of the solutions for the walk kernel
static int walk_layout(const SolDesc &sd, int *S) {
  *S = sd.S;
  if (sd.nsol == 1 && sd.size[0] == 6 && sd.imet == 0 && !sd.metric_const) return LAYOUT_ANI;
  bool iso = !sd.metric_const && sd.S >= 1 && sd.S <= 8;
  for (int s = 0; s < sd.nsol; s++) iso = iso && sd.size[s] != 6;
  return iso ? LAYOUT_ISO : LAYOUT_GEN;
}


template <int LAYOUT, int S, bool NTS = false>
__device__ __forceinline__ unsigned interp_layout(const double *__restrict__ sol, const SolDesc &sd,
                                                  const int *v, const double *phi,
                                                  double *__restrict__ out) {
  if constexpr (LAYOUT == LAYOUT_ANI) {
    double mint[6], r[6];
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const double2 *m = reinterpret_cast<const double2 *>(sol + (int64_t)v[i] * 6);
      double2 a = m[0], b = m[1], c = m[2];
      double mm[6] = {a.x, a.y, b.x, b.y, c.x, c.y};
      double mi[6];
      ok = ok && invmat(mm, mi);
#pragma unroll
      for (int j = 0; j < 6; j++) mint[j] = (i == 0) ? phi[i] * mi[j] : mint[j] + phi[i] * mi[j];
    }
    if (!ok || !invmat(mint, r)) return 0u;
    double2 *o = reinterpret_cast<double2 *>(out);
    o[0] = make_double2(r[0], r[1]);
    o[1] = make_double2(r[2], r[3]);
    o[2] = make_double2(r[4], r[5]);
    return 1u;
  } else if constexpr (LAYOUT == LAYOUT_ISO) {
    double acc[S];
#pragma unroll
    for (int j = 0; j < S; j++) acc[j] = 0.0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const double *row = sol + (int64_t)v[i] * S;
      if constexpr ((S & 1) == 0) {
        // even stride: rows are 16-B aligned (upload pads odd S), 16-B loads
#pragma unroll
        for (int j = 0; j < S; j += 2) {
          const double2 d = *reinterpret_cast<const double2 *>(row + j);
          acc[j] += phi[i] * d.x;
          acc[j + 1] += phi[i] * d.y;
        }
      } else {
#pragma unroll
        for (int j = 0; j < S; j++) acc[j] += phi[i] * row[j];
      }
    }
    if constexpr ((S & 1) == 0) {
#pragma unroll
      for (int j = 0; j < S; j += 2) *reinterpret_cast<double2 *>(out + j) = make_double2(acc[j], acc[j + 1]);
    } else {
#pragma unroll
      for (int j = 0; j < S; j++) stw<NTS>(out + j, acc[j]);
    }
    return (1u << sd.nsol) - 1u;
  } else {
    return interp_bar<4>(sol, sd, v, phi, out);
  }
}

// Near-face cases of the canonical tie rule resolved in place (canonical_tet,
// pmx_kernels.hip, is the general BFS over the containing set; this is the
// same rule for the two shapes that make up almost every tie):
//  * no near face has an interior neighbour: the set is {cur};
//  * exactly one near face f with neighbour n: the set is {cur} if n does not
//    contain p, {cur, n} if it does and n has no further near face with an
//    interior neighbour other than cur -> min(cur, n).
// Returns true when the general BFS is needed (edge / vertex ties, chains).
// On return false, cur/t/lam hold the canonical tet and its barycentrics.
__device__ __forceinline__ bool face_tie(const VolArgs &A, D3 p, int &cur, TetRec &t, double lam[4]) {
  int nnear = 0, f1 = 0;
#pragma unroll
  for (int f = 0; f < 4; f++) {
    const bool nf = t.nb[f] != 0 && lam[f] < TIE_NEAR;
    nnear += nf ? 1 : 0;
    f1 = nf ? f : f1;
  }
  if (nnear == 0) return false;
  if (nnear > 1) return true;
  const int n = pick4(t.nb, f1);
  const TetRec u = A.tets[n];
  if (u.v[0] <= 0) return false;
  const D3 Q[4] = {ld3(A.pts, u.v[0]), ld3(A.pts, u.v[1]), ld3(A.pts, u.v[2]), ld3(A.pts, u.v[3])};
  double mu[4], vu;
  tet_lambda(Q, p, mu, &vu);
  if (!(fmin(fmin(mu[0], mu[1]), fmin(mu[2], mu[3])) > -PMX_EPS)) return false;
  bool more = false;
#pragma unroll
  for (int g = 0; g < 4; g++) more |= (u.nb[g] != 0 && u.nb[g] != cur && mu[g] < TIE_NEAR);
  if (more) return true;
  if (n < cur) {
    cur = n;
    t = u;
#pragma unroll
    for (int f = 0; f < 4; f++) lam[f] = mu[f];
  }
  return false;
}

template <int LAYOUT, int S, bool TIES, int OCC, int BS, int EXP = 0>
__global__ __launch_bounds__(BS, OCC) void k_walk(VolArgs A) {
  const int64_t b = walk_xcd_remap(blockIdx.x, gridDim.x);
  const int64_t j = b * blockDim.x + threadIdx.x;
  unsigned s_cnt = 0, s_sum = 0, s_max = 0, s_min = 0xffffffffu;

  if (j < A.nlist) {
    const int64_t i = A.list[j];
    const Pt4 qq = A.q[i];
    const D3 p{qq.x, qq.y, qq.z};
    int cur = walk_hint(A.grid, A.g, p, A.grid64);
    A.start[i] = cur;
    int ring[WALK_RING];
#pragma unroll
    for (int r = 0; r < WALK_RING; r++) ring[r] = 0;
    int step = 0;
    bool found = false;
    TetRec t = A.tets[cur];
    D3 P[4];
    double lam[4];
    if (t.v[0] <= 0) step = 1;                        // !MG_EOK start: let the scan decide
    else {
      P[0] = ld3(A.pts, t.v[0]); P[1] = ld3(A.pts, t.v[1]);
      P[2] = ld3(A.pts, t.v[2]); P[3] = ld3(A.pts, t.v[3]);
      for (;;) {
        step++;
        double num[4], vol;
        face_nums(P, p, num, &vol);
        if constexpr (EXP == 1) {            // sensitivity: the face arithmetic twice
          D3 Pc[4];
#pragma unroll
          for (int l = 0; l < 4; l++) {
            Pc[l] = P[l];
            asm volatile("" : "+v"(Pc[l].x), "+v"(Pc[l].y), "+v"(Pc[l].z));
          }
          double n2[4], v2;
          face_nums(Pc, p, n2, &v2);
          asm volatile("" ::"v"(n2[0]), "v"(n2[1]), "v"(n2[2]), "v"(n2[3]), "v"(v2));
        }
        if constexpr (EXP == 2) {            // sensitivity: one more tet record gather
          const TetRec e = A.tets[cur + 1];
          asm volatile("" ::"v"(e.v[0]), "v"(e.v[1]), "v"(e.v[2]), "v"(e.v[3]), "v"(e.nb[0]),
                       "v"(e.nb[1]), "v"(e.nb[2]), "v"(e.nb[3]));
        }
        if constexpr (EXP == 3) {            // sensitivity: one more vertex gather
          const Pt4 e = A.pts[t.v[0] + 1];
          asm volatile("" ::"v"(e.x), "v"(e.y), "v"(e.z));
        }
        const double rv = 1.0 / vol;
#pragma unroll
        for (int f = 0; f < 4; f++) lam[f] = -(num[f] * rv);
        double lmin = fmin(fmin(lam[0], lam[1]), fmin(lam[2], lam[3]));
        if (lmin > -PMX_EPS - APPROX_GUARD) {
          // near or inside: the reference's quotients decide
#pragma unroll
          for (int f = 0; f < 4; f++) lam[f] = -num[f] / vol;
          lmin = fmin(fmin(lam[0], lam[1]), fmin(lam[2], lam[3]));
          if (lmin > -PMX_EPS) { found = true; break; }     // src/barycoord_pmmg.c:102-107
        }
        if (step >= A.max_walk) break;
        int rk[4];
        wranks(lam, rk);
#pragma unroll
        for (int r = WALK_RING - 1; r > 0; r--) ring[r] = ring[r - 1];
        ring[0] = cur;
        // first interior, not recently visited neighbour in ascending-lambda
        // order (src/locate_pmmg.c:819-833)
        int next = 0;
#pragma unroll
        for (int r = 0; r < 4; r++) {
          int f = (rk[0] == r) ? 0 : (rk[1] == r) ? 1 : (rk[2] == r) ? 2 : 3;
          int nb = pick4(t.nb, f);
          bool seen = false;
#pragma unroll
          for (int q = 0; q < WALK_RING; q++) seen |= (ring[q] == nb);
          if (!next && nb && !seen) next = nb;
        }
        if (!next) break;
        const TetRec u = A.tets[next];
        cur = next;
        if (u.v[0] <= 0) { t = u; break; }                  // !MG_EOK: let the scan decide
        // shared face: permute the known coordinates, gather the new vertex
        bool m[4][4];
        int nnew = 0, lnew = 0;
#pragma unroll
        for (int l = 0; l < 4; l++) {
#pragma unroll
          for (int k = 0; k < 4; k++) m[l][k] = (u.v[l] == t.v[k]);
          bool any = m[l][0] | m[l][1] | m[l][2] | m[l][3];
          nnew += any ? 0 : 1;
          lnew = any ? lnew : l;
        }
        if (nnew == 1) {
          const D3 pn = ld3(A.pts, pick4(u.v, lnew));
          D3 Q[4];
#pragma unroll
          for (int l = 0; l < 4; l++)
            Q[l] = dsel(m[l][0], P[0], dsel(m[l][1], P[1], dsel(m[l][2], P[2], dsel(m[l][3], P[3], pn))));
#pragma unroll
          for (int l = 0; l < 4; l++) P[l] = Q[l];
        } else {                                               // inconsistent adjacency
          P[0] = ld3(A.pts, u.v[0]); P[1] = ld3(A.pts, u.v[1]);
          P[2] = ld3(A.pts, u.v[2]); P[3] = ld3(A.pts, u.v[3]);
        }
        t = u;
      }
    }
    if (found) {
      double lmn = fmin(fmin(lam[0], lam[1]), fmin(lam[2], lam[3]));
      if (lmn < TIE_NEAR && (!TIES || face_tie(A, p, cur, t, lam))) {
        // within the tolerance of several tets: canonical tet by k_ties
        unsigned slot = atomicAdd(A.tie_count, 1u);
        A.tie_list[slot] = make_int2((int)i, cur);
        A.steps[i] = step;
        found = false;
        step = -1;
      }
    }
    if (found) {
      A.elem[i] = cur;
      A.status[i] = 1;
      A.steps[i] = step;
      const int v[4] = {t.v[0], t.v[1], t.v[2], t.v[3]};
      unsigned wm = interp_layout<LAYOUT, S>(A.sol, A.sd, v, lam, A.out + i * A.sd.S);
      A.wmask[i] = (uint8_t)(wm | A.const_bit);
      s_cnt = 1; s_sum = step; s_max = step; s_min = step;
    } else if (step >= 0) {
      unsigned slot = atomicAdd(A.stuck_count, 1u);
      A.stuck_list[slot] = (int)i;
      A.found[slot] = 0x7fffffff;
      A.bestk[slot] = 0x7fffffff;
      A.best[slot] = ~0ull;
      A.steps[i] = -step;
    }
  }
  wave_stats_w(A.wstats + (b * blockDim.x + threadIdx.x) / 64, s_cnt, s_sum, s_max, s_min);
}

// ---- slot walk (k_walks) -------------------------------------------------------
//
// The walk DIRECTION needs neither the reference's operation order nor the
// tet's own vertex order -- only "found" and the interpolation weights must be
// the reference's quotients.  k_walks therefore walks on slot-ordered state:
//  * slot k holds a vertex id I[k], its coordinates C[k] and the neighbour
//    NB[k] across the face opposite it; a step through the face opposite slot
//    s replaces slot s by the neighbour's fourth vertex (one select per slot,
//    instead of permuting all four coordinates into the new tet's order);
//  * the barycentric numerators are signed sub-volumes about p: with
//    d_k = C_k - p, w0 = d1.(d2 x d3), w1 = -d0.(d2 x d3), w2 = d3.(d0 x d1),
//    w3 = -d2.(d0 x d1) and vol = sum w (2 cross + 4 dot products, no
//    division); every step reflects the slot order's orientation, so the
//    sign flips;
//  * the lane leaves the loop when min w > -(EPS + SLOT_GUARD) vol (the
//    reference's threshold with a margin far above this estimate's error);
//    then, once per lane, the coordinates are put in tet order and the
//    reference's quotients (tet_lambda's operations) decide.  A candidate
//    they reject (|lambda_min + EPS| < guard) continues with the reference-
//    order walk of k_walk.
// The located tet does not depend on the path (unique containing tet, or the
// canonical tet of a tie), so k_walks returns k_walk's results bit for bit.
#define SLOT_GUARD 1.e-10

__device__ __forceinline__ D3 dcross(D3 a, D3 b) {
  return D3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ double ddot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

// one reference-order step decision (k_walk's): the first interior, not
// recently visited neighbour in ascending-lambda order; 0 if none
template <int RG = WALK_RING>
__device__ __forceinline__ int exact_next(const TetRec &t, const double lam[4], int ring[RG],
                                          int cur) {
  int rk[4];
  wranks(lam, rk);
#pragma unroll
  for (int r = RG - 1; r > 0; r--) ring[r] = ring[r - 1];
  ring[0] = cur;
  int next = 0;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    int f = (rk[0] == r) ? 0 : (rk[1] == r) ? 1 : (rk[2] == r) ? 2 : 3;
    int nb = pick4(t.nb, f);
    bool seen = false;
#pragma unroll
    for (int q = 0; q < RG; q++) seen |= (ring[q] == nb);
    if (!next && nb && !seen) next = nb;
  }
  return next;
}

template <int LAYOUT, int S, bool TIES, bool DENSE, int RG = WALK_RING, int NT = 0, int OCC = 1>
__global__ __launch_bounds__(256, OCC) void k_walks(VolArgs A) {
  const int64_t b = walk_xcd_remap(blockIdx.x, gridDim.x);
  const int64_t j = b * blockDim.x + threadIdx.x;
  unsigned s_cnt = 0, s_sum = 0, s_max = 0, s_min = 0xffffffffu;
  // DENSE: the walk's coordinates from the 24-B xyz stream (5.3 vertices per
  // 128-B line instead of 4 for the 32-B Pt4 records)
  auto ldc = [&](int v) -> D3 {
    if constexpr (DENSE) {
      const double *r = A.xyz + (int64_t)v * 3;
      return D3{r[0], r[1], r[2]};
    } else {
      return ld3(A.pts, v);
    }
  };

  if (j < A.nlist) {
    // list order == Morton order of the volume points: both reads coalesced
    // and independent (no list -> point dependent gather)
    const int64_t i = A.list[j];
    const D3 p{A.qv[3 * j], A.qv[3 * j + 1], A.qv[3 * j + 2]};
    int cur = walk_hint(A.grid, A.g, p, A.grid64);
    if (A.rec_start) A.start[i] = cur;
    int ring[RG];
#pragma unroll
    for (int r = 0; r < RG; r++) ring[r] = 0;
    int step = 0;
    bool found = false;
    TetRec t = ldtet<(NT & 1) != 0>(A.tets, cur);
    double lam[4];
    if (t.v[0] <= 0) step = 1;                        // !MG_EOK start: let the scan decide
    else {
      D3 C[4] = {ldc(t.v[0]), ldc(t.v[1]), ldc(t.v[2]), ldc(t.v[3])};
      int I[4] = {t.v[0], t.v[1], t.v[2], t.v[3]};
      int NB[4] = {t.nb[0], t.nb[1], t.nb[2], t.nb[3]};
      bool neg = false, cand = false;
      for (;;) {
        step++;
        D3 d[4];
#pragma unroll
        for (int k = 0; k < 4; k++) d[k] = D3{C[k].x - p.x, C[k].y - p.y, C[k].z - p.z};
        const D3 c23 = dcross(d[2], d[3]), c01 = dcross(d[0], d[1]);
        double w[4] = {ddot(d[1], c23), -ddot(d[0], c23), ddot(d[3], c01), -ddot(d[2], c01)};
        if (neg) {
#pragma unroll
          for (int k = 0; k < 4; k++) w[k] = -w[k];
        }
        const double vol = (w[0] + w[1]) + (w[2] + w[3]);
        const double wmin = fmin(fmin(w[0], w[1]), fmin(w[2], w[3]));
        // near or inside (or a degenerate / inverted tet): the reference decides
        if (!(vol > 0.0) || wmin > -(PMX_EPS + SLOT_GUARD) * vol) { cand = true; break; }
        if (step >= A.max_walk) break;
#pragma unroll
        for (int r = RG - 1; r > 0; r--) ring[r] = ring[r - 1];
        ring[0] = cur;
        // the admissible slot (interior, not recently visited neighbour) with
        // the smallest barycentric
        int sb = -1;
        double wb = 0.0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int nb = NB[k];
          bool seen = false;
#pragma unroll
          for (int q = 0; q < RG; q++) seen |= (ring[q] == nb);
          const bool take = nb && !seen && (sb < 0 || w[k] < wb);
          sb = take ? k : sb;
          wb = take ? w[k] : wb;
        }
        if (sb < 0) break;
        const int next = pick4(NB, sb);
        const TetRec u = ldtet<(NT & 1) != 0>(A.tets, next);
        cur = next;
        t = u;
        if (u.v[0] <= 0) break;                            // !MG_EOK: let the scan decide
        // the neighbour's fourth vertex replaces slot sb
        int nnew = 0, lnew = 0;
#pragma unroll
        for (int l = 0; l < 4; l++) {
          const bool any = (u.v[l] == I[0]) | (u.v[l] == I[1]) | (u.v[l] == I[2]) | (u.v[l] == I[3]);
          nnew += any ? 0 : 1;
          lnew = any ? lnew : l;
        }
        if (nnew != 1) {                                   // inconsistent adjacency: reload
#pragma unroll
          for (int k = 0; k < 4; k++) {
            C[k] = ldc(u.v[k]);
            I[k] = u.v[k];
            NB[k] = u.nb[k];
          }
          neg = false;
          continue;
        }
        const int vn = pick4(u.v, lnew);
        const D3 pn = ldc(vn);
#pragma unroll
        for (int k = 0; k < 4; k++) {
          C[k] = dsel(k == sb, pn, C[k]);
          I[k] = (k == sb) ? vn : I[k];
        }
#pragma unroll
        for (int k = 0; k < 4; k++)
          NB[k] = (u.nb[0] & -(int)(u.v[0] == I[k])) | (u.nb[1] & -(int)(u.v[1] == I[k])) |
                  (u.nb[2] & -(int)(u.v[2] == I[k])) | (u.nb[3] & -(int)(u.v[3] == I[k]));
        neg = !neg;
      }
      if (cand) {
        // coordinates in tet order, then the reference's quotients; a
        // rejected candidate continues in the reference's order (rare)
        D3 P[4];
#pragma unroll
        for (int l = 0; l < 4; l++)
          P[l] = dsel(t.v[l] == I[0], C[0],
                      dsel(t.v[l] == I[1], C[1], dsel(t.v[l] == I[2], C[2], C[3])));
        for (;;) {
          double num[4], vol;
          face_nums(P, p, num, &vol);
#pragma unroll
          for (int f = 0; f < 4; f++) lam[f] = -num[f] / vol;
          const double lmin = fmin(fmin(lam[0], lam[1]), fmin(lam[2], lam[3]));
          if (lmin > -PMX_EPS) { found = true; break; }    // src/barycoord_pmmg.c:102-107
          if (step >= A.max_walk) break;
          const int next = exact_next<RG>(t, lam, ring, cur);
          if (!next) break;
          t = ldtet<(NT & 1) != 0>(A.tets, next);
          cur = next;
          if (t.v[0] <= 0) break;
          step++;
#pragma unroll
          for (int l = 0; l < 4; l++) P[l] = ldc(t.v[l]);
        }
      }
    }
    if (found) {
      double lmn = fmin(fmin(lam[0], lam[1]), fmin(lam[2], lam[3]));
      if (lmn < TIE_NEAR && (!TIES || face_tie(A, p, cur, t, lam))) {
        unsigned slot = atomicAdd(A.tie_count, 1u);
        A.tie_list[slot] = make_int2((int)i, cur);
        A.steps[i] = step;
        found = false;
        step = -1;
      }
    }
    if (found) {
      constexpr bool NTS = (NT & 2) != 0;
      stw<NTS>(A.elem + i, cur);
      stw<NTS>(A.status + i, 1);
      stw<NTS>(A.steps + i, step);
      const int v[4] = {t.v[0], t.v[1], t.v[2], t.v[3]};
      unsigned wm = interp_layout<LAYOUT, S, NTS>(A.sol, A.sd, v, lam, A.out + i * A.sd.S);
      stw<NTS>(A.wmask + i, (uint8_t)(wm | A.const_bit));
      s_cnt = 1; s_sum = step; s_max = step; s_min = step;
    } else if (step >= 0) {
      unsigned slot = atomicAdd(A.stuck_count, 1u);
      A.stuck_list[slot] = (int)i;
      A.found[slot] = 0x7fffffff;
      A.bestk[slot] = 0x7fffffff;
      A.best[slot] = ~0ull;
      A.steps[i] = -step;
    }
  }
  wave_stats_w(A.wstats + (b * blockDim.x + threadIdx.x) / 64, s_cnt, s_sum, s_max, s_min);
}



// OCC: minimum waves per SIMD asked of the register allocator (1 = free);
// BS: threads per block (the waves of one block share a CU and its L1: a
// larger block keeps more Morton-adjacent points on one CU)
template <int LAYOUT, int S, int OCC, int BS>
static void launch_walk_o(const VolArgs &a, int ties, hipStream_t s) {
  const int64_t nb = (a.nlist + BS - 1) / BS;
  constexpr bool X = OCC == 1 && BS == 256;   // default shape
  if (X && ties && a.exp >= 1 && a.exp <= 3) {
    // sensitivity experiments on k_walk
    if (a.exp == 1) hipLaunchKernelGGL((k_walk<LAYOUT, S, true, OCC, BS, X ? 1 : 0>), dim3((unsigned)nb), dim3(BS), 0, s, a);
    else if (a.exp == 2) hipLaunchKernelGGL((k_walk<LAYOUT, S, true, OCC, BS, X ? 2 : 0>), dim3((unsigned)nb), dim3(BS), 0, s, a);
    else hipLaunchKernelGGL((k_walk<LAYOUT, S, true, OCC, BS, X ? 3 : 0>), dim3((unsigned)nb), dim3(BS), 0, s, a);
  } else if (X && ties && a.exp == 4 && a.xyz && !a.ref_walk) {
    // sensitivity experiment: a 2-entry visited ring in the slot walk
    hipLaunchKernelGGL((k_walks<LAYOUT, S, true, true, 2>), dim3((unsigned)nb), dim3(BS), 0, s, a);
  } else if (X && ties && a.exp >= 5 && a.xyz && !a.ref_walk) {
    // sensitivity experiments: non-temporal tet loads (5; r01: +25 % on C3,
    // non-temporal output stores measured +4 % and removed); at least 5 (6)
    // or 6 (7) waves per SIMD asked of the register allocator
    if (a.exp == 5) hipLaunchKernelGGL((k_walks<LAYOUT, S, true, true, WALK_RING, 1>), dim3((unsigned)nb), dim3(BS), 0, s, a);
    else if (a.exp == 6) hipLaunchKernelGGL((k_walks<LAYOUT, S, true, true, WALK_RING, 0, 5>), dim3((unsigned)nb), dim3(BS), 0, s, a);
    else hipLaunchKernelGGL((k_walks<LAYOUT, S, true, true, WALK_RING, 0, 6>), dim3((unsigned)nb), dim3(BS), 0, s, a);
  } else if (X && !a.ref_walk) {
    // production: the slot walk, dense coordinates unless disabled
    if (a.xyz) {
      if (ties) hipLaunchKernelGGL((k_walks<LAYOUT, S, true, true>), dim3((unsigned)nb), dim3(BS), 0, s, a);
      else hipLaunchKernelGGL((k_walks<LAYOUT, S, false, true>), dim3((unsigned)nb), dim3(BS), 0, s, a);
    } else {
      if (ties) hipLaunchKernelGGL((k_walks<LAYOUT, S, true, false>), dim3((unsigned)nb), dim3(BS), 0, s, a);
      else hipLaunchKernelGGL((k_walks<LAYOUT, S, false, false>), dim3((unsigned)nb), dim3(BS), 0, s, a);
    }
  } else if (ties)
    hipLaunchKernelGGL((k_walk<LAYOUT, S, true, OCC, BS>), dim3((unsigned)nb), dim3(BS), 0, s, a);
  else
    hipLaunchKernelGGL((k_walk<LAYOUT, S, false, OCC, BS>), dim3((unsigned)nb), dim3(BS), 0, s, a);
}
template <int LAYOUT, int S>
static void launch_walk_t(const VolArgs &a, int ties, int64_t nb, hipStream_t s) {
  (void)nb;
  if (a.block == 1024) launch_walk_o<LAYOUT, S, 1, 1024>(a, ties, s);
  else if (a.block == 512) launch_walk_o<LAYOUT, S, 1, 512>(a, ties, s);
  else if (a.occ == 5) launch_walk_o<LAYOUT, S, 5, 256>(a, ties, s);
  else launch_walk_o<LAYOUT, S, 1, 256>(a, ties, s);
}

void launch_walk(const VolArgs &a, hipStream_t s) {
  const int64_t nb = (a.nlist + 255) / 256;
  if (nb < 1) return;
  int S = 0;
  const int lay = walk_layout(a.sd, &S);
  const int ties = a.inline_ties;
  if (lay == LAYOUT_ANI) return launch_walk_t<LAYOUT_ANI, 6>(a, ties, nb, s);
  if (lay == LAYOUT_ISO) {
    switch (S) {
      case 1: return launch_walk_t<LAYOUT_ISO, 1>(a, ties, nb, s);
      case 2: return launch_walk_t<LAYOUT_ISO, 2>(a, ties, nb, s);
      case 3: return launch_walk_t<LAYOUT_ISO, 3>(a, ties, nb, s);
      case 4: return launch_walk_t<LAYOUT_ISO, 4>(a, ties, nb, s);
      case 5: return launch_walk_t<LAYOUT_ISO, 5>(a, ties, nb, s);
      case 6: return launch_walk_t<LAYOUT_ISO, 6>(a, ties, nb, s);
      case 7: return launch_walk_t<LAYOUT_ISO, 7>(a, ties, nb, s);
      default: return launch_walk_t<LAYOUT_ISO, 8>(a, ties, nb, s);
    }
  }
  launch_walk_t<LAYOUT_GEN, 0>(a, ties, nb, s);
}

// ---- persistent-lane walk (k_walkp) ----------------------------------------
//
// k_walk runs each wavefront for the LONGEST walk among its 64 lanes: on C2
// the walk-step histogram is 17/33/33/17 % for 1/2/3/4 steps, so every wave
// iterates 4 times for 2.45 useful steps per lane (61 % lane utilisation).
// k_walkp keeps the lanes busy instead:
//  * a persistent grid (occupancy-sized) of waves pulls chunks of 64
//    Morton-consecutive points from per-XCD counters (one atomic per chunk;
//    an XCD's L2 sees a contiguous region, idle XCDs steal from the others);
//  * a lane whose point is located takes the next point of the chunk
//    (ballot rank + shuffles) and starts walking in the same iteration;
//  * located points are queued in LDS (point, tet vertices, barycentrics) and
//    interpolated 64 at a time with every lane active.
// Walk steps, tie handling, stuck points and the interpolation are those of
// k_walk: the outputs are identical.
#define WQ_CAP 128

struct WalkQ {
  int i[WQ_CAP];
  int v[4][WQ_CAP];
  double lam[4][WQ_CAP];
};

__device__ __forceinline__ unsigned long long lanes_below() {
  const int lane = threadIdx.x & 63;
  return lane ? (~0ull >> (64 - lane)) : 0ull;
}

__device__ __forceinline__ int wuni(int x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int LAYOUT, int S>
__device__ __forceinline__ void interp_queued(const VolArgs &A, const WalkQ &Q, int slot) {
  const int i = Q.i[slot];
  const int v[4] = {Q.v[0][slot], Q.v[1][slot], Q.v[2][slot], Q.v[3][slot]};
  const double phi[4] = {Q.lam[0][slot], Q.lam[1][slot], Q.lam[2][slot], Q.lam[3][slot]};
  const unsigned wm = interp_layout<LAYOUT, S>(A.sol, A.sd, v, phi, A.out + (int64_t)i * A.sd.S);
  A.wmask[i] = (uint8_t)(wm | A.const_bit);
}

template <int LAYOUT, int S, bool TIES>
__global__ __launch_bounds__(256) void k_walkp(VolArgs A) {
  __shared__ WalkQ Qs[4];
  const int lane = threadIdx.x & 63;
  WalkQ &Q = Qs[threadIdx.x >> 6];
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  unsigned s_cnt = 0, s_sum = 0, s_max = 0, s_min = 0xffffffffu;

  // chunk stream (wave-uniform state)
  int reg = blockIdx.x & 7, tries = 0, b_cnt = 0, b_used = 0, qn = 0;
  // this lane's element of the current chunk
  int b_i = -1, b_h = 0;
  double b_x = 0.0, b_y = 0.0, b_z = 0.0;

  // this lane's walk
  int i = -1, cur = 0, step = 0;
  bool fresh = false;
  D3 p{0.0, 0.0, 0.0};
  TetRec t;
#pragma unroll
  for (int l = 0; l < 4; l++) { t.v[l] = 0; t.nb[l] = 0; }
  D3 P[4];
#pragma unroll
  for (int l = 0; l < 4; l++) P[l] = D3{0.0, 0.0, 0.0};
  int ring[WALK_RING];
#pragma unroll
  for (int r = 0; r < WALK_RING; r++) ring[r] = 0;
  double lam[4] = {0.0, 0.0, 0.0, 0.0};

  for (;;) {
    // ---- refill idle lanes from the chunk stream
    for (;;) {
      const unsigned long long idle = __ballot(i < 0);
      if (!idle) break;
      if (b_used >= b_cnt) {
        if (tries >= 8) break;
        unsigned long long c = 0;
        if (lane == 0) c = atomicAdd(A.wctr + reg, 64ull);
        c = ((unsigned long long)(unsigned)__shfl((int)(c >> 32), 0) << 32) |
            (unsigned)__shfl((int)(c & 0xffffffffu), 0);
        const int64_t lo = (int64_t)reg * A.region + (int64_t)c;
        const int64_t hi = min((int64_t)(reg + 1) * A.region, A.nlist);
        if (lo >= hi) {
          reg = (reg + 1) & 7;
          tries++;
          continue;
        }
        b_cnt = wuni((int)min((int64_t)64, hi - lo));
        b_used = 0;
        if (lane < b_cnt) {
          const int64_t jj = lo + lane;
          b_i = A.list[jj];
          const Pt4 qq{A.qv[3 * jj], A.qv[3 * jj + 1], A.qv[3 * jj + 2], 0.0};
          b_x = qq.x; b_y = qq.y; b_z = qq.z;
          b_h = walk_hint(A.grid, A.g, D3{b_x, b_y, b_z}, A.grid64);
        }
      }
      const int rank = __popcll(idle & lanes_below());
      const int avail = b_cnt - b_used;
      const int src = (b_used + rank) & 63;
      const int si = __shfl(b_i, src), sh = __shfl(b_h, src);
      const double sx = __shfl(b_x, src), sy = __shfl(b_y, src), sz = __shfl(b_z, src);
      if (i < 0 && rank < avail) {
        i = si;
        p = D3{sx, sy, sz};
        cur = sh;
        fresh = true;
        step = 0;
#pragma unroll
        for (int r = 0; r < WALK_RING; r++) ring[r] = 0;
        A.start[i] = cur;
      }
      b_used = wuni(b_used + min(__popcll(idle), avail));
    }
    if (!__ballot(i >= 0)) break;

    // ---- one walk step for every lane holding a point
    bool done = false, found = false;
    if (i >= 0) {
      const TetRec u = A.tets[cur];
      step++;
      if (u.v[0] <= 0) {
        done = true;                                   // !MG_EOK: let the scan decide
      } else {
        if (fresh) {
          P[0] = ld3(A.pts, u.v[0]); P[1] = ld3(A.pts, u.v[1]);
          P[2] = ld3(A.pts, u.v[2]); P[3] = ld3(A.pts, u.v[3]);
        } else {
          // shared face: permute the known coordinates, gather the new vertex
          bool m[4][4];
          int nnew = 0, lnew = 0;
#pragma unroll
          for (int l = 0; l < 4; l++) {
#pragma unroll
            for (int k = 0; k < 4; k++) m[l][k] = (u.v[l] == t.v[k]);
            const bool any = m[l][0] | m[l][1] | m[l][2] | m[l][3];
            nnew += any ? 0 : 1;
            lnew = any ? lnew : l;
          }
          if (nnew == 1) {
            const D3 pn = ld3(A.pts, pick4(u.v, lnew));
            D3 W[4];
#pragma unroll
            for (int l = 0; l < 4; l++)
              W[l] = dsel(m[l][0], P[0], dsel(m[l][1], P[1], dsel(m[l][2], P[2], dsel(m[l][3], P[3], pn))));
#pragma unroll
            for (int l = 0; l < 4; l++) P[l] = W[l];
          } else {                                     // inconsistent adjacency
            P[0] = ld3(A.pts, u.v[0]); P[1] = ld3(A.pts, u.v[1]);
            P[2] = ld3(A.pts, u.v[2]); P[3] = ld3(A.pts, u.v[3]);
          }
        }
        t = u;
        fresh = false;
        double num[4], vol;
        face_nums(P, p, num, &vol);
        const double rv = 1.0 / vol;
#pragma unroll
        for (int f = 0; f < 4; f++) lam[f] = -(num[f] * rv);
        double lmin = fmin(fmin(lam[0], lam[1]), fmin(lam[2], lam[3]));
        if (lmin > -PMX_EPS - APPROX_GUARD) {
#pragma unroll
          for (int f = 0; f < 4; f++) lam[f] = -num[f] / vol;
          lmin = fmin(fmin(lam[0], lam[1]), fmin(lam[2], lam[3]));
          found = lmin > -PMX_EPS;                     // src/barycoord_pmmg.c:102-107
        }
        if (found || step >= A.max_walk) {
          done = true;
        } else {
          int rk[4];
          wranks(lam, rk);
#pragma unroll
          for (int r = WALK_RING - 1; r > 0; r--) ring[r] = ring[r - 1];
          ring[0] = cur;
          int next = 0;
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int f = (rk[0] == r) ? 0 : (rk[1] == r) ? 1 : (rk[2] == r) ? 2 : 3;
            const int nb = pick4(t.nb, f);
            bool seen = false;
#pragma unroll
            for (int q = 0; q < WALK_RING; q++) seen |= (ring[q] == nb);
            if (!next && nb && !seen) next = nb;
          }
          if (next) cur = next;
          else done = true;
        }
      }
    }
    // ---- finish: located -> LDS queue, near-face ties -> k_ties, else stuck
    bool push = false;
    if (done) {
      bool tie = false;
      if (found) {
        const double lmn = fmin(fmin(lam[0], lam[1]), fmin(lam[2], lam[3]));
        tie = lmn < TIE_NEAR && (!TIES || face_tie(A, p, cur, t, lam));
      }
      if (found && !tie) {
        A.elem[i] = cur;
        A.status[i] = 1;
        A.steps[i] = step;
        push = true;
        s_cnt++; s_sum += step;
        s_max = max(s_max, (unsigned)step);
        s_min = min(s_min, (unsigned)step);
      } else if (found) {
        const unsigned slot = atomicAdd(A.tie_count, 1u);
        A.tie_list[slot] = make_int2(i, cur);
        A.steps[i] = step;
      } else {
        const unsigned slot = atomicAdd(A.stuck_count, 1u);
        A.stuck_list[slot] = i;
        A.found[slot] = 0x7fffffff;
        A.bestk[slot] = 0x7fffffff;
        A.best[slot] = ~0ull;
        A.steps[i] = -step;
      }
    }
    const unsigned long long pm = __ballot(push);
    if (push) {
      const int slot = qn + __popcll(pm & lanes_below());
      Q.i[slot] = i;
#pragma unroll
      for (int l = 0; l < 4; l++) { Q.v[l][slot] = t.v[l]; Q.lam[l][slot] = lam[l]; }
    }
    qn = wuni(qn + __popcll(pm));
    if (done) i = -1;
    if (qn >= 64) {
      wave_sync();
      interp_queued<LAYOUT, S>(A, Q, qn - 64 + lane);
      qn -= 64;
      wave_sync();
    }
  }
  if (qn > 0) {
    wave_sync();
    if (lane < qn) interp_queued<LAYOUT, S>(A, Q, lane);
  }
  // per-wave statistics; records of waves this grid does not have are zeroed
  wave_stats_w(A.wstats + wave, s_cnt, s_sum, s_max, s_min);
  const int64_t nrec = (A.nlist + 63) / 64;
  for (int64_t r = wave + nwaves; r < nrec; r += nwaves)
    if (lane == 0) A.wstats[r] = make_uint4(0, 0, 0, 0xffffffffu);
}

template <int LAYOUT, int S>
static void launch_walkp_t(const VolArgs &a, int ties, hipStream_t s) {
  const void *fn = ties ? (const void *)k_walkp<LAYOUT, S, true> : (const void *)k_walkp<LAYOUT, S, false>;
  int dev = 0, cus = 0, per_cu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, 0);
  const int64_t chunks = (a.nlist + 63) / 64;
  int64_t nb = (int64_t)std::max(per_cu, 1) * std::max(cus, 1);
  nb = std::max<int64_t>(1, std::min<int64_t>(nb, (chunks + 3) / 4));
  if (ties)
    hipLaunchKernelGGL((k_walkp<LAYOUT, S, true>), dim3((unsigned)nb), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((k_walkp<LAYOUT, S, false>), dim3((unsigned)nb), dim3(256), 0, s, a);
}

void launch_walkp(const VolArgs &a, hipStream_t s) {
  if (a.nlist < 1) return;
  int S = 0;
  const int lay = walk_layout(a.sd, &S);
  const int ties = a.inline_ties;
  if (lay == LAYOUT_ANI) return launch_walkp_t<LAYOUT_ANI, 6>(a, ties, s);
  if (lay == LAYOUT_ISO) {
    switch (S) {
      case 1: return launch_walkp_t<LAYOUT_ISO, 1>(a, ties, s);
      case 2: return launch_walkp_t<LAYOUT_ISO, 2>(a, ties, s);
      case 3: return launch_walkp_t<LAYOUT_ISO, 3>(a, ties, s);
      case 4: return launch_walkp_t<LAYOUT_ISO, 4>(a, ties, s);
      case 5: return launch_walkp_t<LAYOUT_ISO, 5>(a, ties, s);
      case 6: return launch_walkp_t<LAYOUT_ISO, 6>(a, ties, s);
      case 7: return launch_walkp_t<LAYOUT_ISO, 7>(a, ties, s);
      default: return launch_walkp_t<LAYOUT_ISO, 8>(a, ties, s);
    }
  }
  launch_walkp_t<LAYOUT_GEN, 0>(a, ties, s);
}
