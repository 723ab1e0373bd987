// pmx_kernels.hip -- gfx950 kernels of the transfer path (volume part).
//
// k_hint_build       uniform grid over the background bbox, cell -> largest
//                    tet index whose centroid falls in it (deterministic)
// k_locate_vol       one thread per new vertex: adjacency walk from the hint
//                    (PMMG_locatePointVol, reference src/locate_pmmg.c:786-883)
//                    fused with PMMG_interp4bar_{iso,ani}
//                    (src/interpmesh_pmmg.c:206-270); stuck lanes are
//                    compacted into a list (wave-aggregated atomic)
// k_exh_find         LDS-staged exhaustive scan for the stuck list: smallest
//                    containing tet index == the reference's first hit in
//                    index order (src/locate_pmmg.c:737-770)
// k_exh_closest[_idx] argmin of |lambda_min|*vol over all tets for points
//                    contained nowhere, then the reference's closest-vertex
//                    barycentrics (src/barycoord_pmmg.c:371-404)
// k_exh_finish       interpolation for the stuck list
#include <algorithm>
#include "pmx_device.h"
#include "pmx_kernels.h"

#define WALK_RING 4

// rank of each value in the stable ascending order (ties: lower index first)
__device__ __forceinline__ void stable_ranks(const double l[4], int rk[4]) {
  rk[0] = rk[1] = rk[2] = rk[3] = 0;
#pragma unroll
  for (int a = 0; a < 4; a++)
#pragma unroll
    for (int b = a + 1; b < 4; b++) {
      // b after a unless l[b] < l[a]
      bool bfirst = l[b] < l[a];
      rk[a] += bfirst ? 1 : 0;
      rk[b] += bfirst ? 0 : 1;
    }
}


__device__ __forceinline__ int clampi(double t, int n) {
  if (!(t > 0.0)) return 0;                 // also catches NaN
  if (t >= (double)(n - 1)) return n - 1;
  return (int)t;
}

__device__ __forceinline__ int64_t cell_of(const GridDesc &g, D3 p, int *c) {
  c[0] = clampi((p.x - g.lo[0]) * g.inv[0], g.dim[0]);
  c[1] = clampi((p.y - g.lo[1]) * g.inv[1], g.dim[1]);
  c[2] = clampi((p.z - g.lo[2]) * g.inv[2], g.dim[2]);
  return (int64_t)c[0] + (int64_t)g.dim[0] * ((int64_t)c[1] + (int64_t)g.dim[1] * c[2]);
}

__device__ int hint_lookup(const int *grid, const GridDesc &g, D3 p) {
  int c[3];
  int k = grid[cell_of(g, p, c)];
  if (k) return k;
  for (int r = 1; r <= 3; r++) {
    for (int dz = -r; dz <= r; dz++)
      for (int dy = -r; dy <= r; dy++)
        for (int dx = -r; dx <= r; dx++) {
          if (max(abs(dx), max(abs(dy), abs(dz))) != r) continue;
          int x = c[0] + dx, y = c[1] + dy, z = c[2] + dz;
          if (x < 0 || y < 0 || z < 0 || x >= g.dim[0] || y >= g.dim[1] || z >= g.dim[2]) continue;
          int kk = grid[(int64_t)x + (int64_t)g.dim[0] * ((int64_t)y + (int64_t)g.dim[1] * z)];
          if (kk) return kk;
        }
  }
  return 1;
}

template <bool MID, bool CENTRAL, bool DX = false, bool FX = false, bool QX = false>
__global__ __launch_bounds__(256) void k_hint_build(const int4 *__restrict__ src, int64_t sstride,
                                                    const Pt4 *__restrict__ pts, int64_t ne,
                                                    int stride, int *__restrict__ grid,
                                                    GridDesc g,
                                                    unsigned long long *__restrict__ grid64,
                                                    const double *__restrict__ xyz = nullptr,
                                                    const float *__restrict__ xyzf = nullptr,
                                                    const unsigned long long *__restrict__ xyzq = nullptr) {
  // one sample per thread; XCD-aware block order: each XCD's L2 serves a
  // contiguous range of samples, i.e. neighbouring tets sharing vertices
  const int64_t n = (ne + stride - 1) / stride;
  const int64_t t = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int64_t k = 1 + t * stride;
  // sampled tet k: from the packed sample stream (sstride 1, coalesced) or
  // from every stride-th record of the 16-B connectivity stream
  const int4 v = src[t * sstride];
  if (v.x <= 0) return;
  D3 m;
  if constexpr (QX) {
    // QX: the vertices' grid coordinates in 21-bit fixed point (HINT_QF
    // fraction bits, packed x | y << 21 | z << 42 at upload): one 8-B gather
    // per vertex, the centroid's cell by integer sums and a shift
    const unsigned long long a = xyzq[v.x], b = xyzq[v.y], c = xyzq[v.z], d = xyzq[v.w];
    const unsigned long long M = (1ull << 21) - 1;
    int cq[3];
#pragma unroll
    for (int ax = 0; ax < 3; ax++) {
      const int sh = 21 * ax;
      const unsigned s4 = (unsigned)((a >> sh) & M) + (unsigned)((b >> sh) & M) +
                          (unsigned)((c >> sh) & M) + (unsigned)((d >> sh) & M);
      cq[ax] = min((int)(s4 >> (HINT_QF + 2)), g.dim[ax] - 1);
    }
    grid[(int64_t)cq[0] + (int64_t)g.dim[0] * ((int64_t)cq[1] + (int64_t)g.dim[1] * cq[2])] = (int)k;
    return;
  } else if constexpr (FX) {
    // FX: centroid from the 12-B single-precision copy of the coordinates (one
    // 12-B gather per vertex instead of 24 B in two loads).  The cell only
    // picks a start tet, and the located tet does not depend on the start.
    auto ldf = [&](int i) -> float3 {
      const float *r = xyzf + 3 * (int64_t)i;
      return make_float3(r[0], r[1], r[2]);
    };
    const float3 a = ldf(v.x), b = ldf(v.y), c = ldf(v.z), d = ldf(v.w);
    m = D3{(double)((a.x + b.x + c.x + d.x) * 0.25f), (double)((a.y + b.y + c.y + d.y) * 0.25f),
           (double)((a.z + b.z + c.z + d.z) * 0.25f)};
  } else if (MID) {
    // midpoint of edge v0-v1: a point of the tet's closure, 2 gathers
    const D3 a = ld3(pts, v.x), b = ld3(pts, v.y);
    m = D3{(a.x + b.x) * 0.5, (a.y + b.y) * 0.5, (a.z + b.z) * 0.5};
  } else {
    // DX: from the dense 24-B coordinates (VolArgs::xyz)
    auto ldp = [&](int i) -> D3 {
      if constexpr (DX) return D3{xyz[3 * (int64_t)i], xyz[3 * (int64_t)i + 1], xyz[3 * (int64_t)i + 2]};
      else return ld3(pts, i);
    };
    const D3 a = ldp(v.x), b = ldp(v.y), c = ldp(v.z), d = ldp(v.w);
    m = D3{(a.x + b.x + c.x + d.x) * 0.25, (a.y + b.y + c.y + d.y) * 0.25,
           (a.z + b.z + c.z + d.z) * 0.25};
  }
  int cc[3];
  const int64_t cell = cell_of(g, m, cc);
  if (CENTRAL) {
    // the sample whose centroid is closest to the cell centre (ties: lowest
    // tet index): deterministic, and a shorter walk from anywhere in the cell
    const double dx = m.x - (g.lo[0] + (cc[0] + 0.5) / g.inv[0]);
    const double dy = m.y - (g.lo[1] + (cc[1] + 0.5) / g.inv[1]);
    const double dz = m.z - (g.lo[2] + (cc[2] + 0.5) / g.inv[2]);
    const float d2 = (float)(dx * dx + dy * dy + dz * dz);
    const unsigned long long key =
        ((unsigned long long)__float_as_uint(d2) << 32) | (unsigned long long)(unsigned)k;
    atomicMin(grid64 + cell, key);
  } else {
    // plain store: any sampled tet of the cell is a valid start; the located
    // tet does not depend on the start (unique containing tet, or the
    // canonical min-index tet of a tie, see canonical_tet)
    grid[cell] = (int)k;
  }
}

// grid coordinates of the vertices in fixed point for k_hint_build<QX>:
// q = (x - lo) * inv * 2^HINT_QF, clamped to [0, dim * 2^HINT_QF - 1]
__global__ __launch_bounds__(256) void k_quant_xyz(const Pt4 *__restrict__ pts, int64_t n, GridDesc g,
                                                   unsigned long long *__restrict__ q) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const Pt4 p = pts[i];
    const double c[3] = {p.x, p.y, p.z};
    unsigned long long r = 0;
#pragma unroll
    for (int a = 0; a < 3; a++) {
      const double t = (c[a] - g.lo[a]) * g.inv[a] * (double)(1 << HINT_QF);
      const long long hi = ((long long)g.dim[a] << HINT_QF) - 1;
      const long long u = !(t > 0.0) ? 0 : (t >= (double)hi ? hi : (long long)t);
      r |= (unsigned long long)u << (21 * a);
    }
    q[i] = r;
  }
}
void launch_quant_xyz(const Pt4 *pts, int64_t n, GridDesc g, unsigned long long *q, hipStream_t s) {
  const int64_t nb = std::min<int64_t>(std::max<int64_t>((n + 255) / 256, 1), 65536);
  hipLaunchKernelGGL(k_quant_xyz, dim3((unsigned)nb), dim3(256), 0, s, pts, n, g, q);
}

__global__ __launch_bounds__(256) void k_fill64(unsigned long long *p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = ~0ull;
}
void launch_fill64(unsigned long long *p, int64_t n, hipStream_t s) {
  const int64_t nb = std::min<int64_t>(std::max<int64_t>((n + 255) / 256, 1), 4096);
  hipLaunchKernelGGL(k_fill64, dim3((unsigned)nb), dim3(256), 0, s, p, n);
}

// connectivity stream out of the tet records: dst[i] = src[i * stride].v
// (a kernel rather than a pitched 2-D copy: no row-count limits at 1e8 tets)
__global__ __launch_bounds__(256) void k_tet_conn(const TetRec *__restrict__ src, int64_t stride,
                                                  int64_t n, int4 *__restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int4 *r = reinterpret_cast<const int4 *>(src + i * stride);
    dst[i] = r[0];
  }
}
void launch_tet_conn(const TetRec *src, int64_t stride, int64_t n, int4 *dst, hipStream_t s) {
  int64_t nb = std::min<int64_t>(std::max<int64_t>((n + 255) / 256, 1), 16384);
  hipLaunchKernelGGL(k_tet_conn, dim3((unsigned)nb), dim3(256), 0, s, src, stride, n, dst);
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
__device__ __noinline__ int canonical_tet(const TetRec *tets, const Pt4 *pts, int k0, D3 p) {
  int vis[TIE_CAP], inq[TIE_CAP];
  int nv = 0, nq = 0, head = 0, best = k0;
  vis[nv++] = k0;
  inq[nq++] = k0;
  while (head < nq) {
    int k = inq[head++];
    TetRec t = tets[k];
    D3 P[4] = {ld3(pts, t.v[0]), ld3(pts, t.v[1]), ld3(pts, t.v[2]), ld3(pts, t.v[3])};
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
      D3 Q[4] = {ld3(pts, u.v[0]), ld3(pts, u.v[1]), ld3(pts, u.v[2]), ld3(pts, u.v[3])};
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

// ---- volume locate + interpolate ------------------------------------------

__device__ __forceinline__ bool in_ring(const int r[WALK_RING], int k) {
  bool h = false;
#pragma unroll
  for (int i = 0; i < WALK_RING; i++) h |= (r[i] == k);
  return h;
}

// Walk statistics: one 4-word record per wavefront (no same-address atomics;
// reduced on demand by pmx_locate_stats_get).  v0 profile: 4 contended
// atomics per wave serialised the whole launch.
__device__ __forceinline__ void wave_stats(uint4 *rec, unsigned cnt, unsigned sum, unsigned mx,
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

// OCC = minimum waves per SIMD requested from the register allocator
// (1 = unconstrained); selected at run time by pmx_run_opts.tune
template <int OCC>
__global__ __launch_bounds__(256, OCC) void k_locate_vol(VolArgs A) {
  int64_t b = A.xcd_swizzle ? xcd_remap(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
  int64_t j = b * blockDim.x + threadIdx.x;
  unsigned s_cnt = 0, s_sum = 0, s_max = 0, s_min = 0xffffffffu;

  if (j < A.nlist) {
    const int64_t i = A.list[j];
    Pt4 qq = A.q[i];
    D3 p{qq.x, qq.y, qq.z};
    int cur = hint_lookup(A.grid, A.g, p);
    if (A.start) A.start[i] = cur;
    int ring[WALK_RING];
#pragma unroll
    for (int r = 0; r < WALK_RING; r++) ring[r] = 0;
    int step = 0;
    bool found = false;
    int v[4];
    double lam[4];
    for (;;) {
      step++;
      TetRec t = A.tets[cur];
      if (t.v[0] <= 0) break;                       // !MG_EOK: let the scan decide
      v[0] = t.v[0]; v[1] = t.v[1]; v[2] = t.v[2]; v[3] = t.v[3];
      D3 P[4] = {ld3(A.pts, v[0]), ld3(A.pts, v[1]), ld3(A.pts, v[2]), ld3(A.pts, v[3])};
      double vol;
      tet_lambda(P, p, lam, &vol);
      // position of face f in the reference's stable ascending order of the
      // barycentrics (glibc qsort, src/barycoord_pmmg.c:306) as ranks: no
      // sorted copy of the doubles is kept live
      int rk[4];
      stable_ranks(lam, rk);
      double lmin = lam[0];
      lmin = (rk[1] == 0) ? lam[1] : lmin;
      lmin = (rk[2] == 0) ? lam[2] : lmin;
      lmin = (rk[3] == 0) ? lam[3] : lmin;
      if (lmin > -PMX_EPS) { found = true; break; }   // src/barycoord_pmmg.c:102-107
      if (step >= A.max_walk) break;
#pragma unroll
      for (int r = WALK_RING - 1; r > 0; r--) ring[r] = ring[r - 1];
      ring[0] = cur;
      // first interior, not recently visited neighbour in ascending-lambda
      // order (src/locate_pmmg.c:819-833)
      int next = 0;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        int f = (rk[0] == r) ? 0 : (rk[1] == r) ? 1 : (rk[2] == r) ? 2 : 3;
        int nb = sel4(t.nb, f);
        if (!next && nb && !in_ring(ring, nb)) next = nb;
      }
      if (!next) break;
      cur = next;
    }
    if (found) {
      // a point within the tolerance of a face/edge/vertex is contained by
      // several tets: take the smallest index among them (start-independent)
      // (resolved by k_ties: keeps the BFS out of this kernel's registers)
      double lmn = fmin(fmin(lam[0], lam[1]), fmin(lam[2], lam[3]));
      if (lmn < TIE_NEAR) {
        unsigned slot = atomicAdd(A.tie_count, 1u);
        A.tie_list[slot] = make_int2((int)i, cur);
        A.steps[i] = step;
        found = false;
        step = -1;                                  // neither found nor stuck
      }
    }
    if (found) {
      A.elem[i] = cur;
      A.status[i] = 1;
      A.steps[i] = step;
      double *out = A.out + i * A.sd.S;
      unsigned wm = interp_bar<4>(A.sol, A.sd, v, lam, out);
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
  wave_stats(A.wstats + (b * blockDim.x + threadIdx.x) / 64, s_cnt, s_sum, s_max, s_min);
}

// ---- tie resolution ----------------------------------------------------------

__device__ void d_ties(const VolArgs &A, unsigned bid, unsigned nblk) {
  const unsigned n = *A.tie_count;
  for (unsigned j = bid * blockDim.x + threadIdx.x; j < n; j += nblk * blockDim.x) {
    int2 e = A.tie_list[j];
    const int64_t i = e.x;
    Pt4 qq = A.q[i];
    D3 p{qq.x, qq.y, qq.z};
    int kc = canonical_tet(A.tets, A.pts, e.y, p);
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
    D3 P[4] = {ld3(A.pts, v[0]), ld3(A.pts, v[1]), ld3(A.pts, v[2]), ld3(A.pts, v[3])};
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
    for (unsigned j = threadIdx.x; j < m; j += blockDim.x) {
      Pt4 qq = A.q[A.list[c0 + j]];
      sp[j] = D3{qq.x, qq.y, qq.z};
    }
    __syncthreads();
    for (int64_t k = 1 + (int64_t)bid * blockDim.x + threadIdx.x; k <= A.ne;
         k += (int64_t)nblk * blockDim.x) {
      TetRec t = A.tets[k];
      if (t.v[0] <= 0) continue;
      D3 P[4] = {ld3(A.pts, t.v[0]), ld3(A.pts, t.v[1]), ld3(A.pts, t.v[2]), ld3(A.pts, t.v[3])};
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
      Pt4 qq = A.q[A.list[c0 + j]];
      sp[j] = D3{qq.x, qq.y, qq.z};
      act[j] = (A.found[c0 + j] == 0x7fffffff);
    }
    __syncthreads();
    for (int64_t k = 1 + (int64_t)bid * blockDim.x + threadIdx.x; k <= A.ne;
         k += (int64_t)nblk * blockDim.x) {
      TetRec t = A.tets[k];
      if (t.v[0] <= 0) continue;
      D3 P[4] = {ld3(A.pts, t.v[0]), ld3(A.pts, t.v[1]), ld3(A.pts, t.v[2]), ld3(A.pts, t.v[3])};
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
    Pt4 qq = A.q[i];
    D3 p{qq.x, qq.y, qq.z};
    int k = A.found[j];
    int st = 1;
    double phi[4];
    if (k == 0x7fffffff) {
      k = A.bestk[j];
      st = 0;
    }
    TetRec t = A.tets[k];
    int v[4] = {t.v[0], t.v[1], t.v[2], t.v[3]};
    D3 P[4] = {ld3(A.pts, v[0]), ld3(A.pts, v[1]), ld3(A.pts, v[2]), ld3(A.pts, v[3])};
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
// Ties, exhaustive scan (find, closest value, closest index) and the final
// interpolation of the scanned points used to be five launches that almost
// always found nothing to do (~4.5 us each).  One launch of FALLBACK_BLOCKS
// co-resident workgroups (1 per CU at most; the kernel admits 4) now reads the
// counters and leaves, or runs the phases separated by a grid barrier
// (MI355X_MICROARCH.md "barrier-counter": release fence + waitcnt before the
// arrive, relaxed agent-scope poll, acquire fence after; bounded spin).
#define FALLBACK_BLOCKS 256

__device__ __forceinline__ unsigned ld_agent(const unsigned *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ void grid_barrier(unsigned *bar, unsigned target) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    atomicAdd(bar, 1u);
    for (long it = 0; ld_agent(bar) < target && it < (1L << 26); it++) __builtin_amdgcn_s_sleep(2);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_fallback(ExhArgs E, VolArgs V) {
  const unsigned nb = gridDim.x, b = blockIdx.x;
  unsigned *bar = V.stuck_count + 4;           // counts[4], zeroed by k_run_init
  if (ld_agent(V.tie_count) == 0 && ld_agent(V.stuck_count) == 0) return;
  d_ties(V, b, nb);
  grid_barrier(bar, nb);
  if (ld_agent(V.stuck_count) == 0) return;
  d_exh_find(E, b, nb);
  grid_barrier(bar, 2 * nb);
  d_exh_closest(E, 0, b, nb);
  grid_barrier(bar, 3 * nb);
  d_exh_closest(E, 1, b, nb);
  grid_barrier(bar, 4 * nb);
  d_exh_finish(E, V, b, nb);
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

// counts[0] volume stuck, [1] surface stuck, [2] surface overflow
__global__ void k_run_init(unsigned *counts) {
  if (threadIdx.x < 8) counts[threadIdx.x] = 0;
}
void launch_run_init(unsigned *counts, hipStream_t s) {
  hipLaunchKernelGGL(k_run_init, dim3(1), dim3(64), 0, s, counts);
}

__global__ __launch_bounds__(256) void k_prologue(uint8_t *wmask, int64_t n, unsigned *counts,
                                                  int *grid, int64_t gcells, int *tgrid,
                                                  int64_t tcells) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
  if (t < 32) counts[t] = 0;
  const int64_t n16 = n / 16;
  for (int64_t i = t; i < n16; i += st) reinterpret_cast<uint4 *>(wmask)[i] = make_uint4(0, 0, 0, 0);
  for (int64_t i = n16 * 16 + t; i < n; i += st) wmask[i] = 0;
  int *gs[2] = {grid, tgrid};
  const int64_t cs[2] = {gcells, tcells};
#pragma unroll
  for (int k = 0; k < 2; k++) {
    int *g = gs[k];
    if (!g) continue;
    const int64_t g4 = cs[k] / 4;
    for (int64_t i = t; i < g4; i += st) reinterpret_cast<int4 *>(g)[i] = make_int4(0, 0, 0, 0);
    for (int64_t i = g4 * 4 + t; i < cs[k]; i += st) g[i] = 0;
  }
}
void launch_prologue(uint8_t *wmask, int64_t n, unsigned *counts, int *grid, int64_t gcells,
                     int *tgrid, int64_t tcells, hipStream_t s) {
  int64_t work = std::max<int64_t>(n / 16, std::max<int64_t>(grid ? gcells / 4 : 0, tgrid ? tcells / 4 : 0));
  int64_t nb = std::min<int64_t>(std::max<int64_t>((work + 255) / 256, 1), 4096);
  hipLaunchKernelGGL(k_prologue, dim3((unsigned)nb), dim3(256), 0, s, wmask, n, counts, grid, gcells,
                     tgrid, tcells);
}

void launch_hint_build(const int4 *tetv, const int4 *packed, const Pt4 *pts, int64_t ne,
                       int stride, int *grid, GridDesc g, int mid, hipStream_t s,
                       unsigned long long *grid64, const double *xyz, const float *xyzf,
                       const unsigned long long *xyzq) {
  const int64_t n = (ne + stride - 1) / stride;
  const int64_t nb = std::max<int64_t>((n + 255) / 256, 1);
  const int4 *src = packed ? packed : tetv + 1;
  const int64_t sstride = packed ? 1 : stride;
  if (grid64)
    hipLaunchKernelGGL((k_hint_build<false, true>), dim3((unsigned)nb), dim3(256), 0, s, src, sstride,
                       pts, ne, stride, grid, g, grid64, nullptr);
  else if (xyzq)
    hipLaunchKernelGGL((k_hint_build<false, false, false, false, true>), dim3((unsigned)nb), dim3(256), 0,
                       s, src, sstride, pts, ne, stride, grid, g, grid64, nullptr, nullptr, xyzq);
  else if (xyzf)
    hipLaunchKernelGGL((k_hint_build<false, false, false, true>), dim3((unsigned)nb), dim3(256), 0, s,
                       src, sstride, pts, ne, stride, grid, g, grid64, nullptr, xyzf);
  else if (mid)
    hipLaunchKernelGGL((k_hint_build<true, false>), dim3((unsigned)nb), dim3(256), 0, s, src, sstride,
                       pts, ne, stride, grid, g, grid64, nullptr);
  else if (xyz)
    hipLaunchKernelGGL((k_hint_build<false, false, true>), dim3((unsigned)nb), dim3(256), 0, s, src,
                       sstride, pts, ne, stride, grid, g, grid64, xyz);
  else
    hipLaunchKernelGGL((k_hint_build<false, false>), dim3((unsigned)nb), dim3(256), 0, s, src, sstride,
                       pts, ne, stride, grid, g, grid64, nullptr);
}
void launch_locate_vol(const VolArgs &a, hipStream_t s) {
  int64_t nb = (a.nlist + 255) / 256;
  if (nb < 1) return;
  switch (a.occ) {
    case 6: hipLaunchKernelGGL(k_locate_vol<6>, dim3((unsigned)nb), dim3(256), 0, s, a); break;
    case 8: hipLaunchKernelGGL(k_locate_vol<8>, dim3((unsigned)nb), dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL(k_locate_vol<1>, dim3((unsigned)nb), dim3(256), 0, s, a); break;
  }
}
void launch_exhaustive(const ExhArgs &e, const VolArgs &v, hipStream_t s) {
  int64_t nb = (e.ne + 255) / 256;
  if (nb > 2048) nb = 2048;
  if (nb < 1) nb = 1;
  (void)nb;
  hipLaunchKernelGGL(k_fallback, dim3(FALLBACK_BLOCKS), dim3(256), 0, s, e, v);
}
void launch_const_metric(const int8_t *kind, int64_t nq, double *out, int S, int off, int size,
                         double hsiz, uint8_t *wmask, int imet, hipStream_t s) {
  int64_t nb = (nq + 255) / 256;
  if (nb > 8192) nb = 8192;
  if (nb < 1) return;
  hipLaunchKernelGGL(k_const_metric, dim3((unsigned)nb), dim3(256), 0, s, kind, nq, out, S, off,
                     size, hsiz, wmask, imet);
}
