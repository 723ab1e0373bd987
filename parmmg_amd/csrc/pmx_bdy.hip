// pmx_bdy.hip -- surface (MG_BDY) part of the transfer path on gfx950.
//
// One thread per boundary vertex runs PMMG_locatePointBdy (reference
// src/locate_pmmg.c:587-723) with its shadow-wedge / shadow-cone tests
// (:209-334) and the PMMG_interp{3,2}bar / PMMG_copyMetrics dispatch of
// src/interpmesh_pmmg.c:550-599.
//
// Device semantics (documented in DESIGN.md): each query starts from the hint
// triangle instead of the previous query's result, and sees the old-mesh point
// flags in the state PMMG_precompute_nodeTrias leaves them (number of incident
// trias), with mesh->base = query ordinal + 1.  The flags a query writes
// (visited trias, wedge/cone marks) are kept in thread-private lists.
#include "pmx_device.h"
#include "pmx_kernels.h"
#include <hipcub/hipcub.hpp>
#include "pmx_internal.h"
#include <algorithm>
#include <cmath>

#define UNSET (-1)

__device__ __constant__ int NXT2d[6] = {1, 2, 0, 1, 2, 0};

struct BdyArgs {
  const double *xyz;        // old vertices, 24 B
  const TriRec *tris;
  const Pt4 *trn;
  const int2 *ntrange;      // fan [lo, hi) in ntlist of vertex l of tria k, at 3 k + l
  const int *ntlist;
  const double *sol;
  SolDesc sd;
  const double *q;          // new points, dense x y z (0-based)
  const int8_t *kind;
  int64_t nq, nt;
  double hausd;
  const int *grid;     // tria hint grid (shares GridDesc with the tet grid)
  GridDesc g;
  double *out;
  uint8_t *wmask;
  int *elem, *status, *steps, *start, *edge, *vertex;
  int *stuck_list;     // bdy exhaustive list
  unsigned *stuck_count;
  int *ovf_list;       // private-list overflow
  unsigned *ovf_count;
  const int *list;       // indices of the boundary points
  int64_t nlist;         // upper bound (launch size); the step's count is *nlist_dev
  const int *nlist_dev;
  uint4 *wstats;         // per-wave walk statistics
  // PMX_RUN_SEQUENTIAL_SURFACE's speculative pass: per point its start tria
  // and mesh->base (null: the hint tria, ordinal + 1), and whether the walk
  // ran a shadow-wedge test (the only path to the point flags)
  const int *seq_start, *seq_base;
  uint8_t *seq_w;
};

// thread-private query state: visited trias + point-flag overrides
template <int CAP> struct RegState {
  int vis[CAP];
  int ovp[CAP], ovf[CAP];
  int nv = 0, no = 0;
  bool over = false;
  __device__ void init(int *, int) {}
  __device__ int &V(int i) { return vis[i]; }
  __device__ int &OP(int i) { return ovp[i]; }
  __device__ int &OF(int i) { return ovf[i]; }
  static constexpr int cap() { return CAP; }
};
struct GlobState {
  int *vis, *ovp, *ovf;
  int nv = 0, no = 0, capv = 0;
  bool over = false;
  __device__ void init(int *ws, int cap) {
    vis = ws; ovp = ws + cap; ovf = ws + 2 * cap; capv = cap;
  }
  __device__ int &V(int i) { return vis[i]; }
  __device__ int &OP(int i) { return ovp[i]; }
  __device__ int &OF(int i) { return ovf[i]; }
};
// GlobState with hashed lists (the sequential mode's overflow pass: walks
// from the predecessors' trias run hundreds of steps, and the linear lists
// make each of them quadratic -- C3: 82-96 ms, a few walks long).  Open
// addressing in per-thread tables tagged with the walk's generation (its
// overflow-list position + 1; the caller zeroes the tables before the pass):
// the same set and map as the lists
struct GlobHashState {
  int2 *vt;                      // visited trias: (tria, gen)
  int4 *ft;                      // point flags: (point, gen, flag, -)
  int mask = 0, gen = 0, nv = 0, no = 0, capv = 0;
  bool over = false;
};
#define GHS_SLOTS 4096           // per table and thread; at most half of them used
__device__ __forceinline__ unsigned ghs_hash(int x) { return (unsigned)x * 2654435761u; }
__device__ bool visited(GlobHashState &s, int t) {
  for (unsigned h = ghs_hash(t) & s.mask;; h = (h + 1) & s.mask) {
    const int2 e = s.vt[h];
    if (e.y != s.gen) return false;
    if (e.x == t) return true;
  }
}
__device__ void mark_visited(GlobHashState &s, int t) {
  unsigned h = ghs_hash(t) & s.mask;
  for (;; h = (h + 1) & s.mask) {
    const int2 e = s.vt[h];
    if (e.y != s.gen) break;
    if (e.x == t) return;
  }
  if (s.nv >= s.capv) { s.over = true; return; }
  s.vt[h] = make_int2(t, s.gen);
  s.nv++;
}
__device__ int get_flag(GlobHashState &s, int p, int cnt) {
  for (unsigned h = ghs_hash(p) & s.mask;; h = (h + 1) & s.mask) {
    const int4 e = s.ft[h];
    if (e.y != s.gen) return cnt;
    if (e.x == p) return e.z;
  }
}
__device__ void set_flag(GlobHashState &s, int p, int f) {
  unsigned h = ghs_hash(p) & s.mask;
  for (;; h = (h + 1) & s.mask) {
    const int4 e = s.ft[h];
    if (e.y != s.gen) break;
    if (e.x == p) { s.ft[h].z = f; return; }
  }
  if (s.no >= s.capv) { s.over = true; return; }
  s.ft[h] = make_int4(p, s.gen, f, 0);
  s.no++;
}

// the reference's own state, for the sequential replay (one lane): tria
// flags tf[] compared with mesh->base, point flags pf[] kept across queries
// (PF_INIT: still the incident-tria count PMMG_precompute_nodeTrias left)
#define PF_INIT ((int)0x80808080)
struct SeqState {
  int *tf, *pf;
  int base;
  bool over = false;
};
// (agent-scope accesses: the replaying lane reads back what it wrote in
// earlier queries, never a stale L1 line)
__device__ __forceinline__ int ld_flag(const int *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_flag(int *p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool visited(SeqState &s, int t) { return ld_flag(s.tf + t) == s.base; }
__device__ __forceinline__ void mark_visited(SeqState &s, int t) { st_flag(s.tf + t, s.base); }
__device__ __forceinline__ int get_flag(SeqState &s, int p, int cnt) {
  const int f = ld_flag(s.pf + p);
  return f == PF_INIT ? cnt : f;
}
__device__ __forceinline__ void set_flag(SeqState &s, int p, int f) { st_flag(s.pf + p, f); }

template <class St> __device__ __forceinline__ int st_cap(const St &s);
template <int C> __device__ __forceinline__ int st_cap(const RegState<C> &) { return C; }
template <> __device__ __forceinline__ int st_cap(const GlobState &s) { return s.capv; }

// RegState: every access at a compile-time index (unrolled, predicated), so
// the lists live in VGPRs; a runtime index would put them in scratch and make
// each visited / flag lookup a dependent memory round trip (r01: the surface
// walk was latency-bound on exactly that)
template <int C> __device__ __forceinline__ bool visited(RegState<C> &s, int t) {
  bool h = false;
#pragma unroll
  for (int i = 0; i < C; i++) h |= (i < s.nv) & (s.vis[i] == t);
  return h;
}
template <int C> __device__ __forceinline__ void mark_visited(RegState<C> &s, int t) {
  if (visited(s, t)) return;
  if (s.nv >= C) { s.over = true; return; }
#pragma unroll
  for (int i = 0; i < C; i++)
    if (i == s.nv) s.vis[i] = t;
  s.nv++;
}
// flag of point p: the query's own override, else the incident-tria count
// PMMG_precompute_nodeTrias leaves (cnt, from the caller's fan record)
template <int C> __device__ __forceinline__ int get_flag(RegState<C> &s, int p, int cnt) {
  bool hit = false;
  int f = 0;
#pragma unroll
  for (int i = 0; i < C; i++) {
    const bool m = (i < s.no) & (s.ovp[i] == p);
    f = m ? s.ovf[i] : f;
    hit |= m;
  }
  return hit ? f : cnt;
}
template <int C> __device__ __forceinline__ void set_flag(RegState<C> &s, int p, int f) {
  bool upd = false;
#pragma unroll
  for (int i = 0; i < C; i++) {
    const bool m = (i < s.no) & (s.ovp[i] == p);
    s.ovf[i] = m ? f : s.ovf[i];
    upd |= m;
  }
  if (upd) return;
  if (s.no >= C) { s.over = true; return; }
#pragma unroll
  for (int i = 0; i < C; i++) {
    s.ovp[i] = (i == s.no) ? p : s.ovp[i];
    s.ovf[i] = (i == s.no) ? f : s.ovf[i];
  }
  s.no++;
}

template <class St> __device__ bool visited(St &s, int t) {
  for (int i = 0; i < s.nv; i++)
    if (s.V(i) == t) return true;
  return false;
}
template <class St> __device__ void mark_visited(St &s, int t) {
  if (visited(s, t)) return;
  if (s.nv >= st_cap(s)) { s.over = true; return; }
  s.V(s.nv++) = t;
}
template <class St> __device__ int get_flag(St &s, int p, int cnt) {
  for (int i = s.no - 1; i >= 0; i--)
    if (s.OP(i) == p) return s.OF(i);
  return cnt;
}
template <class St> __device__ void set_flag(St &s, int p, int f) {
  for (int i = 0; i < s.no; i++)
    if (s.OP(i) == p) { s.OF(i) = f; return; }
  if (s.no >= st_cap(s)) { s.over = true; return; }
  s.OP(s.no) = p;
  s.OF(s.no) = f;
  s.no++;
}

// PMMG_quickarea (src/barycoord_pmmg.c:41-59)
__device__ __forceinline__ double qarea(D3 a, D3 b, D3 c, D3 n) {
  double abx = b.x - a.x, aby = b.y - a.y, abz = b.z - a.z;
  double acx = c.x - a.x, acy = c.y - a.y, acz = c.z - a.z;
  double a0 = aby * acz - abz * acy, a1 = abz * acx - abx * acz, a2 = abx * acy - aby * acx;
  return a0 * n.x + a1 * n.y + a2 * n.z;
}

struct Bary { double val[4]; int idx[4]; };

// PMMG_barycoord2d_compute + sort + isInside (src/barycoord_pmmg.c:191-223,
// :274-284) on the geometry P (area) of a tria with the unit normal n;
// returns the signed normal distance h in b.val[3]
__device__ __forceinline__ bool tria_eval_pre(const D3 P[3], D3 n, double area, D3 p, Bary &b) {
  const D3 c = P[0];
  double h = 0.0;
  h += (p.x - c.x) * n.x;
  h += (p.y - c.y) * n.y;
  h += (p.z - c.z) * n.z;
  D3 q{p.x - h * n.x, p.y - h * n.y, p.z - h * n.z};
  b.val[0] = qarea(q, P[1], P[2], n) / area;
  b.val[1] = qarea(q, P[2], P[0], n) / area;
  b.val[2] = qarea(q, P[0], P[1], n) / area;
  b.idx[0] = 0; b.idx[1] = 1; b.idx[2] = 2;
  b.val[3] = h; b.idx[3] = 3;
  sort3(b.val, b.idx);
  return b.val[0] > -PMX_EPS;
}

__device__ bool tria_eval(const BdyArgs &A, int g, int kn, D3 p, Bary &b) {
  const TriRec t = A.tris[g];
  const Pt4 nn = A.trn[kn];
  const D3 P[3] = {ld3(A.xyz, t.v[0]), ld3(A.xyz, t.v[1]), ld3(A.xyz, t.v[2])};
  return tria_eval_pre(P, D3{nn.x, nn.y, nn.z}, A.trn[g].w, p, b);
}

__device__ __forceinline__ double norm3(double a, double b, double c) {
  double r = 0.0;
  r += a * a;
  r += b * b;
  r += c * c;
  return sqrt(r);
}

// centroid distance of a tria (closest tracking, src/locate_pmmg.c:398-416)
__device__ __forceinline__ double centroid_dist_pre(const D3 P[3], D3 p) {
  double d0 = p.x, d1 = p.y, d2 = p.z;
#pragma unroll
  for (int j = 0; j < 3; j++) {
    d0 -= P[j].x / 3.0;
    d1 -= P[j].y / 3.0;
    d2 -= P[j].z / 3.0;
  }
  return norm3(d0, d1, d2);
}
__device__ __forceinline__ double centroid_dist(const BdyArgs &A, int g, D3 p) {
  const TriRec t = A.tris[g];
  const D3 P[3] = {ld3(A.xyz, t.v[0]), ld3(A.xyz, t.v[1]), ld3(A.xyz, t.v[2])};
  return centroid_dist_pre(P, p);
}

// PMMG_locatePointInTria (src/locate_pmmg.c:385-423), geometry g, normal kn:
// the tria, its normal and its 3 vertices are gathered once; the evaluation,
// the centroid distance and PMMG_locateChkDistTria (:347-366, the same h as
// the evaluation: vertex 0 of g against the normal of kn) share them
template <class St>
__device__ __forceinline__ bool in_tria(const BdyArgs &A, St &s, int g, int kn, D3 p, Bary &b, double &cdist,
                        int &ctria) {
  mark_visited(s, g);
  const TriRec t = A.tris[g];
  const Pt4 nn = A.trn[kn];
  const double area = A.trn[g].w;
  const D3 P[3] = {ld3(A.xyz, t.v[0]), ld3(A.xyz, t.v[1]), ld3(A.xyz, t.v[2])};
  const bool found = tria_eval_pre(P, D3{nn.x, nn.y, nn.z}, area, p, b);
  const double nrm = centroid_dist_pre(P, p);
  if (nrm < cdist) { cdist = nrm; ctria = kn; }
  if (fabs(b.val[3]) > A.hausd) return false;
  return found;
}

// PMMG_locatePointInWedge (src/locate_pmmg.c:286-334)
template <class St>
__device__ int in_wedge(const BdyArgs &A, St &s, int k, int l, D3 p, int base, Bary &b) {
  int i0 = NXT2d[l], i1 = NXT2d[l + 1];   // inxt2[l], iprv2[l]
  TriRec t = A.tris[k];
  int q0 = t.v[i0], q1 = t.v[i1];
  D3 c0 = ld3(A.xyz, q0), c1 = ld3(A.xyz, q1);
  double pv[3] = {p.x - c0.x, p.y - c0.y, p.z - c0.z};
  double a[3] = {c1.x - c0.x, c1.y - c0.y, c1.z - c0.z};
  double n2 = 0.0, alpha = 0.0, dist = 0.0;
  for (int d = 0; d < 3; d++) n2 += a[d] * a[d];
  for (int d = 0; d < 3; d++) alpha += a[d] * pv[d];
  for (int d = 0; d < 3; d++) pv[d] -= (alpha / n2) * a[d];
  for (int d = 0; d < 3; d++) dist += pv[d] * pv[d];
  dist = sqrt(dist);
  if (dist > A.hausd) return UNSET;
  if (alpha < 0.0) { set_flag(s, q1, base); return i0; }
  if (alpha > n2) { set_flag(s, q0, base); return i1; }
  b.idx[0] = 0; b.idx[1] = 1; b.idx[2] = 2;
  b.val[l] = 0.0;
  b.val[i0] = 1.0 - alpha / n2;
  b.val[i1] = alpha / n2;
  return 4;
}

// PMMG_locatePointInCone (src/locate_pmmg.c:209-270)
template <class St>
__device__ bool in_cone(const BdyArgs &A, St &s, int k, int iloc, D3 p, int base) {
  int ip = A.tris[k].v[iloc];
  D3 c0 = ld3(A.xyz, ip);
  set_flag(s, ip, base);
  double pv[3] = {p.x - c0.x, p.y - c0.y, p.z - c0.z};
  double dist = 0.0;
  for (int d = 0; d < 3; d++) dist += pv[d] * pv[d];
  dist = sqrt(dist);
  const int2 fan = A.ntrange[3 * k + iloc];
  for (int f = fan.x; f < fan.y; f++) {
    const int g = A.ntlist[f];
    TriRec t = A.tris[g];
    for (int j = 0; j < 3; j++) {
      int jp = t.v[j];
      if (jp == ip) continue;
      const int2 r = A.ntrange[3 * g + j];
      if (get_flag(s, jp, r.y - r.x) == ip) continue;
      set_flag(s, jp, ip);
      D3 cj = ld3(A.xyz, jp);
      double a[3] = {cj.x - c0.x, cj.y - c0.y, cj.z - c0.z};
      if (dist > A.hausd) return false;
      double alpha = 0.0;
      for (int d = 0; d < 3; d++) alpha += a[d] * pv[d];
      if (alpha > 0.0) return false;
    }
  }
  return true;
}

// ---- interpolation on a boundary triangle --------------------------------

__device__ void interp_tria(const BdyArgs &A, int k, const Bary &b, int edge, int vtx,
                            double *out, unsigned &wm) {
  TriRec t = A.tris[k];
  int v[3] = {t.v[0], t.v[1], t.v[2]};
  double phi[3];
  // PMMG_barycoord_get(phi, barycoord, 3)
  for (int i = 0; i < 3; i++) {
    int id = b.idx[i];
    double val = b.val[i];
    if (id == 0) phi[0] = val;
    if (id == 1) phi[1] = val;
    if (id == 2) phi[2] = val;
  }
  const SolDesc &sd = A.sd;
  for (int s = 0; s < sd.nsol; ++s) {
    if (s == sd.imet && sd.metric_const) continue;
    const int sz = sd.size[s], off = sd.off[s];
    const bool met = (s == sd.imet);
    if (met && vtx != UNSET) {                       // PMMG_copyMetrics
      int src = v[0];
      if (vtx == 1) src = v[1];
      if (vtx == 2) src = v[2];
      for (int j = 0; j < sz; j++) out[off + j] = A.sol[(int64_t)src * sd.S + off + j];
      wm |= 1u << s;
    } else if (met && edge != UNSET) {               // PMMG_interp2bar_{iso,ani}
      int i0 = NXT2d[edge], i1 = NXT2d[edge + 1];
      int va = v[0], vb = v[0];
      double pa = phi[0], pb = phi[0];
      if (i0 == 1) { va = v[1]; pa = phi[1]; }
      if (i0 == 2) { va = v[2]; pa = phi[2]; }
      if (i1 == 1) { vb = v[1]; pb = phi[1]; }
      if (i1 == 2) { vb = v[2]; pb = phi[2]; }
      if (sz == 1) {
        out[off] = pa * A.sol[(int64_t)va * sd.S + off] + pb * A.sol[(int64_t)vb * sd.S + off];
        wm |= 1u << s;
      } else {
        double m0[6], m1[6], mi0[6], mi1[6], mint[6], r[6];
        for (int j = 0; j < 6; j++) {
          m0[j] = A.sol[(int64_t)va * sd.S + off + j];
          m1[j] = A.sol[(int64_t)vb * sd.S + off + j];
        }
        if (!invmat(m0, mi0)) continue;
        if (!invmat(m1, mi1)) continue;
        for (int j = 0; j < 6; j++) mint[j] = pa * mi0[j] + pb * mi1[j];
        if (!invmat(mint, r)) continue;
        for (int j = 0; j < 6; j++) out[off + j] = r[j];
        wm |= 1u << s;
      }
    } else if (sz == 6) {                             // PMMG_interp3bar_ani
      double mi[3][6], mint[6], r[6];
      bool okk = true;
      // unrolled (static indices keep mi in VGPRs); && stops at the first
      // failed inversion like the reference loop
#pragma unroll
      for (int i = 0; i < 3; i++) {
        double m[6];
#pragma unroll
        for (int j = 0; j < 6; j++) m[j] = A.sol[(int64_t)v[i] * sd.S + off + j];
        okk = okk && invmat(m, mi[i]);
      }
      if (!okk) continue;
      for (int j = 0; j < 6; j++) mint[j] = phi[0] * mi[0][j] + phi[1] * mi[1][j] + phi[2] * mi[2][j];
      if (!invmat(mint, r)) continue;
      for (int j = 0; j < 6; j++) out[off + j] = r[j];
      wm |= 1u << s;
    } else {                                          // PMMG_interp3bar_iso
      for (int j = 0; j < sz; j++) {
        double acc = 0.0;
        for (int i = 0; i < 3; i++) acc += phi[i] * A.sol[(int64_t)v[i] * sd.S + off + j];
        out[off + j] = acc;
      }
      wm |= 1u << s;
    }
  }
}

// ---- the walk ----------------------------------------------------------------

// returns 1 found, 2 stuck (needs exhaustive), 3 private-state overflow
template <class St>
__device__ int walk_bdy(const BdyArgs &A, St &s, D3 p, int start, int base, int &k, Bary &b,
                        int &edge, int &vtx, int &step, bool &wedged) {
  wedged = false;
  double cdist = 1.0e10;
  int ctria = 0;
  k = start;
  step = 0;
  edge = UNSET;
  vtx = UNSET;
  bool stuck = false;
  while (step <= A.nt && !stuck) {
    step++;
    TriRec t = A.tris[k];
    if (t.v[0] <= 0) { stuck = true; break; }
    if (in_tria(A, s, k, k, p, b, cdist, ctria)) {
      if (b.val[0] < PMX_EPS) {                        // PMMG_barycoord_isBorder
        if (b.val[1] < PMX_EPS) vtx = b.idx[2];
        else edge = b.idx[0];
      }
      return s.over ? 3 : 1;
    }
    if (s.over) return 3;
    int j;
    for (j = 0; j < 3; j++) {
      int i = b.idx[j];
      int nb = t.nb[0];
      if (i == 1) nb = t.nb[1];
      if (i == 2) nb = t.nb[2];
      if (!nb) continue;
      if (visited(s, nb)) {
        wedged = true;
        int il = in_wedge(A, s, k, i, p, base, b);
        if (s.over) return 3;
        if (il == UNSET) continue;
        if (il == 4) { edge = i; return 1; }
        bool c = in_cone(A, s, k, il, p, base);
        if (s.over) return 3;
        if (c) { vtx = il; return 1; }
        continue;
      }
      k = nb;
      break;
    }
    if (j == 3) stuck = true;
  }
  return 2;
}

__device__ void finish_bdy(const BdyArgs &A, int64_t i, int k, const Bary &b, int edge, int vtx,
                           int status, int step) {
  A.elem[i] = k;
  A.status[i] = status;
  A.steps[i] = step;
  A.edge[i] = edge;
  A.vertex[i] = vtx;
  unsigned wm = 0;
  interp_tria(A, k, b, edge, vtx, A.out + i * A.sd.S, wm);
  A.wmask[i] = (uint8_t)(A.wmask[i] | wm);
}

__device__ int tria_hint(const BdyArgs &A, D3 p);

template <int CAP>
__global__ __launch_bounds__(256) void k_locate_bdy(BdyArgs A) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned s_cnt = 0, s_sum = 0, s_max = 0, s_min = 0xffffffffu;
  if (j < *A.nlist_dev) {
    const int64_t i = A.list[j];
    const D3 p = ld3(A.q, (int)i);
    const int start = A.seq_start ? A.seq_start[i] : tria_hint(A, p);
    const int base = A.seq_base ? A.seq_base[i] : (int)(i + 1);
    A.start[i] = start;
    RegState<CAP> s;
    Bary b;
    int k, edge, vtx, step;
    bool wedged;
    int r = walk_bdy(A, s, p, start, base, k, b, edge, vtx, step, wedged);
    if (A.seq_w) A.seq_w[i] = wedged ? 1 : 0;
    if (r == 1) {
      finish_bdy(A, i, k, b, edge, vtx, 1, step);
      s_cnt = 1; s_sum = (unsigned)step; s_max = (unsigned)step; s_min = (unsigned)step;
    } else if (r == 2) {
      unsigned slot = atomicAdd(A.stuck_count, 1u);
      A.stuck_list[slot] = (int)i;
      A.steps[i] = -step;
    } else {
      unsigned slot = atomicAdd(A.ovf_count, 1u);
      A.ovf_list[slot] = (int)i;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s_cnt += __shfl_xor(s_cnt, o, 64);
    s_sum += __shfl_xor(s_sum, o, 64);
    unsigned a = __shfl_xor(s_max, o, 64), b = __shfl_xor(s_min, o, 64);
    s_max = a > s_max ? a : s_max;
    s_min = b < s_min ? b : s_min;
  }
  if ((threadIdx.x & 63) == 0) A.wstats[j / 64] = make_uint4(s_cnt, s_sum, s_max, s_min);
}

// overflow pass: same walk with large lists in a global workspace
__global__ __launch_bounds__(64) void k_locate_bdy_ovf(BdyArgs A, int *ws, int cap) {
  const unsigned n = *A.ovf_count;
  const unsigned nthr = gridDim.x * blockDim.x;
  const unsigned tid = blockIdx.x * blockDim.x + threadIdx.x;
  for (unsigned j = tid; j < n; j += nthr) {
    int64_t i = A.ovf_list[j];
    const D3 p = ld3(A.q, (int)i);
    GlobState s;
    s.init(ws + (size_t)tid * 3 * cap, cap);
    Bary b;
    int k, edge, vtx, step;
    bool wedged;
    int r = walk_bdy(A, s, p, A.start[i], A.seq_base ? A.seq_base[i] : (int)(i + 1), k, b, edge, vtx, step,
                     wedged);
    if (A.seq_w) A.seq_w[i] = wedged ? 1 : 0;
    if (r == 1) {
      finish_bdy(A, i, k, b, edge, vtx, 1, step);
    } else {
      unsigned slot = atomicAdd(A.stuck_count, 1u);
      A.stuck_list[slot] = (int)i;
      A.steps[i] = -step;
    }
  }
}

// the sequential mode's overflow pass, on hashed lists (workspace:
// ghs_ws_ints() ints per thread, zeroed by the caller)
__global__ __launch_bounds__(64) void k_locate_bdy_ovf_hash(BdyArgs A, int *ws) {
  const unsigned n = *A.ovf_count;
  const unsigned nthr = gridDim.x * blockDim.x;
  const unsigned tid = blockIdx.x * blockDim.x + threadIdx.x;
  int *w = ws + (size_t)tid * (GHS_SLOTS * 6);
  for (unsigned j = tid; j < n; j += nthr) {
    int64_t i = A.ovf_list[j];
    const D3 p = ld3(A.q, (int)i);
    GlobHashState s;
    s.vt = reinterpret_cast<int2 *>(w);
    s.ft = reinterpret_cast<int4 *>(w + 2 * GHS_SLOTS);
    s.mask = GHS_SLOTS - 1;
    s.capv = GHS_SLOTS / 2;
    s.gen = (int)j + 1;
    Bary b;
    int k, edge, vtx, step;
    bool wedged;
    int r = walk_bdy(A, s, p, A.start[i], A.seq_base ? A.seq_base[i] : (int)(i + 1), k, b, edge, vtx, step,
                     wedged);
    if (A.seq_w) A.seq_w[i] = wedged ? 1 : 0;
    if (r == 1) {
      finish_bdy(A, i, k, b, edge, vtx, 1, step);
    } else {
      unsigned slot = atomicAdd(A.stuck_count, 1u);
      A.stuck_list[slot] = (int)i;
      A.steps[i] = -step;
    }
  }
}

// Exhaustive surface search (PMMG_locatePoint_exhaustTria, :477-515):
// one workgroup per stuck point.  First containing tria in index order, else
// the closest tria by centroid distance (lowest index on ties) and the
// reference's re-evaluation with the last tria's geometry.
__global__ __launch_bounds__(256) void k_exh_bdy(BdyArgs A) {
  __shared__ int s_min;
  __shared__ double s_d[256];
  __shared__ int s_k[256];
  const unsigned n = *A.stuck_count;
  for (unsigned j = blockIdx.x; j < n; j += gridDim.x) {
    int64_t i = A.stuck_list[j];
    const D3 p = ld3(A.q, (int)i);
    if (threadIdx.x == 0) s_min = 0x7fffffff;
    __syncthreads();
    RegState<1> dummy;
    for (int64_t t = 1 + threadIdx.x; t <= A.nt; t += blockDim.x) {
      if (A.tris[t].v[0] <= 0) continue;
      Bary b;
      double cd = 1e300;
      int ct = 0;
      dummy.nv = 0;
      dummy.over = false;
      if (in_tria(A, dummy, (int)t, (int)t, p, b, cd, ct)) {
        atomicMin(&s_min, (int)t);
        break;   // later t of this thread are larger
      }
    }
    __syncthreads();
    int kf = s_min;
    if (kf != 0x7fffffff) {
      if (threadIdx.x == 0) {
        Bary b;
        tria_eval(A, kf, kf, p, b);
        finish_bdy(A, i, kf, b, UNSET, UNSET, -1, A.steps[i] - 1);
      }
    } else {
      double best = 1.0e10;
      int bk = 0x7fffffff;
      for (int64_t t = 1 + threadIdx.x; t <= A.nt; t += blockDim.x) {
        if (A.tris[t].v[0] <= 0) continue;
        double d = centroid_dist(A, (int)t, p);
        if (d < best || (d == best && (int)t < bk)) { best = d; bk = (int)t; }
      }
      s_d[threadIdx.x] = best;
      s_k[threadIdx.x] = bk;
      __syncthreads();
      for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
          double d2 = s_d[threadIdx.x + o];
          int k2 = s_k[threadIdx.x + o];
          if (d2 < s_d[threadIdx.x] || (d2 == s_d[threadIdx.x] && k2 < s_k[threadIdx.x])) {
            s_d[threadIdx.x] = d2;
            s_k[threadIdx.x] = k2;
          }
        }
        __syncthreads();
      }
      if (threadIdx.x == 0) {
        int ct = s_k[0];
        Bary b;
        RegState<1> d1;
        double cd = 1e300;
        int cc = 0;
        if (!in_tria(A, d1, (int)A.nt, ct, p, b, cd, cc)) {
          // PMMG_barycoord2d_getClosest (src/barycoord_pmmg.c:324-357)
          TriRec t = A.tris[ct];
          double bd = 0.0;
          int it = 0;
          for (int l = 0; l < 3; l++) {
            D3 c = ld3(A.xyz, t.v[l]);
            double d = norm3(p.x - c.x, p.y - c.y, p.z - c.z);
            if (l == 0 || d < bd) { bd = d; it = l; }
          }
          for (int l = 0; l < 3; l++) { b.idx[l] = l; b.val[l] = (l == it) ? 1.0 : 0.0; }
        }
        finish_bdy(A, i, ct, b, UNSET, UNSET, 0, A.steps[i] - 1);
      }
    }
    __syncthreads();
  }
}

// tria hint grid: cell -> largest tria index whose centroid falls in it
// (deterministic: the surface semantics depend on the start triangle)
__device__ __forceinline__ void tria_hint_one(const TriRec *tris, const double *xyz, int64_t k, int *grid,
                                              const GridDesc &g) {
  TriRec t = tris[k];
  if (t.v[0] <= 0) return;
  D3 a = ld3(xyz, t.v[0]), b = ld3(xyz, t.v[1]), c = ld3(xyz, t.v[2]);
  D3 m{(a.x + b.x + c.x) / 3.0, (a.y + b.y + c.y) / 3.0, (a.z + b.z + c.z) / 3.0};
  int cx = (int)fmin(fmax((m.x - g.lo[0]) * g.inv[0], 0.0), (double)(g.dim[0] - 1));
  int cy = (int)fmin(fmax((m.y - g.lo[1]) * g.inv[1], 0.0), (double)(g.dim[1] - 1));
  int cz = (int)fmin(fmax((m.z - g.lo[2]) * g.inv[2], 0.0), (double)(g.dim[2] - 1));
  atomicMax(&grid[(int64_t)cx + (int64_t)g.dim[0] * ((int64_t)cy + (int64_t)g.dim[1] * cz)], (int)k);
}

// tria hint grid: cell -> largest tria index whose centroid falls in it
// (deterministic: the surface semantics depend on the start triangle)
__global__ __launch_bounds__(256) void k_tria_hint_build(const TriRec *tris, const double *xyz,
                                                         int64_t nt, int *grid, GridDesc g) {
  for (int64_t k = 1 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k <= nt;
       k += (int64_t)gridDim.x * blockDim.x)
    tria_hint_one(tris, xyz, k, grid, g);
}

__device__ int tria_hint(const BdyArgs &A, D3 p) {
  const GridDesc &g = A.g;
  int c[3];
  c[0] = (int)fmin(fmax((p.x - g.lo[0]) * g.inv[0], 0.0), (double)(g.dim[0] - 1));
  c[1] = (int)fmin(fmax((p.y - g.lo[1]) * g.inv[1], 0.0), (double)(g.dim[1] - 1));
  c[2] = (int)fmin(fmax((p.z - g.lo[2]) * g.inv[2], 0.0), (double)(g.dim[2] - 1));
  int k = A.grid[(int64_t)c[0] + (int64_t)g.dim[0] * ((int64_t)c[1] + (int64_t)g.dim[1] * c[2])];
  if (k) return k;
  for (int r = 1; r <= 4; r++)
    for (int dz = -r; dz <= r; dz++)
      for (int dy = -r; dy <= r; dy++)
        for (int dx = -r; dx <= r; dx++) {
          if (max(abs(dx), max(abs(dy), abs(dz))) != r) continue;
          int x = c[0] + dx, y = c[1] + dy, z = c[2] + dz;
          if (x < 0 || y < 0 || z < 0 || x >= g.dim[0] || y >= g.dim[1] || z >= g.dim[2]) continue;
          int kk = A.grid[(int64_t)x + (int64_t)g.dim[0] * ((int64_t)y + (int64_t)g.dim[1] * z)];
          if (kk) return kk;
        }
  return 1;
}

// surface walks are short (1.5 steps on C2): 16 private slots, the rare longer
// walk is redone by k_locate_bdy_ovf with a global workspace (r03: with 8
// slots the overflow pass, one long serial walk per thread, was the C2 surface
// path's tail: surface path 0.287 -> 0.217 ms, step 0.336 -> 0.328 ms with 16;
// C3 within 0.1 %; profiles/r03_c{2,3}_sweep_bdy_cap.log)
#define BDY_CAP 16
#define OVF_CAP 2048
#define OVF_THREADS (64 * 64)

// node -> trias graph (the content of PMMG_precompute_nodeTrias,
// src/locate_pmmg.c:134-195: each boundary vertex's fan of trias in increasing
// tria index, and the fan sizes the point flags start from), rebuilt by every
// step that rebuilds the background's derived data -- the reference builds it
// inside PMMG_interpMetricsAndFields (src/interpmesh_pmmg.c:707).  Sized by
// the surface, not the volume: the 3 nt (vertex, 3 k + l) pairs are radix
// sorted by vertex (stable: fans in tria order), and every pair's slot 3 k + l
// records its vertex's run [lo, hi) -- the surface kernels always reach a
// vertex through a tria that holds it, so no per-vertex offsets over np.
// PMMG_precompute_nodeTrias (src/locate_pmmg.c:134-195): per boundary
// vertex, its incident boundary trias in ascending tria order, i.e. what a
// stable sort of the (vertex, 3 k + l) pairs gives.  Two builds with the same
// output, chosen by size (r03, C2 / C3 steps):
//  * a counting sort over the vertex ids -- count -> exclusive scan over np ->
//    fill at the vertex's offset (slot by atomic, order arbitrary) -> the
//    slot-0 writer sorts its fan (a few entries): its arrays are np-sized;
//  * a 25-bit radix sort of the 3 nt pairs (hipCUB): latency-bound passes
//    whose cost does not grow with np.
// With np > 5 * 3 nt (C3: 16.8 M vertices, 2.3 M pairs) the counting sort's
// memset and scan over np competed with the main stream's derived-data pass
// (step 2.11 -> 2.20 ms); at C2 (1.7 M vertices, 0.5 M pairs) the radix
// sort's passes were the surface stream's critical path (step 0.44 -> 0.36
// ms with the counting sort).  A compacted-id counting sort (bitmap of the
// boundary vertices) lost both: 2.3 M atomicOr on 525 K words serialise.
__global__ __launch_bounds__(256) void k_nt_count(const TriRec *__restrict__ tris, int64_t nt,
                                                  unsigned *__restrict__ cnt) {
  for (int64_t k = 1 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k <= nt;
       k += (int64_t)gridDim.x * blockDim.x) {
    const TriRec t = tris[k];
    if (t.v[0] <= 0) continue;
    for (int l = 0; l < 3; l++) atomicAdd(&cnt[t.v[l]], 1u);
  }
}
__global__ __launch_bounds__(256) void k_nt_fill(const TriRec *__restrict__ tris, int64_t nt,
                                                 const unsigned *__restrict__ off, unsigned *__restrict__ cnt,
                                                 int *__restrict__ list, int2 *__restrict__ range,
                                                 uint8_t *__restrict__ own) {
  for (int64_t k = 1 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k <= nt;
       k += (int64_t)gridDim.x * blockDim.x) {
    const TriRec t = tris[k];
    for (int l = 0; l < 3; l++) {
      if (t.v[0] <= 0) { range[3 * k + l] = make_int2(0, 0); own[3 * k + l] = 0; continue; }
      const int v = t.v[l];
      const unsigned lo = off[v], hi = off[v + 1];
      const unsigned left = atomicSub(&cnt[v], 1u);          // hi - lo, ..., 1
      list[lo + left - 1] = (int)k;
      range[3 * k + l] = make_int2((int)lo, (int)hi);
      own[3 * k + l] = left == 1u ? 1 : 0;                   // exactly one writer per fan
    }
  }
}
__global__ __launch_bounds__(256) void k_nt_sort(int64_t nt, const int2 *__restrict__ range,
                                                 const uint8_t *__restrict__ own, int *__restrict__ list) {
  for (int64_t i = 3 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 3 * (nt + 1);
       i += (int64_t)gridDim.x * blockDim.x) {
    if (!own[i]) continue;
    const int2 r = range[i];
    for (int a = r.x + 1; a < r.y; a++) {                 // insertion sort of the fan
      const int x = list[a];
      int b = a - 1;
      while (b >= r.x && list[b] > x) { list[b + 1] = list[b]; b--; }
      list[b + 1] = x;
    }
  }
}
__global__ __launch_bounds__(256) void k_nt_pairs(const TriRec *__restrict__ tris, int64_t nt,
                                                  unsigned *__restrict__ key, int *__restrict__ val) {
  for (int64_t k = 1 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k <= nt;
       k += (int64_t)gridDim.x * blockDim.x) {
    const TriRec t = tris[k];
    for (int l = 0; l < 3; l++) {
      key[3 * (k - 1) + l] = (unsigned)t.v[l];
      val[3 * (k - 1) + l] = (int)(3 * k + l);
    }
  }
}
__global__ __launch_bounds__(256) void k_nt_runs(const unsigned *__restrict__ key, const int *__restrict__ val,
                                                 int64_t m, int2 *__restrict__ range, int *__restrict__ list) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    list[i] = val[i] / 3;
    if (i > 0 && key[i - 1] == key[i]) continue;           // not the start of a run
    int64_t j = i + 1;
    while (j < m && key[j] == key[i]) j++;
    for (int64_t q = i; q < j; q++) range[val[q]] = make_int2((int)i, (int)j);
  }
}


// The fans by rotation (r05), for a closed manifold surface -- every
// boundary of a ParMmg group's volume mesh, interfaces included: each
// (tria, corner) slot walks its vertex's fan through the tria adjacency
// (Mmg's adjt: edge i opposite vertex i) and writes its tria into the window
// of the fan's owner (its smallest tria) at its rank: the fan's increasing
// tria order of PMMG_precompute_nodeTrias.  One kernel, no atomics, no
// np-sized arrays (the radix sort of C3's 2.3 M (vertex, tria) pairs took
// ~0.26 ms alone on the GPU).  A fan that meets an
// edge without a neighbour (open or non-manifold surface), a neighbour
// without the vertex, or more than FAN_CAP trias counts in *bad: the upload
// runs it once as a check, and a background with any such fan keeps the sort.
#define FAN_CAP 32
// one turn around v from tria k (corner l), the record of each tria in a
// register (one dependent load per step); f(tria, corner of v) per tria, k
// first; false if the fan does not close within FAN_CAP trias
__device__ __forceinline__ int sel3(const int a[3], int i) { return i == 0 ? a[0] : i == 1 ? a[1] : a[2]; }
template <class F>
__device__ __forceinline__ bool fan_turn(const TriRec *__restrict__ tris, int k, int l, const TriRec &t0, F f) {
  const int v = sel3(t0.v, l);
  TriRec tc = t0;
  int cx = (l + 1) % 3, w = sel3(t0.v, (l + 2) % 3);
  f(k, l);
  for (int n = 1;; n++) {
    const int nxt = sel3(tc.nb, cx);               // across the edge {v, w}
    if (nxt == k) return true;                     // closed
    if (nxt <= 0 || n == FAN_CAP) return false;
    tc = tris[nxt];
    const int cv = tc.v[0] == v ? 0 : tc.v[1] == v ? 1 : tc.v[2] == v ? 2 : -1;
    const int cw = tc.v[0] == w ? 0 : tc.v[1] == w ? 1 : tc.v[2] == w ? 2 : -1;
    if (cv < 0 || cw < 0 || cv == cw || tc.v[0] <= 0) return false;
    f(nxt, cv);
    w = sel3(tc.v, 3 - cv - cw);                   // the other edge at v: {v, w'}
    cx = cw;
  }
}
// Every slot walks its fan once: the fan's window is its owner's (the
// smallest tria), and the slot's tria goes to the window at its rank in the
// fan (the number of smaller members) -- the sorted fan without a sort and no
// dependent chain beyond the walk itself.  r05 A/Bs at C3 (rocprof, beside
// the main stream): this 0.12 ms; an owner sorting its fan in global memory
// (a ~35-deep dependent chain) 0.19 ms; only the local minima walking and the
// owner sorting in LDS (2.3 M walks -> 0.8 M, but serial chains in few
// threads) 0.23 ms, step 2.061 vs 2.042 ms (profiles/r05_c3_sweep_fans_owner_lds.log).
// vown (the check only): each fan's owner slot writes its window base at
// its vertex; k_fan_check then finds the vertices whose slots belong to more
// than one fan (two surface sheets touching at a vertex: a group pinched
// there), which the rotation alone cannot see.  No per-vertex counts, no
// np-sized memset: every surface vertex has at least one fan owner, and no
// other vertex is read.  (r06 first version: a per-vertex tria count by
// atomics after an np-sized memset, 0.24 ms at C3 beside the step's prefix.)
__global__ __launch_bounds__(256) void k_fan_rotate(const TriRec *__restrict__ tris, int64_t nt,
                                                    int2 *__restrict__ range, int *__restrict__ list,
                                                    unsigned *__restrict__ bad, int *__restrict__ vown) {
  unsigned nbad = 0;
  for (int64_t i = 3 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 3 * (nt + 1);
       i += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(i / 3), l = (int)(i - 3 * (int64_t)k);
    const TriRec t0 = tris[k];
    if (t0.v[0] <= 0) { range[i] = make_int2(0, 0); continue; }
    int n = 0, rank = 0, own = k, lown = l;
    const bool ok = fan_turn(tris, k, l, t0, [&](int g, int c) {
      n++;
      rank += g < k ? 1 : 0;
      if (g < own) { own = g; lown = c; }
    });
    if (!ok) { nbad++; range[i] = make_int2(0, 0); continue; }
    const int base = (int)((3 * (int64_t)own + lown - 3) * FAN_CAP);
    range[i] = make_int2(base, base + n);
    list[base + rank] = k;
    if (vown && own == k && lown == l) vown[sel3(t0.v, l)] = base;
  }
  for (int o = 32; o > 0; o >>= 1) nbad += __shfl_xor(nbad, o);
  if ((threadIdx.x & 63) == 0 && nbad) atomicAdd(bad, nbad);
}
__global__ __launch_bounds__(256) void k_fan_check(const TriRec *__restrict__ tris, int64_t nt,
                                                   const int2 *__restrict__ range, const int *__restrict__ vown,
                                                   unsigned *__restrict__ bad) {
  unsigned nbad = 0;
  for (int64_t i = 3 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 3 * (nt + 1);
       i += (int64_t)gridDim.x * blockDim.x) {
    const int2 r = range[i];
    if (r.y <= r.x) continue;                      // deleted tria (a failed fan is counted already)
    const int k = (int)(i / 3), l = (int)(i - 3 * (int64_t)k);
    const int v = tris[k].v[l];
    if (vown[v] != r.x) nbad++;
  }
  for (int o = 32; o > 0; o >>= 1) nbad += __shfl_xor(nbad, o);
  if ((threadIdx.x & 63) == 0 && nbad) atomicAdd(bad, nbad);
}

bool pmx_ctx::fan_rotation(hipStream_t s, unsigned *d_bad, bool check) {
  const int64_t m = 3 * nt;
  if (!pmx_dgrow(this, d_ntrange, (size_t)(3 * (nt + 1))) || !pmx_dgrow(this, d_ntlist, (size_t)(m * FAN_CAP)))
    return false;
  if (check && !pmx_dgrow(this, d_ntkey, (size_t)(np + 2))) return false;
  int *vown = check ? reinterpret_cast<int *>(d_ntkey.p) : nullptr;
  const unsigned nb = (unsigned)std::max<int64_t>(1, std::min<int64_t>((m + 255) / 256, 16384));
  hipLaunchKernelGGL(k_fan_rotate, dim3(nb), dim3(256), 0, s, d_tris.p, nt, d_ntrange.p, d_ntlist.p, d_bad,
                     vown);
  if (check)
    hipLaunchKernelGGL(k_fan_check, dim3(nb), dim3(256), 0, s, d_tris.p, nt, (const int2 *)d_ntrange.p,
                       (const int *)vown, d_bad);
  if (hipGetLastError() != hipSuccess) {
    err = "node trias: launch";
    return false;
  }
  return true;
}

// the upload's check: the fans of this background by rotation, their
// failures (open, non-manifold, pinched, over FAN_CAP) into h_nbad[4] (read
// after the upload's final sync).
// PMX_FAN_ROTATION=0 keeps the sort (A/B, tests).
bool pmx_ctx::check_fans(hipStream_t s) {
  fan_rot = false;
  h_nbad[4] = 1u;
  if (nt < 1 || 3 * (nt + 1) * (int64_t)FAN_CAP > (int64_t)INT32_MAX) return true;   // int windows
  const char *e = getenv("PMX_FAN_ROTATION");
  if (e && e[0] == '0') return true;
  // the vertices' fan owners (np-sized, no memset): a vertex where several
  // surface sheets touch has more than one fan
  if (!pmx_dgrow(this, d_wfar, 8)) return false;
  if (!pmx_dgrow(this, d_ntkey, (size_t)(np + 2)) ||
      !pmx_dgrow(this, d_ntrange, (size_t)(3 * (nt + 1))) || !pmx_dgrow(this, d_ntlist, (size_t)(3 * nt * FAN_CAP))) {
    // no room for the check or the fan windows (32 per tria corner): the
    // surface keeps the sort-built fans, the upload goes on
    (void)hipGetLastError();
    err.clear();
    return true;
  }
  if (hipMemsetAsync(d_wfar.p + 3, 0, sizeof(unsigned), s) != hipSuccess) {
    err = "node trias: memset";
    return false;
  }
  if (!fan_rotation(s, d_wfar.p + 3, true)) return false;
  if (hipMemcpyAsync(h_nbad + 4, d_wfar.p + 3, sizeof(unsigned), hipMemcpyDeviceToHost, s) != hipSuccess) {
    err = "node trias: check";
    return false;
  }
  return true;
}

// the counting sort over the vertex ids
static bool node_trias_counting(pmx_ctx *c, hipStream_t s) {
  const int64_t m = 3 * c->nt, np = c->np, nt = c->nt;
  if (!pmx_dgrow(c, c->d_ntkey, (size_t)(2 * (np + 2))) || !pmx_dgrow(c, c->d_ntval, (size_t)(3 * (nt + 1))) ||
      !pmx_dgrow(c, c->d_ntrange, (size_t)(3 * (nt + 1))) || !pmx_dgrow(c, c->d_ntlist, (size_t)m))
    return false;
  unsigned *cnt = c->d_ntkey.p, *off = c->d_ntkey.p + (np + 2);
  uint8_t *own = reinterpret_cast<uint8_t *>(c->d_ntval.p);
  size_t bytes = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, cnt, off, (int)(np + 2), s);
  if (!pmx_dgrow(c, c->d_nttmp, bytes)) return false;
  if (hipMemsetAsync(cnt, 0, (size_t)(np + 2) * sizeof(unsigned), s) != hipSuccess) {
    c->err = "node trias: memset";
    return false;
  }
  const unsigned nb = (unsigned)std::max<int64_t>(1, std::min<int64_t>((nt + 255) / 256, 4096));
  hipLaunchKernelGGL(k_nt_count, dim3(nb), dim3(256), 0, s, c->d_tris.p, nt, cnt);
  if (hipcub::DeviceScan::ExclusiveSum(c->d_nttmp.p, bytes, cnt, off, (int)(np + 2), s) != hipSuccess) {
    c->err = "node trias: scan";
    return false;
  }
  hipLaunchKernelGGL(k_nt_fill, dim3(nb), dim3(256), 0, s, c->d_tris.p, nt, (const unsigned *)off, cnt,
                     c->d_ntlist.p, c->d_ntrange.p, own);
  const unsigned ns = (unsigned)std::max<int64_t>(1, std::min<int64_t>((m + 255) / 256, 4096));
  hipLaunchKernelGGL(k_nt_sort, dim3(ns), dim3(256), 0, s, nt, (const int2 *)c->d_ntrange.p,
                     (const uint8_t *)own, c->d_ntlist.p);
  return true;
}

bool pmx_ctx::build_node_trias(hipStream_t s, int force, bool check) {
  const int64_t m = 3 * nt;
  if (m < 1) return true;
  if (fan_rot && force == 0 && check) {
    // the upload's check again (a FRESH step: what a new background costs):
    // the vertices' fan owners beside the rotation
    return fan_rotation(s, d_wfar.p + 2, true);
  }
  if (fan_rot && force == 0) return fan_rotation(s, d_wfar.p + 2, false);
  if (np <= 5 * m || force == 1) {
    if (!node_trias_counting(this, s)) return false;
    if (hipGetLastError() != hipSuccess) {
      err = "node trias: launch";
      return false;
    }
    return true;
  }
  int bits = 1;
  while (bits < 32 && ((int64_t)1 << bits) <= np) bits++;
  if (!pmx_dgrow(this, d_ntkey, (size_t)(2 * m)) || !pmx_dgrow(this, d_ntval, (size_t)(2 * m)) ||
      !pmx_dgrow(this, d_ntrange, (size_t)(3 * (nt + 1))) || !pmx_dgrow(this, d_ntlist, (size_t)m))
    return false;
  size_t bytes = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const unsigned *)nullptr, (unsigned *)nullptr,
                                     (const int *)nullptr, (int *)nullptr, (int)m, 0, bits, s);
  if (!pmx_dgrow(this, d_nttmp, bytes)) return false;
  const unsigned nb = (unsigned)std::max<int64_t>(1, std::min<int64_t>((nt + 255) / 256, 4096));
  hipLaunchKernelGGL(k_nt_pairs, dim3(nb), dim3(256), 0, s, d_tris.p, nt, d_ntkey.p, d_ntval.p);
  if (hipcub::DeviceRadixSort::SortPairs(d_nttmp.p, bytes, (const unsigned *)d_ntkey.p, d_ntkey.p + m,
                                         (const int *)d_ntval.p, d_ntval.p + m, (int)m, 0, bits, s) !=
      hipSuccess) {
    err = "node trias: sort";
    return false;
  }
  const unsigned nr = (unsigned)std::max<int64_t>(1, std::min<int64_t>((m + 255) / 256, 8192));
  hipLaunchKernelGGL(k_nt_runs, dim3(nr), dim3(256), 0, s, (const unsigned *)d_ntkey.p + m,
                     (const int *)d_ntval.p + m, m, d_ntrange.p, d_ntlist.p);
  if (hipGetLastError() != hipSuccess) {
    err = "node trias: launch";
    return false;
  }
  return true;
}

// the coarser tria hint grid over the background bbox: cells of about 8
// boundary trias.  The grid is 3-D but only its surface cells are used, so it
// is zeroed and rebuilt every step for mostly empty cells; at 2 trias per
// cell it was a 66-MB memset per C3 step beside the volume walk (r02 profile),
// at 8 it is 8.4 MB (surface walks of ~1 more step, latency on the side stream)
bool pmx_ctx::size_tria_grid() {
  double ext[3];
  int64_t cells = 1;
  for (int ax = 0; ax < 3; ax++) ext[ax] = std::max(bbhi[ax] - bblo[ax], 1e-300);
  const double area = 2.0 * (ext[0] * ext[1] + ext[1] * ext[2] + ext[0] * ext[2]);
  const double h = std::sqrt(area / std::max(1.0, (double)nt / 8.0));
  for (int ax = 0; ax < 3; ax++) {
    // 1e-9 slack: libm cbrt/sqrt are not correctly rounded and a cell count
    // of exactly n must not become n+1 (misaligned with a lattice-like mesh)
    int d = (int)std::ceil(ext[ax] / h * (1.0 - 1e-9));
    d = std::max(1, std::min(d, 1024));
    tgd.dim[ax] = d;
    tgd.lo[ax] = bblo[ax];
    tgd.inv[ax] = (double)d / ext[ax];
    cells *= d;
  }
  tcells = nt > 0 ? cells : 0;
  if (tcells && d_tgrid_cap < (size_t)cells) {
    if (d_tgrid) hipFree(d_tgrid);
    d_tgrid = nullptr;
    d_tgrid_cap = 0;
    if (hipMalloc((void **)&d_tgrid, sizeof(int) * (size_t)cells) != hipSuccess) { err = "hipMalloc tgrid"; return false; }
    d_tgrid_cap = (size_t)cells;
  }
  return true;
}

// the surface kernels' arguments for the step's points (tria hint grid tgd)
static BdyArgs bdy_args(pmx_ctx *c, const VolArgs &a) {
  BdyArgs B{};
  B.xyz = c->d_xyz.p; B.tris = c->d_tris.p; B.trn = c->d_trn.p; B.ntrange = c->d_ntrange.p; B.ntlist = c->d_ntlist.p;
  B.sol = c->d_sol.p; B.sd = a.sd; B.q = c->d_qxyz.p; B.kind = c->d_kind.p; B.nq = c->nq; B.nt = c->nt;
  B.hausd = c->hausd; B.grid = c->d_tgrid; B.g = c->tgd;
  B.out = c->d_out.p; B.wmask = c->d_wmask.p; B.elem = c->d_elem.p; B.status = c->d_status.p;
  B.steps = c->d_steps.p; B.start = c->d_start.p; B.edge = c->d_edge.p; B.vertex = c->d_vertex.p;
  B.stuck_list = c->d_blist.p; B.stuck_count = c->d_counts.p + 1;
  B.ovf_list = c->d_olist.p; B.ovf_count = c->d_counts.p + 2;
  B.list = c->d_bdylist.p; B.nlist = c->nq_bdy_ub; B.nlist_dev = c->d_nsel.p + 1; B.wstats = c->d_bstat.p;
  return B;
}

// the walks, their private-list overflow pass and the exhaustive scan
// ovf_threads: the overflow pass's threads, OVF_THREADS unless the caller
// sized the workspace for more (the sequential mode's speculative pass, whose
// walks from the predecessors' trias overflow by the thousand)
static void launch_bdy_walks(const BdyArgs &B, int *ows, int exp, hipStream_t s, int ovf_threads = OVF_THREADS,
                             bool hashed = false) {
  const int64_t nb = (B.nlist + 255) / 256;
  if (exp == 10)                         // A/B: the r01-r03 8-entry private lists
    hipLaunchKernelGGL(k_locate_bdy<BDY_CAP / 2>, dim3((unsigned)nb), dim3(256), 0, s, B);
  else
    hipLaunchKernelGGL(k_locate_bdy<BDY_CAP>, dim3((unsigned)nb), dim3(256), 0, s, B);
  if (hashed)
    hipLaunchKernelGGL(k_locate_bdy_ovf_hash, dim3(ovf_threads / 64), dim3(64), 0, s, B, ows);
  else
    hipLaunchKernelGGL(k_locate_bdy_ovf, dim3(ovf_threads / 64), dim3(64), 0, s, B, ows, OVF_CAP);
  hipLaunchKernelGGL(k_exh_bdy, dim3(256), dim3(256), 0, s, B);
}

bool pmx_ctx::launch_bdy(const VolArgs &a, hipStream_t s) {
  if (nt < 1) { err = "surface points present but the background has no boundary trias"; return false; }
  if (!d_blist.p || d_blist.cap < (size_t)nq) {
    if (d_blist.p) hipFree(d_blist.p);
    if (hipMalloc((void **)&d_blist.p, sizeof(int) * (size_t)std::max<int64_t>(nq, 1)) != hipSuccess) { err = "hipMalloc blist"; return false; }
    d_blist.cap = (size_t)nq;
    if (d_olist.p) hipFree(d_olist.p);
    if (hipMalloc((void **)&d_olist.p, sizeof(int) * (size_t)std::max<int64_t>(nq, 1)) != hipSuccess) { err = "hipMalloc olist"; return false; }
    d_olist.cap = (size_t)nq;
  }
  if (!d_ows.p) {
    if (hipMalloc((void **)&d_ows.p, sizeof(int) * (size_t)OVF_THREADS * 3 * OVF_CAP) != hipSuccess) { err = "hipMalloc ows"; return false; }
    d_ows.cap = (size_t)OVF_THREADS * 3 * OVF_CAP;
  }
  // tria hint grid: sized and allocated with the background
  // (pmx_ctx::size_tria_grid), zeroed and built at the head of the surface
  // path (off the main stream)
  if (hipMemsetAsync(d_tgrid, 0, sizeof(int) * (size_t)tcells, s) != hipSuccess) {
    err = "tria hint grid memset";
    return false;
  }
  {
    int64_t nb = (nt + 255) / 256;
    if (nb > 4096) nb = 4096;
    hipLaunchKernelGGL(k_tria_hint_build, dim3((unsigned)std::max<int64_t>(nb, 1)), dim3(256), 0, s,
                       d_tris.p, d_xyz.p, nt, d_tgrid, tgd);
  }
  launch_bdy_walks(bdy_args(this, a), d_ows.p, a.exp, s);
  return hipGetLastError() == hipSuccess;
}

// ---- PMX_RUN_SEQUENTIAL_SURFACE ---------------------------------------------
//
// The reference runs the surface queries one after the other
// (src/interpmesh_pmmg.c:535-599): in the vertex loop's first-visit order
// through the new tets, each PMMG_locatePointBdy starting from the previous
// one's tria (ifoundTria, :529/:556), with mesh->base counting every locate
// (volume and surface, :521, src/locate_pmmg.c:607/805) and the point flags
// of the shadow tests kept from query to query (PMMG_locatePointInCone marks
// the apex with the base and its scanned neighbours with the apex index, and
// skips a neighbour already marked with it, src/locate_pmmg.c:219,247-249;
// PMMG_locatePointInWedge marks an edge end, :318-323).  A query reads those
// flags only through a wedge test (a walk that meets an already visited
// tria, :640-660).  On the device:
//  1. first-visit keys 4 k + l of every point (k_seq_keys), sorted: the visit
//     order; a scan gives each located point its mesh->base and each
//     surface point its position in the surface sequence;
//  2. a speculative pass of every surface query (the step's walks) starting
//     from the device-semantics result of its predecessor, with its
//     reference base; it records whether the walk ran a wedge test;
//  3. one wavefront replays the sequence (k_seq_resolve): a query whose
//     speculative start is the true one (the previous query's true tria) and
//     whose walk never met the shadow tests keeps its speculative result --
//     it read no carried state; any other is run again by one lane on the
//     reference's own state (tria flags vs base, point flags kept across
//     queries), in order.  A replayed walk that ends stuck hands its point to
//     the exhaustive scan (k_exh_bdy, one launch from the host) and the
//     replay resumes after it.

// the first visit of every new point by the reference's vertex loop: key
// 4 k + l over the valid tets that hold it (atomicMin).  A lane skips the
// vertices its left neighbour (the previous tet) holds: that tet's keys are
// smaller, so the run's leftmost lane gives the minimum (as k_mark_new_tets)
__global__ __launch_bounds__(256) void k_seq_keys(const int4 *__restrict__ tv, int64_t ne,
                                                  unsigned *__restrict__ key) {
  const int64_t st = (int64_t)gridDim.x * blockDim.x;
  const int64_t nit = (ne + st - 1) / st;
  const bool lane0 = (threadIdx.x & 63) == 0;
  for (int64_t it = 0; it < nit; it++) {
    const int64_t k = 1 + it * st + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int4 a = k <= ne ? tv[k] : make_int4(0, 0, 0, 0);
    int4 u;
    u.x = __shfl_up(a.x, 1, 64); u.y = __shfl_up(a.y, 1, 64);
    u.z = __shfl_up(a.z, 1, 64); u.w = __shfl_up(a.w, 1, 64);
    if (lane0 || u.x <= 0) u = make_int4(0, 0, 0, 0);
    if (a.x <= 0) continue;
    const int w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int l = 0; l < 4; l++) {
      const int q = w[l];
      if (q != u.x && q != u.y && q != u.z && q != u.w) atomicMin(key + (q - 1), (unsigned)(4 * k + l));
    }
  }
}
// idx[i] = i; the speculative start (1) and base (0) of every point: a
// surface point the loop never reaches (an orphan, located by a step without
// the marks and reset afterwards) walks from tria 1
__global__ __launch_bounds__(256) void k_seq_iota(int *__restrict__ idx, int *__restrict__ sstart,
                                                  int *__restrict__ sbase, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    idx[i] = (int)i;
    sstart[i] = 1;
    sbase[i] = 0;
  }
}
// per visit-order rank: located (a volume or surface point the loop reaches:
// not NUL, not frozen) in the low word, surface in the high word
__global__ __launch_bounds__(256) void k_seq_flags(const unsigned *__restrict__ skey, const int *__restrict__ sidx,
                                                   const int8_t *__restrict__ kind, int64_t n,
                                                   unsigned long long *__restrict__ val) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const int8_t kd = kind[sidx[r]];
    const bool loc = skey[r] != 0xffffffffu && (kd == KIND_VOL || kd == KIND_BDY);
    val[r] = (unsigned long long)(loc ? 1u : 0u) | ((unsigned long long)(loc && kd == KIND_BDY ? 1u : 0u) << 32);
  }
}
// mesh->base of each located point (1 + the locates before it), the surface
// and the volume sequences; their lengths into nseq[0] / nseq[1]
__global__ __launch_bounds__(256) void k_seq_assign(const int *__restrict__ sidx,
                                                    const unsigned long long *__restrict__ val,
                                                    const unsigned long long *__restrict__ pre, int64_t n,
                                                    int *__restrict__ base, int *__restrict__ seq,
                                                    int *__restrict__ vseq, int *__restrict__ nseq) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long v = val[r], q = pre[r];
    const unsigned located = (unsigned)(q & 0xffffffffull), bdy = (unsigned)(q >> 32);
    if (v & 1ull) {
      const int i = sidx[r];
      base[i] = (int)located + 1;
      if (v >> 32) seq[bdy] = i;
      else vseq[located - bdy] = i;
    }
    if (r == n - 1) {
      const unsigned long long e = q + v;
      nseq[0] = (int)(e >> 32);
      nseq[1] = (int)((e & 0xffffffffull) - (e >> 32));
    }
  }
}
// the speculative start of every surface query: its predecessor's tria from
// the step's (device-semantics) pass; the first query starts at tria 1 (:529)
__global__ __launch_bounds__(256) void k_seq_starts(const int *__restrict__ seq, const int *__restrict__ nseq,
                                                    const int *__restrict__ elem, int *__restrict__ sstart) {
  const int n = *nseq;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x)
    sstart[seq[j]] = j ? elem[seq[j - 1]] : 1;
}

// the replay: one wavefront.  ctl = {next position, start tria of it (-1: the
// tria of the previous query, written by the exhaustive scan), state (0 done,
// 1 stuck: the host scans), stuck point}.  Tria / point flags through
// agent-scope accesses (the lane re-reads what it wrote in earlier queries).
// flags[j] (j < nmax) = surface position j must be looked at by the replay:
// its speculative walk read carried state (a wedge / cone test) or started
// from another tria than its predecessor's speculative result
__global__ __launch_bounds__(256) void k_seq_sflags(const int *__restrict__ seq, const int *__restrict__ nseq_p,
                                                    const int *__restrict__ sstart, const uint8_t *__restrict__ sw,
                                                    const int *__restrict__ elem, int64_t nmax,
                                                    uint8_t *__restrict__ flags) {
  const int n = *nseq_p;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nmax; j += (int64_t)gridDim.x * blockDim.x) {
    bool bad = false;
    if (j < n) {
      const int i = seq[j];
      const int want = j == 0 ? 1 : elem[seq[j - 1]];
      bad = sw[i] || sstart[i] != want;
    }
    flags[j] = bad ? 1 : 0;
  }
}

// the replay, one lane, in visit order over the candidate positions (cand,
// sorted) and the successor of every replayed query; ctl = {next position,
// its start (-1: the tria of the previous point, after a stuck walk the host
// resolved), state (0 done, 1 stuck), the point}.  (r06 first version: the
// wave scanned all positions, 64 at a time.)
__global__ __launch_bounds__(64) void k_seq_resolve(BdyArgs A, const int *__restrict__ seq,
                                                    const int *__restrict__ nseq_p, const int *__restrict__ sstart,
                                                    const uint8_t *__restrict__ sw, const int *__restrict__ sbase,
                                                    int *tf, int *pf, int *ctl, int *stk_list,
                                                    unsigned *stk_count, unsigned *nreplay,
                                                    const int *__restrict__ cand, const int *__restrict__ ncand) {
  if (threadIdx.x != 0) return;
  const int nseq = *nseq_p;
  int j = ctl[0];
  int prev = ctl[1];
  if (j >= nseq) return;
  bool dirty = prev < 0;
  if (prev < 0) prev = A.elem[seq[j - 1]];
  const int nc = *ncand;
  int lo = 0, hi = nc;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cand[mid] < j) lo = mid + 1;
    else hi = mid;
  }
  int pos = lo;
  unsigned replays = 0;
  while (j < nseq) {
    if (!dirty) {
      while (pos < nc && cand[pos] < j) pos++;
      if (pos >= nc) break;
      const int c = cand[pos];
      if (c > j) {
        prev = A.elem[seq[c - 1]];
        j = c;
      }
    }
    const int i = seq[j];
    if (!sw[i] && sstart[i] == prev) {
      prev = A.elem[i];
      dirty = false;
      j++;
      continue;
    }
    const D3 p = ld3(A.q, i);
    SeqState st{tf, pf, sbase[i]};
    Bary b;
    int k, edge, vtx, step;
    bool wedged;
    A.start[i] = prev;
    const int r = walk_bdy(A, st, p, prev, sbase[i], k, b, edge, vtx, step, wedged);
    replays++;
    if (r != 1) {
      A.steps[i] = -step;
      stk_list[0] = i;
      *stk_count = 1u;
      ctl[0] = j;
      ctl[2] = 1;
      ctl[3] = i;
      atomicAdd(nreplay, replays);
      return;
    }
    finish_bdy(A, i, k, b, edge, vtx, 1, step);
    prev = k;
    dirty = true;
    j++;
  }
  ctl[0] = nseq;
  ctl[2] = 0;
  atomicAdd(nreplay, replays);
}

bool pmx_ctx::seq_replay(const VolArgs &a, hipStream_t s, bool surf, bool vol) {
  pmx_ctx *ctx = this;
  auto ck = [&](hipError_t e, const char *what) {
    if (e == hipSuccess) return true;
    ctx->err = std::string("sequential replay: ") + what + ": " + hipGetErrorString(e);
    return false;
  };
  seq_stats[0] = seq_stats[1] = seq_stats[2] = seq_stats[3] = 0;
  if (!surf && !vol) return true;
  if (!have_ntet) {
    err = "PMX_RUN_SEQUENTIAL_*: the first-visit order needs the new tets (points view or pmx_upload_new_tets)";
    return false;
  }
  if (nq < 1) return true;
  if (!ensure_tets(s)) return false;
  const int64_t n = nq;
  size_t sort_b = 0, scan_b = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, sort_b, (const unsigned *)nullptr, (unsigned *)nullptr,
                                     (const int *)nullptr, (int *)nullptr, (int)n, 0, 32, s);
  hipcub::DeviceScan::ExclusiveSum(nullptr, scan_b, (const unsigned long long *)nullptr,
                                   (unsigned long long *)nullptr, (int)n, s);
  if (!pmx_dgrow(this, d_sqkey, (size_t)(2 * n)) || !pmx_dgrow(this, d_sqidx, (size_t)(2 * n)) ||
      !pmx_dgrow(this, d_sqval, (size_t)(2 * n)) || !pmx_dgrow(this, d_sqint, (size_t)(4 * n + 128)) ||
      !pmx_dgrow(this, d_sqw, (size_t)n) || !pmx_dgrow(this, d_sqtmp, std::max(sort_b, scan_b)) ||
      (surf && (!pmx_dgrow(this, d_sqtf, (size_t)(nt + 1)) || !pmx_dgrow(this, d_sqpf, (size_t)(np + 1)))) ||
      (vol && !pmx_dgrow(this, d_sqtv, (size_t)(ne + 1))))
    return false;
  unsigned *key = d_sqkey.p, *key2 = d_sqkey.p + n;
  int *idx = d_sqidx.p, *idx2 = d_sqidx.p + n;
  unsigned long long *val = d_sqval.p, *pre = d_sqval.p + n;
  int *sbase = d_sqint.p, *seq = d_sqint.p + n, *vseq = d_sqint.p + 2 * n, *sstart = d_sqint.p + 3 * n;
  int *ctl = d_sqint.p + 4 * n;                  // [0..3] surface replay, [4..7] volume replay
  int *nseq = ctl + 8;                           // [0] surface, [1] volume
  unsigned *stk_count = (unsigned *)(ctl + 10), *nreplay = (unsigned *)(ctl + 11);   // [11] surface, [12] volume
  int *stk_list = ctl + 13, *vstk_list = ctl + 14;
  unsigned *vcounts = (unsigned *)(ctl + 32);   // the volume fallback's step counters (32 words)
  int *vfound = ctl + 16, *vbestk = ctl + 17;
  const unsigned nbt = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n_ntet + 255) / 256, 8192));
  const unsigned nbp = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192));
  // 1. visit order, bases, sequences
  if (!ck(hipMemsetAsync(key, 0xff, (size_t)n * sizeof(unsigned), s), "memset") ||
      !ck(hipMemsetAsync(ctl, 0, 64 * sizeof(int), s), "memset"))
    return false;
  hipLaunchKernelGGL(k_seq_keys, dim3(nbt), dim3(256), 0, s, (const int4 *)d_ntetv.p, n_ntet, key);
  hipLaunchKernelGGL(k_seq_iota, dim3(nbp), dim3(256), 0, s, idx, sstart, sbase, n);
  if (!ck(hipcub::DeviceRadixSort::SortPairs(d_sqtmp.p, sort_b, (const unsigned *)key, key2, (const int *)idx, idx2,
                                            (int)n, 0, 32, s), "sort"))
    return false;
  hipLaunchKernelGGL(k_seq_flags, dim3(nbp), dim3(256), 0, s, (const unsigned *)key2, (const int *)idx2,
                     (const int8_t *)d_kind.p, n, val);
  if (!ck(hipcub::DeviceScan::ExclusiveSum(d_sqtmp.p, scan_b, (const unsigned long long *)val, pre, (int)n, s),
          "scan"))
    return false;
  hipLaunchKernelGGL(k_seq_assign, dim3(nbp), dim3(256), 0, s, (const int *)idx2, (const unsigned long long *)val,
                     (const unsigned long long *)pre, n, sbase, seq, vseq, nseq);
  if (surf && nq_bdy_ub > 0) {
    // 2. the speculative surface pass
    hipLaunchKernelGGL(k_seq_starts, dim3(nbp), dim3(256), 0, s, (const int *)seq, (const int *)nseq,
                       (const int *)d_elem.p, sstart);
    if (!ck(hipMemsetAsync(d_counts.p + 1, 0, 2 * sizeof(unsigned), s), "memset")) return false;
    BdyArgs B = bdy_args(this, a);
    B.seq_start = sstart;
    B.seq_base = sbase;
    B.seq_w = d_sqw.p;
    // the overflow pass on hashed lists and 2x the threads (C3: 82-96 ms of
    // long speculative walks on linear lists)
    const int seq_ovf = 2 * OVF_THREADS;
    const size_t ws_ints = (size_t)seq_ovf * GHS_SLOTS * 6;
    if (!pmx_dgrow(this, d_ows, ws_ints) ||
        !ck(hipMemsetAsync(d_ows.p, 0, ws_ints * sizeof(int), s), "memset"))
      return false;
    launch_bdy_walks(B, d_ows.p, a.exp, s, seq_ovf, true);
    // 3. the replay, on the reference's state
    if (!ck(hipMemsetAsync(d_sqtf.p, 0, (size_t)(nt + 1) * sizeof(int), s), "memset") ||
        !ck(hipMemsetAsync(d_sqpf.p, 0x80, (size_t)(np + 1) * sizeof(int), s), "memset"))
      return false;
    int hctl[4] = {0, 1, 0, 0};
    if (!ck(hipMemcpyAsync(ctl, hctl, sizeof hctl, hipMemcpyHostToDevice, s), "ctl")) return false;
    // the replay's candidates, in visit order
    {
      size_t sel_b = 0;
      hipcub::CountingInputIterator<int> it(0);
      if (!ck(hipcub::DeviceSelect::Flagged(nullptr, sel_b, it, (const uint8_t *)nullptr, (int *)nullptr,
                                            (int *)nullptr, (int)nq_bdy_ub, s),
              "select") ||
          !pmx_dgrow(this, d_sqflag, (size_t)nq_bdy_ub) || !pmx_dgrow(this, d_sqcand, (size_t)nq_bdy_ub + 1) ||
          !pmx_dgrow(this, d_sqtmp, sel_b))
        return false;
      const unsigned nbs = (unsigned)std::max<int64_t>(1, std::min<int64_t>((nq_bdy_ub + 255) / 256, 8192));
      hipLaunchKernelGGL(k_seq_sflags, dim3(nbs), dim3(256), 0, s, (const int *)seq, (const int *)nseq,
                         (const int *)sstart, (const uint8_t *)d_sqw.p, (const int *)d_elem.p, (int64_t)nq_bdy_ub,
                         d_sqflag.p);
      if (!ck(hipcub::DeviceSelect::Flagged(d_sqtmp.p, sel_b, it, (const uint8_t *)d_sqflag.p, d_sqcand.p + 1,
                                            d_sqcand.p, (int)nq_bdy_ub, s),
              "select"))
        return false;
    }
    BdyArgs X = B;
    X.stuck_list = stk_list;
    X.stuck_count = stk_count;
    for (;;) {
      hipLaunchKernelGGL(k_seq_resolve, dim3(1), dim3(64), 0, s, B, (const int *)seq, (const int *)nseq,
                         (const int *)sstart, (const uint8_t *)d_sqw.p, (const int *)sbase, d_sqtf.p, d_sqpf.p, ctl,
                         stk_list, stk_count, nreplay, (const int *)(d_sqcand.p + 1), (const int *)d_sqcand.p);
      if (!ck(hipMemcpyAsync(hctl, ctl, sizeof hctl, hipMemcpyDeviceToHost, s), "ctl") ||
          !ck(hipStreamSynchronize(s), "sync"))
        return false;
      if (hctl[2] == 0) break;
      // a replayed query ended stuck: the exhaustive scan of that one point
      hipLaunchKernelGGL(k_exh_bdy, dim3(1), dim3(256), 0, s, X);
      hctl[0] += 1;
      hctl[1] = -1;
      hctl[2] = 0;
      if (!ck(hipMemcpyAsync(ctl, hctl, sizeof hctl, hipMemcpyHostToDevice, s), "ctl")) return false;
    }
  }
  if (vol && nq_vol_ub > 0) {
    // the volume: speculative pass from the predecessors' device results, then
    // the replay on the reference's tet flags
    hipLaunchKernelGGL(k_seq_starts, dim3(nbp), dim3(256), 0, s, (const int *)vseq, (const int *)(nseq + 1),
                       (const int *)d_elem.p, sstart);
    SeqVolArgs SV{vseq, nseq + 1, sstart, sbase, d_sqw.p, d_sqtv.p, ctl + 4, vstk_list, nreplay + 1, nullptr, nullptr};
    // the overflow pass's hash tables: generation 0 = empty (positions start at 1)
    if (!pmx_dgrow(this, d_sqows, seqv_ovf_ws_ints()) ||
        !ck(hipMemsetAsync(d_sqows.p, 0, seqv_ovf_ws_ints() * sizeof(int), s), "memset"))
      return false;
    launch_seqv_spec(a, SV, nq_vol_ub, d_sqows.p, s);
    // the replay's candidates: positions whose speculative start may be wrong,
    // in visit order (DeviceSelect keeps the order)
    {
      size_t sel_b = 0;
      hipcub::CountingInputIterator<int> it(0);
      if (!ck(hipcub::DeviceSelect::Flagged(nullptr, sel_b, it, (const uint8_t *)nullptr, (int *)nullptr,
                                            (int *)nullptr, (int)nq_vol_ub, s),
              "select") ||
          !pmx_dgrow(this, d_sqflag, (size_t)nq_vol_ub) || !pmx_dgrow(this, d_sqcand, (size_t)nq_vol_ub + 1) ||
          !pmx_dgrow(this, d_sqtmp, sel_b))
        return false;
      launch_seqv_flags(a, SV, nq_vol_ub, d_sqflag.p, s);
      if (!ck(hipcub::DeviceSelect::Flagged(d_sqtmp.p, sel_b, it, (const uint8_t *)d_sqflag.p, d_sqcand.p + 1,
                                            d_sqcand.p, (int)nq_vol_ub, s),
              "select"))
        return false;
      SV.ncand = d_sqcand.p;
      SV.cand = d_sqcand.p + 1;
    }
    if (!ck(hipMemsetAsync(d_sqtv.p, 0, (size_t)(ne + 1) * sizeof(int), s), "memset")) return false;
    int hctl[4] = {0, 1, 0, 0};
    if (!ck(hipMemcpyAsync(ctl + 4, hctl, sizeof hctl, hipMemcpyHostToDevice, s), "ctl")) return false;
    for (;;) {
      launch_seqv_resolve(a, SV, s);
      if (!ck(hipMemcpyAsync(hctl, ctl + 4, sizeof hctl, hipMemcpyDeviceToHost, s), "ctl") ||
          !ck(hipStreamSynchronize(s), "sync"))
        return false;
      if (hctl[2] == 0) break;
      // a replayed walk got stuck: k_fallback on that one point (its own
      // counters: stuck count 1, no ties, barrier and error words zero)
      const unsigned one = 1u;
      const int imax = 0x7fffffff;
      const unsigned long long umax = ~0ull;
      if (!ck(hipMemsetAsync(vcounts, 0, 32 * sizeof(unsigned), s), "memset") ||
          !ck(hipMemcpyAsync(vcounts, &one, sizeof one, hipMemcpyHostToDevice, s), "fallback") ||
          !ck(hipMemcpyAsync(vfound, &imax, sizeof imax, hipMemcpyHostToDevice, s), "fallback") ||
          !ck(hipMemcpyAsync(vbestk, &imax, sizeof imax, hipMemcpyHostToDevice, s), "fallback") ||
          !ck(hipMemcpyAsync(val, &umax, sizeof umax, hipMemcpyHostToDevice, s), "fallback"))
        return false;
      VolArgs V = a;
      V.stuck_list = vstk_list;
      V.stuck_count = vcounts;
      V.tie_count = vcounts + 3;
      V.found = vfound;
      V.bestk = vbestk;
      V.best = val;
      ExhArgs E{};
      E.xyz = d_xyz.p; E.tets = d_tets.p; E.ne = ne; E.q = d_qxyz.p;
      E.list = vstk_list; E.count = vcounts; E.found = vfound; E.best = val; E.bestk = vbestk;
      E.spin_limit = 1L << 26;
      launch_exhaustive(E, V, fallback_blocks, s);
      if (!ck(hipStreamSynchronize(s), "sync")) return false;
      unsigned derr = 0;
      if (!ck(hipMemcpy(&derr, vcounts + PMX_CNT_ERR, sizeof derr, hipMemcpyDeviceToHost), "fallback")) return false;
      if (derr) { err = "sequential replay: the one-point fallback's grid barrier timed out"; return false; }
      hctl[0] += 1;
      hctl[1] = -1;
      hctl[2] = 0;
      if (!ck(hipMemcpyAsync(ctl + 4, hctl, sizeof hctl, hipMemcpyHostToDevice, s), "ctl")) return false;
    }
  }
  unsigned hr[2];
  int hn[2];
  if (!ck(hipMemcpyAsync(hr, nreplay, sizeof hr, hipMemcpyDeviceToHost, s), "stats") ||
      !ck(hipMemcpyAsync(hn, nseq, sizeof hn, hipMemcpyDeviceToHost, s), "stats") ||
      !ck(hipStreamSynchronize(s), "sync"))
    return false;
  seq_stats[0] = surf ? hr[0] : 0;
  seq_stats[1] = surf ? (unsigned)hn[0] : 0;
  seq_stats[2] = vol ? hr[1] : 0;
  seq_stats[3] = vol ? (unsigned)hn[1] : 0;
  return hipGetLastError() == hipSuccess;
}
