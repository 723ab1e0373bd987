// pmx_device.h -- device-side data layout and geometry for the gfx950 kernels.
//
// HBM layout (all 1-based like Mmg, slot 0 unused):
//   double  xyz[3*(np+1)] 24 B  x, y, z            uploaded as is (no padding)
//   TetRec  tets[ne+1]    32 B  {v[4], nb[4]}      nb[f] = adja/4 (0 = boundary face)
//   double  sol[(np+1)*S]        all background solutions interleaved per vertex
//   TriRec  tris[nt+1]    32 B  {v[3], -, nb[3], -} nb[e] = adjt/3
//   Pt4     trn[nt+1]     32 B  unit normal + |n| (PMMG_precompute_triaNormals)
// New points: Pt4 q[npts] (0-based list), int8 kind[npts].
//
// Floating point: every expression below follows the operation order of the
// reference / restated Mmg helper it cites, and the library is built with
// -ffp-contract=off so that no a*b+c is fused: results are bit-identical to
// the x86-64 oracle (oracle/pmx_oracle.c) on the same inputs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "pmx_wrec.h"      // TetRec and the walk's compact copy WRec

#define PMX_EPS   1.e-6     // MMG5_EPS
#define PMX_EPSD2 1.e-200   // MMG5_EPSD2

struct __align__(32) Pt4 { double x, y, z, w; };
struct __align__(32) TriRec { int v[3]; int pad0; int nb[3]; int pad1; };

struct D3 { double x, y, z; };

// tets[k] through its compact record (WRec, pmx_wrec.h)
__device__ __forceinline__ TetRec wrec_load(const WRec *__restrict__ wr, const TetRec *__restrict__ tets,
                                            int k) {
  const WRec r = wr[k];
  return wrec_decode(r, tets, k);
}

// KIND_SKIP: MG_REQ (copied by PMMG_copyMetricsAndFields_point); KIND_NUL:
// !MG_VOK; KIND_ORPH: in no valid new tet (never visited by the reference)
enum : int8_t { KIND_VOL = 0, KIND_BDY = 1, KIND_SKIP = 2, KIND_NUL = 3, KIND_ORPH = 4 };

struct SolDesc {
  int nsol;
  int S;              // total doubles per vertex
  int imet;           // index of the metric, -1 none
  int metric_const;   // 1: metric set by constant size (not interpolated)
  int size[8];
  int off[8];
};

__device__ __forceinline__ D3 ld3(const Pt4 *p, int i) {
  Pt4 t = p[i];
  return D3{t.x, t.y, t.z};
}
// old-mesh vertices: dense x, y, z (24 B, 5.3 vertices per 128-B line)
__device__ __forceinline__ D3 ld3(const double *__restrict__ xyz, int i) {
  const double *r = xyz + 3 * (int64_t)i;
  return D3{r[0], r[1], r[2]};
}

// MMG5_nonUnitNorPts (restated): (b-a) x (c-a)
__device__ __forceinline__ D3 nonunit_normal(D3 a, D3 b, D3 c) {
  double abx = b.x - a.x, aby = b.y - a.y, abz = b.z - a.z;
  double acx = c.x - a.x, acy = c.y - a.y, acz = c.z - a.z;
  D3 n;
  n.x = aby * acz - abz * acy;
  n.y = abz * acx - abx * acz;
  n.z = abx * acy - aby * acx;
  return n;
}

// MMG5_orvol -> MMG5_det4pt(c0,c1,c2,c3) -> MMG5_det3pt1vec(c0,c1,c2,v),
// v = c3 - c0: [c1-c0 | c2-c0 | v] expanded along v, left to right (restated
// from the public Mmg source; the same expression as oracle/pmx_oracle.c)
__device__ __forceinline__ double orvol(D3 c0, D3 c1, D3 c2, D3 c3) {
  double m00 = c1.x - c0.x, m01 = c2.x - c0.x;
  double m10 = c1.y - c0.y, m11 = c2.y - c0.y;
  double m20 = c1.z - c0.z, m21 = c2.z - c0.z;
  double v0 = c3.x - c0.x, v1 = c3.y - c0.y, v2 = c3.z - c0.z;
  return v0 * (m10 * m21 - m20 * m11) - v1 * (m00 * m21 - m20 * m01) + v2 * (m00 * m11 - m10 * m01);
}

// lambda_f = -((p - c_f) . n_f) / vol, c_f = first vertex of face f in
// MMG5_idir order (reference src/barycoord_pmmg.c:238-257 with the normals
// of src/locate_pmmg.c:101-122 recomputed in registers instead of stored).
__device__ __forceinline__ void tet_lambda(const D3 P[4], D3 p, double lam[4], double *volp) {
  double vol = orvol(P[0], P[1], P[2], P[3]);
  D3 n0 = nonunit_normal(P[1], P[2], P[3]);
  D3 n1 = nonunit_normal(P[0], P[3], P[2]);
  D3 n2 = nonunit_normal(P[0], P[1], P[3]);
  D3 n3 = nonunit_normal(P[0], P[2], P[1]);
  lam[0] = -((p.x - P[1].x) * n0.x + (p.y - P[1].y) * n0.y + (p.z - P[1].z) * n0.z) / vol;
  lam[1] = -((p.x - P[0].x) * n1.x + (p.y - P[0].y) * n1.y + (p.z - P[0].z) * n1.z) / vol;
  lam[2] = -((p.x - P[0].x) * n2.x + (p.y - P[0].y) * n2.y + (p.z - P[0].z) * n2.z) / vol;
  lam[3] = -((p.x - P[0].x) * n3.x + (p.y - P[0].y) * n3.y + (p.z - P[0].z) * n3.z) / vol;
  *volp = vol;
}

// Stable ascending order of 4 (value, index) pairs: adjacent compare-exchange
// (bubble) network == glibc's stable qsort of src/barycoord_pmmg.c:306.
__device__ __forceinline__ void cswap(double &a, double &b, int &ia, int &ib) {
  bool s = a > b;
  double ta = s ? b : a, tb = s ? a : b;
  int tia = s ? ib : ia, tib = s ? ia : ib;
  a = ta; b = tb; ia = tia; ib = tib;
}
__device__ __forceinline__ void sort4(double v[4], int id[4]) {
  cswap(v[0], v[1], id[0], id[1]);
  cswap(v[1], v[2], id[1], id[2]);
  cswap(v[2], v[3], id[2], id[3]);
  cswap(v[0], v[1], id[0], id[1]);
  cswap(v[1], v[2], id[1], id[2]);
  cswap(v[0], v[1], id[0], id[1]);
}
__device__ __forceinline__ void sort3(double v[3], int id[3]) {
  cswap(v[0], v[1], id[0], id[1]);
  cswap(v[1], v[2], id[1], id[2]);
  cswap(v[0], v[1], id[0], id[1]);
}

__device__ __forceinline__ int sel4(const int a[4], int i) {
  int r = a[0];
  r = (i == 1) ? a[1] : r;
  r = (i == 2) ? a[2] : r;
  r = (i == 3) ? a[3] : r;
  return r;
}

// MMG5_invmat (restated from Mmg @889d408; unpinned)
// (both branches produce six scalars and mi is written once: keeps it in VGPRs)
__device__ __forceinline__ bool invmat(const double m[6], double mi[6]) {
  double vmax = fabs(m[1]), t;
  t = fabs(m[2]); if (t > vmax) vmax = t;
  t = fabs(m[4]); if (t > vmax) vmax = t;
  double r0, r1, r2, r3, r4, r5;
  bool ok;
  if (vmax < PMX_EPS) {                       // diagonal metric
    r0 = 1. / m[0];
    r3 = 1. / m[3];
    r5 = 1. / m[5];
    r1 = r2 = r4 = 0.0;
    ok = true;
  } else {
    double vmin = fabs(m[0]);
    vmax = vmin;
#pragma unroll
    for (int k = 1; k < 6; k++) {
      t = fabs(m[k]);
      if (t < vmin) vmin = t;
      else if (t > vmax) vmax = t;
    }
    double aa = m[3] * m[5] - m[4] * m[4];
    double bb = m[4] * m[2] - m[1] * m[5];
    double cc = m[1] * m[4] - m[2] * m[3];
    double det = m[0] * aa + m[1] * bb + m[2] * cc;
    ok = !(vmax == 0.0) && !(fabs(det) < PMX_EPSD2);
    det = 1.0 / det;
    r0 = aa * det;
    r1 = bb * det;
    r2 = cc * det;
    r3 = (m[0] * m[5] - m[2] * m[2]) * det;
    r4 = (m[1] * m[2] - m[0] * m[4]) * det;
    r5 = (m[0] * m[3] - m[1] * m[1]) * det;
  }
  if (ok) {
    mi[0] = r0; mi[1] = r1; mi[2] = r2; mi[3] = r3; mi[4] = r4; mi[5] = r5;
  }
  return ok;
}

// ---- interpolation (shared by the walk and tet-centric kernels) ----------

// PMMG_interp4bar_iso / PMMG_interp3bar_iso (src/interpmesh_pmmg.c:125-149,
// :206-230): out = 0, then += phi_i * old_i in vertex order.
// PMMG_interp4bar_ani / 3bar_ani (:166-190, :247-270): invert, interpolate,
// invert; a failed inversion leaves the output untouched (bit s of wmask).
template <int NV>
__device__ __forceinline__ unsigned interp_bar(const double *__restrict__ sol, const SolDesc &sd,
                                               const int *v, const double *phi,
                                               double *__restrict__ out) {
  unsigned wm = 0;
  for (int s = 0; s < sd.nsol; ++s) {
    if (s == sd.imet && sd.metric_const) continue;
    const int sz = sd.size[s], off = sd.off[s];
    if (sz == 6) {
      // mint_j = ((phi0*mi0_j + phi1*mi1_j) + phi2*mi2_j) + phi3*mi3_j, the
      // reference's left-to-right sum, accumulated one vertex at a time so
      // that only one inverse is live (no scratch)
      double mint[6], r[6];
      bool ok = true;
      // unrolled: the 4 vertex rows are loaded concurrently (a rolled loop
      // measured 6% slower on C2 -- latency, not registers, bounds the walk)
#pragma unroll
      for (int i = 0; i < NV; i++) {
        const int vi = v[i];
        const double ph = phi[i];
        const double *m = sol + (int64_t)vi * sd.S + off;
        double mm[6] = {m[0], m[1], m[2], m[3], m[4], m[5]};
        double mi[6];
        ok = ok && invmat(mm, mi);
#pragma unroll
        for (int j = 0; j < 6; j++) mint[j] = (i == 0) ? ph * mi[j] : mint[j] + ph * mi[j];
      }
      if (!ok) continue;
      if (!invmat(mint, r)) continue;
#pragma unroll
      for (int j = 0; j < 6; j++) out[off + j] = r[j];
      wm |= 1u << s;
    } else {
      for (int j = 0; j < sz; j++) {
        double acc = 0.0;
#pragma unroll
        for (int i = 0; i < NV; i++) acc += phi[i] * sol[(int64_t)v[i] * sd.S + off + j];
        out[off + j] = acc;
      }
      wm |= 1u << s;
    }
  }
  return wm;
}

__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nb) {
  // blocks b and b+8 share an XCD (round-robin dispatch): give each XCD a
  // contiguous range of the Morton-ordered queries so its L2 sees neighbours.
  int64_t xcd = b & 7, r = b >> 3, q = nb >> 3, rem = nb & 7;
  return (xcd < rem) ? xcd * (q + 1) + r : rem * (q + 1) + (xcd - rem) * q + r;
}

