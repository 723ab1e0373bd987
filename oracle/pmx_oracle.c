/*
 * pmx_oracle.c -- CPU restatement of the reference transfer path.
 *
 * TEST INFRASTRUCTURE ONLY (see pmx_oracle.h).  PARITY UNPINNED.
 *
 * Every routine cites the reference file:line whose semantics it restates.
 * It is written for sequential clarity, not speed, with the exact floating
 * point operation order of the reference (build: -O2 -ffp-contract=off).
 */
#include "pmx_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define ORC_EPS   1.e-6     /* MMG5_EPS   */
#define ORC_EPSD2 1.e-200   /* MMG5_EPSD2 */
#define ORC_UNSET (-1)      /* PMMG_UNSET, src/libparmmgtypes.h:236 */
#define TAG_REQ   4         /* MG_REQ */
#define TAG_BDY   16        /* MG_BDY */
#define TAG_NUL   16384     /* MG_NUL */

/* MMG5_idir: vertices of face f (opposite vertex f), outward orientation */
static const int FV[4][3] = {{1,2,3},{0,3,2},{0,1,3},{0,2,1}};
static const int NXT2[6] = {1,2,0,1,2,0};   /* MMG5_inxt2 */
static const int PRV2[3] = {2,0,1};         /* MMG5_iprv2 */

typedef struct { int idx; double val; } bcoord;

struct orc_ctx {
  int64_t np, ne, nt;
  const double *xyz;
  const int *tet, *adja, *tria, *adjt;
  double hausd;
  /* reference precomputes */
  double *fn;      /* 12*(ne+1): PMMG_precompute_faceAreas  src/locate_pmmg.c:101-122 */
  double *tvol;    /* ne+1: pt->qual = MMG5_orvol                   :110       */
  double *trn;     /* 3*(nt+1): PMMG_precompute_triaNormals          :68-90   */
  double *trarea;  /* nt+1: ptr->qual = |n|                          :84      */
  int    *ntria;   /* nodeTrias CSR (reference layout)               :134-195 */
  int    *ptmp;    /* point tmp = offset into ntria                          */
  /* mutable flags */
  int    *pflag, *pflag0, *tflag, *trflag;
  int     base;
  /* fresh (device-semantics) mode: the point flags a query wrote, restored
   * from pflag0 before the next query (O(touched) instead of O(np)) */
  int    *touched;
  int64_t ntouched, captouched;
  int     track;
};

static void set_pflag(orc_ctx *o, int i, int v) {
  if (o->track) {
    if (o->ntouched == o->captouched) {
      int64_t c = o->captouched ? 2 * o->captouched : 64;
      int *t = (int *)realloc(o->touched, sizeof(int) * (size_t)c);
      if (!t) abort();
      o->touched = t;
      o->captouched = c;
    }
    o->touched[o->ntouched++] = i;
  }
  o->pflag[i] = v;
}

static const double *PT(const orc_ctx *o, int i) { return &o->xyz[3*(int64_t)i]; }

/* ---- restated Mmg helpers (unpinned) --------------------------------- */

/* MMG5_nonUnitNorPts: (p2-p1) x (p3-p1) */
static void nonunit_normal(const double *a, const double *b, const double *c, double *n) {
  double abx = b[0]-a[0], aby = b[1]-a[1], abz = b[2]-a[2];
  double acx = c[0]-a[0], acy = c[1]-a[1], acz = c[2]-a[2];
  n[0] = aby*acz - abz*acy;
  n[1] = abz*acx - abx*acz;
  n[2] = abx*acy - aby*acx;
}

/* MMG5_orvol -> MMG5_det4pt(c0,c1,c2,c3) -> MMG5_det3pt1vec(c0,c1,c2,v) with
 * v = c3 - c0: the 3x3 determinant [c1-c0 | c2-c0 | v] expanded along v,
 *   v0*(m10*m21 - m20*m11) - v1*(m00*m21 - m20*m01) + v2*(m00*m11 - m10*m01)
 * (public Mmg source, src/common/tools.c; evaluated left to right) */
static double orvol(const double *c0, const double *c1, const double *c2, const double *c3) {
  double m00 = c1[0]-c0[0], m01 = c2[0]-c0[0];
  double m10 = c1[1]-c0[1], m11 = c2[1]-c0[1];
  double m20 = c1[2]-c0[2], m21 = c2[2]-c0[2];
  double v0 = c3[0]-c0[0], v1 = c3[1]-c0[1], v2 = c3[2]-c0[2];
  return v0*(m10*m21 - m20*m11) - v1*(m00*m21 - m20*m01) + v2*(m00*m11 - m10*m01);
}

int orc_invmat(const double *m, double *mi) {
  double aa, bb, cc, det, vmin, vmax, t;
  int k;
  vmax = fabs(m[1]);
  t = fabs(m[2]); if (t > vmax) vmax = t;
  t = fabs(m[4]); if (t > vmax) vmax = t;
  if (vmax < ORC_EPS) {                 /* diagonal */
    mi[0] = 1./m[0];
    mi[3] = 1./m[3];
    mi[5] = 1./m[5];
    mi[1] = mi[2] = mi[4] = 0.0;
    return 1;
  }
  vmin = vmax = fabs(m[0]);
  for (k = 1; k < 6; k++) {
    t = fabs(m[k]);
    if (t < vmin) vmin = t;
    else if (t > vmax) vmax = t;
  }
  if (vmax == 0.0) return 0;
  aa = m[3]*m[5] - m[4]*m[4];
  bb = m[4]*m[2] - m[1]*m[5];
  cc = m[1]*m[4] - m[2]*m[3];
  det = m[0]*aa + m[1]*bb + m[2]*cc;
  if (fabs(det) < ORC_EPSD2) return 0;
  det = 1.0 / det;
  mi[0] = aa*det;
  mi[1] = bb*det;
  mi[2] = cc*det;
  mi[3] = (m[0]*m[5] - m[2]*m[2])*det;
  mi[4] = (m[1]*m[2] - m[0]*m[4])*det;
  mi[5] = (m[0]*m[3] - m[1]*m[1])*det;
  return 1;
}

void orc_constant_size(int64_t npts, int size, double hsiz, double *m) {
  int64_t i;
  for (i = 0; i < npts; i++) {
    if (size == 1) m[i] = hsiz;
    else {
      double v = 1.0 / (hsiz*hsiz);
      m[6*i+0] = v; m[6*i+1] = 0.0; m[6*i+2] = 0.0;
      m[6*i+3] = v; m[6*i+4] = 0.0; m[6*i+5] = v;
    }
  }
}

/* ---- context ---------------------------------------------------------- */

orc_ctx *orc_create(int64_t np, int64_t ne, int64_t nt, const double *xyz,
                    const int *tet, const int *adja, const int *tria,
                    const int *adjt, double hausd) {
  orc_ctx *o = (orc_ctx *)calloc(1, sizeof(orc_ctx));
  int64_t k, ip, nbp;
  int *cnt;
  if (!o) return NULL;
  o->np = np; o->ne = ne; o->nt = nt;
  o->xyz = xyz; o->tet = tet; o->adja = adja; o->tria = tria; o->adjt = adjt;
  o->hausd = hausd;
  o->fn     = (double *)calloc((size_t)(12*(ne+1)), sizeof(double));
  o->tvol   = (double *)calloc((size_t)(ne+1), sizeof(double));
  o->trn    = (double *)calloc((size_t)(3*(nt+1)), sizeof(double));
  o->trarea = (double *)calloc((size_t)(nt+1), sizeof(double));
  o->ptmp   = (int *)calloc((size_t)(np+1), sizeof(int));
  o->pflag  = (int *)calloc((size_t)(np+1), sizeof(int));
  o->pflag0 = (int *)calloc((size_t)(np+1), sizeof(int));
  o->tflag  = (int *)calloc((size_t)(ne+1), sizeof(int));
  o->trflag = (int *)calloc((size_t)(nt+1), sizeof(int));
  cnt       = (int *)calloc((size_t)(np+1), sizeof(int));

  /* face normals and signed volumes: src/locate_pmmg.c:101-122 */
  for (k = 1; k <= ne; k++) {
    const int *v = &tet[4*k];
    int f;
    o->tvol[k] = orvol(PT(o,v[0]), PT(o,v[1]), PT(o,v[2]), PT(o,v[3]));
    for (f = 0; f < 4; f++)
      nonunit_normal(PT(o,v[FV[f][0]]), PT(o,v[FV[f][1]]), PT(o,v[FV[f][2]]), &o->fn[12*k+3*f]);
  }
  /* unit tria normals and areas: src/locate_pmmg.c:68-90 */
  for (k = 1; k <= nt; k++) {
    double *n = &o->trn[3*k], r;
    nonunit_normal(PT(o,tria[3*k]), PT(o,tria[3*k+1]), PT(o,tria[3*k+2]), n);
    o->trarea[k] = sqrt(n[0]*n[0] + n[1]*n[1] + n[2]*n[2]);
    r = 1.0 / o->trarea[k];
    n[0] *= r; n[1] *= r; n[2] *= r;
  }
  /* node -> trias graph, reference layout: src/locate_pmmg.c:134-195 */
  nbp = 0;
  for (k = 1; k <= nt; k++) {
    int l;
    for (l = 0; l < 3; l++) {
      int q = tria[3*k+l];
      if (!cnt[q]) nbp++;
      cnt[q]++;
    }
  }
  o->ntria = (int *)calloc((size_t)(nbp + 3*nt + 1), sizeof(int));
  o->ptmp[1] = 0;
  for (ip = 2; ip <= np; ip++)
    o->ptmp[ip] = cnt[ip-1] ? o->ptmp[ip-1] + cnt[ip-1] + 1 : o->ptmp[ip-1];
  for (ip = 1; ip <= np; ip++) {
    if (!cnt[ip]) continue;
    o->ntria[o->ptmp[ip]] = cnt[ip];
    o->pflag0[ip] = 0;
  }
  {
    int *fill = (int *)calloc((size_t)(np+1), sizeof(int));
    for (k = 1; k <= nt; k++) {
      int l;
      for (l = 0; l < 3; l++) {
        int q = tria[3*k+l];
        o->ntria[o->ptmp[q] + 1 + fill[q]++] = (int)k;
      }
    }
    /* the reference leaves point->flag = number of incident trias */
    for (ip = 1; ip <= np; ip++) o->pflag0[ip] = fill[ip];
    free(fill);
  }
  free(cnt);
  orc_reset(o);
  return o;
}

void orc_destroy(orc_ctx *o) {
  if (!o) return;
  free(o->fn); free(o->tvol); free(o->trn); free(o->trarea); free(o->ntria);
  free(o->ptmp); free(o->pflag); free(o->pflag0); free(o->tflag); free(o->trflag);
  free(o->touched);
  free(o);
}

void orc_reset(orc_ctx *o) {
  memcpy(o->pflag, o->pflag0, sizeof(int) * (size_t)(o->np+1));
  memset(o->tflag, 0, sizeof(int) * (size_t)(o->ne+1));
  memset(o->trflag, 0, sizeof(int) * (size_t)(o->nt+1));
  o->base = 0;
}

/* ---- barycentric coordinates ------------------------------------------ */

/* stable ascending order (glibc qsort = merge sort for these sizes):
 * src/barycoord_pmmg.c:89-100,300-310 */
static void bsort(bcoord *b, int n) {
  int i, j;
  for (i = 1; i < n; i++) {
    bcoord x = b[i];
    for (j = i; j > 0 && b[j-1].val > x.val; j--) b[j] = b[j-1];
    b[j] = x;
  }
}

/* src/barycoord_pmmg.c:238-257 then :300-310; inside test :102-107 */
static int tet_eval(const orc_ctx *o, int k, const double *p, bcoord *b) {
  const int *v = &o->tet[4*(int64_t)k];
  double vol = o->tvol[k];
  int f;
  for (f = 0; f < 4; f++) {
    const double *n = &o->fn[12*(int64_t)k + 3*f];
    const double *c = PT(o, v[FV[f][0]]);
    b[f].val = -((p[0]-c[0])*n[0] + (p[1]-c[1])*n[1] + (p[2]-c[2])*n[2]) / vol;
    b[f].idx = f;
  }
  bsort(b, 4);
  return b[0].val > -ORC_EPS;
}

/* src/locate_pmmg.c:441-461 */
static int in_tetra(orc_ctx *o, int k, const double *p, bcoord *b, double *cdist, int *ctet) {
  int found;
  double d;
  o->tflag[k] = o->base;
  found = tet_eval(o, k, p, b);
  d = fabs(b[0].val) * o->tvol[k];
  if (d < *cdist) { *cdist = d; *ctet = k; }
  return found;
}

static double dist3(const double *p, const double *c) {
  double d0 = p[0]-c[0], d1 = p[1]-c[1], d2 = p[2]-c[2];
  return sqrt(d0*d0 + d1*d1 + d2*d2);
}

/* src/barycoord_pmmg.c:371-404 */
static void tet_closest_vertex(const orc_ctx *o, int k, const double *p, bcoord *b) {
  const int *v = &o->tet[4*(int64_t)k];
  double best = dist3(p, PT(o, v[0])), d;
  int i, it = 0;
  for (i = 1; i < 4; i++) {
    d = dist3(p, PT(o, v[i]));
    if (d < best) { best = d; it = i; }
  }
  for (i = 0; i < 4; i++) { b[i].val = 0.0; b[i].idx = i; }
  b[it].val = 1.0;
}

int orc_tet_contains(orc_ctx *o, int k, const double *p, double *lmin) {
  bcoord b[4];
  int r = tet_eval(o, k, p, b);
  if (lmin) *lmin = b[0].val;
  return r;
}

/* ---- volume location: src/locate_pmmg.c:786-883 + :737-770 ------------ */

static int locate_vol(orc_ctx *o, const double *p, int *elem, bcoord *b, int *steps) {
  const int64_t ne = o->ne;
  int cur, ctet = 0, stuck = 0;
  int64_t step = 0, s;
  double cdist = 1.0e10;

  cur = *elem ? *elem : 1;
  o->base++;
  while (step <= ne && !stuck) {
    int i;
    const int *adj;
    step++;
    if (o->tet[4*(int64_t)cur] <= 0) continue;           /* MG_EOK */
    if (in_tetra(o, cur, p, b, &cdist, &ctet)) break;
    /* first unvisited interior neighbour in ascending lambda order :819-833 */
    adj = &o->adja[4*(int64_t)(cur-1)+1];
    for (i = 0; i < 4; i++) {
      int nb = adj[b[i].idx] / 4;
      if (!nb) continue;
      if (o->tflag[nb] == o->base) continue;
      cur = nb;
      break;
    }
    if (i == 4) stuck = 1;
  }
  s = stuck ? -step : step;
  *elem = cur;

  if (step > ne) {
    *elem = ctet;
    tet_closest_vertex(o, ctet, p, b);
    *steps = (int)s;
    return 0;
  }
  if (!stuck) { *steps = (int)s; return 1; }

  /* exhaustive scan in index order, skipping visited tets :743-759 */
  {
    int64_t k;
    for (k = 1; k <= ne; k++) {
      s--;
      if (o->tet[4*k] <= 0) continue;
      if (o->tflag[k] == o->base) continue;
      if (in_tetra(o, (int)k, p, b, &cdist, &ctet)) break;
    }
    *steps = (int)s;
    if (k <= ne) { *elem = (int)k; return -1; }
    *elem = ctet;
    tet_closest_vertex(o, ctet, p, b);
    return 0;
  }
}

int orc_locate_vol(orc_ctx *o, const double *p, int *elem, double *phi, int *steps) {
  bcoord b[4];
  int i, r = locate_vol(o, p, elem, b, steps);
  for (i = 0; i < 4; i++) phi[b[i].idx] = b[i].val;     /* PMMG_barycoord_get */
  return r;
}

/* ---- surface location: src/locate_pmmg.c:209-723 ------------------------ */

/* PMMG_quickarea, src/barycoord_pmmg.c:41-59 */
static double qarea(const double *a, const double *b, const double *c, const double *n) {
  double abx = b[0]-a[0], aby = b[1]-a[1], abz = b[2]-a[2];
  double acx = c[0]-a[0], acy = c[1]-a[1], acz = c[2]-a[2];
  double a0 = aby*acz - abz*acy, a1 = abz*acx - abx*acz, a2 = abx*acy - aby*acx;
  return a0*n[0] + a1*n[1] + a2*n[2];
}

/* src/barycoord_pmmg.c:191-223 (geometry of tria g, normal of tria kn),
 * sorted :274-284 */
static int tria_eval(const orc_ctx *o, int g, int kn, const double *p, bcoord *b) {
  const int *v = &o->tria[3*(int64_t)g];
  const double *n = &o->trn[3*(int64_t)kn];
  const double *c = PT(o, v[0]);
  double h = 0.0, q[3], area = o->trarea[g];
  int d, e;
  for (d = 0; d < 3; d++) h += (p[d]-c[d])*n[d];
  for (d = 0; d < 3; d++) q[d] = p[d] - h*n[d];
  for (e = 0; e < 3; e++) {
    b[e].val = qarea(q, PT(o, v[NXT2[e]]), PT(o, v[NXT2[e+1]]), n) / area;
    b[e].idx = e;
  }
  b[3].val = h; b[3].idx = 3;
  bsort(b, 3);
  return b[0].val > -ORC_EPS;
}

/* PMMG_locatePointInTria (src/locate_pmmg.c:385-423) on the geometry of
 * tria g with the normal of tria kn (they differ only in the quirk of
 * PMMG_locatePoint_exhaustTria :504-509). */
static int in_tria_g(orc_ctx *o, int g, int kn, const double *p, bcoord *b,
                     double *cdist, int *ctria) {
  const int *v = &o->tria[3*(int64_t)g];
  const double *n = &o->trn[3*(int64_t)kn];
  double dd[3], nrm, h;
  int found, j, d;
  const double *c0;
  o->trflag[g] = o->base;
  found = tria_eval(o, g, kn, p, b);
  for (d = 0; d < 3; d++) dd[d] = p[d];
  for (j = 0; j < 3; j++) {
    const double *c = PT(o, v[j]);
    for (d = 0; d < 3; d++) dd[d] -= c[d]/3.0;
  }
  nrm = 0;
  for (d = 0; d < 3; d++) nrm += dd[d]*dd[d];
  nrm = sqrt(nrm);
  if (nrm < *cdist) { *cdist = nrm; *ctria = kn; }
  /* PMMG_locateChkDistTria :347-366 */
  c0 = PT(o, v[0]);
  h = 0.0;
  for (d = 0; d < 3; d++) h += (p[d]-c0[d])*n[d];
  if (fabs(h) > o->hausd) return 0;
  return found;
}
static int in_tria(orc_ctx *o, int k, const double *p, bcoord *b, double *cdist, int *ctria) {
  return in_tria_g(o, k, k, p, b, cdist, ctria);
}

int orc_tria_contains(orc_ctx *o, int k, const double *p) {
  bcoord b[4];
  double cd = 1e300;
  int ct = 0, saved = o->trflag[k];
  int r = in_tria(o, k, p, b, &cd, &ct);
  o->trflag[k] = saved;
  return r;
}

/* src/barycoord_pmmg.c:324-357 */
static void tria_closest_vertex(const orc_ctx *o, int k, const double *p, bcoord *b) {
  const int *v = &o->tria[3*(int64_t)k];
  double best = dist3(p, PT(o, v[0])), d;
  int i, it = 0;
  for (i = 1; i < 3; i++) {
    d = dist3(p, PT(o, v[i]));
    if (d < best) { best = d; it = i; }
  }
  for (i = 0; i < 3; i++) { b[i].val = 0.0; b[i].idx = i; }
  b[it].val = 1.0;
}

/* PMMG_locatePointInCone, src/locate_pmmg.c:209-270 */
static int in_cone(orc_ctx *o, int k, int iloc, const double *p) {
  int ip = o->tria[3*(int64_t)k+iloc];
  const double *c0 = PT(o, ip);
  const int *fan = &o->ntria[o->ptmp[ip]];
  double pv[3], dist = 0.0;
  int t, j, d;
  set_pflag(o, ip, o->base);
  for (d = 0; d < 3; d++) pv[d] = p[d] - c0[d];
  for (d = 0; d < 3; d++) dist += pv[d]*pv[d];
  dist = sqrt(dist);
  for (t = 0; t < fan[0]; t++) {
    const int *v = &o->tria[3*(int64_t)fan[t+1]];
    for (j = 0; j < 3; j++) {
      int jp = v[j];
      double a[3], alpha;
      if (jp == ip) continue;
      if (o->pflag[jp] == ip) continue;
      set_pflag(o, jp, ip);
      for (d = 0; d < 3; d++) a[d] = PT(o, jp)[d] - c0[d];
      if (dist > o->hausd) return 0;
      alpha = 0.0;
      for (d = 0; d < 3; d++) alpha += a[d]*pv[d];
      if (alpha > 0.0) return 0;
    }
  }
  return 1;
}

/* PMMG_locatePointInWedge, src/locate_pmmg.c:286-334 */
static int in_wedge(orc_ctx *o, int k, int l, const double *p, bcoord *b) {
  int i0 = NXT2[l], i1 = PRV2[l];
  int q0 = o->tria[3*(int64_t)k+i0], q1 = o->tria[3*(int64_t)k+i1];
  const double *c0 = PT(o, q0), *c1 = PT(o, q1);
  double pv[3], a[3], n2 = 0.0, alpha = 0.0, dist = 0.0;
  int d;
  for (d = 0; d < 3; d++) pv[d] = p[d] - c0[d];
  for (d = 0; d < 3; d++) a[d] = c1[d] - c0[d];
  for (d = 0; d < 3; d++) n2 += a[d]*a[d];
  for (d = 0; d < 3; d++) alpha += a[d]*pv[d];
  for (d = 0; d < 3; d++) pv[d] -= (alpha/n2)*a[d];
  for (d = 0; d < 3; d++) dist += pv[d]*pv[d];
  dist = sqrt(dist);
  if (dist > o->hausd) return ORC_UNSET;
  if (alpha < 0.0) { set_pflag(o, q1, o->base); return i0; }
  if (alpha > n2)  { set_pflag(o, q0, o->base); return i1; }
  for (d = 0; d < 3; d++) b[d].idx = d;
  b[l].val  = 0.0;
  b[i0].val = 1.0 - alpha/n2;
  b[i1].val = alpha/n2;
  return 4;
}

/* src/locate_pmmg.c:587-723 (foundConvex :531-569 has no observable effect:
 * it compares an uninitialised h with itself and never updates) */
static int locate_bdy(orc_ctx *o, const double *p, int *elem, int *edge, int *vtx,
                      bcoord *b, int *steps) {
  const int64_t nt = o->nt;
  int cur, ctria = 0, stuck = 0;
  int64_t step = 0, s;
  double cdist = 1.0e10;

  cur = *elem ? *elem : 1;
  o->base++;
  *edge = ORC_UNSET; *vtx = ORC_UNSET;
  while (step <= nt && !stuck) {
    const int *adj;
    int j;
    step++;
    if (o->tria[3*(int64_t)cur] <= 0) continue;
    if (in_tria(o, cur, p, b, &cdist, &ctria)) {
      /* PMMG_barycoord_isBorder, src/barycoord_pmmg.c:109-120 */
      if (b[0].val < ORC_EPS) {
        if (b[1].val < ORC_EPS) *vtx = b[2].idx;
        else *edge = b[0].idx;
      }
      break;
    }
    adj = &o->adjt[3*(int64_t)(cur-1)+1];
    for (j = 0; j < 3; j++) {
      int i = b[j].idx, nb = adj[i] / 3, il;
      if (!nb) continue;
      if (o->trflag[nb] == o->base) {
        il = in_wedge(o, cur, i, p, b);
        if (il == ORC_UNSET) continue;
        if (il == 4) { *edge = i; *steps = (int)step; *elem = cur; return 1; }
        if (in_cone(o, cur, il, p)) { *vtx = il; *steps = (int)step; *elem = cur; return 1; }
        continue;
      }
      cur = nb;
      break;
    }
    if (j == 3) stuck = 1;
  }
  s = stuck ? -step : step;
  if (step > nt) {
    *elem = ctria;
    tria_closest_vertex(o, ctria, p, b);
    *steps = (int)s;
    return 0;
  }
  *elem = cur;
  if (!stuck) { *steps = (int)s; return 1; }

  /* PMMG_locatePoint_exhaustTria, src/locate_pmmg.c:477-515 */
  {
    int64_t k;
    int last = 0;
    for (k = 1; k <= nt; k++) {
      s--;
      last = (int)k;
      if (o->tria[3*k] <= 0) continue;
      if (o->trflag[k] == o->base) continue;
      if (in_tria(o, (int)k, p, b, &cdist, &ctria)) break;
    }
    *steps = (int)s;
    if (k <= nt) { *elem = (int)k; return -1; }
    *elem = ctria;
    /* the reference re-evaluates with the geometry of the last scanned tria
     * and the normal of the closest one (:504-509) */
    if (!in_tria_g(o, last, ctria, p, b, &cdist, &ctria))
      tria_closest_vertex(o, *elem, p, b);
    return 0;
  }
}

int orc_locate_bdy(orc_ctx *o, const double *p, int *elem, int *edge, int *vertex,
                   int *bary_idx, double *bary_val, int *steps) {
  bcoord b[4];
  int i, r;
  for (i = 0; i < 4; i++) { b[i].idx = i; b[i].val = 0.0; }
  r = locate_bdy(o, p, elem, edge, vertex, b, steps);
  for (i = 0; i < 4; i++) { bary_idx[i] = b[i].idx; bary_val[i] = b[i].val; }
  return r;
}

/* ---- interpolation: src/interpmesh_pmmg.c:50-296 ----------------------- */

/* phi[i] = value of the barycoord entry whose idx is i: PMMG_barycoord_get */
static void unpermute(const bcoord *b, int ndim, double *phi) {
  int i;
  for (i = 0; i < ndim; i++) phi[b[i].idx] = b[i].val;
}

/* PMMG_interp{4,3}bar_iso: zero, then accumulate vertex by vertex */
static void interp_iso(int nv, const int *v, const double *phi, int size,
                       const double *old, double *out) {
  int i, j;
  for (j = 0; j < size; j++) out[j] = 0.0;
  for (i = 0; i < nv; i++)
    for (j = 0; j < size; j++) out[j] += phi[i] * old[(int64_t)v[i]*size + j];
}

/* PMMG_interp{4,3}bar_ani: inverse, interpolate, invert */
static int interp_ani(int nv, const int *v, const double *phi, const double *old, double *out) {
  double mi[4][6], mint[6];
  int i, s;
  for (i = 0; i < nv; i++)
    if (!orc_invmat(&old[6*(int64_t)v[i]], mi[i])) return 0;
  for (s = 0; s < 6; s++) {
    if (nv == 4) mint[s] = phi[0]*mi[0][s] + phi[1]*mi[1][s] + phi[2]*mi[2][s] + phi[3]*mi[3][s];
    else         mint[s] = phi[0]*mi[0][s] + phi[1]*mi[1][s] + phi[2]*mi[2][s];
  }
  return orc_invmat(mint, out);
}

/* PMMG_interp2bar_{iso,ani} :50-110 (edge l of tria v) */
static int interp_edge(const int *v, int l, const double *phi, int size,
                       const double *old, double *out) {
  int i0 = NXT2[l], i1 = PRV2[l];
  if (size == 1) {
    out[0] = phi[i0]*old[v[i0]] + phi[i1]*old[v[i1]];
    return 1;
  } else {
    double mi[2][6], mint[6];
    int s;
    if (!orc_invmat(&old[6*(int64_t)v[i0]], mi[0])) return 0;
    if (!orc_invmat(&old[6*(int64_t)v[i1]], mi[1])) return 0;
    for (s = 0; s < 6; s++) mint[s] = phi[i0]*mi[0][s] + phi[i1]*mi[1][s];
    return orc_invmat(mint, out);
  }
}

int orc_interp_points(orc_ctx *o, int64_t npts, const double *pxyz, const int *ptag,
                      const int64_t *order, int nsol, const int *size,
                      const double *const *oldsol, double *const *newsol, int imet,
                      const int *start_vol, const int *start_bdy, int fresh,
                      int *elem, int *status, int *steps, int *edge, int *vertex) {
  int64_t it;
  int cur_vol = 1, cur_bdy = 1;      /* src/interpmesh_pmmg.c:529 */
  orc_reset(o);
  o->ntouched = 0;
  o->track = fresh != 0;
  for (it = 0; it < npts; it++) {
    int64_t ip = order ? order[it] : it;
    const double *p = &pxyz[3*ip];
    int tag = ptag ? ptag[ip] : 0;
    int s, r, st = 0, e = ORC_UNSET, vx = ORC_UNSET, k;
    bcoord b[4];
    double phi[4];
    if (tag >= TAG_NUL) continue;                 /* MG_VOK */
    if (tag & TAG_REQ) continue;                  /* copied, :546-549 */
    if (fresh) {
      /* device semantics: flags as left by nodeTrias, base = ordinal+1 */
      int64_t q;
      for (q = 0; q < o->ntouched; q++) o->pflag[o->touched[q]] = o->pflag0[o->touched[q]];
      o->ntouched = 0;
      o->base = (int)ip;
    }
    if (tag & TAG_BDY) {
      const int *v;
      int i;
      k = start_bdy ? start_bdy[ip] : cur_bdy;
      if (k < 1 || k > o->nt) k = 1;
      for (i = 0; i < 4; i++) { b[i].idx = i; b[i].val = 0.0; }
      r = locate_bdy(o, p, &k, &e, &vx, b, &st);
      cur_bdy = k;
      v = &o->tria[3*(int64_t)k];
      unpermute(b, 3, phi);
      for (s = 0; s < nsol; s++) {
        double *out = &newsol[s][(int64_t)size[s]*ip];
        if (s == imet) {
          if (vx != ORC_UNSET) {                  /* PMMG_copyMetrics :285-296 */
            int j;
            for (j = 0; j < size[s]; j++) out[j] = oldsol[s][(int64_t)size[s]*v[vx] + j];
          } else if (e != ORC_UNSET) {
            interp_edge(v, e, phi, size[s], oldsol[s], out);
          } else if (size[s] == 6) {
            interp_ani(3, v, phi, oldsol[s], out);
          } else {
            interp_iso(3, v, phi, size[s], oldsol[s], out);
          }
        } else if (size[s] == 6) {
          interp_ani(3, v, phi, oldsol[s], out);
        } else {
          interp_iso(3, v, phi, size[s], oldsol[s], out);
        }
      }
    } else {
      const int *v;
      k = start_vol ? start_vol[ip] : cur_vol;
      if (k < 1 || k > o->ne) k = 1;              /* invalid start: first tet */
      r = locate_vol(o, p, &k, b, &st);
      cur_vol = k;
      v = &o->tet[4*(int64_t)k];
      unpermute(b, 4, phi);
      for (s = 0; s < nsol; s++) {
        double *out = &newsol[s][(int64_t)size[s]*ip];
        if (size[s] == 6) interp_ani(4, v, phi, oldsol[s], out);
        else interp_iso(4, v, phi, size[s], oldsol[s], out);
      }
    }
    if (elem) elem[ip] = k;
    if (status) status[ip] = r;
    if (steps) steps[ip] = st;
    if (edge) edge[ip] = e;
    if (vertex) vertex[ip] = vx;
  }
  o->track = 0;
  return 1;
}
