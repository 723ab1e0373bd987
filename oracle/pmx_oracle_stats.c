/*
 * pmx_oracle_stats.c -- CPU restatement of the quality / edge-length
 * statistics (TEST INFRASTRUCTURE ONLY, PARITY UNPINNED: the per-element
 * arithmetic is Mmg's and Mmg is absent from the container).
 *
 *   orc_tetra_qual  MMG3D_tetraQual -> MMG5_caltet_iso / MMG5_caltet33_ani
 *                   (called from reference src/quality_pmmg.c:720-733)
 *   orc_tetra_qual_rid  the same with metRidTyp: 1 with a size-6 metric is
 *                   MMG5_orcal -> MMG5_caltet_ani, whose mean metric
 *                   (MMG5_moymet) leaves out the non-singular ridge points
 *                   (their stored metric is Mmg's two-sided ridge metric)
 *   orc_qualhisto   MMG3D_computeInqua statistics as aggregated by
 *                   PMMG_qualhisto (src/quality_pmmg.c:156-261)
 *   orc_prilen      MMG3D_computePrilen (centralized branch of PMMG_prilen,
 *                   src/quality_pmmg.c:646-651; same loop as the distributed
 *                   one at :506-564): hash every tet edge, then pop them in
 *                   (k ascending, ia ascending) order.
 *   orc_prilen_full the same with metRidTyp and Mmg's surface data (xTetra
 *                   edge tags, point / xPoint normals): the length kernels the
 *                   reference selects at :462-466 and :527-531 --
 *                   MMG5_lenSurfEdg33_ani / MMG5_lenSurfEdg_iso for the
 *                   parallel edges, MMG5_lenedg33_ani / MMG5_lenedg(_ani|_iso)
 *                   for the tet edges -- restated from the public Mmg sources
 *                   (MMG5_lenEdg, MMG5_buildridmet, MMG5_lenedgspl_ani with
 *                   MMG5_moymet, MMG5_lenedgCoor_ani/_iso; unpinned).
 */
#include "pmx_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define ALPHAD 20.7846097   /* MMG3D_ALPHAD */
#define EPS    1.e-6
#define EPSD2  1.e-200
#define TAG_GEO 2
#define TAG_REQ 4
#define TAG_NOM 8
#define TAG_CRN 32
#define TAG_REF 1
#define TAG_BDY 16

static const int IARE[6][2] = {{0,1},{0,2},{0,3},{1,2},{1,3},{2,3}};

static double caltet_iso(const double *a, const double *b, const double *c, const double *d) {
  double abx = b[0]-a[0], aby = b[1]-a[1], abz = b[2]-a[2];
  double acx = c[0]-a[0], acy = c[1]-a[1], acz = c[2]-a[2];
  double adx = d[0]-a[0], ady = d[1]-a[1], adz = d[2]-a[2];
  double v1 = acy*adz - acz*ady, v2 = acz*adx - acx*adz, v3 = acx*ady - acy*adx;
  double vol = abx*v1 + aby*v2 + abz*v3, rap;
  double bcx, bcy, bcz, bdx, bdy, bdz, cdx, cdy, cdz;
  if (vol <= 0.) return 0.0;
  bcx = c[0]-b[0]; bcy = c[1]-b[1]; bcz = c[2]-b[2];
  bdx = d[0]-b[0]; bdy = d[1]-b[1]; bdz = d[2]-b[2];
  cdx = d[0]-c[0]; cdy = d[1]-c[1]; cdz = d[2]-c[2];
  rap  = abx*abx + aby*aby + abz*abz;
  rap += acx*acx + acy*acy + acz*acz;
  rap += adx*adx + ady*ady + adz*adz;
  rap += bcx*bcx + bcy*bcy + bcz*bcz;
  rap += bdx*bdx + bdy*bdy + bdz*bdz;
  rap += cdx*cdx + cdy*cdy + cdz*cdz;
  if (rap < EPSD2) return 0.0;
  rap = rap * sqrt(rap);
  return vol / rap;
}

static double mlen2(const double *m, double x, double y, double z) {
  return m[0]*x*x + m[3]*y*y + m[5]*z*z + 2.0*(m[1]*x*y + m[2]*x*z + m[4]*y*z);
}

/* MMG5_caltet33_ani / MMG5_caltet_ani past their mean metric mm */
static double caltet_ani_mm(const double *a, const double *b, const double *c, const double *d,
                            const double *mm) {
  double det, rap, num, vol;
  double abx = b[0]-a[0], aby = b[1]-a[1], abz = b[2]-a[2];
  double acx = c[0]-a[0], acy = c[1]-a[1], acz = c[2]-a[2];
  double adx = d[0]-a[0], ady = d[1]-a[1], adz = d[2]-a[2];
  double bcx, bcy, bcz, bdx, bdy, bdz, cdx, cdy, cdz;
  vol = abx*(acy*adz - acz*ady) + aby*(acz*adx - acx*adz) + abz*(acx*ady - acy*adx);
  if (vol <= 0.) return 0.0;
  det = mm[0]*(mm[3]*mm[5] - mm[4]*mm[4]) - mm[1]*(mm[1]*mm[5] - mm[2]*mm[4])
      + mm[2]*(mm[1]*mm[4] - mm[2]*mm[3]);
  if (det < EPSD2) return 0.0;
  det = sqrt(det) * vol;
  bcx = c[0]-b[0]; bcy = c[1]-b[1]; bcz = c[2]-b[2];
  bdx = d[0]-b[0]; bdy = d[1]-b[1]; bdz = d[2]-b[2];
  cdx = d[0]-c[0]; cdy = d[1]-c[1]; cdz = d[2]-c[2];
  rap  = mlen2(mm, abx, aby, abz);
  rap += mlen2(mm, acx, acy, acz);
  rap += mlen2(mm, adx, ady, adz);
  rap += mlen2(mm, bcx, bcy, bcz);
  rap += mlen2(mm, bdx, bdy, bdz);
  rap += mlen2(mm, cdx, cdy, cdz);
  if (rap < EPSD2) return 0.0;
  num = sqrt(rap) * rap;
  return det / num;
}

/* MMG5_caltet33_ani: the plain mean of the 4 vertex metrics */
static double caltet_ani(const double *a, const double *b, const double *c, const double *d,
                         const double *ma, const double *mb, const double *mc, const double *md) {
  double mm[6];
  int i;
  for (i = 0; i < 6; i++) mm[i] = 0.25 * (ma[i] + mb[i] + mc[i] + md[i]);
  return caltet_ani_mm(a, b, c, d, mm);
}

static int ridge_pt(unsigned tg);

/* MMG5_caltet_ani (metRidTyp = 1): MMG5_moymet's mean over the vertices that
 * are not non-singular ridge points (MG_SIN || MG_NOM || !MG_GEO), summed in
 * vertex order and scaled by 1/n; no such vertex: quality 0 (moymet fails) */
static double caltet_ani_rid(const double *xyz, const double *met, const int *v, const uint16_t *tag) {
  double mm[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0}, dd;
  int i, j, n = 0;
  for (j = 0; j < 4; j++) {
    if (tag && ridge_pt(tag[v[j]])) continue;
    n++;
    for (i = 0; i < 6; i++) mm[i] += met[6*(int64_t)v[j] + i];
  }
  if (!n) return 0.0;
  dd = 1. / n;
  for (i = 0; i < 6; i++) mm[i] = mm[i] * dd;
  return caltet_ani_mm(&xyz[3*v[0]], &xyz[3*v[1]], &xyz[3*v[2]], &xyz[3*v[3]], mm);
}

void orc_tetra_qual_rid(int64_t ne, const double *xyz, const int *tet, const double *met, int msize,
                        const uint16_t *tag, int metRidTyp, double *qual) {
  int64_t k;
  qual[0] = 0.0;
  for (k = 1; k <= ne; k++) {
    const int *v = &tet[4*k];
    if (v[0] <= 0) { qual[k] = 0.0; continue; }
    if (met && msize == 6 && metRidTyp)
      qual[k] = caltet_ani_rid(xyz, met, v, tag);
    else if (met && msize == 6)
      qual[k] = caltet_ani(&xyz[3*v[0]], &xyz[3*v[1]], &xyz[3*v[2]], &xyz[3*v[3]],
                           &met[6*v[0]], &met[6*v[1]], &met[6*v[2]], &met[6*v[3]]);
    else
      qual[k] = caltet_iso(&xyz[3*v[0]], &xyz[3*v[1]], &xyz[3*v[2]], &xyz[3*v[3]]);
  }
}

void orc_tetra_qual(int64_t ne, const double *xyz, const int *tet, const double *met, int msize,
                    double *qual) {
  int64_t k;
  qual[0] = 0.0;
  for (k = 1; k <= ne; k++) {
    const int *v = &tet[4*k];
    if (v[0] <= 0) { qual[k] = 0.0; continue; }
    if (met && msize == 6)
      qual[k] = caltet_ani(&xyz[3*v[0]], &xyz[3*v[1]], &xyz[3*v[2]], &xyz[3*v[3]],
                           &met[6*v[0]], &met[6*v[1]], &met[6*v[2]], &met[6*v[3]]);
    else
      qual[k] = caltet_iso(&xyz[3*v[0]], &xyz[3*v[1]], &xyz[3*v[2]], &xyz[3*v[3]]);
  }
}

/* a non-singular ridge point: !(MG_SIN || MG_NOM) && MG_GEO (MG_SIN = CRN|REQ) */
static int ridge_pt(unsigned tg) {
  int sin = (tg & TAG_CRN) || (tg & TAG_REQ);
  return !(sin || (TAG_NOM & tg)) && (tg & TAG_GEO);
}
static int tet_4ridge(const int *v, const uint16_t *tag) {
  int i;
  if (!tag) return 0;
  for (i = 0; i < 4; i++)
    if (!ridge_pt(tag[v[i]])) return 0;
  return 1;
}

void orc_qualhisto_tags(int64_t ne, const int *tet, const double *qual, const uint16_t *tag,
                        orc_qualstats *st) {
  int64_t k;
  orc_qualhisto(ne, tet, qual, st);
  for (k = 1; k <= ne; k++)
    if (tet[4*k] > 0 && tet_4ridge(&tet[4*k], tag)) st->nrid++;
}

void orc_qualhisto(int64_t ne, const int *tet, const double *qual, orc_qualstats *st) {
  int64_t k;
  int i;
  memset(st, 0, sizeof *st);
  st->min = 2.0;
  st->max = 0.0;
  for (k = 1; k <= ne; k++) {
    double rap;
    int ir;
    if (tet[4*k] <= 0) continue;
    st->ne++;
    rap = ALPHAD * qual[k];
    if (rap < st->min) { st->min = rap; st->iel = k; }
    if (rap > 0.5) st->med++;
    if (rap > 0.12) st->good++;
    st->avg += rap;
    if (rap > st->max) st->max = rap;
    ir = (int)(5.0 * rap);
    if (ir > 4) ir = 4;
    st->his[ir] += 1;
  }
  (void)i;
}

/* ---- edge lengths -------------------------------------------------------- */

static uint64_t hkey(int a, int b) { return ((uint64_t)(uint32_t)a << 32) | (uint32_t)b; }

static double len_iso(const double *xyz, const double *met, int p1, int p2) {
  const double *c1 = &xyz[3*p1], *c2 = &xyz[3*p2];
  double h1 = met[p1], h2 = met[p2], l, r;
  l = (c2[0]-c1[0])*(c2[0]-c1[0]) + (c2[1]-c1[1])*(c2[1]-c1[1]) + (c2[2]-c1[2])*(c2[2]-c1[2]);
  l = sqrt(l);
  r = h2 / h1 - 1.0;
  return (fabs(r) < EPS) ? (l / h1) : (l / (h2 - h1) * log1p(r));
}

static double len_ani(const double *xyz, const double *met, int p1, int p2) {
  const double *c1 = &xyz[3*p1], *c2 = &xyz[3*p2];
  double ux = c2[0]-c1[0], uy = c2[1]-c1[1], uz = c2[2]-c1[2];
  double dd1 = mlen2(&met[6*p1], ux, uy, uz), dd2 = mlen2(&met[6*p2], ux, uy, uz);
  if (dd1 <= 0.0) dd1 = 0.0;
  if (dd2 <= 0.0) dd2 = 0.0;
  return (sqrt(dd1) + sqrt(dd2) + 4.0*sqrt(0.5*(dd1 + dd2))) / 6.0;
}

/* ---- Mmg's surface-aware lengths in a tensor metric (restated, unpinned) ---- */

/* MG_SIN(tag) || (tag & MG_NOM): a singular or non-manifold point, whose
 * stored metric is a plain tensor */
static int sin_or_nom(unsigned tg) { return (tg & TAG_CRN) || (tg & TAG_REQ) || (tg & TAG_NOM); }

typedef struct {
  const double *xyz, *met;           /* met: 6 per point (size-6 metric)  */
  const uint16_t *tag;               /* point tags, NULL: none            */
  const orc_surface *sf;             /* surface data, NULL: none          */
} lctx;

static const double ZERO3[3] = {0.0, 0.0, 0.0};
static unsigned ptag_of(const lctx *L, int ip) { return L->tag ? L->tag[ip] : 0u; }
/* MMG5_Point.n (the tangent at a ridge point, in mmg3d) */
static const double *pn_of(const lctx *L, int ip) {
  return (L->sf && L->sf->n) ? &L->sf->n[3*(int64_t)ip] : ZERO3;
}
/* mesh->xpoint[p->xp].n1 / .n2 (xp 0: Mmg's unused, zeroed entry 0) */
static const double *xn_of(const lctx *L, int ip, int which) {
  int xp;
  const double *a;
  if (!L->sf || !L->sf->xp) return ZERO3;
  xp = L->sf->xp[ip];
  a = which ? L->sf->n2 : L->sf->n1;
  return (a && xp > 0) ? &a[3*(int64_t)xp] : ZERO3;
}

/* MMG5_buildridmet: the metric of ridge point np0 in the direction u, from its
 * ridge storage m = (tangent size, in-surface sizes of sides 1 and 2, normal
 * sizes of sides 1 and 2): the side whose normal is the more orthogonal to u,
 * basis (t, n x t, n), mr = R diag(m0, dv, dn) R^T */
static void buildridmet(const lctx *L, int np0, double ux, double uy, double uz, double mr[6]) {
  const double *m = &L->met[6*(int64_t)np0], *t = pn_of(L, np0);
  const double *n1 = xn_of(L, np0, 0), *n2 = xn_of(L, np0, 1);
  double ps1, ps2, dv, dn, u[3], r[3][3];
  ps1 = ux*n1[0] + uy*n1[1] + uz*n1[2];
  ps2 = ux*n2[0] + uy*n2[1] + uz*n2[2];
  if (fabs(ps2) < fabs(ps1)) {
    n1 = n2;
    dv = m[2];
    dn = m[4];
  } else {
    dv = m[1];
    dn = m[3];
  }
  r[0][0] = t[0]; r[1][0] = t[1]; r[2][0] = t[2];
  u[0] = n1[1]*t[2] - n1[2]*t[1];
  u[1] = n1[2]*t[0] - n1[0]*t[2];
  u[2] = n1[0]*t[1] - n1[1]*t[0];
  r[0][1] = u[0]; r[1][1] = u[1]; r[2][1] = u[2];
  r[0][2] = n1[0]; r[1][2] = n1[1]; r[2][2] = n1[2];
  mr[0] = m[0]*r[0][0]*r[0][0] + dv*r[0][1]*r[0][1] + dn*r[0][2]*r[0][2];
  mr[1] = m[0]*r[0][0]*r[1][0] + dv*r[0][1]*r[1][1] + dn*r[0][2]*r[1][2];
  mr[2] = m[0]*r[0][0]*r[2][0] + dv*r[0][1]*r[2][1] + dn*r[0][2]*r[2][2];
  mr[3] = m[0]*r[1][0]*r[1][0] + dv*r[1][1]*r[1][1] + dn*r[1][2]*r[1][2];
  mr[4] = m[0]*r[1][0]*r[2][0] + dv*r[1][1]*r[2][1] + dn*r[1][2]*r[2][2];
  mr[5] = m[0]*r[2][0]*r[2][0] + dv*r[2][1]*r[2][1] + dn*r[2][2]*r[2][2];
}

/* the tangent of the curve under edge [p, p + u] at p (MMG5_lenEdg's
 * gammaprim): u itself at a singular / non-manifold point; along the point's
 * tangent on a ridge edge (isedg); else u projected on the tangent plane of
 * the side closest to it (ridge point), of its xPoint normal (reference
 * point), of its point normal (any other) */
static void gammaprim(const lctx *L, int ip, double ux, double uy, double uz, int isedg, double g[3]) {
  const unsigned tg = ptag_of(L, ip);
  const double *n1;
  double ps1, ps2;
  if (sin_or_nom(tg)) {
    g[0] = ux; g[1] = uy; g[2] = uz;
    return;
  }
  if (isedg) {
    const double *t = pn_of(L, ip);
    ps1 = ux*t[0] + uy*t[1] + uz*t[2];
    g[0] = ps1*t[0]; g[1] = ps1*t[1]; g[2] = ps1*t[2];
    return;
  }
  if (TAG_GEO & tg) {
    const double *n2 = xn_of(L, ip, 1);
    n1 = xn_of(L, ip, 0);
    ps1 = ux*n1[0] + uy*n1[1] + uz*n1[2];
    ps2 = ux*n2[0] + uy*n2[1] + uz*n2[2];
    if (fabs(ps2) < fabs(ps1)) {
      n1 = n2;
      ps1 = ps2;
    }
  } else if (TAG_REF & tg) {
    n1 = xn_of(L, ip, 0);
    ps1 = ux*n1[0] + uy*n1[1] + uz*n1[2];
  } else {
    n1 = pn_of(L, ip);
    ps1 = ux*n1[0] + uy*n1[1] + uz*n1[2];
  }
  g[0] = ux - ps1*n1[0];
  g[1] = uy - ps1*n1[1];
  g[2] = uz - ps1*n1[2];
}

static double qform(const double *m, const double *g) {
  return m[0]*g[0]*g[0] + m[3]*g[1]*g[1] + m[5]*g[2]*g[2] + 2.0*m[1]*g[0]*g[1] + 2.0*m[2]*g[0]*g[2] +
         2.0*m[4]*g[1]*g[2];
}

/* MMG5_lenEdg: length of a surface edge along the curve, from the end
 * tangents; a negative quadratic form counts as 1 */
static double lenEdg(const lctx *L, int np0, int np1, const double *m0, const double *m1, int isedg) {
  const double *c0 = &L->xyz[3*(int64_t)np0], *c1 = &L->xyz[3*(int64_t)np1];
  double ux = c1[0] - c0[0], uy = c1[1] - c0[1], uz = c1[2] - c0[2], g0[3], g1[3], l0, l1;
  gammaprim(L, np0, ux, uy, uz, isedg, g0);
  gammaprim(L, np1, -ux, -uy, -uz, isedg, g1);
  l0 = qform(m0, g0);
  l1 = qform(m1, g1);
  if (l0 < 0.) l0 = 1.;
  if (l1 < 0.) l1 = 1.;
  return 0.5*(sqrt(l0) + sqrt(l1));
}

/* MMG5_lenSurfEdg33_ani (classic storage) / MMG5_lenSurfEdg_ani (ridge
 * storage: the metric of a non-singular ridge endpoint rebuilt per direction) */
static double lenSurfEdg_ani(const lctx *L, int np0, int np1, int isedg, int ridmet) {
  const double *c0 = &L->xyz[3*(int64_t)np0], *c1 = &L->xyz[3*(int64_t)np1];
  double ux = c1[0] - c0[0], uy = c1[1] - c0[1], uz = c1[2] - c0[2], m0[6], m1[6];
  int i;
  for (i = 0; i < 6; i++) {
    m0[i] = L->met[6*(int64_t)np0 + i];
    m1[i] = L->met[6*(int64_t)np1 + i];
  }
  if (ridmet) {
    const unsigned t0 = ptag_of(L, np0), t1 = ptag_of(L, np1);
    if (!sin_or_nom(t0) && (TAG_GEO & t0)) buildridmet(L, np0, ux, uy, uz, m0);
    if (!sin_or_nom(t1) && (TAG_GEO & t1)) buildridmet(L, np1, ux, uy, uz, m1);
  }
  return lenEdg(L, np0, np1, m0, m1, isedg);
}

/* MMG5_lenedgCoor_ani */
static double lenedgCoor_ani(const double *ca, const double *cb, const double *sa, const double *sb) {
  double ux = cb[0]-ca[0], uy = cb[1]-ca[1], uz = cb[2]-ca[2];
  double dd1 = mlen2(sa, ux, uy, uz), dd2 = mlen2(sb, ux, uy, uz);
  if (dd1 <= 0.0) dd1 = 0.0;
  if (dd2 <= 0.0) dd2 = 0.0;
  return (sqrt(dd1) + sqrt(dd2) + 4.0*sqrt(0.5*(dd1 + dd2))) / 6.0;
}

/* MMG5_moymet: the mean metric of tet v over its vertices that are not
 * non-singular ridge points (0 if none) */
static int moymet(const lctx *L, const int *v, double mm[6]) {
  int i, j, n = 0;
  double dd;
  for (i = 0; i < 6; i++) mm[i] = 0.0;
  for (j = 0; j < 4; j++) {
    if (ridge_pt(ptag_of(L, v[j]))) continue;
    n++;
    for (i = 0; i < 6; i++) mm[i] += L->met[6*(int64_t)v[j] + i];
  }
  if (!n) return 0;
  dd = 1. / n;
  for (i = 0; i < 6; i++) mm[i] = mm[i] * dd;
  return n;
}

/* MMG5_lenedg_ani (ridmet) / MMG5_lenedg33_ani of local edge ia of tet v */
static double lenedg_ani(const lctx *L, const int *v, int xt, int ia, int ridmet) {
  const int ip1 = v[IARE[ia][0]], ip2 = v[IARE[ia][1]];
  int i;
  if (xt && L->sf && L->sf->xtag) {
    const unsigned et = L->sf->xtag[6*(int64_t)xt + ia];
    if (et & TAG_BDY) return lenSurfEdg_ani(L, ip1, ip2, (et & TAG_GEO) != 0, ridmet);
  }
  {
    double m1[6], m2[6];
    for (i = 0; i < 6; i++) {
      m1[i] = L->met[6*(int64_t)ip1 + i];
      m2[i] = L->met[6*(int64_t)ip2 + i];
    }
    if (ridmet) {                     /* MMG5_lenedgspl_ani */
      if (ridge_pt(ptag_of(L, ip1)) && !moymet(L, v, m1)) return 0.0;
      if (ridge_pt(ptag_of(L, ip2)) && !moymet(L, v, m2)) return 0.0;
    }
    return lenedgCoor_ani(&L->xyz[3*(int64_t)ip1], &L->xyz[3*(int64_t)ip2], m1, m2);
  }
}

/* MMG5_lenSurfEdg_iso on a size-6 metric as the reference calls it for the
 * parallel edges with metRidTyp = 1 (src/quality_pmmg.c:466): h = met->m[ip],
 * the flat array read as if it were isotropic */
static double len_iso_flat(const double *xyz, const double *met, int p1, int p2) {
  const double *c1 = &xyz[3*p1], *c2 = &xyz[3*p2];
  double h1 = met[p1], h2 = met[p2], l, r;
  l = (c2[0]-c1[0])*(c2[0]-c1[0]) + (c2[1]-c1[1])*(c2[1]-c1[1]) + (c2[2]-c1[2])*(c2[2]-c1[2]);
  l = sqrt(l);
  r = h2 / h1 - 1.0;
  return (fabs(r) < EPS) ? (l / h1) : (l / (h2 - h1) * log1p(r));
}

/* open-addressing set of unordered edges (key = min << 32 | max) */
typedef struct { uint64_t cap, mask, *tab; uint8_t *popped; } eset;
static int eset_init(eset *e, int64_t nmax) {
  e->cap = 1;
  while (e->cap < (uint64_t)(2 * nmax + 16)) e->cap <<= 1;
  e->mask = e->cap - 1;
  e->tab = (uint64_t *)calloc(e->cap, sizeof(uint64_t));
  e->popped = (uint8_t *)calloc(e->cap, 1);
  return e->tab && e->popped;
}
static void eset_free(eset *e) { free(e->tab); free(e->popped); }
/* slot of the edge (inserted if absent and ins); -1 if absent */
static int64_t eset_slot(eset *e, int a, int b, int ins) {
  int lo = a < b ? a : b, hi = a < b ? b : a;
  uint64_t key = hkey(lo, hi), h = (key * 0x9e3779b97f4a7c15ULL) >> 20;
  while (e->tab[h & e->mask] && e->tab[h & e->mask] != key) h++;
  if (!e->tab[h & e->mask]) {
    if (!ins) return -1;
    e->tab[h & e->mask] = key;
  }
  return (int64_t)(h & e->mask);
}

static void len_count(orc_lenstats *st, double len, int np_, int nq_) {
  static const double bd[9] = {0.0, 0.3, 0.6, 0.7071, 0.9, 1.3, 1.4142, 2.0, 5.0};
  int i;
  if (!len) { st->nullEdge++; return; }
  st->avlen += len;
  st->ned++;
  if (len < st->lmin) { st->lmin = len; st->amin = np_; st->bmin = nq_; }
  if (len > st->lmax) { st->lmax = len; st->amax = np_; st->bmax = nq_; }
  for (i = 0; i < 8; i++)
    if (bd[i] <= len && len < bd[i+1]) { st->hl[i]++; break; }
  if (i == 8) st->hl[8]++;
}

int orc_prilen_full(int64_t np, int64_t ne, const double *xyz, const int *tet,
                    const double *met, int msize, const uint16_t *tag, int metRidTyp,
                    const orc_surface *sf, int64_t npar, const int *pa, const int *pb,
                    const int *powner, const uint16_t *ptag, int myrank, int exact_once,
                    orc_lenstats *st) {
  eset e;
  int64_t k, i;
  lctx L;
  const int ani33 = !metRidTyp && msize == 6;     /* :462, :527 */
  (void)np;
  L.xyz = xyz; L.met = met; L.tag = tag; L.sf = sf;
  if (!eset_init(&e, 6 * ne)) { eset_free(&e); return 0; }
  memset(st, 0, sizeof *st);
  st->lmin = 1.e30;
  st->lmax = 0.0;
  /* MMG5_hashEdge of every edge of every valid tet (:421-440) */
  for (k = 1; k <= ne; k++) {
    const int *v = &tet[4*k];
    int ia;
    if (v[0] <= 0) continue;
    for (ia = 0; ia < 6; ia++) eset_slot(&e, v[IARE[ia][0]], v[IARE[ia][1]], 1);
  }
  /* 1) owned parallel edges, in communicator order (:445-502):
   *    MMG5_lenSurfEdg33_ani (classic tensor storage) or MMG5_lenSurfEdg_iso
   *    -- the latter also for a size-6 metric with metRidTyp = 1, as written */
  for (i = 0; i < npar; i++) {
    int64_t s = eset_slot(&e, pa[i], pb[i], 0);
    double len;
    if (powner[i] != myrank) {
      if (exact_once && s >= 0) e.popped[s] = 1;    /* not ours: never counted here */
      continue;
    }
    if (s < 0 || e.popped[s]) continue;            /* MMG5_hashPop failed */
    e.popped[s] = 1;
    if (ani33)
      len = lenSurfEdg_ani(&L, pa[i], pb[i], ptag && (ptag[i] & TAG_GEO), 0);
    else if (msize == 6)
      len = len_iso_flat(xyz, met, pa[i], pb[i]);
    else
      len = len_iso(xyz, met, pa[i], pb[i]);
    len_count(st, len, pa[i], pb[i]);
  }
  /* 2) the other edges, (k, ia) order, ridge-only tets skipped (:505-564):
   *    MMG5_lenedg33_ani, or MMG5_lenedg = lenedg_ani / lenedg_iso (the iso
   *    surface and volume formulas coincide) */
  for (k = 1; k <= ne; k++) {
    const int *v = &tet[4*k];
    const int xt = (sf && sf->xt) ? sf->xt[k] : 0;
    int ia;
    if (v[0] <= 0) continue;
    if (tet_4ridge(v, tag)) continue;
    for (ia = 0; ia < 6; ia++) {
      int np_ = v[IARE[ia][0]], nq_ = v[IARE[ia][1]];
      int64_t s = eset_slot(&e, np_, nq_, 0);
      double len;
      if (e.popped[s]) continue;                    /* MMG5_hashPop returned 0 */
      e.popped[s] = 1;
      if (msize == 6) len = lenedg_ani(&L, v, xt, ia, !ani33);
      else len = len_iso(xyz, met, np_, nq_);
      len_count(st, len, np_, nq_);
    }
  }
  eset_free(&e);
  return 1;
}

int orc_prilen_dist(int64_t np, int64_t ne, const double *xyz, const int *tet,
                    const double *met, int msize, const uint16_t *tag, int64_t npar,
                    const int *pa, const int *pb, const int *powner, int myrank, int exact_once,
                    orc_lenstats *st) {
  return orc_prilen_full(np, ne, xyz, tet, met, msize, tag, 0, NULL, npar, pa, pb, powner, NULL, myrank,
                         exact_once, st);
}

int orc_prilen(int64_t np, int64_t ne, const double *xyz, const int *tet, const double *met,
               int msize, orc_lenstats *st) {
  return orc_prilen_dist(np, ne, xyz, tet, met, msize, NULL, 0, NULL, NULL, NULL, 0, 0, st);
}
