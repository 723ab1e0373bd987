/*
 * pmx_oracle.h -- CPU restatement of ParMmg's post-remesh transfer path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this code, and only as the checker.
 * The product path (parmmg_amd, libpmx_transfer.so) never links it.
 *
 * PARITY UNPINNED: the reference hot path (src/locate_pmmg.c,
 * src/barycoord_pmmg.c, src/interpmesh_pmmg.c) cannot be compiled here without
 * the absent Mmg headers, and the reference ships no golden vectors for this
 * path (its CTest suite checks exit codes only; WaveSurface locate KATs live in
 * the external testparmmg repo).  The restatement is therefore pinned only by
 * self-consistency properties (see DESIGN.md "Oracle").  The Mmg helpers
 * (MMG5_orvol, MMG5_nonUnitNorPts, MMG5_invmat, quality, edge length) are
 * restated from the public Mmg sources @889d408 and are unpinned as well.
 *
 * Conventions follow the reference: old-mesh arrays are 1-based (slot 0
 * unused), adja[4*(k-1)+1+f] = 4*k'+f', adjt[3*(k-1)+1+e] = 3*k'+e'.
 */
#ifndef PMX_ORACLE_H
#define PMX_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_ctx orc_ctx;

/* hausd: surface distance threshold (mesh->info.hausd). */
orc_ctx *orc_create(int64_t np, int64_t ne, int64_t nt,
                    const double *xyz, const int *tet, const int *adja,
                    const int *tria, const int *adjt, double hausd);
void     orc_destroy(orc_ctx *o);

/* Reset the mutable state exactly as the reference does at the start of
 * PMMG_interpMetricsAndFields_mesh (src/interpmesh_pmmg.c:515-526) after
 * PMMG_precompute_nodeTrias (src/locate_pmmg.c:134-195). */
void orc_reset(orc_ctx *o);

/* PMMG_locatePointVol (src/locate_pmmg.c:786-883).  *elem is the start tet
 * in / found tet out.  phi[4]: barycentric coordinates un-permuted (index =
 * local vertex).  Returns 1 found, -1 found by exhaustive search, 0 closest. */
int orc_locate_vol(orc_ctx *o, const double *p, int *elem, double *phi, int *steps);

/* PMMG_locatePointBdy (src/locate_pmmg.c:587-723).  ip is unused by the
 * reference; edge/vertex are -1 when unset.  bary[8] receives the reference's
 * barycoord array as (idx,val) pairs: idx in bary_idx[4], val in bary_val[4]. */
int orc_locate_bdy(orc_ctx *o, const double *p, int *elem, int *edge, int *vertex,
                   int *bary_idx, double *bary_val, int *steps);

/* 1 if the point is inside tet k by the reference predicate (lambda_min > -EPS) */
int orc_tet_contains(orc_ctx *o, int k, const double *p, double *lmin);
int orc_tria_contains(orc_ctx *o, int k, const double *p);

/* MMG5_invmat restatement; returns 1 ok, 0 fail (mi untouched). */
int orc_invmat(const double *m, double *mi);

/*
 * PMMG_interpMetricsAndFields_mesh (src/interpmesh_pmmg.c:477-649) over an
 * explicit list of new points.
 *   npts, pxyz[3*npts], ptag[npts]      new points (0-based list)
 *   order[npts] or NULL                 visitation order (first visit of each
 *                                       vertex in the new-tet loop :535-545)
 *   nsol, size[nsol], oldsol[nsol]      solutions; oldsol[s] = size*(np+1) doubles
 *   newsol[nsol]                        outputs, size*npts doubles (in/out: left
 *                                       untouched where the reference leaves them)
 *   imet                                index of the metric in the list or -1
 *   start_vol/start_bdy                 NULL = reference carry-over of the found
 *                                       element (:528-532); else per-point start
 *   fresh                               0 = reference semantics (point flags
 *                                       persist across queries); 1 = point flags
 *                                       restored to their post-nodeTrias state
 *                                       before every query (GPU semantics)
 *   elem/status/steps/edge/vertex       per-point outputs (may be NULL)
 * Returns 1.
 */
int orc_interp_points(orc_ctx *o, int64_t npts, const double *pxyz, const int *ptag,
                      const int64_t *order, int nsol, const int *size,
                      const double *const *oldsol, double *const *newsol, int imet,
                      const int *start_vol, const int *start_bdy, int fresh,
                      int *elem, int *status, int *steps, int *edge, int *vertex);

/* MMG3D_Set_constantSize restatement: iso m=hsiz, ani diag(1/hsiz^2). */
void orc_constant_size(int64_t npts, int size, double hsiz, double *m);

/* ---- statistics (restated Mmg per-element kernels; unpinned) ---------- */
typedef struct {
  int64_t ne;            /* counted elements */
  double  max, min, avg; /* alpha*q */
  int64_t iel;           /* first element realising min (1-based) */
  int64_t good, med;
  int64_t his[5];
  int64_t nrid;          /* OUTQUA: elements with 4 ridge vertices */
} orc_qualstats;

/* per-tet quality (MMG3D_tetraQual -> MMG5_caltet_iso / caltet33_ani) */
void orc_tetra_qual(int64_t ne, const double *xyz, const int *tet,
                    const double *met, int msize, double *qual /* ne+1 */);
void orc_tetra_qual_rid(int64_t ne, const double *xyz, const int *tet, const double *met, int msize,
                        const uint16_t *tag, int metRidTyp, double *qual);
/* histogram of MMG3D_computeInqua-style statistics over qual[1..ne]; with
 * point tags (np+1, or NULL), MMG3D_computeOutqua's nrid */
void orc_qualhisto(int64_t ne, const int *tet, const double *qual, orc_qualstats *st);
void orc_qualhisto_tags(int64_t ne, const int *tet, const double *qual, const uint16_t *tag,
                        orc_qualstats *st);

typedef struct {
  int64_t ned, nullEdge;
  double  avlen, lmin, lmax;
  int64_t amin, bmin, amax, bmax;
  int64_t hl[9];
} orc_lenstats;
/* unique-edge length histogram (MMG3D_computePrilen, centralized) */
int orc_prilen(int64_t np, int64_t ne, const double *xyz, const int *tet,
               const double *met, int msize, orc_lenstats *st);
/* PMMG_computePrilen (src/quality_pmmg.c:370-574): point tags (np+1 or NULL:
 * tets with 4 ridge vertices skipped, :509-517) and npar parallel edges
 * pa[i] -> pb[i] owned by rank powner[i]: owned ones first in list order,
 * then every other edge in (k, ia) order; exact_once: the non-owned parallel
 * edges are not counted (the reference counts them, its warning :585-586). */
int orc_prilen_dist(int64_t np, int64_t ne, const double *xyz, const int *tet,
                    const double *met, int msize, const uint16_t *tag, int64_t npar,
                    const int *pa, const int *pb, const int *powner, int myrank, int exact_once,
                    orc_lenstats *st);

/* Mmg's surface data, as Mmg holds it (all 1-based; NULL members: absent):
 * xt[k] = tetra[k].xt (0: no xTetra), xtag[6*x + ia] = xtetra[x].tag[ia],
 * n[3*ip] = point[ip].n, xp[ip] = point[ip].xp, n1/n2[3*x] = xpoint[x].n1/n2 */
typedef struct {
  const int      *xt;
  const uint16_t *xtag;
  const double   *n;
  const int      *xp;
  const double   *n1, *n2;
} orc_surface;
/* PMMG_computePrilen / MMG3D_computePrilen with metRidTyp and the surface
 * data (NULL: no xTetra, zero normals); ptag[i] = the parallel edge's tag
 * (MMG5_hGet on the parallel-edge hash, :456; NULL: 0) */
int orc_prilen_full(int64_t np, int64_t ne, const double *xyz, const int *tet,
                    const double *met, int msize, const uint16_t *tag, int metRidTyp,
                    const orc_surface *sf, int64_t npar, const int *pa, const int *pb,
                    const int *powner, const uint16_t *ptag, int myrank, int exact_once,
                    orc_lenstats *st);

#ifdef __cplusplus
}
#endif
#endif
