/*
 * pmx_transfer.h -- C ABI of the MI355X-native ParMmg transfer path.
 *
 * Replaces, behind ParMmg's own seams, the reference interface:
 *   PMMG_interpMetricsAndFields(PMMG_pParMesh, int *permNodGlob)
 *       reference src/parmmg.h:472, def src/interpmesh_pmmg.c:663-741,
 *       sole caller src/libparmmg1.c:829  -> PMX_interpMetricsAndFields
 *   PMMG_copyMetricsAndFields_point(...)
 *       reference src/parmmg.h:473, def src/interpmesh_pmmg.c:432-446,
 *       caller src/libparmmg1.c:792       -> PMX_copyMetricsAndFields_point
 *   PMMG_locatePointVol / PMMG_locatePointBdy (src/locate_pmmg.h:63-68) and
 *   PMMG_interp{4,3,2}bar_{iso,ani} selected by PMMG_setfunc
 *       (src/parmmgexterns.c:4-6, src/libparmmg_tools.c:595-612)
 *                                          -> pmx_run (batched, on device)
 *   PMMG_tetraQual / PMMG_qualhisto / PMMG_prilen (src/parmmg.h:564-566,
 *       def src/quality_pmmg.c:156-346,591-733)
 *                                          -> pmx_tetra_qual / pmx_qualhisto /
 *                                             pmx_prilen
 *
 * Rules (ParMmg conventions): plain C, pointers + sizes, no torch types.
 * Host memory is caller owned; device buffers are owned by the context.
 * Functions return 1 on success and 0 on failure (pmx_last_error() says why).
 * One host thread per context, one context per GPU (rank -> device by
 * rank % ndev).  Mesh arrays are 1-based exactly as in Mmg: slot 0 unused,
 * adja[4*(k-1)+1+f] = 4*k'+f', adjt[3*(k-1)+1+e] = 3*k'+e'.
 */
#ifndef PMX_TRANSFER_H
#define PMX_TRANSFER_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PMX_TAG_REQ   4        /* MG_REQ */
#define PMX_TAG_BDY   16       /* MG_BDY */
#define PMX_TAG_NUL   16384    /* MG_NUL */
#define PMX_MAX_SOLS  8        /* metric + fields per group */

typedef struct pmx_ctx pmx_ctx;

/* Strided view of an Mmg-style AoS mesh.  Pass e.g.
 *   point_c = &mesh->point[0].c[0], point_stride = sizeof(MMG5_Point),
 *   tetra_v = &mesh->tetra[0].v[0], tetra_stride = sizeof(MMG5_Tetra).
 * Strides are in BYTES.  Entries 1..n are read. */
typedef struct {
  int64_t       np, ne, nt;
  const double *point_c;  int64_t point_stride;
  const int    *tetra_v;  int64_t tetra_stride;
  const int    *adja;                       /* 4*ne+5 ints, may be NULL */
  const int    *tria_v;   int64_t tria_stride;
  const int    *adjt;                       /* 3*nt+4 ints, may be NULL  */
  double        hausd;                      /* mesh->info.hausd          */
} pmx_mesh_view;

/* A solution on the mesh vertices: m[size*ip + j], ip = 1..np (Mmg layout). */
typedef struct {
  int           size;     /* 1 scalar/iso metric, 3 vector, 6 tensor/ani metric */
  double       *m;
} pmx_sol_view;

/* New points to transfer onto: c[ip] at (const char*)c + ip*stride, ip=first..last;
 * tag as uint16_t at (const char*)tag + ip*tag_stride (MMG5_Point.tag).
 * Optional new tets (tetra_v != NULL, entries 1..ne, stride in bytes, vertex
 * indices in the same numbering as ip): only the points of valid tets
 * (v[0] > 0) are located, as in the reference's vertex loop over the new tets
 * (src/interpmesh_pmmg.c:535-541); the others are left untouched (a constant
 * size metric is still written on every valid point).  NULL: every point.
 * The tets also stay on the device (pmx_new_mesh_qual, pmx_promote_background).
 * They are read, validated and sent by the first pmx_run on these points,
 * once its step is enqueued (their DMA overlaps the step and the download; a
 * vertex outside [first, last] fails that pmx_run): the array must stay
 * valid until then. */
typedef struct {
  int64_t         first, last;
  const double   *c;    int64_t stride;
  const uint16_t *tag;  int64_t tag_stride;
  const int      *tetra_v;  int64_t tetra_stride;  int64_t ne;
} pmx_points_view;

/* Localisation statistics (reference PMMG_locateStats, src/locate_pmmg.h:45-50) */
typedef struct {
  int64_t nvol, nbdy;        /* located points by path            */
  int64_t nexhaust;          /* exhaustive searches               */
  int64_t nclosest;          /* not found -> closest element      */
  int64_t stepmin, stepmax;  /* |steps| over every located point, */
  double  stepav;            /* exhaustive ones included, as
                                PMMG_locate_postprocessing (src/locate_pmmg.c:
                                995-1028); an exhaustive point counts its walk
                                steps + 1 (the reference adds every tet it
                                scanned); no point: stepmin = the background's
                                ne, stepav 0                          */
} pmx_locate_stats;

/* ---- context ---------------------------------------------------------- */
/* A context owns one stream's device buffers and a pinned host staging arena
 * (hipHostMalloc, grown on demand, kept until pmx_destroy): about 36 B per
 * background tet + (24 + 8*S) B per background vertex, or 65 B per new vertex,
 * whichever upload is larger.  Host gathers/scatters of 2^18 elements or more
 * use PMX_HOST_THREADS threads (default min(8, hardware threads));
 * PMX_HOST_THREADS_MIN overrides that threshold. */
pmx_ctx    *pmx_create(int device);
void        pmx_destroy(pmx_ctx *ctx);
/* ctx == NULL: the last error of a call made without a context (this thread) */
const char *pmx_last_error(pmx_ctx *ctx);
/* Run on an external HIP stream (hipStream_t passed as void*); NULL = own. */
int         pmx_set_stream(pmx_ctx *ctx, void *hip_stream);
int         pmx_synchronize(pmx_ctx *ctx);
/* Device and build identification. */
int         pmx_device_info(pmx_ctx *ctx, char *buf, int buflen);

/* ---- background (old) group -------------------------------------------- */
/* AoS -> SoA conversion on the host, then upload.  imet = index of the
 * metric in sols[] (or -1).  If adja is NULL it is rebuilt from tetra_v by
 * device face matching (overlapped with the solutions' upload; half the tet
 * bytes over PCIe -- the faster choice for a valid conforming mesh, whose
 * face adjacency is unique; non-manifold faces fail the upload).
 * Every argument is checked before the context changes; on failure the
 * context holds no background (pmx_run refuses until a good upload). */
int pmx_upload_background(pmx_ctx *ctx, const pmx_mesh_view *old_mesh,
                          int nsol, const pmx_sol_view *old_sols, int imet);

/* ---- new points -------------------------------------------------------- */
int pmx_upload_points(pmx_ctx *ctx, const pmx_points_view *pts);

/* ---- the hot path (device resident) ------------------------------------ */
typedef struct {
  int    hint_stride;              /* hint grid built from every k-th tet,
                                      0 -> default                           */
  int    max_walk;                 /* walk step cap before exhaustive, 0=auto */
  double hsiz;                     /* >0: constant-size metric shortcut
                                      (src/interpmesh_pmmg.c:497-512)        */
  int    timing;                   /* record per-kernel HIP events           */
  int    flags;                    /* PMX_RUN_* (0 = production defaults)    */
} pmx_run_opts;

/* pmx_run_opts.flags */
#define PMX_RUN_REFERENCE_WALK   0x1  /* volume walk in the reference's order
                                         (k_walk) instead of the slot walk    */
#define PMX_RUN_NO_INLINE_TIES   0x2  /* every near-face point to the tie BFS */
#define PMX_RUN_RECORD_STARTS    0x4  /* keep each volume walk's start tet    */
#define PMX_RUN_SERIAL_SURFACE   0x8  /* surface path on the main stream      */
#define PMX_RUN_FRESH_BACKGROUND 0x10 /* redo every device pass the uploads
                                         ran on the raw arrays (derived data,
                                         fan check, device-built layouts, the
                                         orphan marks of the new tets): one
                                         ParMmg iteration per step            */
#define PMX_RUN_SEQUENTIAL_SURFACE 0x40 /* the reference's SEQUENTIAL surface
                                         semantics (src/interpmesh_pmmg.c:
                                         528-599, src/locate_pmmg.c:209-334):
                                         the boundary points in the vertex
                                         loop's first-visit order through the
                                         new tets, each query starting from the
                                         previous one's tria, the point flags
                                         of the shadow cone / wedge tests and
                                         mesh->base carried over.  Needs the new
                                         tets (points view or
                                         pmx_upload_new_tets).  Default: every
                                         query fresh from its hint tria        */
#define PMX_RUN_SEQUENTIAL_VOLUME 0x80 /* the reference's sequential volume
                                         walk (src/locate_pmmg.c:786-883 from
                                         the previous volume point's tet,
                                         src/interpmesh_pmmg.c:529,606): ties
                                         resolved by the reference's own path,
                                         a walk into a deleted tet returning
                                         the closest tet it visited.  Needs
                                         the new tets.  Default: the canonical
                                         (smallest-index) tet of a tie, and
                                         the exhaustive scan after a deleted
                                         tet                                  */
#define PMX_RUN_DEBUG_BARRIER_TIMEOUT 0x100 /* test hook: the fallback's grid
                                         barriers do not wait (the step must
                                         then fail, never return silently)   */
#define PMX_RUN_EAGER_DOWNLOAD   0x20 /* the step's fields start down into
                                         pinned staging as soon as it ends
                                         (overlapping the host work that
                                         follows pmx_run); pmx_download then
                                         only scatters them.  For callers that
                                         always download (the ParMmg seam
                                         sets it)                             */

/* Locate every uploaded new point in the background group and interpolate all
 * background solutions onto it.  Results stay on the device.  Asynchronous:
 * device-side failures (a fallback grid barrier that timed out) are reported
 * by the next pmx_synchronize / pmx_download, which then return 0. */
int pmx_run(pmx_ctx *ctx, const pmx_run_opts *opts);

/* Copy results to the host.  new_sols[s].m receives size*(npts) doubles in
 * point-list order (entries of REQ points and of failed tensor inversions are
 * left untouched).  elem/status/steps may be NULL.  Every host output call
 * takes the capacity its arrays were allocated for and returns 0 (nothing
 * written, pmx_last_error says why) when the device holds more: here
 * npts_cap rows -- size*npts_cap doubles per solution, npts_cap ints for
 * elem/status/steps -- with npts = last - first + 1 of the points view. */
int pmx_download(pmx_ctx *ctx, const pmx_sol_view *new_sols, int64_t npts_cap, int *elem,
                 int *status, int *steps);
/* Per-point start element used by the device walk (debug/parity).  Volume
 * points' starts are recorded only by a pmx_run with PMX_RUN_RECORD_STARTS;
 * surface points' always.  cap: ints in start (>= npts). */
int pmx_download_starts(pmx_ctx *ctx, int *start, int64_t cap);
/* Per-point reference-style extras for boundary points: edge/vertex (-1
 * unset).  cap: ints in each array (>= npts). */
int pmx_download_border(pmx_ctx *ctx, int *edge, int *vertex, int64_t cap);
/* 1 when the context holds a step's results on its current points (a pmx_run
 * after the last pmx_upload_points), 0 otherwise -- e.g. a group whose
 * interpolation had nothing to locate (src/interpmesh_pmmg.c:497-512). */
int pmx_step_ready(pmx_ctx *ctx);
int pmx_locate_stats_get(pmx_ctx *ctx, pmx_locate_stats *st);
/* After a PMX_RUN_SEQUENTIAL_SURFACE step: the boundary points the reference
 * would locate (*nseq) and how many of them the device replayed one by one on
 * the reference's state (*nreplay; the others kept their speculative result:
 * same start tria as the reference, no shadow-wedge test on the way). */
int pmx_seq_surface_stats(pmx_ctx *ctx, int64_t *nseq, int64_t *nreplay);
/* The same for the volume points of a PMX_RUN_SEQUENTIAL_VOLUME step. */
int pmx_seq_volume_stats(pmx_ctx *ctx, int64_t *nseq, int64_t *nreplay);
/* Lane utilisation of the last step's walks (path 0 volume, 1 surface): a
 * wave iterates until its longest walk ends, so step_sum / lane_steps is the
 * fraction of lane-steps that did work.  Over the walk's per-wave records:
 * located points, their summed steps, 64 x the longest walk of each wave,
 * and the waves by their longest walk (entry 15: 15 steps or more). */
typedef struct {
  int64_t waves, located, step_sum, lane_steps;
  int64_t wave_max_hist[16];
} pmx_wave_stats;
int pmx_locate_wave_stats(pmx_ctx *ctx, int path, pmx_wave_stats *st);

/* Device pointers of the resident result buffers (for collectives / chaining):
 * which = 0 packed solutions [npts][S], 1 elem, 2 status. */
void *pmx_device_buffer(pmx_ctx *ctx, int which);
/* Device memory on the context's GPU for a C caller (zeroed): e.g. the
 * per-group partial records of the _device statistics functions. */
void *pmx_device_alloc(pmx_ctx *ctx, size_t bytes);
int pmx_device_free(pmx_ctx *ctx, void *p);
/* Copy bytes of device memory (e.g. such partial records) to the host, after
 * the context stream's earlier work; blocking. */
int pmx_device_download(pmx_ctx *ctx, void *host, const void *dev, size_t bytes);
/* and the other way (e.g. an empty partial record of a rank without a group) */
int pmx_device_upload(pmx_ctx *ctx, void *dev, const void *host, size_t bytes);
/* Inspection: copy the volume hint grid of the last run to host (cap cells);
 * returns the number of cells (0 on error). */
int64_t pmx_debug_hint_grid(pmx_ctx *ctx, int *host, int64_t cap);

/* ---- background topology on the device (the old-group
 * snapshot of src/grpsplit_pmmg.c:207-418) ------------------------------- */

/* Tet face adjacency, Mmg layout: adja[4*(k-1)+1+f] = 4*k'+f' (0 = boundary),
 * 4*ne+5 ints.  Replaces MMG3D_hashTetra's adjacency (called by ParMmg at
 * src/libparmmg1.c:272, src/distributemesh_pmmg.c:1185, src/metis_pmmg.c:756).
 * Tets with v[0] <= 0 are skipped.  Returns 1, or 0 on error / non-manifold
 * faces (pmx_last_error).  pmx_upload_background builds it the same way when
 * its mesh view has adja == NULL. */
int pmx_build_adja(pmx_ctx *ctx, int64_t ne, int64_t np, const int *tetra_v,
                   int64_t tetra_stride, int *adja);

/* Boundary trias (faces with adja 0) in (tet, face) order, vertices in
 * MMG5_idir order: tria[3*k+j], k = 1..nt (row 0 unused, maxnt rows at most);
 * and, if adjt != NULL, their edge adjacency adjt[3*(k-1)+1+e] = 3*k'+e'
 * (edge e = vertices (e+1)%3, (e+2)%3; 0 unless exactly 2 trias share it).
 * Replaces MMG5_chkBdryTria + MMG3D_hashTria on the snapshot
 * (src/grpsplit_pmmg.c:403-414).  Returns nt, or -1 on error. */
int64_t pmx_build_bdry(pmx_ctx *ctx, int64_t ne, int64_t np, const int *tetra_v,
                       int64_t tetra_stride, const int *adja, int *tria, int64_t maxnt,
                       int *adjt);

/* Device time (ms) of the last pmx_build_adja / pmx_build_bdry. */
double pmx_topo_ms(pmx_ctx *ctx);

/* Kernel timing of the last pmx_run with opts.timing != 0, in ms:
 * which = 0 hint build, 1 volume locate+interp, 2 surface locate+interp,
 * 3 exhaustive fallback, 4 total. */
double pmx_kernel_ms(pmx_ctx *ctx, int which);
/* Forget recorded kernel timings. */
int    pmx_timing_reset(pmx_ctx *ctx);

/* ---- drop-in mirrors of the reference seams ------------------------------ */
typedef struct {
  pmx_mesh_view    mesh;        /* new mesh (only points are read)            */
  pmx_points_view  points;      /* its vertices (first=1,last=np typically)   */
  pmx_sol_view    *met;         /* new metric (written), or NULL              */
  pmx_sol_view    *fields;      /* new fields (written), nsols entries        */
  int              nsols;
  double           hsiz;        /* mesh->info.hsiz                            */
  pmx_mesh_view    old_mesh;    /* background snapshot (old_listgrp)          */
  pmx_sol_view    *old_met;
  pmx_sol_view    *old_fields;
} pmx_group;

/* PMMG_interpMetricsAndFields (src/interpmesh_pmmg.c:663-741): loop on
 * groups; inputMet = parmesh->info.inputMet.  Returns 1 ok / 0 fail. */
int PMX_interpMetricsAndFields(pmx_ctx *ctx, int ngrp, pmx_group *grps,
                               const int *permNodGlob, int inputMet);

/* The same with one context per group: group g on ctxs[g] (caller-owned, all
 * on one device, e.g. kept across ParMmg iterations).  Every group's step is
 * enqueued before the first download, and each context keeps its group's new
 * points, new tets and results until its next upload -- so that
 * PMMG_tetraQual (src/libparmmg1.c:845) can run on them without a re-upload
 * (pmx_new_mesh_qual_synced).  Errors in pmx_last_error(ctxs[0]). */
int PMX_interpMetricsAndFields_groups(pmx_ctx *const *ctxs, int ngrp, pmx_group *grps,
                                      const int *permNodGlob, int inputMet);

/* PMMG_copyMetricsAndFields_point (src/interpmesh_pmmg.c:432-446) on the
 * caller's host arrays (a host loop: nothing to do on the device). Old-point
 * tags are read through old_tag (uint16_t, stride bytes).  ctx may be NULL
 * (the reference calls it at src/libparmmg1.c:792, before the first
 * interpolation): errors then in pmx_last_error(NULL), per host thread. */
int PMX_copyMetricsAndFields_point(pmx_ctx *ctx, pmx_group *grp,
                                   const uint16_t *old_tag, int64_t old_tag_stride,
                                   const int *permNodGlob, int renum, int inputMet);

/* The same copy on device-resident data (PMMG_copySol_point, :311-358),
 * after a pmx_run: rows of the new points that the step did not write take
 * the background's values of its MG_REQ points (old ip -> new point
 * permNodGlob[ip], or ip; points-view numbering).  Equivalent to the
 * reference's copy before the interpolation, which then overwrites the rows
 * it writes.  Needs the background's point tags on the device (promoted, or
 * pmx_upload_point_tags); copy_metric: the metric too (inputMet and no
 * -hsiz, :378).  The copied rows count as written (pmx_download,
 * pmx_promote_background). */
int pmx_copy_required(pmx_ctx *ctx, const int *permNodGlob, int copy_metric);

/* ---- Medit files ---------------------------------
 * The wire format of the path's inputs and outputs: ParMmg reads/writes them
 * through Mmg (src/inout_pmmg.c:440-991 -> MMG3D_loadMesh / saveMesh /
 * loadSol / saveSol).  ASCII .mesh/.sol and binary .meshb/.solb (chosen by
 * the extension; binary versions 1-4 read, 2-4 written).  Arrays in Mmg's
 * layout (1-based, slot 0 untouched; tensors (11,12,13,22,23,33), converted
 * from/to Medit's (11,12,22,13,23,33)).  Keywords other than Vertices,
 * Tetrahedra, Triangles, RequiredVertices (mesh) and SolAtVertices (solution)
 * are skipped.  No context: errors in pmx_medit_last_error() (per thread). */
typedef struct {
  int64_t np, ne, nt, nreq;    /* vertices, tetrahedra, triangles, required vertices */
  int     dim, version;
} pmx_medit_info;
const char *pmx_medit_last_error(void);
int pmx_medit_mesh_info(const char *path, pmx_medit_info *info);
/* sized = the counts the arrays were allocated for (pmx_medit_mesh_info of
 * the same file): the read fails, writing nothing past them, if the file's
 * counts differ (changed file) or a keyword block appears twice.
 * xyz[3*(np+1)], tet[4*(ne+1)] required; vref[np+1], tetref[ne+1],
 * tria[3*(nt+1)], triaref[nt+1], req[nreq] may be NULL */
int pmx_medit_mesh_read(const char *path, const pmx_medit_info *sized, double *xyz, int *vref, int *tet,
                        int *tetref, int *tria, int *triaref, int *req);
int pmx_medit_mesh_write(const char *path, int64_t np, const double *xyz, const int *vref, int64_t ne,
                         const int *tet, const int *tetref, int64_t nt, const int *tria, const int *triaref,
                         int64_t nreq, const int *req);
/* solutions at vertices: types 1 scalar, 2 vector (3), 3 symmetric tensor (6) */
int pmx_medit_sol_info(const char *path, int64_t *np, int *nsol, int *types);
/* fields[s]: size(types[s])*(np+1); np, nsol, types = what the fields were
 * sized for (pmx_medit_sol_info): a different header fails the read */
int pmx_medit_sol_read(const char *path, int64_t np, int nsol, const int *types, double **fields);
int pmx_medit_sol_write(const char *path, int64_t np, int nsol, const int *types,
                        const double *const *fields);

/* ---- statistics ---------------------------------------------------------- */
/* Reference: PMMG_tetraQual / PMMG_qualhisto / PMMG_prilen (src/parmmg.h:564-566,
 * def src/quality_pmmg.c:156-733).  The per-element arithmetic is Mmg's,
 * restated (MMG5_caltet_iso / caltet33_ani, MMG5_lenEdg*; unpinned). */
#define PMX_INQUA  0          /* PMMG_INQUA : before the remesh                */
#define PMX_OUTQUA 1          /* PMMG_OUTQUA: after it (counts nrid, below)    */
#define PMX_LESQUA 2          /* mesh->info.optimLES: MMG3D_computeLESqua
                                 (src/quality_pmmg.c:221-224) -- not restated:
                                 the statistics calls refuse it (return 0)     */
#define PMX_TAG_GEO    2      /* MG_GEO  */
#define PMX_TAG_PARBDY 8192   /* MG_PARBDY */

/* Per-group partials as written to device memory by the *_device functions:
 * plain 8-byte fields, no padding (all-gathered as int64 words). */
typedef struct {
  double  avg, max, min;       /* alpha*q: SUM, max, min                     */
  int64_t iel, ne, np, good, med, nrid;
  int64_t his[5];
  int64_t iel_grp;             /* filled by the host fold                    */
} pmx_qual_part;               /* 15 x 8 B */
typedef struct {
  double  avlen, lmin, lmax;   /* avlen is the SUM over edges                */
  int64_t amin, bmin, amax, bmax, ned, nullEdge;
  int64_t hl[9];
} pmx_len_part;                /* 18 x 8 B */

/* ---- device residency across ParMmg iterations -------------------------
 * PMMG_update_oldGrps (src/libparmmg1.c:653) makes the group's current mesh
 * -- this iteration's new mesh with its interpolated metric and fields, and
 * the frozen points' copies (PMMG_copyMetricsAndFields_point, :792) -- the
 * next interpolation's background.  On the device that mesh already exists:
 * the new points, their tags and the step's results.  Replaces the
 * background upload (pmx_upload_background) of the next iteration when the
 * group was not renumbered in between (no load balancing of this group).
 *
 * pmx_upload_new_tets: the new mesh's tets (tetra_v as in pmx_mesh_view,
 * vertex indices in the last points view's numbering, !MG_EOK entries kept
 * as deleted) -- after pmx_upload_points, once per iteration (they also
 * serve pmx_new_mesh_qual).  A points view with tetra_v uploads them too
 * (packed and sent by the first pmx_run, the orphan marks made from them on
 * the device): no separate call needed then.
 *
 * pmx_promote_background: after a pmx_run on those points, the new points
 * (view first must be 1) become the background vertices 1..np, the step's
 * results its solutions (same list as the step), their tags its point tags.
 * Rows the step did not write (points not located, frozen, NUL, failed
 * interpolations) take the caller's values from sols[], in pmx_download's
 * point-list layout (entry 0 = point 1) -- the arrays pmx_download wrote into.  m: the new mesh --
 * np, ne (= the uploaded new tets), nt / tria_v / adjt / hausd of its
 * boundary trias (host, Mmg numbering), adja (optional: Mmg's mesh->adja,
 * else built on the device); point_c and tetra_v are not read.  Only the
 * trias (and adja when given) cross PCIe.  The new points and results are
 * consumed: upload the next iteration's points before the next pmx_run. */
int pmx_upload_new_tets(pmx_ctx *ctx, const int *tetra_v, int64_t tetra_stride, int64_t ne);
/* on: every points upload with new tets also builds, on a stream of its own
 * and while the step on those points runs, the next background's tet
 * records (face adjacency from the device-resident new tets); the following
 * pmx_promote_background (with m->adja = NULL) only swaps them in.  Off by
 * default: the drop-in path does not promote. */
int pmx_set_residency(pmx_ctx *ctx, int on);
int pmx_promote_background(pmx_ctx *ctx, const pmx_mesh_view *m, int nsol, const pmx_sol_view *sols);

/* Results (one group, or reduced over groups and ranks). */
typedef struct {
  int64_t ne, np;
  double  max, min, avg;       /* alpha*q, avg is the SUM (reference avg_cur) */
  int64_t iel;                 /* element realising min (1-based, in its group) */
  int64_t good, med;
  int64_t his[5];
  int64_t nrid;                /* OUTQUA: tets whose 4 vertices are ridge points */
  int     iel_grp, cpu;        /* group and rank of iel                      */
} pmx_qual_stats;

typedef struct {
  int64_t ned, nullEdge;
  double  avlen, lmin, lmax;   /* avlen is the SUM over edges                */
  int64_t amin, bmin, amax, bmax;
  int64_t hl[9];
  int     cpu_min, cpu_max;
} pmx_len_stats;

/* Point tags of the uploaded background (MMG5_Point.tag through a stride):
 * ridge points for the length loop's filter (src/quality_pmmg.c:509-517) and
 * OUTQUA's nrid.  NULL: no tags.  Kept until the next background upload. */
int pmx_upload_point_tags(pmx_ctx *ctx, const uint16_t *tag, int64_t tag_stride);

/* Quality of every background tet in the uploaded metric
 * (MMG3D_tetraQual(mesh, met, metRidTyp), src/quality_pmmg.c:726).  metRidTyp
 * 0 or 1: identical arithmetic for a size-1 metric (or none); with a size-6
 * metric 1 is MMG5_caltet_ani's ridge-aware mean (needs the point tags,
 * pmx_upload_point_tags: refused without them).  Result stays on the device;
 * qual may be NULL, else it holds qual_cap doubles (>= ne+1). */
int pmx_tetra_qual(pmx_ctx *ctx, int metRidTyp, double *qual, int64_t qual_cap);

/* PMMG_count_nodes_par (src/quality_pmmg.c:33-80) for the uploaded group:
 * the group's points in the internal node communicator (idx_ip[i] -> slot
 * idx_comm[i], nitem_grp entries) count when they claim their slot
 * (intvalues[slot] == 0 -> base; intvalues is the rank's array of nitem
 * slots, in/out, pre-marked by the caller for nodes a higher rank counts,
 * :196-209); every other point counts when a valid tet touches it.  The
 * count is the group's np in the next qualhisto partial. */
int pmx_count_nodes(pmx_ctx *ctx, const int *idx_ip, const int *idx_comm, int64_t nitem_grp,
                    int *intvalues, int64_t nitem, int base, int64_t *np);

/* The per-group part of PMMG_qualhisto (src/quality_pmmg.c:216-261) on the
 * uploaded group: opt PMX_INQUA / PMX_OUTQUA (PMX_LESQUA is refused); use_stored: the qualities of the
 * last pmx_tetra_qual.  Partial written to dev_result (pmx_qual_part, device
 * memory) on the context stream. */
int pmx_qualhisto_device(pmx_ctx *ctx, int opt, int use_stored, void *dev_result);
int pmx_qualhisto(pmx_ctx *ctx, int opt, pmx_qual_stats *st);

/* Parallel (interface) edges of the group for the distributed PMMG_prilen
 * (src/quality_pmmg.c:398-502): edge i joins a[i] -> b[i] (mesh->edge
 * orientation) and is owned by rank owner[i] (the lowest rank sharing it).
 * The owned edges are measured first, in list order, each once; the rank's
 * tet loop then measures every other edge -- the non-owned parallel edges
 * too, as the reference does (its warning at :585-586: interface edges are
 * counted by every rank holding them) unless exact_once is set. */
typedef struct {
  int64_t         n;
  const int      *a, *b, *owner;
  int             myrank;
  int             exact_once;
  /* the edge's tag from the parallel-edge hash (MMG5_hGet(&hpar, a, b, &ref,
   * &tag), :456): its MG_GEO bit is the isedg of MMG5_lenSurfEdg33_ani for a
   * tensor metric (:463).  NULL: 0 */
  const uint16_t *tag;
} pmx_par_edges;

/* Mmg's surface data of the uploaded group, read through strides as Mmg holds
 * it (1-based; pass &mesh->tetra[0].xt, sizeof(MMG5_Tetra);
 * &mesh->xtetra[0].tag[0], sizeof(MMG5_xTetra); &mesh->point[0].n[0] and
 * &mesh->point[0].xp, sizeof(MMG5_Point); &mesh->xpoint[0].n1[0] / .n2[0],
 * sizeof(MMG5_xPoint)).  The edge lengths in a tensor metric need it
 * (src/quality_pmmg.c:463,528,531 -> MMG5_lenedg33_ani / MMG5_lenedg_ani:
 * an edge tagged MG_BDY in its tet's xTetra is measured along the curved
 * surface from the point normals / ridge tangents, MMG5_lenSurfEdg33_ani /
 * MMG5_lenSurfEdg_ani, and with metRidTyp = 1 a ridge point's metric is rebuilt
 * per direction from its two xPoint normals, MMG5_buildridmet).  Never
 * uploaded after the background (or a NULL view): no tet has an xTetra and
 * every normal is 0 -- what Mmg holds for a mesh it never analysed.  Kept
 * until the next background upload; refused (0) if an index is out of range. */
typedef struct {
  int64_t         nxt, nxp;                     /* xTetra / xPoint counts   */
  const int      *tetra_xt;    int64_t tetra_stride;
  const uint16_t *xtetra_tag;  int64_t xtetra_stride;
  const double   *point_n;     const int *point_xp;  int64_t point_stride;
  const double   *xpoint_n1;   const double *xpoint_n2;  int64_t xpoint_stride;
} pmx_surface_view;
int pmx_upload_surface(pmx_ctx *ctx, const pmx_surface_view *sv);

/* PMMG_prilen on the uploaded group: centralized (par == NULL, the
 * MMG3D_computePrilen branch) or distributed (PMMG_computePrilen).  Tets whose
 * 4 vertices are ridge points (pmx_upload_point_tags) are skipped.  metRidTyp
 * (src/quality_pmmg.c:462-466,527-531): 0 or 1 for a size-1 metric (the same
 * lengths); with a size-6 metric 0 = classic storage (MMG5_lenedg33_ani /
 * MMG5_lenSurfEdg33_ani), 1 = Mmg's ridge storage (MMG5_lenedg_ani; the
 * parallel edges, as the reference writes them, MMG5_lenSurfEdg_iso on the
 * metric array read as isotropic: h = met->m[ip]), which needs the point tags
 * (refused without).  Surface edges use pmx_upload_surface's data. */
int pmx_prilen_device(pmx_ctx *ctx, int metRidTyp, const pmx_par_edges *par, void *dev_result);
int pmx_prilen(pmx_ctx *ctx, int metRidTyp, const pmx_par_edges *par, pmx_len_stats *st);

/* PMMG_tetraQual(parmesh, metRidTyp) on the NEW mesh right after the
 * interpolation (src/libparmmg1.c:845, metRidTyp = 1; a size-6 metric
 * takes MMG5_caltet_ani's ridge-aware mean as in pmx_tetra_qual): the new tets (1-based records through a stride,
 * vertex indices in the last points view's numbering) are uploaded as by
 * pmx_upload_new_tets -- or tetra_v = NULL: the ones already uploaded; the
 * coordinates and the interpolated metric are the step's device-resident
 * points and results.  qual (host, qual_cap doubles >= ne+1) and/or
 * dev_result (the qualhisto partial of the new mesh, opt as above; np = the
 * points) may be NULL.  Needs a pmx_run on those points. */
int pmx_new_mesh_qual(pmx_ctx *ctx, const int *tetra_v, int64_t tetra_stride, int64_t ne, int opt,
                      int metRidTyp, double *qual, int64_t qual_cap, void *dev_result);

/* PMMG_tetraQual(parmesh, metRidTyp) on the new mesh of the last step
 * (src/libparmmg1.c:845, right after PMMG_interpMetricsAndFields) in the
 * caller's metric array met (Mmg layout, the points view's numbering; NULL
 * or met->m NULL: no metric): the device already holds the new points, the
 * new tets (the points view must have carried them) and the interpolated
 * metric; only the rows the step did not write -- frozen points the caller
 * filled (PMMG_copyMetricsAndFields_point), failed tensor inversions -- are
 * sent, or the whole array when the step interpolated no metric (-hsiz, Mmg's
 * own metric).  dev_result as in pmx_new_mesh_qual.  qual: the qualities of
 * tets 1..ne through qual_stride bytes -- 0 or 8: a dense array of ne+1
 * doubles, every entry written (deleted tets 0, qual[0] = 0); any larger
 * stride: an AoS field such as &mesh->tetra[0].qual with sizeof(MMG5_Tetra),
 * written for the valid tets only (MMG3D_tetraQual skips !MG_EOK) -- straight
 * from pinned staging, no intermediate array.  qual_cap: the records the
 * array holds (entries 0 .. qual_cap-1; >= ne+1, e.g. mesh->nemax+1). */
int pmx_new_mesh_qual_synced(pmx_ctx *ctx, const pmx_sol_view *met, int opt, int metRidTyp, double *qual,
                             int64_t qual_stride, int64_t qual_cap, void *dev_result);

/* The reduction across groups and ranks (the reference's MPI_Reduce with its
 * custom operators, src/quality_pmmg.c:82-144, :265-307, :661-676), as host
 * folds in (rank, group) order -- deterministic; ties go to the first:
 *   pmx_qual_fold: parts[i] of rank[i] (nondecreasing; NULL = one group per
 *     rank), groups folded as PMMG_qualhisto's loop, then ranks;
 *   pmx_len_fold:  one part per rank, with the reference's operator
 *     (a smaller lmin also takes the other rank's amax/bmax, :125-131). */
int pmx_qual_fold(const pmx_qual_part *parts, const int *rank, int n, pmx_qual_stats *out);
int pmx_len_fold(const pmx_len_part *parts, int n, pmx_len_stats *out);

/* RCCL: one all-gather of the ranks' device partials on the context stream,
 * then the fold.  comm is an ncclComm_t (void *): pmx_comm_unique_id on one
 * rank (broadcast the bytes, e.g. MPI_Bcast on parmesh->comm), pmx_comm_init
 * on every rank. */
int pmx_comm_unique_id(char *id, int len);
int pmx_comm_init(pmx_ctx *ctx, void **comm, int nranks, const char *id, int rank);
int pmx_comm_destroy(void *comm);
/* dev_parts: this rank's ngrp group partials (pmx_qual_part, contiguous in
 * device memory), merged on the host before the all-gather. */
int pmx_qualhisto_allreduce(pmx_ctx *ctx, void *comm, int nranks, const void *dev_parts, int ngrp,
                            pmx_qual_stats *out);
int pmx_prilen_allreduce(pmx_ctx *ctx, void *comm, int nranks, const void *dev_part,
                         pmx_len_stats *out);

#ifdef __cplusplus
}
#endif
#endif
