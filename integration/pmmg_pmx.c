/*
 * pmmg_pmx.c -- ParMmg's transfer-path seams, re-implemented over the MI355X
 * C ABI (include/pmx_transfer.h).  Linked into ParMmg in place of
 * src/interpmesh_pmmg.c, src/locate_pmmg.c, src/barycoord_pmmg.c and the five
 * functions below of src/quality_pmmg.c; every definition has
 * the reference's exact signature, return convention and caller:
 *
 *   PMMG_copyMetricsAndFields_point  src/parmmg.h:473   caller src/libparmmg1.c:792
 *   PMMG_interpMetricsAndFields      src/parmmg.h:472   caller src/libparmmg1.c:829
 *   PMMG_tetraQual                   src/parmmg.h:566   caller src/libparmmg1.c:845
 *   PMMG_qualhisto                   src/parmmg.h:564   callers src/libparmmg1.c:910,
 *                                                       src/libparmmg.c:175,318
 *   PMMG_prilen                      src/parmmg.h:565   callers src/libparmmg1.c:964,
 *                                                       src/libparmmg.c:185
 *
 * Compiled by tests/c/adapter_demo.c against a test-local parmmg.h
 * (tests/c/pmmg_stub/) that declares the few fields read here.
 */
#include <float.h>
#include "parmmg.h"
#include "pmx_transfer.h"

/* one device context per MPI rank for the statistics (rank -> device
 * rank % ndev), created by the first seam that needs the device */
static pmx_ctx *PMMG_pmx = NULL;
/* RCCL communicator of the statistics' reduction (nprocs > 1) */
static void *PMMG_pmx_comm = NULL;

/* one context per group for the interpolation, kept across iterations: each
 * group's new points, new tets and interpolated metric stay on the device
 * from PMMG_interpMetricsAndFields (:829) to PMMG_tetraQual (:845), which
 * then sends only the rows the step did not write.  The bookkeeping (a few
 * words per group) is plain heap memory, outside ParMmg's accounting like the
 * device memory itself. */
typedef struct {
  const void *mesh, *point, *tetra;    /* the new mesh the step ran on */
  int         np, ne, valid;
} pmx_grp_state;
static pmx_ctx      **PMMG_pmx_grp = NULL;
static pmx_grp_state *PMMG_pmx_state = NULL;
static int            PMMG_pmx_ngrp = 0;

static pmx_ctx *pmx(PMMG_pParMesh parmesh) {
  if (!PMMG_pmx) PMMG_pmx = pmx_create(parmesh->myrank);
  if (!PMMG_pmx) fprintf(stderr, "  ## Error: no HIP device for the transfer path.\n");
  return PMMG_pmx;
}

/* the group contexts 0..ngrp-1 (created on demand, on the rank's device) */
static pmx_ctx **pmx_groups(PMMG_pParMesh parmesh, int ngrp) {
  int i;
  if (ngrp > PMMG_pmx_ngrp) {
    pmx_ctx **c = (pmx_ctx **)realloc(PMMG_pmx_grp, (size_t)ngrp * sizeof *c);
    pmx_grp_state *st;
    if (!c) return NULL;
    PMMG_pmx_grp = c;
    st = (pmx_grp_state *)realloc(PMMG_pmx_state, (size_t)ngrp * sizeof *st);
    if (!st) return NULL;
    PMMG_pmx_state = st;
    for (i = PMMG_pmx_ngrp; i < ngrp; i++) {
      PMMG_pmx_grp[i] = NULL;
      memset(&PMMG_pmx_state[i], 0, sizeof PMMG_pmx_state[i]);
    }
    PMMG_pmx_ngrp = ngrp;
  }
  for (i = 0; i < ngrp; i++) {
    if (!PMMG_pmx_grp[i]) PMMG_pmx_grp[i] = pmx_create(parmesh->myrank);
    if (!PMMG_pmx_grp[i]) {
      fprintf(stderr, "  ## Error: no HIP device for the transfer path.\n");
      return NULL;
    }
  }
  return PMMG_pmx_grp;
}

/* the RCCL communicator, created once by every rank of parmesh->comm: rank
 * 0's id and its success broadcast together, and every rank's readiness
 * agreed, so that either all ranks enter RCCL's collective initialisation or
 * none does */
static void *pmx_comm(PMMG_pParMesh parmesh, pmx_ctx *ctx) {
  char id[257];
  int ok;
  if (PMMG_pmx_comm) return PMMG_pmx_comm;
  memset(id, 0, sizeof id);
  if (parmesh->myrank == 0) id[0] = (char)(pmx_comm_unique_id(id + 1, 256) > 0);
  MPI_Bcast(id, (int)sizeof id, MPI_BYTE, 0, parmesh->comm);
  ok = id[0] && ctx != NULL;
  MPI_Allreduce(MPI_IN_PLACE, &ok, 1, MPI_INT, MPI_MIN, parmesh->comm);
  if (!ok) return NULL;
  if (!pmx_comm_init(ctx, &PMMG_pmx_comm, parmesh->nprocs, id + 1, parmesh->myrank)) return NULL;
  return PMMG_pmx_comm;
}

static void view_mesh(MMG5_pMesh m, pmx_mesh_view *v) {
  v->np = m->np; v->ne = m->ne; v->nt = m->nt;
  v->point_c = &m->point[0].c[0];  v->point_stride = sizeof(MMG5_Point);
  v->tetra_v = &m->tetra[0].v[0];  v->tetra_stride = sizeof(MMG5_Tetra);
  /* NULL: the device rebuilds the same adjacency by face matching, overlapped
   * with the rest of the upload (16 B/tet less over PCIe) */
  v->adja    = NULL;
  v->tria_v  = m->nt ? &m->tria[0].v[0] : NULL; v->tria_stride = sizeof(MMG5_Tria);
  v->adjt    = m->adjt;
  v->hausd   = m->info.hausd;
}

static void view_sol(MMG5_pSol s, pmx_sol_view *v) { v->size = s->size; v->m = s->m; }

static int pmx_fail(pmx_ctx *ctx, const char *who) {
  fprintf(stderr, "  ## Error: %s: %s\n", who, pmx_last_error(ctx));
  return 0;
}

/* ---- the interpolation seams ---------------------------------------------- */

/* src/interpmesh_pmmg.c:432-446: the frozen (MG_REQ) points' metric and fields
 * copied from the old mesh (through Scotch's permNodGlob when renumbered).  A
 * host loop in the library: works before any context exists (iteration 0
 * calls it before the first interpolation). */
int PMMG_copyMetricsAndFields_point(MMG5_pMesh mesh, MMG5_pMesh oldMesh, MMG5_pSol met,
                                    MMG5_pSol oldMet, MMG5_pSol field, MMG5_pSol oldField,
                                    int *permNodGlob, uint8_t inputMet) {
  pmx_group g;
  pmx_sol_view m, om, fl[PMX_MAX_SOLS], ofl[PMX_MAX_SOLS];
  int j;
  if (mesh->nsols > PMX_MAX_SOLS) {
    fprintf(stderr, "  ## Error: %s: more than %d solution fields.\n", __func__, PMX_MAX_SOLS);
    return 0;
  }
  memset(&g, 0, sizeof g);
  view_mesh(oldMesh, &g.old_mesh);
  if (met) view_sol(met, &m);
  if (oldMet) view_sol(oldMet, &om);
  g.met = met && met->m ? &m : NULL;
  g.old_met = oldMet && oldMet->m ? &om : NULL;
  for (j = 0; j < mesh->nsols; j++) { view_sol(&field[j], &fl[j]); view_sol(&oldField[j], &ofl[j]); }
  g.fields = fl; g.old_fields = ofl; g.nsols = mesh->nsols; g.hsiz = mesh->info.hsiz;
  if (!PMX_copyMetricsAndFields_point(PMMG_pmx, &g, &oldMesh->point[0].tag, sizeof(MMG5_Point),
                                      permNodGlob, oldMesh->info.renum, inputMet))
    return pmx_fail(PMMG_pmx, __func__);
  return 1;
}

/* src/interpmesh_pmmg.c:663-741: every group in one call, each on its own
 * context (group g+1's upload overlaps group g's step); the contexts keep the
 * groups' new meshes and results for PMMG_tetraQual */
int PMMG_interpMetricsAndFields(PMMG_pParMesh parmesh, int *permNodGlob) {
  int ngrp = parmesh->ngrp, igrp, j, ier;
  pmx_group *g;
  pmx_sol_view *sv;
  pmx_ctx **ctxs = pmx_groups(parmesh, ngrp > 0 ? ngrp : 1);
  if (!ctxs) return 0;
  for (igrp = 0; igrp < PMMG_pmx_ngrp; igrp++) PMMG_pmx_state[igrp].valid = 0;
  PMMG_CALLOC(parmesh, g, ngrp, pmx_group, "pmx groups", return 0);
  PMMG_CALLOC(parmesh, sv, ngrp * 2 * (PMX_MAX_SOLS + 1), pmx_sol_view, "pmx sols",
              PMMG_DEL_MEM(parmesh, g, pmx_group, "pmx groups"); return 0);
  for (igrp = 0; igrp < ngrp; igrp++) {
    PMMG_pGrp G = &parmesh->listgrp[igrp], O = &parmesh->old_listgrp[igrp];
    MMG5_pMesh mesh = G->mesh;
    pmx_sol_view *met = sv + igrp * 2 * (PMX_MAX_SOLS + 1), *omet = met + 1,
                 *fl = met + 2, *ofl = fl + PMX_MAX_SOLS;
    if (mesh->nsols > PMX_MAX_SOLS) {
      fprintf(stderr, "  ## Error: %s: more than %d solution fields.\n", __func__, PMX_MAX_SOLS);
      PMMG_DEL_MEM(parmesh, sv, pmx_sol_view, "pmx sols");
      PMMG_DEL_MEM(parmesh, g, pmx_group, "pmx groups");
      return 0;
    }
    /* the new mesh: its points (located) and tets (only the vertices of valid
     * tets are visited, src/interpmesh_pmmg.c:535-541) */
    view_mesh(mesh, &g[igrp].mesh);
    g[igrp].points.first = 1; g[igrp].points.last = mesh->np;
    g[igrp].points.c = &mesh->point[0].c[0];  g[igrp].points.stride = sizeof(MMG5_Point);
    g[igrp].points.tag = &mesh->point[0].tag; g[igrp].points.tag_stride = sizeof(MMG5_Point);
    view_sol(G->met, met); view_sol(O->met, omet);
    g[igrp].met = G->met->m ? met : NULL;  g[igrp].old_met = O->met->m ? omet : NULL;
    for (j = 0; j < mesh->nsols; j++) { view_sol(&G->field[j], &fl[j]); view_sol(&O->field[j], &ofl[j]); }
    g[igrp].fields = fl; g[igrp].old_fields = ofl; g[igrp].nsols = mesh->nsols;
    g[igrp].hsiz = mesh->info.hsiz;
    view_mesh(O->mesh, &g[igrp].old_mesh);
  }
  ier = PMX_interpMetricsAndFields_groups(ctxs, ngrp, g, permNodGlob, parmesh->info.inputMet);
  if (!ier) pmx_fail(ctxs[0], __func__);
  /* resident only where the group's context ran a step: a group with nothing
   * to locate (no metric and no field, or -hsiz and no field, reference
   * :497-512) keeps no new mesh on the device, and its PMMG_tetraQual takes
   * the upload path */
  for (igrp = 0; ier && igrp < ngrp; igrp++) {
    MMG5_pMesh mesh = parmesh->listgrp[igrp].mesh;
    pmx_grp_state *st = &PMMG_pmx_state[igrp];
    st->mesh = mesh; st->point = mesh->point; st->tetra = mesh->tetra;
    st->np = mesh->np; st->ne = mesh->ne; st->valid = pmx_step_ready(ctxs[igrp]);
  }
  PMMG_DEL_MEM(parmesh, sv, pmx_sol_view, "pmx sols");
  PMMG_DEL_MEM(parmesh, g, pmx_group, "pmx groups");
  return ier;
}

/* ---- the statistics seams --------------------------------------------------- */

/* a group's mesh + metric on the device for the statistics: tets, points,
 * metric, point tags and -- for the lengths in a tensor metric, which Mmg
 * measures along the curved surface (MMG5_lenedg33_ani / MMG5_lenedg_ani) --
 * Mmg's xTetra edge tags and point / xPoint normals, read in place */
static int upload_stats_group(pmx_ctx *ctx, MMG5_pMesh mesh, MMG5_pSol met) {
  pmx_mesh_view v;
  pmx_sol_view s;
  pmx_surface_view sv;
  int ns = 0;
  view_mesh(mesh, &v);
  v.nt = 0; v.tria_v = NULL; v.adjt = NULL;
  v.adja = mesh->adja;                       /* Mmg's, when it has one */
  if (met && met->m) { view_sol(met, &s); ns = 1; }
  if (!pmx_upload_background(ctx, &v, ns, &s, ns ? 0 : -1)) return 0;
  if (!pmx_upload_point_tags(ctx, &mesh->point[0].tag, sizeof(MMG5_Point))) return 0;
  if (!(ns && met->size == 6 && (mesh->xtetra || mesh->xpoint))) return 1;
  memset(&sv, 0, sizeof sv);
  if (mesh->xtetra && mesh->xt > 0) {
    sv.nxt = mesh->xt;
    sv.tetra_xt = &mesh->tetra[0].xt;              sv.tetra_stride = sizeof(MMG5_Tetra);
    sv.xtetra_tag = (const uint16_t *)&mesh->xtetra[0].tag[0]; sv.xtetra_stride = sizeof(MMG5_xTetra);
  }
  sv.point_n = &mesh->point[0].n[0];  sv.point_xp = &mesh->point[0].xp;  sv.point_stride = sizeof(MMG5_Point);
  if (mesh->xpoint && mesh->xp > 0) {
    sv.nxp = mesh->xp;
    sv.xpoint_n1 = &mesh->xpoint[0].n1[0];  sv.xpoint_n2 = &mesh->xpoint[0].n2[0];
    sv.xpoint_stride = sizeof(MMG5_xPoint);
  }
  return pmx_upload_surface(ctx, &sv);
}

/* the group's new mesh of the last interpolation is still the one the
 * group holds: ParMmg calls PMMG_tetraQual right after the interpolation
 * (src/libparmmg1.c:829 -> :845), nothing changes the mesh in between */
static int pmx_resident(int igrp, MMG5_pMesh mesh) {
  const pmx_grp_state *st;
  if (igrp >= PMMG_pmx_ngrp) return 0;
  st = &PMMG_pmx_state[igrp];
  return st->valid && st->mesh == (const void *)mesh && st->point == (const void *)mesh->point &&
         st->tetra == (const void *)mesh->tetra && st->np == mesh->np && st->ne == mesh->ne;
}

/* src/quality_pmmg.c:720-733: MMG3D_tetraQual on every group, pt->qual set.
 * After the interpolation the new mesh is on the device already: only the
 * metric rows the step did not write cross PCIe (pmx_new_mesh_qual_synced);
 * any other mesh is uploaded. */
int PMMG_tetraQual(PMMG_pParMesh parmesh, int8_t metRidTyp) {
  int igrp, k, ok;
  double *q = NULL;
  for (igrp = 0; igrp < parmesh->ngrp; igrp++) {
    PMMG_pGrp grp = &parmesh->listgrp[igrp];
    MMG5_pMesh mesh = grp->mesh;
    pmx_ctx *ctx;
    if (pmx_resident(igrp, mesh)) {
      /* the qualities straight into tetra[k].qual (valid tets only) */
      pmx_sol_view mv;
      ctx = PMMG_pmx_grp[igrp];
      PMMG_pmx_state[igrp].valid = 0;            /* one use per interpolation */
      if (grp->met && grp->met->m) view_sol(grp->met, &mv);
      ok = pmx_new_mesh_qual_synced(ctx, grp->met && grp->met->m ? &mv : NULL, PMX_INQUA, metRidTyp,
                                    &mesh->tetra[0].qual, sizeof(MMG5_Tetra), (int64_t)mesh->ne + 1, NULL);
    } else {
      ctx = pmx(parmesh);
      PMMG_MALLOC(parmesh, q, mesh->ne + 1, double, "qual", return 0);
      ok = ctx && upload_stats_group(ctx, mesh, grp->met) &&
           pmx_tetra_qual(ctx, metRidTyp, q, (int64_t)mesh->ne + 1);
      if (ok)
        for (k = 1; k <= mesh->ne; k++)
          if (MG_EOK(&mesh->tetra[k])) mesh->tetra[k].qual = q[k];
      PMMG_DEL_MEM(parmesh, q, double, "qual");
    }
    if (!ok) {
      if (ctx) pmx_fail(ctx, __func__);
      fprintf(stderr, "\n  ## Quality computation problem.\n");
      return 0;
    }
  }
  return 1;
}

/* src/quality_pmmg.c:156-346.  Per group: the device partial (MMG3D_computeInqua
 * / computeOutqua restated; optimLES is refused by the library) and the node
 * count of PMMG_count_nodes_par (:33-80); then the groups folded as the
 * reference's loop and the ranks reduced with its operators (one RCCL
 * all-gather + a rank-ordered fold instead of 12 MPI_Reduce), printed by
 * rank 0 through Mmg's display as the reference does.  Distributed: every
 * rank reaches the agreement on its local result (MPI_Allreduce MIN) whatever
 * failed before it, and all ranks enter the RCCL calls or none does. */
int PMMG_qualhisto(PMMG_pParMesh parmesh, int opt, int isCentral) {
  PMMG_pInt_comm int_node_comm = parmesh->int_node_comm;
  PMMG_pExt_comm ext_node_comm;
  pmx_qual_part *parts = NULL;
  pmx_qual_stats st;
  void *d_parts = NULL;
  int *intvalues = NULL, his[PMMG_QUAL_HISSIZE];
  int i, k, igrp, ier = 1, optimLES;
  const int dist = !isCentral && parmesh->nprocs > 1;
  pmx_ctx *ctx = pmx(parmesh);
  if (!ctx) ier = 0;
  optimLES = (parmesh->ngrp && parmesh->listgrp[0].mesh) ? parmesh->listgrp[0].mesh->info.optimLES : 0;
  /* nodes shared with a higher rank are counted there (:196-209) */
  if (ier && int_node_comm) {
    PMMG_CALLOC(parmesh, int_node_comm->intvalues, int_node_comm->nitem, int, "intvalues", ier = 0);
    intvalues = int_node_comm->intvalues;
    for (k = 0; ier && k < parmesh->next_node_comm; k++) {
      ext_node_comm = &parmesh->ext_node_comm[k];
      if (parmesh->myrank > ext_node_comm->color_out) continue;
      for (i = 0; i < ext_node_comm->nitem; i++) intvalues[ext_node_comm->int_comm_index[i]] = 1;
    }
  }
  if (ier) {
    d_parts = pmx_device_alloc(ctx, (size_t)(parmesh->ngrp > 0 ? parmesh->ngrp : 1) * sizeof(pmx_qual_part));
    if (!d_parts) ier = 0;
  }
  for (igrp = 0; ier && igrp < parmesh->ngrp; igrp++) {
    PMMG_pGrp grp = &parmesh->listgrp[igrp];
    MMG5_pMesh mesh = grp->mesh;
    int64_t np;
    int dopt = mesh->info.optimLES ? PMX_LESQUA : (opt == PMMG_INQUA ? PMX_INQUA : PMX_OUTQUA);
    if (!upload_stats_group(ctx, mesh, grp->met)) { ier = 0; break; }
    if (int_node_comm) {
      mesh->base++;                                /* PMMG_count_nodes_par, :41-42 */
      if (!pmx_count_nodes(ctx, grp->node2int_node_comm_index1, grp->node2int_node_comm_index2,
                           grp->nitem_int_node_comm, intvalues, int_node_comm->nitem, mesh->base, &np)) {
        ier = 0;
        break;
      }
    }
    if (!pmx_qualhisto_device(ctx, dopt, 0, (pmx_qual_part *)d_parts + igrp)) { ier = 0; break; }
  }
  if (!ier && ctx) pmx_fail(ctx, __func__);
  if (parmesh->info.imprim0 > PMMG_VERB_VERSION) {
    if (dist) MPI_Allreduce(MPI_IN_PLACE, &ier, 1, MPI_INT, MPI_MIN, parmesh->comm);
    if (ier && !dist) {
      /* this rank's groups, folded as the reference's group loop */
      PMMG_MALLOC(parmesh, parts, parmesh->ngrp > 0 ? parmesh->ngrp : 1, pmx_qual_part, "parts", ier = 0);
      if (ier && parmesh->ngrp > 0) {
        ier = pmx_synchronize(ctx) &&
              pmx_device_download(ctx, parts, d_parts, sizeof(pmx_qual_part) * (size_t)parmesh->ngrp);
        if (ier) {
          int *rk;
          PMMG_CALLOC(parmesh, rk, parmesh->ngrp, int, "ranks", ier = 0);
          if (ier) {
            ier = pmx_qual_fold(parts, rk, parmesh->ngrp, &st);
            PMMG_DEL_MEM(parmesh, rk, int, "ranks");
          }
        }
      }
      st.cpu = parmesh->myrank;
    } else if (ier) {
      void *comm = pmx_comm(parmesh, ctx);
      ier = comm && pmx_qualhisto_allreduce(ctx, comm, parmesh->nprocs, d_parts, parmesh->ngrp, &st);
    }
    if (ier && parmesh->myrank == 0) {
      if (parmesh->info.imprim > PMMG_VERB_VERSION) {
        fprintf(stdout, "\n  -- PARALLEL MESH QUALITY");
        if (optimLES) fprintf(stdout, " (LES)");
        fprintf(stdout, "  %lld   %lld\n", (long long)st.np, (long long)st.ne);
        fprintf(stdout, "     BEST   %8.6f  AVRG.   %8.6f  WRST.   %8.6f (", st.max,
                st.avg / (double)st.ne, st.min);
        if (parmesh->ngrp > 1) fprintf(stdout, "GROUP %d - ", st.iel_grp);
        if (parmesh->nprocs > 1) fprintf(stdout, "PROC %d - ", st.cpu);
        fprintf(stdout, "ELT %lld)\n", (long long)st.iel);
      }
      for (i = 0; i < PMMG_QUAL_HISSIZE; i++) his[i] = (int)st.his[i];
      ier = MMG3D_displayQualHisto_internal(st.ne, st.max, st.avg, st.min, (int)st.iel, (int)st.good,
                                            (int)st.med, his, (int)st.nrid, optimLES,
                                            parmesh->info.imprim);
    }
    if (!ier && ctx) pmx_fail(ctx, __func__);
  }
  if (parts) PMMG_DEL_MEM(parmesh, parts, pmx_qual_part, "parts");
  if (d_parts) pmx_device_free(ctx, d_parts);
  if (int_node_comm && int_node_comm->intvalues) PMMG_DEL_MEM(parmesh, int_node_comm->intvalues, int, "intvalues");
  return ier;
}

/* src/quality_pmmg.c:370-709 (one group per rank, as the reference requires):
 * centralized = MMG3D_computePrilen, distributed = PMMG_computePrilen with
 * the parallel edges owned by the lowest rank measured first (:398-502); the
 * ranks reduced with PMMG_compute_lenStats' operator (:106-144).  As in the
 * reference, a rank with more than one group fails the call and a rank with no
 * group or no metric takes part with an empty partial (:620-675); the local
 * results are agreed by every rank before the RCCL calls (the reference
 * reduces ier first, :664), so all ranks enter them or none does. */
int PMMG_prilen(PMMG_pParMesh parmesh, int8_t metRidTyp, int isCentral) {
  static double bd[9] = {0.0, 0.3, 0.6, 0.7071, 0.9, 1.3, 1.4142, 2.0, 5.0};
  pmx_len_stats st;
  pmx_par_edges par;
  MMG5_HGeom hpar;
  MMG5_pMesh mesh = NULL;
  MMG5_pSol met = NULL;
  void *d_part = NULL;
  int *pa = NULL, *pb = NULL, *po = NULL, *intvalues, hl[9];
  uint16_t *pt = NULL;
  int i, k, ier = 1, dist = 0, have = 0;
  const int reduce = !isCentral && parmesh->nprocs > 1;
  pmx_ctx *ctx;
  if (parmesh->ngrp > 1) {
    printf("  ## Warning:%s: this function must be called with at most 1"
           "group per processor. Exit function.\n", __func__);
    ier = 0;
  }
  if (ier && parmesh->ngrp == 1) {
    mesh = parmesh->listgrp[0].mesh;
    met = parmesh->listgrp[0].met;
    have = met && met->m;
  }
  if (!reduce && !have) return ier;      /* nothing measured, nothing to reduce */
  ctx = pmx(parmesh);
  if (!ctx) ier = 0;
  memset(&par, 0, sizeof par);
  if (ier && have && !isCentral) {
    /* the parallel edges and their owner (lowest rank holding them, :398-419) */
    PMMG_pInt_comm int_edge_comm;
    PMMG_pGrp grp = &parmesh->listgrp[0];
    memset(&hpar, 0, sizeof hpar);
    if (PMMG_hashPar(mesh, &hpar) != PMMG_SUCCESS) ier = 0;
    if (ier && !PMMG_build_edgeComm(parmesh, mesh, &hpar)) ier = 0;
    if (ier) {
      dist = 1;
      int_edge_comm = parmesh->int_edge_comm;
      PMMG_MALLOC(parmesh, int_edge_comm->intvalues, int_edge_comm->nitem, int, "intvalues", ier = 0);
      intvalues = ier ? int_edge_comm->intvalues : NULL;
      if (ier) {
        for (i = 0; i < int_edge_comm->nitem; i++) intvalues[i] = parmesh->myrank;
        for (k = 0; k < parmesh->next_edge_comm; k++) {
          PMMG_pExt_comm ext = &parmesh->ext_edge_comm[k];
          for (i = 0; i < ext->nitem; i++)
            if (ext->color_out < intvalues[ext->int_comm_index[i]]) intvalues[ext->int_comm_index[i]] = ext->color_out;
        }
        PMMG_MALLOC(parmesh, pa, grp->nitem_int_edge_comm, int, "par a", ier = 0);
        PMMG_MALLOC(parmesh, pb, grp->nitem_int_edge_comm, int, "par b", ier = 0);
        PMMG_MALLOC(parmesh, po, grp->nitem_int_edge_comm, int, "par owner", ier = 0);
        PMMG_MALLOC(parmesh, pt, grp->nitem_int_edge_comm, uint16_t, "par tag", ier = 0);
      }
      if (ier) {
        for (i = 0; i < grp->nitem_int_edge_comm; i++) {
          const int ia = grp->edge2int_edge_comm_index1[i];
          int ref;
          int16_t tag = 0;
          pa[i] = mesh->edge[ia].a;
          pb[i] = mesh->edge[ia].b;
          po[i] = intvalues[grp->edge2int_edge_comm_index2[i]];
          /* :456: an edge missing from the parallel-edge hash is not measured
           * in step 1 (it stays in the edge hash for the tet loop): no owner */
          if (!MMG5_hGet(&hpar, pa[i], pb[i], &ref, &tag)) po[i] = -1;
          pt[i] = (uint16_t)tag;
        }
        par.n = grp->nitem_int_edge_comm;
        par.a = pa; par.b = pb; par.owner = po; par.tag = pt;
        par.myrank = parmesh->myrank;
        par.exact_once = 0;                         /* the reference's counts (:585-586) */
      }
    }
  }
  if (ier && have) ier = upload_stats_group(ctx, mesh, met);
  if (!reduce) {
    if (ier) ier = pmx_prilen(ctx, metRidTyp, dist ? &par : NULL, &st);
    st.cpu_min = st.cpu_max = parmesh->myrank;
  } else {
    if (ier) {
      d_part = pmx_device_alloc(ctx, sizeof(pmx_len_part));
      if (!d_part) ier = 0;
    }
    if (ier && have) ier = pmx_prilen_device(ctx, metRidTyp, &par, d_part);
    if (ier && !have) {
      /* the empty partial of a rank without a metric (:633-640) */
      pmx_len_part e;
      memset(&e, 0, sizeof e);
      e.lmin = DBL_MAX;
      ier = pmx_device_upload(ctx, d_part, &e, sizeof e);
    }
    if (!ier && ctx) pmx_fail(ctx, __func__);
    MPI_Allreduce(MPI_IN_PLACE, &ier, 1, MPI_INT, MPI_MIN, parmesh->comm);
    if (ier) {
      void *comm = pmx_comm(parmesh, ctx);
      ier = comm && pmx_prilen_allreduce(ctx, comm, parmesh->nprocs, d_part, &st);
    }
  }
  if (!ier && ctx) pmx_fail(ctx, __func__);
  if (d_part) pmx_device_free(ctx, d_part);
  if (pa) PMMG_DEL_MEM(parmesh, pa, int, "par a");
  if (pb) PMMG_DEL_MEM(parmesh, pb, int, "par b");
  if (po) PMMG_DEL_MEM(parmesh, po, int, "par owner");
  if (pt) PMMG_DEL_MEM(parmesh, pt, uint16_t, "par tag");
  if (dist) {
    /* the reference's cleanup (:566-571) */
    if (parmesh->int_edge_comm) PMMG_DEL_MEM(parmesh, parmesh->int_edge_comm->intvalues, int, "intvalues");
    PMMG_edge_comm_free(parmesh);
    MMG5_DEL_MEM(mesh, hpar.geom);
    MMG5_DEL_MEM(mesh, mesh->edge);
    mesh->na = 0;
  }
  if (!ier) return 0;
  if (parmesh->myrank == parmesh->info.root) {
    const double avlen = st.avlen / (double)st.ned;
    fprintf(stdout, "\n  -- RESULTING EDGE LENGTHS (ROUGH EVAL.) %d \n", (int)st.ned);
    fprintf(stdout, "     AVERAGE LENGTH         %12.4f\n", avlen);
    fprintf(stdout, "     SMALLEST EDGE LENGTH   %12.4f   %6d %6d", st.lmin, (int)st.amin, (int)st.bmin);
    if (parmesh->nprocs > 1) fprintf(stdout, " (PROC %d)\n", st.cpu_min);
    else fprintf(stdout, "\n");
    fprintf(stdout, "     LARGEST  EDGE LENGTH   %12.4f   %6d %6d", st.lmax, (int)st.amax, (int)st.bmax);
    if (parmesh->nprocs > 1) fprintf(stdout, " (PROC %d)\n", st.cpu_max);
    else fprintf(stdout, "\n");
    for (i = 0; i < 9; i++) hl[i] = (int)st.hl[i];
    MMG5_displayLengthHisto_internal((int)st.ned, (int)st.amin, (int)st.bmin, st.lmin, (int)st.amax,
                                     (int)st.bmax, st.lmax, (int)st.nullEdge, bd, hl, 1,
                                     parmesh->info.imprim);
  }
  return 1;
}
