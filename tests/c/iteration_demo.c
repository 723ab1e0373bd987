/*
 * iteration_demo.c -- two ParMmg iterations driven from C with the background
 * kept on the GPU (INTEGRATION.md "Device residency"), the quality of the new
 * mesh in the interpolated metric and the RCCL statistics reduction (one
 * rank), the way ParMmg's host loop would call them:
 *
 *   iteration 1: background M1 (host upload) -> new mesh M2 (points + tets),
 *                step, fields down, PMMG_tetraQual on M2 (src/libparmmg1.c:845),
 *                PMMG_qualhisto's reduction (src/quality_pmmg.c:275-306);
 *   iteration 2: background = M2 promoted on the device (PMMG_update_oldGrps,
 *                src/libparmmg1.c:653) -> new mesh M3, step, fields down.
 *
 * Check: iteration 2's fields equal, bit for bit, those of a second context
 * that uploads M2 with iteration 1's fields from the host.  Meshes: jittered
 * Kuhn cubes from the repository's generator (parmmg_amd/csrc/meshgen.c).
 * Prints "iteration ok" and exits 0 on success.  Needs a GPU.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pmx_transfer.h"

void pmg_kuhn_counts(int n, int64_t *np, int64_t *ne, int64_t *nt);
int64_t pmg_kuhn_cube(int n, uint64_t seed, double jitter, double *xyz, int *tet, int *adja, int *tria,
                      int *adjt);

typedef struct {
  int64_t np, ne, nt;
  double *xyz;
  int *tet, *adja, *tria, *adjt;
  uint16_t *tag;
} Mesh;

static int kuhn(int n, uint64_t seed, Mesh *m) {
  pmg_kuhn_counts(n, &m->np, &m->ne, &m->nt);
  m->xyz = calloc((size_t)(m->np + 1) * 3, sizeof(double));
  m->tet = calloc((size_t)(m->ne + 1) * 4, sizeof(int));
  m->adja = calloc((size_t)(4 * m->ne + 5), sizeof(int));
  m->tria = calloc((size_t)(m->nt + 1) * 3, sizeof(int));
  m->adjt = calloc((size_t)(3 * m->nt + 4), sizeof(int));
  m->tag = calloc((size_t)(m->np + 1), sizeof(uint16_t));
  if (pmg_kuhn_cube(n, seed, 0.15, m->xyz, m->tet, m->adja, m->tria, m->adjt) != m->nt) return 0;
  for (int64_t i = 1; i <= m->np; i++) {   /* boundary vertices: MG_BDY */
    const double *x = m->xyz + 3 * i;
    for (int a = 0; a < 3; a++)
      if (x[a] == 0.0 || x[a] == 1.0) m->tag[i] = PMX_TAG_BDY;
  }
  return 1;
}

static void view(const Mesh *m, pmx_mesh_view *v) {
  memset(v, 0, sizeof *v);
  v->np = m->np; v->ne = m->ne; v->nt = m->nt;
  v->point_c = m->xyz; v->point_stride = 24;
  v->tetra_v = m->tet; v->tetra_stride = 16;
  v->adja = m->adja;
  v->tria_v = m->tria; v->tria_stride = 12;
  v->adjt = m->adjt;
  v->hausd = 0.01;
}

static void points(const Mesh *m, pmx_points_view *pv) {
  memset(pv, 0, sizeof *pv);
  pv->first = 1; pv->last = m->np;
  pv->c = m->xyz; pv->stride = 24;
  pv->tag = m->tag; pv->tag_stride = 2;
  pv->tetra_v = m->tet; pv->tetra_stride = 16; pv->ne = m->ne;
}

#define CK(x) do { if (!(x)) { fprintf(stderr, "%s: %s\n", #x, pmx_last_error(ctx)); return 1; } } while (0)

int main(void) {
  Mesh m1, m2, m3;
  if (!kuhn(6, 11, &m1) || !kuhn(7, 22, &m2) || !kuhn(5, 33, &m3)) return 1;
  /* background fields: iso size h = 0.05 + 0.1 x, a scalar level set */
  double *h1 = calloc((size_t)m1.np + 1, sizeof(double)), *ls1 = calloc((size_t)m1.np + 1, sizeof(double));
  for (int64_t i = 1; i <= m1.np; i++) {
    const double *x = m1.xyz + 3 * i;
    h1[i] = 0.05 + 0.1 * x[0];
    ls1[i] = sqrt((x[0] - .5) * (x[0] - .5) + (x[1] - .5) * (x[1] - .5) + (x[2] - .5) * (x[2] - .5)) - .3;
  }
  pmx_ctx *ctx = pmx_create(0);
  if (!ctx) { fprintf(stderr, "no device\n"); return 1; }
  CK(pmx_set_residency(ctx, 1));
  pmx_mesh_view v1, v2;
  pmx_points_view p2, p3;
  view(&m1, &v1); view(&m2, &v2);
  points(&m2, &p2); points(&m3, &p3);
  pmx_sol_view old1[2] = {{1, h1}, {1, ls1}};
  /* iteration 1 */
  CK(pmx_upload_background(ctx, &v1, 2, old1, 0));
  CK(pmx_upload_points(ctx, &p2));
  pmx_run_opts o;
  memset(&o, 0, sizeof o);
  CK(pmx_run(ctx, &o));
  double *h2 = calloc((size_t)m2.np + 1, sizeof(double)), *ls2 = calloc((size_t)m2.np + 1, sizeof(double));
  /* pmx_download writes in point-list order: entry 0 = point 1 (Mmg's m[1]) */
  pmx_sol_view new2[2] = {{1, h2 + 1}, {1, ls2 + 1}};
  CK(pmx_download(ctx, new2, m2.np, NULL, NULL, NULL));
  /* quality of the new mesh in the interpolated metric, reduced over the
   * (one-rank) RCCL communicator */
  const int stats = getenv("PMX_DEMO_NO_STATS") == NULL;
  pmx_qual_stats qs;
  memset(&qs, 0, sizeof qs);
  if (stats) {
  char id[256];
  int idlen = pmx_comm_unique_id(id, sizeof id);
  void *comm = NULL;
  if (idlen <= 0) { fprintf(stderr, "pmx_comm_unique_id failed\n"); return 1; }
  CK(pmx_comm_init(ctx, &comm, 1, id, 0));
  void *d = NULL;
  if (!(d = pmx_device_alloc(ctx, sizeof(pmx_qual_part)))) { fprintf(stderr, "%s\n", pmx_last_error(ctx)); return 1; }
  CK(pmx_new_mesh_qual(ctx, NULL, 0, 0, PMX_INQUA, 1, NULL, 0, d));
  CK(pmx_qualhisto_allreduce(ctx, comm, 1, d, 1, &qs));
  if (qs.ne != m2.ne || qs.np != m2.np || qs.min <= 0.0 || qs.max > 1.0 + 1e-12) {
    fprintf(stderr, "new-mesh statistics: ne %lld np %lld min %g max %g\n", (long long)qs.ne,
            (long long)qs.np, qs.min, qs.max);
    return 1;
  }
  pmx_device_free(ctx, d);
  pmx_comm_destroy(comm);
  }
  /* iteration 2: M2 promoted, new mesh M3 */
  CK(pmx_promote_background(ctx, &v2, 2, new2));
  CK(pmx_upload_points(ctx, &p3));
  CK(pmx_run(ctx, &o));
  double *h3 = calloc((size_t)m3.np + 1, sizeof(double)), *ls3 = calloc((size_t)m3.np + 1, sizeof(double));
  pmx_sol_view new3[2] = {{1, h3 + 1}, {1, ls3 + 1}};
  CK(pmx_download(ctx, new3, m3.np, NULL, NULL, NULL));
  /* the same iteration 2 from a host upload of M2 and iteration 1's fields */
  pmx_ctx *ref = pmx_create(0);
  double *h3r = calloc((size_t)m3.np + 1, sizeof(double)), *ls3r = calloc((size_t)m3.np + 1, sizeof(double));
  pmx_sol_view new3r[2] = {{1, h3r + 1}, {1, ls3r + 1}};
  if (!ref || !pmx_upload_background(ref, &v2, 2, (pmx_sol_view[2]){{1, h2}, {1, ls2}}, 0) || !pmx_upload_points(ref, &p3) ||
      !pmx_run(ref, &o) || !pmx_download(ref, new3r, m3.np, NULL, NULL, NULL)) {
    fprintf(stderr, "reference context: %s\n", ref ? pmx_last_error(ref) : "create");
    return 1;
  }
  {
    int64_t nd = 0, nb = 0, first = -1;
    for (int64_t i = 1; i <= m3.np; i++)
      if (memcmp(h3 + i, h3r + i, 8) || memcmp(ls3 + i, ls3r + i, 8)) {
        nd++;
        nb += m3.tag[i] ? 1 : 0;
        if (first < 0) first = i;
      }
    if (nd) {
      fprintf(stderr, "promoted background differs from the host upload: %lld points (%lld surface), "
              "first %lld: h %.17g vs %.17g, ls %.17g vs %.17g\n", (long long)nd, (long long)nb,
              (long long)first, h3[first], h3r[first], ls3[first], ls3r[first]);
      return 1;
    }
  }
  pmx_destroy(ref);
  pmx_destroy(ctx);
  printf("iteration ok: %lld + %lld new points, new-mesh quality min %.4f\n", (long long)m2.np,
         (long long)m3.np, qs.min);
  return 0;
}
