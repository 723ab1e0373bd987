/*
 * adapter_demo.c -- ParMmg's own seams, as integration/pmmg_pmx.c defines them
 * (exact reference signatures), driven in the reference's call order of one
 * remesh iteration (src/libparmmg1.c):
 *
 *   :792  PMMG_copyMetricsAndFields_point   (before any device context exists)
 *   :829  PMMG_interpMetricsAndFields
 *   :845  PMMG_tetraQual(parmesh, 1)
 *   :910  PMMG_qualhisto(parmesh, PMMG_OUTQUA, 0)
 *   :964  PMMG_prilen(parmesh, 1, 0)
 * and the input-side calls of src/libparmmg.c:175,185 (centralized).
 *
 * The ParMmg structures come from the test-local tests/c/pmmg_stub/parmmg.h.
 * Inputs: raw arrays in <dir> written by tests/test_capi.py (a background
 * group and a new mesh in Mmg's 1-based layout); the background's boundary
 * trias and their adjacency are built on the device (pmx_build_adja /
 * pmx_build_bdry, the snapshot's MMG5_chkBdryTria + MMG3D_hashTria).
 * Outputs: <dir>/out_{met,fld,qual}.bin and, on stdout, what the adapter
 * handed Mmg's display functions (one JSON object per line).
 *
 * usage: adapter_demo <dir> full|refuse_ani|refuse_les
 */
#include "parmmg.h"
#include "pmx_transfer.h"

static void *rd(const char *dir, const char *name, size_t bytes) {
  char path[1024];
  FILE *f;
  void *p = calloc(bytes ? bytes : 1, 1);
  snprintf(path, sizeof path, "%s/%s", dir, name);
  f = fopen(path, "rb");
  if (!f || fread(p, 1, bytes, f) != bytes) {
    fprintf(stderr, "cannot read %s\n", path);
    exit(2);
  }
  fclose(f);
  return p;
}
static void wr(const char *dir, const char *name, const void *p, size_t bytes) {
  char path[1024];
  FILE *f;
  snprintf(path, sizeof path, "%s/%s", dir, name);
  f = fopen(path, "wb");
  if (!f || fwrite(p, 1, bytes, f) != bytes || fclose(f) != 0) {
    fprintf(stderr, "cannot write %s\n", path);
    exit(2);
  }
}

/* ---- the Mmg / ParMmg helpers the adapter calls (recorded) ---------------- */
int MMG3D_displayQualHisto_internal(int64_t ne, double max, double avg, double min, int iel, int good,
                                    int med, int his[PMMG_QUAL_HISSIZE], int nrid, int optimLES,
                                    int imprim) {
  (void)imprim;
  printf("{\"qualhisto\": {\"ne\": %lld, \"max\": %.17g, \"avg\": %.17g, \"min\": %.17g, \"iel\": %d, "
         "\"good\": %d, \"med\": %d, \"his\": [%d, %d, %d, %d, %d], \"nrid\": %d, \"optimLES\": %d}}\n",
         (long long)ne, max, avg, min, iel, good, med, his[0], his[1], his[2], his[3], his[4], nrid,
         optimLES);
  return 1;
}
int MMG5_displayLengthHisto_internal(int ned, int amin, int bmin, double lmin, int amax, int bmax,
                                     double lmax, int nullEdge, double *bd, int *hl, int8_t shift,
                                     int imprim) {
  (void)bd; (void)shift; (void)imprim;
  printf("{\"prilen\": {\"ned\": %d, \"amin\": %d, \"bmin\": %d, \"lmin\": %.17g, \"amax\": %d, "
         "\"bmax\": %d, \"lmax\": %.17g, \"nullEdge\": %d, \"hl\": [%d, %d, %d, %d, %d, %d, %d, %d, %d]}}\n",
         ned, amin, bmin, lmin, amax, bmax, lmax, nullEdge, hl[0], hl[1], hl[2], hl[3], hl[4], hl[5], hl[6],
         hl[7], hl[8]);
  return 1;
}
/* one rank: no parallel edges */
static PMMG_Int_comm edge_comm;
int PMMG_hashPar(MMG5_pMesh mesh, MMG5_HGeom *pHash) { (void)mesh; pHash->geom = NULL; return PMMG_SUCCESS; }
int PMMG_build_edgeComm(PMMG_pParMesh parmesh, MMG5_pMesh mesh, MMG5_HGeom *hpar) {
  (void)mesh; (void)hpar;
  memset(&edge_comm, 0, sizeof edge_comm);
  parmesh->int_edge_comm = &edge_comm;
  parmesh->next_edge_comm = 0;
  parmesh->listgrp[0].nitem_int_edge_comm = 0;
  return 1;
}
void PMMG_edge_comm_free(PMMG_pParMesh parmesh) { parmesh->int_edge_comm = NULL; }
int MPI_Bcast(void *buf, int count, int type, int root, MPI_Comm comm) {
  (void)buf; (void)count; (void)type; (void)root; (void)comm;
  fprintf(stderr, "MPI_Bcast reached with one rank\n");
  exit(3);
}

/* ---- mesh assembly ----------------------------------------------------------- */
static MMG5_pMesh make_mesh(int64_t np, int64_t ne, const double *xyz, const int *tet, const uint16_t *tag) {
  MMG5_pMesh m = calloc(1, sizeof *m);
  int64_t i;
  m->np = (int)np; m->ne = (int)ne;
  m->point = calloc((size_t)np + 1, sizeof(MMG5_Point));
  m->tetra = calloc((size_t)ne + 1, sizeof(MMG5_Tetra));
  for (i = 1; i <= np; i++) {
    memcpy(m->point[i].c, xyz + 3 * i, 3 * sizeof(double));
    m->point[i].tag = tag[i];
  }
  for (i = 1; i <= ne; i++) memcpy(m->tetra[i].v, tet + 4 * i, 4 * sizeof(int));
  m->info.hausd = 0.01;
  m->info.hsiz = 0.0;
  return m;
}

int main(int argc, char **argv) {
  const char *dir = argc > 1 ? argv[1] : ".";
  const char *mode = argc > 2 ? argv[2] : "full";
  long long np, ne, np2, ne2;
  int msize, fsize, ier;
  int64_t i, nt;
  char path[1024];
  FILE *f;
  snprintf(path, sizeof path, "%s/sizes.txt", dir);
  f = fopen(path, "r");
  if (!f || fscanf(f, "%lld %lld %lld %lld %d %d", &np, &ne, &np2, &ne2, &msize, &fsize) != 6) return 2;
  fclose(f);

  double *oxyz = rd(dir, "old_xyz.bin", (size_t)(np + 1) * 24);
  int *otet = rd(dir, "old_tet.bin", (size_t)(ne + 1) * 16);
  uint16_t *otag = rd(dir, "old_tag.bin", (size_t)(np + 1) * 2);
  double *omet = rd(dir, "old_met.bin", (size_t)(np + 1) * msize * 8);
  double *ofld = rd(dir, "old_fld.bin", (size_t)(np + 1) * fsize * 8);
  double *nxyz = rd(dir, "new_xyz.bin", (size_t)(np2 + 1) * 24);
  int *ntet = rd(dir, "new_tet.bin", (size_t)(ne2 + 1) * 16);
  uint16_t *ntag = rd(dir, "new_tag.bin", (size_t)(np2 + 1) * 2);

  /* the background group: its snapshot's boundary trias + adjacency, built
   * by the device builders (their own context) */
  MMG5_pMesh old = make_mesh(np, ne, oxyz, otet, otag);
  {
    pmx_ctx *topo = pmx_create(0);
    int *adja = calloc((size_t)(4 * ne + 5), sizeof(int));
    int *tria = calloc((size_t)(4 * ne + 1) * 3, sizeof(int));
    int *adjt = calloc((size_t)(12 * ne + 4), sizeof(int));
    if (!topo || !pmx_build_adja(topo, ne, np, otet, 16, adja)) return 4;
    nt = pmx_build_bdry(topo, ne, np, otet, 16, adja, tria, 4 * ne, adjt);
    if (nt < 0) return 4;
    old->nt = (int)nt;
    old->tria = calloc((size_t)nt + 1, sizeof(MMG5_Tria));
    for (i = 1; i <= nt; i++) memcpy(old->tria[i].v, tria + 3 * i, 3 * sizeof(int));
    old->adjt = adjt;
    old->adja = adja;
    free(tria);
    pmx_destroy(topo);
  }
  MMG5_pMesh mesh = make_mesh(np2, ne2, nxyz, ntet, ntag);
  mesh->nsols = 1;
  MMG5_Sol oldmet = {(int)np, msize, omet}, oldfld = {(int)np, fsize, ofld};
  MMG5_Sol met = {(int)np2, msize, calloc((size_t)(np2 + 1) * msize, 8)};
  MMG5_Sol fld = {(int)np2, fsize, calloc((size_t)(np2 + 1) * fsize, 8)};
  for (i = 0; i < (np2 + 1) * msize; i++) met.m[i] = -7.0;
  for (i = 0; i < (np2 + 1) * fsize; i++) fld.m[i] = -7.0;

  PMMG_Grp grp, ogrp;
  memset(&grp, 0, sizeof grp);
  memset(&ogrp, 0, sizeof ogrp);
  grp.mesh = mesh; grp.met = &met; grp.field = &fld;
  ogrp.mesh = old; ogrp.met = &oldmet; ogrp.field = &oldfld;
  PMMG_ParMesh pm;
  memset(&pm, 0, sizeof pm);
  pm.myrank = 0; pm.nprocs = 1; pm.ngrp = 1;
  pm.listgrp = &grp; pm.old_listgrp = &ogrp;
  pm.info.imprim = 5; pm.info.imprim0 = 5; pm.info.root = 0; pm.info.inputMet = 1;

  if (!strcmp(mode, "refuse_les")) {
    mesh->info.optimLES = 1;
    ier = PMMG_qualhisto(&pm, PMMG_INQUA, 1);
    printf("{\"call\": \"qualhisto_les\", \"ret\": %d}\n", ier);
    return 0;
  }
  /* src/libparmmg1.c:792 -- no device context exists yet */
  ier = PMMG_copyMetricsAndFields_point(mesh, old, &met, &oldmet, &fld, &oldfld, NULL, pm.info.inputMet);
  printf("{\"call\": \"copy\", \"ret\": %d}\n", ier);
  if (!ier) return 1;
  /* :829 */
  ier = PMMG_interpMetricsAndFields(&pm, NULL);
  printf("{\"call\": \"interp\", \"ret\": %d}\n", ier);
  if (!ier) return 1;
  wr(dir, "out_met.bin", met.m, (size_t)(np2 + 1) * msize * 8);
  wr(dir, "out_fld.bin", fld.m, (size_t)(np2 + 1) * fsize * 8);
  if (!strcmp(mode, "refuse_ani")) {
    /* :845 with an anisotropic metric: Mmg's ridge metric storage, refused */
    ier = PMMG_tetraQual(&pm, 1);
    printf("{\"call\": \"tetraqual_ani_1\", \"ret\": %d}\n", ier);
    ier = PMMG_prilen(&pm, 1, 0);
    printf("{\"call\": \"prilen_ani_1\", \"ret\": %d}\n", ier);
    ier = PMMG_tetraQual(&pm, 0);
    printf("{\"call\": \"tetraqual_ani_0\", \"ret\": %d}\n", ier);
    return 0;
  }
  /* :845 */
  ier = PMMG_tetraQual(&pm, 1);
  printf("{\"call\": \"tetraqual\", \"ret\": %d}\n", ier);
  if (!ier) return 1;
  {
    double *q = calloc((size_t)ne2 + 1, sizeof(double));
    for (i = 1; i <= ne2; i++) q[i] = mesh->tetra[i].qual;
    wr(dir, "out_qual.bin", q, (size_t)(ne2 + 1) * 8);
    free(q);
  }
  /* :910 */
  ier = PMMG_qualhisto(&pm, PMMG_OUTQUA, 0);
  printf("{\"call\": \"qualhisto_out\", \"ret\": %d}\n", ier);
  if (!ier) return 1;
  /* :964 */
  ier = PMMG_prilen(&pm, 1, 0);
  printf("{\"call\": \"prilen_1_dist\", \"ret\": %d}\n", ier);
  if (!ier) return 1;
  /* src/libparmmg.c:175,185 (centralized input) */
  ier = PMMG_qualhisto(&pm, PMMG_INQUA, 1);
  printf("{\"call\": \"qualhisto_in\", \"ret\": %d}\n", ier);
  if (!ier) return 1;
  ier = PMMG_prilen(&pm, 0, 1);
  printf("{\"call\": \"prilen_0_central\", \"ret\": %d}\n", ier);
  if (!ier) return 1;
  printf("{\"adapter\": \"ok\"}\n");
  return 0;
}
