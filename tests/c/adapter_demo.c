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
 * Mode "iterate": two ParMmg iterations.  Iteration 1 as above up to :845;
 * then iteration 2 with TWO groups (a group context each, kept from
 * iteration 1): group 0's background is iteration 1's new mesh with its
 * interpolated metric and field (PMMG_update_oldGrps, :653), its new mesh
 * <dir>/new2_*; group 1 repeats iteration 1's inputs.  Every PMMG_tetraQual
 * (:845) on the device-resident new meshes is followed by a second call that
 * takes the re-upload path (the resident state is used once): both written
 * out (out_q{1,2a,2b}_{res,upl}.bin) for a bit-for-bit comparison.
 *
 * usage: adapter_demo <dir> full|ani|refuse_les|iterate|nolocate|hsiz_nofield|twoproc_prilen|twoproc_qualhisto
 */
#define _POSIX_C_SOURCE 200809L
#include <signal.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>
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
int MMG5_hGet(MMG5_HGeom *hash, int a, int b, int *ref, int16_t *tag) {
  (void)hash; (void)a; (void)b;
  *ref = 0; *tag = 0;
  return 0;
}
int PMMG_build_edgeComm(PMMG_pParMesh parmesh, MMG5_pMesh mesh, MMG5_HGeom *hpar) {
  (void)mesh; (void)hpar;
  memset(&edge_comm, 0, sizeof edge_comm);
  parmesh->int_edge_comm = &edge_comm;
  parmesh->next_edge_comm = 0;
  parmesh->listgrp[0].nitem_int_edge_comm = 0;
  return 1;
}
void PMMG_edge_comm_free(PMMG_pParMesh parmesh) { parmesh->int_edge_comm = NULL; }
/* MPI: never reached with one rank; for the two-process mode a shim over a
 * socketpair (rank 0 = parent, rank 1 = forked child), blocking, in call order */
static int mpi_fd = -1, mpi_rank = 0;
static void xfer(void *out, const void *in, size_t n) {
  /* rank 0 writes then reads, rank 1 reads then writes: no deadlock for n < the socket buffer */
  if (mpi_rank == 0) {
    if (write(mpi_fd, in, n) != (ssize_t)n || read(mpi_fd, out, n) != (ssize_t)n) exit(5);
  } else {
    if (read(mpi_fd, out, n) != (ssize_t)n || write(mpi_fd, in, n) != (ssize_t)n) exit(5);
  }
}
int MPI_Bcast(void *buf, int count, int type, int root, MPI_Comm comm) {
  char tmp[4096];
  (void)type; (void)comm;
  if (mpi_fd < 0) {
    fprintf(stderr, "MPI_Bcast reached with one rank\n");
    exit(3);
  }
  if (count > (int)sizeof tmp) exit(5);
  xfer(tmp, buf, (size_t)count);
  if (mpi_rank != root) memcpy(buf, tmp, (size_t)count);
  printf("{\"mpi\": \"bcast\", \"rank\": %d}\n", mpi_rank);
  return 0;
}
int MPI_Allreduce(const void *sendbuf, void *recvbuf, int count, int type, int op, MPI_Comm comm) {
  int mine[64], other[64], i;
  (void)comm;
  if (mpi_fd < 0) {
    fprintf(stderr, "MPI_Allreduce reached with one rank\n");
    exit(3);
  }
  if (type != MPI_INT || op != MPI_MIN || count > 64) exit(5);
  memcpy(mine, sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf, (size_t)count * sizeof(int));
  xfer(other, mine, (size_t)count * sizeof(int));
  for (i = 0; i < count; i++) ((int *)recvbuf)[i] = mine[i] < other[i] ? mine[i] : other[i];
  printf("{\"mpi\": \"allreduce\", \"rank\": %d, \"value\": %d}\n", mpi_rank, ((int *)recvbuf)[0]);
  fflush(stdout);
  return 0;
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

/* :845 twice: the device-resident new mesh, then the re-upload path */
static int qual_twice(const char *dir, const char *tag, PMMG_pParMesh pm) {
  char name[64];
  int g, k, ier;
  /* the deleted tets keep the -1 (MMG3D_tetraQual skips !MG_EOK) */
  for (g = 0; g < pm->ngrp; g++)
    for (k = 1; k <= pm->listgrp[g].mesh->ne; k++) pm->listgrp[g].mesh->tetra[k].qual = -1.0;
  for (int pass = 0; pass < 2; pass++) {
    ier = PMMG_tetraQual(pm, 1);
    printf("{\"call\": \"tetraqual_%s_%s\", \"ret\": %d}\n", tag, pass ? "upl" : "res", ier);
    if (!ier) return 0;
    for (g = 0; g < pm->ngrp; g++) {
      MMG5_pMesh m = pm->listgrp[g].mesh;
      double *q = calloc((size_t)m->ne + 1, sizeof(double));
      for (k = 1; k <= m->ne; k++) q[k] = m->tetra[k].qual;
      snprintf(name, sizeof name, "out_q%s%c_%s.bin", tag, pm->ngrp > 1 ? 'a' + g : '_', pass ? "upl" : "res");
      wr(dir, name, q, (size_t)(m->ne + 1) * 8);
      for (k = 1; k <= m->ne; k++) m->tetra[k].qual = -1.0;
      free(q);
    }
  }
  return 1;
}

static int iterate(const char *dir, PMMG_pParMesh pm, MMG5_pMesh mesh, MMG5_pMesh old, MMG5_pSol met,
                   MMG5_pSol fld, MMG5_pSol oldmet, MMG5_pSol oldfld, int msize, int fsize) {
  long long np3, ne3;
  char path[1024];
  FILE *f;
  int ier, g;
  int64_t i;
  if (!qual_twice(dir, "1", pm)) return 1;
  /* iteration 2 (:653): iteration 1's new mesh, metric and field become group
   * 0's background (a snapshot copy, as PMMG_update_oldGrps makes) */
  snprintf(path, sizeof path, "%s/sizes2.txt", dir);
  f = fopen(path, "r");
  if (!f || fscanf(f, "%lld %lld", &np3, &ne3) != 2) return 2;
  fclose(f);
  double *xyz1 = calloc((size_t)mesh->np + 1, 24);
  int *tet1 = calloc((size_t)mesh->ne + 1, 16);
  uint16_t *tag1 = calloc((size_t)mesh->np + 1, 2);
  for (i = 1; i <= mesh->np; i++) {
    memcpy(xyz1 + 3 * i, mesh->point[i].c, 24);
    tag1[i] = mesh->point[i].tag;
  }
  for (i = 1; i <= mesh->ne; i++) memcpy(tet1 + 4 * i, mesh->tetra[i].v, 16);
  MMG5_pMesh bg = make_mesh(mesh->np, mesh->ne, xyz1, tet1, tag1);
  {
    pmx_ctx *topo = pmx_create(0);
    int *adja = calloc((size_t)(4 * bg->ne + 5), sizeof(int));
    int *tria = calloc((size_t)(4 * bg->ne + 1) * 3, sizeof(int));
    int *adjt = calloc((size_t)(12 * bg->ne + 4), sizeof(int));
    int64_t nt;
    if (!topo || !pmx_build_adja(topo, bg->ne, bg->np, tet1, 16, adja)) return 4;
    nt = pmx_build_bdry(topo, bg->ne, bg->np, tet1, 16, adja, tria, 4 * bg->ne, adjt);
    if (nt < 0) return 4;
    bg->nt = (int)nt;
    bg->tria = calloc((size_t)nt + 1, sizeof(MMG5_Tria));
    for (i = 1; i <= nt; i++) memcpy(bg->tria[i].v, tria + 3 * i, 3 * sizeof(int));
    bg->adjt = adjt;
    bg->adja = adja;
    free(tria);
    pmx_destroy(topo);
  }
  MMG5_Sol bgmet = {mesh->np, msize, calloc((size_t)(mesh->np + 1) * msize, 8)};
  MMG5_Sol bgfld = {mesh->np, fsize, calloc((size_t)(mesh->np + 1) * fsize, 8)};
  memcpy(bgmet.m, met->m, (size_t)(mesh->np + 1) * msize * 8);
  memcpy(bgfld.m, fld->m, (size_t)(mesh->np + 1) * fsize * 8);
  double *x3 = rd(dir, "new2_xyz.bin", (size_t)(np3 + 1) * 24);
  int *t3 = rd(dir, "new2_tet.bin", (size_t)(ne3 + 1) * 16);
  uint16_t *g3 = rd(dir, "new2_tag.bin", (size_t)(np3 + 1) * 2);
  MMG5_pMesh m3 = make_mesh(np3, ne3, x3, t3, g3);
  m3->nsols = 1;
  MMG5_Sol met3 = {(int)np3, msize, calloc((size_t)(np3 + 1) * msize, 8)};
  MMG5_Sol fld3 = {(int)np3, fsize, calloc((size_t)(np3 + 1) * fsize, 8)};
  for (i = 0; i < (np3 + 1) * msize; i++) met3.m[i] = -7.0;
  for (i = 0; i < (np3 + 1) * fsize; i++) fld3.m[i] = -7.0;
  /* group 1: iteration 1's inputs again, fresh output arrays */
  MMG5_Sol met1 = {mesh->np, msize, calloc((size_t)(mesh->np + 1) * msize, 8)};
  MMG5_Sol fld1 = {mesh->np, fsize, calloc((size_t)(mesh->np + 1) * fsize, 8)};
  for (i = 0; i < (mesh->np + 1) * msize; i++) met1.m[i] = -7.0;
  for (i = 0; i < (mesh->np + 1) * fsize; i++) fld1.m[i] = -7.0;
  PMMG_Grp grps[2], ogrps[2];
  memset(grps, 0, sizeof grps);
  memset(ogrps, 0, sizeof ogrps);
  grps[0].mesh = m3; grps[0].met = &met3; grps[0].field = &fld3;
  ogrps[0].mesh = bg; ogrps[0].met = &bgmet; ogrps[0].field = &bgfld;
  grps[1].mesh = mesh; grps[1].met = &met1; grps[1].field = &fld1;
  ogrps[1].mesh = old; ogrps[1].met = oldmet; ogrps[1].field = oldfld;
  pm->ngrp = 2;
  pm->listgrp = grps;
  pm->old_listgrp = ogrps;
  for (g = 0; g < 2; g++) {
    ier = PMMG_copyMetricsAndFields_point(grps[g].mesh, ogrps[g].mesh, grps[g].met, ogrps[g].met,
                                          grps[g].field, ogrps[g].field, NULL, pm->info.inputMet);
    if (!ier) return 1;
  }
  ier = PMMG_interpMetricsAndFields(pm, NULL);
  printf("{\"call\": \"interp2\", \"ret\": %d}\n", ier);
  if (!ier) return 1;
  wr(dir, "out2_met.bin", met3.m, (size_t)(np3 + 1) * msize * 8);
  wr(dir, "out2_fld.bin", fld3.m, (size_t)(np3 + 1) * fsize * 8);
  wr(dir, "out2b_met.bin", met1.m, (size_t)(mesh->np + 1) * msize * 8);
  wr(dir, "out2b_fld.bin", fld1.m, (size_t)(mesh->np + 1) * fsize * 8);
  wr(dir, "bg2_met.bin", bgmet.m, (size_t)(mesh->np + 1) * msize * 8);
  wr(dir, "bg2_fld.bin", bgfld.m, (size_t)(mesh->np + 1) * fsize * 8);
  if (!qual_twice(dir, "2", pm)) return 1;
  /* more than one group: PMMG_prilen fails as the reference's does (:623-627) */
  ier = PMMG_prilen(pm, 1, 0);
  printf("{\"call\": \"prilen_2grp\", \"ret\": %d}\n", ier);
  printf("{\"adapter\": \"ok\"}\n");
  return 0;
}

/* Mode "twoproc_<case>": two ranks (fork + socketpair MPI shim) on the
 * statistics seams; rank 1 fails locally (<case> = prilen: two groups, the
 * reference's refusal; qualhisto: an upload it cannot do), rank 0 does not.
 * Both must agree on the failure and return 0 without entering a collective
 * the other rank skips (no hang: each rank has a 120 s alarm). */
static int twoproc(const char *dir, const char *which, MMG5_pMesh mesh, MMG5_pSol met, MMG5_pSol fld) {
  int sv[2], ier, status = 0;
  pid_t pid;
  if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) return 6;
  fflush(stdout);
  pid = fork();
  if (pid < 0) return 6;
  mpi_rank = pid == 0 ? 1 : 0;
  mpi_fd = sv[mpi_rank];
  close(sv[1 - mpi_rank]);
  alarm(120);
  {
    PMMG_Grp grps[2];
    PMMG_ParMesh pm;
    memset(grps, 0, sizeof grps);
    memset(&pm, 0, sizeof pm);
    grps[0].mesh = mesh; grps[0].met = met; grps[0].field = fld;
    grps[1] = grps[0];
    pm.myrank = mpi_rank; pm.nprocs = 2; pm.ngrp = 1;
    pm.listgrp = grps; pm.old_listgrp = grps;
    pm.info.imprim = 5; pm.info.imprim0 = 5; pm.info.root = 0; pm.info.inputMet = 1;
    if (!strcmp(which, "prilen")) {
      if (mpi_rank == 1) pm.ngrp = 2;                  /* :623-627: fails on this rank */
      ier = PMMG_prilen(&pm, 0, 0);
    } else {
      MMG5_Mesh bad;
      if (mpi_rank == 1) {                             /* a tet with a vertex past np */
        bad = *mesh;
        bad.tetra = calloc((size_t)mesh->ne + 1, sizeof(MMG5_Tetra));
        memcpy(bad.tetra, mesh->tetra, ((size_t)mesh->ne + 1) * sizeof(MMG5_Tetra));
        bad.tetra[1].v[2] = mesh->np + 5;
        grps[0].mesh = &bad;
      }
      ier = PMMG_qualhisto(&pm, PMMG_INQUA, 0);
    }
    printf("{\"call\": \"%s_rank%d\", \"ret\": %d}\n", which, mpi_rank, ier);
    fflush(stdout);
  }
  (void)dir;
  if (mpi_rank == 1) _exit(0);
  if (waitpid(pid, &status, 0) != pid || !WIFEXITED(status) || WEXITSTATUS(status) != 0) return 7;
  return 0;
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

  if (!strncmp(mode, "twoproc_", 8)) {
    /* before any HIP call: the ranks are forked processes */
    MMG5_pMesh m2 = make_mesh(np2, ne2, nxyz, ntet, ntag);
    MMG5_Sol met2 = {(int)np2, msize, calloc((size_t)(np2 + 1) * msize, 8)};
    MMG5_Sol fld2 = {(int)np2, fsize, calloc((size_t)(np2 + 1) * fsize, 8)};
    for (i = 0; i < (np2 + 1) * msize; i++) met2.m[i] = msize == 1 ? 0.05 : ((i % 6 == 0 || i % 6 == 3 || i % 6 == 5) ? 400.0 : 0.0);
    return twoproc(dir, mode + 8, m2, &met2, &fld2);
  }
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

  if (!strcmp(mode, "nolocate") || !strcmp(mode, "hsiz_nofield")) {
    /* a group whose interpolation has nothing to locate (reference
     * src/interpmesh_pmmg.c:497-512): no input metric and no field, or -hsiz
     * and no field.  Its context runs no step, so :845 must take the upload
     * path (and not fail on a "resident" mesh the device does not hold). */
    double *q = calloc((size_t)ne2 + 1, sizeof(double));
    mesh->nsols = 0;
    if (!strcmp(mode, "nolocate")) pm.info.inputMet = 0;
    else mesh->info.hsiz = 0.05;
    for (i = 0; i < (np2 + 1) * msize; i++) met.m[i] = 0.05;   /* Mmg's own metric */
    ier = PMMG_interpMetricsAndFields(&pm, NULL);
    printf("{\"call\": \"interp\", \"ret\": %d}\n", ier);
    for (i = 1; i <= ne2; i++) mesh->tetra[i].qual = -1.0;
    ier = PMMG_tetraQual(&pm, 1);
    printf("{\"call\": \"tetraqual\", \"ret\": %d}\n", ier);
    for (i = 1; i <= ne2; i++) q[i] = mesh->tetra[i].qual;
    wr(dir, "out_qual.bin", q, (size_t)(ne2 + 1) * 8);
    wr(dir, "out_met.bin", met.m, (size_t)(np2 + 1) * msize * 8);
    free(q);
    return 0;
  }
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
  if (!strcmp(mode, "ani")) {
    /* :845 with an anisotropic metric (Mmg's ridge metric storage): the
     * quality on the device-resident new mesh; then the lengths of :964 with
     * the new mesh's surface data (xTetra edge tags, point / xPoint normals,
     * as MMG3D_analys leaves them; files written by the test) */
    double *q = calloc((size_t)ne2 + 1, sizeof(double));
    long long nxt, nxp;
    ier = PMMG_tetraQual(&pm, 1);
    printf("{\"call\": \"tetraqual_ani_1\", \"ret\": %d}\n", ier);
    for (i = 1; i <= ne2; i++) q[i] = mesh->tetra[i].qual;
    wr(dir, "out_qual_ani1.bin", q, (size_t)(ne2 + 1) * 8);
    snprintf(path, sizeof path, "%s/surf_sizes.txt", dir);
    f = fopen(path, "r");
    if (!f || fscanf(f, "%lld %lld", &nxt, &nxp) != 2) return 2;
    fclose(f);
    {
      int *xt = rd(dir, "new_xt.bin", (size_t)(ne2 + 1) * 4);
      uint16_t *xtag = rd(dir, "new_xtag.bin", (size_t)(nxt + 1) * 12);
      double *pn = rd(dir, "new_pn.bin", (size_t)(np2 + 1) * 24);
      int *xp = rd(dir, "new_xp.bin", (size_t)(np2 + 1) * 4);
      double *n1 = rd(dir, "new_n1.bin", (size_t)(nxp + 1) * 24), *n2 = rd(dir, "new_n2.bin", (size_t)(nxp + 1) * 24);
      mesh->xt = (int)nxt; mesh->xp = (int)nxp;
      mesh->xtetra = calloc((size_t)nxt + 1, sizeof(MMG5_xTetra));
      mesh->xpoint = calloc((size_t)nxp + 1, sizeof(MMG5_xPoint));
      for (i = 1; i <= ne2; i++) mesh->tetra[i].xt = xt[i];
      for (i = 1; i <= nxt; i++) memcpy(mesh->xtetra[i].tag, xtag + 6 * i, 12);
      for (i = 1; i <= np2; i++) { memcpy(mesh->point[i].n, pn + 3 * i, 24); mesh->point[i].xp = xp[i]; }
      for (i = 1; i <= nxp; i++) { memcpy(mesh->xpoint[i].n1, n1 + 3 * i, 24); memcpy(mesh->xpoint[i].n2, n2 + 3 * i, 24); }
    }
    ier = PMMG_prilen(&pm, 1, 0);
    printf("{\"call\": \"prilen_ani_1\", \"ret\": %d}\n", ier);
    ier = PMMG_prilen(&pm, 0, 1);
    printf("{\"call\": \"prilen_ani_0_central\", \"ret\": %d}\n", ier);
    ier = PMMG_tetraQual(&pm, 0);
    printf("{\"call\": \"tetraqual_ani_0\", \"ret\": %d}\n", ier);
    for (i = 1; i <= ne2; i++) q[i] = mesh->tetra[i].qual;
    wr(dir, "out_qual_ani0.bin", q, (size_t)(ne2 + 1) * 8);
    free(q);
    return 0;
  }
  if (!strcmp(mode, "iterate")) return iterate(dir, &pm, mesh, old, &met, &fld, &oldmet, &oldfld, msize, fsize);
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
