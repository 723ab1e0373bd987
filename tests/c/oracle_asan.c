/*
 * oracle_asan.c -- the CPU-side C of the repository (oracle/ restatement and
 * the mesh generator parmmg_amd/csrc/meshgen.c) driven end to end, built
 * with -fsanitize=address,undefined by tests/test_sanitizers.py (SURVEY.md
 * section 5: "the CPU restatement runs under ASan/UBSan").  Test
 * infrastructure only.
 *
 * Kuhn cube, volume + surface points, sequential and device-semantics runs,
 * exhaustive/closest fallbacks (points outside the cube), quality, length
 * statistics with and without point tags.  Checks the linear field is
 * reproduced in the volume and the counts are the analytic ones; every heap
 * block is freed (LeakSanitizer).  Prints "oracle asan ok".
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "pmx_oracle.h"

void pmg_kuhn_counts(int n, int64_t *np, int64_t *ne, int64_t *nt);
int64_t pmg_kuhn_cube(int n, uint64_t seed, double jitter, double *xyz, int *tet, int *adja,
                      int *tria, int *adjt);
int64_t pmg_new_points_count(int n, int with_surface);
int64_t pmg_new_points(int n, uint64_t seed, double jitter, int with_surface, int morton,
                       double *xyz, int *tag);
int64_t pmg_build_adja(int64_t ne, const int *tet, int *adja);

static double lin(const double *x) { return 1.0 + 2.0 * x[0] - 3.0 * x[1] + 0.5 * x[2]; }

int main(void) {
  const int n = 6;
  int64_t np, ne, nt;
  pmg_kuhn_counts(n, &np, &ne, &nt);
  double *xyz = calloc((size_t)(np + 1) * 3, sizeof(double));
  int *tet = calloc((size_t)(ne + 1) * 4, sizeof(int));
  int *adja = calloc((size_t)(4 * ne + 5), sizeof(int));
  int *tria = calloc((size_t)(nt + 1) * 3, sizeof(int));
  int *adjt = calloc((size_t)(3 * nt + 4), sizeof(int));
  if (pmg_kuhn_cube(n, 20250117, 0.15, xyz, tet, adja, tria, adjt) != nt) return 1;
  /* the CPU adjacency builder agrees with the generator's */
  int *adja2 = calloc((size_t)(4 * ne + 5), sizeof(int));
  if (pmg_build_adja(ne, tet, adja2) != 0) return 2;
  for (int64_t i = 1; i <= 4 * ne; i++)
    if (adja[i] != adja2[i]) return 3;

  const int64_t nq = pmg_new_points_count(n, 1) + 40;
  double *q = calloc((size_t)nq * 3, sizeof(double));
  int *tag = calloc((size_t)nq, sizeof(int));
  pmg_new_points(n, 12345, 0.3, 1, 1, q, tag);
  for (int64_t i = nq - 40; i < nq; i++) {      /* outside: exhaustive + closest */
    q[3 * i] = -0.2 + 0.01 * (double)(i % 7);
    q[3 * i + 1] = 1.1;
    q[3 * i + 2] = 0.5;
    tag[i] = 0;
  }
  double *m0 = calloc((size_t)(np + 1), sizeof(double));
  double *m1 = calloc((size_t)(np + 1) * 6, sizeof(double));
  for (int64_t i = 1; i <= np; i++) {
    m0[i] = lin(&xyz[3 * i]);
    m1[6 * i] = m1[6 * i + 3] = m1[6 * i + 5] = 400.0 + 10.0 * xyz[3 * i];
    m1[6 * i + 1] = 1.0;
  }
  const int size[2] = {1, 6};
  const double *old[2] = {m0, m1};
  double *o0 = calloc((size_t)nq, sizeof(double)), *o1 = calloc((size_t)nq * 6, sizeof(double));
  double *out[2] = {o0, o1};
  int *elem = calloc((size_t)nq, sizeof(int)), *status = calloc((size_t)nq, sizeof(int));
  int *steps = calloc((size_t)nq, sizeof(int)), *edge = calloc((size_t)nq, sizeof(int));
  int *vertex = calloc((size_t)nq, sizeof(int));
  orc_ctx *o = orc_create(np, ne, nt, xyz, tet, adja, tria, adjt, 0.01);
  int bad = 0;
  for (int fresh = 0; fresh < 2; fresh++) {
    orc_interp_points(o, nq, q, tag, NULL, 2, size, old, out, 1, NULL, NULL, fresh, elem, status,
                      steps, edge, vertex);
    for (int64_t i = 0; i < nq - 40; i++)
      if (tag[i] == 0 && fabs(o0[i] - lin(&q[3 * i])) > 1e-12) bad++;
    for (int64_t i = nq - 40; i < nq; i++)
      if (status[i] != 0) bad++;
  }
  double *qual = calloc((size_t)(ne + 1), sizeof(double));
  orc_tetra_qual(ne, xyz, tet, m1, 6, qual);
  orc_qualstats qs;
  orc_qualhisto(ne, tet, qual, &qs);
  if (qs.ne != ne || qs.his[0] + qs.his[1] + qs.his[2] + qs.his[3] + qs.his[4] != ne) bad++;
  orc_lenstats ls;
  orc_prilen(np, ne, xyz, tet, m1, 6, &ls);
  const int64_t nedges = 3LL * n * (n + 1) * (n + 1) + 3LL * n * n * (n + 1) + (int64_t)n * n * n;
  if (ls.ned + ls.nullEdge != nedges) bad++;
  orc_destroy(o);
  free(xyz); free(tet); free(adja); free(adja2); free(tria); free(adjt); free(q); free(tag);
  free(m0); free(m1); free(o0); free(o1); free(elem); free(status); free(steps); free(edge);
  free(vertex); free(qual);
  if (bad) { fprintf(stderr, "oracle asan: %d mismatches\n", bad); return 4; }
  printf("oracle asan ok\n");
  return 0;
}
