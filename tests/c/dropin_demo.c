/*
 * dropin_demo.c -- the drop-in seam driven from C, the way ParMmg's host code
 * would call it: Mmg-style AoS point/tetra records read
 * through strided views, one group, PMX_interpMetricsAndFields in place of
 * PMMG_interpMetricsAndFields (reference src/interpmesh_pmmg.c:663-741,
 * caller src/libparmmg1.c:829), no adjacency given (built on the device).
 *
 * Old mesh: Kuhn cube [0,1]^3, n cells per axis, 6 tets per cell.  Old
 * solutions: iso metric h = 0.05 + 0.1 x and a linear vector field; both are
 * reproduced exactly (to rounding) by barycentric interpolation, so every
 * interior new point is checked against the analytic value.  One new point is
 * MG_REQ: the seam must leave its entries untouched (the reference copies
 * them in PMMG_copyMetricsAndFields_point instead).
 *
 * Prints "dropin ok" and exits 0 on success.  Needs a GPU.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pmx_transfer.h"

/* the fields of MMG5_Point / MMG5_Tetra the seam reads, in an AoS record of a
 * different size than ours: the views carry the stride */
typedef struct { double c[3]; double n[3]; int ref, xp, tmp, flag, s; uint16_t tag; int8_t tagdel; } MockPoint;
typedef struct { double qual; int v[4]; int ref, base, mark, xt, flag; int16_t tag; } MockTetra;

static double hfun(const double *x) { return 0.05 + 0.1 * x[0]; }
static void ufun(const double *x, double *u) {
  u[0] = 1.0 + 2.0 * x[0] - 3.0 * x[1] + 0.5 * x[2];
  u[1] = -x[0] + 4.0 * x[2];
  u[2] = 0.25 + x[1];
}

static double orvol(const MockPoint *p, const int *v) {
  const double *a = p[v[0]].c, *b = p[v[1]].c, *c = p[v[2]].c, *d = p[v[3]].c;
  double u[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  double w[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
  double z[3] = {d[0] - a[0], d[1] - a[1], d[2] - a[2]};
  return u[0] * (w[1] * z[2] - w[2] * z[1]) - u[1] * (w[0] * z[2] - w[2] * z[0]) +
         u[2] * (w[0] * z[1] - w[1] * z[0]);
}

int main(void) {
  const int n = 6, n1 = n + 1;
  const int64_t np = (int64_t)n1 * n1 * n1, ne = 6LL * n * n * n;
  MockPoint *pt = calloc((size_t)np + 1, sizeof *pt);
  MockTetra *te = calloc((size_t)ne + 1, sizeof *te);
  double *met = calloc((size_t)np + 1, sizeof(double));
  double *vel = calloc((size_t)(np + 1) * 3, sizeof(double));
#define VID(i, j, k) (1 + (i) + n1 * ((j) + n1 * (k)))
  for (int k = 0; k < n1; k++)
    for (int j = 0; j < n1; j++)
      for (int i = 0; i < n1; i++) {
        MockPoint *p = &pt[VID(i, j, k)];
        p->c[0] = (double)i / n; p->c[1] = (double)j / n; p->c[2] = (double)k / n;
        met[VID(i, j, k)] = hfun(p->c);
        ufun(p->c, vel + 3 * VID(i, j, k));
      }
  /* Kuhn: the 6 monotone paths from corner (0,0,0) to (1,1,1) of each cell */
  static const int perm[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};
  int64_t kt = 1;
  for (int k = 0; k < n; k++)
    for (int j = 0; j < n; j++)
      for (int i = 0; i < n; i++)
        for (int q = 0; q < 6; q++) {
          int c[3] = {i, j, k};
          int *v = te[kt].v;
          v[0] = VID(c[0], c[1], c[2]);
          for (int s = 0; s < 3; s++) {
            c[perm[q][s]]++;
            v[s + 1] = VID(c[0], c[1], c[2]);
          }
          if (orvol(pt, v) < 0.0) { int t = v[2]; v[2] = v[3]; v[3] = t; }
          kt++;
        }

  /* new mesh: interior points (LCG jitter), the last one MG_REQ */
  const int64_t nn = 500;
  MockPoint *npt = calloc((size_t)nn + 1, sizeof *npt);
  double *nmet = calloc((size_t)nn + 1, sizeof(double));
  double *nvel = calloc((size_t)(nn + 1) * 3, sizeof(double));
  uint64_t s = 12345;
  for (int64_t ip = 1; ip <= nn; ip++) {
    for (int a = 0; a < 3; a++) {
      s = s * 6364136223846793005ULL + 1442695040888963407ULL;
      npt[ip].c[a] = 0.05 + 0.9 * (double)(s >> 11) / 9007199254740992.0;
    }
    nmet[ip] = -1.0;   /* sentinels: must be overwritten, except for REQ */
    nvel[3 * ip] = nvel[3 * ip + 1] = nvel[3 * ip + 2] = -1.0;
  }
  npt[nn].tag = PMX_TAG_REQ;

  pmx_ctx *ctx = pmx_create(0);
  if (!ctx) { fprintf(stderr, "pmx_create failed (no GPU?)\n"); return 1; }
  pmx_mesh_view old = {0};
  old.np = np; old.ne = ne; old.nt = 0;
  old.point_c = &pt[0].c[0]; old.point_stride = sizeof(MockPoint);
  old.tetra_v = &te[0].v[0]; old.tetra_stride = sizeof(MockTetra);
  old.adja = NULL;           /* rebuilt on the device (pmx_build_adja) */
  old.hausd = 0.01;
  pmx_sol_view old_met = {1, met}, old_vel = {3, vel};
  pmx_sol_view new_met = {1, nmet}, new_vel = {3, nvel};
  pmx_group g;
  memset(&g, 0, sizeof g);
  g.points.first = 1; g.points.last = nn;
  g.points.c = &npt[0].c[0]; g.points.stride = sizeof(MockPoint);
  g.points.tag = &npt[0].tag; g.points.tag_stride = sizeof(MockPoint);
  g.met = &new_met; g.fields = &new_vel; g.nsols = 1; g.hsiz = 0.0;
  g.old_mesh = old; g.old_met = &old_met; g.old_fields = &old_vel;
  if (!PMX_interpMetricsAndFields(ctx, 1, &g, NULL, 1)) {
    fprintf(stderr, "PMX_interpMetricsAndFields: %s\n", pmx_last_error(ctx));
    return 1;
  }
  int bad = 0;
  for (int64_t ip = 1; ip <= nn; ip++) {
    double u[3];
    ufun(npt[ip].c, u);
    if (ip == nn) {
      bad += nmet[ip] != -1.0 || nvel[3 * ip] != -1.0;
      continue;
    }
    bad += fabs(nmet[ip] - hfun(npt[ip].c)) > 1e-13;
    for (int a = 0; a < 3; a++) bad += fabs(nvel[3 * ip + a] - u[a]) > 1e-12;
  }
  pmx_destroy(ctx);
  if (bad) { fprintf(stderr, "dropin: %d mismatches\n", bad); return 1; }
  printf("dropin ok: %lld new points through PMX_interpMetricsAndFields\n", (long long)nn);
  return 0;
}
