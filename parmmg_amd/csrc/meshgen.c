/*
 * meshgen.c -- synthetic background/new meshes for the transfer path
 * (test fixtures and bench inputs; NOT part of the product path).
 *
 * Produces the same data the reference's background snapshot holds after
 * PMMG_create_oldGrp (reference src/grpsplit_pmmg.c:207-418):
 *   - points      xyz[3*(np+1)]          1-based, slot 0 unused
 *   - tetrahedra  tet[4*(ne+1)]          1-based, positively oriented (orvol>0)
 *   - adjacency   adja[4*ne+5]           Mmg encoding adja[4*(k-1)+1+f] = 4*k'+f'
 *                                        (reference src/grpsplit_pmmg.c:344-348)
 *   - boundary    tria[3*(nt+1)]         outward faces, vertex order of MMG5_idir
 *   - surface adj adjt[3*nt+4]           adjt[3*(k-1)+1+e] = 3*k'+e'
 *                                        (read at reference src/locate_pmmg.c:539,631)
 *
 * Kuhn (Freudenthal) cube: n^3 cells, 6 tets per cell, ne = 6n^3,
 * np = (n+1)^3, nt = 12n^2 (SURVEY.md section 8 notation).  Jitter is applied
 * to every coordinate that is not on a boundary plane, so the boundary stays
 * exactly planar.  RNG: counter-based splitmix64, reproducible in parallel.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* Cap the OpenMP team (the Python loader passes the process's CPU share: a
 * GPU box's affinity set is 256 CPUs under a 16-CPU cgroup quota, and 256
 * spinning libgomp threads throttled by that quota can stall a parallel
 * region for minutes). */
void pmg_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
#else
  (void)n;
#endif
}

/* face f of a tet is opposite local vertex f; its vertices in MMG5_idir order */
static const int FACEV[4][3] = {{1,2,3},{0,3,2},{0,1,3},{0,2,1}};
/* triangle edge e is opposite local vertex e: (e+1)%3, (e+2)%3 */

static const int PERM[6][3]  = {{0,1,2},{0,2,1},{1,0,2},{1,2,0},{2,0,1},{2,1,0}};
static const int PARITY[6]   = {+1,-1,-1,+1,+1,-1};

static uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
/* uniform in (-1,1) */
static double usym(uint64_t seed, uint64_t ctr) {
  double u = (double)(mix64(seed ^ mix64(ctr)) >> 11) * 0x1.0p-53;
  return 2.0 * u - 1.0;
}

/* corner offsets of local vertex l of Kuhn tet type p */
static void kuhn_corners(int p, int off[4][3]) {
  int c[3] = {0,0,0};
  int l, a;
  for (a = 0; a < 3; a++) off[0][a] = 0;
  for (l = 1; l < 4; l++) {
    c[PERM[p][l-1]] = 1;
    for (a = 0; a < 3; a++) off[l][a] = c[a];
  }
  if (PARITY[p] < 0) {      /* odd permutation: swap local 2,3 -> orvol > 0 */
    int t[3];
    memcpy(t, off[2], sizeof t); memcpy(off[2], off[3], sizeof t); memcpy(off[3], t, sizeof t);
  }
}

/* neighbour table: for tet type p, face f -> cell shift d, type q, face g */
typedef struct { int d[3]; int q, g; } nbr_t;
static nbr_t NBR[6][4];
static int nbr_ready = 0;

static int same_set(int a[3][3], int b[3][3]) {
  int i, j, hit;
  for (i = 0; i < 3; i++) {
    hit = 0;
    for (j = 0; j < 3; j++)
      if (a[i][0]==b[j][0] && a[i][1]==b[j][1] && a[i][2]==b[j][2]) hit = 1;
    if (!hit) return 0;
  }
  return 1;
}

static void build_nbr_table(void) {
  int p, f, q, g, a, i;
  int off[4][3], offq[4][3], F[3][3], G[3][3];
  if (nbr_ready) return;
  for (p = 0; p < 6; p++) {
    kuhn_corners(p, off);
    for (f = 0; f < 4; f++) {
      int d[3] = {0,0,0};
      for (i = 0; i < 3; i++) memcpy(F[i], off[FACEV[f][i]], sizeof F[i]);
      for (a = 0; a < 3; a++) {
        if (F[0][a] == F[1][a] && F[1][a] == F[2][a]) d[a] = F[0][a] ? 1 : -1;
      }
      NBR[p][f].q = -1;
      for (q = 0; q < 6; q++) {
        if (q == p && !d[0] && !d[1] && !d[2]) continue;
        kuhn_corners(q, offq);
        for (g = 0; g < 4; g++) {
          for (i = 0; i < 3; i++)
            for (a = 0; a < 3; a++) G[i][a] = offq[FACEV[g][i]][a] + d[a];
          if (same_set(F, G)) {
            memcpy(NBR[p][f].d, d, sizeof d);
            NBR[p][f].q = q; NBR[p][f].g = g;
          }
        }
      }
    }
  }
  nbr_ready = 1;
}

void pmg_kuhn_counts(int n, int64_t *np, int64_t *ne, int64_t *nt) {
  *np = (int64_t)(n+1)*(n+1)*(n+1);
  *ne = 6LL*n*n*n;
  *nt = 12LL*n*n;
}

/* Build the jittered Kuhn cube.  Returns nt (number of boundary trias), or -1. */
int64_t pmg_kuhn_cube(int n, uint64_t seed, double jitter,
                      double *xyz, int *tet, int *adja, int *tria, int *adjt) {
  const int64_t n1 = n + 1;
  int64_t np, ne, nt;
  int64_t iv, cell, k, nb;
  pmg_kuhn_counts(n, &np, &ne, &nt);
  if (ne >= 0x1FFFFFFF) return -1;     /* 4*ne must fit an int (adja encoding) */
  build_nbr_table();

  xyz[0] = xyz[1] = xyz[2] = 0.0;
#pragma omp parallel for schedule(static)
  for (iv = 0; iv < np; iv++) {
    int64_t ijk[3] = { iv % n1, (iv / n1) % n1, iv / (n1*n1) };
    int a;
    for (a = 0; a < 3; a++) {
      double j = 0.0;
      if (ijk[a] > 0 && ijk[a] < n) j = jitter * usym(seed, (uint64_t)(3*iv + a));
      xyz[3*(iv+1)+a] = ((double)ijk[a] + j) / (double)n;
    }
  }

  tet[0] = tet[1] = tet[2] = tet[3] = 0;
  adja[0] = 0;
#pragma omp parallel for schedule(static)
  for (cell = 0; cell < (int64_t)n*n*n; cell++) {
    int64_t c[3] = { cell % n, (cell / n) % n, cell / ((int64_t)n*n) };
    int p, l, f, off[4][3];
    for (p = 0; p < 6; p++) {
      int64_t kk = 1 + 6*cell + p;
      kuhn_corners(p, off);
      for (l = 0; l < 4; l++) {
        int64_t vi = c[0]+off[l][0], vj = c[1]+off[l][1], vk = c[2]+off[l][2];
        tet[4*kk+l] = (int)(1 + vi + n1*(vj + n1*vk));
      }
      for (f = 0; f < 4; f++) {
        const nbr_t *t = &NBR[p][f];
        int64_t d0 = c[0]+t->d[0], d1 = c[1]+t->d[1], d2 = c[2]+t->d[2];
        int val = 0;
        if (d0 >= 0 && d0 < n && d1 >= 0 && d1 < n && d2 >= 0 && d2 < n) {
          int64_t kn = 1 + 6*(d0 + (int64_t)n*(d1 + (int64_t)n*d2)) + t->q;
          val = (int)(4*kn + t->g);
        }
        adja[4*(kk-1)+1+f] = val;
      }
    }
  }
  adja[4*ne+1] = adja[4*ne+2] = adja[4*ne+3] = adja[4*ne+4] = 0;

  /* boundary triangles, in (tet, face) order */
  nb = 0;
  tria[0] = tria[1] = tria[2] = 0;
  for (k = 1; k <= ne; k++) {
    int f;
    for (f = 0; f < 4; f++) {
      if (adja[4*(k-1)+1+f]) continue;
      nb++;
      tria[3*nb+0] = tet[4*k+FACEV[f][0]];
      tria[3*nb+1] = tet[4*k+FACEV[f][1]];
      tria[3*nb+2] = tet[4*k+FACEV[f][2]];
    }
  }
  if (nb != nt) return -1;
  if (adjt) {
    extern int pmg_build_adjt(int64_t nt, const int *tria, int *adjt);
    if (!pmg_build_adjt(nt, tria, adjt)) return -1;
  }
  return nt;
}

/* ---------------------------------------------------------------------- */
/* generic face matching (any tet mesh), sort based                        */
typedef struct { int a, b, c; int owner; } fkey_t;   /* owner = 4*k+f */

static int cmp_fkey(const void *x, const void *y) {
  const fkey_t *p = (const fkey_t *)x, *q = (const fkey_t *)y;
  if (p->a != q->a) return p->a < q->a ? -1 : 1;
  if (p->b != q->b) return p->b < q->b ? -1 : 1;
  if (p->c != q->c) return p->c < q->c ? -1 : 1;
  return p->owner < q->owner ? -1 : (p->owner > q->owner);
}
static void sort3(int *v) {
  int t;
  if (v[0] > v[1]) { t=v[0]; v[0]=v[1]; v[1]=t; }
  if (v[1] > v[2]) { t=v[1]; v[1]=v[2]; v[2]=t; }
  if (v[0] > v[1]) { t=v[0]; v[0]=v[1]; v[1]=t; }
}

/* adja[4*(k-1)+1+f] = 4*k'+f' or 0.  Returns the number of non-manifold
 * faces found (0 for a valid mesh), or -1 on allocation failure. */
int64_t pmg_build_adja(int64_t ne, const int *tet, int *adja) {
  fkey_t *keys;
  int64_t k, i, nbad = 0;
  keys = (fkey_t *)malloc(sizeof(fkey_t) * (size_t)(4*ne));
  if (!keys) return -1;
  for (k = 1; k <= ne; k++) {
    int f;
    for (f = 0; f < 4; f++) {
      int v[3] = { tet[4*k+FACEV[f][0]], tet[4*k+FACEV[f][1]], tet[4*k+FACEV[f][2]] };
      sort3(v);
      keys[4*(k-1)+f].a = v[0]; keys[4*(k-1)+f].b = v[1]; keys[4*(k-1)+f].c = v[2];
      keys[4*(k-1)+f].owner = (int)(4*k + f);
    }
  }
  qsort(keys, (size_t)(4*ne), sizeof(fkey_t), cmp_fkey);
  memset(adja, 0, sizeof(int) * (size_t)(4*ne+5));
  for (i = 0; i < 4*ne; ) {
    int64_t j = i + 1;
    while (j < 4*ne && keys[j].a == keys[i].a && keys[j].b == keys[i].b && keys[j].c == keys[i].c) j++;
    if (j - i == 2) {
      int o1 = keys[i].owner, o2 = keys[i+1].owner;
      adja[4*(o1/4-1)+1+o1%4] = o2;
      adja[4*(o2/4-1)+1+o2%4] = o1;
    } else if (j - i > 2) {
      nbad++;
    }
    i = j;
  }
  free(keys);
  return nbad;
}

/* Boundary faces in (tet, face) order, vertices in MMG5_idir order. */
int64_t pmg_build_bdry(int64_t ne, const int *tet, const int *adja, int *tria, int64_t maxnt) {
  int64_t k, nb = 0;
  for (k = 1; k <= ne; k++) {
    int f;
    for (f = 0; f < 4; f++) {
      if (adja[4*(k-1)+1+f]) continue;
      nb++;
      if (nb > maxnt) return -1;
      tria[3*nb+0] = tet[4*k+FACEV[f][0]];
      tria[3*nb+1] = tet[4*k+FACEV[f][1]];
      tria[3*nb+2] = tet[4*k+FACEV[f][2]];
    }
  }
  return nb;
}

typedef struct { int a, b; int owner; } ekey_t;       /* owner = 3*k+e */
static int cmp_ekey(const void *x, const void *y) {
  const ekey_t *p = (const ekey_t *)x, *q = (const ekey_t *)y;
  if (p->a != q->a) return p->a < q->a ? -1 : 1;
  if (p->b != q->b) return p->b < q->b ? -1 : 1;
  return p->owner < q->owner ? -1 : (p->owner > q->owner);
}

/* Surface adjacency.  Manifold edges only; an edge with != 2 trias stays 0. */
int pmg_build_adjt(int64_t nt, const int *tria, int *adjt) {
  ekey_t *keys;
  int64_t k, i;
  keys = (ekey_t *)malloc(sizeof(ekey_t) * (size_t)(3*nt + 1));
  if (!keys) return 0;
  for (k = 1; k <= nt; k++) {
    int e;
    for (e = 0; e < 3; e++) {
      int a = tria[3*k + (e+1)%3], b = tria[3*k + (e+2)%3];
      ekey_t *q = &keys[3*(k-1)+e];
      q->a = a < b ? a : b; q->b = a < b ? b : a; q->owner = (int)(3*k+e);
    }
  }
  qsort(keys, (size_t)(3*nt), sizeof(ekey_t), cmp_ekey);
  memset(adjt, 0, sizeof(int) * (size_t)(3*nt+4));
  for (i = 0; i < 3*nt; ) {
    int64_t j = i + 1;
    while (j < 3*nt && keys[j].a == keys[i].a && keys[j].b == keys[i].b) j++;
    if (j - i == 2) {
      int o1 = keys[i].owner, o2 = keys[i+1].owner;
      adjt[3*(o1/3-1)+1+o1%3] = o2;
      adjt[3*(o2/3-1)+1+o2%3] = o1;
    }
    i = j;
  }
  free(keys);
  return 1;
}

/* ---------------------------------------------------------------------- */
/* New vertices: jittered cell centres (volume, tag 0) plus jittered face
 * cell centres on the 6 cube faces (tag MG_BDY=16), Morton ordered.       */
typedef struct { uint64_t key; int64_t idx; } mkey_t;
static int cmp_mkey(const void *x, const void *y) {
  const mkey_t *p = (const mkey_t *)x, *q = (const mkey_t *)y;
  if (p->key != q->key) return p->key < q->key ? -1 : 1;
  return p->idx < q->idx ? -1 : (p->idx > q->idx);
}
static uint64_t spread21(uint64_t v) {
  v &= 0x1fffff;
  v = (v | v << 32) & 0x1f00000000ffffULL;
  v = (v | v << 16) & 0x1f0000ff0000ffULL;
  v = (v | v << 8)  & 0x100f00f00f00f00fULL;
  v = (v | v << 4)  & 0x10c30c30c30c30c3ULL;
  v = (v | v << 2)  & 0x1249249249249249ULL;
  return v;
}
static uint64_t morton3(const double *p) {
  uint64_t q[3];
  int a;
  for (a = 0; a < 3; a++) {
    double t = p[a];
    if (t < 0.0) t = 0.0;
    if (t > 1.0) t = 1.0;
    q[a] = (uint64_t)(t * 2097151.0);
  }
  return spread21(q[0]) | (spread21(q[1]) << 1) | (spread21(q[2]) << 2);
}

int64_t pmg_new_points_count(int n, int with_surface) {
  return (int64_t)n*n*n + (with_surface ? 6LL*n*n : 0);
}

/* xyz[3*count] (0-based list), tag[count]; returns count */
int64_t pmg_new_points(int n, uint64_t seed, double jitter, int with_surface,
                       int morton, double *xyz, int *tag) {
  int64_t nv = (int64_t)n*n*n, ns = with_surface ? 6LL*n*n : 0, cnt = nv + ns, i;
  double *tmp = (double *)malloc(sizeof(double) * (size_t)(3*cnt));
  int *ttmp = (int *)malloc(sizeof(int) * (size_t)cnt);
  mkey_t *keys = NULL;
  if (!tmp || !ttmp) { free(tmp); free(ttmp); return -1; }
#pragma omp parallel for schedule(static)
  for (i = 0; i < nv; i++) {
    int64_t c[3] = { i % n, (i / n) % n, i / ((int64_t)n*n) };
    int a;
    for (a = 0; a < 3; a++)
      tmp[3*i+a] = ((double)c[a] + 0.5 + jitter * usym(seed, (uint64_t)(3*i+a))) / (double)n;
    ttmp[i] = 0;
  }
#pragma omp parallel for schedule(static)
  for (i = 0; i < ns; i++) {
    int64_t face = i / ((int64_t)n*n), r = i % ((int64_t)n*n);
    int axis = (int)(face / 2), side = (int)(face % 2);
    int64_t u = r % n, v = r / n;
    int a1 = (axis+1)%3, a2 = (axis+2)%3;
    double *p = &tmp[3*(nv+i)];
    p[axis] = side ? 1.0 : 0.0;
    p[a1] = ((double)u + 0.5 + jitter * usym(seed ^ 0x5bd1e995ULL, (uint64_t)(2*i)))   / (double)n;
    p[a2] = ((double)v + 0.5 + jitter * usym(seed ^ 0x5bd1e995ULL, (uint64_t)(2*i+1))) / (double)n;
    ttmp[nv+i] = 16;
  }
  if (morton) {
    keys = (mkey_t *)malloc(sizeof(mkey_t) * (size_t)cnt);
    if (!keys) { free(tmp); free(ttmp); return -1; }
#pragma omp parallel for schedule(static)
    for (i = 0; i < cnt; i++) { keys[i].key = morton3(&tmp[3*i]); keys[i].idx = i; }
    qsort(keys, (size_t)cnt, sizeof(mkey_t), cmp_mkey);
#pragma omp parallel for schedule(static)
    for (i = 0; i < cnt; i++) {
      int64_t s = keys[i].idx;
      xyz[3*i] = tmp[3*s]; xyz[3*i+1] = tmp[3*s+1]; xyz[3*i+2] = tmp[3*s+2];
      tag[i] = ttmp[s];
    }
    free(keys);
  } else {
    memcpy(xyz, tmp, sizeof(double) * (size_t)(3*cnt));
    memcpy(tag, ttmp, sizeof(int) * (size_t)cnt);
  }
  free(tmp); free(ttmp);
  return cnt;
}

/* Oriented volume check (6V): the sign only (the generator's own expansion). */
int64_t pmg_count_inverted(int64_t ne, const double *xyz, const int *tet) {
  int64_t k, bad = 0;
#pragma omp parallel for reduction(+:bad)
  for (k = 1; k <= ne; k++) {
    const double *a = &xyz[3*tet[4*k]], *b = &xyz[3*tet[4*k+1]];
    const double *c = &xyz[3*tet[4*k+2]], *d = &xyz[3*tet[4*k+3]];
    double bx = b[0]-a[0], by = b[1]-a[1], bz = b[2]-a[2];
    double cx = c[0]-a[0], cy = c[1]-a[1], cz = c[2]-a[2];
    double dx = d[0]-a[0], dy = d[1]-a[1], dz = d[2]-a[2];
    double v = bx*(cy*dz-cz*dy) + by*(cz*dx-cx*dz) + bz*(cx*dy-cy*dx);
    if (!(v > 0.0)) bad++;
  }
  return bad;
}
