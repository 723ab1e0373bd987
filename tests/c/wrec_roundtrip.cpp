// Round trip of the walk's compact tet records (parmmg_amd/csrc/pmx_wrec.h),
// host-only (g++, ASan/UBSan): every valid tet decodes to its record, through
// the packed fields, through a far neighbour field resolved from the full
// record, or through the whole-tet escape; deltas at the field limits,
// boundary faces, deleted tets.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include "pmx_wrec.h"

static int check(const std::vector<TetRec> &tets, long long *nesc, long long *nfar) {
  int bad = 0;
  for (size_t k = 1; k < tets.size(); k++) {
    WRec r;
    wrec_encode(tets[k], (int64_t)k, r);
    if ((r.w[3] >> 28) & WREC_ESC) (*nesc)++;
    const TetRec t = wrec_decode(r, tets.data(), (int)k);
    if (tets[k].v[0] <= 0) {                     // deleted: only the flag matters
      bad += t.v[0] != tets[k].v[0];
      continue;
    }
    for (int i = 0; i < 4; i++) {
      *nfar += t.nb[i] < 0;
      bad += t.nb[i] < 0 && t.nb[i] != -(i + 1);
      bad += (t.v[i] != tets[k].v[i]) + (wrec_resolve(t.nb[i], tets.data(), (int)k) != tets[k].nb[i]);
    }
  }
  return bad;
}

int main() {
  std::mt19937_64 rng(20260117);
  const int n = 1 << 18;
  std::vector<TetRec> tets(n + 1);
  tets[0] = TetRec{{0, 0, 0, 0}, {0, 0, 0, 0}};
  const int edge[] = {0, 1, -1, (1 << 19) - 1, -(1 << 19), 1 << 19, -(1 << 19) - 1};
  const int nedge[] = {0, 1, -1, (1 << 23) - 1, -(1 << 23) + 1, 1 << 23, -(1 << 23)};
  for (int k = 1; k <= n; k++) {
    TetRec &t = tets[k];
    const int mode = (int)(rng() % 8);
    const int v0 = 1 + (int)(rng() % 200000000);
    t.v[0] = mode == 0 ? -(int)(rng() % 5) : v0;  // some deleted tets
    for (int i = 1; i < 4; i++) {
      int d = (int)(rng() % 131072) - 65536;
      if (mode == 1) d = edge[rng() % 7];            // at and past the 20-bit limits
      if (mode == 2) d = (int)(rng() % 2000000) - 1000000;
      long long v = (long long)v0 + d;
      t.v[i] = (int)(v < 1 ? 1 : v);
    }
    for (int f = 0; f < 4; f++) {
      long long d = (long long)(rng() % 800000) - 400000;
      if (mode == 3) d = nedge[rng() % 7];           // at and past the 24-bit limits
      long long nb = (long long)k + d;
      t.nb[f] = (rng() % 6 == 0 || nb < 1 || nb > 2000000000LL) ? 0 : (int)nb;
    }
  }
  long long nesc = 0, nfar = 0;
  const int bad = check(tets, &nesc, &nfar);
  printf("wrec roundtrip: %d tets, %lld escaped, %lld far neighbour fields, %d mismatches\n", n, nesc, nfar,
         bad);
  if (bad || nesc == 0 || nesc == n || nfar == 0) return 1;
  printf("wrec roundtrip ok\n");
  return 0;
}
