// ASan/UBSan driver of the library's Medit I/O (parmmg_amd/csrc/pmx_medit.hip,
// host code, compiled here with g++): a small mesh and three solutions
// written and read back, ASCII and binary, compared bit for bit.
#include <cstdio>
#include <cstring>
#include <vector>
#include "pmx_transfer.h"

static int check(int ok, const char *what) {
  if (!ok) { fprintf(stderr, "%s: %s\n", what, pmx_medit_last_error()); return 0; }
  return 1;
}

int main(int argc, char **argv) {
  const char *dir = argc > 1 ? argv[1] : ".";
  const int np = 5, ne = 2, nt = 3, nreq = 2;
  std::vector<double> xyz = {0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 1, 0.1, 0.2, 0.3};
  std::vector<int> vref = {0, 1, 2, 3, 4, 5}, tet = {0, 0, 0, 0, 1, 2, 3, 4, 2, 3, 4, 5}, tetref = {0, 7, 8};
  std::vector<int> tria = {0, 0, 0, 1, 2, 3, 1, 2, 4, 2, 3, 5}, triaref = {0, 1, 1, 2}, req = {2, 5};
  std::vector<double> s1(np + 1), s3(3 * (np + 1)), s6(6 * (np + 1));
  for (int i = 0; i < (int)s1.size(); i++) s1[i] = 0.5 + i;
  for (int i = 0; i < (int)s3.size(); i++) s3[i] = 1.0 / (i + 1);
  for (int i = 0; i < (int)s6.size(); i++) s6[i] = 3.0 * i - 1.25;
  const char *ext[2][2] = {{"mesh", "sol"}, {"meshb", "solb"}};
  for (int b = 0; b < 2; b++) {
    char pm[512], ps[512];
    snprintf(pm, sizeof pm, "%s/asan.%s", dir, ext[b][0]);
    snprintf(ps, sizeof ps, "%s/asan.%s", dir, ext[b][1]);
    if (!check(pmx_medit_mesh_write(pm, np, xyz.data(), vref.data(), ne, tet.data(), tetref.data(), nt,
                                    tria.data(), triaref.data(), nreq, req.data()), "mesh write")) return 1;
    pmx_medit_info info;
    if (!check(pmx_medit_mesh_info(pm, &info), "mesh info")) return 1;
    if (info.np != np || info.ne != ne || info.nt != nt || info.nreq != nreq) return 1;
    std::vector<double> x2(3 * (np + 1));
    std::vector<int> v2(np + 1), t2(4 * (ne + 1)), tr2(ne + 1), f2(3 * (nt + 1)), fr2(nt + 1), q2(nreq);
    if (!check(pmx_medit_mesh_read(pm, &info, x2.data(), v2.data(), t2.data(), tr2.data(), f2.data(),
                                   fr2.data(), q2.data()), "mesh read")) return 1;
    if (memcmp(x2.data() + 3, xyz.data() + 3, 3 * np * sizeof(double)) || t2 != tet || q2 != req ||
        memcmp(f2.data() + 3, tria.data() + 3, 3 * nt * sizeof(int)))
      return 1;
    const int types[3] = {1, 2, 3};
    const double *fields[3] = {s1.data(), s3.data(), s6.data()};
    if (!check(pmx_medit_sol_write(ps, np, 3, types, fields), "sol write")) return 1;
    int64_t n2 = 0;
    int ns = 0, ty[8] = {0};
    if (!check(pmx_medit_sol_info(ps, &n2, &ns, ty), "sol info") || n2 != np || ns != 3) return 1;
    std::vector<double> r1(np + 1), r3(3 * (np + 1)), r6(6 * (np + 1));
    double *out[3] = {r1.data(), r3.data(), r6.data()};
    if (!check(pmx_medit_sol_read(ps, n2, ns, ty, out), "sol read")) return 1;
    // arrays sized for a smaller file than the one read: refused, nothing written past them
    pmx_medit_info small = info;
    small.np = np - 2;
    std::vector<double> xs(3 * (small.np + 1));
    if (pmx_medit_mesh_read(pm, &small, xs.data(), nullptr, t2.data(), nullptr, nullptr, nullptr, nullptr))
      return 1;
    std::vector<double> rs(np - 1);
    double *outs[1] = {rs.data()};
    const int t1[1] = {1};
    if (pmx_medit_sol_read(ps, np - 2, 1, t1, outs)) return 1;
    if (memcmp(r1.data() + 1, s1.data() + 1, np * 8) || memcmp(r3.data() + 3, s3.data() + 3, 3 * np * 8) ||
        memcmp(r6.data() + 6, s6.data() + 6, 6 * np * 8))
      return 1;
  }
  {
    // a repeated Vertices block whose first copy is larger than the last one
    // (the counts an info pass would size from): refused without overflow
    char pd[512];
    snprintf(pd, sizeof pd, "%s/dup.mesh", dir);
    FILE *f = fopen(pd, "w");
    if (!f) return 1;
    fprintf(f, "MeshVersionFormatted 2\nDimension 3\nVertices\n6\n");
    for (int k = 0; k < 6; k++) fprintf(f, "%d 0 0 0\n", k);
    fprintf(f, "Vertices\n2\n0 0 0 0\n1 0 0 0\nTetrahedra\n0\nEnd\n");
    fclose(f);
    pmx_medit_info di;
    if (pmx_medit_mesh_info(pd, &di) || !strstr(pmx_medit_last_error(), "duplicate")) return 1;
    di.np = 2; di.ne = 0; di.nt = 0; di.nreq = 0;
    std::vector<double> xd(3 * 3);
    std::vector<int> td(4);
    if (pmx_medit_mesh_read(pd, &di, xd.data(), nullptr, td.data(), nullptr, nullptr, nullptr, nullptr)) return 1;
    // a binary block whose next position points back at itself: refused, no loop
    char pb[512];
    snprintf(pb, sizeof pb, "%s/loop.meshb", dir);
    f = fopen(pb, "wb");
    if (!f) return 1;
    const int32_t hdr[2] = {1, 2}, dimkw[3] = {3, 8, 3};   // Dimension block: next = its own header (8)
    fwrite(hdr, 4, 2, f);
    fwrite(dimkw, 4, 3, f);
    fclose(f);
    if (pmx_medit_mesh_info(pb, &di) || !strstr(pmx_medit_last_error(), "position")) return 1;
  }
  pmx_medit_info none{};
  if (pmx_medit_mesh_read("/nonexistent.mesh", &none, xyz.data(), nullptr, tet.data(), nullptr, nullptr,
                          nullptr, nullptr))
    return 1;
  printf("medit asan ok\n");
  return 0;
}
