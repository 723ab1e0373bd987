// pmx_medit.hip -- Medit mesh / solution files in the C library (host code).
//
// the wire format of the transfer path's inputs and
// outputs.  ParMmg reads and writes them through Mmg (src/inout_pmmg.c:440-991
// -> MMG3D_loadMesh / MMG3D_saveMesh / MMG3D_loadSol / MMG3D_saveSol); the
// formats are restated here from the public Medit / libMeshb descriptions:
//
//   .mesh / .sol   ASCII: keywords by name, counts, records; unknown keywords
//                  are skipped (tokens up to the next alphabetic one).
//   .meshb / .solb binary: int32 1 (endianness), int32 version; then keyword
//                  blocks: int32 code, the absolute position of the next
//                  block (int32 for version <= 2, int64 from 3), a count for
//                  the keywords that carry one (int32 up to version 3, int64
//                  at 4), records.  Reals are float32 at version 1, float64
//                  from 2; integers int64 at version 4.  Codes: Dimension 3,
//                  Vertices 4, Triangles 6, Tetrahedra 8, RequiredVertices 15,
//                  End 54, SolAtVertices 62 (+ int32 ntypes, int32 types).
//
// Arrays are Mmg's (1-based, slot 0 untouched): xyz[3*(np+1)], refs[n+1],
// tet[4*(ne+1)], tria[3*(nt+1)], solutions [size*(np+1)] with Mmg's tensor
// order (11,12,13,22,23,33); files hold Medit's (11,12,22,13,23,33).
// Binary parity is unpinned (the reference holds no binary file); the ASCII
// reader is checked against the reference's own libexamples meshes.
#include <algorithm>
#include <cctype>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "pmx_transfer.h"

namespace {

thread_local std::string g_err;

int fail(const std::string &what) {
  g_err = what;
  return 0;
}

enum : int { KW_DIM = 3, KW_VERT = 4, KW_TRI = 6, KW_TET = 8, KW_REQV = 15, KW_END = 54, KW_SOLV = 62 };

bool ends_with(const std::string &s, const char *suf) {
  const size_t n = strlen(suf);
  return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}
bool is_binary(const char *path) {
  const std::string p(path);
  return ends_with(p, ".meshb") || ends_with(p, ".solb");
}

// ---- ASCII ---------------------------------------------------------------------

struct Text {
  std::vector<char> buf;
  size_t i = 0;
  bool load(const char *path) {
    FILE *f = fopen(path, "rb");
    if (!f) return false;
    fseek(f, 0, SEEK_END);
    const long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    buf.resize((size_t)std::max(n, 0L) + 1);
    const size_t got = n > 0 ? fread(buf.data(), 1, (size_t)n, f) : 0;
    fclose(f);
    buf[got] = 0;
    buf.resize(got + 1);
    return true;
  }
  void skip_ws() {
    for (;;) {
      while (buf[i] && isspace((unsigned char)buf[i])) i++;
      if (buf[i] == '#') {                       // comment line
        while (buf[i] && buf[i] != '\n') i++;
        continue;
      }
      return;
    }
  }
  bool at_end() {
    skip_ws();
    return !buf[i];
  }
  bool next_is_word() {
    skip_ws();
    return isalpha((unsigned char)buf[i]);
  }
  std::string word() {
    skip_ws();
    const size_t s = i;
    while (buf[i] && !isspace((unsigned char)buf[i])) i++;
    return std::string(buf.data() + s, i - s);
  }
  bool integer(int64_t &v) {
    skip_ws();
    char *e = nullptr;
    v = strtoll(buf.data() + i, &e, 10);
    if (e == buf.data() + i) return false;
    i = (size_t)(e - buf.data());
    return true;
  }
  bool real(double &v) {
    skip_ws();
    char *e = nullptr;
    v = strtod(buf.data() + i, &e);
    if (e == buf.data() + i) return false;
    i = (size_t)(e - buf.data());
    return true;
  }
  void skip_block() {                            // an unknown keyword's data
    while (!at_end() && !next_is_word()) word();
  }
};

// ---- binary --------------------------------------------------------------------

struct Bin {
  FILE *f = nullptr;
  int ver = 0;
  long size = 0;
  ~Bin() {
    if (f) fclose(f);
  }
  bool open(const char *path) {
    f = fopen(path, "rb");
    if (!f) return false;
    if (fseek(f, 0, SEEK_END) != 0 || (size = ftell(f)) < 8 || fseek(f, 0, SEEK_SET) != 0) return false;
    int32_t code = 0, v = 0;
    if (fread(&code, 4, 1, f) != 1 || fread(&v, 4, 1, f) != 1) return false;
    if (code != 1) return false;                 // other endianness: not supported
    ver = v;
    return ver >= 1 && ver <= 4;
  }
  bool i32(int32_t &x) { return fread(&x, 4, 1, f) == 1; }
  bool pos(int64_t &p) {
    if (ver >= 3) return fread(&p, 8, 1, f) == 1;
    int32_t q;
    if (fread(&q, 4, 1, f) != 1) return false;
    p = q;
    return true;
  }
  bool count(int64_t &n) {
    if (ver == 4) return fread(&n, 8, 1, f) == 1;
    int32_t q;
    if (fread(&q, 4, 1, f) != 1) return false;
    n = q;
    return true;
  }
  bool integer(int64_t &x) {
    if (ver == 4) return fread(&x, 8, 1, f) == 1;
    int32_t q;
    if (fread(&q, 4, 1, f) != 1) return false;
    x = q;
    return true;
  }
  bool real(double &x) {
    if (ver == 1) {
      float q;
      if (fread(&q, 4, 1, f) != 1) return false;
      x = q;
      return true;
    }
    return fread(&x, 8, 1, f) == 1;
  }
  // the next block's absolute position must move forward and stay in the
  // file (a malformed position would loop or re-read blocks)
  bool next_ok(int64_t next, long at) const { return next <= 0 || (next > at && next <= size); }
};

struct BinOut {
  FILE *f = nullptr;
  int ver = 0;
  ~BinOut() {
    if (f) fclose(f);
  }
  // flush and close, reporting buffered data that could not be written
  bool close() {
    const bool good = fflush(f) == 0 && !ferror(f);
    const bool closed = fclose(f) == 0;
    f = nullptr;
    return good && closed;
  }
  void i32(int32_t x) { fwrite(&x, 4, 1, f); }
  void integer(int64_t x) {
    if (ver == 4) fwrite(&x, 8, 1, f);
    else i32((int32_t)x);
  }
  void real(double x) { fwrite(&x, 8, 1, f); }
  // keyword header; the next-block position is patched when the block ends
  long begin(int kw, bool with_count, int64_t n) {
    i32(kw);
    const long at = ftell(f);
    if (ver >= 3) { int64_t z = 0; fwrite(&z, 8, 1, f); }
    else i32(0);
    if (with_count) {
      if (ver == 4) fwrite(&n, 8, 1, f);
      else i32((int32_t)n);
    }
    return at;
  }
  void end(long at) {
    const long here = ftell(f);
    fseek(f, at, SEEK_SET);
    if (ver >= 3) { int64_t p = here; fwrite(&p, 8, 1, f); }
    else { int32_t p = (int32_t)here; fwrite(&p, 4, 1, f); }
    fseek(f, here, SEEK_SET);
  }
};

// Medit (11,12,22,13,23,33) <-> Mmg (11,12,13,22,23,33): positions 2 and 3
inline int tensor_perm(int j) { return j == 2 ? 3 : j == 3 ? 2 : j; }
inline int type_size(int t) { return t == 1 ? 1 : t == 2 ? 3 : t == 3 ? 6 : 0; }

// the common reader: sizes only (out == nullptr) or the data
struct MeshOut {
  double *xyz;
  int *vref, *tet, *tetref, *tria, *triaref, *req;
};

// a keyword block's count: each keyword at most once, and in the read pass
// the count the caller's arrays were sized from (pmx_medit_mesh_info)
bool block_count(const char *kw, int64_t n, int64_t *slot, bool *seen, const pmx_medit_info *expect,
                 int64_t expected) {
  if (*seen) return fail(std::string("duplicate ") + kw + " block");
  *seen = true;
  *slot = n;
  if (expect && n != expected)
    return fail(std::string(kw) + " count differs from the one the arrays were sized for");
  return true;
}

int read_mesh(const char *path, pmx_medit_info *info, const MeshOut *out, const pmx_medit_info *expect) {
  pmx_medit_info I{};
  I.dim = 3;
  bool seen[4] = {false, false, false, false};
  auto count_of = [&](const char *name, int64_t n) -> bool {
    const std::string k(name);
    if (k == "Vertices") return block_count(name, n, &I.np, &seen[0], expect, expect ? expect->np : 0);
    if (k == "Tetrahedra") return block_count(name, n, &I.ne, &seen[1], expect, expect ? expect->ne : 0);
    if (k == "Triangles") return block_count(name, n, &I.nt, &seen[2], expect, expect ? expect->nt : 0);
    return block_count(name, n, &I.nreq, &seen[3], expect, expect ? expect->nreq : 0);
  };
  if (is_binary(path)) {
    Bin b;
    if (!b.open(path)) return fail(std::string("cannot open or not a native-endian .meshb: ") + path);
    I.version = b.ver;
    for (;;) {
      int32_t kw;
      int64_t next;
      const long at = ftell(b.f);
      if (!b.i32(kw) || !b.pos(next)) return fail("truncated .meshb");
      if (!b.next_ok(next, at)) return fail("bad .meshb block position");
      if (kw == KW_END) break;
      if (kw == KW_DIM) {
        int32_t d;
        if (!b.i32(d)) return fail("truncated .meshb");
        I.dim = d;
        if (d != 3) return fail("only 3-D meshes");
      } else if (kw == KW_VERT || kw == KW_TET || kw == KW_TRI || kw == KW_REQV) {
        int64_t n;
        if (!b.count(n) || n < 0) return fail("bad .meshb count");
        if (!count_of(kw == KW_VERT ? "Vertices" : kw == KW_TET ? "Tetrahedra" : kw == KW_TRI ? "Triangles"
                                                                                   : "RequiredVertices", n))
          return 0;
        if (out) {
          for (int64_t k = 1; k <= n; k++) {
            int64_t x, ref = 0;
            if (kw == KW_VERT) {
              for (int a = 0; a < 3; a++) {
                double c;
                if (!b.real(c)) return fail("truncated Vertices");
                out->xyz[3 * k + a] = c;
              }
              if (!b.integer(ref)) return fail("truncated Vertices");
              if (out->vref) out->vref[k] = (int)ref;
            } else if (kw == KW_TET || kw == KW_TRI) {
              const int nv = kw == KW_TET ? 4 : 3;
              int *dst = kw == KW_TET ? out->tet : out->tria;
              for (int a = 0; a < nv; a++) {
                if (!b.integer(x)) return fail("truncated elements");
                if (dst) dst[nv * k + a] = (int)x;
              }
              if (!b.integer(ref)) return fail("truncated elements");
              int *r = kw == KW_TET ? out->tetref : out->triaref;
              if (r) r[k] = (int)ref;
            } else {
              if (!b.integer(x)) return fail("truncated RequiredVertices");
              if (out->req) out->req[k - 1] = (int)x;
            }
          }
        }
      }
      if (next <= 0) break;
      if (fseek(b.f, (long)next, SEEK_SET) != 0) return fail("bad .meshb block position");
    }
  } else {
    Text t;
    if (!t.load(path)) return fail(std::string("cannot open ") + path);
    I.version = 1;
    while (!t.at_end()) {
      if (!t.next_is_word()) { t.word(); continue; }
      const std::string kw = t.word();
      int64_t n = 0;
      if (kw == "End") break;
      if (kw == "MeshVersionFormatted") {
        if (!t.integer(n)) return fail("bad MeshVersionFormatted");
        I.version = (int)n;
      } else if (kw == "Dimension") {
        if (!t.integer(n)) return fail("bad Dimension");
        I.dim = (int)n;
        if (n != 3) return fail("only 3-D meshes");
      } else if (kw == "Vertices" || kw == "Tetrahedra" || kw == "Triangles" || kw == "RequiredVertices") {
        if (!t.integer(n) || n < 0) return fail("bad count after " + kw);
        const int nv = kw == "Vertices" ? 0 : kw == "Tetrahedra" ? 4 : kw == "Triangles" ? 3 : 1;
        if (!count_of(kw.c_str(), n)) return 0;
        for (int64_t k = 1; k <= n; k++) {
          int64_t x, ref = 0;
          if (nv == 0) {
            for (int a = 0; a < 3; a++) {
              double c;
              if (!t.real(c)) return fail("truncated Vertices");
              if (out) out->xyz[3 * k + a] = c;
            }
            if (!t.integer(ref)) return fail("truncated Vertices");
            if (out && out->vref) out->vref[k] = (int)ref;
          } else if (nv == 1) {
            if (!t.integer(x)) return fail("truncated RequiredVertices");
            if (out && out->req) out->req[k - 1] = (int)x;
          } else {
            int *dst = out ? (nv == 4 ? out->tet : out->tria) : nullptr;
            for (int a = 0; a < nv; a++) {
              if (!t.integer(x)) return fail("truncated " + kw);
              if (dst) dst[nv * k + a] = (int)x;
            }
            if (!t.integer(ref)) return fail("truncated " + kw);
            int *r = out ? (nv == 4 ? out->tetref : out->triaref) : nullptr;
            if (r) r[k] = (int)ref;
          }
        }
      } else {
        t.skip_block();
      }
    }
  }
  // a block the arrays were sized for that the file no longer holds
  if (expect && (I.np != expect->np || I.ne != expect->ne || I.nt != expect->nt || I.nreq != expect->nreq))
    return fail("mesh counts differ from the ones the arrays were sized for");
  if (info) *info = I;
  return 1;
}

struct SolIn {
  int64_t np = 0;
  int nsol = 0, types[PMX_MAX_SOLS] = {0}, version = 0;
};

// the read pass: the header must be the one the fields were sized for
bool sol_header_ok(const SolIn &S, const SolIn *expect) {
  if (!expect) return true;
  bool same = S.np == expect->np && S.nsol == expect->nsol;
  for (int s = 0; same && s < S.nsol; s++) same = S.types[s] == expect->types[s];
  return same ? true : fail("SolAtVertices header differs from the one the fields were sized for");
}

int read_sol(const char *path, SolIn &S, double **fields, const SolIn *expect) {
  auto store = [&](int64_t k, int s, int j, double v) {
    const int sz = type_size(S.types[s]);
    const int jj = sz == 6 ? tensor_perm(j) : j;
    if (fields && fields[s]) fields[s][k * sz + jj] = v;
  };
  if (is_binary(path)) {
    Bin b;
    if (!b.open(path)) return fail(std::string("cannot open or not a native-endian .solb: ") + path);
    S.version = b.ver;
    bool found = false;
    for (;;) {
      int32_t kw;
      int64_t next;
      const long at = ftell(b.f);
      if (!b.i32(kw) || !b.pos(next)) return fail("truncated .solb");
      if (!b.next_ok(next, at)) return fail("bad .solb block position");
      if (kw == KW_END) break;
      if (kw == KW_DIM) {
        int32_t d;
        if (!b.i32(d) || d != 3) return fail("only 3-D solutions");
      } else if (kw == KW_SOLV) {
        if (found) return fail("duplicate SolAtVertices block");
        int64_t n;
        int32_t nt;
        if (!b.count(n) || !b.i32(nt) || nt < 1 || nt > PMX_MAX_SOLS) return fail("bad SolAtVertices header");
        S.np = n;
        S.nsol = nt;
        for (int s = 0; s < nt; s++) {
          int32_t ty;
          if (!b.i32(ty) || !type_size(ty)) return fail("unsupported solution type");
          S.types[s] = ty;
        }
        found = true;
        if (!sol_header_ok(S, expect)) return 0;
        if (fields) {
          for (int64_t k = 1; k <= n; k++)
            for (int s = 0; s < nt; s++)
              for (int j = 0; j < type_size(S.types[s]); j++) {
                double v;
                if (!b.real(v)) return fail("truncated SolAtVertices");
                store(k, s, j, v);
              }
        }
      }
      if (next <= 0) break;
      if (fseek(b.f, (long)next, SEEK_SET) != 0) return fail("bad .solb block position");
    }
    return found ? 1 : fail("no SolAtVertices");
  }
  Text t;
  if (!t.load(path)) return fail(std::string("cannot open ") + path);
  while (!t.at_end()) {
    if (!t.next_is_word()) { t.word(); continue; }
    const std::string kw = t.word();
    int64_t n = 0;
    if (kw == "End") break;
    if (kw == "MeshVersionFormatted") {
      if (!t.integer(n)) return fail("bad MeshVersionFormatted");
      S.version = (int)n;
    } else if (kw == "Dimension") {
      if (!t.integer(n) || n != 3) return fail("only 3-D solutions");
    } else if (kw == "SolAtVertices") {
      int64_t nt;
      if (!t.integer(n) || !t.integer(nt) || nt < 1 || nt > PMX_MAX_SOLS) return fail("bad SolAtVertices header");
      S.np = n;
      S.nsol = (int)nt;
      for (int s = 0; s < S.nsol; s++) {
        int64_t ty;
        if (!t.integer(ty) || !type_size((int)ty)) return fail("unsupported solution type");
        S.types[s] = (int)ty;
      }
      if (!sol_header_ok(S, expect)) return 0;
      if (!fields) return 1;
      for (int64_t k = 1; k <= n; k++)
        for (int s = 0; s < S.nsol; s++)
          for (int j = 0; j < type_size(S.types[s]); j++) {
            double v;
            if (!t.real(v)) return fail("truncated SolAtVertices");
            store(k, s, j, v);
          }
      return 1;
    } else {
      t.skip_block();
    }
  }
  return fail("no SolAtVertices");
}

}  // namespace

extern "C" {

const char *pmx_medit_last_error(void) { return g_err.c_str(); }

int pmx_medit_mesh_info(const char *path, pmx_medit_info *info) {
  if (!path || !info) return fail("pmx_medit_mesh_info: null argument");
  return read_mesh(path, info, nullptr, nullptr);
}

int pmx_medit_mesh_read(const char *path, const pmx_medit_info *sized, double *xyz, int *vref, int *tet,
                        int *tetref, int *tria, int *triaref, int *req) {
  if (!path || !sized || !xyz || !tet) return fail("pmx_medit_mesh_read: null argument");
  MeshOut o{xyz, vref, tet, tetref, tria, triaref, req};
  return read_mesh(path, nullptr, &o, sized);
}

int pmx_medit_mesh_write(const char *path, int64_t np, const double *xyz, const int *vref, int64_t ne,
                         const int *tet, const int *tetref, int64_t nt, const int *tria, const int *triaref,
                         int64_t nreq, const int *req) {
  if (!path || np < 0 || ne < 0 || nt < 0 || nreq < 0 || (np && !xyz) || (ne && !tet) || (nt && !tria) ||
      (nreq && !req))
    return fail("pmx_medit_mesh_write: bad arguments");
  if (is_binary(path)) {
    BinOut b;
    b.f = fopen(path, "wb");
    if (!b.f) return fail(std::string("cannot create ") + path);
    // version 2 (float64, 32-bit positions) while the file stays below 2 GiB
    // and the counts fit, else 3 / 4
    const double bytes = 64.0 + np * 32.0 + ne * 20.0 + nt * 16.0 + nreq * 4.0;
    b.ver = (np >= (1LL << 31) || ne >= (1LL << 31)) ? 4 : bytes >= 2.0e9 ? 3 : 2;
    b.i32(1);
    b.i32(b.ver);
    long at = b.begin(KW_DIM, false, 0);
    b.i32(3);
    b.end(at);
    at = b.begin(KW_VERT, true, np);
    for (int64_t k = 1; k <= np; k++) {
      for (int a = 0; a < 3; a++) b.real(xyz[3 * k + a]);
      b.integer(vref ? vref[k] : 0);
    }
    b.end(at);
    at = b.begin(KW_TET, true, ne);
    for (int64_t k = 1; k <= ne; k++) {
      for (int a = 0; a < 4; a++) b.integer(tet[4 * k + a]);
      b.integer(tetref ? tetref[k] : 0);
    }
    b.end(at);
    if (nt) {
      at = b.begin(KW_TRI, true, nt);
      for (int64_t k = 1; k <= nt; k++) {
        for (int a = 0; a < 3; a++) b.integer(tria[3 * k + a]);
        b.integer(triaref ? triaref[k] : 0);
      }
      b.end(at);
    }
    if (nreq) {
      at = b.begin(KW_REQV, true, nreq);
      for (int64_t k = 0; k < nreq; k++) b.integer(req[k]);
      b.end(at);
    }
    at = b.begin(KW_END, false, 0);
    (void)at;                                    // End: next position 0
    if (!b.close()) return fail(std::string("write error: ") + path);
    return 1;
  }
  FILE *f = fopen(path, "w");
  if (!f) return fail(std::string("cannot create ") + path);
  fprintf(f, "MeshVersionFormatted 2\n\nDimension 3\n\nVertices\n%lld\n", (long long)np);
  for (int64_t k = 1; k <= np; k++)
    fprintf(f, "%.17g %.17g %.17g %d\n", xyz[3 * k], xyz[3 * k + 1], xyz[3 * k + 2], vref ? vref[k] : 0);
  fprintf(f, "\nTetrahedra\n%lld\n", (long long)ne);
  for (int64_t k = 1; k <= ne; k++)
    fprintf(f, "%d %d %d %d %d\n", tet[4 * k], tet[4 * k + 1], tet[4 * k + 2], tet[4 * k + 3],
            tetref ? tetref[k] : 0);
  if (nt) {
    fprintf(f, "\nTriangles\n%lld\n", (long long)nt);
    for (int64_t k = 1; k <= nt; k++)
      fprintf(f, "%d %d %d %d\n", tria[3 * k], tria[3 * k + 1], tria[3 * k + 2], triaref ? triaref[k] : 0);
  }
  if (nreq) {
    fprintf(f, "\nRequiredVertices\n%lld\n", (long long)nreq);
    for (int64_t k = 0; k < nreq; k++) fprintf(f, "%d\n", req[k]);
  }
  fprintf(f, "\nEnd\n");
  bool bad = fflush(f) != 0 || ferror(f) != 0;
  bad = fclose(f) != 0 || bad;
  return bad ? fail(std::string("write error: ") + path) : 1;
}

int pmx_medit_sol_info(const char *path, int64_t *np, int *nsol, int *types) {
  if (!path || !np || !nsol) return fail("pmx_medit_sol_info: null argument");
  SolIn S;
  if (!read_sol(path, S, nullptr, nullptr)) return 0;
  *np = S.np;
  *nsol = S.nsol;
  if (types)
    for (int s = 0; s < S.nsol; s++) types[s] = S.types[s];
  return 1;
}

int pmx_medit_sol_read(const char *path, int64_t np, int nsol, const int *types, double **fields) {
  if (!path || !fields || !types || nsol < 1 || nsol > PMX_MAX_SOLS || np < 0)
    return fail("pmx_medit_sol_read: bad arguments");
  SolIn E, S;
  E.np = np;
  E.nsol = nsol;
  for (int s = 0; s < nsol; s++) E.types[s] = types[s];
  return read_sol(path, S, fields, &E);
}

int pmx_medit_sol_write(const char *path, int64_t np, int nsol, const int *types, const double *const *fields) {
  if (!path || np < 0 || nsol < 1 || nsol > PMX_MAX_SOLS || !types || !fields)
    return fail("pmx_medit_sol_write: bad arguments");
  for (int s = 0; s < nsol; s++)
    if (!type_size(types[s]) || !fields[s]) return fail("pmx_medit_sol_write: bad solution");
  if (is_binary(path)) {
    BinOut b;
    b.f = fopen(path, "wb");
    if (!b.f) return fail(std::string("cannot create ") + path);
    int width = 0;
    for (int s = 0; s < nsol; s++) width += type_size(types[s]);
    const double bytes = 64.0 + np * 8.0 * width;
    b.ver = np >= (1LL << 31) ? 4 : bytes >= 2.0e9 ? 3 : 2;
    b.i32(1);
    b.i32(b.ver);
    long at = b.begin(KW_DIM, false, 0);
    b.i32(3);
    b.end(at);
    at = b.begin(KW_SOLV, true, np);
    b.i32(nsol);
    for (int s = 0; s < nsol; s++) b.i32(types[s]);
    for (int64_t k = 1; k <= np; k++)
      for (int s = 0; s < nsol; s++) {
        const int sz = type_size(types[s]);
        for (int j = 0; j < sz; j++) b.real(fields[s][k * sz + (sz == 6 ? tensor_perm(j) : j)]);
      }
    b.end(at);
    b.begin(KW_END, false, 0);
    if (!b.close()) return fail(std::string("write error: ") + path);
    return 1;
  }
  FILE *f = fopen(path, "w");
  if (!f) return fail(std::string("cannot create ") + path);
  fprintf(f, "MeshVersionFormatted 2\n\nDimension 3\n\nSolAtVertices\n%lld\n%d", (long long)np, nsol);
  for (int s = 0; s < nsol; s++) fprintf(f, " %d", types[s]);
  fprintf(f, "\n");
  for (int64_t k = 1; k <= np; k++) {
    bool first = true;
    for (int s = 0; s < nsol; s++) {
      const int sz = type_size(types[s]);
      for (int j = 0; j < sz; j++) {
        fprintf(f, first ? "%.17g" : " %.17g", fields[s][k * sz + (sz == 6 ? tensor_perm(j) : j)]);
        first = false;
      }
    }
    fprintf(f, "\n");
  }
  fprintf(f, "\nEnd\n");
  bool bad = fflush(f) != 0 || ferror(f) != 0;
  bad = fclose(f) != 0 || bad;
  return bad ? fail(std::string("write error: ") + path) : 1;
}

}  // extern "C"
