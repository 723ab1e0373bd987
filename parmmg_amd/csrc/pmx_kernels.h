// pmx_kernels.h -- kernel argument blocks and launchers (host <-> device).
#pragma once
#include "pmx_device.h"

struct GridDesc {
  int dim[3];
  double lo[3];
  double inv[3];
  int qf[3];        // fraction bits of the fixed-point grid coordinates:
                    // dim << qf fits 21 bits (qf = 21 - ceil(log2 dim))
};

// cell (x, y, z) of the volume hint grid, row-major.  (r03: 4x4x4 blocks of
// 64 cells, so that a wave of Morton-ordered points reads its hint cells from
// a few lines, left the walk within 0.5 % and made the surface path overlap it
// worse: C3 step 2.09 -> 2.19 ms, profiles/r03_c3_sweep_grid_priority.log.)
__host__ __device__ inline int64_t gcell(const GridDesc &g, int x, int y, int z) {
  return (int64_t)x + (int64_t)g.dim[0] * ((int64_t)y + (int64_t)g.dim[1] * z);
}

// counters of one step (d_counts, zeroed by the prologue):
//   [0] volume stuck, [1] surface stuck, [2] surface overflow, [3] volume ties,
//   [4] k_fallback grid-barrier arrivals, [7] device error flags (PMX_DERR_*)
#define PMX_CNT_ERR 7
#define PMX_DERR_BARRIER 1u         // a grid barrier gave up waiting (co-residency lost)

struct VolArgs {
  const double *xyz;            // old vertices, 24 B (x, y, z), 1-based
  const TetRec *tets;
  const WRec *wrec;             // the walk's compact copy of tets (null: walk on tets)
  const double *sol;
  SolDesc sd;
  const double *q;              // new points as uploaded, dense x y z (0-based)
  const int8_t *kind;
  int64_t nq, ne;
  const int *grid;
  const uint4 *hrec;            // exp 13: the hint cells with their start record inline
  GridDesc g;
  double *out;
  uint8_t *wmask;
  int *elem, *status, *steps, *start;
  int *stuck_list;
  unsigned *stuck_count;
  int2 *tie_list;               // (point, found tet) of points near a face
  unsigned *tie_count;
  int *found, *bestk;
  unsigned long long *best;
  const int *list;              // indices of the volume points (input order kept)
  int64_t nlist;                // upper bound (launch size); the step's count is *nlist_dev
  const int *nlist_dev;
  uint4 *wstats;                // per-wave {located, sum steps, max, min}
  int max_walk;
  unsigned const_bit;           // wmask bit of a constant-size metric (0 if none)
  int inline_ties;              // resolve face ties in place
  int ref_walk;                 // 1: k_walk (reference-order walk) instead of k_walks
  int rec_start;                // write the start tet of every point (diagnostics)
  int far;                      // the compact records have far neighbour fields (pmx_wrec.h)
  int exp;                      // measurement switch (tools/walk_pmc.sh): 0 production,
                                // 4 no interpolation, 5 hint + hint record only,
                                // 17 a record with a far neighbour field read whole,
                                // 18 compact records whatever their far fields,
                                // (pmx_run) 19 / 20 fans on the main stream
};

struct ExhArgs {
  const double *xyz;
  const TetRec *tets;
  int64_t ne;
  const double *q;
  const int *list;
  const unsigned *count;
  int *found;
  unsigned long long *best;
  int *bestk;
  long spin_limit;              // grid-barrier poll budget (debug: 0 forces a timeout)
};

// volume hint grid from every stride-th tet: `packed` = the host-packed
// connectivity of tets 1, 1+stride, ... (stride == PMX_HINT_STRIDE), else the
// tet records are read strided
void launch_hint_build(const int4 *packed, const int *kidx, const TetRec *tets, int64_t ne, int stride, int *grid,
                       GridDesc g, const unsigned long long *xyzq, const double *xyz, hipStream_t s,
                       bool v0 = false, int bs = 256, int64_t nsamp = -1);
void launch_hint_inline(const int *grid, int64_t cells, const WRec *wr, uint4 *hrec, hipStream_t s);
// per-background derived data: fixed-point grid coordinates of the vertices
// (hint centroids) and the unit normals of the boundary trias
// (PMMG_precompute_triaNormals, src/locate_pmmg.c:68-90), one launch
void launch_bg_derive(const double *xyz, int64_t np, GridDesc g, unsigned long long *xyzq,
                      const TriRec *tris, int64_t nt, Pt4 *trn, hipStream_t s);
void launch_walk(const VolArgs &a, hipStream_t s);
void launch_exhaustive(const ExhArgs &e, const VolArgs &v, int blocks, hipStream_t s);
void launch_const_metric(const int8_t *kind, int64_t nq, double *out, int S, int off, int size,
                         double hsiz, uint8_t *wmask, int imet, hipStream_t s);
// the step's first launch zeroes up to PMX_ZERO_MAX device ranges
#define PMX_ZERO_MAX 3
struct ZeroRanges {
  void *p[PMX_ZERO_MAX];
  int64_t bytes[PMX_ZERO_MAX];
  int n;
  void add(void *ptr, int64_t b) {
    if (ptr && b > 0) { p[n] = ptr; bytes[n] = b; n++; }
  }
};
void launch_prologue(const ZeroRanges &z, hipStream_t s);
void launch_tet_conn(const TetRec *src, int64_t n, int4 *dst, hipStream_t s);
// device residency (pmx_promote_background): new points + results -> background
void launch_promote(const double *qxyz, const double *out, const uint16_t *qtag, int64_t n, int S, double *xyz,
                    double *sol, uint16_t *ptag, hipStream_t s);
// points in no valid new tet (mk == 0) after a step: rows back to untouched
void launch_mark_new_tets(const int4 *tv, int64_t ne, uint8_t *mk, int64_t nmk, hipStream_t s);
struct OrphanRows {
  uint8_t *wmask;
  int *elem, *status, *steps, *start, *edge, *vertex;
  int8_t *kind;
};
void launch_orphans(const uint8_t *mk, int64_t n, uint8_t keep, const OrphanRows &r, hipStream_t s);
void launch_patch_rows(const int4 *ent, const double *vals, int64_t n, int S, double *sol, hipStream_t s);
// new points, every step (the tag dispatch of the reference's vertex loop,
// src/interpmesh_pmmg.c:541-560): kinds (mark != NULL: the orphan marks of
// the new tets, 0 = in no valid new tet) and the order-preserving compaction into
// the volume / surface lists; counts into nsel[0..1].  tcnt: scratch of cls_tiles(n) int2.
#define CLS_TILE 16384               // 4 rounds of 256 threads x 16 points
inline int64_t cls_tiles(int64_t n) { return (n + CLS_TILE - 1) / CLS_TILE; }
void launch_classify(const uint16_t *tag, const uint8_t *mk, int64_t n, int2 *tcnt, int8_t *kind, int *vlist,
                     int *blist, int *nsel, hipStream_t s);

void launch_build_tetrec(const int4 *tv, const int *adja, int64_t ne, int stride, TetRec *tets, int4 *sample,
                         hipStream_t s);
// the vertex-owner sample (k_vmin_owner): out[i] / kidx[i] the i-th vertex's
// owner tet in vertex order; owner np + 1 words, flag and pos np + 1 ints each,
// tmp owner_scan_temp_bytes(np) bytes; the sample count into *h_count (pinned)
size_t owner_scan_temp_bytes(int64_t np);
bool launch_owner_sample(const TetRec *tets, int64_t ne, int64_t np, unsigned *owner, int *flag, int *pos,
                         int4 *out, int *kidx, unsigned *d_count, unsigned *h_count, void *tmp, size_t tmp_bytes,
                         hipStream_t s);
// the walk's compact records from the tet records (slots 0..ne)
// (*h_nfar, pinned, when stream s gets there: the tets with a far neighbour
// field, pmx_wrec.h; d_nfar one device word)
void launch_build_wrec(const TetRec *tets, int64_t ne, WRec *wr, unsigned *d_nfar, unsigned *h_nfar,
                       hipStream_t s);
// PMX_RUN_SEQUENTIAL_VOLUME (pmx_walk.hip): the volume sequence (point
// indices in the reference's visit order, its length on the device), each
// point's speculative start and mesh->base, the speculation's "sure" flags,
// the replay's tet flags (ne + 1, base compare), its control words and
// one-point stuck list, the replay count
struct SeqVolArgs {
  const int *vseq;
  const int *nvseq;
  const int *sstart, *sbase;
  uint8_t *sure;
  int *tf;
  int *ctl;
  int *stk_list;
  unsigned *nreplay;
  const int *cand, *ncand;   // the positions whose speculative start may be wrong (sorted)
};
// the speculative pass and its overflow pass (workspace: seqv_ovf_ws_ints() ints)
size_t seqv_ovf_ws_ints();
void launch_seqv_spec(const VolArgs &a, const SeqVolArgs &s, int64_t nmax, int *ws, hipStream_t st);
void launch_seqv_resolve(const VolArgs &a, const SeqVolArgs &s, hipStream_t st);
// flags[j] (j < nmax) = position j of the volume sequence must be checked by
// the replay: not sure, or its start is not its predecessor's speculative tet
void launch_seqv_flags(const VolArgs &a, const SeqVolArgs &s, int64_t nmax, uint8_t *flags, hipStream_t st);
// workgroups of k_fallback that can be co-resident with `share` other
// launches of it on this device (0 on error)
int fallback_coresident_blocks(int device, int share);

struct StatArgs {
  // vertex v at xyz[xstride * (v - vbase)] (background: dense xyz, stride 3,
  // base 0; new mesh: the uploaded Pt4 points, stride 4, base = first index);
  // its metric at sol[S * (v - vbase) + moff], its tag at ptag[v - vbase]
  const double *xyz;
  int xstride, vbase;
  const TetRec *tets;           // records with neighbours (background only)
  const int4 *tetv;             // connectivity stream (v only)
  int64_t ne;
  const double *sol;
  int S, msize, moff;
  const uint16_t *ptag;         // point tags or null (no ridge points)
  // quality with metRidTyp = 1 and a tensor metric (MMG5_caltet_ani): the
  // mean metric leaves out the non-singular ridge points of these tags
  // (null: every vertex counts)
  const uint16_t *rtag;
  int ridmet;
  // edge lengths in a tensor metric along the curved surface (pmx_upload_surface;
  // null: no xTetra, zero normals): per tet the xTetra edge tags (bit 2 ia
  // MG_BDY, 2 ia + 1 MG_GEO), per point MMG5_Point.n and its xPoint index,
  // per xPoint n1 | n2 (6 doubles, entry 0 zero)
  const uint16_t *etag;
  const double *pn, *xpn;
  const int *pxp;
  // distributed prilen: sorted (min << 32 | max) keys of the parallel edges
  // the tet loop must skip, and a per-point prefilter
  const unsigned long long *par_key;
  int64_t npar;
  const uint8_t *par_pt;
  // k_prilen's tet schedule: 0 = one contiguous range per workgroup; C > 0 =
  // a moving front (each XCD's range dealt out in chunks of C batches,
  // round-robin over that XCD's workgroups, all co-resident)
  int sched_chunk;
};
