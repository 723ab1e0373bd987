// pmx_kernels.h -- kernel argument blocks and launchers (host <-> device).
#pragma once
#include "pmx_device.h"

struct GridDesc {
  int dim[3];
  double lo[3];
  double inv[3];
};

struct VolArgs {
  const Pt4 *pts;
  const TetRec *tets;
  const double *sol;
  SolDesc sd;
  const Pt4 *q;
  const int8_t *kind;
  int64_t nq, ne;
  const int *grid;
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
  const int *list;              // indices of the volume points (Morton order kept)
  int64_t nlist;
  uint4 *wstats;                // per-wave {located, sum steps, max, min}
  int max_walk;
  unsigned const_bit;           // wmask bit of a constant-size metric (0 if none)
  int occ;                      // k_locate_vol register/occupancy variant
  int xcd_swizzle;
  int inline_ties;               // k_walk: resolve face ties in place
  const double *qv;             // coordinates of the volume points in list order (xyz, 24 B)
  unsigned long long *wctr;     // k_walkp: per-XCD-region chunk counters [8]
  int64_t region;               // k_walkp: points per region (multiple of 64)
  int block;                    // k_walk threads per block (256 / 512 / 1024)
  const unsigned long long *grid64;  // central hint grid (null: plain int grid)
  int exp;                      // k_walk sensitivity experiment (0 = production)
  const double *xyz;            // dense 24-B coordinates (k_build_xyz), null: use pts
  int ref_walk;                 // 1: k_walk (reference-order walk) instead of k_walks
  int rec_start;                // k_walks: write the start tet of every point (diagnostics)
};

struct ExhArgs {
  const Pt4 *pts;
  const TetRec *tets;
  int64_t ne;
  const Pt4 *q;
  const int *list;
  const unsigned *count;
  int *found;
  unsigned long long *best;
  int *bestk;
};

void launch_hint_build(const int4 *tetv, const int4 *packed, const Pt4 *pts, int64_t ne,
                       int stride, int *grid, GridDesc g, int mid, hipStream_t s,
                       unsigned long long *grid64 = nullptr, const double *xyz = nullptr,
                       const float *xyzf = nullptr, const unsigned long long *xyzq = nullptr);
// fraction bits of the fixed-point grid coordinates (dim <= 4096: 12 + 9 = 21 bits)
#define HINT_QF 9
void launch_hint_build_fused(const int4 *packed, int64_t ne, int stride, int *grid, GridDesc g,
                             const unsigned long long *xyzq, const TriRec *tris, const Pt4 *pts,
                             int64_t nt, int *tgrid, GridDesc tg, hipStream_t s);
void launch_quant_xyz(const Pt4 *pts, int64_t n, GridDesc g, unsigned long long *q, hipStream_t s);
void launch_fill64(unsigned long long *p, int64_t n, hipStream_t s);
void launch_locate_vol(const VolArgs &a, hipStream_t s);
void launch_walk(const VolArgs &a, hipStream_t s);
void launch_walkp(const VolArgs &a, hipStream_t s);
void launch_build_xyz(const Pt4 *pts, int64_t n, double *out, float *outf, hipStream_t s);
void launch_tet_conn(const TetRec *src, int64_t stride, int64_t n, int4 *dst, hipStream_t s);
void launch_exhaustive(const ExhArgs &e, const VolArgs &v, hipStream_t s);
void launch_const_metric(const int8_t *kind, int64_t nq, double *out, int S, int off, int size,
                         double hsiz, uint8_t *wmask, int imet, hipStream_t s);
void launch_run_init(unsigned *counts, hipStream_t s);
void launch_prologue(uint8_t *wmask, int64_t n, unsigned *counts, int *grid, int64_t gcells,
                     int *tgrid, int64_t tcells, hipStream_t s);

struct StatArgs {
  const Pt4 *pts;
  const double *xyz;            // dense 24-B coordinates (k_build_xyz); null: pts
  const TetRec *tets;
  const int4 *tetv;             // connectivity stream (v only)
  int64_t ne;
  const double *sol;
  int S, msize, moff;
  const uint16_t *ptag;
};
