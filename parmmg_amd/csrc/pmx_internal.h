// pmx_internal.h -- the context object behind the C ABI (host only).
#pragma once
#include <hip/hip_runtime.h>
#include <string>
#include <vector>
#include "pmx_transfer.h"
#include "pmx_kernels.h"

template <class T> struct DevBuf {
  T *p = nullptr;
  size_t cap = 0;
};

struct pmx_ctx {
  int device = 0;
  hipStream_t own = nullptr, stream = nullptr;
  // the surface path runs on `side`, forked after the prologue and joined
  // before the fallback: it overlaps the volume hint build and walk
  hipStream_t side = nullptr;
  hipStream_t side_lo = nullptr;        // lowest-priority side stream (tune bit 30)
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  std::string err;
  // pinned host staging arena (hipHostMalloc, grown on demand, reused across
  // steps): point uploads and result downloads go through it as async DMA
  // instead of pageable copies (PCIe-inclusive rate)
  void *h_stage = nullptr;
  size_t h_stage_cap = 0;

  // background group
  bool have_bg = false;
  int64_t np = 0, ne = 0, nt = 0;
  double hausd = 0.0;
  SolDesc sd{};
  GridDesc grid{};
  int64_t gcells = 0;
  double bblo[3]{}, bbhi[3]{};
  DevBuf<Pt4> d_pts;
  DevBuf<TetRec> d_tets;
  DevBuf<double> d_sol;
  DevBuf<double> d_xyz;                 // dense coordinates, 3 doubles per vertex
  DevBuf<float> d_xyzf;                 // the same in single precision (hint centroids)
  DevBuf<unsigned long long> d_xyzq;    // fixed-point grid coordinates (hint centroids)
  DevBuf<TriRec> d_tris;
  DevBuf<Pt4> d_trn;
  DevBuf<int> d_grid;
  DevBuf<unsigned long long> d_grid64;    // central-hint grid: (dist2 f32 bits << 32 | tet) minima
  DevBuf<int> d_ntoff, d_ntlist;
  std::vector<int> h_ntoff, h_ntlist;

  // new points and results
  bool have_pts = false, ran = false;
  int64_t nq = 0, nq_vol = 0, nq_bdy = 0;
  int out_S = -1;
  DevBuf<Pt4> d_q;
  DevBuf<int8_t> d_kind;
  DevBuf<uint8_t> d_wmask;
  DevBuf<double> d_out;
  DevBuf<int> d_elem, d_status, d_steps, d_start, d_edge, d_vertex;
  DevBuf<int> d_list, d_found, d_bestk;
  DevBuf<int2> d_ties;
  // tet-centric volume path
  DevBuf<int4> d_tetv;                  // connectivity stream (16 B / tet)
  DevBuf<int4> d_tets_s;                // packed sample: tets 1, 1+S, 1+2S.. (S = hint stride)
  DevBuf<unsigned> d_qcnt, d_qstart;
  DevBuf<int> d_qcell, d_qslot, d_tbest;
  DevBuf<Pt4> d_qs;
  DevBuf<unsigned long long> d_tests;
  DevBuf<char> d_scan_tmp;
  int tests_blocks = 0;
  bool tet_mode = false;
  DevBuf<unsigned long long> d_best;
  DevBuf<unsigned> d_counts;            // [0] vol stuck, [1] bdy stuck, [2] bdy overflow
  DevBuf<int> d_vollist, d_bdylist;     // compacted point lists per path
  DevBuf<double> d_qv;                  // volume points, dense xyz in list order
  DevBuf<uint4> d_vstat, d_bstat;       // per-wave walk statistics
  DevBuf<int> d_blist, d_olist, d_ows;
  int *d_tgrid = nullptr;
  size_t d_tgrid_cap = 0;
  GridDesc tgd{};
  bool tria_hint_fused = false;         // this step's tria hint built with the volume hint
  int64_t tcells = 0;

  // statistics
  DevBuf<double> d_qual;
  DevBuf<unsigned long long> d_red;
  DevBuf<uint8_t> d_emask;              // prilen: per-tet mask of edges whose shell is rotated
  DevBuf<uint32_t> d_elist;             // prilen: compacted (tet*8 + edge) list
  DevBuf<unsigned> d_bcount;            // prilen: per-block counts -> offsets, [nb] total
  bool have_qual = false;

  // timing
  double topo_ms = 0.0;                 // device time of the last topology build
  std::vector<hipEvent_t> events;
  int ev_used = 0;

  hipEvent_t *next_event_slot();
  void free_all();
  void host_build_node_trias(const std::vector<TriRec> &tr);
  bool launch_bdy(const VolArgs &a, const pmx_run_opts &o, hipStream_t s);
  bool size_tria_grid();
  bool launch_tet_locate(const VolArgs &a, const pmx_run_opts &o, hipStream_t s);
};

bool pmx_ctx_build_adja_host(pmx_ctx *ctx, const pmx_mesh_view *m, std::vector<int> &adja);
void launch_tria_normals(const TriRec *tris, const Pt4 *pts, int64_t nt, Pt4 *trn, hipStream_t s);
extern "C" int pmx_timing_reset(pmx_ctx *ctx);
