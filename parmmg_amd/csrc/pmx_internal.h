// pmx_internal.h -- the context object behind the C ABI (host only).
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include <functional>
#include <string>
#include <vector>
#include "pmx_transfer.h"
#include "pmx_kernels.h"

template <class T> struct DevBuf {
  T *p = nullptr;
  size_t cap = 0;
};

// hint grid from every 4th tet: 1/4 of the stores and of the tet bytes of a
// full build, at ~0.5 extra walk step (r01 measurements)
#define PMX_HINT_STRIDE 4
// pmx_run_opts.flags bits 16-23: the walk's measurement switch (VolArgs.exp; tools/walk_pmc.sh)
#define PMX_RUN_EXP_SHIFT 16
// the walk takes the 32-B tet records instead of the compact ones when more
// than 1/PMX_WREC_FAR_DIV of the tets have a far neighbour field (pmx_wrec.h)
#define PMX_WREC_FAR_DIV 16

struct pmx_ctx {
  int device = 0;
  hipStream_t own = nullptr, stream = nullptr;
  // the surface path runs on `side`, forked after the volume hint build and
  // joined before the fallback: it overlaps the volume walk
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_fork2 = nullptr, ev_join = nullptr;
  hipEvent_t ev_dl[8] = {};             // chunked download: one per chunk
  std::string err;
  int fallback_blocks = 0;              // co-resident k_fallback workgroups
  int fallback_share = 0;               // live contexts on the device they were sized for
  // PMX_interpMetricsAndFields: a second context on the same device, groups
  // alternate between the two (created on first use, destroyed with this one)
  pmx_ctx *peer = nullptr;
  // pinned host staging arena (hipHostMalloc, grown on demand, reused across
  // steps): uploads and downloads go through it as async DMA
  void *h_stage = nullptr;
  size_t h_stage_cap = 0;

  // background group (raw uploads)
  bool have_bg = false;
  int64_t np = 0, ne = 0, nt = 0;
  double hausd = 0.0;
  SolDesc sd{};
  GridDesc grid{};
  int64_t gcells = 0;
  double bblo[3]{}, bbhi[3]{};
  DevBuf<double> d_xyz;                 // old vertices, x y z (24 B), slot 0 unused
  DevBuf<TetRec> d_tets;
  DevBuf<WRec> d_wrec;                  // the walk's compact copy of d_tets (built with it)
  DevBuf<unsigned> d_wfar;              // [0] / [1] far-field counters of d_wrec / d_wrec_next, [2] / [3] bad fans (step / upload check), [4] owner-sample count
  DevBuf<double> d_sol;
  DevBuf<int4> d_tets_s;                // hint sample: every 4th tet (default, packed with the tets) or one owner tet per vertex (order_hint_samples)
  DevBuf<int> d_tets_sk;                // its tet indices (samples_sorted)
  bool samples_sorted = false;
  bool samples_owner = false;           // the vertex-owner sample: nsamp entries
  // decided at each background upload / promotion (environment, A/B):
  // compact_recs -- the walk's 24-B records d_wrec are built (PMX_WALK_RECORDS=compact;
  //   default: the walk reads the 32-B records, no per-background pass);
  // sample_mode -- PMX_HINT_SAMPLE_ORDER: 0 (default) every 4th tet, packed by the host
  //   with the tet records (or by k_build_tetrec), 2 one owner tet per vertex (device passes)
  bool compact_recs = false;
  int sample_mode = 0;
  // d_btv holds this background's raw connectivity and its adjacency was
  // built on the device (an upload without Mmg's adja)
  bool bg_btv = false;
  int64_t nsamp = 0;
  DevBuf<unsigned> d_skey;              // order_hint_samples scratch: keys / owners, indices / flags, records, temp
  DevBuf<int> d_sidx;
  DevBuf<int4> d_salt;
  DevBuf<char> d_stmp;
  DevBuf<TriRec> d_tris;
  // node -> trias fans (built on the device, in the step): ntlist = trias
  // sorted by (vertex, index), ntrange[3 k + l] = the run of vertex l of tria k
  DevBuf<int> d_ntlist, d_ntval;
  DevBuf<unsigned> d_ntkey;
  DevBuf<int2> d_ntrange;
  DevBuf<char> d_nttmp;
  bool have_csr = false;
  // derived from the raw uploads on the device (k_bg_derive), by the first
  // step after an upload or by every step with PMX_RUN_FRESH_BACKGROUND
  bool have_derived = false;
  DevBuf<unsigned long long> d_xyzq;    // fixed-point grid coordinates (hint centroids)
  DevBuf<Pt4> d_trn;                    // tria unit normals + areas
  DevBuf<int> d_grid;
  // statistics only: 16-B connectivity stream, derived on first use
  bool have_tetv = false;
  DevBuf<int4> d_tetv;

  // new points and results
  bool have_pts = false, ran = false;
  int64_t nq = 0;
  // volume / surface point counts: upper bounds from the host's tag pass
  // (launch sizes); the exact counts are the step's classification (d_nsel)
  int64_t nq_vol_ub = 0, nq_bdy_ub = 0;
  int out_S = -1;                       // solution width the results were computed for
  int64_t out_n = -1;                   // point count the results were computed for
  DevBuf<int8_t> d_kind;
  DevBuf<uint8_t> d_wmask;
  DevBuf<double> d_out;
  DevBuf<int> d_elem, d_status, d_steps, d_start, d_edge, d_vertex;
  DevBuf<int> d_list, d_found, d_bestk;
  DevBuf<int2> d_ties;
  DevBuf<unsigned long long> d_best;
  DevBuf<unsigned> d_counts;            // step counters, see pmx_kernels.h
  DevBuf<int> d_vollist, d_bdylist;     // compacted point lists per path
  DevBuf<double> d_qxyz;                // new points as uploaded (dense xyz)
  DevBuf<uint8_t> d_qmark;              // orphan marks (points of valid new tets), uploaded when needed
  DevBuf<int> d_nsel;                   // compaction counts: volume, surface
  DevBuf<int2> d_ctile;                 // classification tile counts
  DevBuf<uint4> d_vstat, d_bstat;       // per-wave walk statistics
  DevBuf<uint4> d_hrec;                 // exp 13: hint cells with their start record inline
  DevBuf<int> d_blist, d_olist, d_ows;
  // PMX_RUN_SEQUENTIAL_SURFACE (pmx_bdy.hip seq_surface): visit keys / order,
  // located / surface flags and their scan, bases | sequence | speculative
  // starts | control words, wedge flags, cub scratch, the replay's tria and
  // point flags; seq_stats = {replayed queries, surface sequence length}
  DevBuf<unsigned> d_sqkey;
  DevBuf<int> d_sqidx, d_sqint, d_sqtf, d_sqpf, d_sqtv, d_sqows;
  DevBuf<unsigned long long> d_sqval;
  DevBuf<uint8_t> d_sqw, d_sqflag;
  DevBuf<int> d_sqcand;                 // [0] count, then the volume replay's candidate positions
  DevBuf<char> d_sqtmp;
  unsigned seq_stats[4] = {0, 0, 0, 0};   // surface replays / sequence, volume replays / sequence
  int64_t seq_stats_n = -1;             // -1: the last step was not sequential
  int *d_tgrid = nullptr;
  size_t d_tgrid_cap = 0;
  GridDesc tgd{};
  int64_t tcells = 0;

  // group seams (pmx_groups.hip): constant-size metric of a step without a
  // background, and the frozen-point copy (buffers reused across calls)
  DevBuf<double> d_cmet;
  DevBuf<int> d_cperm, d_ccnt;         // pmx_copy_required

  // statistics
  DevBuf<double> d_qual;
  DevBuf<unsigned long long> d_red;
  bool have_qual = false;
  bool have_ptag = false;               // background point tags (pmx_upload_point_tags)
  DevBuf<uint16_t> d_ptag;
  // Mmg's surface data of the background (pmx_upload_surface): per tet the
  // xTetra edge tags packed 2 bits per edge (BDY, GEO); per point MMG5_Point.n
  // and its xPoint index; per xPoint n1, n2
  bool have_surf = false;
  DevBuf<uint16_t> d_etag;
  DevBuf<double> d_pn, d_xpn;
  DevBuf<int> d_pxp;
  DevBuf<uint16_t> d_pedge_tag;         // prilen: tags of the owned parallel edges
  // prilen, edge-bucket variant (PMX_PRILEN_BUCKETS=1, A/B of the shell
  // rotation): per-vertex counts / offsets / cursors and the candidate records
  DevBuf<unsigned> d_pbcnt, d_pboff;
  DevBuf<int4> d_pbrec;
  DevBuf<char> d_pbtmp;
  int64_t stat_np = -1;                 // node count of pmx_count_nodes (-1: np)
  DevBuf<uint8_t> d_touch;
  DevBuf<int> d_cidx, d_intv;
  DevBuf<double> d_pub;                 // public partial records of the host wrappers
  DevBuf<unsigned long long> d_pkey;    // prilen: excluded parallel edges (sorted keys)
  DevBuf<uint8_t> d_ppt;
  DevBuf<int2> d_pedge;                 // prilen: owned parallel edges (step 1)
  DevBuf<int4> d_ntetv;                 // the new tets (pmx_upload_new_tets), 1-based
  bool have_ntet = false;               //   vertex = points-view index - first + 1
  int64_t n_ntet = 0;
  double qlo[3]{}, qhi[3]{};            // bbox of the uploaded new points
  // device adjacency of promoted backgrounds (pmx_topo.hip), reused buffers
  DevBuf<int> d_adja;
  DevBuf<int4> d_btv;                   // background connectivity when its adjacency is built here
  DevBuf<unsigned> d_tcnt, d_toff, d_tbad;
  DevBuf<int4> d_trec;
  DevBuf<char> d_ttmp;
  DevBuf<int4> d_pent;                  // promote: patched rows
  DevBuf<double> d_pval;
  // residency (pmx_set_residency): the next background's tet records, built
  // from the new tets on the `topo` stream while the current step runs
  bool residency = false;
  hipStream_t topo = nullptr;
  hipEvent_t ev_topo = nullptr;
  bool next_topo = false;               // d_tets_next / d_tets_s_next are being built
  DevBuf<TetRec> d_tets_next;
  DevBuf<WRec> d_wrec_next;
  DevBuf<int4> d_tets_s_next;
  // [2] / [3]: tets of d_wrec / d_wrec_next with a far neighbour field (pmx_wrec.h), [4]: bad fans,
  // [5]: entries of the vertex-owner hint sample
  unsigned *h_nbad = nullptr;           // pinned [2]: non-manifold faces of that build, [1] of a background upload's
  DevBuf<double> d_nqual;
  bool have_qtag = false;               // raw tags of the new points
  DevBuf<uint16_t> d_qtag;
  int64_t pts_first = 0;                // points view's first index
  // the new tets of the points view: packed (validated, orphan marks) and
  // sent by the first pmx_run after the upload, once its step is enqueued --
  // their DMA on `up` overlaps the step and the results' download (the step
  // itself never reads them); consumers wait for ev_tets (ensure_tets)
  hipStream_t up = nullptr;
  hipEvent_t ev_tets = nullptr;
  char *h_tets = nullptr;               // pinned copy of the current new tets (int4, 0 = deleted);
  size_t h_tets_cap = 0;                // not the shared arena: it outlives the step (qualities' validity)
  bool tets_pending = false;            // view kept, not packed yet
  bool view_tets = false;               // the points view carried new tets (orphans exist by definition)
  bool tets_inflight = false;           // DMA issued on `up`, ev_tets recorded
  pmx_points_view tview{};
  bool orph_marks = false;              // d_qmark holds the device's marks of the packed new tets
  bool orph_fixed = true;               // the last step's orphan rows reset (fix_orphans)
  unsigned last_const_bit = 0;          // wmask bit of the last step's constant-size metric
  // PMX_RUN_EAGER_DOWNLOAD: the last step's fields (n * S doubles) and write
  // masks (n bytes) copied into h_out as soon as the step ends, in eager_nch
  // chunks (ev_eg); 0 = no such copy, or the results changed since
  char *h_out = nullptr;
  size_t h_out_cap = 0;
  int eager_nch = 0;
  hipEvent_t ev_eg[4] = {};
  DevBuf<double> d_gather;              // all-gathered partials

  // timing
  double topo_ms = 0.0;                 // device time of the last topology build
  std::vector<hipEvent_t> events;
  int ev_used = 0;

  hipEvent_t *next_event_slot();
  void free_all();
  bool order_hint_samples(int64_t ne, int64_t nverts, hipStream_t s);
  // PMX_RUN_FRESH_BACKGROUND: the per-background device passes of an upload
  // (face matching + records when the device built the adjacency, compact
  // records, owner sample), again on stream s (pmx_capi.hip)
  bool rederive(hipStream_t s);
  // the orphan marks of the new tets on stream s: d_qmark[j] = 1 when a valid
  // new tet holds point j (the reference's vertex loop, src/interpmesh_pmmg.c:535-541)
  bool mark_new_tets(hipStream_t s);
  // the fans by rotation (closed manifold surface, checked at the upload:
  // fan_rot) or by a sort; force 1: the counting sort
  bool fan_rot = false;
  bool fan_rotation(hipStream_t s, unsigned *d_bad, bool check = false);
  bool check_fans(hipStream_t s);
  // from d_tris, np, nt (pmx_bdy.hip); check: the rotation also re-counts every
  // vertex's trias, the upload's fan check (a FRESH step redoes it)
  bool build_node_trias(hipStream_t s, int force = 0, bool check = false);
  // the new points: kinds, lists (pmx_capi.hip); marks: the orphan marks
  // (d_qmark) classify points in no valid new tet as KIND_ORPH
  bool classify(hipStream_t s, bool marks = false);
  bool launch_bdy(const VolArgs &a, hipStream_t s);
  // PMX_RUN_SEQUENTIAL_SURFACE / _VOLUME after the step's passes, on stream s
  // (synchronises the host: a replayed query that ends stuck is scanned by a
  // launch of its own; pmx_bdy.hip)
  bool seq_replay(const VolArgs &a, hipStream_t s, bool surf, bool vol);
  bool size_tria_grid();
  bool pack_new_tets();                   // the pending new tets: pack, send on `up`, residency build
  bool ensure_tets(hipStream_t s);        // d_ntetv valid for work on stream s
  bool fix_orphans();                     // the last step's rows of orphan points: untouched
  bool eager_download();                  // issue the eager copies of the step just enqueued
  int4 *grow_htets(int64_t ne);           // h_tets for ne + 1 records (ev_tets already waited)
  // device error word of the last step (after a stream sync): 0 = none
  bool check_device_errors();
};

// grow-only device buffer (contents not kept); false + ctx->err on failure
template <class T> inline bool pmx_dgrow(pmx_ctx *ctx, DevBuf<T> &b, size_t n) {
  if (n <= b.cap && b.p) return true;
  if (b.p) hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  const hipError_t e = hipMalloc((void **)&b.p, std::max<size_t>(n, 1) * sizeof(T));
  if (e != hipSuccess) {
    ctx->err = std::string("hipMalloc: ") + hipGetErrorString(e);
    b.p = nullptr;
    return false;
  }
  b.cap = n;
  return true;
}
// the context's pinned staging arena, at least `bytes` (pmx_capi.hip)
char *pmx_hstage(pmx_ctx *ctx, size_t bytes);
// qualities dev[0..ne] (stream order) into the caller's array: stride 8
// (dense) writes qual[0..ne] with qual[0] = 0; any other stride (bytes, an
// AoS field such as &MMG5_Tetra[0].qual) writes only the tets that are valid
// in h_tets (deleted tets keep their value, as MMG3D_tetraQual skips
// !MG_EOK).  Chunked through the pinned arena, each chunk's host scatter
// overlapping the next one's DMA (pmx_capi.hip).
bool pmx_download_qual(pmx_ctx *ctx, const double *dev, int64_t ne, double *qual, int64_t stride);
// f(i0, i1) over [lo, hi) on the host pool (pmx_capi.hip)
void pmx_par_for(int64_t lo, int64_t hi, const std::function<void(int64_t, int64_t)> &f);

// face adjacency of device connectivity (1-based int4, slot 0 unused) into
// dadja (Mmg layout, 4 ne + 5 ints), context-owned scratch; false on a
// non-manifold face or a failure (ctx->err)
// h_nbad != NULL: asynchronous on stream s, the non-manifold count lands in
// *h_nbad (pinned) when the stream gets there; NULL: checked before returning
bool pmx_ctx_build_adja_device(pmx_ctx *ctx, const int4 *tv, int64_t ne, int64_t np, int *dadja,
                               hipStream_t s, unsigned *h_nbad);
extern "C" int pmx_timing_reset(pmx_ctx *ctx);
// error of a call made without a context (pmx_last_error(NULL), per thread)
void pmx_set_noctx_error(const char *msg);
