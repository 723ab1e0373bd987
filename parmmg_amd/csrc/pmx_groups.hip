// pmx_groups.hip -- drop-in mirrors of the reference's group-level seams.
//
// PMX_interpMetricsAndFields      <- PMMG_interpMetricsAndFields
//                                    (reference src/interpmesh_pmmg.c:663-741)
// PMX_copyMetricsAndFields_point  <- PMMG_copyMetricsAndFields_point
//                                    (reference src/interpmesh_pmmg.c:311-446)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstring>
#include <vector>

#include "pmx_internal.h"
#include <string>

// MMG3D_Set_constantSize on the new points of the last pmx_upload_points,
// without a background (the reference's -hsiz shortcut, :501-506, also when no
// field needs a locate): written into the caller's Mmg-layout metric from
// entry `first` on, every valid point (kind != KIND_NUL)
static int constant_metric(pmx_ctx *ctx, const pmx_sol_view *met, int64_t first, double hsiz) {
  const int64_t n = ctx->nq;
  const int sz = met->size;
  if (n == 0) return 1;
  if (sz != 1 && sz != 6) { ctx->err = "constant size: metric size must be 1 or 6"; return 0; }
  if (!pmx_dgrow(ctx, ctx->d_cmet, (size_t)(n * sz))) return 0;
  hipStream_t s = ctx->stream;
  if (hipMemsetAsync(ctx->d_wmask.p, 0, (size_t)n, s) != hipSuccess) {
    ctx->err = "constant size: memset";
    return 0;
  }
  if (!ctx->classify(s)) return 0;       // kinds of the new points (NUL rows stay untouched)
  launch_const_metric(ctx->d_kind.p, n, ctx->d_cmet.p, sz, 0, sz, hsiz, ctx->d_wmask.p, 0, s);
  char *st = pmx_hstage(ctx, (size_t)n * sz * sizeof(double) + (size_t)n + 256);
  if (!st) return 0;
  double *h = (double *)st;
  uint8_t *wm = (uint8_t *)(st + (size_t)n * sz * sizeof(double));
  if (hipMemcpyAsync(h, ctx->d_cmet.p, (size_t)n * sz * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipMemcpyAsync(wm, ctx->d_wmask.p, (size_t)n, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    ctx->err = "constant size: download";
    return 0;
  }
  double *dst = met->m + first * sz;
  for (int64_t i = 0; i < n; i++)
    if (wm[i]) memcpy(dst + i * sz, h + i * sz, sizeof(double) * (size_t)sz);
  return 1;
}

// The group loop of PMMG_interpMetricsAndFields (src/interpmesh_pmmg.c:690-730)
// over contexts: group g on ctxs[g]; a context's pending download is done
// before the context takes its next group, the rest after every step is
// enqueued, so a group's host staging and upload overlap the steps of the
// groups before it.  A failing group makes the call fail but the other groups
// are still processed (reference :715-721); errors go to `ectx`.
static int interp_groups(pmx_ctx *ectx, pmx_ctx *const *ctxs, int ngrp, pmx_group *grps, int inputMet) {
  int ier = 1;
  std::string first_err;
  auto fail = [&](pmx_ctx *c) {
    ier = 0;
    if (first_err.empty()) first_err = c->err;
  };
  struct Pending {
    bool on = false;
    int ns = 0;
    int64_t cap = 0;                       // rows the caller's arrays hold from `first` on
    pmx_sol_view news[PMX_MAX_SOLS];
  };
  std::vector<Pending> pend((size_t)std::max(ngrp, 1));
  auto finish = [&](int g) {
    if (!pend[g].on) return;
    pend[g].on = false;
    if (!pmx_download(ctxs[g], pend[g].news, pend[g].cap, nullptr, nullptr, nullptr)) fail(ctxs[g]);
  };
  for (int g = 0; g < ngrp; g++) {
    pmx_ctx *X = ctxs[g];
    for (int h = 0; h < g; h++)             // the context's previous group, if any
      if (ctxs[h] == X) finish(h);
    pmx_group &G = grps[g];
    // reference :497-512: with -hsiz the metric is the constant one (written
    // whenever there is a metric array), otherwise it is interpolated when the
    // user gave one
    const bool cst = (inputMet == 1) && G.hsiz > 0.0 && G.met && G.met->m;
    const bool ismet = (inputMet == 1) && !(G.hsiz > 0.0) && G.met && G.met->m && G.old_met &&
                       G.old_met->m;
    if (G.nsols < 0 || G.nsols > PMX_MAX_SOLS || (G.nsols > 0 && (!G.fields || !G.old_fields))) {
      X->err = "PMX_interpMetricsAndFields: bad field list";
      fail(X);
      continue;
    }
    X->ran = false;                          // no step of this call yet on this context
    if (!ismet && !cst && G.nsols == 0) continue;   // nothing to do (:508-512)
    // the points of the new mesh's valid tets only (:535-541)
    pmx_points_view pv = G.points;
    if (!pv.tetra_v && G.mesh.tetra_v && G.mesh.ne > 0) {
      pv.tetra_v = G.mesh.tetra_v;
      pv.tetra_stride = G.mesh.tetra_stride;
      pv.ne = G.mesh.ne;
    }
    if (!pmx_upload_points(X, &pv)) { fail(X); continue; }
    if (cst && !constant_metric(X, G.met, G.points.first, G.hsiz)) { fail(X); continue; }
    if (!ismet && G.nsols == 0) continue;            // constant metric only: no locate
    pmx_sol_view olds[PMX_MAX_SOLS];
    Pending &P = pend[g];
    int ns = 0, imet = -1;
    if (ismet) {
      olds[ns] = *G.old_met;
      P.news[ns] = *G.met;
      imet = ns++;
    }
    bool bad = false;
    for (int j = 0; j < G.nsols; j++) {
      if (ns >= PMX_MAX_SOLS) { bad = true; break; }
      olds[ns] = G.old_fields[j];
      P.news[ns] = G.fields[j];
      ns++;
    }
    if (bad) { X->err = "PMX_interpMetricsAndFields: too many solution fields"; fail(X); continue; }
    if (!pmx_upload_background(X, &G.old_mesh, ns, olds, imet)) { fail(X); continue; }
    // the background upload invalidated nothing of the points; run the step
    pmx_run_opts o{};
    o.flags = PMX_RUN_EAGER_DOWNLOAD;        // every group is downloaded below
    // PMX_SEQUENTIAL=surface|volume|all: the reference's sequential
    // semantics (PMX_RUN_SEQUENTIAL_*; the points view carries the new tets)
    static const int seqf = [] {
      const char *e = getenv("PMX_SEQUENTIAL");
      if (!e) return 0;
      const std::string v(e);
      return (v == "surface" ? PMX_RUN_SEQUENTIAL_SURFACE : 0) | (v == "volume" ? PMX_RUN_SEQUENTIAL_VOLUME : 0) |
             (v == "all" || v == "1" ? PMX_RUN_SEQUENTIAL_SURFACE | PMX_RUN_SEQUENTIAL_VOLUME : 0);
    }();
    o.flags |= seqf;
    if (!pmx_run(X, &o)) { fail(X); continue; }
    // outputs in Mmg layout start at point index `first`
    for (int k = 0; k < ns; k++)
      if (P.news[k].m) P.news[k].m += (int64_t)P.news[k].size * G.points.first;
    P.ns = ns;
    // Mmg's arrays hold entries 0..np of the new mesh (its view's np when
    // given, else the points view's last)
    P.cap = (G.mesh.np > 0 ? G.mesh.np : G.points.last) + 1 - G.points.first;
    P.on = true;
  }
  for (int g = 0; g < ngrp; g++) finish(g);
  if (!ier) ectx->err = first_err;
  return ier;
}

extern "C" {

// Groups alternate between the context and a second one on the same device
// (created on first use): group g+1's host staging and upload overlap group
// g's step on the other context's streams, and group g's download waits until
// the context is needed again (g+2).
int PMX_interpMetricsAndFields(pmx_ctx *ctx, int ngrp, pmx_group *grps, const int *permNodGlob,
                               int inputMet) {
  (void)permNodGlob;  // only used by the frozen-point copy, as in the reference (:477-484)
  if (!ctx || ngrp < 0 || (ngrp > 0 && !grps)) return 0;
  hipSetDevice(ctx->device);
  if (ngrp > 1 && !ctx->peer) {
    ctx->peer = pmx_create(ctx->device);
    if (!ctx->peer) { ctx->err = "PMX_interpMetricsAndFields: second context"; return 0; }
  }
  std::vector<pmx_ctx *> cs((size_t)std::max(ngrp, 1));
  for (int g = 0; g < ngrp; g++) cs[(size_t)g] = (ngrp > 1 && (g & 1)) ? ctx->peer : ctx;
  return interp_groups(ctx, cs.data(), ngrp, grps, inputMet);
}

// One context per group (the caller's, e.g. kept across ParMmg iterations):
// every group's new points, new tets and results stay on its context for
// pmx_new_mesh_qual_synced until that context's next upload.
int PMX_interpMetricsAndFields_groups(pmx_ctx *const *ctxs, int ngrp, pmx_group *grps,
                                      const int *permNodGlob, int inputMet) {
  (void)permNodGlob;
  if (ngrp < 0 || (ngrp > 0 && (!ctxs || !grps))) return 0;
  for (int g = 0; g < ngrp; g++)
    if (!ctxs[g]) return 0;
  if (ngrp == 0) return 1;
  hipSetDevice(ctxs[0]->device);
  return interp_groups(ctxs[0], ctxs, ngrp, grps, inputMet);
}

}  // extern "C"

// copy of frozen (MG_REQ) points, optionally through the Scotch permutation
// (PMMG_copySol_point, src/interpmesh_pmmg.c:311-358).  The caller's arrays
// are host arrays, both sides: a host loop (an O(np) tag scan, REQ rows
// copied); no device round trip, so no context is needed either -- the
// reference calls it (src/libparmmg1.c:792) before the first interpolation
// has created one.  ctx may be NULL: errors then go to pmx_last_error(NULL).
// The device-resident variant is pmx_copy_required (below).
extern "C" int PMX_copyMetricsAndFields_point(pmx_ctx *ctx, pmx_group *G, const uint16_t *old_tag,
                                              int64_t old_tag_stride, const int *permNodGlob,
                                              int renum, int inputMet) {
  auto fail = [&](const char *msg) {
    if (ctx) ctx->err = msg;
    else pmx_set_noctx_error(msg);
    return 0;
  };
  if (!G) return fail("PMX_copyMetricsAndFields_point: null group");
  const int64_t np = G->old_mesh.np;
  std::vector<const pmx_sol_view *> olds, news;
  if (inputMet && G->hsiz <= 0.0 && G->met && G->old_met) {   // :378
    olds.push_back(G->old_met);
    news.push_back(G->met);
  }
  if (G->nsols < 0 || G->nsols > PMX_MAX_SOLS || (G->nsols > 0 && (!G->fields || !G->old_fields)))
    return fail("PMX_copyMetricsAndFields_point: bad field list");
  for (int j = 0; j < G->nsols; j++) {
    olds.push_back(&G->old_fields[j]);
    news.push_back(&G->fields[j]);
  }
  if (olds.empty() || np < 1) return 1;
  if (!old_tag) return fail("PMX_copyMetricsAndFields_point: old point tags required");
  for (size_t k = 0; k < olds.size(); k++)
    if (!olds[k]->m || olds[k]->size != news[k]->size)
      return fail("PMX_copyMetricsAndFields_point: null or mismatched solution");
  const bool use_perm = renum && permNodGlob;   // :328 (!oldMesh->info.renum || !permNodGlob)
  for (int64_t ip = 1; ip <= np; ip++) {
    const unsigned t = *(const uint16_t *)((const char *)old_tag + ip * old_tag_stride);
    if (t >= PMX_TAG_NUL || !(t & PMX_TAG_REQ)) continue;   // !MG_VOK / not frozen
    const int64_t dst = use_perm ? permNodGlob[ip] : ip;
    for (size_t k = 0; k < olds.size(); k++) {
      if (!news[k]->m) continue;
      const int sz = olds[k]->size;
      memcpy(news[k]->m + dst * sz, olds[k]->m + ip * sz, sizeof(double) * (size_t)sz);
    }
  }
  return 1;
}

// the same copy on device-resident data, after a step: rows of the new
// points the step did not write take the background's values of the old
// frozen points mapped to them -- equivalent to the reference's copy before
// the interpolation, which then overwrites the rows it writes
__global__ __launch_bounds__(256) void k_copy_required(const uint16_t *__restrict__ ptag, const int *__restrict__ perm,
                                                       int64_t np, int64_t first, int64_t n, const double *__restrict__ sol,
                                                       int S, SolDesc sd, unsigned smask, double *__restrict__ out,
                                                       uint8_t *__restrict__ wmask, unsigned *__restrict__ nbad) {
  for (int64_t ip = 1 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; ip <= np;
       ip += (int64_t)gridDim.x * blockDim.x) {
    const unsigned t = ptag[ip];
    if (t >= PMX_TAG_NUL || !(t & PMX_TAG_REQ)) continue;
    const int64_t j = (perm ? (int64_t)perm[ip] : ip) - first;
    if (j < 0 || j >= n) { atomicAdd(nbad, 1u); continue; }
    unsigned w = wmask[j];
    for (int s = 0; s < sd.nsol; s++) {
      const unsigned bit = 1u << s;
      if (!(smask & bit) || (w & bit)) continue;
      for (int c = 0; c < sd.size[s]; c++) out[j * S + sd.off[s] + c] = sol[ip * S + sd.off[s] + c];
      w |= bit;
    }
    wmask[j] = (uint8_t)w;
  }
}

extern "C" int pmx_copy_required(pmx_ctx *ctx, const int *permNodGlob, int copy_metric) {
  if (!ctx) return 0;
  hipSetDevice(ctx->device);
  if (!ctx->ran || !ctx->have_pts || ctx->out_n != ctx->nq || ctx->out_S != ctx->sd.S) {
    ctx->err = "pmx_copy_required: no step has run on the current uploads";
    return 0;
  }
  if (!ctx->have_ptag) { ctx->err = "pmx_copy_required: the background's point tags are not on the device"; return 0; }
  if (!ctx->fix_orphans()) return 0;
  const int64_t np = ctx->np;
  hipStream_t s = ctx->stream;
  if (permNodGlob) {
    if (!pmx_dgrow(ctx, ctx->d_cperm, (size_t)(np + 1))) return 0;
    if (hipMemcpyAsync(ctx->d_cperm.p, permNodGlob, (size_t)(np + 1) * sizeof(int), hipMemcpyHostToDevice, s) !=
        hipSuccess) {
      ctx->err = "pmx_copy_required: permutation upload";
      return 0;
    }
  }
  if (!pmx_dgrow(ctx, ctx->d_ccnt, 1) || hipMemsetAsync(ctx->d_ccnt.p, 0, sizeof(int), s) != hipSuccess) return 0;
  ctx->eager_nch = 0;                        // the results change: no eager copy of them
  unsigned smask = (1u << ctx->sd.nsol) - 1u;
  if (!copy_metric && ctx->sd.imet >= 0) smask &= ~(1u << ctx->sd.imet);
  const int64_t nb = std::max<int64_t>(1, std::min<int64_t>((np + 255) / 256, 4096));
  hipLaunchKernelGGL(k_copy_required, dim3((unsigned)nb), dim3(256), 0, s, ctx->d_ptag.p,
                     permNodGlob ? ctx->d_cperm.p : nullptr, np, ctx->pts_first, ctx->nq, ctx->d_sol.p,
                     ctx->sd.S, ctx->sd, smask, ctx->d_out.p, ctx->d_wmask.p, (unsigned *)ctx->d_ccnt.p);
  unsigned bad = 0;
  if (hipMemcpyAsync(&bad, ctx->d_ccnt.p, sizeof bad, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    ctx->err = "pmx_copy_required: launch";
    return 0;
  }
  if (bad) { ctx->err = "pmx_copy_required: a frozen point maps outside the new points"; return 0; }
  return 1;
}
