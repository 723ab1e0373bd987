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
  if (hipMemsetAsync(ctx->d_wmask.p, 0, (size_t)n, s) != hipSuccess) { ctx->err = "constant size: memset"; return 0; }
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

extern "C" {

int PMX_interpMetricsAndFields(pmx_ctx *ctx, int ngrp, pmx_group *grps, const int *permNodGlob,
                               int inputMet) {
  (void)permNodGlob;  // only used by the frozen-point copy, as in the reference (:477-484)
  if (!ctx || ngrp < 0 || (ngrp > 0 && !grps)) return 0;
  hipSetDevice(ctx->device);
  // a failing group makes the call fail but the other groups are still
  // processed (reference :715-721)
  int ier = 1;
  std::string first_err;
  auto fail = [&]() {
    ier = 0;
    if (first_err.empty()) first_err = ctx->err;
  };
  for (int g = 0; g < ngrp; g++) {
    pmx_group &G = grps[g];
    // reference :497-512: with -hsiz the metric is the constant one (written
    // whenever there is a metric array), otherwise it is interpolated when the
    // user gave one
    const bool cst = (inputMet == 1) && G.hsiz > 0.0 && G.met && G.met->m;
    const bool ismet = (inputMet == 1) && !(G.hsiz > 0.0) && G.met && G.met->m && G.old_met &&
                       G.old_met->m;
    if (G.nsols < 0 || G.nsols > PMX_MAX_SOLS || (G.nsols > 0 && (!G.fields || !G.old_fields))) {
      ctx->err = "PMX_interpMetricsAndFields: bad field list";
      fail();
      continue;
    }
    if (!ismet && !cst && G.nsols == 0) continue;   // nothing to do (:508-512)
    // the points of the new mesh's valid tets only (:535-541)
    pmx_points_view pv = G.points;
    if (!pv.tetra_v && G.mesh.tetra_v && G.mesh.ne > 0) {
      pv.tetra_v = G.mesh.tetra_v;
      pv.tetra_stride = G.mesh.tetra_stride;
      pv.ne = G.mesh.ne;
    }
    if (!pmx_upload_points(ctx, &pv)) { fail(); continue; }
    if (cst && !constant_metric(ctx, G.met, G.points.first, G.hsiz)) { fail(); continue; }
    if (!ismet && G.nsols == 0) continue;            // constant metric only: no locate
    pmx_sol_view olds[PMX_MAX_SOLS], news[PMX_MAX_SOLS];
    int ns = 0, imet = -1;
    if (ismet) {
      olds[ns] = *G.old_met;
      news[ns] = *G.met;
      imet = ns++;
    }
    bool bad = false;
    for (int j = 0; j < G.nsols; j++) {
      if (ns >= PMX_MAX_SOLS) { bad = true; break; }
      olds[ns] = G.old_fields[j];
      news[ns] = G.fields[j];
      ns++;
    }
    if (bad) { ctx->err = "PMX_interpMetricsAndFields: too many solution fields"; fail(); continue; }
    if (!pmx_upload_background(ctx, &G.old_mesh, ns, olds, imet)) { fail(); continue; }
    // the background upload invalidated nothing of the points; run the step
    pmx_run_opts o{};
    if (!pmx_run(ctx, &o)) { fail(); continue; }
    // outputs in Mmg layout start at point index `first`
    for (int s = 0; s < ns; s++)
      if (news[s].m) news[s].m += (int64_t)news[s].size * G.points.first;
    if (!pmx_download(ctx, news, nullptr, nullptr, nullptr)) fail();
  }
  if (!ier) ctx->err = first_err;
  return ier;
}

}  // extern "C"

// copy of frozen (MG_REQ) points, optionally through the Scotch permutation
// (PMMG_copySol_point, src/interpmesh_pmmg.c:311-358): compacted (dest, values)
__global__ void k_copy_req(const uint16_t *tag, const int *perm, int64_t np, const double *old,
                           int S, int *cnt, int *dst, double *vals) {
  for (int64_t ip = 1 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; ip <= np;
       ip += (int64_t)gridDim.x * blockDim.x) {
    unsigned t = tag[ip];
    if (t >= PMX_TAG_NUL) continue;          // MG_VOK
    if (!(t & PMX_TAG_REQ)) continue;
    int slot = atomicAdd(cnt, 1);
    dst[slot] = perm ? perm[ip] : (int)ip;
    for (int j = 0; j < S; j++) vals[(int64_t)slot * S + j] = old[ip * S + j];
  }
}

extern "C" int PMX_copyMetricsAndFields_point(pmx_ctx *ctx, pmx_group *G, const uint16_t *old_tag,
                                              int64_t old_tag_stride, const int *permNodGlob,
                                              int renum, int inputMet) {
  if (!ctx || !G) return 0;
  hipSetDevice(ctx->device);
  const int64_t np = G->old_mesh.np;
  std::vector<const pmx_sol_view *> olds, news;
  if (inputMet && G->hsiz <= 0.0 && G->met && G->old_met) {   // :378
    olds.push_back(G->old_met);
    news.push_back(G->met);
  }
  for (int j = 0; j < G->nsols; j++) {
    olds.push_back(&G->old_fields[j]);
    news.push_back(&G->fields[j]);
  }
  if (olds.empty() || np < 1) return 1;
  if (!old_tag) { ctx->err = "PMX_copyMetricsAndFields_point: old point tags required"; return 0; }
  int S = 0;
  for (auto *s : olds) {
    if (!s->m) { ctx->err = "PMX_copyMetricsAndFields_point: null solution"; return 0; }
    S += s->size;
  }
  const bool use_perm = renum && permNodGlob;
  // staging (pinned, reused): tags | permutation | interleaved old solutions
  const size_t b_tag = ((size_t)(np + 1) * 2 + 255) & ~(size_t)255;
  const size_t b_perm = use_perm ? (((size_t)(np + 1) * 4 + 255) & ~(size_t)255) : 0;
  const size_t b_sol = (size_t)(np + 1) * S * sizeof(double);
  char *st = pmx_hstage(ctx, b_tag + b_perm + b_sol);
  if (!st) return 0;
  uint16_t *ht = (uint16_t *)st;
  int *hp = (int *)(st + b_tag);
  double *hs = (double *)(st + b_tag + b_perm);
  ht[0] = 0;
  for (int64_t ip = 1; ip <= np; ip++)
    ht[ip] = *(const uint16_t *)((const char *)old_tag + ip * old_tag_stride);
  if (use_perm) memcpy(hp, permNodGlob, (size_t)(np + 1) * 4);
  {
    int off = 0;
    for (auto *s : olds) {
      for (int64_t ip = 1; ip <= np; ip++)
        for (int j = 0; j < s->size; j++) hs[(size_t)ip * S + off + j] = s->m[ip * s->size + j];
      off += s->size;
    }
  }
  hipStream_t s = ctx->stream;
  if (!pmx_dgrow(ctx, ctx->d_ctag, (size_t)(np + 1)) || !pmx_dgrow(ctx, ctx->d_cold, (size_t)(np + 1) * S) ||
      !pmx_dgrow(ctx, ctx->d_ccnt, 1) || !pmx_dgrow(ctx, ctx->d_cdst, (size_t)(np + 1)) ||
      !pmx_dgrow(ctx, ctx->d_cvals, (size_t)(np + 1) * S) ||
      (use_perm && !pmx_dgrow(ctx, ctx->d_cperm, (size_t)(np + 1))))
    return 0;
  bool okk = hipMemcpyAsync(ctx->d_ctag.p, ht, (size_t)(np + 1) * 2, hipMemcpyHostToDevice, s) == hipSuccess &&
             hipMemcpyAsync(ctx->d_cold.p, hs, b_sol, hipMemcpyHostToDevice, s) == hipSuccess &&
             (!use_perm || hipMemcpyAsync(ctx->d_cperm.p, hp, (size_t)(np + 1) * 4, hipMemcpyHostToDevice, s) == hipSuccess) &&
             hipMemsetAsync(ctx->d_ccnt.p, 0, 4, s) == hipSuccess;
  int n = 0;
  if (okk) {
    const int64_t nb = std::min<int64_t>((np + 255) / 256, 4096);
    hipLaunchKernelGGL(k_copy_req, dim3((unsigned)nb), dim3(256), 0, s, ctx->d_ctag.p,
                       use_perm ? ctx->d_cperm.p : nullptr, np, ctx->d_cold.p, S, ctx->d_ccnt.p,
                       ctx->d_cdst.p, ctx->d_cvals.p);
    okk = hipMemcpyAsync(&n, ctx->d_ccnt.p, 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
          hipStreamSynchronize(s) == hipSuccess;
  }
  if (okk && n > 0) {
    // the arena is free again (the uploads completed): the compacted entries
    int *hd = (int *)st;
    double *hv = (double *)(st + (((size_t)n * 4 + 255) & ~(size_t)255));
    okk = hipMemcpyAsync(hd, ctx->d_cdst.p, (size_t)n * 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
          hipMemcpyAsync(hv, ctx->d_cvals.p, (size_t)n * S * 8, hipMemcpyDeviceToHost, s) == hipSuccess &&
          hipStreamSynchronize(s) == hipSuccess;
    if (okk) {
      for (int q = 0; q < n; q++) {
        int off = 0;
        for (size_t k = 0; k < news.size(); k++) {
          const int sz = olds[k]->size;
          if (news[k]->m)
            for (int j = 0; j < sz; j++) news[k]->m[(int64_t)hd[q] * sz + j] = hv[(size_t)q * S + off + j];
          off += sz;
        }
      }
    }
  }
  if (!okk) ctx->err = "PMX_copyMetricsAndFields_point: device copy failed";
  return okk ? 1 : 0;
}
