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

extern "C" {

int PMX_interpMetricsAndFields(pmx_ctx *ctx, int ngrp, pmx_group *grps, const int *permNodGlob,
                               int inputMet) {
  (void)permNodGlob;  // only used by the REQ copy, as in the reference (:477-484)
  if (!ctx) return 0;
  int ier = 1;
  for (int g = 0; g < ngrp; g++) {
    pmx_group &G = grps[g];
    const bool ismet = (inputMet == 1) && G.met && G.old_met && G.met->m && G.old_met->m;
    const bool cst = ismet && G.hsiz > 0.0;
    // reference early exit :509-512 (constant metric still set, :501-506)
    if (!ismet && G.nsols <= 0) continue;
    pmx_sol_view olds[PMX_MAX_SOLS], news[PMX_MAX_SOLS];
    int ns = 0, imet = -1;
    if (ismet) {
      olds[ns] = *G.old_met;
      news[ns] = *G.met;
      imet = ns++;
    }
    for (int j = 0; j < G.nsols; j++) {
      if (ns >= PMX_MAX_SOLS) { ctx->err = "too many solution fields"; return 0; }
      olds[ns] = G.old_fields[j];
      news[ns] = G.fields[j];
      ns++;
    }
    if (!pmx_upload_background(ctx, &G.old_mesh, ns, olds, imet)) return 0;
    if (!pmx_upload_points(ctx, &G.points)) return 0;
    pmx_run_opts o{};
    o.hsiz = cst ? G.hsiz : 0.0;
    if (!pmx_run(ctx, &o)) return 0;
    // outputs in Mmg layout start at point index `first`
    for (int s = 0; s < ns; s++)
      if (news[s].m) news[s].m += (int64_t)news[s].size * G.points.first;
    if (!pmx_download(ctx, news, nullptr, nullptr, nullptr)) ier = 0;
  }
  return ier;
}

}  // extern "C"

// copy of frozen (MG_REQ) points, optionally through the Scotch permutation
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
  if (inputMet && G->hsiz <= 0.0 && G->met && G->old_met) {   // :382
    olds.push_back(G->old_met);
    news.push_back(G->met);
  }
  for (int j = 0; j < G->nsols; j++) {
    olds.push_back(&G->old_fields[j]);
    news.push_back(&G->fields[j]);
  }
  if (olds.empty() || np < 1) return 1;
  int S = 0;
  for (auto *s : olds) S += s->size;
  std::vector<uint16_t> ht((size_t)(np + 1), 0);
  for (int64_t ip = 1; ip <= np; ip++)
    ht[(size_t)ip] = *(const uint16_t *)((const char *)old_tag + ip * old_tag_stride);
  std::vector<double> hs((size_t)(np + 1) * S, 0.0);
  {
    int off = 0;
    for (auto *s : olds) {
      for (int64_t ip = 1; ip <= np; ip++)
        for (int j = 0; j < s->size; j++) hs[(size_t)ip * S + off + j] = s->m[ip * s->size + j];
      off += s->size;
    }
  }
  const bool use_perm = renum && permNodGlob;
  uint16_t *dt = nullptr;
  int *dp = nullptr, *dcnt = nullptr, *ddst = nullptr;
  double *dold = nullptr, *dvals = nullptr;
  bool okk = hipMalloc((void **)&dt, ht.size() * 2) == hipSuccess &&
             hipMalloc((void **)&dold, hs.size() * 8) == hipSuccess &&
             hipMalloc((void **)&dcnt, 4) == hipSuccess &&
             hipMalloc((void **)&ddst, (size_t)(np + 1) * 4) == hipSuccess &&
             hipMalloc((void **)&dvals, (size_t)(np + 1) * S * 8) == hipSuccess &&
             (!use_perm || hipMalloc((void **)&dp, (size_t)(np + 1) * 4) == hipSuccess);
  int n = 0;
  if (okk) {
    hipStream_t st = ctx->stream;
    hipMemcpyAsync(dt, ht.data(), ht.size() * 2, hipMemcpyHostToDevice, st);
    hipMemcpyAsync(dold, hs.data(), hs.size() * 8, hipMemcpyHostToDevice, st);
    if (use_perm) hipMemcpyAsync(dp, permNodGlob, (size_t)(np + 1) * 4, hipMemcpyHostToDevice, st);
    hipMemsetAsync(dcnt, 0, 4, st);
    int64_t nb = std::min<int64_t>((np + 255) / 256, 4096);
    hipLaunchKernelGGL(k_copy_req, dim3((unsigned)nb), dim3(256), 0, st, dt, dp, np, dold, S,
                       dcnt, ddst, dvals);
    okk = hipStreamSynchronize(st) == hipSuccess &&
          hipMemcpy(&n, dcnt, 4, hipMemcpyDeviceToHost) == hipSuccess;
    if (okk && n > 0) {
      std::vector<int> hd((size_t)n);
      std::vector<double> hv((size_t)n * S);
      okk = hipMemcpy(hd.data(), ddst, (size_t)n * 4, hipMemcpyDeviceToHost) == hipSuccess &&
            hipMemcpy(hv.data(), dvals, (size_t)n * S * 8, hipMemcpyDeviceToHost) == hipSuccess;
      if (okk) {
        for (int q = 0; q < n; q++) {
          int off = 0;
          for (size_t s = 0; s < news.size(); s++) {
            const int sz = olds[s]->size;
            for (int j = 0; j < sz; j++)
              news[s]->m[(int64_t)hd[(size_t)q] * sz + j] = hv[(size_t)q * S + off + j];
            off += sz;
          }
        }
      }
    }
  }
  hipFree(dt); hipFree(dp); hipFree(dcnt); hipFree(ddst); hipFree(dold); hipFree(dvals);
  if (!okk) ctx->err = "PMX_copyMetricsAndFields_point: device copy failed";
  return okk ? 1 : 0;
}
