// pmx_capi.hip -- host side of the C ABI declared in include/pmx_transfer.h.
//
// Converts Mmg-style AoS (strided) meshes and solutions into the SoA device
// layout of pmx_device.h, owns the device buffers of one GPU, and sequences
// the kernels of one transfer step on one HIP stream.
#include <hip/hip_runtime.h>
#include <sched.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include <hipcub/hipcub.hpp>
#include "pmx_transfer.h"
#include "pmx_kernels.h"
#include "pmx_internal.h"

// events per recorded step: 0 start, 7 derived data built, 1 hint built,
// 2 volume walk done, 3/5 surface path start (node -> trias fans) / end (side
// stream), 6 joined, 4 end
#define PMX_EV_PER_RUN 8

// errors of the calls that work without a context (per host thread)
static thread_local std::string noctx_err;

// live contexts per device in this process (the fallback grids share the GPU)
static std::atomic<int> &live_contexts(int device) {
  static std::atomic<int> n[64];
  return n[device & 63];
}
void pmx_set_noctx_error(const char *msg) { noctx_err = msg; }

static bool ok(pmx_ctx *c, hipError_t e, const char *what) {
  if (e == hipSuccess) return true;
  c->err = std::string(what) + ": " + hipGetErrorString(e);
  return false;
}
#define CK(x) do { if (!ok(ctx, (x), #x)) return 0; } while (0)

template <class T> static bool dgrow(pmx_ctx *ctx, DevBuf<T> &b, size_t n) {
  return pmx_dgrow(ctx, b, n);
}
// pinned staging of at least `bytes`, 25 % slack so that a slowly growing
// ParMmg group does not re-pin every iteration.  Every arena copy is on the
// context's stream and no call waits for its last one (pmx_upload_points
// returns with its coordinates still in flight): the arena is handed out only
// once that stream has drained, so no host write, read or re-pin races a DMA.
char *pmx_hstage(pmx_ctx *ctx, size_t bytes) {
  if (!ok(ctx, hipStreamSynchronize(ctx->stream), "pmx_hstage: stream")) return nullptr;
  if (bytes <= ctx->h_stage_cap && ctx->h_stage) return (char *)ctx->h_stage;
  if (ctx->h_stage) hipHostFree(ctx->h_stage);
  ctx->h_stage = nullptr;
  ctx->h_stage_cap = 0;
  const size_t cap = std::max<size_t>(bytes + bytes / 4, 1 << 20);
  if (!ok(ctx, hipHostMalloc(&ctx->h_stage, cap, hipHostMallocDefault), "hipHostMalloc")) return nullptr;
  ctx->h_stage_cap = cap;
  return (char *)ctx->h_stage;
}
static char *hstage(pmx_ctx *ctx, size_t bytes) { return pmx_hstage(ctx, bytes); }
static size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

// The process's CPU share: the CPUs it may run on, capped by a cgroup v2 CPU
// quota (cpu.max "quota period"; a GPU box of this pool: 16 of 256).
static unsigned cpu_share() {
  cpu_set_t set;
  unsigned n = 0;
  if (sched_getaffinity(0, sizeof set, &set) == 0) n = (unsigned)CPU_COUNT(&set);
  if (!n) n = std::max(1u, std::thread::hardware_concurrency());
  if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    long long period = 0;
    if (fscanf(f, "%31s %lld", q, &period) == 2 && period > 0 && strcmp(q, "max") != 0) {
      const long long quota = atoll(q);
      if (quota > 0) n = std::min<unsigned>(n, (unsigned)std::max(1LL, (quota + period - 1) / period));
    }
    fclose(f);
  }
  return n;
}
// host gathers/scatters of large AoS arrays split over the CPU share
// (PMX_HOST_THREADS overrides; at most 32).  Measured on a GPU box (16-CPU
// quota of 256, C3 resident cycle, tools/trace_resident.py): 8 threads 89-95
// ms, 16 threads 67-71 ms, 24 threads (throttled by the quota) 77 ms.
// Ranges below PMX_HOST_THREADS_MIN elements (default 2^18) stay serial.
static unsigned host_threads() {
  static const unsigned T = [] {
    const char *e = getenv("PMX_HOST_THREADS");
    unsigned t = e ? (unsigned)std::max(1, atoi(e)) : cpu_share();
    return std::min(t, 32u);
  }();
  return T;
}
// streaming (non-temporal) 16-B stores into the pinned staging: the host
// never reads those lines again, and a plain store first reads each line for
// ownership (a third of the packing traffic).  PMX_NT_STORES=0: plain stores,
// for the A/B.  A pass ends with a full fence before its DMA is issued.
typedef int pmx_v4i __attribute__((ext_vector_type(4)));
static bool nt_stores() {
  static const bool on = [] {
    const char *e = getenv("PMX_NT_STORES");
    return !(e && e[0] == '0');
  }();
  return on;
}
static inline void st4(int4 *p, int a, int b, int c, int d, bool nt) {
  if (nt) {
    const pmx_v4i v = {a, b, c, d};
    __builtin_nontemporal_store(v, (pmx_v4i *)p);
  } else {
    *p = make_int4(a, b, c, d);
  }
}
static int64_t host_threads_min() {
  static const int64_t M = [] {
    const char *e = getenv("PMX_HOST_THREADS_MIN");
    return e ? std::max<int64_t>(1, atoll(e)) : (int64_t)(1 << 18);
  }();
  return M;
}
// PMX_TRACE=1: host phase timings of the staging calls on stderr
namespace {
struct Trace {
  const char *who;
  bool on;
  std::chrono::steady_clock::time_point t0, last;
  explicit Trace(const char *w) : who(w), on(getenv("PMX_TRACE") != nullptr) {
    if (on) t0 = last = std::chrono::steady_clock::now();
  }
  void mark(const char *what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[pmx] %s %-22s %8.3f ms\n", who, what,
            std::chrono::duration<double, std::milli>(now - last).count());
    last = now;
  }
};
}  // namespace

// a persistent pool of host_threads()-1 workers (thread creation per pass
// cost ~0.1 ms per pass and dominated the chunked copies); the calling thread
// takes part.  One job at a time (a mutex serialises concurrent callers).
namespace {
struct HostPool {
  std::mutex run_m;                      // one job at a time
  std::mutex m;
  std::condition_variable cv, done_cv;
  std::vector<std::thread> th;
  const std::function<void(int)> *job = nullptr;
  int njob = 0;
  std::atomic<int> next{0};
  int active = 0;
  unsigned gen = 0;
  bool stop = false;
  explicit HostPool(unsigned nworkers) {
    for (unsigned i = 0; i < nworkers; i++) th.emplace_back([this] { work(); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> g(m);
      stop = true;
    }
    cv.notify_all();
    for (auto &t : th) t.join();
  }
  void drain(const std::function<void(int)> &f, int n) {
    for (int i = next.fetch_add(1); i < n; i = next.fetch_add(1)) f(i);
  }
  void work() {
    unsigned seen = 0;
    for (;;) {
      const std::function<void(int)> *f;
      int n;
      {
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, [&] { return stop || gen != seen; });
        if (stop) return;
        seen = gen;
        f = job;
        n = njob;
        if (!f) continue;                  // woke after that job had finished
        active++;
      }
      drain(*f, n);
      {
        std::lock_guard<std::mutex> g(m);
        if (--active == 0) done_cv.notify_all();
      }
    }
  }
  void run(const std::function<void(int)> &f, int n) {
    std::lock_guard<std::mutex> r(run_m);
    {
      std::lock_guard<std::mutex> g(m);
      job = &f;
      njob = n;
      next.store(0);
      gen++;
    }
    cv.notify_all();
    drain(f, n);
    std::unique_lock<std::mutex> g(m);
    done_cv.wait(g, [&] { return active == 0 && next.load() >= n; });
    job = nullptr;
  }
};
HostPool &host_pool() {
  static HostPool *p = new HostPool(host_threads() - 1);   // never destroyed: no exit-time joins
  return *p;
}
}  // namespace

// f(chunk, lo, hi) over C contiguous chunks of [lo, hi); returns C
template <class F> static int par_chunks(int64_t lo, int64_t hi, F f) {
  const int64_t n = hi - lo;
  const int C = (host_threads() <= 1 || n < host_threads_min()) ? 1 : (int)host_threads();
  if (C == 1) { f(0, lo, hi); return 1; }
  const int64_t chunk = (n + C - 1) / C;
  const std::function<void(int)> job = [&](int i) {
    const int64_t a = lo + (int64_t)i * chunk, b = std::min(hi, a + chunk);
    f(i, a, std::max(a, b));
  };
  host_pool().run(job, C);
  return C;
}
template <class F> static void par_for(int64_t lo, int64_t hi, F f) {
  par_chunks(lo, hi, [&](int, int64_t a, int64_t b) { if (a < b) f(a, b); });
}
void pmx_par_for(int64_t lo, int64_t hi, const std::function<void(int64_t, int64_t)> &f) {
  par_for(lo, hi, f);
}

bool pmx_download_qual(pmx_ctx *ctx, const double *dev, int64_t ne, double *qual, int64_t stride) {
  const bool dense = stride == (int64_t)sizeof(double);
  const int4 *htv = (const int4 *)ctx->h_tets;
  if (!dense && (!htv || ctx->h_tets_cap < (size_t)(ne + 1) * sizeof(int4))) {
    ctx->err = "qualities: strided output needs the new tets' host copy";
    return false;
  }
  hipStream_t s = ctx->stream;
  char *st = hstage(ctx, (size_t)(ne + 1) * sizeof(double));
  if (!st) return false;
  const double *h = (const double *)st;
  char *out = (char *)qual;
  const bool nt_q = !dense && nt_stores() && ((uintptr_t)out % 8) == 0 && stride % 8 == 0;
  const int64_t nch = std::max<int64_t>(1, std::min<int64_t>(8, (ne + 1) >> 20));
  for (int64_t c = 0; c < nch; c++) {
    const int64_t lo = (ne + 1) * c / nch, hi = (ne + 1) * (c + 1) / nch;
    CK(hipMemcpyAsync(st + lo * 8, dev + lo, (size_t)(hi - lo) * 8, hipMemcpyDeviceToHost, s));
    CK(hipEventRecord(ctx->ev_dl[c], s));
  }
  for (int64_t c = 0; c < nch; c++) {
    const int64_t lo = (ne + 1) * c / nch, hi = (ne + 1) * (c + 1) / nch;
    CK(hipEventSynchronize(ctx->ev_dl[c]));
    if (dense) {
      par_for(lo, hi, [&](int64_t k0, int64_t k1) { memcpy(qual + k0, h + k0, (size_t)(k1 - k0) * 8); });
    } else if (nt_q) {
      // streaming 8-B stores into the records (8-B aligned field and stride):
      // no read for ownership of the caller's record lines
      par_for(std::max<int64_t>(lo, 1), hi, [&](int64_t k0, int64_t k1) {
        for (int64_t k = k0; k < k1; k++)
          if (htv[k].x) {
            long long bits;
            memcpy(&bits, &h[k], sizeof bits);
            __builtin_nontemporal_store(bits, (long long *)(out + k * stride));
          }
        std::atomic_thread_fence(std::memory_order_seq_cst);
      });
    } else {
      par_for(std::max<int64_t>(lo, 1), hi, [&](int64_t k0, int64_t k1) {
        for (int64_t k = k0; k < k1; k++)
          if (htv[k].x) memcpy(out + k * stride, &h[k], sizeof(double));   // any record alignment
      });
    }
  }
  if (dense) qual[0] = 0.0;
  return true;
}

// the pinned copy of the new tets, ne + 1 records
int4 *pmx_ctx::grow_htets(int64_t ne) {
  const size_t bytes = (size_t)(ne + 1) * sizeof(int4);
  if (bytes > h_tets_cap) {
    if (h_tets) hipHostFree(h_tets);
    h_tets = nullptr;
    h_tets_cap = 0;
    if (hipHostMalloc((void **)&h_tets, bytes, hipHostMallocDefault) != hipSuccess) {
      err = "pinned staging of the new tets";
      return nullptr;
    }
    h_tets_cap = bytes;
  }
  return (int4 *)h_tets;
}

template <class T> static void dfree(DevBuf<T> &b) {
  if (b.p) hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
}

bool pmx_ctx::check_device_errors() {
  if (!ran || !d_counts.p) return true;
  unsigned e = 0;
  if (hipMemcpy(&e, d_counts.p + PMX_CNT_ERR, sizeof e, hipMemcpyDeviceToHost) != hipSuccess) {
    err = "reading the step's device error word failed";
    return false;
  }
  if (e & PMX_DERR_BARRIER) {
    err = "k_fallback: a grid barrier timed out (workgroups not co-resident); the step's "
          "results are invalid";
    return false;
  }
  return true;
}

// boundary triangles of a mesh view -> TriRec records, validated against np
static bool stage_trias(pmx_ctx *ctx, const pmx_mesh_view *m, int64_t np, std::vector<TriRec> &htr) {
  const int64_t nt = m->nt;
  htr.assign((size_t)(nt + 1), TriRec{});
  if (nt < 1) return true;
  const char *rc = (const char *)m->tria_v;
  for (int64_t k = 1; k <= nt; k++) {
    const int *v = (const int *)(rc + k * m->tria_stride);
    TriRec &r = htr[(size_t)k];
    for (int l = 0; l < 3; l++) {
      r.v[l] = v[l];
      const int a = m->adjt[3 * (k - 1) + 1 + l];
      r.nb[l] = a / 3;
      if (v[l] < 1 || v[l] > np || a < 0 || a / 3 > nt) {
        ctx->err = "tria vertex or adjacency index out of range";
        return false;
      }
    }
  }
  return true;
}

// the volume hint grid over the background bbox [lo, hi] (about one cell per
// 6 tets) and the surface (tria) grid
static bool setup_grids(pmx_ctx *ctx, const double lo[3], const double hi[3], int64_t ne) {
  double ext[3], vol = 1.0;
  for (int a = 0; a < 3; a++) {
    ext[a] = std::max(hi[a] - lo[a], 1e-300);
    vol *= ext[a];
  }
  double target = std::max(1.0, (double)ne / 6.0);
  double h = std::cbrt(vol / target);
  GridDesc g;
  int64_t cells = 1;
  for (int a = 0; a < 3; a++) {
    // 1e-9 slack: libm cbrt is not correctly rounded, and 255.00000000000003
    // cells must stay 255 (r01: C3 got 256 per axis, misaligned with the
    // mesh: 10% empty cells, 0.73 instead of 0.44 cells start distance)
    int d = (int)std::ceil(ext[a] / h * (1.0 - 1e-9));
    d = std::max(1, std::min(d, 4096));
    g.dim[a] = d;
    int bits = 0;
    while ((1 << bits) < d) bits++;
    g.qf[a] = 21 - bits;
    g.lo[a] = lo[a];
    g.inv[a] = (double)d / ext[a];
    cells *= d;
  }
  ctx->grid = g;
  ctx->gcells = cells;
  for (int a = 0; a < 3; a++) { ctx->bblo[a] = lo[a]; ctx->bbhi[a] = hi[a]; }
  if (!ctx->size_tria_grid()) return false;
  return pmx_dgrow(ctx, ctx->d_grid, (size_t)cells);
}

// the background's derived layouts, decided per upload / promotion (A/B
// switches): PMX_WALK_RECORDS=compact builds the
// walk's 24-B records (a device pass per background: 1.26 ms at C3 for a walk
// 2 % faster); PMX_HINT_SAMPLE_ORDER=2 the vertex-owner hint sample (three
// device passes per background, 1.26 ms at C3, for a hint build 0.03 ms
// faster on a lexicographic numbering).  Defaults: neither -- no device pass
// per background beyond what every step does.
static bool env_compact_records() {
  const char *e = getenv("PMX_WALK_RECORDS");
  return e && strcmp(e, "compact") == 0;
}
static int env_sample_mode() {
  const char *e = getenv("PMX_HINT_SAMPLE_ORDER");
  return (e && atoi(e) == 2) ? 2 : 0;
}

extern "C" {

pmx_ctx *pmx_create(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return nullptr;
  if (device < 0) device = 0;
  device %= n;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  pmx_ctx *ctx = new pmx_ctx();
  ctx->device = device;
  // PMX_SIDE_CUS=N (measurement): the side stream on CUs [0, N), the main
  // stream on the rest (hipExtStreamCreateWithCUMask)
  int side_cus = 0;
  if (const char *e = getenv("PMX_SIDE_CUS")) side_cus = atoi(e);
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device);
  std::vector<uint32_t> mside, mmain;
  if (side_cus > 0 && side_cus < ncu) {
    mside.assign((size_t)(ncu + 31) / 32, 0u);
    mmain.assign((size_t)(ncu + 31) / 32, 0u);
    for (int c = 0; c < ncu; c++) (c < side_cus ? mside : mmain)[c / 32] |= 1u << (c % 32);
  }
  // HIP maps a process's streams onto a few hardware queues (4 by default,
  // GPU_MAX_HW_QUEUES) in creation order: a second context's streams share
  // the first one's queues, and two streams on one queue run one after the
  // other.  Contexts alternate their creation order so that the second one's
  // main and surface streams land on the first one's idle residency (topo)
  // and short-lived orphan-mark (up) queues instead of behind its walk
  // (PMX_interpMetricsAndFields runs two groups' steps side by side).
  static std::atomic<unsigned> n_created{0};
  const bool odd = (n_created.fetch_add(1) & 1u) != 0;
  // PMX_STREAM_PRIO=1 (A/B): the main stream at the device's greatest
  // priority, the orphan-mark stream at its least, so that the walk's
  // critical prefix (derived data, hint build) is dispatched first
  static const bool prio = [] {
    const char *e = getenv("PMX_STREAM_PRIO");
    return e && e[0] == '1';
  }();
  int p_least = 0, p_greatest = 0;
  if (prio) hipDeviceGetStreamPriorityRange(&p_least, &p_greatest);
  auto mk_main = [&] {
    if (mmain.empty() && prio) return hipStreamCreateWithPriority(&ctx->own, hipStreamNonBlocking, p_greatest);
    return mmain.empty() ? hipStreamCreateWithFlags(&ctx->own, hipStreamNonBlocking)
                         : hipExtStreamCreateWithCUMask(&ctx->own, (uint32_t)mmain.size(), mmain.data());
  };
  auto mk_up = [&] {
    return prio ? hipStreamCreateWithPriority(&ctx->up, hipStreamNonBlocking, p_least)
                : hipStreamCreateWithFlags(&ctx->up, hipStreamNonBlocking);
  };
  auto mk_side = [&] {
    return mside.empty() ? hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking)
                         : hipExtStreamCreateWithCUMask(&ctx->side, (uint32_t)mside.size(), mside.data());
  };
  bool sok;
  if (!odd)
    sok = mk_main() == hipSuccess && mk_side() == hipSuccess && mk_up() == hipSuccess &&
          hipStreamCreateWithFlags(&ctx->topo, hipStreamNonBlocking) == hipSuccess;
  else
    sok = hipStreamCreateWithFlags(&ctx->topo, hipStreamNonBlocking) == hipSuccess && mk_up() == hipSuccess &&
          mk_main() == hipSuccess && mk_side() == hipSuccess;
  ctx->stream = ctx->own;
  if (!sok ||
      hipEventCreateWithFlags(&ctx->ev_topo, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_tets, hipEventDisableTiming) != hipSuccess ||
      hipHostMalloc((void **)&ctx->h_nbad, 8 * sizeof(unsigned), hipHostMallocDefault) != hipSuccess ||
      [&] {
        for (auto &e : ctx->ev_dl)
          if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return true;
        for (auto &e : ctx->ev_eg)
          if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return true;
        return false;
      }() ||
      hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_fork2, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming) != hipSuccess) {
    pmx_destroy(ctx);
    return nullptr;
  }
  // the fallback's grid barrier needs every workgroup resident at once: size
  // its grid from the occupancy query, sharing the GPU with every live
  // context of this process (at least two: ParMmg groups of one rank, C4: 2
  // per GPU, PMX_interpMetricsAndFields' peer); re-sized in pmx_run when
  // contexts come and go.  Contexts of other processes on the same GPU are
  // not counted: one rank per GPU is the supported deployment.
  live_contexts(device)++;
  ctx->fallback_share = std::max(2, live_contexts(device).load());
  ctx->fallback_blocks = fallback_coresident_blocks(device, ctx->fallback_share);
  if (ctx->fallback_blocks < 1) {
    pmx_destroy(ctx);
    return nullptr;
  }
  return ctx;
}

void pmx_destroy(pmx_ctx *ctx) {
  if (!ctx) return;
  if (ctx->fallback_share > 0) live_contexts(ctx->device)--;
  if (ctx->peer) pmx_destroy(ctx->peer);
  ctx->peer = nullptr;
  hipSetDevice(ctx->device);
  if (ctx->stream) hipStreamSynchronize(ctx->stream);
  if (ctx->side) hipStreamSynchronize(ctx->side);
  if (ctx->topo) hipStreamSynchronize(ctx->topo);
  if (ctx->up) hipStreamSynchronize(ctx->up);
  ctx->free_all();
  for (auto &e : ctx->events) hipEventDestroy(e);
  if (ctx->ev_fork) hipEventDestroy(ctx->ev_fork);
  if (ctx->ev_fork2) hipEventDestroy(ctx->ev_fork2);
  if (ctx->ev_join) hipEventDestroy(ctx->ev_join);
  if (ctx->side) hipStreamDestroy(ctx->side);
  if (ctx->topo) hipStreamDestroy(ctx->topo);
  if (ctx->ev_topo) hipEventDestroy(ctx->ev_topo);
  if (ctx->ev_tets) hipEventDestroy(ctx->ev_tets);
  if (ctx->up) hipStreamDestroy(ctx->up);
  if (ctx->h_tets) hipHostFree(ctx->h_tets);
  for (auto &e : ctx->ev_dl)
    if (e) hipEventDestroy(e);
  for (auto &e : ctx->ev_eg)
    if (e) hipEventDestroy(e);
  if (ctx->h_out) hipHostFree(ctx->h_out);
  if (ctx->h_nbad) hipHostFree(ctx->h_nbad);
  if (ctx->own) hipStreamDestroy(ctx->own);
  delete ctx;
}

const char *pmx_last_error(pmx_ctx *ctx) {
  if (ctx) return ctx->err.c_str();
  return noctx_err.empty() ? "null context" : noctx_err.c_str();
}

int pmx_set_stream(pmx_ctx *ctx, void *s) {
  if (!ctx) return 0;
  ctx->stream = s ? (hipStream_t)s : ctx->own;
  return 1;
}

int pmx_synchronize(pmx_ctx *ctx) {
  if (!ctx) return 0;
  hipSetDevice(ctx->device);
  CK(hipStreamSynchronize(ctx->stream));
  return ctx->check_device_errors() ? 1 : 0;
}

int pmx_device_info(pmx_ctx *ctx, char *buf, int buflen) {
  if (!ctx) return 0;
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, ctx->device));
  snprintf(buf, (size_t)buflen, "%s %s CUs=%d HBM=%.1fGB", p.name, p.gcnArchName,
           p.multiProcessorCount, (double)p.totalGlobalMem / 1e9);
  return 1;
}

// ---- background upload ------------------------------------------------------

static bool check_background(pmx_ctx *ctx, const pmx_mesh_view *m, int nsol, const pmx_sol_view *sols,
                             int imet) {
  if (m->np < 1 || m->ne < 1 || m->nt < 0 || m->np >= (1LL << 31) - 1 || 4 * m->ne >= (1LL << 31)) {
    ctx->err = "pmx_upload_background: mesh sizes out of range";
    return false;
  }
  if (!m->point_c || !m->tetra_v || m->point_stride < 24 || m->tetra_stride < 16) {
    ctx->err = "pmx_upload_background: point_c / tetra_v missing or strides too small";
    return false;
  }
  if (nsol < 0 || nsol > PMX_MAX_SOLS || imet < -1 || imet >= nsol || (nsol > 0 && !sols)) {
    ctx->err = "pmx_upload_background: bad solution list";
    return false;
  }
  for (int s = 0; s < nsol; s++) {
    if (sols[s].size != 1 && sols[s].size != 3 && sols[s].size != 6) {
      ctx->err = "pmx_upload_background: solution size must be 1, 3 or 6";
      return false;
    }
    if (!sols[s].m) {
      ctx->err = "pmx_upload_background: null solution";
      return false;
    }
  }
  if (m->nt > 0 && (!m->tria_v || !m->adjt || m->tria_stride < 12)) {
    ctx->err = "pmx_upload_background: nt > 0 requires tria_v and adjt";
    return false;
  }
  return true;
}

int pmx_upload_background(pmx_ctx *ctx, const pmx_mesh_view *m, int nsol,
                          const pmx_sol_view *sols, int imet) {
  if (!ctx) return 0;
  // whatever happens below, the context holds no usable background until the
  // upload has completed (a failed call must not leave sizes that disagree
  // with the device buffers)
  ctx->have_bg = ctx->ran = ctx->have_derived = ctx->have_tetv = ctx->have_qual = false;
  ctx->eager_nch = 0;
  ctx->have_ptag = ctx->have_csr = ctx->have_surf = ctx->fan_rot = false;
  ctx->stat_np = -1;
  if (!m) { ctx->err = "pmx_upload_background: null mesh"; return 0; }
  hipSetDevice(ctx->device);
  if (!check_background(ctx, m, nsol, sols, imet)) return 0;
  const int64_t np = m->np, ne = m->ne, nt = m->nt;
  const bool dev_adja = m->adja == nullptr;   // no MMG3D_hashTetra on the host: device face matching
  ctx->compact_recs = env_compact_records();
  ctx->sample_mode = env_sample_mode();
  ctx->bg_btv = false;
  // the host packs the every-4th-tet hint sample with the tet records (the
  // device-adjacency path: k_build_tetrec writes it)
  const bool host_sample = !dev_adja && ctx->sample_mode == 0;
  // a residency build of the next background's records shares the adjacency
  // scratch: let it finish (its result, in the *_next buffers, is kept)
  if (ctx->next_topo) CK(hipStreamSynchronize(ctx->topo));
  Trace tr("background");
  SolDesc sd{};
  sd.nsol = nsol;
  sd.imet = imet;
  int S = 0;
  for (int s = 0; s < nsol; s++) {
    sd.size[s] = sols[s].size;
    sd.off[s] = S;
    S += sols[s].size;
  }
  sd.S = S;
  const int64_t ns = (ne + PMX_HINT_STRIDE - 1) / PMX_HINT_STRIDE;
  const size_t hs_n = (size_t)(np + 1) * std::max(S, 1);
  // pinned staging: xyz | tets (TetRec, or int4 when the device builds the
  // adjacency) | packed hint sample | solutions; each part goes down as soon
  // as it is packed (the tets in chunks), one sync at the end
  const size_t trec = dev_adja ? sizeof(int4) : sizeof(TetRec);
  const size_t o_p = 0, o_t = o_p + al256((size_t)(np + 1) * 24),
               o_h = o_t + al256((size_t)(ne + 1) * trec),
               o_s = o_h + al256(host_sample ? (size_t)ns * sizeof(int4) : 0),
               total = o_s + al256(hs_n * sizeof(double));
  CK(hipStreamSynchronize(ctx->stream));   // the arena may still feed an earlier copy
  char *stg = hstage(ctx, total);
  if (!stg) return 0;
  // any return after the topology fork first waits for that stream (a later
  // call may regrow the buffers its kernels use)
  struct StreamGuard {
    hipStream_t s = nullptr;
    ~StreamGuard() { if (s) hipStreamSynchronize(s); }
  } topo_guard;
  if (!dgrow(ctx, ctx->d_xyz, (size_t)(np + 1) * 3) || !dgrow(ctx, ctx->d_tets, (size_t)(ne + 1)) ||
      (ctx->compact_recs && !dgrow(ctx, ctx->d_wrec, (size_t)(ne + 1))) || !dgrow(ctx, ctx->d_wfar, 8) ||
      !dgrow(ctx, ctx->d_tets_s, (size_t)std::max<int64_t>(ns, 1)) || !dgrow(ctx, ctx->d_sol, hs_n) ||
      !dgrow(ctx, ctx->d_tris, (size_t)(nt + 1)) || !dgrow(ctx, ctx->d_trn, (size_t)(nt + 1)) ||
      !dgrow(ctx, ctx->d_xyzq, (size_t)(np + 1)) ||
      (dev_adja && (!dgrow(ctx, ctx->d_btv, (size_t)(ne + 1)) || !dgrow(ctx, ctx->d_adja, (size_t)(4 * ne + 5)))))
    return 0;
  hipStream_t st = ctx->stream;

  // points -> dense xyz (24 B), bounding box per chunk
  double *hp = (double *)(stg + o_p);
  hp[0] = hp[1] = hp[2] = 0.0;
  const char *pc = (const char *)m->point_c;
  double blo[64][3], bhi[64][3];
  const int nch = par_chunks(1, np + 1, [&](int c, int64_t i0, int64_t i1) {
    double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
    for (int64_t i = i0; i < i1; i++) {
      const double *cc = (const double *)(pc + i * m->point_stride);
      for (int a = 0; a < 3; a++) {
        hp[3 * i + a] = cc[a];
        lo[a] = std::min(lo[a], cc[a]);
        hi[a] = std::max(hi[a], cc[a]);
      }
    }
    for (int a = 0; a < 3; a++) { blo[c][a] = lo[a]; bhi[c][a] = hi[a]; }
  });
  double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
  for (int c = 0; c < nch; c++)
    for (int a = 0; a < 3; a++) { lo[a] = std::min(lo[a], blo[c][a]); hi[a] = std::max(hi[a], bhi[c][a]); }
  CK(hipMemcpyAsync(ctx->d_xyz.p, hp, (size_t)(np + 1) * 24, hipMemcpyHostToDevice, st));
  tr.mark("points");
  // tets -> TetRec with neighbour tet index (or the bare connectivity), + the
  // packed hint sample (the connectivity of every PMX_HINT_STRIDE-th tet,
  // contiguous: the hint build streams ne/4 * 16 B instead of touching every
  // line of the tet records); in chunks, each DMA'd while the next is packed
  TetRec *ht = (TetRec *)(stg + o_t);
  int4 *htv = (int4 *)(stg + o_t);
  int4 *hh = (int4 *)(stg + o_h);
  if (dev_adja) htv[0] = make_int4(0, 0, 0, 0);
  else memset(&ht[0], 0, sizeof(TetRec));
  const char *tc = (const char *)m->tetra_v;
  const int *adja_in = m->adja;
  bool bad = false;
  const bool ntst = nt_stores();
  const int64_t ntc = std::max<int64_t>(1, std::min<int64_t>(8, ne >> 20));
  for (int64_t c = 0; c < ntc; c++) {
    const int64_t klo = (c == 0) ? 0 : 1 + ne * c / ntc, khi = 1 + ne * (c + 1) / ntc;
    par_for(std::max<int64_t>(klo, 1), khi, [&](int64_t k0, int64_t k1) {
      bool b = false;
      for (int64_t k = k0; k < k1; k++) {
        const int *v = (const int *)(tc + k * m->tetra_stride);
        // indices the kernels will gather through: a valid tet (v[0] > 0,
        // MG_EOK) must name vertices 1..np and neighbours 0..ne
        const bool valid = v[0] > 0;
        if (dev_adja) {
          if (!valid) { st4(&htv[k], 0, 0, 0, 0, ntst); }
          else {
            for (int l = 0; l < 4; l++)
              if (v[l] < 1 || v[l] > np) b = true;
            st4(&htv[k], v[0], v[1], v[2], v[3], ntst);
          }
        } else {
          TetRec &r = ht[(size_t)k];
          for (int l = 0; l < 4; l++) {
            r.v[l] = v[l];
            const int a = adja_in[4 * (k - 1) + 1 + l];
            r.nb[l] = a / 4;
            if (valid && (v[l] < 1 || v[l] > np || a < 0 || a / 4 > ne)) b = true;
          }
        }
        if (host_sample && (k - 1) % PMX_HINT_STRIDE == 0)
          hh[(k - 1) / PMX_HINT_STRIDE] = make_int4(v[0], v[1], v[2], v[3]);
      }
      if (b) __atomic_store_n(&bad, true, __ATOMIC_RELAXED);
      std::atomic_thread_fence(std::memory_order_seq_cst);
    });
    if (bad) break;
    if (dev_adja)
      CK(hipMemcpyAsync(ctx->d_btv.p + klo, htv + klo, (size_t)(khi - klo) * sizeof(int4), hipMemcpyHostToDevice, st));
    else
      CK(hipMemcpyAsync(ctx->d_tets.p + klo, ht + klo, (size_t)(khi - klo) * sizeof(TetRec), hipMemcpyHostToDevice,
                        st));
  }
  if (bad) {
    ctx->err = "pmx_upload_background: tet vertex or adjacency index out of range";
    return 0;
  }
  ctx->h_nbad[2] = 0;                        // no far fields unless compact records are built
  if (!dev_adja) {
    if (host_sample)
      CK(hipMemcpyAsync(ctx->d_tets_s.p, hh, (size_t)ns * sizeof(int4), hipMemcpyHostToDevice, st));
    if (ctx->compact_recs) launch_build_wrec(ctx->d_tets.p, ne, ctx->d_wrec.p, ctx->d_wfar.p, ctx->h_nbad + 2, st);
    // the owner sample (mode 2) while the host packs the solutions and trias
    if (!ctx->order_hint_samples(ne, np, st)) return 0;
  }
  if (dev_adja) {
    // face matching on the device (pmx_topo.hip), then the tet records and
    // the hint sample from the device connectivity -- on the topology stream
    // as soon as the connectivity is down, overlapping the solutions' and
    // trias' packing and DMA; joined before the final sync
    CK(hipEventRecord(ctx->ev_fork, st));
    CK(hipStreamWaitEvent(ctx->topo, ctx->ev_fork, 0));
    topo_guard.s = ctx->topo;
    ctx->h_nbad[1] = 0;                      // [0] belongs to a pending residency build
    if (!pmx_ctx_build_adja_device(ctx, ctx->d_btv.p, ne, np, ctx->d_adja.p, ctx->topo, ctx->h_nbad + 1))
      return 0;
    launch_build_tetrec(ctx->d_btv.p, ctx->d_adja.p, ne, PMX_HINT_STRIDE, ctx->d_tets.p, ctx->d_tets_s.p,
                        ctx->topo);
    if (ctx->compact_recs)
      launch_build_wrec(ctx->d_tets.p, ne, ctx->d_wrec.p, ctx->d_wfar.p, ctx->h_nbad + 2, ctx->topo);
    if (!ctx->order_hint_samples(ne, np, ctx->topo)) return 0;
    CK(hipEventRecord(ctx->ev_join, ctx->topo));
  }
  tr.mark("tets");
  // solutions -> interleaved [np+1][S], in blocks of 1024 rows (each row's
  // line written while it is in cache, not once per solution) and chunks
  // whose DMA overlaps the packing of the next
  double *hs = (double *)(stg + o_s);
  // row 0: Mmg's unused slot, as the caller holds it (no kernel reads a
  // vertex 0 -- but PMMG_prilen's parallel edges with a tensor metric and
  // metRidTyp = 1 read met->m[ip] flat, src/quality_pmmg.c:466, i.e. row 0
  // for ip < 6)
  memset(hs, 0, (size_t)std::max(S, 1) * sizeof(double));
  for (int s = 0; s < nsol; s++)
    for (int j = 0; j < sols[s].size; j++) hs[sd.off[s] + j] = sols[s].m[j];
  if (S == 0) {
    memset(hs, 0, hs_n * sizeof(double));
    CK(hipMemcpyAsync(ctx->d_sol.p, hs, hs_n * sizeof(double), hipMemcpyHostToDevice, st));
  } else {
    const int64_t nsc = std::max<int64_t>(1, std::min<int64_t>(4, (np * S) >> 21));
    for (int64_t c = 0; c < nsc; c++) {
      const int64_t r0 = (c == 0) ? 0 : 1 + np * c / nsc, r1 = 1 + np * (c + 1) / nsc;
      par_for(std::max<int64_t>(r0, 1), r1, [&](int64_t i0, int64_t i1) {
        for (int64_t b0 = i0; b0 < i1; b0 += 1024) {
          const int64_t b1 = std::min(i1, b0 + 1024);
          for (int s = 0; s < nsol; s++) {
            const int sz = sols[s].size, off = sd.off[s];
            const double *src = sols[s].m;
            for (int64_t i = b0; i < b1; i++)
              for (int j = 0; j < sz; j++) hs[(size_t)i * S + off + j] = src[i * sz + j];
          }
        }
      });
      CK(hipMemcpyAsync(ctx->d_sol.p + r0 * S, hs + r0 * S, (size_t)((r1 - r0) * S) * sizeof(double),
                        hipMemcpyHostToDevice, st));
    }
  }
  tr.mark("solutions");
  // boundary triangles
  std::vector<TriRec> htr;
  if (!stage_trias(ctx, m, np, htr)) return 0;
  ctx->np = np; ctx->ne = ne; ctx->nt = nt; ctx->hausd = m->hausd;
  ctx->sd = sd;
  if (!setup_grids(ctx, lo, hi, ne)) return 0;
  CK(hipMemcpyAsync(ctx->d_tris.p, htr.data(), htr.size() * sizeof(TriRec), hipMemcpyHostToDevice, st));
  if (!ctx->check_fans(st)) return 0;
  // the node -> trias fans are the step's (pmx_run: PMMG_precompute_nodeTrias
  // runs inside the reference's call)
  if (dev_adja) CK(hipStreamWaitEvent(st, ctx->ev_join, 0));
  CK(hipGetLastError());
  tr.mark("trias + topology");
  CK(hipStreamSynchronize(ctx->stream));   // host staging vectors die here
  tr.mark("sync");
  if (dev_adja && ctx->h_nbad[1]) {
    ctx->err = "pmx_upload_background: non-manifold tet faces";
    return 0;
  }
  ctx->fan_rot = ctx->nt > 0 && ctx->h_nbad[4] == 0;
  ctx->nsamp = ctx->samples_owner ? (int64_t)ctx->h_nbad[5] : 0;
  ctx->bg_btv = dev_adja;
  ctx->have_bg = true;
  return 1;
}

int pmx_upload_points(pmx_ctx *ctx, const pmx_points_view *pv) {
  if (!ctx) return 0;
  ctx->have_pts = ctx->ran = false;
  ctx->have_ntet = false;                  // the new tets belong to the points
  Trace tr("points");
  if (ctx->next_topo) {                     // its buffers are about to be reused
    CK(hipStreamSynchronize(ctx->topo));
    ctx->next_topo = false;
  }
  if (ctx->tets_inflight) {                 // d_ntetv / h_tets are about to be reused
    CK(hipEventSynchronize(ctx->ev_tets));
    ctx->tets_inflight = false;
  }
  ctx->tets_pending = false;
  ctx->orph_marks = false;
  ctx->orph_fixed = true;
  ctx->eager_nch = 0;
  if (!pv) { ctx->err = "pmx_upload_points: null view"; return 0; }
  hipSetDevice(ctx->device);
  const int64_t n = pv->last - pv->first + 1;
  if (n < 0 || n >= (1LL << 31) || pv->first < 0 || (n > 0 && (!pv->c || pv->stride < 24))) {
    ctx->err = "pmx_upload_points: bad range or coordinates";
    return 0;
  }
  if (pv->tetra_v && (pv->ne < 0 || pv->tetra_stride < 16)) {
    ctx->err = "pmx_upload_points: bad new-tet view";
    return 0;
  }
  const size_t nn = (size_t)std::max<int64_t>(n, 1);
  // The host packs and sends only what the device cannot derive -- dense
  // coordinates (24 B), tags (2 B), the new tets (16 B) -- in a pinned
  // staging arena, chunked so that DMA overlaps packing.  The kinds, the
  // per-path lists (order-preserving compaction), the list-ordered volume
  // coordinates and the orphan marks are the step's work (pmx_run), as the
  // vertex loop and its tag dispatch are inside the reference's call
  // (src/interpmesh_pmmg.c:535-560).  The host's tag pass gives the launch
  // sizes (upper bounds: orphans are found on the device).
  const int64_t ntet = pv->tetra_v ? pv->ne : 0;
  const size_t o_x = 0, o_tg = o_x + al256(nn * 3 * sizeof(double)),
               total = o_tg + al256(pv->tag ? nn * 2 : 0);
  CK(hipStreamSynchronize(ctx->stream));   // the arena may still feed an earlier copy
  char *st = hstage(ctx, total);
  if (!st) return 0;
  double *hx = (double *)(st + o_x);
  uint16_t *htg = (uint16_t *)(st + o_tg);
  const char *pc = (const char *)pv->c;
  const char *tg = (const char *)pv->tag;
  if (!dgrow(ctx, ctx->d_qxyz, nn * 3) || !dgrow(ctx, ctx->d_kind, nn) || !dgrow(ctx, ctx->d_qmark, nn + 64) ||   // + 64: the marks' word-wide flush
      !dgrow(ctx, ctx->d_nsel, 2) || !dgrow(ctx, ctx->d_vollist, nn) || !dgrow(ctx, ctx->d_bdylist, nn) ||
      !dgrow(ctx, ctx->d_ctile, (size_t)std::max<int64_t>(cls_tiles(n), 1)) ||
      (tg && !dgrow(ctx, ctx->d_qtag, nn)) || (ntet && !dgrow(ctx, ctx->d_ntetv, (size_t)(ntet + 1))))
    return 0;
  // coordinates (+ bounding box: a promoted background's hint grid) and tags
  // (+ the per-path upper bounds)
  double qlo[64][3], qhi[64][3];
  int64_t cvol[64], cbdy[64];
  const int C = par_chunks(0, n, [&](int ci, int64_t j0, int64_t j1) {
    double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
    int64_t nv = 0, nb = 0;
    for (int64_t j = j0; j < j1; j++) {
      const double *c = (const double *)(pc + (pv->first + j) * pv->stride);
      for (int ax = 0; ax < 3; ax++) {
        hx[3 * j + ax] = c[ax];
        lo[ax] = std::min(lo[ax], c[ax]);
        hi[ax] = std::max(hi[ax], c[ax]);
      }
      if (tg) {
        const uint16_t t = *(const uint16_t *)(tg + (pv->first + j) * pv->tag_stride);
        htg[j] = t;
        const bool live = t < PMX_TAG_NUL && !(t & PMX_TAG_REQ);
        nv += (live && !(t & PMX_TAG_BDY)) ? 1 : 0;
        nb += (live && (t & PMX_TAG_BDY)) ? 1 : 0;
      }
    }
    for (int ax = 0; ax < 3; ax++) { qlo[ci][ax] = lo[ax]; qhi[ci][ax] = hi[ax]; }
    cvol[ci] = tg ? nv : j1 - j0;
    cbdy[ci] = nb;
  });
  ctx->nq_vol_ub = ctx->nq_bdy_ub = 0;
  for (int i = 0; i < C; i++) {
    ctx->nq_vol_ub += cvol[i];
    ctx->nq_bdy_ub += cbdy[i];
  }
  for (int ax = 0; ax < 3; ax++) {
    ctx->qlo[ax] = HUGE_VAL;
    ctx->qhi[ax] = -HUGE_VAL;
    for (int i = 0; i < C; i++) {
      ctx->qlo[ax] = std::min(ctx->qlo[ax], qlo[i][ax]);
      ctx->qhi[ax] = std::max(ctx->qhi[ax], qhi[i][ax]);
    }
  }
  if (n) {
    CK(hipMemcpyAsync(ctx->d_qxyz.p, hx, (size_t)n * 3 * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    if (tg) CK(hipMemcpyAsync(ctx->d_qtag.p, htg, (size_t)n * 2, hipMemcpyHostToDevice, ctx->stream));
  }
  tr.mark("coords");
  // the new tets are packed and sent by the first step on these points
  // (pack_new_tets): their DMA overlaps the step and the download
  ctx->tview = *pv;
  ctx->tets_pending = ntet > 0;
  ctx->view_tets = ntet > 0;
  ctx->nq = n;
  if (!dgrow(ctx, ctx->d_wmask, nn)) return 0;
  if (!dgrow(ctx, ctx->d_elem, nn)) return 0;
  if (!dgrow(ctx, ctx->d_status, nn)) return 0;
  if (!dgrow(ctx, ctx->d_steps, nn)) return 0;
  // points a step never locates (NUL, frozen, orphans) report element 0
  CK(hipMemsetAsync(ctx->d_elem.p, 0, nn * sizeof(int), ctx->stream));
  CK(hipMemsetAsync(ctx->d_status.p, 0, nn * sizeof(int), ctx->stream));
  CK(hipMemsetAsync(ctx->d_steps.p, 0, nn * sizeof(int), ctx->stream));
  if (!dgrow(ctx, ctx->d_start, nn)) return 0;
  if (!dgrow(ctx, ctx->d_edge, nn)) return 0;
  if (!dgrow(ctx, ctx->d_vertex, nn)) return 0;
  // start 0, edge / vertex unset (-1) for every point no step writes
  CK(hipMemsetAsync(ctx->d_start.p, 0, nn * sizeof(int), ctx->stream));
  CK(hipMemsetAsync(ctx->d_edge.p, 0xff, nn * sizeof(int), ctx->stream));
  CK(hipMemsetAsync(ctx->d_vertex.p, 0xff, nn * sizeof(int), ctx->stream));
  if (!dgrow(ctx, ctx->d_list, nn)) return 0;
  if (!dgrow(ctx, ctx->d_found, nn)) return 0;
  if (!dgrow(ctx, ctx->d_bestk, nn)) return 0;
  if (!dgrow(ctx, ctx->d_best, nn)) return 0;
  if (!dgrow(ctx, ctx->d_ties, nn)) return 0;
  if (!dgrow(ctx, ctx->d_counts, 32)) return 0;
  // one record per wave (sized for every point on one path)
  if (!dgrow(ctx, ctx->d_vstat, (nn + 255) / 256 * 4 + 4)) return 0;
  if (!dgrow(ctx, ctx->d_bstat, (nn + 255) / 256 * 4 + 4)) return 0;
  // no wait for the copies: the step queues behind them, and the next host
  // use of the arena waits for the stream (pmx_hstage)
  ctx->have_qtag = tg && n;
  ctx->pts_first = pv->first;
  // orphans (points in no valid new tet) are known once the tets are packed,
  // after the step: the step locates them too and fix_orphans resets their
  // rows before any consumer reads them (the reference never visits them,
  // src/interpmesh_pmmg.c:535-541)
  ctx->have_pts = true;
  ctx->have_ntet = ntet > 0;
  ctx->n_ntet = ntet;
  return 1;
}

// ---- the new tets, after the step (pack_new_tets) ------------------------------

// The points view's new tets (vertex = view index - first + 1), validated and
// packed in chunks into their own pinned staging (the shared arena serves the
// download meanwhile), each chunk's DMA on `up` overlapping the packing of
// the next.  Once they are on the device, a kernel on the same stream marks
// the points of valid tets -- the reference's vertex loop over the new tets
// (src/interpmesh_pmmg.c:535-541) -- so that the points in no valid tet
// (orphans: untouched, the reference never visits them) are known to
// fix_orphans.  With residency the next background's tet records are built
// from them on the topo stream once they have arrived.
bool pmx_ctx::pack_new_tets() {
  pmx_ctx *ctx = this;                     // CK()
  if (!tets_pending) return true;
  tets_pending = false;
  const pmx_points_view *pv = &tview;
  const int64_t n = nq, ntet = pv->ne;
  Trace tr("new tets");
  int4 *htv = grow_htets(ntet);
  if (!htv) return false;
  const char *tc = (const char *)pv->tetra_v;
  bool bad = false;
  htv[0] = make_int4(0, 0, 0, 0);
  const bool nt = nt_stores();
  const int64_t nch = std::max<int64_t>(1, std::min<int64_t>(8, ntet >> 20));
  for (int64_t c = 0; c < nch; c++) {
    const int64_t lo = (c == 0) ? 0 : 1 + ntet * c / nch, hi = 1 + ntet * (c + 1) / nch;
    par_for(std::max<int64_t>(lo, 1), hi, [&](int64_t k0, int64_t k1) {
      bool b = false;
      for (int64_t k = k0; k < k1; k++) {
        const int *v = (const int *)(tc + k * pv->tetra_stride);
        if (v[0] <= 0) { st4(&htv[k], 0, 0, 0, 0, nt); continue; }   // !MG_EOK
        int w[4];
        for (int l = 0; l < 4; l++) {
          int64_t jj = (int64_t)v[l] - pv->first;
          if (jj < 0 || jj >= n) { b = true; jj = 0; }
          w[l] = (int)(jj + 1);
        }
        st4(&htv[k], w[0], w[1], w[2], w[3], nt);
      }
      if (b) __atomic_store_n(&bad, true, __ATOMIC_RELAXED);
      std::atomic_thread_fence(std::memory_order_seq_cst);
    });
    if (bad) break;
    CK(hipMemcpyAsync(d_ntetv.p + lo, htv + lo, (size_t)(hi - lo) * sizeof(int4), hipMemcpyHostToDevice, up));
  }
  if (!bad && n > 0) {
    // the orphan marks, on the device once the tets are there (the host's
    // byte stores into a point-sized array cost as much as the packing)
    CK(hipMemsetAsync(d_qmark.p, 0, (size_t)n, up));
    launch_mark_new_tets(d_ntetv.p, ntet, d_qmark.p, n, up);
    CK(hipGetLastError());
    orph_marks = true;
  }
  CK(hipEventRecord(ev_tets, up));
  tets_inflight = true;
  if (bad) {
    err = "pmx_run: new tet vertex outside [first, last] of the points view";
    have_ntet = false;
    return false;
  }
  tr.mark("pack + dma issued");
  // residency: the next background's tet records (face adjacency built on
  // the device) on the topo stream, after the tets' DMA, while the step and
  // the download go on
  if (residency && ntet > 0) {
    const int64_t ns = (ntet + PMX_HINT_STRIDE - 1) / PMX_HINT_STRIDE;
    if (!dgrow(this, d_adja, (size_t)(4 * ntet + 5)) || !dgrow(this, d_tets_next, (size_t)(ntet + 1)) ||
        (compact_recs && !dgrow(this, d_wrec_next, (size_t)(ntet + 1))) || !dgrow(this, d_wfar, 8) ||
        !dgrow(this, d_tets_s_next, (size_t)std::max<int64_t>(ns, 1)))
      return false;
    *h_nbad = 0;
    CK(hipStreamWaitEvent(topo, ev_tets, 0));
    if (!pmx_ctx_build_adja_device(this, d_ntetv.p, ntet, n, d_adja.p, topo, h_nbad)) return false;
    launch_build_tetrec(d_ntetv.p, d_adja.p, ntet, PMX_HINT_STRIDE, d_tets_next.p, d_tets_s_next.p, topo);
    h_nbad[3] = 0;
    if (compact_recs) launch_build_wrec(d_tets_next.p, ntet, d_wrec_next.p, d_wfar.p + 1, h_nbad + 3, topo);
    CK(hipEventRecord(ev_topo, topo));
    next_topo = true;
  }
  return true;
}

// the new tets on the device before work on stream s reads them
bool pmx_ctx::ensure_tets(hipStream_t s) {
  pmx_ctx *ctx = this;
  if (tets_pending && !pack_new_tets()) return false;
  if (tets_inflight) CK(hipStreamWaitEvent(s, ev_tets, 0));
  return true;
}

// The last step located every live point; the orphans' rows go back to
// "never visited" -- no written solution bit (a constant-size metric stays:
// MMG3D_Set_constantSize writes every valid point), element / status / steps
// 0 -- on the stream, before any consumer of the results.
bool pmx_ctx::fix_orphans() {
  pmx_ctx *ctx = this;
  if (orph_fixed) return true;
  orph_fixed = true;
  if (!ran || !orph_marks || nq == 0) return true;
  if (tets_inflight) CK(hipStreamWaitEvent(stream, ev_tets, 0));   // the marks are written on `up`
  OrphanRows r{d_wmask.p, d_elem.p, d_status.p, d_steps.p, d_start.p, d_edge.p, d_vertex.p, d_kind.p};
  launch_orphans(d_qmark.p, nq, (uint8_t)last_const_bit, r, stream);
  CK(hipGetLastError());
  return true;
}

// The hint sample, once the tets are on the device and np set
// (sample_mode, PMX_HINT_SAMPLE_ORDER at the upload): 0 every 4th tet in tet
// order, packed with the tet records (nothing to do here); 2 one tet per
// vertex, in vertex order (k_vmin_owner; its count lands in h_nbad[5], nsamp
// after the upload's sync) -- A/Bs in DESIGN.md section 7 r05 / r06.  (r05's
// mode 1, the every-4th-tet sample sorted by smallest vertex, was dropped in
// r06: its sort could not be redone by a FRESH step.)
bool pmx_ctx::order_hint_samples(int64_t ne, int64_t np, hipStream_t s) {
  samples_sorted = samples_owner = false;
  if (sample_mode != 2 || np < 1 || ne < 1) return true;
  const size_t tb = owner_scan_temp_bytes(np);
  if (!dgrow(this, d_skey, (size_t)(np + 2)) || !dgrow(this, d_sidx, (size_t)(2 * (np + 1))) ||
      !dgrow(this, d_salt, (size_t)(np + 1)) || !dgrow(this, d_tets_sk, (size_t)(np + 1)) ||
      !dgrow(this, d_stmp, std::max<size_t>(tb, 1)) || !dgrow(this, d_wfar, 8))
    return false;
  if (!launch_owner_sample(d_tets.p, ne, np, d_skey.p, d_sidx.p, d_sidx.p + (np + 1), d_salt.p, d_tets_sk.p,
                           d_wfar.p + 4, h_nbad + 5, d_stmp.p, tb, s)) {
    err = "hint sample: vertex owners";
    return false;
  }
  std::swap(d_tets_s, d_salt);
  samples_sorted = samples_owner = true;
  return true;
}

// PMX_RUN_FRESH_BACKGROUND: the device passes an upload runs on the raw
// arrays, again, in stream order on s -- a ParMmg iteration brings a new
// background (PMMG_update_oldGrps, src/libparmmg1.c:653) and the reference
// recomputes its derived data inside the call (src/interpmesh_pmmg.c:514-518)
bool pmx_ctx::rederive(hipStream_t s) {
  pmx_ctx *ctx = this;                     // CK()
  if (bg_btv) {
    // face matching of the uploaded connectivity, then the tet records and
    // the every-4th-tet sample (MMG3D_hashTetra's adjacency on the device)
    if (!pmx_ctx_build_adja_device(this, d_btv.p, ne, np, d_adja.p, s, h_nbad + 1)) return false;
    launch_build_tetrec(d_btv.p, d_adja.p, ne, PMX_HINT_STRIDE, d_tets.p, d_tets_s.p, s);
  }
  if (compact_recs) launch_build_wrec(d_tets.p, ne, d_wrec.p, d_wfar.p, h_nbad + 2, s);
  if (sample_mode == 2 && !order_hint_samples(ne, np, s)) return false;
  CK(hipGetLastError());
  return true;
}

// the orphan marks from the device copy of the new tets (d_ntetv), on s
bool pmx_ctx::mark_new_tets(hipStream_t s) {
  pmx_ctx *ctx = this;
  if (nq < 1) return true;
  CK(hipMemsetAsync(d_qmark.p, 0, (size_t)nq, s));
  launch_mark_new_tets(d_ntetv.p, n_ntet, d_qmark.p, nq, s);
  CK(hipGetLastError());
  return true;
}

// ---- the step ---------------------------------------------------------------

static void fill_vol_args(pmx_ctx *ctx, const SolDesc &sd, const pmx_run_opts &opts, VolArgs &A) {
  A.xyz = ctx->d_xyz.p; A.tets = ctx->d_tets.p; A.wrec = ctx->d_wrec.p; A.sol = ctx->d_sol.p; A.sd = sd;
  A.q = ctx->d_qxyz.p; A.kind = ctx->d_kind.p; A.nq = ctx->nq; A.ne = ctx->ne;
  A.grid = ctx->d_grid.p; A.g = ctx->grid;
  A.out = ctx->d_out.p; A.wmask = ctx->d_wmask.p;
  A.elem = ctx->d_elem.p; A.status = ctx->d_status.p; A.steps = ctx->d_steps.p;
  A.start = ctx->d_start.p;
  A.stuck_list = ctx->d_list.p; A.stuck_count = ctx->d_counts.p;
  A.tie_list = ctx->d_ties.p; A.tie_count = ctx->d_counts.p + 3;
  A.found = ctx->d_found.p; A.bestk = ctx->d_bestk.p; A.best = ctx->d_best.p;
  A.list = ctx->d_vollist.p; A.nlist = ctx->nq_vol_ub; A.nlist_dev = ctx->d_nsel.p; A.wstats = ctx->d_vstat.p;
  A.max_walk = opts.max_walk > 0 ? opts.max_walk : 512;
  A.const_bit = sd.metric_const ? (1u << sd.imet) : 0u;
  A.inline_ties = (opts.flags & PMX_RUN_NO_INLINE_TIES) ? 0 : 1;
  A.ref_walk = (opts.flags & PMX_RUN_REFERENCE_WALK) ? 1 : 0;
  A.rec_start = (opts.flags & PMX_RUN_RECORD_STARTS) ? 1 : 0;
  A.exp = (opts.flags >> PMX_RUN_EXP_SHIFT) & 0xff;
  // the compact records resolve a far neighbour field when a walk crosses it
  // (a dependent read of the 32-B record); with many such tets the walk on
  // the 32-B records is faster (r05, C3: lex 0 % of the tets, compact 2 %
  // faster; 9 %, 32-B 1.5 % faster; appended 41 %, 32-B 5.5 % faster --
  // DESIGN.md section 7).  exp 18: compact records always
  if (!ctx->compact_recs ||
      (A.exp != 18 && (uint64_t)ctx->h_nbad[2] * PMX_WREC_FAR_DIV > (uint64_t)std::max<int64_t>(ctx->ne, 1)))
    A.wrec = nullptr;
  A.far = ctx->h_nbad[2] > 0 ? 1 : 0;
}

// pmx_run_opts.flags: the public PMX_RUN_* bits, plus the experiment switch
// in bits 16-23 (VolArgs.exp).  Switches that keep the results bit for bit
// (A/Bs of layouts, launch shapes and stream order) are always accepted; the
// measurement switches that skip work (4: no interpolation, 5: hint only)
// only when PMX_EXPERIMENTS=1 is set in the environment; anything else is
// refused, so that a stray bit never changes results silently.
static bool run_flags_valid(int flags, std::string *err) {
  const int pub = PMX_RUN_REFERENCE_WALK | PMX_RUN_NO_INLINE_TIES | PMX_RUN_RECORD_STARTS |
                  PMX_RUN_SERIAL_SURFACE | PMX_RUN_FRESH_BACKGROUND | PMX_RUN_DEBUG_BARRIER_TIMEOUT |
                  PMX_RUN_EAGER_DOWNLOAD | PMX_RUN_SEQUENTIAL_SURFACE | PMX_RUN_SEQUENTIAL_VOLUME;
  if (flags & ~(pub | (0xff << PMX_RUN_EXP_SHIFT))) {
    *err = "pmx_run: unknown flag bits";
    return false;
  }
  const int e = (flags >> PMX_RUN_EXP_SHIFT) & 0xff;
  switch (e) {
    case 0: case 6: case 9: case 10: case 11: case 12: case 13: case 15: case 16: case 17: case 18: case 19: case 20: case 21: case 22: case 23: case 24: case 25: case 26:
      return true;
    case 4: case 5: case 14: {
      const char *v = getenv("PMX_EXPERIMENTS");
      if (v && v[0] == '1') return true;
      *err = "pmx_run: measurement switch needs PMX_EXPERIMENTS=1";
      return false;
    }
    default:
      *err = "pmx_run: unknown experiment switch";
      return false;
  }
}

int pmx_run(pmx_ctx *ctx, const pmx_run_opts *o) {
  if (!ctx) return 0;
  ctx->ran = false;
  ctx->eager_nch = 0;
  if (!ctx->have_bg || !ctx->have_pts) { ctx->err = "pmx_run: upload background and points first"; return 0; }
  hipSetDevice(ctx->device);
  pmx_run_opts opts{};
  if (o) opts = *o;
  if (opts.hint_stride < 0 || opts.max_walk < 0) { ctx->err = "pmx_run: bad options"; return 0; }
  if (!run_flags_valid(opts.flags, &ctx->err)) return 0;
  const int64_t n = ctx->nq;
  const int S = ctx->sd.S;
  if (!dgrow(ctx, ctx->d_out, (size_t)std::max<int64_t>(n * S, 1))) return 0;
  SolDesc sd = ctx->sd;
  sd.metric_const = (opts.hsiz > 0.0 && sd.imet >= 0) ? 1 : 0;

  hipEvent_t *ev = nullptr;
  if (opts.timing) ev = ctx->next_event_slot();

  hipStream_t st = ctx->stream;
  // everything below is one iteration's device work on the uploaded raw
  // arrays: the per-background derived data (with PMX_RUN_FRESH_BACKGROUND,
  // or after an upload), the points' classification and compaction, the
  // node -> trias CSR (surface points only), hint grids, walks, fallback.
  // FRESH also redoes every device pass of the uploads (rederive: records,
  // samples, face matching; the fan check; the orphan marks of the new
  // tets): the step is then what a ParMmg iteration costs the device.
  const bool fresh = (opts.flags & PMX_RUN_FRESH_BACKGROUND) != 0;
  const bool derive = !ctx->have_derived || fresh;
  const bool csr = ctx->nq_bdy_ub > 0 && (!ctx->have_csr || fresh);
  // the orphan marks inside the step (FRESH with new tets): the new tets'
  // DMA must have landed (a pending points view is packed now)
  const bool marks = fresh && ctx->have_ntet && n > 0;
  if (marks && !ctx->ensure_tets(st)) return 0;
  if (ev) CK(hipEventRecord(ev[0], st));
  // one prologue kernel zeroes the write masks, the counters and the hint grid
  ZeroRanges z{};
  z.add(ctx->d_wmask.p, n);
  z.add(ctx->d_counts.p, 32 * sizeof(unsigned));
  z.add(ctx->d_grid.p, ctx->gcells * (int64_t)sizeof(int));
  launch_prologue(z, st);
  // the node -> trias fans (PMMG_precompute_nodeTrias, surface points only)
  // on the side stream from the start of the step: a small radix sort that
  // overlaps the derived data, the classification and the hint build
  const bool bdy = ctx->nq_bdy_ub > 0;
  const bool serial = (opts.flags & PMX_RUN_SERIAL_SURFACE) != 0;
  // (r03: the surface stream at the highest priority measured the same,
  // C3 2.093 vs 2.095 ms, profiles/r03_c3_sweep_surface_priority.log)
  hipStream_t side = ctx->side;
  hipStream_t ss = serial ? st : side;
  if (bdy && !serial) {
    CK(hipEventRecord(ctx->ev_fork, st));
    CK(hipStreamWaitEvent(side, ctx->ev_fork, 0));
  }
  // (on the side stream only once it has been forked from the main one: an
  // unforked side stream's event could precede ev[0])
  if (ev) CK(hipEventRecord(ev[3], bdy ? ss : st));
  // exp 19 (A/B): the fans on the main stream ahead of the derived data (a
  // few short kernels there, instead of passes starved on the side stream);
  // exp 20: the same with the counting sort over the vertex ids
  const int exp0 = (opts.flags >> PMX_RUN_EXP_SHIFT) & 0xff;
  // exp 25 (A/B, r06): the fans (and a FRESH step's fan check) on the side
  // stream after the classification, beside the walk instead of the prefix
  const bool fans_late = exp0 == 25 && bdy && !serial;
  if (bdy && csr && !fans_late) {
    if (!ctx->build_node_trias(exp0 == 19 || exp0 == 20 ? st : ss, exp0 == 20 ? 1 : 0, fresh)) return 0;
    ctx->have_csr = true;
  }
  // the orphan marks on `up`, beside the derived data and the hint build
  // (the classification waits for them)
  // exp 26 (A/B): the marks start after the derived data (which they slow
  // by sharing the memory system), beside the latency-bound hint build only
  const bool marks_after_derive = marks && exp0 == 26;
  auto launch_marks = [&]() -> bool {
    CK(hipEventRecord(ctx->ev_fork, st));
    CK(hipStreamWaitEvent(ctx->up, ctx->ev_fork, 0));
    if (!ctx->mark_new_tets(ctx->up)) return false;
    CK(hipEventRecord(ctx->ev_tets, ctx->up));
    ctx->tets_inflight = true;
    return true;
  };
  if (marks && !marks_after_derive && !launch_marks()) return 0;
  // exp 15 (A/B): no fixed-point copy of the vertices -- the hint build
  // quantises the sampled tets' vertices itself -- and the tria normals on
  // the surface stream
  const int exp = (opts.flags >> PMX_RUN_EXP_SHIFT) & 0xff;
  const bool hint_xyz = exp == 15 && (opts.hint_stride == 0 || opts.hint_stride == PMX_HINT_STRIDE);
  if (derive) {
    if (hint_xyz)
      launch_bg_derive(ctx->d_xyz.p, 0, ctx->grid, ctx->d_xyzq.p, ctx->d_tris.p, ctx->nt, ctx->d_trn.p,
                       (bdy && !serial) ? side : st);
    else if (bdy && !serial) {
      // the tria normals only feed the surface path: on its stream (r05:
      // the main stream's derived-data pass is the vertices alone)
      launch_bg_derive(ctx->d_xyz.p, ctx->np, ctx->grid, ctx->d_xyzq.p, ctx->d_tris.p, 0, ctx->d_trn.p, st);
      launch_bg_derive(ctx->d_xyz.p, 0, ctx->grid, ctx->d_xyzq.p, ctx->d_tris.p, ctx->nt, ctx->d_trn.p, side);
    } else {
      launch_bg_derive(ctx->d_xyz.p, ctx->np, ctx->grid, ctx->d_xyzq.p, ctx->d_tris.p, ctx->nt,
                       ctx->d_trn.p, st);
    }
    ctx->have_derived = !hint_xyz;
  }
  if (fresh && !ctx->rederive(st)) return 0;
  if (marks_after_derive && !launch_marks()) return 0;
  if (ev) CK(hipEventRecord(ev[7], st));
  // with the marks in the step, the hint build (which does not depend on the
  // points) goes ahead of the classification, beside the marks
  const int stride = opts.hint_stride > 0 ? opts.hint_stride : PMX_HINT_STRIDE;
  const bool packed = stride == PMX_HINT_STRIDE;
  bool any_interp = false;
  for (int s = 0; s < sd.nsol; s++)
    if (!(s == sd.imet && sd.metric_const)) any_interp = true;
  GridDesc g_hint = ctx->grid;
  auto hint_build = [&]() {
    launch_hint_build(packed ? ctx->d_tets_s.p : nullptr,
                      packed && ctx->samples_sorted ? ctx->d_tets_sk.p : nullptr, ctx->d_tets.p, ctx->ne,
                      stride, ctx->d_grid.p, g_hint, hint_xyz ? nullptr : ctx->d_xyzq.p, ctx->d_xyz.p, st,
                      exp == 16, exp == 21 ? 1024 : exp == 22 ? 64 : 256,
                      packed && ctx->samples_owner ? ctx->nsamp : -1);
  };
  // exp 23 (A/B): the marks beside the walk instead -- the points
  // classified without them, the orphans located and their rows reset at the
  // end of the step (k_orphans), the r05 order of the hint build
  const bool marks_late = marks && exp == 23;
  const bool hint_first = marks && !marks_late && any_interp;
  if (hint_first) hint_build();
  if (marks && !marks_late) CK(hipStreamWaitEvent(st, ctx->ev_tets, 0));
  if (!ctx->classify(st, marks && !marks_late)) return 0;
  if (sd.metric_const)
    launch_const_metric(ctx->d_kind.p, n, ctx->d_out.p, S, sd.off[sd.imet], sd.size[sd.imet],
                        opts.hsiz, ctx->d_wmask.p, sd.imet, st);
  // reference early exit (src/interpmesh_pmmg.c:508-512): nothing to locate
  if (!any_interp && bdy && !serial) {
    CK(hipEventRecord(ctx->ev_join, side));
    CK(hipStreamWaitEvent(st, ctx->ev_join, 0));
  }
  if (any_interp) {
    VolArgs A{};
    fill_vol_args(ctx, sd, opts, A);
    // the surface path on the side stream as soon as the points are
    // classified, latency-bound beside the hint build and the volume walk
    // (r03 A/B, profiles/r03_c{2,3,4}_sweep_surface_fork.log: C2 step 0.346 ->
    // 0.338 ms, C3 / C4 within 0.1 %); exp 9: forked after the hint build
    // (r01-r03 order: the r01 sweep had the hint build 40 % slower beside it)
    auto fork_surface = [&]() -> bool {
      if (!bdy || serial) return true;
      CK(hipEventRecord(ctx->ev_fork2, st));
      CK(hipStreamWaitEvent(side, ctx->ev_fork2, 0));
      if (fans_late && csr) {
        if (!ctx->build_node_trias(side, 0, fresh)) return false;
        ctx->have_csr = true;
      }
      if (!ctx->launch_bdy(A, side)) return false;
      if (ev) CK(hipEventRecord(ev[5], side));
      CK(hipEventRecord(ctx->ev_join, side));
      return true;
    };
    const bool early = A.exp != 9;
    if (early && !fork_surface()) return 0;
    if (!hint_first) hint_build();
    if (exp == 13 && A.wrec) {
      if (!dgrow(ctx, ctx->d_hrec, (size_t)(2 * ctx->gcells))) return 0;
      launch_hint_inline(ctx->d_grid.p, ctx->gcells, ctx->d_wrec.p, ctx->d_hrec.p, st);
      A.hrec = ctx->d_hrec.p;
    }
    if (ev) CK(hipEventRecord(ev[1], st));
    if (!early && !fork_surface()) return 0;
    if (ctx->nq_vol_ub) launch_walk(A, st);
    if (ev) CK(hipEventRecord(ev[2], st));
    if (bdy && !serial) {
      CK(hipStreamWaitEvent(st, ctx->ev_join, 0));     // surface path done
    } else if (bdy) {
      if (!ctx->launch_bdy(A, st)) return 0;
      if (ev) CK(hipEventRecord(ev[5], st));
    } else if (ev) {
      CK(hipEventRecord(ev[5], st));
    }
    if (ev) CK(hipEventRecord(ev[6], st));
    ExhArgs E{};
    E.xyz = ctx->d_xyz.p; E.tets = ctx->d_tets.p; E.ne = ctx->ne; E.q = ctx->d_qxyz.p;
    E.list = ctx->d_list.p; E.count = ctx->d_counts.p; E.found = ctx->d_found.p;
    E.best = ctx->d_best.p; E.bestk = ctx->d_bestk.p;
    E.spin_limit = (opts.flags & PMX_RUN_DEBUG_BARRIER_TIMEOUT) ? 0L : (1L << 26);
    const int share = std::max(2, live_contexts(ctx->device).load());
    if (share != ctx->fallback_share) {
      const int fb = fallback_coresident_blocks(ctx->device, share);
      if (fb < 1) { ctx->err = "pmx_run: occupancy query failed"; return 0; }
      ctx->fallback_blocks = fb;
      ctx->fallback_share = share;
    }
    if (ctx->nq_vol_ub) launch_exhaustive(E, A, ctx->fallback_blocks, st);
    // the reference's sequential semantics, after every default result
    ctx->seq_stats_n = -1;
    const bool sq_s = bdy && (opts.flags & PMX_RUN_SEQUENTIAL_SURFACE);
    const bool sq_v = ctx->nq_vol_ub > 0 && (opts.flags & PMX_RUN_SEQUENTIAL_VOLUME);
    if (opts.flags & (PMX_RUN_SEQUENTIAL_SURFACE | PMX_RUN_SEQUENTIAL_VOLUME)) {
      if (!ctx->seq_replay(A, st, sq_s, sq_v)) return 0;
      ctx->seq_stats_n = 1;
    }
    if (marks_late) {
      CK(hipStreamWaitEvent(st, ctx->ev_tets, 0));
      OrphanRows rr{ctx->d_wmask.p, ctx->d_elem.p, ctx->d_status.p, ctx->d_steps.p, ctx->d_start.p,
                    ctx->d_edge.p, ctx->d_vertex.p, ctx->d_kind.p};
      launch_orphans(ctx->d_qmark.p, n, (uint8_t)(sd.metric_const ? (1u << sd.imet) : 0u), rr, st);
    }
    if (ev) CK(hipEventRecord(ev[4], st));
  } else if (ev) {
    for (int k = 1; k < PMX_EV_PER_RUN; k++)
      if (k != 7 && k != 3) CK(hipEventRecord(ev[k], st));
  }
  CK(hipGetLastError());
  // the step located every live point: the orphans' rows are reset by the
  // first consumer of these results (fix_orphans); the new tets are packed
  // and sent now, while the device runs the step
  ctx->last_const_bit = sd.metric_const ? (1u << sd.imet) : 0u;
  // with the marks in the step, the orphans were never located (KIND_ORPH):
  // nothing to reset
  ctx->orph_fixed = marks;
  if (marks) ctx->orph_marks = true;
  ctx->out_S = S;
  ctx->out_n = n;
  if ((opts.flags & PMX_RUN_EAGER_DOWNLOAD) && !ctx->eager_download()) return 0;
  if (ctx->tets_pending && !ctx->pack_new_tets()) return 0;
  ctx->ran = true;
  return 1;
}

// The fields and write masks of the step just enqueued, down into h_out (its
// own pinned buffer: the arena stays free for the calls in between) in chunks
// on the step's stream.  The orphan reset (fix_orphans, later) changes masks
// only: pmx_download takes them again.
bool pmx_ctx::eager_download() {
  pmx_ctx *ctx = this;
  eager_nch = 0;
  const int64_t n = nq;
  const int S = sd.S;
  if (n == 0 || S == 0) return true;
  const size_t o_wm = al256((size_t)(n * S) * sizeof(double)), bytes = o_wm + al256((size_t)n);
  if (bytes > h_out_cap) {
    CK(hipStreamSynchronize(stream));      // an earlier eager copy may still land in it
    if (h_out) hipHostFree(h_out);
    h_out = nullptr;
    h_out_cap = 0;
    if (hipHostMalloc((void **)&h_out, bytes + bytes / 4, hipHostMallocDefault) != hipSuccess) {
      err = "pmx_run: pinned staging of the eager download";
      return false;
    }
    h_out_cap = bytes + bytes / 4;
  }
  const int nch = (int)std::max<int64_t>(1, std::min<int64_t>(4, (n * S) >> 21));
  for (int c = 0; c < nch; c++) {
    const int64_t lo = n * c / nch, hi = n * (c + 1) / nch;
    CK(hipMemcpyAsync(h_out + (size_t)(lo * S) * sizeof(double), d_out.p + lo * S,
                      (size_t)((hi - lo) * S) * sizeof(double), hipMemcpyDeviceToHost, stream));
    CK(hipMemcpyAsync(h_out + o_wm + lo, d_wmask.p + lo, (size_t)(hi - lo), hipMemcpyDeviceToHost, stream));
    CK(hipEventRecord(ev_eg[c], stream));
  }
  eager_nch = nch;
  return true;
}

// results of the last step, consistent with the current uploads
static bool results_ready(pmx_ctx *ctx, const char *who) {
  if (!ctx->ran || !ctx->have_pts || !ctx->have_bg || ctx->out_n != ctx->nq || ctx->out_S != ctx->sd.S) {
    ctx->err = std::string(who) + ": no step has run on the current uploads";
    return false;
  }
  return true;
}

// The step's rows [i0, i1) of the packed fields h (S doubles per point) into
// the caller's per-solution arrays where the write mask has the solution's
// bit.  In blocks of 1024 points, so that every solution reads a block of h
// from cache (solution by solution over the whole range read h once per
// solution).
static void scatter_rows(const pmx_ctx *ctx, const pmx_sol_view *new_sols, const double *h, const uint8_t *wm,
                         int64_t i0, int64_t i1) {
  const int S = ctx->sd.S;
  // streaming 8-B stores (no read for ownership of the caller's lines; the
  // arrays are far larger than the caches anyway); PMX_NT_STORES=0: plain
  const bool nt = nt_stores();
  for (int64_t b0 = i0; b0 < i1; b0 += 1024) {
    const int64_t b1 = std::min(i1, b0 + 1024);
    for (int s = 0; s < ctx->sd.nsol; s++) {
      double *dst = new_sols[s].m;
      if (!dst) continue;
      const int sz = ctx->sd.size[s], off = ctx->sd.off[s];
      const unsigned bit = 1u << s;
      for (int64_t i = b0; i < b1; i++) {
        if (!(wm[i] & bit)) continue;
        const double *src = h + i * S + off;
        double *d = dst + i * sz;
        if (nt) {
          for (int j = 0; j < sz; j++) {
            long long bits;
            memcpy(&bits, &src[j], sizeof bits);
            __builtin_nontemporal_store(bits, (long long *)&d[j]);
          }
        } else {
          for (int j = 0; j < sz; j++) d[j] = src[j];
        }
      }
    }
  }
  if (nt) std::atomic_thread_fence(std::memory_order_seq_cst);   // the caller reads them next
}

// pmx_download after a PMX_RUN_EAGER_DOWNLOAD step: the fields are (being)
// copied into h_out; each chunk is scattered once it has landed.  elem /
// status / steps come down as usual (after fix_orphans).
static int download_eager(pmx_ctx *ctx, const pmx_sol_view *new_sols, int *elem, int *status, int *steps) {
  const int64_t n = ctx->nq;
  const int S = ctx->sd.S;
  const double *h = (const double *)ctx->h_out;
  const uint8_t *wm = (const uint8_t *)(ctx->h_out + al256((size_t)(n * S) * sizeof(double)));
  // the eager copy holds the step's masks; with new tets, the orphan reset
  // (fix_orphans, enqueued by pmx_download after them) changed some: take the
  // masks again (n bytes)
  if (ctx->orph_marks) {
    CK(hipMemcpyAsync(const_cast<uint8_t *>(wm), ctx->d_wmask.p, (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
    CK(hipStreamSynchronize(ctx->stream));
  }
  const bool want_int = elem || status || steps;
  const size_t o_el = 0, o_st = o_el + al256((size_t)n * sizeof(int)), o_sp = o_st + al256((size_t)n * sizeof(int)),
               total = o_sp + al256((size_t)n * sizeof(int));
  char *st = nullptr;
  if (want_int) {
    st = hstage(ctx, total);               // waits for the stream: the eager chunks have landed
    if (!st) return 0;
    if (elem) CK(hipMemcpyAsync(st + o_el, ctx->d_elem.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    if (status) CK(hipMemcpyAsync(st + o_st, ctx->d_status.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    if (steps) CK(hipMemcpyAsync(st + o_sp, ctx->d_steps.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  }
  const int nch = ctx->eager_nch;
  for (int c = 0; c < nch; c++) {
    const int64_t lo = n * c / nch, hi = n * (c + 1) / nch;
    CK(hipEventSynchronize(ctx->ev_eg[c]));
    par_for(lo, hi, [&](int64_t i0, int64_t i1) { scatter_rows(ctx, new_sols, h, wm, i0, i1); });
  }
  if (want_int) {
    CK(hipStreamSynchronize(ctx->stream));
    if (elem) memcpy(elem, st + o_el, (size_t)n * sizeof(int));
    if (status) memcpy(status, st + o_st, (size_t)n * sizeof(int));
    if (steps) memcpy(steps, st + o_sp, (size_t)n * sizeof(int));
  }
  return 1;
}

// the caller's host arrays must hold the points of the step (npts rows):
// refused before anything is written (r04: an output sized by a wrong count
// was written past on the host)
static bool check_cap(pmx_ctx *ctx, const char *who, int64_t cap, int64_t need) {
  if (cap >= need) return true;
  ctx->err = std::string(who) + ": output capacity " + std::to_string(cap) + " < " + std::to_string(need) +
             " entries needed";
  return false;
}

int pmx_download(pmx_ctx *ctx, const pmx_sol_view *new_sols, int64_t npts_cap, int *elem, int *status,
                 int *steps) {
  if (!ctx) return 0;
  if (!results_ready(ctx, "pmx_download")) return 0;
  if (!check_cap(ctx, "pmx_download", npts_cap, ctx->nq)) return 0;
  hipSetDevice(ctx->device);
  if (!ctx->fix_orphans()) return 0;
  const int64_t n = ctx->nq;
  const int S = ctx->sd.S;
  CK(hipStreamSynchronize(ctx->stream));
  if (!ctx->check_device_errors()) return 0;
  if (n == 0) return 1;   // empty step: nothing to copy
  // every device -> host copy lands in the pinned arena (async DMA, one sync),
  // then the host scatters into the caller's (pageable, strided) arrays
  const bool want_sol = new_sols && S > 0;
  if (want_sol && ctx->eager_nch > 0) return download_eager(ctx, new_sols, elem, status, steps);
  const size_t o_out = 0, o_wm = o_out + al256(want_sol ? (size_t)(n * S) * sizeof(double) : 0),
               o_el = o_wm + al256(want_sol ? (size_t)n : 0), o_st = o_el + al256((size_t)n * sizeof(int)),
               o_sp = o_st + al256((size_t)n * sizeof(int)), total = o_sp + al256((size_t)n * sizeof(int));
  char *st = hstage(ctx, total);
  if (!st) return 0;
  const double *h = (const double *)(st + o_out);
  const uint8_t *wm = (const uint8_t *)(st + o_wm);
  // the fields in chunks: a chunk's scatter into the caller's arrays overlaps
  // the DMA of the next one
  const int64_t nch = want_sol ? std::max<int64_t>(1, std::min<int64_t>(4, (n * S) >> 21)) : 0;
  for (int64_t c = 0; c < nch; c++) {
    const int64_t lo = n * c / nch, hi = n * (c + 1) / nch;
    CK(hipMemcpyAsync(st + o_out + (size_t)(lo * S) * sizeof(double), ctx->d_out.p + lo * S,
                      (size_t)((hi - lo) * S) * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    CK(hipMemcpyAsync(st + o_wm + lo, ctx->d_wmask.p + lo, (size_t)(hi - lo), hipMemcpyDeviceToHost, ctx->stream));
    CK(hipEventRecord(ctx->ev_dl[c], ctx->stream));
  }
  if (elem) CK(hipMemcpyAsync(st + o_el, ctx->d_elem.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  if (status) CK(hipMemcpyAsync(st + o_st, ctx->d_status.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  if (steps) CK(hipMemcpyAsync(st + o_sp, ctx->d_steps.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  for (int64_t c = 0; c < nch; c++) {
    const int64_t lo = n * c / nch, hi = n * (c + 1) / nch;
    CK(hipEventSynchronize(ctx->ev_dl[c]));
    par_for(lo, hi, [&](int64_t i0, int64_t i1) { scatter_rows(ctx, new_sols, h, wm, i0, i1); });
  }
  CK(hipStreamSynchronize(ctx->stream));
  if (elem) memcpy(elem, st + o_el, (size_t)n * sizeof(int));
  if (status) memcpy(status, st + o_st, (size_t)n * sizeof(int));
  if (steps) memcpy(steps, st + o_sp, (size_t)n * sizeof(int));
  return 1;
}

int pmx_download_starts(pmx_ctx *ctx, int *start, int64_t cap) {
  if (!ctx || !start) return 0;
  if (!results_ready(ctx, "pmx_download_starts")) return 0;
  if (!check_cap(ctx, "pmx_download_starts", cap, ctx->nq)) return 0;
  hipSetDevice(ctx->device);
  if (!ctx->fix_orphans()) return 0;
  CK(hipStreamSynchronize(ctx->stream));
  if (!ctx->check_device_errors()) return 0;
  if (ctx->nq == 0) return 1;
  CK(hipMemcpy(start, ctx->d_start.p, (size_t)ctx->nq * sizeof(int), hipMemcpyDeviceToHost));
  return 1;
}

int pmx_download_border(pmx_ctx *ctx, int *edge, int *vertex, int64_t cap) {
  if (!ctx) return 0;
  if (!results_ready(ctx, "pmx_download_border")) return 0;
  if (!check_cap(ctx, "pmx_download_border", cap, ctx->nq)) return 0;
  hipSetDevice(ctx->device);
  if (!ctx->fix_orphans()) return 0;
  CK(hipStreamSynchronize(ctx->stream));
  if (!ctx->check_device_errors()) return 0;
  if (ctx->nq == 0) return 1;
  if (edge) CK(hipMemcpy(edge, ctx->d_edge.p, (size_t)ctx->nq * sizeof(int), hipMemcpyDeviceToHost));
  if (vertex) CK(hipMemcpy(vertex, ctx->d_vertex.p, (size_t)ctx->nq * sizeof(int), hipMemcpyDeviceToHost));
  return 1;
}

int pmx_locate_stats_get(pmx_ctx *ctx, pmx_locate_stats *st) {
  if (!ctx || !st) return 0;
  if (!results_ready(ctx, "pmx_locate_stats_get")) return 0;
  hipSetDevice(ctx->device);
  if (!ctx->fix_orphans()) return 0;
  CK(hipStreamSynchronize(ctx->stream));
  if (!ctx->check_device_errors()) return 0;
  // per point, over the points the reference visits (kind VOL / BDY; orphans
  // are KIND_ORPH once fix_orphans has run, NUL / frozen points never
  // located): steps > 0 located by a walk, steps < 0 by an exhaustive scan
  // (the reference's ppt->s sign, src/locate_pmmg.c:840-844), status 0 the
  // closest element (not contained anywhere)
  const int64_t n = ctx->nq;
  std::vector<int> status((size_t)std::max<int64_t>(n, 1)), steps((size_t)std::max<int64_t>(n, 1));
  std::vector<int8_t> kind((size_t)std::max<int64_t>(n, 1));
  if (n) {
    CK(hipMemcpy(status.data(), ctx->d_status.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost));
    CK(hipMemcpy(steps.data(), ctx->d_steps.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost));
    CK(hipMemcpy(kind.data(), ctx->d_kind.p, (size_t)n, hipMemcpyDeviceToHost));
  }
  // PMMG_locate_postprocessing (src/locate_pmmg.c:995-1028): |steps| of every
  // visited point, the exhaustive ones (steps < 0) included, min / max / mean
  memset(st, 0, sizeof *st);
  int64_t located = 0, sum = 0, mx = 0, mn = ctx->ne;
  for (int64_t i = 0; i < n; i++) {
    const int8_t k = kind[(size_t)i];
    if (k != KIND_VOL && k != KIND_BDY) continue;
    (k == KIND_VOL ? st->nvol : st->nbdy)++;
    int64_t s = steps[(size_t)i];
    if (s < 0) {
      st->nexhaust++;
      s = -s;
    }
    if (status[(size_t)i] == 0) st->nclosest++;
    located++;
    sum += s;
    mx = std::max<int64_t>(mx, s);
    mn = std::min<int64_t>(mn, s);
  }
  st->stepmax = mx;
  st->stepmin = mn;
  st->stepav = located ? (double)sum / (double)located : 0.0;
  return 1;
}

int pmx_locate_wave_stats(pmx_ctx *ctx, int path, pmx_wave_stats *st) {
  if (!ctx || !st || (path != 0 && path != 1)) {
    if (ctx) ctx->err = "pmx_locate_wave_stats: bad arguments";
    return 0;
  }
  if (!results_ready(ctx, "pmx_locate_wave_stats")) return 0;
  if (!ctx->fix_orphans()) return 0;
  int nsel[2] = {0, 0};
  CK(hipStreamSynchronize(ctx->stream));
  if (!ctx->check_device_errors()) return 0;
  if (ctx->nq) CK(hipMemcpy(nsel, ctx->d_nsel.p, sizeof nsel, hipMemcpyDeviceToHost));
  memset(st, 0, sizeof *st);
  const int64_t npath = nsel[path];
  if (!npath) return 1;
  std::vector<uint4> w((size_t)((npath + 255) / 256 * 4));
  CK(hipMemcpy(w.data(), path ? ctx->d_bstat.p : ctx->d_vstat.p, w.size() * sizeof(uint4),
               hipMemcpyDeviceToHost));
  for (const uint4 &r : w) {
    if (!r.x) continue;
    st->waves++;
    st->located += r.x;
    st->step_sum += r.y;
    st->lane_steps += 64 * (int64_t)r.z;
    st->wave_max_hist[std::min<unsigned>(r.z, 15u)]++;
  }
  return 1;
}

int pmx_seq_surface_stats(pmx_ctx *ctx, int64_t *nseq, int64_t *nreplay) {
  if (!ctx || !nseq || !nreplay) return 0;
  if (ctx->seq_stats_n < 0 || !ctx->ran) {
    ctx->err = "pmx_seq_surface_stats: the last step did not run PMX_RUN_SEQUENTIAL_SURFACE / _VOLUME";
    return 0;
  }
  *nseq = ctx->seq_stats[1];
  *nreplay = ctx->seq_stats[0];
  return 1;
}

int pmx_seq_volume_stats(pmx_ctx *ctx, int64_t *nseq, int64_t *nreplay) {
  if (!ctx || !nseq || !nreplay) return 0;
  if (ctx->seq_stats_n < 0 || !ctx->ran) {
    ctx->err = "pmx_seq_volume_stats: the last step did not run PMX_RUN_SEQUENTIAL_SURFACE / _VOLUME";
    return 0;
  }
  *nseq = ctx->seq_stats[3];
  *nreplay = ctx->seq_stats[2];
  return 1;
}

int pmx_step_ready(pmx_ctx *ctx) {
  return ctx && ctx->ran && ctx->have_pts && ctx->have_bg && ctx->out_n == ctx->nq && ctx->out_S == ctx->sd.S;
}

void *pmx_device_buffer(pmx_ctx *ctx, int which) {
  if (!ctx) return nullptr;
  // the orphan rows reset before a caller chains on the results (enqueued on
  // the context stream, which the caller orders its own work after)
  if (ctx->ran && (which == 0 || which == 1 || which == 2)) {
    hipSetDevice(ctx->device);
    if (!ctx->fix_orphans()) return nullptr;
  }
  switch (which) {
    case 0: return ctx->d_out.p;
    case 1: return ctx->d_elem.p;
    case 2: return ctx->d_status.p;
    default: return nullptr;
  }
}

void *pmx_device_alloc(pmx_ctx *ctx, size_t bytes) {
  if (!ctx) return nullptr;
  hipSetDevice(ctx->device);
  void *p = nullptr;
  const hipError_t e = hipMalloc(&p, std::max<size_t>(bytes, 1));
  if (e != hipSuccess) {
    ctx->err = std::string("pmx_device_alloc: ") + hipGetErrorString(e);
    return nullptr;
  }
  if (hipMemset(p, 0, std::max<size_t>(bytes, 1)) != hipSuccess) {
    hipFree(p);
    ctx->err = "pmx_device_alloc: memset";
    return nullptr;
  }
  return p;
}

int pmx_device_free(pmx_ctx *ctx, void *p) {
  if (!ctx) return 0;
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->stream);
  return (p == nullptr || hipFree(p) == hipSuccess) ? 1 : 0;
}

int pmx_device_download(pmx_ctx *ctx, void *host, const void *dev, size_t bytes) {
  if (!ctx) return 0;
  if (!host || !dev) { ctx->err = "pmx_device_download: null pointer"; return 0; }
  hipSetDevice(ctx->device);
  CK(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  return 1;
}

int pmx_device_upload(pmx_ctx *ctx, void *dev, const void *host, size_t bytes) {
  if (!ctx) return 0;
  if (!host || !dev) { ctx->err = "pmx_device_upload: null pointer"; return 0; }
  hipSetDevice(ctx->device);
  CK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  return 1;
}

int64_t pmx_debug_hint_grid(pmx_ctx *ctx, int *host, int64_t cap) {
  if (!ctx || !ctx->ran || !host) return 0;
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) return 0;
  const int64_t n = std::min<int64_t>(cap, ctx->gcells);
  if (hipMemcpy(host, ctx->d_grid.p, sizeof(int) * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess)
    return 0;
  return ctx->gcells;
}

int pmx_timing_reset(pmx_ctx *ctx) {
  if (!ctx) return 0;
  ctx->ev_used = 0;
  return 1;
}

double pmx_kernel_ms(pmx_ctx *ctx, int which) {
  if (!ctx || ctx->ev_used == 0 || which < 0 || which > 5) return -1.0;
  hipStreamSynchronize(ctx->stream);
  double tot = 0.0;
  for (int r = 0; r < ctx->ev_used; r++) {
    hipEvent_t *e = &ctx->events[(size_t)r * PMX_EV_PER_RUN];
    float ms = 0.f;
    // 0 hint (prologue + derived data + hint build), 1 volume walk, 2 surface
    // path, 3 fallback, 4 total, 5 derived data (prologue included)
    static const int from[6] = {0, 1, 3, 6, 0, 0}, to[6] = {1, 2, 5, 4, 4, 7};
    hipEventElapsedTime(&ms, e[from[which]], e[to[which]]);
    tot += ms;
  }
  return tot / ctx->ev_used;
}

// ---- device residency across ParMmg iterations --------------------------------
//
// PMMG_update_oldGrps (src/libparmmg1.c:653) makes the group's current mesh --
// the previous iteration's new mesh with its interpolated metric and fields
// -- the next interpolation's background.  The new points, their tags and the
// step's results are already on the device; with the new tets uploaded once
// (pmx_upload_new_tets, also used by pmx_new_mesh_qual) the next background
// needs only its boundary trias from the host.

int pmx_set_residency(pmx_ctx *ctx, int on) {
  if (!ctx) return 0;
  ctx->residency = on != 0;
  return 1;
}

int pmx_upload_new_tets(pmx_ctx *ctx, const int *tetra_v, int64_t tetra_stride, int64_t ne) {
  if (!ctx) return 0;
  if (!ctx->have_pts) { ctx->err = "pmx_upload_new_tets: upload the new points first"; return 0; }
  if (!tetra_v || ne < 1 || tetra_stride < 16 || 4 * ne >= (1LL << 31)) {
    ctx->err = "pmx_upload_new_tets: bad new tets";
    return 0;
  }
  hipSetDevice(ctx->device);
  const int64_t first = ctx->pts_first, n = ctx->nq;
  if (ctx->ran && ctx->view_tets) {
    // the last step took its orphans from the points view's tets (never
    // located, or located and reset): other tets would need another step.
    // The same tets are accepted (their pinned copy, packed by that step, is
    // compared row by row); nothing changes on a refusal.
    if (ctx->tets_inflight) {
      CK(hipEventSynchronize(ctx->ev_tets));
      ctx->tets_inflight = false;
    }
    const int4 *old = (const int4 *)ctx->h_tets;
    bool same = old && !ctx->tets_pending && ne == ctx->tview.ne;
    const char *tc0 = (const char *)tetra_v;
    for (int64_t k = 1; same && k <= ne; k++) {
      const int *v = (const int *)(tc0 + k * tetra_stride);
      if (v[0] > 0)
        for (int l = 0; l < 4; l++)
          if ((int64_t)v[l] - first < 0 || (int64_t)v[l] - first >= n) {
            ctx->err = "pmx_upload_new_tets: tet vertex outside the uploaded points";
            return 0;
          }
      const int4 o = old[k];
      same = v[0] <= 0 ? o.x == 0
                       : (o.x == (int)(v[0] - first + 1) && o.y == (int)(v[1] - first + 1) &&
                          o.z == (int)(v[2] - first + 1) && o.w == (int)(v[3] - first + 1));
    }
    if (!same) {
      ctx->err = "pmx_upload_new_tets: the last step took its orphans from the points view's new tets; "
                 "other tets need another pmx_run";
      return 0;
    }
  }
  ctx->have_ntet = false;
  if (ctx->next_topo) {                     // built from other tets: drop it
    CK(hipStreamSynchronize(ctx->topo));
    ctx->next_topo = false;
  }
  ctx->tets_pending = false;                // these tets replace the points view's
  if (ctx->tets_inflight) {
    CK(hipEventSynchronize(ctx->ev_tets));
    ctx->tets_inflight = false;
  }
  // packed into the pinned copy of the new tets (a strided quality output
  // reads their validity there)
  int4 *h = ctx->grow_htets(ne);
  if (!h) return 0;
  h[0] = make_int4(0, 0, 0, 0);
  const char *tc = (const char *)tetra_v;
  bool bad = false;
  const bool nt = nt_stores();
  // vertices renumbered from the points view (first..last) to 1..n: the
  // numbering of a promoted background
  par_for(1, ne + 1, [&](int64_t k0, int64_t k1) {
    bool b = false;
    for (int64_t k = k0; k < k1; k++) {
      const int *v = (const int *)(tc + k * tetra_stride);
      if (v[0] <= 0) { st4(&h[k], 0, 0, 0, 0, nt); continue; }   // !MG_EOK
      int w[4];
      for (int l = 0; l < 4; l++) {
        const int64_t j = (int64_t)v[l] - first;
        if (j < 0 || j >= n) b = true;
        w[l] = (int)(j + 1);
      }
      st4(&h[k], w[0], w[1], w[2], w[3], nt);
    }
    if (b) __atomic_store_n(&bad, true, __ATOMIC_RELAXED);
    std::atomic_thread_fence(std::memory_order_seq_cst);
  });
  if (bad) { ctx->err = "pmx_upload_new_tets: tet vertex outside the uploaded points"; return 0; }
  if (!dgrow(ctx, ctx->d_ntetv, (size_t)(ne + 1))) return 0;
  CK(hipMemcpyAsync(ctx->d_ntetv.p, h, (size_t)(ne + 1) * sizeof(int4), hipMemcpyHostToDevice, ctx->stream));
  if (ctx->view_tets && n > 0) {
    // these tets replace the points view's: the reference visits the points
    // of THEIR valid tets (src/interpmesh_pmmg.c:535-541), so the orphan
    // marks come from them (a step already run has its orphan rows reset
    // from these marks by the next consumer of its results)
    CK(hipMemsetAsync(ctx->d_qmark.p, 0, (size_t)n, ctx->stream));
    launch_mark_new_tets(ctx->d_ntetv.p, ne, ctx->d_qmark.p, n, ctx->stream);
    CK(hipGetLastError());
    ctx->orph_marks = true;
    if (ctx->ran) ctx->orph_fixed = false;
  }
  CK(hipStreamSynchronize(ctx->stream));
  ctx->n_ntet = ne;
  ctx->have_ntet = true;
  return 1;
}

int pmx_promote_background(pmx_ctx *ctx, const pmx_mesh_view *m, int nsol, const pmx_sol_view *sols) {
  if (!ctx) return 0;
  if (!m) { ctx->err = "pmx_promote_background: null mesh"; return 0; }
  if (!ctx->ran || !ctx->have_pts || ctx->out_n != ctx->nq || ctx->out_S != ctx->sd.S) {
    ctx->err = "pmx_promote_background: no step has run on the current uploads";
    return 0;
  }
  if (!ctx->have_ntet) { ctx->err = "pmx_promote_background: upload the new tets first"; return 0; }
  if (ctx->pts_first != 1) {
    ctx->err = "pmx_promote_background: the points view must start at 1 (Mmg numbering)";
    return 0;
  }
  const int64_t n = ctx->nq, ne = ctx->n_ntet, nt = m->nt;
  if (m->np != n || m->ne != ne || n < 1) {
    ctx->err = "pmx_promote_background: mesh sizes differ from the uploaded points / new tets";
    return 0;
  }
  if (nt < 0 || (nt > 0 && (!m->tria_v || !m->adjt || m->tria_stride < 12))) {
    ctx->err = "pmx_promote_background: nt > 0 requires tria_v and adjt";
    return 0;
  }
  const SolDesc sd = ctx->sd;
  if (nsol != sd.nsol || (nsol > 0 && !sols)) {
    ctx->err = "pmx_promote_background: solution list differs from the step's";
    return 0;
  }
  for (int s = 0; s < nsol; s++)
    if (sols[s].size != sd.size[s]) {
      ctx->err = "pmx_promote_background: solution size differs from the step's";
      return 0;
    }
  if (m->adja) {
    // the walks gather through these: every neighbour of a valid tet must
    // name a face of 1..ne (as pmx_upload_background checks)
    bool badj = false;
    par_chunks(1, ne + 1, [&](int, int64_t k0, int64_t k1) {
      bool b = false;
      for (int64_t k = k0; k < k1 && !b; k++) {
        if (m->tetra_v && *(const int *)((const char *)m->tetra_v + k * m->tetra_stride) <= 0) continue;
        for (int f = 0; f < 4; f++) {
          const int a = m->adja[4 * (k - 1) + 1 + f];
          if (a < 0 || a / 4 > ne) b = true;
        }
      }
      if (b) __atomic_store_n(&badj, true, __ATOMIC_RELAXED);
    });
    if (badj) { ctx->err = "pmx_promote_background: adjacency entry out of range"; return 0; }
  }
  hipSetDevice(ctx->device);
  Trace tr("promote");
  hipStream_t st = ctx->stream;
  if (!ctx->fix_orphans() || !ctx->ensure_tets(st)) return 0;
  CK(hipStreamSynchronize(st));
  if (!ctx->check_device_errors()) return 0;
  tr.mark("sync");
  const int S = sd.S;
  // rows the step did not write keep the caller's values (Mmg's own, or the
  // frozen-point copy): which ones, from the write masks
  char *stg = hstage(ctx, (size_t)n);
  if (!stg) return 0;
  CK(hipMemcpyAsync(stg, ctx->d_wmask.p, (size_t)n, hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  const uint8_t *wm = (const uint8_t *)stg;
  const unsigned full = (1u << nsol) - 1u;
  // per chunk, then concatenated in chunk order
  std::vector<std::vector<int4>> cent(64);
  std::vector<std::vector<double>> cval(64);
  bool missing = false;
  const int nch = par_chunks(0, n, [&](int c, int64_t j0, int64_t j1) {
    for (int64_t j = j0; j < j1; j++) {
      if ((wm[j] & full) == full) continue;      // every solution written (the common case)
      for (int s = 0; s < nsol; s++) {
        if (wm[j] & (1u << s)) continue;
        const int sz = sd.size[s];
        if (!sols[s].m) { __atomic_store_n(&missing, true, __ATOMIC_RELAXED); continue; }
        cent[(size_t)c].push_back(make_int4((int)(j + 1), sd.off[s], sz, 0));
        const double *src = sols[s].m + j * sz;   // pmx_download's layout
        for (int q = 0; q < 6; q++) cval[(size_t)c].push_back(q < sz ? src[q] : 0.0);
      }
    }
  });
  if (missing) {
    ctx->err = "pmx_promote_background: a row the step did not write needs the caller's solution";
    return 0;
  }
  std::vector<int4> ent;
  std::vector<double> vals;
  for (int c = 0; c < nch; c++) {
    ent.insert(ent.end(), cent[(size_t)c].begin(), cent[(size_t)c].end());
    vals.insert(vals.end(), cval[(size_t)c].begin(), cval[(size_t)c].end());
  }
  tr.mark("unwritten rows");
  // boundary trias of the new mesh (the host's: Mmg's numbering)
  std::vector<TriRec> htr;
  if (!stage_trias(ctx, m, n, htr)) return 0;
  tr.mark("trias");
  // the background invalid until this completes
  ctx->have_bg = ctx->have_derived = ctx->have_tetv = ctx->have_qual = ctx->have_ptag = ctx->have_csr = ctx->have_surf = false;
  ctx->bg_btv = false;                     // records from the new tets (or the caller's adja), not d_btv
  ctx->stat_np = -1;
  const int64_t ns = (ne + PMX_HINT_STRIDE - 1) / PMX_HINT_STRIDE;
  if (!dgrow(ctx, ctx->d_xyz, (size_t)(n + 1) * 3) || !dgrow(ctx, ctx->d_sol, (size_t)(n + 1) * std::max(S, 1)) ||
      !dgrow(ctx, ctx->d_tets, (size_t)(ne + 1)) || !dgrow(ctx, ctx->d_tets_s, (size_t)std::max<int64_t>(ns, 1)) ||
      !dgrow(ctx, ctx->d_adja, (size_t)(4 * ne + 5)) || !dgrow(ctx, ctx->d_tris, (size_t)(nt + 1)) ||
      !dgrow(ctx, ctx->d_trn, (size_t)(nt + 1)) || !dgrow(ctx, ctx->d_xyzq, (size_t)(n + 1)))
    return 0;
  const bool tags = ctx->have_qtag;
  if (tags && !dgrow(ctx, ctx->d_ptag, (size_t)(n + 1))) return 0;
  launch_promote(ctx->d_qxyz.p, ctx->d_out.p, tags ? ctx->d_qtag.p : nullptr, n, S, ctx->d_xyz.p, ctx->d_sol.p,
                 tags ? ctx->d_ptag.p : nullptr, st);
  if (!ent.empty()) {
    if (!dgrow(ctx, ctx->d_pent, ent.size()) || !dgrow(ctx, ctx->d_pval, vals.size())) return 0;
    CK(hipMemcpyAsync(ctx->d_pent.p, ent.data(), ent.size() * sizeof(int4), hipMemcpyHostToDevice, st));
    CK(hipMemcpyAsync(ctx->d_pval.p, vals.data(), vals.size() * sizeof(double), hipMemcpyHostToDevice, st));
    launch_patch_rows(ctx->d_pent.p, ctx->d_pval.p, (int64_t)ent.size(), S, ctx->d_sol.p, st);
  }
  // tet records: prepared while the step ran (residency on), else from the
  // caller's Mmg adjacency (mesh->adja after remeshing) or one built here
  tr.mark("promote launch");
  const bool prepared = ctx->next_topo;
  if (prepared) {                          // the residency build shares d_adja: wait for it
    CK(hipEventSynchronize(ctx->ev_topo));
    tr.mark("wait topo");
    ctx->next_topo = false;
  }
  if (prepared && !m->adja) {
    if (*ctx->h_nbad) { ctx->err = "pmx_promote_background: non-manifold tet faces"; return 0; }
    std::swap(ctx->d_tets, ctx->d_tets_next);
    std::swap(ctx->d_wrec, ctx->d_wrec_next);
    ctx->h_nbad[2] = ctx->h_nbad[3];
    std::swap(ctx->d_tets_s, ctx->d_tets_s_next);
  } else {
    if (m->adja) {
      CK(hipMemcpyAsync(ctx->d_adja.p, m->adja, (size_t)(4 * ne + 5) * sizeof(int), hipMemcpyHostToDevice, st));
    } else if (!pmx_ctx_build_adja_device(ctx, ctx->d_ntetv.p, ne, n, ctx->d_adja.p, st, nullptr)) {
      return 0;
    }
    if ((ctx->compact_recs && !dgrow(ctx, ctx->d_wrec, (size_t)(ne + 1))) || !dgrow(ctx, ctx->d_wfar, 8)) return 0;
    launch_build_tetrec(ctx->d_ntetv.p, ctx->d_adja.p, ne, PMX_HINT_STRIDE, ctx->d_tets.p, ctx->d_tets_s.p, st);
    ctx->h_nbad[2] = 0;
    if (ctx->compact_recs) launch_build_wrec(ctx->d_tets.p, ne, ctx->d_wrec.p, ctx->d_wfar.p, ctx->h_nbad + 2, st);
  }
  ctx->np = n;
  ctx->ne = ne;
  ctx->nt = nt;
  ctx->hausd = m->hausd;
  tr.mark("tet records");
  if (!setup_grids(ctx, ctx->qlo, ctx->qhi, ne)) return 0;
  if (!ctx->order_hint_samples(ne, ctx->np, st)) return 0;
  tr.mark("grids");
  CK(hipMemcpyAsync(ctx->d_tris.p, htr.data(), htr.size() * sizeof(TriRec), hipMemcpyHostToDevice, st));
  if (!ctx->check_fans(st)) return 0;
  CK(hipGetLastError());
  CK(hipStreamSynchronize(st));            // host vectors die here
  ctx->fan_rot = ctx->nt > 0 && ctx->h_nbad[4] == 0;
  ctx->nsamp = ctx->samples_owner ? (int64_t)ctx->h_nbad[5] : 0;
  tr.mark("uploads + sync");
  ctx->have_ptag = tags;
  // the points and the results were consumed: the next step needs new points
  ctx->have_pts = ctx->ran = ctx->have_ntet = false;
  ctx->have_bg = true;
  return 1;
}

}  // extern "C"

// ---- pmx_ctx members ----------------------------------------------------------

// the new points' classification and compaction on stream s (the marks, if
// any, zeroed beforehand)
bool pmx_ctx::classify(hipStream_t s, bool marks) {
  if (nq < 1) return true;
  launch_classify(have_qtag ? d_qtag.p : nullptr, marks ? d_qmark.p : nullptr, nq, d_ctile.p, d_kind.p, d_vollist.p, d_bdylist.p,
                  d_nsel.p, s);
  if (hipGetLastError() != hipSuccess) {
    err = "classification: launch failed";
    return false;
  }
  return true;
}

hipEvent_t *pmx_ctx::next_event_slot() {
  size_t need = (size_t)(ev_used + 1) * PMX_EV_PER_RUN;
  while (events.size() < need) {
    hipEvent_t e;
    hipEventCreate(&e);
    events.push_back(e);
  }
  hipEvent_t *r = &events[(size_t)ev_used * PMX_EV_PER_RUN];
  ev_used++;
  return r;
}

void pmx_ctx::free_all() {
  if (h_stage) hipHostFree(h_stage);
  h_stage = nullptr;
  h_stage_cap = 0;
  dfree(d_xyz); dfree(d_tets); dfree(d_wrec); dfree(d_wrec_next); dfree(d_wfar); dfree(d_skey); dfree(d_sidx); dfree(d_salt); dfree(d_stmp); dfree(d_tets_sk); dfree(d_sol); dfree(d_tets_s); dfree(d_tris);
  dfree(d_ntlist); dfree(d_ntval); dfree(d_ntkey); dfree(d_ntrange); dfree(d_nttmp); dfree(d_xyzq); dfree(d_trn); dfree(d_grid); dfree(d_tetv);
  dfree(d_kind); dfree(d_qmark); dfree(d_ctile); dfree(d_nsel); dfree(d_wmask); dfree(d_out); dfree(d_elem); dfree(d_status);
  dfree(d_steps); dfree(d_start); dfree(d_edge); dfree(d_vertex); dfree(d_list); dfree(d_found);
  dfree(d_bestk); dfree(d_best); dfree(d_ties); dfree(d_counts); dfree(d_vollist); dfree(d_bdylist);
  dfree(d_vstat); dfree(d_bstat); dfree(d_hrec);
  dfree(d_sqkey); dfree(d_sqidx); dfree(d_sqint); dfree(d_sqtf); dfree(d_sqpf); dfree(d_sqtv); dfree(d_sqows); dfree(d_sqval);
  dfree(d_sqw);
  dfree(d_sqtmp);
  dfree(d_sqflag);
  dfree(d_sqcand);
  dfree(d_qual); dfree(d_red); dfree(d_blist); dfree(d_olist); dfree(d_ows);
  dfree(d_ptag); dfree(d_touch); dfree(d_cidx); dfree(d_intv); dfree(d_pub); dfree(d_pkey);
  dfree(d_ppt); dfree(d_pedge); dfree(d_ntetv); dfree(d_nqual); dfree(d_qtag); dfree(d_gather);
  dfree(d_adja); dfree(d_tcnt); dfree(d_toff); dfree(d_tbad); dfree(d_trec); dfree(d_ttmp);
  dfree(d_pent); dfree(d_pval); dfree(d_tets_next); dfree(d_tets_s_next);
  next_topo = false;
  dfree(d_cmet); dfree(d_cperm); dfree(d_ccnt);
  if (d_tgrid) hipFree(d_tgrid);
  d_tgrid = nullptr;
  d_tgrid_cap = 0;
  have_bg = have_pts = ran = have_derived = have_tetv = have_qual = have_ptag = have_qtag = have_csr = false;
  have_surf = false;
  dfree(d_etag); dfree(d_pn); dfree(d_xpn); dfree(d_pxp); dfree(d_pedge_tag);
  dfree(d_pbcnt); dfree(d_pboff); dfree(d_pbrec); dfree(d_pbtmp);
  have_ntet = false;
  stat_np = -1;
}

