// pmx_stats.hip -- quality and edge-length statistics on gfx950.
//
// pmx_tetra_qual       <- PMMG_tetraQual -> MMG3D_tetraQual (reference
//                         src/quality_pmmg.c:720-733; per-tet kernels restated
//                         from Mmg MMG5_caltet_iso / MMG5_caltet33_ani, unpinned)
// pmx_qualhisto[_device] <- the per-group part of PMMG_qualhisto
//                         (src/quality_pmmg.c:156-261): MMG3D_computeInqua /
//                         computeOutqua statistics (5 bins, min + location,
//                         max, sum, good, med; OUTQUA: nrid) and the group's
//                         node count (PMMG_count_nodes_par, :33-80)
// pmx_prilen[_device]  <- PMMG_prilen / PMMG_computePrilen (src/quality_pmmg.c:
//                         370-709): owned parallel edges first, then every
//                         other unique edge in (k, ia) hash-pop order
// pmx_new_mesh_qual    <- PMMG_tetraQual on the new mesh right after the
//                         interpolation (src/libparmmg1.c:845), in the
//                         device-resident interpolated metric (no re-upload)
// pmx_qual_fold / pmx_len_fold, pmx_*_allreduce <- the reference's MPI_Reduce
//                         with its custom ops (:82-144, :265-307, :661-676):
//                         one RCCL all-gather of the per-rank partials, then
//                         the reference's operators folded in rank order
//
// Histograms are one pass over the mesh: per-thread accumulation, a wavefront
// reduction, one partial record per workgroup, and a two-level final
// reduction in workgroup order (deterministic sums).  Unique edges are
// enumerated without a hash table: tet k owns its local edge ia iff k is the
// smallest admissible tet index in the edge shell, found by rotating around
// the edge through the adjacency (early exit on the first smaller index) --
// the first occurrence in the reference's (k ascending, ia ascending)
// hash-pop order, so endpoints and orientation of every length match it.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <unordered_set>
#include <type_traits>
#include <mutex>
#include <vector>
#include "pmx_internal.h"

#define ALPHAD 20.7846097          // MMG3D_ALPHAD (12*sqrt(3))
#define TAG_GEO 2
#define TAG_REQ 4
#define TAG_NOM 8
#define TAG_CRN 32
#define TAG_REF 1
#define LEN_STEP2 (1LL << 40)      // keys of tet edges: LEN_STEP2 + 6*k + ia

__constant__ int IARE[6][2] = {{0, 1}, {0, 2}, {0, 3}, {1, 2}, {1, 3}, {2, 3}};

// MMG5_caltet_iso (restated)
__device__ double caltet_iso(D3 a, D3 b, D3 c, D3 d) {
  double abx = b.x - a.x, aby = b.y - a.y, abz = b.z - a.z;
  double acx = c.x - a.x, acy = c.y - a.y, acz = c.z - a.z;
  double adx = d.x - a.x, ady = d.y - a.y, adz = d.z - a.z;
  double v1 = acy * adz - acz * ady;
  double v2 = acz * adx - acx * adz;
  double v3 = acx * ady - acy * adx;
  double vol = abx * v1 + aby * v2 + abz * v3;
  if (vol <= 0.) return 0.0;
  double bcx = c.x - b.x, bcy = c.y - b.y, bcz = c.z - b.z;
  double bdx = d.x - b.x, bdy = d.y - b.y, bdz = d.z - b.z;
  double cdx = d.x - c.x, cdy = d.y - c.y, cdz = d.z - c.z;
  double rap = abx * abx + aby * aby + abz * abz;
  rap += acx * acx + acy * acy + acz * acz;
  rap += adx * adx + ady * ady + adz * adz;
  rap += bcx * bcx + bcy * bcy + bcz * bcz;
  rap += bdx * bdx + bdy * bdy + bdz * bdz;
  rap += cdx * cdx + cdy * cdy + cdz * cdz;
  if (rap < PMX_EPSD2) return 0.0;
  rap = rap * sqrt(rap);
  return vol / rap;
}

__device__ __forceinline__ double mlen2(const double *m, double x, double y, double z) {
  return m[0] * x * x + m[3] * y * y + m[5] * z * z + 2.0 * (m[1] * x * y + m[2] * x * z + m[4] * y * z);
}

// MMG5_caltet33_ani / MMG5_caltet_ani (restated) past their mean metric mm
__device__ double caltet_ani_mm(D3 a, D3 b, D3 c, D3 d, const double mm[6]) {
  double abx = b.x - a.x, aby = b.y - a.y, abz = b.z - a.z;
  double acx = c.x - a.x, acy = c.y - a.y, acz = c.z - a.z;
  double adx = d.x - a.x, ady = d.y - a.y, adz = d.z - a.z;
  double vol = abx * (acy * adz - acz * ady) + aby * (acz * adx - acx * adz) + abz * (acx * ady - acy * adx);
  if (vol <= 0.) return 0.0;
  double det = mm[0] * (mm[3] * mm[5] - mm[4] * mm[4]) - mm[1] * (mm[1] * mm[5] - mm[2] * mm[4]) +
               mm[2] * (mm[1] * mm[4] - mm[2] * mm[3]);
  if (det < PMX_EPSD2) return 0.0;
  det = sqrt(det) * vol;
  double bcx = c.x - b.x, bcy = c.y - b.y, bcz = c.z - b.z;
  double bdx = d.x - b.x, bdy = d.y - b.y, bdz = d.z - b.z;
  double cdx = d.x - c.x, cdy = d.y - c.y, cdz = d.z - c.z;
  double rap = mlen2(mm, abx, aby, abz);
  rap += mlen2(mm, acx, acy, acz);
  rap += mlen2(mm, adx, ady, adz);
  rap += mlen2(mm, bcx, bcy, bcz);
  rap += mlen2(mm, bdx, bdy, bdz);
  rap += mlen2(mm, cdx, cdy, cdz);
  if (rap < PMX_EPSD2) return 0.0;
  double num = sqrt(rap) * rap;
  return det / num;
}

// MMG5_caltet33_ani: the plain mean of the 4 vertex metrics
__device__ double caltet_ani(D3 a, D3 b, D3 c, D3 d, const double *ma, const double *mb,
                             const double *mc, const double *md) {
  double mm[6];
  for (int i = 0; i < 6; i++) mm[i] = 0.25 * (ma[i] + mb[i] + mc[i] + md[i]);
  return caltet_ani_mm(a, b, c, d, mm);
}

// vertex v of the statistics' mesh (the background: dense xyz; the new mesh:
// the uploaded Pt4 points, shifted by the first point index)
__device__ __forceinline__ D3 sld3(const StatArgs &A, int v) {
  const double *r = A.xyz + (int64_t)A.xstride * (v - A.vbase);
  return D3{r[0], r[1], r[2]};
}
__device__ __forceinline__ const double *smet(const StatArgs &A, int v) {
  return A.sol + (int64_t)(v - A.vbase) * A.S + A.moff;
}
__device__ __forceinline__ unsigned stag(const StatArgs &A, int v) { return A.ptag[v - A.vbase]; }

// a vertex that is a non-singular ridge point: !(MG_SIN || MG_NOM) && MG_GEO
__device__ __forceinline__ bool ridge_pt(unsigned tg) {
  const bool sin = (tg & TAG_CRN) || (tg & TAG_REQ);
  return !(sin || (TAG_NOM & tg)) && (tg & TAG_GEO);
}
// all 4 vertices are non-singular ridge points: skipped by the length loop
// (reference src/quality_pmmg.c:509-517), counted by MMG3D_computeOutqua's nrid
__device__ __forceinline__ bool tet_4ridge(const StatArgs &A, const int v[4]) {
  if (!A.ptag) return false;
  bool all = true;
#pragma unroll
  for (int i = 0; i < 4; i++) all = all && ridge_pt(stag(A, v[i]));
  return all;
}

// MMG5_caltet_ani (metRidTyp = 1): MMG5_moymet's mean over the vertices that
// are not non-singular ridge points (their stored metric is Mmg's two-sided
// ridge metric), summed in vertex order and scaled by 1/n; none: quality 0
__device__ double caltet_ani_rid(const StatArgs &A, const int v[4], D3 a, D3 b, D3 c, D3 d) {
  double mm[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  int n = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    if (A.rtag && ridge_pt(A.rtag[v[j] - A.vbase])) continue;
    n++;
    const double *m = smet(A, v[j]);
#pragma unroll
    for (int i = 0; i < 6; i++) mm[i] += m[i];
  }
  if (!n) return 0.0;
  const double dd = 1. / n;
#pragma unroll
  for (int i = 0; i < 6; i++) mm[i] = mm[i] * dd;
  return caltet_ani_mm(a, b, c, d, mm);
}

template <bool ANI>
__device__ double tet_quality(const StatArgs &A, const int v[4]) {
  D3 a = sld3(A, v[0]), b = sld3(A, v[1]), c = sld3(A, v[2]), d = sld3(A, v[3]);
  if (ANI && A.ridmet) return caltet_ani_rid(A, v, a, b, c, d);
  if (ANI) return caltet_ani(a, b, c, d, smet(A, v[0]), smet(A, v[1]), smet(A, v[2]), smet(A, v[3]));
  return caltet_iso(a, b, c, d);
}

// ---- quality histogram ------------------------------------------------------------

struct QualPart {
  double avg, max, min;
  long long iel, ne, good, med, his[5], nrid;
};

__device__ __forceinline__ void qual_merge(QualPart &x, const QualPart &y) {
  x.avg += y.avg;
  x.max = fmax(x.max, y.max);
  if (y.min < x.min || (y.min == x.min && y.iel < x.iel)) { x.min = y.min; x.iel = y.iel; }
  x.ne += y.ne; x.good += y.good; x.med += y.med; x.nrid += y.nrid;
  for (int i = 0; i < 5; i++) x.his[i] += y.his[i];
}
__device__ __forceinline__ void qual_init(QualPart &p) {
  p.avg = 0.0; p.max = 0.0; p.min = 2.0; p.iel = 0x7fffffffffffffffLL;
  p.ne = 0; p.good = 0; p.med = 0; p.nrid = 0;
  for (int i = 0; i < 5; i++) p.his[i] = 0;
}

// quality of every tet (+ optional histogram partials in the same pass).
// ANI: the metric is a 6-component tensor (compiled apart: the iso variant
// does not carry the tensor path's registers).  OUT: MMG3D_computeOutqua's
// count of tets with 4 ridge vertices.
// Each workgroup takes a contiguous tet range, 256 tets per iteration, the
// next iteration's connectivity loaded before this one's vertex gathers (two
// dependent levels in flight).  Counts are wave-uniform (ballot + popcount,
// scalar registers); sum and extrema per lane, reduced by a fixed shuffle
// tree and the 4 waves in order (deterministic), so the workgroup needs no
// 256-entry LDS reduction buffer (occupancy no longer LDS-bound).
// MODE (compiled apart, no run-time branches in the loop): QM_STORE every
// tet's quality into qual, no partials (MMG3D_tetraQual); QM_HISTO the
// partials of freshly computed qualities, nothing stored; QM_STORED the
// partials of the qualities already in qual (OUTQUA after tetraQual).
enum { QM_STORE = 0, QM_HISTO = 1, QM_STORED = 2 };
template <bool ANI, bool OUT, int MODE>
__global__ __launch_bounds__(256) void k_qual(StatArgs A, double *qual, QualPart *parts) {
  constexpr bool use_stored = MODE == QM_STORED;
  __shared__ QualPart sh[4];
  double avg = 0.0, qmax = 0.0, qmin = 2.0;
  long long iel = 0x7fffffffffffffffLL;
  unsigned cne = 0, cgood = 0, cmed = 0, cnrid = 0, chis[5] = {0, 0, 0, 0, 0};
  // contiguous chunk per block; each XCD gets a contiguous run of chunks so
  // the next z-layer's points (another chunk) are in its own L2
  const int64_t lb = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t per = (A.ne + gridDim.x - 1) / gridDim.x;
  const int64_t k0 = 1 + lb * per, k1 = min(A.ne, k0 + per - 1), kstep = blockDim.x;
  // 16-B connectivity stream: the neighbours are not needed here
  int4 cv = (k0 + (int64_t)threadIdx.x <= k1) ? A.tetv[k0 + threadIdx.x] : make_int4(0, 0, 0, 0);
  // the vertex rows are loaded for every lane (an invalid tet reads row 0 and
  // discards the result), then the next connectivity: loads return in
  // order, so a prefetch issued before the gathers (r05) made every gather
  // wait for it -- the prefetch hid nothing.  The ridge-storage mean
  // (OUTQUA with a tensor metric) keeps the tag-dependent loads.
  const bool pre = !(ANI && A.ridmet);
  for (int64_t kb = k0; kb <= k1; kb += kstep) {   // uniform over the block
    const int64_t k = kb + threadIdx.x;
    const bool in = k <= k1;
    const int v[4] = {cv.x, cv.y, cv.z, cv.w};
    const bool valid = in && v[0] > 0;
    const int64_t kn = k + kstep;
    double q = 0.0;
    bool rid4 = false;
    if (use_stored || pre) {
      const int vb = A.vbase;
      const int w[4] = {valid ? v[0] : vb, valid ? v[1] : vb, valid ? v[2] : vb, valid ? v[3] : vb};
      unsigned tg[4] = {0u, 0u, 0u, 0u};
      if (OUT && A.ptag) {
#pragma unroll
        for (int i = 0; i < 4; i++) tg[i] = stag(A, w[i]);
      }
      double qs = 0.0;
      D3 P[4];
      double mv[ANI ? 4 : 1][6];
      if constexpr (use_stored) {
        qs = qual[in ? k : k1];
      } else {
#pragma unroll
        for (int i = 0; i < 4; i++) P[i] = sld3(A, w[i]);
        if constexpr (ANI) {
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const double *m = smet(A, w[i]);
#pragma unroll
            for (int j = 0; j < 6; j++) mv[i][j] = m[j];
          }
        }
      }
      cv = A.tetv[kn <= k1 ? kn : k1];
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (use_stored) {
        q = qs;
      } else if constexpr (ANI) {
        q = caltet_ani(P[0], P[1], P[2], P[3], mv[0], mv[1], mv[2], mv[3]);
      } else {
        q = caltet_iso(P[0], P[1], P[2], P[3]);
      }
      if (OUT && A.ptag) rid4 = ridge_pt(tg[0]) && ridge_pt(tg[1]) && ridge_pt(tg[2]) && ridge_pt(tg[3]);
    } else {
      if (kn <= k1) cv = A.tetv[kn];
      if (valid) q = tet_quality<ANI>(A, v);
      if (OUT && valid) rid4 = tet_4ridge(A, v);
    }
    // !MG_EOK: no quality (0, not a stale value)
    if (MODE == QM_STORE && in && !valid) qual[k] = 0.0;
    double rap = 0.0;
    if (valid) {
      if (MODE == QM_STORE) qual[k] = q;
      rap = ALPHAD * q;
      if (MODE != QM_STORE) {
        if (rap < qmin || (rap == qmin && k < iel)) { qmin = rap; iel = k; }
        avg += rap;
        qmax = fmax(qmax, rap);
      }
    }
    if (MODE == QM_STORE) continue;
    cne += (unsigned)__popcll(__ballot(valid));
    cgood += (unsigned)__popcll(__ballot(valid && rap > 0.12));
    cmed += (unsigned)__popcll(__ballot(valid && rap > 0.5));
    if (OUT) cnrid += (unsigned)__popcll(__ballot(valid && rid4));
    int ir = (int)(5.0 * rap);
    ir = ir < 4 ? ir : 4;
    // the bin from three bit ballots (scalar mask algebra) instead of five
    // per-bin ones
    const unsigned long long V = __ballot(valid), B0 = __ballot(ir & 1), B1 = __ballot(ir & 2),
                             B2 = __ballot(ir & 4);
    const unsigned long long L = V & ~B2;            // bins 0-3
    chis[0] += (unsigned)__popcll(L & ~B1 & ~B0);
    chis[1] += (unsigned)__popcll(L & ~B1 & B0);
    chis[2] += (unsigned)__popcll(L & B1 & ~B0);
    chis[3] += (unsigned)__popcll(L & B1 & B0);
    chis[4] += (unsigned)__popcll(V & B2);
  }
  if (MODE == QM_STORE) return;
  // the same tree on every lane (the lower lane's value first)
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double ya = __shfl_xor(avg, o, 64), ymx = __shfl_xor(qmax, o, 64), ymn = __shfl_xor(qmin, o, 64);
    const long long yi = __shfl_xor(iel, o, 64);
    avg = (threadIdx.x & o) == 0 ? avg + ya : ya + avg;
    qmax = fmax(qmax, ymx);
    if (ymn < qmin || (ymn == qmin && yi < iel)) { qmin = ymn; iel = yi; }
  }
  if ((threadIdx.x & 63) == 0) {
    QualPart p;
    p.avg = avg; p.max = qmax; p.min = qmin; p.iel = iel;
    p.ne = cne; p.good = cgood; p.med = cmed; p.nrid = cnrid;
#pragma unroll
    for (int i = 0; i < 5; i++) p.his[i] = chis[i];
    sh[threadIdx.x >> 6] = p;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    QualPart r = sh[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); w++) qual_merge(r, sh[w]);
    parts[lb] = r;
  }
}

// fixed-order reduction of n partials (launched twice: FINAL_GRID blocks, then
// one); the last level writes the public pmx_qual_part (np from the node count)
__global__ __launch_bounds__(256) void k_qual_final(const QualPart *parts, int n, QualPart *res,
                                                    pmx_qual_part *pub, long long np) {
  __shared__ QualPart sh[256];
  QualPart p;
  qual_init(p);
  const int pb = (n + gridDim.x - 1) / gridDim.x;
  const int lo = blockIdx.x * pb, hi = min(n, lo + pb);
  int per = (hi - lo + 255) / 256;
  for (int b = lo + threadIdx.x * per; b < min(hi, lo + (int)(threadIdx.x + 1) * per); b++)
    qual_merge(p, parts[b]);
  sh[threadIdx.x] = p;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) qual_merge(sh[threadIdx.x], sh[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  if (res) res[blockIdx.x] = sh[0];
  if (pub) {
    const QualPart &r = sh[0];
    pmx_qual_part o;
    o.avg = r.avg; o.max = r.max; o.min = r.min;
    o.iel = r.ne ? r.iel : 0;
    o.ne = r.ne; o.np = np; o.good = r.good; o.med = r.med; o.nrid = r.nrid;
    for (int i = 0; i < 5; i++) o.his[i] = r.his[i];
    o.iel_grp = 0;
    *pub = o;
  }
}

// ---- node count (PMMG_count_nodes_par, src/quality_pmmg.c:33-80) ------------------

// points touched by a valid tet
__global__ __launch_bounds__(256) void k_touch(const int4 *__restrict__ tv, int64_t ne,
                                               uint8_t *__restrict__ touched) {
  for (int64_t k = 1 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k <= ne;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int4 v = tv[k];
    if (v.x <= 0) continue;
    touched[v.x] = 1; touched[v.y] = 1; touched[v.z] = 1; touched[v.w] = 1;
  }
}
// points of the internal node communicator count when they claim their slot
// (intvalues[idx] == 0 -> base); the other points when a valid tet touches them
__global__ __launch_bounds__(256) void k_count_nodes(const uint8_t *__restrict__ touched, int64_t np,
                                                     const int *__restrict__ comm_idx,
                                                     int *__restrict__ intvalues, int base,
                                                     unsigned long long *__restrict__ count) {
  unsigned c = 0;
  for (int64_t ip = 1 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; ip <= np;
       ip += (int64_t)gridDim.x * blockDim.x) {
    const int idx = comm_idx ? comm_idx[ip] : -1;
    if (idx >= 0) c += atomicCAS(&intvalues[idx], 0, base) == 0 ? 1u : 0u;
    else c += touched[ip] ? 1u : 0u;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(count, (unsigned long long)c);
}

// ---- edge lengths ---------------------------------------------------------------

struct LenPart {
  double avlen, lmin, lmax;
  long long kmin, kmax;          // first-occurrence keys of the extremal edges
  long long ned, nul, hl[9];
};

__device__ __forceinline__ int pick_v(const TetRec &t, int l) {
  return (t.v[0] & -(int)(l == 0)) | (t.v[1] & -(int)(l == 1)) | (t.v[2] & -(int)(l == 2)) |
         (t.v[3] & -(int)(l == 3));
}
__device__ __forceinline__ int pick_nb(const TetRec &t, int l) {
  return (t.nb[0] & -(int)(l == 0)) | (t.nb[1] & -(int)(l == 1)) | (t.nb[2] & -(int)(l == 2)) |
         (t.nb[3] & -(int)(l == 3));
}


// log1p as glibc computes it (sysdeps/ieee754/dbl-64/s_log1p.c: Sun's fdlibm
// algorithm with its polynomial in the pairwise (Estrin) form glibc uses),
// restated so that the lengths are the reference's bit for bit on a glibc
// host -- ocml's log1p differs from it in the last ulp now and then.
// Checked against glibc 2.35's log1p on 5e7 inputs over (-0.49, 20) and
// tiny / huge ranges: no difference (tests/test_oracle.py pins the C twin of
// this code against the host's log1p).  Needs -ffp-contract=off (the
// library's flag): every product and sum rounded as in the C source.
__device__ double pmx_log1p(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01, Lp3 = 2.857142874366239149e-01,
               Lp4 = 2.222219843214978396e-01, Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01,
               Lp7 = 1.479819860511658591e-01;
  double f = 0.0, c = 0.0, u;
  int hx = __double2hiint(x), hu = 0, k = 1;
  const int ax = hx & 0x7fffffff;
  if (hx < 0x3FDA827A) {                          // x < 0.41422
    if (ax >= 0x3ff00000) return x == -1.0 ? -__builtin_inf() : (x - x) / (x - x);   // x <= -1
    if (ax < 0x3e200000) return ax < 0x3c900000 ? x : x - x * x * 0.5;                // |x| < 2^-29
    if (hx > 0 || hx <= (int)0xbfd2bec3) { k = 0; f = x; hu = 1; }                     // -0.2929 < x < 0.41422
  } else if (hx >= 0x7ff00000) {
    return x + x;
  }
  if (k != 0) {
    if (hx < 0x43400000) {
      u = 1.0 + x;
      hu = __double2hiint(u);
      k = (hu >> 20) - 1023;
      c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0);  // correction term
      c /= u;
    } else {
      u = x;
      hu = __double2hiint(u);
      k = (hu >> 20) - 1023;
      c = 0.0;
    }
    hu &= 0x000fffff;
    if (hu < 0x6a09e) {
      u = __hiloint2double(hu | 0x3ff00000, __double2loint(u));            // normalise u
    } else {
      k += 1;
      u = __hiloint2double(hu | 0x3fe00000, __double2loint(u));            // normalise u / 2
      hu = (0x00100000 - hu) >> 2;
    }
    f = u - 1.0;
  }
  const double hfsq = 0.5 * f * f;
  const double dk = (double)k;
  if (hu == 0) {                                   // |f| < 2^-20
    if (f == 0.0) {
      if (k == 0) return 0.0;
      c += dk * ln2_lo;
      return dk * ln2_hi + c;
    }
    const double R = hfsq * (1.0 - 0.66666666666666666 * f);
    if (k == 0) return f - R;
    return dk * ln2_hi - ((R - (dk * ln2_lo + c)) - f);
  }
  const double s = f / (2.0 + f);
  const double z = s * s;
  const double R1 = z * Lp1, z2 = z * z, R2 = Lp2 + z * Lp3, z4 = z2 * z2, R3 = Lp4 + z * Lp5, z6 = z4 * z2,
               R4 = Lp6 + z * Lp7;
  const double R = R1 + z2 * R2 + z4 * R3 + z6 * R4;
  if (k == 0) return f - (hfsq - s * (hfsq + R));
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + (dk * ln2_lo + c))) - f);
}

// MMG5_lenEdg_iso in two halves: the loads (the sizes issued with the
// coordinates -- the scheduler otherwise places them after the wait for the
// coordinates, a second round trip) and the arithmetic, so that a caller can
// put work between them
struct IsoEdge { D3 c1, c2; double h1, h2; };
__device__ __forceinline__ IsoEdge iso_edge_load(const StatArgs &A, int p1, int p2) {
  IsoEdge e;
  e.c1 = sld3(A, p1);
  e.c2 = sld3(A, p2);
  e.h1 = smet(A, p1)[0];
  e.h2 = smet(A, p2)[0];
  __builtin_amdgcn_sched_barrier(0);
  return e;
}
template <bool TWO = false>   // TWO (A/B): the two-branch form, two divisions in a mixed wave
__device__ __forceinline__ double iso_edge_len(const IsoEdge &e) {
  double ux = e.c2.x - e.c1.x, uy = e.c2.y - e.c1.y, uz = e.c2.z - e.c1.z;
  double l = ux * ux + uy * uy + uz * uz;
  l = sqrt(l);
  double r = e.h2 / e.h1 - 1.0;
  if constexpr (TWO) return (fabs(r) < PMX_EPS) ? (l / e.h1) : (l / (e.h2 - e.h1) * pmx_log1p(r));
  // one division for both branches (l / h1 or l / (h2 - h1): the same
  // correctly rounded quotients as the two-branch form, one instead of two
  // in a wave whose lanes take both)
  const bool flat = fabs(r) < PMX_EPS;
  const double q = l / (flat ? e.h1 : (e.h2 - e.h1));
  return flat ? q : q * pmx_log1p(r);
}

// MMG5_lenEdg_iso / lenEdg33_ani (restated, unpinned; the surface lengths
// MMG5_lenSurfEdg_iso / lenSurfEdg33_ani of the parallel edges take the same
// formulas in classic metric storage)
template <bool ANI, bool TWO = false>
__device__ __forceinline__ double edge_len_t(const StatArgs &A, int p1, int p2) {
  if (ANI) {
    D3 c1 = sld3(A, p1), c2 = sld3(A, p2);
    double ux = c2.x - c1.x, uy = c2.y - c1.y, uz = c2.z - c1.z;
    const double *m1 = smet(A, p1), *m2 = smet(A, p2);
    double dd1 = mlen2(m1, ux, uy, uz);
    double dd2 = mlen2(m2, ux, uy, uz);
    if (dd1 <= 0.0) dd1 = 0.0;
    if (dd2 <= 0.0) dd2 = 0.0;
    return (sqrt(dd1) + sqrt(dd2) + 4.0 * sqrt(0.5 * (dd1 + dd2))) / 6.0;
  }
  const IsoEdge e = iso_edge_load(A, p1, p2);
  return iso_edge_len<TWO>(e);
}
__device__ double edge_len(const StatArgs &A, int p1, int p2) {
  return A.msize == 6 ? edge_len_t<true>(A, p1, p2) : edge_len_t<false>(A, p1, p2);
}

// ---- Mmg's surface-aware lengths in a tensor metric (restated from the public
// Mmg sources, unpinned; the oracle's orc_prilen_full, oracle/pmx_oracle_stats.c,
// is the same restatement in C).  The background's arrays: vbase 0, xstride 3.

// MG_SIN(tag) || (tag & MG_NOM): the stored metric is a plain tensor
__device__ __forceinline__ bool sin_or_nom(unsigned tg) { return (tg & (TAG_CRN | TAG_REQ | TAG_NOM)) != 0; }
__device__ __forceinline__ unsigned ptag_or0(const StatArgs &A, int ip) { return A.ptag ? A.ptag[ip] : 0u; }
// MMG5_Point.n (a ridge point's tangent, in mmg3d); zeros without surface data
__device__ __forceinline__ D3 pn_of(const StatArgs &A, int ip) {
  if (!A.pn) return D3{0.0, 0.0, 0.0};
  const double *r = A.pn + 3 * (int64_t)ip;
  return D3{r[0], r[1], r[2]};
}
// mesh->xpoint[p->xp].n1 / .n2 (entry 0: zeros)
__device__ __forceinline__ D3 xn_of(const StatArgs &A, int ip, int which) {
  if (!A.pxp) return D3{0.0, 0.0, 0.0};
  const double *r = A.xpn + 6 * (int64_t)A.pxp[ip] + 3 * which;
  return D3{r[0], r[1], r[2]};
}

// MMG5_buildridmet: ridge point np0's metric in the direction u, from its
// ridge storage m = (tangent size, in-surface sizes of sides 1 / 2, normal
// sizes of sides 1 / 2): the side whose normal is the more orthogonal to u,
// basis (t, n x t, n), mr = R diag(m0, dv, dn) R^T
__device__ void buildridmet(const StatArgs &A, int np0, double ux, double uy, double uz, double mr[6]) {
  const double *m = smet(A, np0);
  const D3 t = pn_of(A, np0);
  D3 n1 = xn_of(A, np0, 0);
  const D3 n2 = xn_of(A, np0, 1);
  const double ps1 = ux * n1.x + uy * n1.y + uz * n1.z;
  const double ps2 = ux * n2.x + uy * n2.y + uz * n2.z;
  double dv, dn;
  if (fabs(ps2) < fabs(ps1)) {
    n1 = n2;
    dv = m[2];
    dn = m[4];
  } else {
    dv = m[1];
    dn = m[3];
  }
  double r[3][3];
  r[0][0] = t.x; r[1][0] = t.y; r[2][0] = t.z;
  r[0][1] = n1.y * t.z - n1.z * t.y;
  r[1][1] = n1.z * t.x - n1.x * t.z;
  r[2][1] = n1.x * t.y - n1.y * t.x;
  r[0][2] = n1.x; r[1][2] = n1.y; r[2][2] = n1.z;
  mr[0] = m[0] * r[0][0] * r[0][0] + dv * r[0][1] * r[0][1] + dn * r[0][2] * r[0][2];
  mr[1] = m[0] * r[0][0] * r[1][0] + dv * r[0][1] * r[1][1] + dn * r[0][2] * r[1][2];
  mr[2] = m[0] * r[0][0] * r[2][0] + dv * r[0][1] * r[2][1] + dn * r[0][2] * r[2][2];
  mr[3] = m[0] * r[1][0] * r[1][0] + dv * r[1][1] * r[1][1] + dn * r[1][2] * r[1][2];
  mr[4] = m[0] * r[1][0] * r[2][0] + dv * r[1][1] * r[2][1] + dn * r[1][2] * r[2][2];
  mr[5] = m[0] * r[2][0] * r[2][0] + dv * r[2][1] * r[2][1] + dn * r[2][2] * r[2][2];
}

// the tangent at ip of the curve under the edge [ip, ip + u] (MMG5_lenEdg's
// gammaprim): u at a singular / non-manifold point; along the point's tangent
// on a ridge edge (isedg); else u projected on the tangent plane of the side
// nearest to it (ridge point), of its xPoint normal (MG_REF), of its normal
__device__ D3 gammaprim(const StatArgs &A, int ip, double ux, double uy, double uz, bool isedg) {
  const unsigned tg = ptag_or0(A, ip);
  if (sin_or_nom(tg)) return D3{ux, uy, uz};
  if (isedg) {
    const D3 t = pn_of(A, ip);
    const double ps1 = ux * t.x + uy * t.y + uz * t.z;
    return D3{ps1 * t.x, ps1 * t.y, ps1 * t.z};
  }
  D3 n1;
  double ps1;
  if (TAG_GEO & tg) {
    n1 = xn_of(A, ip, 0);
    const D3 n2 = xn_of(A, ip, 1);
    ps1 = ux * n1.x + uy * n1.y + uz * n1.z;
    const double ps2 = ux * n2.x + uy * n2.y + uz * n2.z;
    if (fabs(ps2) < fabs(ps1)) {
      n1 = n2;
      ps1 = ps2;
    }
  } else if (TAG_REF & tg) {
    n1 = xn_of(A, ip, 0);
    ps1 = ux * n1.x + uy * n1.y + uz * n1.z;
  } else {
    n1 = pn_of(A, ip);
    ps1 = ux * n1.x + uy * n1.y + uz * n1.z;
  }
  return D3{ux - ps1 * n1.x, uy - ps1 * n1.y, uz - ps1 * n1.z};
}

__device__ __forceinline__ double qform(const double *m, D3 g) {
  return m[0] * g.x * g.x + m[3] * g.y * g.y + m[5] * g.z * g.z + 2.0 * m[1] * g.x * g.y + 2.0 * m[2] * g.x * g.z +
         2.0 * m[4] * g.y * g.z;
}

// MMG5_lenSurfEdg33_ani (ridmet 0, classic storage) / MMG5_lenSurfEdg_ani
// (ridmet 1: a non-singular ridge endpoint's metric rebuilt per direction),
// both through MMG5_lenEdg: the mean of the end tangents' lengths, a negative
// quadratic form counting as 1
__device__ double len_surf_ani(const StatArgs &A, int np0, int np1, bool isedg, bool ridmet) {
  const D3 c0 = sld3(A, np0), c1 = sld3(A, np1);
  const double ux = c1.x - c0.x, uy = c1.y - c0.y, uz = c1.z - c0.z;
  double m0[6], m1[6];
  const double *s0 = smet(A, np0), *s1 = smet(A, np1);
#pragma unroll
  for (int i = 0; i < 6; i++) { m0[i] = s0[i]; m1[i] = s1[i]; }
  if (ridmet) {
    const unsigned t0 = ptag_or0(A, np0), t1 = ptag_or0(A, np1);
    if (!sin_or_nom(t0) && (TAG_GEO & t0)) buildridmet(A, np0, ux, uy, uz, m0);
    if (!sin_or_nom(t1) && (TAG_GEO & t1)) buildridmet(A, np1, ux, uy, uz, m1);
  }
  const D3 g0 = gammaprim(A, np0, ux, uy, uz, isedg);
  const D3 g1 = gammaprim(A, np1, -ux, -uy, -uz, isedg);
  double l0 = qform(m0, g0), l1 = qform(m1, g1);
  if (l0 < 0.) l0 = 1.;
  if (l1 < 0.) l1 = 1.;
  return 0.5 * (sqrt(l0) + sqrt(l1));
}

// MMG5_moymet: the mean metric of tet v over its vertices that are not
// non-singular ridge points (false if none)
__device__ bool moymet(const StatArgs &A, const int *v, double mm[6]) {
  int n = 0;
#pragma unroll
  for (int i = 0; i < 6; i++) mm[i] = 0.0;
  for (int j = 0; j < 4; j++) {
    if (ridge_pt(ptag_or0(A, v[j]))) continue;
    n++;
    const double *m = smet(A, v[j]);
#pragma unroll
    for (int i = 0; i < 6; i++) mm[i] += m[i];
  }
  if (!n) return false;
  const double dd = 1. / n;
#pragma unroll
  for (int i = 0; i < 6; i++) mm[i] = mm[i] * dd;
  return true;
}

// MMG5_lenedg_ani (ridmet) / MMG5_lenedg33_ani of local edge ia = (ip1, ip2)
// of tet v (its packed xTetra edge tags et): a boundary edge of the xTetra along the
// surface, any other straight (MMG5_lenedgCoor_ani), a non-singular ridge
// endpoint then taking the tet's mean metric (MMG5_lenedgspl_ani)
__device__ double len_tet_ani(const StatArgs &A, const int *v, int ia, int ip1, int ip2, unsigned et) {
  if ((et >> (2 * ia)) & 1u) return len_surf_ani(A, ip1, ip2, ((et >> (2 * ia + 1)) & 1u) != 0, A.ridmet != 0);
  double m1[6], m2[6];
  const double *s1 = smet(A, ip1), *s2 = smet(A, ip2);
#pragma unroll
  for (int i = 0; i < 6; i++) { m1[i] = s1[i]; m2[i] = s2[i]; }
  if (A.ridmet) {
    if (ridge_pt(ptag_or0(A, ip1)) && !moymet(A, v, m1)) return 0.0;
    if (ridge_pt(ptag_or0(A, ip2)) && !moymet(A, v, m2)) return 0.0;
  }
  const D3 c1 = sld3(A, ip1), c2 = sld3(A, ip2);
  const double ux = c2.x - c1.x, uy = c2.y - c1.y, uz = c2.z - c1.z;
  double dd1 = mlen2(m1, ux, uy, uz), dd2 = mlen2(m2, ux, uy, uz);
  if (dd1 <= 0.0) dd1 = 0.0;
  if (dd2 <= 0.0) dd2 = 0.0;
  return (sqrt(dd1) + sqrt(dd2) + 4.0 * sqrt(0.5 * (dd1 + dd2))) / 6.0;
}

// MMG5_lenSurfEdg_iso on a size-6 metric as the reference calls it for the
// parallel edges with metRidTyp = 1 (src/quality_pmmg.c:466): h = met->m[ip],
// the Mmg array (6 per point) read flat, i.e. component ip % 6 of point ip / 6
__device__ double len_iso_flat(const StatArgs &A, int p1, int p2) {
  const D3 c1 = sld3(A, p1), c2 = sld3(A, p2);
  const double h1 = A.sol[(int64_t)(p1 / 6) * A.S + A.moff + p1 % 6];
  const double h2 = A.sol[(int64_t)(p2 / 6) * A.S + A.moff + p2 % 6];
  double l = (c2.x - c1.x) * (c2.x - c1.x) + (c2.y - c1.y) * (c2.y - c1.y) + (c2.z - c1.z) * (c2.z - c1.z);
  l = sqrt(l);
  const double r = h2 / h1 - 1.0;
  const bool flat = fabs(r) < PMX_EPS;
  const double q = l / (flat ? h1 : (h2 - h1));
  return flat ? q : q * pmx_log1p(r);
}

__device__ __forceinline__ void len_merge(LenPart &x, const LenPart &y) {
  x.avlen += y.avlen;
  if (y.lmin < x.lmin || (y.lmin == x.lmin && y.kmin < x.kmin)) { x.lmin = y.lmin; x.kmin = y.kmin; }
  if (y.lmax > x.lmax || (y.lmax == x.lmax && y.kmax < x.kmax)) { x.lmax = y.lmax; x.kmax = y.kmax; }
  x.ned += y.ned;
  x.nul += y.nul;
  for (int i = 0; i < 9; i++) x.hl[i] += y.hl[i];
}
__device__ __forceinline__ void len_init(LenPart &p) {
  p.avlen = 0.0; p.lmin = 1.e30; p.lmax = 0.0;
  p.kmin = 0x7fffffffffffffffLL; p.kmax = 0x7fffffffffffffffLL;
  p.ned = 0; p.nul = 0;
  for (int i = 0; i < 9; i++) p.hl[i] = 0;
}

__constant__ double BD[9] = {0.0, 0.3, 0.6, 0.7071, 0.9, 1.3, 1.4142, 2.0, 5.0};

// the edge (a, b) is measured elsewhere: an owned parallel edge of step 1 (or,
// exact_once, a parallel edge of another rank).  Sorted (min, max) keys,
// prefiltered by a per-point flag.
__device__ __forceinline__ bool par_excluded(const StatArgs &A, int a, int b) {
  if (!A.npar || !A.par_pt[a] || !A.par_pt[b]) return false;
  const unsigned long long key = ((unsigned long long)(unsigned)min(a, b) << 32) | (unsigned)max(a, b);
  int64_t lo = 0, hi = A.npar;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (A.par_key[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo < A.npar && A.par_key[lo] == key;
}

// Edge-length accumulator.  add() is called by every lane of a wave in
// converged control flow ("on" = this lane has an edge).  The histogram and
// the null-edge count are workgroup counters in LDS (one ds_add per edge);
// the sum and the extrema are per lane, reduced in a fixed tree at store().
// (Wave-uniform counters in scalar registers spilled to VGPR lanes: ~900
// readlane/writelane VALU instructions in the loop.)
struct LenAcc {
  unsigned *cnt;                       // LDS [10]: hl[0..8], null edges
  double avlen = 0.0, lmin = 1.e30, lmax = 0.0;
  long long kmin = 0x7fffffffffffffffLL, kmax = 0x7fffffffffffffffLL;
  __device__ explicit LenAcc(unsigned *lds) : cnt(lds) {
    if (threadIdx.x < 10) cnt[threadIdx.x] = 0u;
    __syncthreads();
  }
  __device__ void add(bool on, double len, long long key) {
    if (!on) return;
    if (len == 0.0) { atomicAdd(&cnt[9], 1u); return; }
    // bin i: BD[i] <= len < BD[i+1]; 8: len >= 5, negative or NaN -- the
    // number of bounds BD[1..8] at or below len
    int bin = 0;
#pragma unroll
    for (int i = 1; i < 9; i++) bin += (len >= BD[i]) ? 1 : 0;
    if (!(len >= 0.0)) bin = 8;
    atomicAdd(&cnt[bin], 1u);
    avlen += len;
    if (len < lmin || (len == lmin && key < kmin)) { lmin = len; kmin = key; }
    if (len > lmax || (len == lmax && key < kmax)) { lmax = len; kmax = key; }
  }
  // add() for a lane whose keys strictly increase from call to call (k_prilen:
  // lane t takes ring entry head + t of every round, and the ring is in key
  // order): an equal length never has the smaller key, so the extrema need no
  // key tie-break (the cross-lane tie-breaks stay in store())
  __device__ void add_ordered(bool on, double len, long long key) {
    if (!on) return;
    if (len == 0.0) { atomicAdd(&cnt[9], 1u); return; }
    int bin = 0;
#pragma unroll
    for (int i = 1; i < 9; i++) bin += (len >= BD[i]) ? 1 : 0;
    if (!(len >= 0.0)) bin = 8;
    atomicAdd(&cnt[bin], 1u);
    avlen += len;
    if (len < lmin) { lmin = len; kmin = key; }
    if (len > lmax) { lmax = len; kmax = key; }
  }
  // one LenPart per workgroup: wave shuffles of the per-lane fields, the 4
  // wave results in order, the LDS counters
  __device__ void store(LenPart *out) const {
    __shared__ LenPart wsh[4];
    double s = avlen, lo = lmin, hi = lmax;
    long long klo = kmin, khi = kmax;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double ys = __shfl_xor(s, o, 64), ylo = __shfl_xor(lo, o, 64), yhi = __shfl_xor(hi, o, 64);
      const long long yklo = __shfl_xor(klo, o, 64), ykhi = __shfl_xor(khi, o, 64);
      // the same tree on every lane: the lower lane's value first, so all
      // lanes agree bitwise
      const bool low = (threadIdx.x & o) == 0;
      s = low ? s + ys : ys + s;
      if (ylo < lo || (ylo == lo && yklo < klo)) { lo = ylo; klo = yklo; }
      if (yhi > hi || (yhi == hi && ykhi < khi)) { hi = yhi; khi = ykhi; }
    }
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
      LenPart p;
      p.avlen = s; p.lmin = lo; p.lmax = hi; p.kmin = klo; p.kmax = khi;
      p.ned = 0; p.nul = 0;
      for (int i = 0; i < 9; i++) p.hl[i] = 0;
      wsh[threadIdx.x >> 6] = p;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      LenPart r = wsh[0];
      for (int w = 1; w < (int)(blockDim.x >> 6); w++) len_merge(r, wsh[w]);
      r.ned = 0;
      for (int i = 0; i < 9; i++) { r.hl[i] = cnt[i]; r.ned += cnt[i]; }   // every non-null length has a bin
      r.nul = cnt[9];
      *out = r;
    }
  }
};

// IARE and the two other local vertices of edge ia, as nibble tables (no
// constant-memory load for a per-lane index)
__device__ __forceinline__ int iare0(int ia) { return (0x211000 >> (4 * ia)) & 15; }
__device__ __forceinline__ int iare1(int ia) { return (0x332321 >> (4 * ia)) & 15; }
__device__ __forceinline__ int oth0(int ia) { return (0x000112 >> (4 * ia)) & 15; }
__device__ __forceinline__ int oth1(int ia) { return (0x123233 >> (4 * ia)) & 15; }

__device__ __forceinline__ bool rec_4ridge(const StatArgs &A, const TetRec &t) {
  const int v[4] = {t.v[0], t.v[1], t.v[2], t.v[3]};
  return tet_4ridge(A, v);
}

// One rotation step around the edge (a, b): the shell entered tet r through
// its face (a, b, keep); the next tet is across the face (a, b, w) of r, i.e.
// opposite keep, and w (the sum of r's vertices minus a, b, keep, in modular
// arithmetic) is the vertex of the face crossed next.
__device__ __forceinline__ int rotate_step(const TetRec &r, int a, int b, int &keep) {
  const bool e0 = r.v[0] == keep, e1 = r.v[1] == keep, e2 = r.v[2] == keep;
  const int nb = e0 ? r.nb[0] : e1 ? r.nb[1] : e2 ? r.nb[2] : r.nb[3];
  keep = (int)((unsigned)r.v[0] + (unsigned)r.v[1] + (unsigned)r.v[2] + (unsigned)r.v[3] -
               (unsigned)a - (unsigned)b - (unsigned)keep);
  return nb;
}

// A shell record: from the workgroup's LDS batches when the tet is one of
// them (the current and the previous batch of 256 records: the in-cell and
// x-neighbour shells of a lexicographic numbering), else from HBM.
// L (lean): the batch bases and the tet index in 32-bit arithmetic (tet
// indices < 2^31; the no-batch sentinel is 2^31 modulo 2^32): prilen is
// VALU-bound, and these are on every shell step.
template <bool L>
__device__ __forceinline__ TetRec shell_rec(const StatArgs &A, const TetRec (*srec)[256], long long kb0,
                                            long long kb1, int c) {
  int idx;
  if constexpr (L) {
    const unsigned d0 = (unsigned)c - (unsigned)kb0, d1 = (unsigned)c - (unsigned)kb1;
    idx = d0 < 256u ? (int)d0 : (d1 < 256u ? 256 + (int)d1 : -1);
  } else {
    const unsigned long long d0 = (unsigned long long)((long long)c - kb0);
    const unsigned long long d1 = (unsigned long long)((long long)c - kb1);
    idx = d0 < 256ull ? (int)d0 : (d1 < 256ull ? 256 + (int)d1 : -1);
  }
  // one LDS index into both batches.  The LDS read is unconditional (slot 0
  // for a miss) and only a miss loads from HBM: with both loads conditional
  // the compiler merges them into one flat load through a selected pointer
  // (r06 ISA: flat_load_dwordx4, which waits on both memory counters)
  const int4 *l = reinterpret_cast<const int4 *>(&srec[0][0]) + 2 * (idx < 0 ? 0 : idx);
  int4 lv = l[0], ln = l[1];
  // (opaque to the optimiser: it would otherwise sink the LDS read into the
  // hit branch and merge the two again)
  asm volatile("" : "+v"(lv.x), "+v"(lv.y), "+v"(lv.z), "+v"(lv.w), "+v"(ln.x), "+v"(ln.y), "+v"(ln.z), "+v"(ln.w));
  if (idx < 0) {
    const int4 *g = reinterpret_cast<const int4 *>(A.tets) + 2 * (int64_t)c;
    lv = g[0];
    ln = g[1];
  }
  return TetRec{{lv.x, lv.y, lv.z, lv.w}, {ln.x, ln.y, ln.z, ln.w}};
}

// A shell record from HBM / L2, unconditionally (index 0: the unused slot
// 0).  No LDS path and no select on the loaded value: with either, the
// compiler turns the load into a branch (a select of a single-use load
// becomes a branch), and a conditional load makes it wait for every load in
// flight at the next join -- here the number of loads in flight is the same
// on every path, so the length's arithmetic overlaps the second step's
// records.
__device__ __forceinline__ TetRec shell_rec_g(const StatArgs &A, int c) {
  const int4 *g = reinterpret_cast<const int4 *>(A.tets) + 2 * (int64_t)c;
  const int4 gv = g[0], gn = g[1];
  return TetRec{{gv.x, gv.y, gv.z, gv.w}, {gn.x, gn.y, gn.z, gn.w}};
}

// True iff no admissible tet with index < k contains the edge (a, b) of tet
// k.  The shell is rotated from k through the two faces of k that contain the
// edge (cursors c0, c1; keep0/keep1 = the vertex of the face just crossed),
// both directions advanced together: a smaller index is met after min(d0, d1)
// steps, and a closed shell is covered when the cursors meet.  r0/r1 are the
// records of c0/c1, loaded by the caller (with the edge's points, in one
// round trip) and then one step ahead; without point tags an index alone
// decides, so a record is only loaded when the rotation goes on through it.
template <bool TAGS, bool L>
__device__ __forceinline__ bool owns_edge(const StatArgs &A, const TetRec (*srec)[256], long long kb0, long long kb1,
                                          int64_t k64, int a, int b, int c0, int c1, int keep0, int keep1,
                                          TetRec r0, TetRec r1) {
  using KT = typename std::conditional<L, int, int64_t>::type;
  const KT k = (KT)k64;
  for (int guard = 0; guard < 4096; guard++) {
    if (c0 == (int)k) c0 = 0;                    // a direction that wrapped around
    if (c1 == (int)k) c1 = 0;
    if (!c0 && !c1) return true;                 // both ends reached: every tet seen
    if (!TAGS && ((c0 && c0 < k) || (c1 && c1 < k))) return false;
    if (c0 && c0 == c1) {                        // the cursors meet on one tet
      if (!TAGS) return true;                  // its index was checked above
      return !(c0 < k && !rec_4ridge(A, r0));
    }
    int n0 = 0, n1 = 0;
    if (c0) {
      if (TAGS && c0 < k && !rec_4ridge(A, r0)) return false;
      n0 = rotate_step(r0, a, b, keep0);
    }
    if (c1) {
      if (TAGS && c1 < k && !rec_4ridge(A, r1)) return false;
      n1 = rotate_step(r1, a, b, keep1);
    }
    // closed shell: the next tet of one direction is the one the other just saw
    if (c0 && c1 && (n0 == c1 || n1 == c0)) return true;
    c0 = c0 ? n0 : 0;
    c1 = c1 ? n1 : 0;
    const bool need0 = c0 && c0 != (int)k, need1 = c1 && c1 != (int)k;
    if (!TAGS) {                               // decided by the indices: no load
      if ((need0 && c0 < k) || (need1 && c1 < k)) return false;
      if (need0 && c0 == c1) return true;
    }
    if (need0) r0 = shell_rec<L>(A, srec, kb0, kb1, c0);
    if (need1) r1 = shell_rec<L>(A, srec, kb0, kb1, c1);
  }
  return true;
}

// owns_edge without point tags, as straight-line selects for the first two
// rotation steps (a Kuhn shell of 4 or 6 tets is decided there: the two
// cursors meet), then owns_edge's loop for a longer shell.  The same
// decisions in the same order as owns_edge<false, L>; the loop's early
// returns become a "decided" mask, so the wave issues no branch per check.
// The steps are separate calls so that the caller can put work between them:
// k_prilen evaluates the edge's length while the second step's records load.
template <bool L, bool G>
struct FlatRot {
  int c0, c1, keep0, keep1;
  TetRec r0, r1;
  int i0, i1;                                      // where r0 / r1 were loaded from
  bool done = false, own = true;
  __device__ __forceinline__ void step(const StatArgs &A, const TetRec (*srec)[256], long long kb0, long long kb1,
                                       int64_t k64, int a, int b) {
    using KT = typename std::conditional<L, int, int64_t>::type;
    const KT k = (KT)k64;
    c0 = (c0 == (int)k) ? 0 : c0;
    c1 = (c1 == (int)k) ? 0 : c1;
    // the checks of owns_edge's loop head, first decision wins
    const bool d_end = !c0 && !c1;
    const bool d_small = (c0 && c0 < k) || (c1 && c1 < k);
    const bool d_meet = c0 && c0 == c1;
    own = done ? own : (d_end ? true : (d_small ? false : true));
    done = done || d_end || d_small || d_meet;
    const int n0 = c0 ? rotate_step(r0, a, b, keep0) : 0;
    const int n1 = c1 ? rotate_step(r1, a, b, keep1) : 0;
    const bool d_closed = c0 && c1 && (n0 == c1 || n1 == c0);
    done = done || d_closed;                       // own stays true
    c0 = c0 ? n0 : 0;
    c1 = c1 ? n1 : 0;
    const bool need0 = c0 && c0 != (int)k, need1 = c1 && c1 != (int)k;
    const bool d_small2 = (need0 && c0 < k) || (need1 && c1 < k);
    own = done ? own : !d_small2;
    done = done || d_small2 || (need0 && c0 == c1);
    if constexpr (G) {
      // a record not needed is reloaded from where it came (same value)
      i0 = (!done && need0) ? c0 : i0;
      i1 = (!done && need1) ? c1 : i1;
      r0 = shell_rec_g(A, i0);
      r1 = shell_rec_g(A, i1);
    } else {
      if (!done && need0) r0 = shell_rec<L>(A, srec, kb0, kb1, c0);
      if (!done && need1) r1 = shell_rec<L>(A, srec, kb0, kb1, c1);
    }
  }
  __device__ __forceinline__ bool finish(const StatArgs &A, const TetRec (*srec)[256], long long kb0, long long kb1,
                                         int64_t k64, int a, int b) {
    if (done) return own;
    return owns_edge<false, L>(A, srec, kb0, kb1, k64, a, b, c0, c1, keep0, keep1, r0, r1);
  }
};

// ---- prilen: unique edges by shell ownership, one pass ------------------------
//
// Each workgroup walks a contiguous range of tets, 256 records per batch:
//  1. every thread reads its tet record (prefetched one batch ahead, kept in a
//     double-buffered LDS array), drops the edges a smaller face neighbour
//     owns (no point tags) and queues the others, in (k, ia) order, in an LDS
//     ring;
//  2. the ring is consumed in full rounds of 256 edges -- one per thread:
//     the edge's points and the first shell step's records are loaded in one
//     round trip, the length is computed, the shell rotation decides whether
//     it counts.  Fewer than 256 left over wait for the next batch, unless
//     they belong to the previous batch, whose LDS records are about to be
//     overwritten (then a partial round).
// (r01 ran the phases as separate launches through a global list: 6.25 ms at
// 125M tets; a fused version with one round trip per dependent load and
// partial rounds after every batch: 7.2 ms.)
#define LEN_QCAP 2048                 // > 255 left over + 6 * 256 queued
// SURF (tensor metrics with surface data or ridge storage): every length by
// len_tet_ani from the owner tet's xTetra edge tags and vertices.
// X (measurement only, PMX_PRILEN_EXP): bits 0-1 with PMX_EXPERIMENTS=1 give
// wrong results by design -- bit 0 no length evaluation (1.0), bit 1 no shell
// rotation (every candidate counts), the VALU breakdown of the r05 verdict's
// item 6; bit 2 (4: same results) the rotation as owns_edge's loop from the
// first step instead of owns_edge_flat (r05's kernel, for the A/B).
template <bool ANI, bool TAGS, bool PAR, int W = 1, bool L = false, bool SURF = false, int X = 0>
__global__ __launch_bounds__(256, W) void k_prilen(StatArgs A, LenPart *parts) {
  __shared__ TetRec srec[2][256];
  __shared__ unsigned short q[LEN_QCAP + 2];     // + the spare entry of unset slots
  __shared__ unsigned wcnt[4];
  __shared__ long long kbase[2];                 // first tet of each LDS buffer
  __shared__ unsigned lcnt[10];
  LenAcc acc(lcnt);
  // The tets a workgroup takes, batch by batch (kb = first tet of a batch,
  // valid while kb <= k1):
  //  * contiguous (sched_chunk 0): XCD-contiguous ranges, one per workgroup;
  //    the shells and points of the next z-layer of cells are another
  //    range's, read by the same L2;
  //  * front (sched_chunk C): each XCD's eighth of the tets is dealt out in
  //    chunks of C batches, round-robin over the XCD's co-resident
  //    workgroups, so the XCD works on one contiguous window that moves
  //    forward: a +y shell (a few batches ahead) is a batch another
  //    workgroup of the same L2 loads about then.
  // Either way a workgroup's batches come in increasing tet order (the ring's
  // keys stay ordered).
  const unsigned tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t C = A.sched_chunk;
  int64_t lb, k0, k1, jump = 0, xlo = 1;
  if (C == 0) {
    lb = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t per = (A.ne + gridDim.x - 1) / gridDim.x;
    k0 = 1 + lb * per;
    k1 = min(A.ne, k0 + per - 1);
  } else {
    lb = blockIdx.x;
    const int64_t x = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int64_t G = ((int64_t)gridDim.x - x + 7) >> 3;     // this XCD's workgroups
    xlo = 1 + x * A.ne / 8;
    k1 = (x + 1) * A.ne / 8;
    k0 = xlo + j * C * 256;
    jump = (G - 1) * C * 256;
  }
  auto next_batch = [&](int64_t kb) -> int64_t {
    if (C == 0) return kb + 256;
    return kb + 256 + (((kb - xlo) >> 8) % C == C - 1 ? jump : 0);
  };
  unsigned head = 0, tail = 0;                   // ring positions (uniform)
  // each batch's records go to an LDS buffer; the next batch's are loaded at
  // the start of the batch and written to the other buffer after its rounds,
  // so the load is in flight during them (loaded from a clamped index: no
  // merge copy that would wait for it; records past k1 are never used)
  const int4 *recs = reinterpret_cast<const int4 *>(A.tets);
  {
    const int64_t kn = max<int64_t>(1, min(k0 + (int64_t)tid, A.ne));
    int4 *srow = reinterpret_cast<int4 *>(&srec[0][tid]);
    srow[0] = recs[2 * kn];
    srow[1] = recs[2 * kn + 1];
    // no second batch yet: a base no index reaches, in 64 and in 32 bits
    if (tid == 0) { kbase[0] = k0; kbase[1] = -(1LL << 40) + (1LL << 31); }
    __syncthreads();
  }

  int buf = 0;
  for (int64_t kb = k0;; buf ^= 1) {
    const bool more = kb <= k1;
    if (!more && head == tail) break;
    const unsigned prev_end = tail;              // entries before it: the previous batch
    const int64_t kbn = next_batch(kb);
    const int64_t kn = max<int64_t>(1, min(kbn + (int64_t)tid, A.ne));
    const int4 pv = recs[2 * kn], pn = recs[2 * kn + 1];
    if (more) {
      const int64_t k = kb + tid;
      const TetRec t = srec[buf][tid];
      unsigned m = 0;
      if (k <= k1) {
        const int v[4] = {t.v[0], t.v[1], t.v[2], t.v[3]};
        if (t.v[0] > 0 && !(TAGS && tet_4ridge(A, v))) {
          m = 0x3fu;
          if constexpr (!TAGS) {
            // a face neighbour with a smaller index disowns the face's three
            // edges (those not through the opposite local vertex f):
            // f = 0: edges 3,4,5; 1: 1,2,5; 2: 0,2,4; 3: 0,1,3 -- the same
            // test as "n0 or n1 smaller" per edge, n0/n1 = the neighbours
            // across the two faces that hold it
            const unsigned emask[4] = {0x38u, 0x26u, 0x15u, 0x0bu};
#pragma unroll
            for (int f = 0; f < 4; f++) {
              const int n = t.nb[f];
              bool sm;
              if constexpr (L) sm = (unsigned)n - 1u < (unsigned)k - 1u;   // 1 <= n < k
              else sm = n && n < k;
              m &= sm ? ~emask[f] : ~0u;
            }
          }
        }
      }
      // ring positions in (thread, ia) order: the wave's exclusive prefix of
      // the per-thread counts through one ballot per edge slot (mbcnt), the
      // wave totals in LDS
      unsigned pre = 0, wtot = 0;
#pragma unroll
      for (int ia = 0; ia < 6; ia++) {
        const unsigned long long bb = __ballot((m >> ia) & 1u);
        pre = __builtin_amdgcn_mbcnt_hi((unsigned)(bb >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bb, pre));
        wtot += (unsigned)__popcll(bb);
      }
      if (lane == 0) wcnt[wv] = wtot;
      __syncthreads();
      unsigned base = 0, total = 0;
      for (unsigned w = 0; w < 4; w++) {
        base += (w < wv) ? wcnt[w] : 0u;
        total += wcnt[w];
      }
      total = __builtin_amdgcn_readfirstlane(total);
      unsigned pos = tail + base + pre;
      // unconditional stores: an unset slot writes the spare entry q[LEN_QCAP]
#pragma unroll
      for (int ia = 0; ia < 6; ia++) {
        const unsigned bit = (m >> ia) & 1u;
        q[bit ? (pos & (LEN_QCAP - 1)) : LEN_QCAP] = (unsigned short)((buf << 11) | (tid << 3) | ia);
        pos += bit;
      }
      __syncthreads();
      tail += total;
    }
    // full rounds; a partial one while entries of the previous batch remain
    // (their LDS records are rewritten next); everything once the tets ran out
    const unsigned avail = tail - head;
    unsigned nr = avail >> 8;
    if (!more) nr = (avail + 255u) >> 8;
    else if (head + (nr << 8) < prev_end) nr++;
    const long long kb0 = kbase[0], kb1 = kbase[1];   // fixed during the rounds
    for (unsigned r = 0; r < nr; r++) {
      const unsigned cnt = min(256u, tail - head);
      bool on = false;
      double len = 0.0;
      long long key = 0;
      if (tid < cnt) {
        const unsigned it = q[(head + tid) & (LEN_QCAP - 1)];
        const int eb = (int)(it >> 11), slot = (int)((it >> 3) & 255u), ia = (int)(it & 7u);
        // the record's fields by LDS address (no per-lane selects)
        const int *sv = srec[eb][slot].v, *sn = srec[eb][slot].nb;
        const int64_t kk = (eb ? kb1 : kb0) + slot;
        const int o0 = oth0(ia), o1 = oth1(ia);
        const int a = sv[iare0(ia)], b = sv[iare1(ia)], keep0 = sv[o1], keep1 = sv[o0];
        const int c0 = sn[o0], c1 = sn[o1];
        // the first rotation step's records, issued with the points' loads
        TetRec r0{}, r1{};
        // FLAT: the rotation's first two steps as straight-line selects (no
        // point tags); GREC (X bit 3): the flat steps' records always from
        // HBM / L2, no LDS path; EARLY (X bit 4): the first step before the
        // length (its records wanted first), the second step's loads in flight
        // during the length's arithmetic
        constexpr bool FLAT = !(X & 6) && !TAGS;
        constexpr bool GREC = FLAT && (X & 8);
        constexpr bool EARLY = FLAT && (X & 16) && !ANI && !SURF && !(X & 1);
        if constexpr (GREC) {
          r0 = shell_rec_g(A, c0);
          r1 = shell_rec_g(A, c1);
        } else if constexpr (!(X & 2)) {
          if (c0) r0 = shell_rec<L>(A, srec, kb0, kb1, c0);
          if (c1) r1 = shell_rec<L>(A, srec, kb0, kb1, c1);
        }
        FlatRot<L, GREC> fr{c0, c1, keep0, keep1, r0, r1, c0, c1};
        if constexpr (EARLY) {
          const IsoEdge e = iso_edge_load(A, a, b);   // in flight during the step
          fr.step(A, srec, kb0, kb1, kk, a, b);
          len = iso_edge_len(e);
        } else if constexpr (SURF) {
          const int vv[4] = {sv[0], sv[1], sv[2], sv[3]};
          len = len_tet_ani(A, vv, ia, a, b, A.etag ? (unsigned)A.etag[kk] : 0u);
        } else if constexpr (X & 1) {
          len = 1.0 + 1e-9 * (double)(a & 7);
        } else {
          len = edge_len_t<ANI, (X & 128) != 0>(A, a, b);
        }
        if constexpr (X & 2) on = true;
        else if constexpr (FLAT) {
          if constexpr (!EARLY) fr.step(A, srec, kb0, kb1, kk, a, b);
          fr.step(A, srec, kb0, kb1, kk, a, b);
          on = fr.finish(A, srec, kb0, kb1, kk, a, b) && !(PAR && par_excluded(A, a, b));
        } else
          on = owns_edge<TAGS, L>(A, srec, kb0, kb1, kk, a, b, c0, c1, keep0, keep1, r0, r1) &&
               !(PAR && par_excluded(A, a, b));
        if constexpr (L) key = LEN_STEP2 + (long long)(6u * (unsigned)kk + (unsigned)ia);   // 6 ne < 2^32
        else key = LEN_STEP2 + 6 * kk + ia;
      }
      if constexpr (L) acc.add_ordered(on, len, key);
      else acc.add(on, len, key);
      head += cnt;
    }
    if (more) {                                  // no entry of the previous batch is left
      __syncthreads();                           // ... once every wave is past its rounds
      int4 *srow = reinterpret_cast<int4 *>(&srec[buf ^ 1][tid]);
      srow[0] = pv;
      srow[1] = pn;
      if (tid == 0) kbase[buf ^ 1] = kbn;
    }
    __syncthreads();                             // srec, wcnt, kbase rewritten next
    kb = kbn;
  }
  acc.store(parts + lb);
}

// ---- prilen, edge-bucket variant (A/B of the shell rotation) --------------------
//
// The r04 verdict's alternative to the rotation: unique edges through buckets
// of the smaller endpoint instead of shell walks.  The face-neighbour filter
// of k_prilen keeps the candidates (a tet's edge no smaller face neighbour
// disowns: 1.0015 per unique edge on Kuhn meshes); each candidate goes to the
// bucket of its smaller endpoint (counts and placement aggregated per
// workgroup in an LDS hash, one global atomic per distinct bucket -- the
// LDS-aggregated bucketing of pmx_topo.hip); an edge's owner is its candidate
// with the smallest key 6 k + ia in the bucket (the reference's first
// occurrence), found by scanning the bucket.  Point tags (the 4-ridge
// filter disables the face filter) and the surface-aware tensor lengths keep
// the rotation.  Selected by PMX_PRILEN_BUCKETS=1.
#define PB_HT 2048
__device__ __forceinline__ int pb_slot(int *keys, int a) {
  unsigned h = ((unsigned)a * 2654435761u) >> (32 - 11);
  for (;;) {
    const int old = atomicCAS(&keys[h], -1, a);
    if (old == -1 || old == a) return (int)h;
    h = (h + 1) & (PB_HT - 1);
  }
}
// the candidate edges of tet k (bit ia): valid tet, no smaller face neighbour
// on either face containing the edge
__device__ __forceinline__ unsigned pb_cands(const TetRec &t, int64_t k) {
  unsigned m = 0;
  if (t.v[0] <= 0) return 0;
#pragma unroll
  for (int ia = 0; ia < 6; ia++) {
    const int n0 = pick_nb(t, oth0(ia)), n1 = pick_nb(t, oth1(ia));
    if ((n0 && n0 < k) || (n1 && n1 < k)) continue;
    m |= 1u << ia;
  }
  return m;
}
// PASS 0 counts, PASS 1 places: records {a, b, 6 k + ia, 0} in the reference's
// orientation (a = v[IARE[ia][0]]), bucket = min(a, b)
template <int PASS>
__global__ __launch_bounds__(256) void k_pb_bucket(const TetRec *__restrict__ tets, int64_t ne,
                                                   unsigned *__restrict__ cnt, int4 *__restrict__ rec) {
  __shared__ int keys[PB_HT];
  __shared__ unsigned cnts[PB_HT];
  for (int i = threadIdx.x; i < PB_HT; i += blockDim.x) { keys[i] = -1; cnts[i] = 0u; }
  __syncthreads();
  const int64_t k = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x + 1;
  TetRec t{};
  unsigned m = 0;
  int slot[6];
  unsigned rank[6];
  if (k <= ne) {
    t = tets[k];
    m = pb_cands(t, k);
#pragma unroll
    for (int ia = 0; ia < 6; ia++) {
      slot[ia] = 0;
      rank[ia] = 0;
      if (!((m >> ia) & 1u)) continue;
      const int a = pick_v(t, iare0(ia)), b = pick_v(t, iare1(ia));
      slot[ia] = pb_slot(keys, min(a, b));
      rank[ia] = atomicAdd(&cnts[slot[ia]], 1u);
    }
  }
  __syncthreads();
  if (PASS == 0) {
    for (int i = threadIdx.x; i < PB_HT; i += blockDim.x)
      if (keys[i] >= 0) atomicAdd(cnt + keys[i], cnts[i]);
    return;
  }
  // one reservation per bucket: the workgroup's run starts there
  for (int i = threadIdx.x; i < PB_HT; i += blockDim.x)
    if (keys[i] >= 0) cnts[i] = atomicAdd(cnt + keys[i], cnts[i]);
  __syncthreads();
#pragma unroll
  for (int ia = 0; ia < 6; ia++) {
    if (!((m >> ia) & 1u)) continue;
    const int a = pick_v(t, iare0(ia)), b = pick_v(t, iare1(ia));
    rec[cnts[slot[ia]] + rank[ia]] = make_int4(a, b, (int)(6u * (unsigned)k + (unsigned)ia), 0);
  }
}
// one thread per candidate: the owner (smallest key among the bucket's
// candidates of the same edge) measures it
template <bool ANI, bool PAR>
__global__ __launch_bounds__(256) void k_pb_edges(StatArgs A, const int4 *__restrict__ rec, int64_t nrec,
                                                  const unsigned *__restrict__ off, LenPart *parts) {
  __shared__ unsigned lcnt[10];
  LenAcc acc(lcnt);
  const int64_t lb = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t per = ((nrec + gridDim.x - 1) / gridDim.x + 255) / 256 * 256;
  const int64_t r0 = lb * per, r1 = min(nrec, r0 + per);
  for (int64_t rb = r0; rb < r0 + per; rb += blockDim.x) {   // uniform trip count
    const int64_t r = rb + threadIdx.x;
    bool on = false;
    double len = 0.0;
    long long key = 0;
    if (r < r1) {
      const int4 e = rec[r];
      const int lo = min(e.x, e.y), hi = max(e.x, e.y);
      const unsigned me = (unsigned)e.z;
      const unsigned b0 = off[lo], b1 = off[lo + 1];
      bool own = true;
      for (unsigned q = b0; q < b1; q++) {
        const int4 o = rec[q];
        own = own && !(max(o.x, o.y) == hi && (unsigned)o.z < me);
      }
      on = own && !(PAR && par_excluded(A, e.x, e.y));
      if (on) len = edge_len_t<ANI>(A, e.x, e.y);
      key = LEN_STEP2 + (long long)me;
    }
    acc.add(on, len, key);
  }
  acc.store(parts + lb);
}

// step 1 of the distributed prilen: the owned parallel edges, in list order,
// each once (src/quality_pmmg.c:445-502); one workgroup.  The kernel the
// reference selects at :462-466: MMG5_lenSurfEdg33_ani for a tensor metric in
// classic storage (isedg from the edge's hash tag), else MMG5_lenSurfEdg_iso
// -- for a tensor metric with metRidTyp = 1 on the flat array, as written
__global__ __launch_bounds__(256) void k_prilen_par(StatArgs A, const int2 *edges, const uint16_t *etags,
                                                    int64_t n, LenPart *part) {
  __shared__ unsigned lcnt[10];
  LenAcc acc(lcnt);
  for (int64_t base = 0; base < n; base += blockDim.x) {
    const int64_t i = base + threadIdx.x;
    const bool on = i < n;
    double len = 0.0;
    if (on) {
      const int2 e = edges[i];
      if (A.msize != 6) len = edge_len(A, e.x, e.y);
      else if (A.ridmet) len = len_iso_flat(A, e.x, e.y);
      else len = len_surf_ani(A, e.x, e.y, etags && (etags[i] & TAG_GEO), false);
    }
    acc.add(on, len, i);
  }
  acc.store(part);
}

// fixed-order reduction; the last level resolves the extremal edges' endpoints
// (step-1 keys: the list entry; step-2 keys: the tet's local edge)
__global__ __launch_bounds__(256) void k_prilen_final(const LenPart *parts, int n, LenPart *res,
                                                      pmx_len_part *pub, const TetRec *tets,
                                                      const int2 *par_edges) {
  __shared__ LenPart sh[256];
  LenPart p;
  len_init(p);
  const int pb = (n + gridDim.x - 1) / gridDim.x;
  const int lo = blockIdx.x * pb, hi = min(n, lo + pb);
  int per = (hi - lo + 255) / 256;
  for (int b = lo + threadIdx.x * per; b < min(hi, lo + (int)(threadIdx.x + 1) * per); b++)
    len_merge(p, parts[b]);
  sh[threadIdx.x] = p;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) len_merge(sh[threadIdx.x], sh[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  if (res) res[blockIdx.x] = sh[0];
  if (pub) {
    const LenPart &r = sh[0];
    pmx_len_part o;
    o.avlen = r.avlen; o.lmin = r.ned ? r.lmin : 1.e30; o.lmax = r.lmax;
    o.ned = r.ned; o.nullEdge = r.nul;
    for (int i = 0; i < 9; i++) o.hl[i] = r.hl[i];
    o.amin = o.bmin = o.amax = o.bmax = 0;
    long long keys[2] = {r.kmin, r.kmax};
    long long ab[2][2] = {{0, 0}, {0, 0}};
    for (int j = 0; j < 2 && r.ned; j++) {
      const long long key = keys[j];
      if (key >= LEN_STEP2) {
        const long long kk = (key - LEN_STEP2) / 6;
        const int ia = (int)((key - LEN_STEP2) % 6);
        const TetRec t = tets[kk];
        ab[j][0] = pick_v(t, IARE[ia][0]);
        ab[j][1] = pick_v(t, IARE[ia][1]);
      } else {
        ab[j][0] = par_edges[key].x;
        ab[j][1] = par_edges[key].y;
      }
    }
    o.amin = ab[0][0]; o.bmin = ab[0][1]; o.amax = ab[1][0]; o.bmax = ab[1][1];
    *pub = o;
  }
}

// ---- the new mesh (PMMG_tetraQual after the interpolation) ----------------------

__global__ __launch_bounds__(256) void k_conn_from_host(const int4 *__restrict__ src, int64_t n,
                                                       int4 *__restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

// ---- host side ------------------------------------------------------------------

// partial records per pass: a function of ne only (the fixed-order final
// reduction then gives the same sums on every run); enough workgroups to fill
// 256 CUs several times over, each a contiguous range of >= 2048 tets
#define FINAL_GRID 64
static int stat_blocks(int64_t ne) {
  return (int)std::max<int64_t>(256, std::min<int64_t>(16384, ne / 2048));
}

static bool ensure_tetv(pmx_ctx *ctx) {
  if (ctx->have_tetv) return true;
  if (!pmx_dgrow(ctx, ctx->d_tetv, (size_t)(ctx->ne + 1))) return false;
  launch_tet_conn(ctx->d_tets.p, ctx->ne + 1, ctx->d_tetv.p, ctx->stream);
  ctx->have_tetv = true;
  return true;
}

// the statistics' view of the background group
static bool stat_args(pmx_ctx *ctx, StatArgs &A) {
  if (!ctx->have_bg) { ctx->err = "statistics: upload a group first"; return false; }
  // the 16-B connectivity stream of the quality pass, derived from the tet
  // records on the first statistics call after an upload (the transfer step
  // itself does not need it)
  if (!ensure_tetv(ctx)) return false;
  A = StatArgs{};
  A.xyz = ctx->d_xyz.p;
  A.xstride = 3;
  A.vbase = 0;
  A.tets = ctx->d_tets.p;
  A.tetv = ctx->d_tetv.p;
  A.ne = ctx->ne;
  A.sol = ctx->d_sol.p;
  A.S = ctx->sd.S;
  A.msize = ctx->sd.imet >= 0 ? ctx->sd.size[ctx->sd.imet] : 0;
  A.moff = ctx->sd.imet >= 0 ? ctx->sd.off[ctx->sd.imet] : 0;
  A.ptag = ctx->have_ptag ? ctx->d_ptag.p : nullptr;
  return true;
}

static bool ensure_red(pmx_ctx *ctx, size_t bytes) {
  return pmx_dgrow(ctx, ctx->d_red, (bytes + 7) / 8);
}

// qualhisto partial of the mesh described by A (background or new mesh)
static int qual_partial(pmx_ctx *ctx, const StatArgs &A, int opt, double *qual_dev, int use_stored,
                        pmx_qual_part *pub, long long np) {
  const int nb = stat_blocks(A.ne);
  if (!ensure_red(ctx, sizeof(QualPart) * (nb + FINAL_GRID + 1))) return 0;
  QualPart *parts = (QualPart *)ctx->d_red.p;
  hipStream_t s = ctx->stream;
  const bool ani = A.msize == 6, out = opt == PMX_OUTQUA && A.ptag;
  double *q = use_stored ? qual_dev : nullptr;
  // MMG3D_computeInqua takes MMG5_caltet33_ani (classic storage);
  // MMG3D_computeOutqua MMG5_orcal -> MMG5_caltet_ani, the ridge-storage mean
  // (ridge points left out, caltet_ani_rid) -- unless the caller's stored
  // qualities are used
  StatArgs B = A;
  if (ani && opt == PMX_OUTQUA && !use_stored) {
    B.ridmet = 1;
    B.rtag = A.ptag;
  }
  using KQ = void (*)(StatArgs, double *, QualPart *);
  static const KQ kq[2][2][2] = {
      {{k_qual<false, false, QM_HISTO>, k_qual<false, false, QM_STORED>},
       {k_qual<false, true, QM_HISTO>, k_qual<false, true, QM_STORED>}},
      {{k_qual<true, false, QM_HISTO>, k_qual<true, false, QM_STORED>},
       {k_qual<true, true, QM_HISTO>, k_qual<true, true, QM_STORED>}}};
  hipLaunchKernelGGL(kq[ani][out][use_stored ? 1 : 0], dim3(nb), dim3(256), 0, s, B, q, parts);
  QualPart *mid = parts + nb;
  hipLaunchKernelGGL(k_qual_final, dim3(FINAL_GRID), dim3(256), 0, s, parts, nb, mid,
                     (pmx_qual_part *)nullptr, 0LL);
  hipLaunchKernelGGL(k_qual_final, dim3(1), dim3(256), 0, s, mid, FINAL_GRID, (QualPart *)nullptr, pub, np);
  if (hipGetLastError() != hipSuccess) { ctx->err = "qualhisto: launch failed"; return 0; }
  return 1;
}

static void qual_to_stats(const pmx_qual_part &r, pmx_qual_stats *st) {
  memset(st, 0, sizeof *st);
  st->ne = r.ne; st->np = r.np; st->max = r.max; st->min = r.min; st->avg = r.avg;
  st->iel = r.iel; st->good = r.good; st->med = r.med; st->nrid = r.nrid;
  for (int i = 0; i < 5; i++) st->his[i] = r.his[i];
  st->iel_grp = (int)r.iel_grp;
  st->cpu = 0;
}
static void len_to_stats(const pmx_len_part &r, pmx_len_stats *st) {
  memset(st, 0, sizeof *st);
  st->ned = r.ned; st->nullEdge = r.nullEdge; st->avlen = r.avlen; st->lmin = r.lmin; st->lmax = r.lmax;
  st->amin = r.amin; st->bmin = r.bmin; st->amax = r.amax; st->bmax = r.bmax;
  for (int i = 0; i < 9; i++) st->hl[i] = r.hl[i];
  st->cpu_min = st->cpu_max = 0;
}

extern "C" {

int pmx_upload_point_tags(pmx_ctx *ctx, const uint16_t *tag, int64_t stride) {
  if (!ctx) return 0;
  ctx->have_ptag = false;
  if (!ctx->have_bg) { ctx->err = "pmx_upload_point_tags: upload a background first"; return 0; }
  if (!tag) return 1;                       // no tags: no ridge points
  hipSetDevice(ctx->device);
  const int64_t np = ctx->np;
  char *st = pmx_hstage(ctx, (size_t)(np + 1) * 2);
  if (!st) return 0;
  uint16_t *h = (uint16_t *)st;
  h[0] = 0;
  for (int64_t i = 1; i <= np; i++) h[i] = *(const uint16_t *)((const char *)tag + i * stride);
  if (!pmx_dgrow(ctx, ctx->d_ptag, (size_t)(np + 1))) return 0;
  if (hipMemcpyAsync(ctx->d_ptag.p, h, (size_t)(np + 1) * 2, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess) {
    ctx->err = "pmx_upload_point_tags: copy";
    return 0;
  }
  ctx->have_ptag = true;
  return 1;
}

// Mmg's surface data of the background: packed on the host (the xTetra edge
// tags to 2 bits per edge of each tet, the normals and xPoint indices as
// arrays), checked, uploaded.  Replaces the previous upload's.
int pmx_upload_surface(pmx_ctx *ctx, const pmx_surface_view *sv) {
  if (!ctx) return 0;
  ctx->have_surf = false;
  if (!ctx->have_bg) { ctx->err = "pmx_upload_surface: upload a background first"; return 0; }
  if (!sv) return 1;                        // no surface data: no xTetra, zero normals
  const char *who = "pmx_upload_surface";
  const int64_t np = ctx->np, ne = ctx->ne, nxt = sv->nxt, nxp = sv->nxp;
  if (nxt < 0 || nxp < 0 || (nxt > 0 && (!sv->tetra_xt || !sv->xtetra_tag || sv->tetra_stride < 4 ||
                                        sv->xtetra_stride < 12)) ||
      (!sv->point_n != !sv->point_xp) || (sv->point_n && sv->point_stride < 24) ||
      (nxp > 0 && (!sv->xpoint_n1 || !sv->xpoint_n2 || sv->xpoint_stride < 24))) {
    ctx->err = std::string(who) + ": bad view";
    return 0;
  }
  hipSetDevice(ctx->device);
  std::vector<uint16_t> et((size_t)(ne + 1), 0);
  std::vector<double> pn((size_t)(np + 1) * 3, 0.0), xpn((size_t)(nxp + 1) * 6, 0.0);
  std::vector<int> pxp((size_t)(np + 1), 0);
  std::atomic<bool> bad{false};
  if (nxt > 0)
    pmx_par_for(1, ne + 1, [&](int64_t k0, int64_t k1) {
      for (int64_t k = k0; k < k1; k++) {
        const int xt = *(const int *)((const char *)sv->tetra_xt + k * sv->tetra_stride);
        if (xt == 0) continue;
        if (xt < 0 || xt > nxt) { bad = true; continue; }
        const uint16_t *tg = (const uint16_t *)((const char *)sv->xtetra_tag + (int64_t)xt * sv->xtetra_stride);
        unsigned b = 0;
        for (int ia = 0; ia < 6; ia++)
          b |= ((tg[ia] & PMX_TAG_BDY) ? 1u : 0u) << (2 * ia) | ((tg[ia] & PMX_TAG_GEO) ? 1u : 0u) << (2 * ia + 1);
        et[(size_t)k] = (uint16_t)b;
      }
    });
  if (sv->point_n)
    pmx_par_for(1, np + 1, [&](int64_t i0, int64_t i1) {
      for (int64_t i = i0; i < i1; i++) {
        const double *n = (const double *)((const char *)sv->point_n + i * sv->point_stride);
        const int xp = *(const int *)((const char *)sv->point_xp + i * sv->point_stride);
        if (xp < 0 || xp > nxp) { bad = true; continue; }
        pxp[(size_t)i] = xp;
        for (int c = 0; c < 3; c++) pn[(size_t)(3 * i + c)] = n[c];
      }
    });
  for (int64_t x = 1; x <= nxp; x++) {
    const double *n1 = (const double *)((const char *)sv->xpoint_n1 + x * sv->xpoint_stride);
    const double *n2 = (const double *)((const char *)sv->xpoint_n2 + x * sv->xpoint_stride);
    for (int c = 0; c < 3; c++) { xpn[(size_t)(6 * x + c)] = n1[c]; xpn[(size_t)(6 * x + 3 + c)] = n2[c]; }
  }
  if (bad) { ctx->err = std::string(who) + ": an xTetra or xPoint index is out of range"; return 0; }
  hipStream_t s = ctx->stream;
  if (!pmx_dgrow(ctx, ctx->d_etag, et.size()) || !pmx_dgrow(ctx, ctx->d_pn, pn.size()) ||
      !pmx_dgrow(ctx, ctx->d_pxp, pxp.size()) || !pmx_dgrow(ctx, ctx->d_xpn, xpn.size()))
    return 0;
  if (hipMemcpyAsync(ctx->d_etag.p, et.data(), et.size() * 2, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(ctx->d_pn.p, pn.data(), pn.size() * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(ctx->d_pxp.p, pxp.data(), pxp.size() * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(ctx->d_xpn.p, xpn.data(), xpn.size() * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    ctx->err = std::string(who) + ": copy";
    return 0;
  }
  ctx->have_surf = true;
  return 1;
}

// metRidTyp selects Mmg's ridge-metric storage (src/quality_pmmg.c:462,527,
// 726).  For a size-1 metric (or none) both values take the same isotropic
// arithmetic.  With a size-6 metric:
//  * the quality (MMG3D_tetraQual: 0 -> MMG5_caltet33_ani, 1 -> MMG5_orcal ->
//    MMG5_caltet_ani) is restated for both: 1 averages the metric over the
//    vertices that are not non-singular ridge points (MMG5_moymet), which
//    needs the point tags (caltet_ani_rid);
//  * the edge lengths (0: MMG5_lenedg33_ani, 1: MMG5_lenedg_ani) measure the
//    xTetra's boundary edges along the curved surface (pmx_upload_surface),
//    and 1 rebuilds a ridge point's metric per direction (MMG5_buildridmet)
//    or takes the tet's mean (MMG5_lenedgspl_ani): len_tet_ani.
static bool check_met_rid_typ(pmx_ctx *ctx, int metRidTyp, int msize, const char *who, bool lengths) {
  if (metRidTyp != 0 && metRidTyp != 1) {
    ctx->err = std::string(who) + ": metRidTyp must be 0 or 1";
    return false;
  }
  (void)msize;
  (void)lengths;
  return true;
}

int pmx_tetra_qual(pmx_ctx *ctx, int metRidTyp, double *qual, int64_t qual_cap) {
  if (!ctx) return 0;
  hipSetDevice(ctx->device);
  StatArgs A;
  if (!stat_args(ctx, A)) return 0;
  if (!check_met_rid_typ(ctx, metRidTyp, A.msize, "pmx_tetra_qual", false)) return 0;
  if (qual && qual_cap < ctx->ne + 1) {
    ctx->err = "pmx_tetra_qual: qual holds " + std::to_string(qual_cap) + " doubles, ne+1 = " +
               std::to_string(ctx->ne + 1) + " needed";
    return 0;
  }
  A.ridmet = metRidTyp == 1 && A.msize == 6;
  A.rtag = A.ptag;
  if (A.ridmet && !A.rtag) {
    ctx->err = "pmx_tetra_qual: metRidTyp = 1 with a tensor metric needs the point tags (pmx_upload_point_tags)";
    return 0;
  }
  if (!pmx_dgrow(ctx, ctx->d_qual, (size_t)(ctx->ne + 1))) return 0;
  if (A.msize == 6)
    hipLaunchKernelGGL((k_qual<true, false, QM_STORE>), dim3(stat_blocks(ctx->ne)), dim3(256), 0, ctx->stream, A,
                       ctx->d_qual.p, (QualPart *)nullptr);
  else
    hipLaunchKernelGGL((k_qual<false, false, QM_STORE>), dim3(stat_blocks(ctx->ne)), dim3(256), 0, ctx->stream, A,
                       ctx->d_qual.p, (QualPart *)nullptr);
  if (hipGetLastError() != hipSuccess) { ctx->err = "k_qual launch"; return 0; }
  ctx->have_qual = true;
  if (qual) {
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) return 0;
    if (hipMemcpy(qual, ctx->d_qual.p, sizeof(double) * (size_t)(ctx->ne + 1), hipMemcpyDeviceToHost) != hipSuccess) return 0;
    qual[0] = 0.0;
  }
  return 1;
}

int pmx_count_nodes(pmx_ctx *ctx, const int *idx_ip, const int *idx_comm, int64_t nitem_grp,
                    int *intvalues, int64_t nitem, int base, int64_t *np_out) {
  if (!ctx || !np_out) return 0;
  hipSetDevice(ctx->device);
  StatArgs A;
  if (!stat_args(ctx, A)) return 0;
  if (nitem_grp < 0 || nitem < 0 || (nitem_grp > 0 && (!idx_ip || !idx_comm || !intvalues))) {
    ctx->err = "pmx_count_nodes: bad communicator arrays";
    return 0;
  }
  const int64_t np = ctx->np;
  hipStream_t s = ctx->stream;
  // point -> communicator slot (-1: not in the internal communicator)
  std::vector<int> cidx;
  if (nitem_grp > 0) {
    cidx.assign((size_t)(np + 1), -1);
    for (int64_t i = 0; i < nitem_grp; i++) {
      if (idx_ip[i] < 1 || idx_ip[i] > np || idx_comm[i] < 0 || idx_comm[i] >= nitem) {
        ctx->err = "pmx_count_nodes: communicator index out of range";
        return 0;
      }
      cidx[(size_t)idx_ip[i]] = idx_comm[i];
    }
  }
  if (!pmx_dgrow(ctx, ctx->d_touch, (size_t)(np + 1)) || !pmx_dgrow(ctx, ctx->d_cidx, cidx.size() + 1) ||
      !pmx_dgrow(ctx, ctx->d_intv, (size_t)std::max<int64_t>(nitem, 1)) || !ensure_red(ctx, 64))
    return 0;
  unsigned long long *cnt = ctx->d_red.p;
  bool okk = hipMemsetAsync(ctx->d_touch.p, 0, (size_t)(np + 1), s) == hipSuccess &&
             hipMemsetAsync(cnt, 0, 8, s) == hipSuccess;
  if (okk && nitem_grp > 0)
    okk = hipMemcpyAsync(ctx->d_cidx.p, cidx.data(), cidx.size() * 4, hipMemcpyHostToDevice, s) == hipSuccess &&
          hipMemcpyAsync(ctx->d_intv.p, intvalues, (size_t)nitem * 4, hipMemcpyHostToDevice, s) == hipSuccess;
  if (!okk) { ctx->err = "pmx_count_nodes: copy"; return 0; }
  const int64_t nbt = std::min<int64_t>((ctx->ne + 255) / 256, 16384);
  hipLaunchKernelGGL(k_touch, dim3((unsigned)std::max<int64_t>(nbt, 1)), dim3(256), 0, s, A.tetv, ctx->ne,
                     ctx->d_touch.p);
  const int64_t nbp = std::min<int64_t>((np + 255) / 256, 16384);
  hipLaunchKernelGGL(k_count_nodes, dim3((unsigned)std::max<int64_t>(nbp, 1)), dim3(256), 0, s,
                     ctx->d_touch.p, np, nitem_grp > 0 ? ctx->d_cidx.p : nullptr, ctx->d_intv.p, base, cnt);
  unsigned long long c = 0;
  okk = hipMemcpyAsync(&c, cnt, 8, hipMemcpyDeviceToHost, s) == hipSuccess &&
        (nitem_grp == 0 || hipMemcpyAsync(intvalues, ctx->d_intv.p, (size_t)nitem * 4, hipMemcpyDeviceToHost, s) == hipSuccess) &&
        hipStreamSynchronize(s) == hipSuccess;
  if (!okk) { ctx->err = "pmx_count_nodes: launch"; return 0; }
  *np_out = (int64_t)c;
  ctx->stat_np = (int64_t)c;
  return 1;
}

int pmx_qualhisto_device(pmx_ctx *ctx, int opt, int use_stored, void *dev_result) {
  if (!ctx || !dev_result) return 0;
  if (opt == PMX_LESQUA) {
    // MMG3D_computeLESqua (src/quality_pmmg.c:221-224, selected at run time by
    // mesh->info.optimLES): Mmg's LES quality is not restated here
    ctx->err = "pmx_qualhisto: the optimLES quality (MMG3D_computeLESqua) is not supported";
    return 0;
  }
  if (opt != PMX_INQUA && opt != PMX_OUTQUA) {
    ctx->err = "pmx_qualhisto: opt must be PMX_INQUA, PMX_OUTQUA or PMX_LESQUA";
    return 0;
  }
  hipSetDevice(ctx->device);
  StatArgs A;
  if (!stat_args(ctx, A)) return 0;
  if (use_stored && !ctx->have_qual) { ctx->err = "pmx_qualhisto: no stored quality"; return 0; }
  const long long np = ctx->stat_np >= 0 ? ctx->stat_np : ctx->np;
  return qual_partial(ctx, A, opt, ctx->d_qual.p, use_stored, (pmx_qual_part *)dev_result, np);
}

int pmx_qualhisto(pmx_ctx *ctx, int opt, pmx_qual_stats *st) {
  if (!ctx || !st) return 0;
  hipSetDevice(ctx->device);
  if (!pmx_dgrow(ctx, ctx->d_pub, 32)) return 0;
  if (!pmx_qualhisto_device(ctx, opt, 0, ctx->d_pub.p)) return 0;
  pmx_qual_part r;
  if (hipMemcpyAsync(&r, ctx->d_pub.p, sizeof r, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess) {
    ctx->err = "pmx_qualhisto: download";
    return 0;
  }
  qual_to_stats(r, st);
  return 1;
}

int pmx_prilen_device(pmx_ctx *ctx, int metRidTyp, const pmx_par_edges *par, void *dev_result) {
  // metRidTyp (src/quality_pmmg.c:462,527): 0 or 1 give the same lengths for a
  // size-1 metric (MMG5_lenedg = lenedg_iso, MMG5_lenSurfEdg_iso); with a
  // size-6 metric 1 selects Mmg's ridge storage: refused, not approximated
  if (!ctx || !dev_result) return 0;
  if (ctx->have_bg && ctx->sd.imet >= 0 &&
      !check_met_rid_typ(ctx, metRidTyp, ctx->sd.size[ctx->sd.imet], "pmx_prilen", true))
    return 0;
  if (metRidTyp != 0 && metRidTyp != 1) { ctx->err = "pmx_prilen: metRidTyp must be 0 or 1"; return 0; }
  hipSetDevice(ctx->device);
  StatArgs A;
  if (!stat_args(ctx, A)) return 0;
  if (ctx->sd.imet < 0) { ctx->err = "pmx_prilen: no metric"; return 0; }
  if (ctx->ne >= (1LL << 29)) { ctx->err = "pmx_prilen: ne >= 2^29 per group"; return 0; }
  const bool ani = ctx->sd.size[ctx->sd.imet] == 6;
  A.ridmet = metRidTyp == 1 && ani;
  if (A.ridmet && !A.ptag) {
    ctx->err = "pmx_prilen: metRidTyp = 1 with a tensor metric needs the point tags (pmx_upload_point_tags)";
    return 0;
  }
  if (ctx->have_surf) {
    A.etag = ctx->d_etag.p;
    A.pn = ctx->d_pn.p;
    A.pxp = ctx->d_pxp.p;
    A.xpn = ctx->d_xpn.p;
  }
  hipStream_t s = ctx->stream;
  // parallel edges (host): step-1 list (owned, first occurrence, list order)
  // and the sorted keys of the edges step 2 must not count
  std::vector<int2> own;
  std::vector<uint16_t> own_tag;
  std::vector<unsigned long long> excl;
  std::vector<uint8_t> ppt;
  if (par && par->n > 0) {
    if (!par->a || !par->b || !par->owner) { ctx->err = "pmx_prilen: bad parallel edges"; return 0; }
    std::unordered_set<unsigned long long> popped;
    for (int64_t i = 0; i < par->n; i++) {
      const int a = par->a[i], b = par->b[i];
      if (a < 1 || b < 1 || a > ctx->np || b > ctx->np || a == b) {
        ctx->err = "pmx_prilen: parallel edge vertex out of range";
        return 0;
      }
      const unsigned long long key = ((unsigned long long)(unsigned)std::min(a, b) << 32) | (unsigned)std::max(a, b);
      if (par->owner[i] == par->myrank) {
        // MMG5_hashPop succeeds once per edge: a repeated entry is not counted
        if (popped.insert(key).second) {
          own.push_back(make_int2(a, b));
          own_tag.push_back(par->tag ? par->tag[i] : (uint16_t)0);
        }
        excl.push_back(key);
      } else if (par->exact_once) {
        excl.push_back(key);
      }
    }
    std::sort(excl.begin(), excl.end());
    excl.erase(std::unique(excl.begin(), excl.end()), excl.end());
    ppt.assign((size_t)(ctx->np + 1), 0);
    for (unsigned long long key : excl) {
      ppt[(size_t)(key >> 32)] = 1;
      ppt[(size_t)(key & 0xffffffffu)] = 1;
    }
  }
  // the schedule (PMX_PRILEN_SCHED=C: the moving front in chunks of C
  // batches, grid = the co-resident workgroups; unset: contiguous ranges)
  static const int sched = [] {
    const char *e = getenv("PMX_PRILEN_SCHED");
    return e ? std::max(0, atoi(e)) : 0;
  }();
  using KFn = void (*)(StatArgs, LenPart *);
  // variants: metric kind x point tags x parallel edges (each drops the
  // other paths' registers and branches)
  // the isotropic variants held to 5 waves per SIMD (96 VGPRs, a few
  // spills): 2 % faster at the C5 share; the anisotropic ones spill too
  // much there (4.46 instead of 3.63 ms) and keep the compiler's choice
  static const KFn kfn[16] = {
      k_prilen<false, false, false, 5>,        k_prilen<false, false, true, 5>,
      k_prilen<false, true, false, 5>,         k_prilen<false, true, true, 5>,
      k_prilen<true, false, false>,            k_prilen<true, false, true>,
      k_prilen<true, true, false>,             k_prilen<true, true, true>,
      k_prilen<false, false, false, 5, true>,  k_prilen<false, false, true, 5, true>,
      k_prilen<false, true, false, 5, true>,   k_prilen<false, true, true, 5, true>,
      k_prilen<true, false, false, 1, true>,   k_prilen<true, false, true, 1, true>,
      k_prilen<true, true, false, 1, true>,    k_prilen<true, true, true, 1, true>};
  // lean 32-bit index arithmetic while 6 ne + 5 fits 32 bits (PMX_PRILEN_WIDE=1:
  // the 64-bit variant, for the A/B)
  static const bool wide = getenv("PMX_PRILEN_WIDE") != nullptr;
  const bool lean = !wide && A.ne < 700000000LL;
  const int sel = (lean ? 8 : 0) | (ani ? 4 : 0) | (A.ptag ? 2 : 0) |
                  (par && par->n > 0 && !excl.empty() ? 1 : 0);
  // tensor metrics measured along the surface / in ridge storage
  // (len_tet_ani): the owner tet's xTetra tags and vertices per edge
  static const KFn kfs[8] = {
      k_prilen<true, false, false, 1, false, true>, k_prilen<true, false, true, 1, false, true>,
      k_prilen<true, true, false, 1, false, true>,  k_prilen<true, true, true, 1, false, true>,
      k_prilen<true, false, false, 1, true, true>,  k_prilen<true, false, true, 1, true, true>,
      k_prilen<true, true, false, 1, true, true>,   k_prilen<true, true, true, 1, true, true>};
  const bool surf = ani && (ctx->have_surf || A.ridmet);
  KFn kern = surf ? kfs[(lean ? 4 : 0) | (sel & 3)] : kfn[sel];
  // measurement variants of the default iso kernel: PMX_PRILEN_EXP=1..3 with
  // PMX_EXPERIMENTS=1 (results wrong by design: the VALU breakdown), 4 the r05
  // rotation loop, 8 / 16 / 24 the flat rotation's record and order variants,
  // 32 / 33 the default at 6 / 4 waves per SIMD (same results)
  {
    static const int xp = [] {
      const char *e = getenv("PMX_PRILEN_EXP"), *x = getenv("PMX_EXPERIMENTS");
      const int v = e ? atoi(e) : 0;
      if (v == 4 || v == 8 || v == 16 || v == 24 || v == 32 || v == 33 || v == 128) return v;
      return (e && x && x[0] == '1') ? std::max(0, std::min(3, v)) : 0;
    }();
    KFn kv = nullptr;
    switch (xp) {
      case 1: kv = k_prilen<false, false, false, 5, true, false, 1>; break;
      case 2: kv = k_prilen<false, false, false, 5, true, false, 2>; break;
      case 3: kv = k_prilen<false, false, false, 5, true, false, 3>; break;
      case 4: kv = k_prilen<false, false, false, 5, true, false, 4>; break;
      case 8: kv = k_prilen<false, false, false, 5, true, false, 8>; break;
      case 16: kv = k_prilen<false, false, false, 5, true, false, 16>; break;
      case 24: kv = k_prilen<false, false, false, 5, true, false, 24>; break;
      case 32: kv = k_prilen<false, false, false, 6, true, false, 0>; break;    // 6 waves / SIMD
      case 33: kv = k_prilen<false, false, false, 4, true, false, 0>; break;    // 4 waves / SIMD
      case 128: kv = k_prilen<false, false, false, 5, true, false, 128>; break; // two-division length
      default: break;
    }
    if (kv && sel == 8 && !surf) kern = kv;
  }
  int nb = stat_blocks(ctx->ne);
  A.sched_chunk = 0;
  if (sched > 0) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess ||
        per_cu < 1 || cus < 8) {
      ctx->err = "pmx_prilen: occupancy query";
      return 0;
    }
    nb = per_cu * cus / 8 * 8;
    A.sched_chunk = sched;
  }
  // the edge-bucket variant (A/B): no point tags, no surface-aware tensor path
  static const bool buckets = [] {
    const char *e = getenv("PMX_PRILEN_BUCKETS");
    return e && e[0] == '1';
  }();
  const bool use_pb = buckets && !A.ptag && !surf;
  int64_t npb = 0;
  if (use_pb) {
    const int64_t np = ctx->np;
    if (!pmx_dgrow(ctx, ctx->d_pbcnt, (size_t)(np + 2)) || !pmx_dgrow(ctx, ctx->d_pboff, (size_t)(np + 2)))
      return 0;
    size_t tb = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, tb, ctx->d_pbcnt.p, ctx->d_pboff.p, (int)(np + 2), s);
    if (!pmx_dgrow(ctx, ctx->d_pbtmp, tb)) return 0;
    const unsigned nbt = (unsigned)std::max<int64_t>((ctx->ne + 255) / 256, 1);
    if (hipMemsetAsync(ctx->d_pbcnt.p, 0, (size_t)(np + 2) * sizeof(unsigned), s) != hipSuccess) return 0;
    hipLaunchKernelGGL(k_pb_bucket<0>, dim3(nbt), dim3(256), 0, s, (const TetRec *)ctx->d_tets.p, ctx->ne,
                       ctx->d_pbcnt.p, (int4 *)nullptr);
    if (hipcub::DeviceScan::ExclusiveSum(ctx->d_pbtmp.p, tb, ctx->d_pbcnt.p, ctx->d_pboff.p, (int)(np + 2), s) !=
        hipSuccess) {
      ctx->err = "pmx_prilen: bucket scan";
      return 0;
    }
    unsigned tot = 0;
    if (hipMemcpyAsync(&tot, ctx->d_pboff.p + np + 1, sizeof tot, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      ctx->err = "pmx_prilen: bucket total";
      return 0;
    }
    npb = tot;
    if (!pmx_dgrow(ctx, ctx->d_pbrec, (size_t)std::max<int64_t>(npb, 1)) ||
        hipMemcpyAsync(ctx->d_pbcnt.p, ctx->d_pboff.p, (size_t)(np + 2) * sizeof(unsigned), hipMemcpyDeviceToDevice,
                       s) != hipSuccess)
      return 0;
    hipLaunchKernelGGL(k_pb_bucket<1>, dim3(nbt), dim3(256), 0, s, (const TetRec *)ctx->d_tets.p, ctx->ne,
                       ctx->d_pbcnt.p, ctx->d_pbrec.p);
  }
  if (!ensure_red(ctx, sizeof(LenPart) * ((size_t)nb + 1 + FINAL_GRID + 1))) return 0;
  LenPart *parts = (LenPart *)ctx->d_red.p;
  A.npar = (int64_t)excl.size();
  if (A.npar) {
    if (!pmx_dgrow(ctx, ctx->d_pkey, excl.size()) || !pmx_dgrow(ctx, ctx->d_ppt, ppt.size()) ||
        !pmx_dgrow(ctx, ctx->d_pedge, std::max<size_t>(own.size(), 1)) ||
        !pmx_dgrow(ctx, ctx->d_pedge_tag, std::max<size_t>(own.size(), 1)))
      return 0;
    if (hipMemcpyAsync(ctx->d_pkey.p, excl.data(), excl.size() * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(ctx->d_ppt.p, ppt.data(), ppt.size(), hipMemcpyHostToDevice, s) != hipSuccess ||
        (!own.empty() && hipMemcpyAsync(ctx->d_pedge.p, own.data(), own.size() * sizeof(int2), hipMemcpyHostToDevice, s) != hipSuccess) ||
        (!own.empty() && hipMemcpyAsync(ctx->d_pedge_tag.p, own_tag.data(), own_tag.size() * sizeof(uint16_t),
                                        hipMemcpyHostToDevice, s) != hipSuccess)) {
      ctx->err = "pmx_prilen: parallel edge upload";
      return 0;
    }
    A.par_key = ctx->d_pkey.p;
    A.par_pt = ctx->d_ppt.p;
  }
  // partials: [0] step 1 (owned parallel edges), [1..nb] step 2 (tet edges)
  if (!own.empty())
    hipLaunchKernelGGL(k_prilen_par, dim3(1), dim3(256), 0, s, A, ctx->d_pedge.p,
                       (const uint16_t *)ctx->d_pedge_tag.p, (int64_t)own.size(), parts);
  else
    hipLaunchKernelGGL(k_prilen_par, dim3(1), dim3(256), 0, s, A, (const int2 *)nullptr, (const uint16_t *)nullptr,
                       (int64_t)0, parts);
  if (use_pb) {
    using KP = void (*)(StatArgs, const int4 *, int64_t, const unsigned *, LenPart *);
    static const KP kp[2][2] = {{k_pb_edges<false, false>, k_pb_edges<false, true>},
                                {k_pb_edges<true, false>, k_pb_edges<true, true>}};
    hipLaunchKernelGGL(kp[ani ? 1 : 0][A.npar ? 1 : 0], dim3(nb), dim3(256), 0, s, A, (const int4 *)ctx->d_pbrec.p,
                       npb, (const unsigned *)ctx->d_pboff.p, parts + 1);
  } else {
    hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 0, s, A, parts + 1);
  }
  LenPart *mid = parts + 1 + nb;
  hipLaunchKernelGGL(k_prilen_final, dim3(FINAL_GRID), dim3(256), 0, s, parts, nb + 1, mid,
                     (pmx_len_part *)nullptr, ctx->d_tets.p, (const int2 *)ctx->d_pedge.p);
  hipLaunchKernelGGL(k_prilen_final, dim3(1), dim3(256), 0, s, mid, FINAL_GRID, (LenPart *)nullptr,
                     (pmx_len_part *)dev_result, ctx->d_tets.p, (const int2 *)ctx->d_pedge.p);
  if (hipGetLastError() != hipSuccess) { ctx->err = "pmx_prilen: launch failed"; return 0; }
  return 1;
}

int pmx_prilen(pmx_ctx *ctx, int metRidTyp, const pmx_par_edges *par, pmx_len_stats *st) {
  if (!ctx || !st) return 0;
  hipSetDevice(ctx->device);
  if (!pmx_dgrow(ctx, ctx->d_pub, 32)) return 0;
  if (!pmx_prilen_device(ctx, metRidTyp, par, ctx->d_pub.p)) return 0;
  pmx_len_part r;
  if (hipMemcpyAsync(&r, ctx->d_pub.p, sizeof r, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess) {
    ctx->err = "pmx_prilen: download";
    return 0;
  }
  len_to_stats(r, st);
  return 1;
}

// the quality pass over the device-resident new mesh (the step's points and
// the uploaded new tets), in the metric at sol[S * j + moff] (msize 0: none)
static int new_mesh_qual_core(pmx_ctx *ctx, const char *who, int opt, int metRidTyp, double *qual,
                              int64_t qstride, void *dev_result, const double *sol, int S, int msize, int moff) {
  const int64_t ne = ctx->n_ntet;
  const int64_t n = ctx->nq;
  hipStream_t s = ctx->stream;
  if (!pmx_dgrow(ctx, ctx->d_nqual, (size_t)(ne + 1))) return 0;
  StatArgs A{};
  A.xyz = ctx->d_qxyz.p;                  // the new points, dense x y z
  A.xstride = 3;
  A.vbase = 1;
  A.tetv = ctx->d_ntetv.p;
  A.ne = ne;
  A.sol = sol;
  A.S = S;
  A.msize = msize;
  A.moff = moff;
  A.ptag = (opt == PMX_OUTQUA && ctx->have_qtag) ? ctx->d_qtag.p : nullptr;
  if (!check_met_rid_typ(ctx, metRidTyp, A.msize, who, false)) return 0;
  A.ridmet = metRidTyp == 1 && A.msize == 6;
  A.rtag = ctx->have_qtag ? ctx->d_qtag.p : nullptr;
  if (A.ridmet && !A.rtag) {
    // MMG5_moymet leaves the ridge points out: without their tags the mean
    // would silently be the plain one
    ctx->err = std::string(who) + ": metRidTyp = 1 with a tensor metric needs the new points' tags (points view tag)";
    return 0;
  }
  if (dev_result && opt != PMX_INQUA && opt != PMX_OUTQUA) {
    ctx->err = std::string(who) + (opt == PMX_LESQUA ? ": the optimLES quality (MMG3D_computeLESqua) is not supported"
                                                      : ": opt must be PMX_INQUA or PMX_OUTQUA");
    return 0;
  }
  const int nb = stat_blocks(ne);
  if (A.msize == 6)
    hipLaunchKernelGGL((k_qual<true, false, QM_STORE>), dim3(nb), dim3(256), 0, s, A, ctx->d_nqual.p, (QualPart *)nullptr);
  else
    hipLaunchKernelGGL((k_qual<false, false, QM_STORE>), dim3(nb), dim3(256), 0, s, A, ctx->d_nqual.p, (QualPart *)nullptr);
  if (dev_result && !qual_partial(ctx, A, opt, ctx->d_nqual.p, 1, (pmx_qual_part *)dev_result, n)) return 0;
  if (hipGetLastError() != hipSuccess) { ctx->err = std::string(who) + ": launch"; return 0; }
  if (qual && !pmx_download_qual(ctx, ctx->d_nqual.p, ne, qual, qstride)) {
    ctx->err = std::string(who) + ": " + ctx->err;
    return 0;
  }
  return 1;
}

int pmx_new_mesh_qual(pmx_ctx *ctx, const int *tetra_v, int64_t tetra_stride, int64_t ne, int opt,
                      int metRidTyp, double *qual, int64_t qual_cap, void *dev_result) {
  if (!ctx) return 0;
  hipSetDevice(ctx->device);
  if (!ctx->ran || !ctx->have_pts || ctx->out_n != ctx->nq) {
    ctx->err = "pmx_new_mesh_qual: run a step on the new points first";
    return 0;
  }
  // the new tets: given here (uploaded, as pmx_upload_new_tets), or NULL for
  // the ones already uploaded; vertex j+1 = new point j
  if (tetra_v) {
    if (!pmx_upload_new_tets(ctx, tetra_v, tetra_stride, ne)) return 0;
  } else if (!ctx->have_ntet) {
    ctx->err = "pmx_new_mesh_qual: no new tets uploaded";
    return 0;
  } else if (!ctx->ensure_tets(ctx->stream)) {
    return 0;
  }
  if (qual && qual_cap < ctx->n_ntet + 1) {
    ctx->err = "pmx_new_mesh_qual: qual holds " + std::to_string(qual_cap) + " doubles, ne+1 = " +
               std::to_string(ctx->n_ntet + 1) + " needed";
    return 0;
  }
  // the interpolated metric, in the step's output rows (a constant-size
  // metric of the step is there too)
  const int msize = ctx->sd.imet >= 0 ? ctx->sd.size[ctx->sd.imet] : 0;
  const int moff = ctx->sd.imet >= 0 ? ctx->sd.off[ctx->sd.imet] : 0;
  return new_mesh_qual_core(ctx, "pmx_new_mesh_qual", opt, metRidTyp, qual, 8, dev_result, ctx->d_out.p, ctx->sd.S,
                            msize, moff);
}

// PMMG_tetraQual after PMMG_interpMetricsAndFields on the caller's metric
// array: the step's own rows where it wrote the metric, and only the rows it
// did not write (frozen points that PMMG_copyMetricsAndFields_point filled on
// the host, failed tensor inversions) sent to the device; a metric the step
// did not interpolate (-hsiz constant size, or Mmg's own) is sent whole.
int pmx_new_mesh_qual_synced(pmx_ctx *ctx, const pmx_sol_view *met, int opt, int metRidTyp, double *qual,
                             int64_t qual_stride, int64_t qual_cap, void *dev_result) {
  if (!ctx) return 0;
  hipSetDevice(ctx->device);
  const char *who = "pmx_new_mesh_qual_synced";
  const int64_t qs = qual_stride ? qual_stride : (int64_t)sizeof(double);
  if (qs < (int64_t)sizeof(double)) { ctx->err = std::string(who) + ": bad quality stride"; return 0; }
  if (!ctx->ran || !ctx->have_pts || ctx->out_n != ctx->nq) {
    ctx->err = std::string(who) + ": run a step on the new points first";
    return 0;
  }
  if (!ctx->have_ntet) { ctx->err = std::string(who) + ": the step's points view had no new tets"; return 0; }
  if (qual && qual_cap < ctx->n_ntet + 1) {
    ctx->err = std::string(who) + ": qual holds " + std::to_string(qual_cap) + " records, ne+1 = " +
               std::to_string(ctx->n_ntet + 1) + " needed";
    return 0;
  }
  if (!ctx->ensure_tets(ctx->stream) || !ctx->fix_orphans()) return 0;
  const int64_t n = ctx->nq, first = ctx->pts_first;
  hipStream_t s = ctx->stream;
  if (!met || !met->m) return new_mesh_qual_core(ctx, who, opt, metRidTyp, qual, qs, dev_result, nullptr, 0, 0, 0);
  const int sz = met->size;
  if (sz != 1 && sz != 6) { ctx->err = std::string(who) + ": metric size must be 1 or 6"; return 0; }
  const double *hm = met->m + first * sz;      // Mmg layout: entry of point `first`
  const int im = ctx->sd.imet;
  if (im >= 0 && ctx->sd.size[im] == sz) {
    // the step's metric: patch the rows it did not write from the caller's array
    std::vector<uint8_t> wm((size_t)std::max<int64_t>(n, 1));
    if (n && (hipMemcpyAsync(wm.data(), ctx->d_wmask.p, (size_t)n, hipMemcpyDeviceToHost, s) != hipSuccess ||
              hipStreamSynchronize(s) != hipSuccess)) {
      ctx->err = std::string(who) + ": write masks";
      return 0;
    }
    // the unwritten rows, found by the host pool (per-chunk lists joined in order)
    std::vector<int4> ent;
    std::vector<double> val;
    {
      std::mutex mu;
      std::vector<std::pair<int64_t, std::vector<int>>> rows;
      pmx_par_for(0, n, [&](int64_t j0, int64_t j1) {
        std::vector<int> r;
        for (int64_t j = j0; j < j1; j++)
          if (!(wm[(size_t)j] & (1u << im))) r.push_back((int)j);
        std::lock_guard<std::mutex> g(mu);
        rows.emplace_back(j0, std::move(r));
      });
      std::sort(rows.begin(), rows.end(),
                [](const std::pair<int64_t, std::vector<int>> &a, const std::pair<int64_t, std::vector<int>> &b) {
                  return a.first < b.first;
                });
      for (const auto &r : rows)
        for (int j : r.second) {
          ent.push_back(make_int4(j, ctx->sd.off[im], sz, 0));
          for (int c = 0; c < 6; c++) val.push_back(c < sz ? hm[(int64_t)j * sz + c] : 0.0);
        }
    }
    const int64_t ne_ = (int64_t)ent.size();
    if (ne_) {
      if (!pmx_dgrow(ctx, ctx->d_pent, (size_t)ne_) || !pmx_dgrow(ctx, ctx->d_pval, (size_t)ne_ * 6)) return 0;
      if (hipMemcpyAsync(ctx->d_pent.p, ent.data(), (size_t)ne_ * sizeof(int4), hipMemcpyHostToDevice, s) !=
              hipSuccess ||
          hipMemcpyAsync(ctx->d_pval.p, val.data(), (size_t)ne_ * 6 * sizeof(double), hipMemcpyHostToDevice, s) !=
              hipSuccess) {
        ctx->err = std::string(who) + ": patch upload";
        return 0;
      }
      launch_patch_rows(ctx->d_pent.p, ctx->d_pval.p, ne_, ctx->sd.S, ctx->d_out.p, s);
      ctx->eager_nch = 0;                    // the results changed
      // the rows are the caller's now (pmx_download / pmx_promote_background
      // then give the same values)
      const uint8_t bit = (uint8_t)(1u << im);
      for (int64_t e = 0; e < ne_; e++) wm[(size_t)ent[(size_t)e].x] |= bit;
      if (hipMemcpyAsync(ctx->d_wmask.p, wm.data(), (size_t)n, hipMemcpyHostToDevice, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess) {
        ctx->err = std::string(who) + ": write masks";
        return 0;
      }
    }
    return new_mesh_qual_core(ctx, who, opt, metRidTyp, qual, qs, dev_result, ctx->d_out.p, ctx->sd.S, sz,
                              ctx->sd.off[im]);
  }
  // no metric in the step: the caller's whole array
  if (!pmx_dgrow(ctx, ctx->d_cmet, (size_t)std::max<int64_t>(n * sz, 1))) return 0;
  if (n && (hipMemcpyAsync(ctx->d_cmet.p, hm, (size_t)(n * sz) * sizeof(double), hipMemcpyHostToDevice, s) !=
                hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)) {
    ctx->err = std::string(who) + ": metric upload";
    return 0;
  }
  return new_mesh_qual_core(ctx, who, opt, metRidTyp, qual, qs, dev_result, ctx->d_cmet.p, sz, sz, 0);
}

// ---- the reduction across ranks (host folds + RCCL) --------------------------------

int pmx_qual_fold(const pmx_qual_part *parts, const int *rank, int n, pmx_qual_stats *out) {
  if (!parts || !out || n < 1) return 0;
  // per rank: the groups in order (PMMG_qualhisto's loop, :216-261: sums,
  // strict max, strict min -> first group on ties); then the ranks in order
  // with the reduce operators (:275-306, custom op :82-98: strict min ->
  // lowest rank on ties)
  memset(out, 0, sizeof *out);
  bool first_rank = true;
  int i = 0;
  while (i < n) {
    const int r = rank ? rank[i] : i;
    pmx_qual_stats g;
    memset(&g, 0, sizeof g);
    g.max = 0.0;          // reference max = DBL_MIN; every partial's max is >= 0
    g.min = 1.e300;       // DBL_MAX
    int grp = 0;
    const int i0 = i;
    while (i < n && (rank ? rank[i] : i) == r) i++;
    const bool single = i - i0 == 1;          // an already merged rank partial
    for (int j = i0; j < i; j++, grp++) {
      const pmx_qual_part &p = parts[j];
      g.np += p.np; g.ne += p.ne; g.avg += p.avg; g.med += p.med; g.good += p.good; g.nrid += p.nrid;
      if (p.max > g.max) g.max = p.max;
      if (p.ne && p.min < g.min) { g.min = p.min; g.iel = p.iel; g.iel_grp = single ? (int)p.iel_grp : grp; }
      for (int h = 0; h < 5; h++) g.his[h] += p.his[h];
    }
    g.cpu = r;
    if (first_rank) {
      *out = g;
      first_rank = false;
      continue;
    }
    out->np += g.np; out->ne += g.ne; out->avg += g.avg; out->med += g.med; out->good += g.good;
    out->nrid += g.nrid;
    if (g.max > out->max) out->max = g.max;
    if (g.min < out->min) { out->min = g.min; out->iel = g.iel; out->iel_grp = g.iel_grp; out->cpu = g.cpu; }
    for (int h = 0; h < 5; h++) out->his[h] += g.his[h];
  }
  return 1;
}

int pmx_len_fold(const pmx_len_part *parts, int n, pmx_len_stats *out) {
  if (!parts || !out || n < 1) return 0;
  // PMMG_compute_lenStats (:106-144) applied in rank order: sums; a strictly
  // smaller lmin takes lmin, amin/bmin AND amax/bmax (the reference's quirk)
  // and cpu_min; a strictly larger lmax takes lmax, amax/bmax and cpu_max
  len_to_stats(parts[0], out);
  out->cpu_min = out->cpu_max = 0;
  for (int r = 1; r < n; r++) {
    const pmx_len_part &in = parts[r];
    out->avlen += in.avlen;
    out->ned += in.ned;
    out->nullEdge += in.nullEdge;
    for (int j = 0; j < 9; j++) out->hl[j] += in.hl[j];
    if (in.lmin < out->lmin) {
      out->lmin = in.lmin; out->amin = in.amin; out->bmin = in.bmin;
      out->amax = in.amax; out->bmax = in.bmax; out->cpu_min = r;
    }
    if (in.lmax > out->lmax) {
      out->lmax = in.lmax; out->amax = in.amax; out->bmax = in.bmax; out->cpu_max = r;
    }
  }
  return 1;
}

int pmx_comm_unique_id(char *id, int len) {
  if (!id || len < (int)sizeof(ncclUniqueId)) return 0;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return 0;
  memcpy(id, &u, sizeof u);
  return (int)sizeof u;
}

int pmx_comm_init(pmx_ctx *ctx, void **comm, int nranks, const char *id, int rank) {
  if (!ctx || !comm || !id || nranks < 1 || rank < 0 || rank >= nranks) return 0;
  hipSetDevice(ctx->device);
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  ncclComm_t c;
  const ncclResult_t r = ncclCommInitRank(&c, nranks, u, rank);
  if (r != ncclSuccess) { ctx->err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r); return 0; }
  *comm = (void *)c;
  return 1;
}

int pmx_comm_destroy(void *comm) {
  if (!comm) return 0;
  return ncclCommDestroy((ncclComm_t)comm) == ncclSuccess ? 1 : 0;
}

// one all-gather of each rank's partial (records of `bytes`), on the context stream
static bool gather_parts(pmx_ctx *ctx, void *comm, int nranks, const void *dev_part, size_t bytes,
                         std::vector<char> &host) {
  hipStream_t s = ctx->stream;
  if (!pmx_dgrow(ctx, ctx->d_gather, (size_t)nranks * bytes / 8 + 1)) return false;
  const ncclResult_t r = ncclAllGather(dev_part, ctx->d_gather.p, bytes / 8, ncclInt64, (ncclComm_t)comm, s);
  if (r != ncclSuccess) { ctx->err = std::string("ncclAllGather: ") + ncclGetErrorString(r); return false; }
  host.resize((size_t)nranks * bytes);
  if (hipMemcpyAsync(host.data(), ctx->d_gather.p, host.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    ctx->err = "stats all-gather: download";
    return false;
  }
  return true;
}

int pmx_qualhisto_allreduce(pmx_ctx *ctx, void *comm, int nranks, const void *dev_parts, int ngrp,
                            pmx_qual_stats *out) {
  if (!ctx || !comm || !dev_parts || !out || nranks < 1 || ngrp < 1) return 0;
  hipSetDevice(ctx->device);
  hipStream_t s = ctx->stream;
  // the rank's groups merged first (PMMG_qualhisto's group loop), then one
  // record per rank all-gathered
  std::vector<pmx_qual_part> g((size_t)ngrp);
  if (hipMemcpyAsync(g.data(), dev_parts, g.size() * sizeof(pmx_qual_part), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    ctx->err = "pmx_qualhisto_allreduce: download";
    return 0;
  }
  pmx_qual_stats m;
  std::vector<int> zero((size_t)ngrp, 0);
  pmx_qual_fold(g.data(), zero.data(), ngrp, &m);
  pmx_qual_part mine;
  mine.avg = m.avg; mine.max = m.max; mine.min = m.min; mine.iel = m.iel; mine.ne = m.ne; mine.np = m.np;
  mine.good = m.good; mine.med = m.med; mine.nrid = m.nrid;
  for (int h = 0; h < 5; h++) mine.his[h] = m.his[h];
  mine.iel_grp = m.iel_grp;
  if (!pmx_dgrow(ctx, ctx->d_pub, 32) ||
      hipMemcpyAsync(ctx->d_pub.p, &mine, sizeof mine, hipMemcpyHostToDevice, s) != hipSuccess) {
    ctx->err = "pmx_qualhisto_allreduce: upload";
    return 0;
  }
  std::vector<char> h;
  if (!gather_parts(ctx, comm, nranks, ctx->d_pub.p, sizeof(pmx_qual_part), h)) return 0;
  return pmx_qual_fold((const pmx_qual_part *)h.data(), nullptr, nranks, out);
}

int pmx_prilen_allreduce(pmx_ctx *ctx, void *comm, int nranks, const void *dev_part, pmx_len_stats *out) {
  if (!ctx || !comm || !dev_part || !out || nranks < 1) return 0;
  hipSetDevice(ctx->device);
  std::vector<char> h;
  if (!gather_parts(ctx, comm, nranks, dev_part, sizeof(pmx_len_part), h)) return 0;
  return pmx_len_fold((const pmx_len_part *)h.data(), nranks, out);
}

}  // extern "C"
