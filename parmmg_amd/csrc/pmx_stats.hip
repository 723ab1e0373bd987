// pmx_stats.hip -- quality and edge-length statistics on gfx950.
//
// pmx_tetra_qual  <- PMMG_tetraQual -> MMG3D_tetraQual (reference
//                    src/quality_pmmg.c:720-733; per-tet kernels restated from
//                    Mmg MMG5_caltet_iso / MMG5_caltet33_ani, unpinned)
// pmx_qualhisto   <- PMMG_qualhisto per-group part (src/quality_pmmg.c:156-261)
//                    with MMG3D_computeInqua's histogram (5 bins)
// pmx_prilen      <- PMMG_prilen / MMG3D_computePrilen (src/quality_pmmg.c:370-709)
//
// Both histograms are one pass over the mesh: per-thread accumulation, a
// wavefront/LDS tree per workgroup, one partial record per workgroup, and a
// two-level final reduction in workgroup order (deterministic sums).
// Unique edges are enumerated without a hash table: tet k owns its local edge
// ia iff k is the smallest admissible tet index in the edge shell, found by
// rotating around the edge through the adjacency (early exit on the first
// smaller index) -- this is the first occurrence in the reference's
// (k ascending, ia ascending) hash-pop order, so endpoints and orientation of
// every length match the reference.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdlib>
#include <vector>
#include "pmx_internal.h"

#define ALPHAD 20.7846097          // MMG3D_ALPHAD (12*sqrt(3))
#define TAG_GEO 2
#define TAG_REQ 4
#define TAG_NOM 8
#define TAG_CRN 32

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

// MMG5_caltet33_ani (restated): quality in the mean vertex metric
__device__ double caltet_ani(D3 a, D3 b, D3 c, D3 d, const double *ma, const double *mb,
                             const double *mc, const double *md) {
  double mm[6];
  for (int i = 0; i < 6; i++) mm[i] = 0.25 * (ma[i] + mb[i] + mc[i] + md[i]);
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

struct QualPart {
  double avg, max, min;
  long long iel, ne, good, med, his[5];
};

__device__ __forceinline__ D3 sld3(const StatArgs &A, int i) { return ld3(A.xyz, i); }

template <bool ANI>
__device__ double tet_quality(const StatArgs &A, int64_t k, const TetRec &t) {
  D3 a = sld3(A, t.v[0]), b = sld3(A, t.v[1]), c = sld3(A, t.v[2]), d = sld3(A, t.v[3]);
  if (ANI) {
    const double *m = A.sol;
    return caltet_ani(a, b, c, d, m + (int64_t)t.v[0] * A.S + A.moff, m + (int64_t)t.v[1] * A.S + A.moff,
                      m + (int64_t)t.v[2] * A.S + A.moff, m + (int64_t)t.v[3] * A.S + A.moff);
  }
  return caltet_iso(a, b, c, d);
}

// quality of every tet (+ optional histogram partials in the same pass)
// ANI: the metric is a 6-component tensor (compiled apart: the iso variant
// does not carry the tensor path's registers)
template <bool ANI>
__global__ __launch_bounds__(256) void k_qual(StatArgs A, double *qual, QualPart *parts,
                                              int use_stored) {
  __shared__ QualPart sh[256];
  // thread-local accumulators with 32-bit counts (a thread sees < 2^32 tets):
  // half the registers of QualPart's 64-bit fields
  double avg = 0.0, qmax = 0.0, qmin = 2.0;
  long long iel = 0x7fffffffffffffffLL;
  unsigned cne = 0, cgood = 0, cmed = 0, chis[5] = {0, 0, 0, 0, 0};
  const int64_t per = (A.ne + gridDim.x - 1) / gridDim.x;       // contiguous chunk per block
  const int64_t k0 = 1 + (int64_t)blockIdx.x * per, k1 = min(A.ne, k0 + per - 1);
  for (int64_t k = k0 + threadIdx.x; k <= k1; k += blockDim.x) {
    // 16-B connectivity stream: the neighbours are not needed here
    const int4 cv = A.tetv[k];
    TetRec t;
    t.v[0] = cv.x; t.v[1] = cv.y; t.v[2] = cv.z; t.v[3] = cv.w;
    if (t.v[0] <= 0) continue;
    double q = use_stored ? qual[k] : tet_quality<ANI>(A, k, t);
    if (!use_stored && qual) qual[k] = q;
    if (!parts) continue;
    double rap = ALPHAD * q;
    cne++;
    if (rap < qmin || (rap == qmin && k < iel)) { qmin = rap; iel = k; }
    if (rap > 0.5) cmed++;
    if (rap > 0.12) cgood++;
    avg += rap;
    qmax = fmax(qmax, rap);
    int ir = (int)(5.0 * rap);
    ir = ir < 4 ? ir : 4;
    // predicated, static indices: the histogram stays in VGPRs (no scratch)
#pragma unroll
    for (int i = 0; i < 5; i++) chis[i] += (i == ir) ? 1u : 0u;
  }
  if (!parts) return;
  QualPart p;
  p.avg = avg; p.max = qmax; p.min = qmin; p.iel = iel;
  p.ne = cne; p.good = cgood; p.med = cmed;
#pragma unroll
  for (int i = 0; i < 5; i++) p.his[i] = chis[i];
  sh[threadIdx.x] = p;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      QualPart &x = sh[threadIdx.x];
      const QualPart &y = sh[threadIdx.x + o];
      x.avg += y.avg;
      x.max = fmax(x.max, y.max);
      if (y.min < x.min || (y.min == x.min && y.iel < x.iel)) { x.min = y.min; x.iel = y.iel; }
      x.ne += y.ne; x.good += y.good; x.med += y.med;
      for (int i = 0; i < 5; i++) x.his[i] += y.his[i];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) parts[blockIdx.x] = sh[0];
}

__global__ __launch_bounds__(256) void k_qual_final(const QualPart *parts, int n, QualPart *res) {
  __shared__ QualPart sh[256];
  QualPart p;
  p.avg = 0.0; p.max = 0.0; p.min = 2.0; p.iel = 0x7fffffffffffffffLL; p.ne = 0; p.good = 0; p.med = 0;
  for (int i = 0; i < 5; i++) p.his[i] = 0;
  // this block's contiguous range, contiguous sub-ranges per thread: the
  // summation order is fixed (launched twice: FINAL_GRID blocks, then one)
  const int pb = (n + gridDim.x - 1) / gridDim.x;
  const int lo = blockIdx.x * pb, hi = min(n, lo + pb);
  int per = (hi - lo + 255) / 256;
  for (int b = lo + threadIdx.x * per; b < min(hi, lo + (int)(threadIdx.x + 1) * per); b++) {
    const QualPart &y = parts[b];
    p.avg += y.avg;
    p.max = fmax(p.max, y.max);
    if (y.min < p.min || (y.min == p.min && y.iel < p.iel)) { p.min = y.min; p.iel = y.iel; }
    p.ne += y.ne; p.good += y.good; p.med += y.med;
    for (int i = 0; i < 5; i++) p.his[i] += y.his[i];
  }
  sh[threadIdx.x] = p;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      QualPart &x = sh[threadIdx.x];
      const QualPart &y = sh[threadIdx.x + o];
      x.avg += y.avg;
      x.max = fmax(x.max, y.max);
      if (y.min < x.min || (y.min == x.min && y.iel < x.iel)) { x.min = y.min; x.iel = y.iel; }
      x.ne += y.ne; x.good += y.good; x.med += y.med;
      for (int i = 0; i < 5; i++) x.his[i] += y.his[i];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) res[blockIdx.x] = sh[0];
}

// ---- edge lengths ---------------------------------------------------------------

struct LenPart {
  double avlen, lmin, lmax;
  long long kmin, kmax;          // first-occurrence key 6*k+ia of the extremal edges
  long long ned, nul, hl[9];
};

// a tet is skipped when all 4 vertices are non-singular ridge points
// (reference src/quality_pmmg.c:509-517)
__device__ __forceinline__ bool tet_admissible(const StatArgs &A, const TetRec &t) {
  if (!A.ptag) return true;
  int n = 0;
  for (int i = 0; i < 4; i++) {
    unsigned tg = A.ptag[t.v[i]];
    bool sin = (tg & TAG_CRN) || (tg & TAG_REQ);
    if (!(sin || (TAG_NOM & tg)) && (tg & TAG_GEO)) continue;
    n++;
  }
  return n > 0;
}

__device__ __forceinline__ int pick_v(const TetRec &t, int l) {
  return (t.v[0] & -(int)(l == 0)) | (t.v[1] & -(int)(l == 1)) | (t.v[2] & -(int)(l == 2)) |
         (t.v[3] & -(int)(l == 3));
}
__device__ __forceinline__ int pick_nb(const TetRec &t, int l) {
  return (t.nb[0] & -(int)(l == 0)) | (t.nb[1] & -(int)(l == 1)) | (t.nb[2] & -(int)(l == 2)) |
         (t.nb[3] & -(int)(l == 3));
}

__device__ __forceinline__ int loc_of(const TetRec &t, int p) {
  int l = 3;
  if (t.v[0] == p) l = 0;
  else if (t.v[1] == p) l = 1;
  else if (t.v[2] == p) l = 2;
  return l;
}

// MMG5_lenEdg_iso / lenEdg_ani (restated, unpinned)
__device__ double edge_len(const StatArgs &A, int p1, int p2) {
  D3 c1 = sld3(A, p1), c2 = sld3(A, p2);
  double ux = c2.x - c1.x, uy = c2.y - c1.y, uz = c2.z - c1.z;
  if (A.msize == 6) {
    const double *m1 = A.sol + (int64_t)p1 * A.S + A.moff, *m2 = A.sol + (int64_t)p2 * A.S + A.moff;
    double dd1 = mlen2(m1, ux, uy, uz);
    double dd2 = mlen2(m2, ux, uy, uz);
    if (dd1 <= 0.0) dd1 = 0.0;
    if (dd2 <= 0.0) dd2 = 0.0;
    return (sqrt(dd1) + sqrt(dd2) + 4.0 * sqrt(0.5 * (dd1 + dd2))) / 6.0;
  }
  double h1 = A.sol[(int64_t)p1 * A.S + A.moff], h2 = A.sol[(int64_t)p2 * A.S + A.moff];
  double l = ux * ux + uy * uy + uz * uz;
  l = sqrt(l);
  double r = h2 / h1 - 1.0;
  return (fabs(r) < PMX_EPS) ? (l / h1) : (l / (h2 - h1) * log1p(r));
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

// ---- prilen: unique edges by shell ownership, compacted ------------------------
//
// Tet k owns its local edge ia iff no admissible tet of smaller index shares
// it (the first occurrence in the reference's (k, ia) hash-pop order).  A
// per-thread loop over tets rotating each shell in turn left ~1 lane in 6
// with a shell to rotate on a lattice-ordered mesh (r01: 40 ms at 125M tets),
// so the shells to rotate are compacted first:
//  1. k_len_mark: per tet, edges decided without a load -- disowned by a
//     smaller face neighbour (no point tags), or owned because both faces
//     around the edge are boundary faces (shell = {k}, measured right away) --
//     and a 6-bit mask of the edges whose shell must be rotated;
//  2. k_len_scan + k_len_compact: those (tet, edge) pairs, in (k, ia) order,
//     into a list (deterministic positions: block counts + exclusive scan);
//  3. k_len_rotate: one list entry per thread, every lane rotating a shell.
// Sums are reduced in a fixed order (phase-1 partials, then phase-3 partials,
// two-level final reduction): the result does not depend on the schedule.

__device__ __forceinline__ void edge_others(int ia, int &o0, int &o1) {
  const int i0 = IARE[ia][0], i1 = IARE[ia][1];
  o0 = (i0 != 0 && i1 != 0) ? 0 : (i0 != 1 && i1 != 1) ? 1 : 2;
  o1 = 6 - i0 - i1 - o0;
}

struct LenAcc {
  double avlen = 0.0, lmin = 1.e30, lmax = 0.0;
  long long kmin = 0x7fffffffffffffffLL, kmax = 0x7fffffffffffffffLL;
  unsigned ned = 0, nul = 0, hl[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  __device__ void add(const StatArgs &A, const TetRec &t, int64_t k, int ia) {
    const int np_ = pick_v(t, IARE[ia][0]), nq_ = pick_v(t, IARE[ia][1]);
    const double len = edge_len(A, np_, nq_);
    if (!(len != 0.0)) { if (len == 0.0) { nul++; return; } }
    const long long key = 6 * k + ia;
    avlen += len;
    ned++;
    if (len < lmin || (len == lmin && key < kmin)) { lmin = len; kmin = key; }
    if (len > lmax || (len == lmax && key < kmax)) { lmax = len; kmax = key; }
    int bin = 8;
#pragma unroll
    for (int i = 7; i >= 0; i--) bin = (BD[i] <= len && len < BD[i + 1]) ? i : bin;
#pragma unroll
    for (int i = 0; i < 9; i++) hl[i] += (i == bin) ? 1u : 0u;
  }
  __device__ void store(LenPart *sh, LenPart *out) const {
    LenPart p;
    p.avlen = avlen; p.lmin = lmin; p.lmax = lmax; p.kmin = kmin; p.kmax = kmax;
    p.ned = ned; p.nul = nul;
#pragma unroll
    for (int i = 0; i < 9; i++) p.hl[i] = hl[i];
    sh[threadIdx.x] = p;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if ((int)threadIdx.x < o) len_merge(sh[threadIdx.x], sh[threadIdx.x + o]);
      __syncthreads();
    }
    if (threadIdx.x == 0) *out = sh[0];
  }
};

__device__ __forceinline__ unsigned block_sum(unsigned v, unsigned *sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  return sh[0] + sh[1] + sh[2] + sh[3];
}

__global__ __launch_bounds__(256) void k_len_mark(StatArgs A, LenPart *parts, uint8_t *emask,
                                                  unsigned *bcount) {
  __shared__ LenPart sh[256];
  __shared__ unsigned shc[4];
  LenAcc acc;
  unsigned cnt = 0;
  const int64_t per = (A.ne + gridDim.x - 1) / gridDim.x;
  const int64_t k0 = 1 + (int64_t)blockIdx.x * per, k1 = min(A.ne, k0 + per - 1);
  for (int64_t k = k0 + threadIdx.x; k <= k1; k += blockDim.x) {
    const TetRec t = A.tets[k];
    unsigned m = 0;
    if (t.v[0] > 0 && tet_admissible(A, t)) {
      for (int ia = 0; ia < 6; ia++) {
        int o0, o1;
        edge_others(ia, o0, o1);
        const int n0 = pick_nb(t, o0), n1 = pick_nb(t, o1);
        if (!A.ptag && ((n0 && n0 < k) || (n1 && n1 < k))) continue;   // disowned
        if (!n0 && !n1) { acc.add(A, t, k, ia); continue; }             // shell = {k}
        m |= 1u << ia;
      }
    }
    emask[k] = (uint8_t)m;
    cnt += __popc(m);
  }
  const unsigned tot = block_sum(cnt, shc);
  if (threadIdx.x == 0) bcount[blockIdx.x] = tot;
  acc.store(sh, parts + blockIdx.x);
}

// exclusive scan of the per-block counts (one workgroup; n <= 16384)
__global__ __launch_bounds__(256) void k_len_scan(unsigned *bcount, int n, unsigned *total) {
  __shared__ unsigned sh[256];
  const int per = (n + 255) / 256;
  const int b0 = threadIdx.x * per, b1 = min(n, b0 + per);
  unsigned s = 0;
  for (int b = b0; b < b1; b++) s += bcount[b];
  sh[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned run = 0;
    for (int i = 0; i < 256; i++) { unsigned v = sh[i]; sh[i] = run; run += v; }
    *total = run;
  }
  __syncthreads();
  unsigned run = sh[threadIdx.x];
  for (int b = b0; b < b1; b++) { unsigned v = bcount[b]; bcount[b] = run; run += v; }
}

__global__ __launch_bounds__(256) void k_len_compact(const uint8_t *emask, int64_t ne,
                                                     const unsigned *boff, uint32_t *list) {
  __shared__ unsigned sh[256];
  const int64_t per = (ne + gridDim.x - 1) / gridDim.x;
  const int64_t k0 = 1 + (int64_t)blockIdx.x * per, k1 = min(ne, k0 + per - 1);
  unsigned base = boff[blockIdx.x];
  for (int64_t kb = k0; kb <= k1; kb += blockDim.x) {
    const int64_t k = kb + threadIdx.x;
    const unsigned m = (k <= k1) ? emask[k] : 0u;
    const unsigned c = __popc(m);
    // block-wide exclusive scan of c (Hillis-Steele in LDS)
    sh[threadIdx.x] = c;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
      const unsigned v = (int)threadIdx.x >= o ? sh[threadIdx.x - o] : 0u;
      __syncthreads();
      sh[threadIdx.x] += v;
      __syncthreads();
    }
    unsigned pos = base + sh[threadIdx.x] - c;
    const unsigned stot = sh[255];
    for (int ia = 0; ia < 6; ia++)
      if ((m >> ia) & 1u) list[pos++] = (uint32_t)(k * 8 + ia);
    base += stot;
    __syncthreads();
  }
}

// True iff no admissible tet with index < k contains edge ia of tet k.  The
// shell is rotated from k through the two faces of k that contain the edge,
// both directions advanced together (two independent loads in flight): a
// smaller index is met after min(d0, d1) steps, and a closed shell is covered
// when the two cursors meet, in half the dependent steps.
__device__ bool owns_edge_bidir(const StatArgs &A, int64_t k, const TetRec &t0, int ia) {
  const int i0 = IARE[ia][0], i1 = IARE[ia][1];
  const int a = pick_v(t0, i0), b = pick_v(t0, i1);
  int o0, o1;
  edge_others(ia, o0, o1);
  int c0 = pick_nb(t0, o0), c1 = pick_nb(t0, o1);
  int keep0 = pick_v(t0, o1), keep1 = pick_v(t0, o0);
  for (int guard = 0; guard < 4096; guard++) {
    if (c0 == (int)k) c0 = 0;                    // a direction that wrapped around
    if (c1 == (int)k) c1 = 0;
    if (!c0 && !c1) return true;                 // both ends reached: every tet seen
    if (!A.ptag && ((c0 && c0 < k) || (c1 && c1 < k))) return false;
    if (c0 && c0 == c1) {                        // the cursors meet on one tet
      const TetRec t = A.tets[c0];
      return !(c0 < k && tet_admissible(A, t));
    }
    TetRec t0r, t1r;
    if (c0) t0r = A.tets[c0];
    if (c1) t1r = A.tets[c1];
    int n0 = 0, n1 = 0;
    if (c0) {
      if (c0 < k && tet_admissible(A, t0r)) return false;
      n0 = pick_nb(t0r, loc_of(t0r, keep0));
      int nk = 0;
#pragma unroll
      for (int l = 0; l < 4; l++) {
        const int v = t0r.v[l];
        nk = (v != a && v != b && v != keep0) ? v : nk;
      }
      keep0 = nk;
    }
    if (c1) {
      if (c1 < k && tet_admissible(A, t1r)) return false;
      n1 = pick_nb(t1r, loc_of(t1r, keep1));
      int nk = 0;
#pragma unroll
      for (int l = 0; l < 4; l++) {
        const int v = t1r.v[l];
        nk = (v != a && v != b && v != keep1) ? v : nk;
      }
      keep1 = nk;
    }
    // closed shell: the next tet of one direction is the one the other just saw
    if (c0 && c1 && (n0 == c1 || n1 == c0)) return true;
    c0 = c0 ? n0 : 0;
    c1 = c1 ? n1 : 0;
  }
  return true;
}

__global__ __launch_bounds__(256) void k_len_rotate(StatArgs A, const uint32_t *list,
                                                    const unsigned *total, LenPart *parts) {
  __shared__ LenPart sh[256];
  LenAcc acc;
  const int64_t n = *total;
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t e0 = (int64_t)blockIdx.x * per, e1 = min(n, e0 + per);
  for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
    const uint32_t it = list[e];
    const int64_t k = it >> 3;
    const int ia = (int)(it & 7u);
    const TetRec t = A.tets[k];
    if (owns_edge_bidir(A, k, t, ia)) acc.add(A, t, k, ia);
  }
  acc.store(sh, parts + blockIdx.x);
}

__global__ __launch_bounds__(256) void k_prilen_final(const LenPart *parts, int n, LenPart *res) {
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
  if (threadIdx.x == 0) res[blockIdx.x] = sh[0];
}

// ---- C ABI ----------------------------------------------------------------------

// partial records per pass: a function of ne only (the fixed-order final
// reduction then gives the same sums on every run); enough workgroups to fill
// 256 CUs several times over, each a contiguous range of >= 2048 tets
#define FINAL_GRID 64
static int stat_blocks(int64_t ne) {
  return (int)std::max<int64_t>(256, std::min<int64_t>(16384, ne / 2048));
}

static bool stat_args(pmx_ctx *ctx, StatArgs &A) {
  if (!ctx->have_bg) { ctx->err = "statistics: upload a group first"; return false; }
  // the 16-B connectivity stream of the quality pass, derived from the tet
  // records on the first statistics call after an upload (the transfer step
  // itself does not need it)
  if (!ctx->have_tetv) {
    if (ctx->d_tetv.cap < (size_t)(ctx->ne + 1)) {
      if (ctx->d_tetv.p) hipFree(ctx->d_tetv.p);
      ctx->d_tetv.p = nullptr;
      ctx->d_tetv.cap = 0;
      if (hipMalloc((void **)&ctx->d_tetv.p, sizeof(int4) * (size_t)(ctx->ne + 1)) != hipSuccess) {
        ctx->err = "statistics: hipMalloc tetv";
        return false;
      }
      ctx->d_tetv.cap = (size_t)(ctx->ne + 1);
    }
    launch_tet_conn(ctx->d_tets.p, ctx->ne + 1, ctx->d_tetv.p, ctx->stream);
    ctx->have_tetv = true;
  }
  A.xyz = ctx->d_xyz.p;
  A.tets = ctx->d_tets.p;
  A.tetv = ctx->d_tetv.p;
  A.ne = ctx->ne;
  A.sol = ctx->d_sol.p;
  A.S = ctx->sd.S;
  A.msize = ctx->sd.imet >= 0 ? ctx->sd.size[ctx->sd.imet] : 0;
  A.moff = ctx->sd.imet >= 0 ? ctx->sd.off[ctx->sd.imet] : 0;
  A.ptag = nullptr;
  return true;
}

template <class T> static bool dgrow_t(pmx_ctx *ctx, DevBuf<T> &b, size_t n) {
  if (b.p && b.cap >= n) return true;
  if (b.p) hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  if (hipMalloc((void **)&b.p, n * sizeof(T)) != hipSuccess) { ctx->err = "hipMalloc prilen"; return false; }
  b.cap = n;
  return true;
}
static bool dgrow_u8(pmx_ctx *ctx, DevBuf<uint8_t> &b, size_t n) { return dgrow_t(ctx, b, n); }
static bool dgrow_u32(pmx_ctx *ctx, DevBuf<uint32_t> &b, size_t n) { return dgrow_t(ctx, b, n); }
static bool dgrow_u32(pmx_ctx *ctx, DevBuf<unsigned> &b, size_t n, int) { return dgrow_t(ctx, b, n); }

static bool ensure_red(pmx_ctx *ctx, size_t bytes) {
  size_t n = (bytes + 7) / 8;
  if (ctx->d_red.cap >= n && ctx->d_red.p) return true;
  if (ctx->d_red.p) hipFree(ctx->d_red.p);
  ctx->d_red.p = nullptr;
  if (hipMalloc((void **)&ctx->d_red.p, n * 8) != hipSuccess) { ctx->err = "hipMalloc stats"; return false; }
  ctx->d_red.cap = n;
  return true;
}

extern "C" {

int pmx_tetra_qual(pmx_ctx *ctx, double *qual) {
  if (!ctx) return 0;
  hipSetDevice(ctx->device);
  StatArgs A{};
  if (!stat_args(ctx, A)) return 0;
  if (ctx->d_qual.cap < (size_t)(ctx->ne + 1)) {
    if (ctx->d_qual.p) hipFree(ctx->d_qual.p);
    if (hipMalloc((void **)&ctx->d_qual.p, sizeof(double) * (size_t)(ctx->ne + 1)) != hipSuccess) {
      ctx->err = "hipMalloc qual";
      return 0;
    }
    ctx->d_qual.cap = (size_t)(ctx->ne + 1);
  }
  if (A.msize == 6)
    hipLaunchKernelGGL(k_qual<true>, dim3(stat_blocks(ctx->ne)), dim3(256), 0, ctx->stream, A,
                       ctx->d_qual.p, (QualPart *)nullptr, 0);
  else
    hipLaunchKernelGGL(k_qual<false>, dim3(stat_blocks(ctx->ne)), dim3(256), 0, ctx->stream, A,
                       ctx->d_qual.p, (QualPart *)nullptr, 0);
  if (hipGetLastError() != hipSuccess) { ctx->err = "k_qual launch"; return 0; }
  ctx->have_qual = true;
  if (qual) {
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) return 0;
    if (hipMemcpy(qual, ctx->d_qual.p, sizeof(double) * (size_t)(ctx->ne + 1), hipMemcpyDeviceToHost) != hipSuccess) return 0;
    qual[0] = 0.0;
  }
  return 1;
}

int pmx_qualhisto_device(pmx_ctx *ctx, int use_stored, void *dev_result) {
  StatArgs A{};
  if (!stat_args(ctx, A)) return 0;
  if (use_stored && !ctx->have_qual) { ctx->err = "pmx_qualhisto: no stored quality"; return 0; }
  if (!ensure_red(ctx, sizeof(QualPart) * (stat_blocks(ctx->ne) + FINAL_GRID + 1))) return 0;
  QualPart *parts = (QualPart *)ctx->d_red.p;
  if (A.msize == 6)
    hipLaunchKernelGGL(k_qual<true>, dim3(stat_blocks(ctx->ne)), dim3(256), 0, ctx->stream, A,
                       use_stored ? ctx->d_qual.p : (double *)nullptr, parts, use_stored);
  else
    hipLaunchKernelGGL(k_qual<false>, dim3(stat_blocks(ctx->ne)), dim3(256), 0, ctx->stream, A,
                       use_stored ? ctx->d_qual.p : (double *)nullptr, parts, use_stored);
  QualPart *mid = parts + stat_blocks(ctx->ne);
  QualPart *res = dev_result ? (QualPart *)dev_result : mid + FINAL_GRID;
  hipLaunchKernelGGL(k_qual_final, dim3(FINAL_GRID), dim3(256), 0, ctx->stream, parts,
                     stat_blocks(ctx->ne), mid);
  hipLaunchKernelGGL(k_qual_final, dim3(1), dim3(256), 0, ctx->stream, mid, FINAL_GRID, res);
  return hipGetLastError() == hipSuccess;
}

int pmx_qualhisto(pmx_ctx *ctx, pmx_qual_stats *st) {
  if (!ctx || !st) return 0;
  hipSetDevice(ctx->device);
  if (!pmx_qualhisto_device(ctx, 0, nullptr)) return 0;
  QualPart r;
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) return 0;
  if (hipMemcpy(&r, (QualPart *)ctx->d_red.p + stat_blocks(ctx->ne) + FINAL_GRID, sizeof r, hipMemcpyDeviceToHost) != hipSuccess) return 0;
  st->ne = r.ne;
  st->np = ctx->np;
  st->max = r.max;
  st->min = r.min;
  st->avg = r.avg;
  st->iel = r.ne ? r.iel : 0;
  st->good = r.good;
  st->med = r.med;
  for (int i = 0; i < 5; i++) st->his[i] = r.his[i];
  return 1;
}

// result slot of the prilen reduction in d_red (after both partial arrays)
static int64_t len_res_slot(pmx_ctx *ctx) { return 2 * (int64_t)stat_blocks(ctx->ne) + FINAL_GRID; }

int pmx_prilen_device(pmx_ctx *ctx, const uint16_t *dtag, void *dev_result) {
  StatArgs A{};
  if (!stat_args(ctx, A)) return 0;
  if (ctx->sd.imet < 0) { ctx->err = "pmx_prilen: no metric"; return 0; }
  if (ctx->ne >= (1LL << 29)) { ctx->err = "pmx_prilen: ne >= 2^29 per group"; return 0; }
  A.ptag = dtag;
  const int nb = stat_blocks(ctx->ne);
  if (!ensure_red(ctx, sizeof(LenPart) * (2 * (size_t)nb + FINAL_GRID + 1))) return 0;
  LenPart *parts = (LenPart *)ctx->d_red.p;
  LenPart *res = dev_result ? (LenPart *)dev_result : parts + len_res_slot(ctx);
  if (!dgrow_u8(ctx, ctx->d_emask, (size_t)(ctx->ne + 1)) ||
      !dgrow_u32(ctx, ctx->d_elist, (size_t)(6 * ctx->ne + 1)) ||
      !dgrow_u32(ctx, ctx->d_bcount, (size_t)nb + 1))
    return 0;
  unsigned *bc = ctx->d_bcount.p, *total = ctx->d_bcount.p + nb;
  hipLaunchKernelGGL(k_len_mark, dim3(nb), dim3(256), 0, ctx->stream, A, parts, ctx->d_emask.p, bc);
  hipLaunchKernelGGL(k_len_scan, dim3(1), dim3(256), 0, ctx->stream, bc, nb, total);
  hipLaunchKernelGGL(k_len_compact, dim3(nb), dim3(256), 0, ctx->stream, ctx->d_emask.p, ctx->ne, bc,
                     ctx->d_elist.p);
  hipLaunchKernelGGL(k_len_rotate, dim3(nb), dim3(256), 0, ctx->stream, A, ctx->d_elist.p, total,
                     parts + nb);
  LenPart *mid = parts + 2 * nb;
  hipLaunchKernelGGL(k_prilen_final, dim3(FINAL_GRID), dim3(256), 0, ctx->stream, parts, 2 * nb, mid);
  hipLaunchKernelGGL(k_prilen_final, dim3(1), dim3(256), 0, ctx->stream, mid, FINAL_GRID, res);
  return hipGetLastError() == hipSuccess;
}

int pmx_prilen(pmx_ctx *ctx, const uint16_t *point_tag, int64_t tag_stride, int metRidTyp,
               pmx_len_stats *st) {
  (void)metRidTyp;   // classic storage only: met->size 1 or 6 on every point
  if (!ctx || !st) return 0;
  hipSetDevice(ctx->device);
  uint16_t *dtag = nullptr;
  if (point_tag) {
    std::vector<uint16_t> h((size_t)(ctx->np + 1), 0);
    for (int64_t i = 1; i <= ctx->np; i++)
      h[(size_t)i] = *(const uint16_t *)((const char *)point_tag + i * tag_stride);
    if (hipMalloc((void **)&dtag, h.size() * 2) != hipSuccess) return 0;
    hipMemcpy(dtag, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  }
  int r = pmx_prilen_device(ctx, dtag, nullptr);
  LenPart res;
  if (r) {
    r = hipStreamSynchronize(ctx->stream) == hipSuccess &&
        hipMemcpy(&res, (LenPart *)ctx->d_red.p + len_res_slot(ctx), sizeof res, hipMemcpyDeviceToHost) == hipSuccess;
  }
  if (dtag) hipFree(dtag);
  if (!r) return 0;
  st->ned = res.ned;
  st->nullEdge = res.nul;
  st->avlen = res.avlen;
  st->lmin = res.ned ? res.lmin : 1.e30;
  st->lmax = res.lmax;
  st->amin = st->bmin = st->amax = st->bmax = 0;
  // endpoints from the first-occurrence keys
  if (res.ned) {
    TetRec t;
    int64_t k = res.kmin / 6;
    int ia = (int)(res.kmin % 6);
    static const int ia0[6] = {0, 0, 0, 1, 1, 2}, ia1[6] = {1, 2, 3, 2, 3, 3};
    hipMemcpy(&t, ctx->d_tets.p + k, sizeof t, hipMemcpyDeviceToHost);
    st->amin = t.v[ia0[ia]];
    st->bmin = t.v[ia1[ia]];
    k = res.kmax / 6;
    ia = (int)(res.kmax % 6);
    hipMemcpy(&t, ctx->d_tets.p + k, sizeof t, hipMemcpyDeviceToHost);
    st->amax = t.v[ia0[ia]];
    st->bmax = t.v[ia1[ia]];
  }
  for (int i = 0; i < 9; i++) st->hl[i] = res.hl[i];
  return 1;
}

}  // extern "C"
