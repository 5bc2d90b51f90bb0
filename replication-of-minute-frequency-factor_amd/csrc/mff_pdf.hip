// mff_pdf.hip — doc_pdf60..95: the frame-wide average rank (CM:1006-1138).
//
// The reference ranks `close.last().over(code,date) / close` over ALL rows of the day
// frame (CM:1015-1017: `.rank()` is outside `.over`), then reports, per stock-day, the
// rank of the level where the cumulative volume share first exceeds p.  Stage 1 emits
// that level's key q (the "query", 5 per stock-day).  The rank of q among the day's
// keys is n_less(q) + (n_eq(q) + 1) / 2 (S6 'average'), computed here without sorting
// the day's ~240*S keys:
//   1. sort    — per day, the 5*S (x R ranks) queries as total-order u64 (mff_sort.h);
//   2. count   — per (day, chunk of 256 stocks) workgroup, every local key c_last/c_b
//                finds its bin among the sorted queries (lower_bound: LDS splitters,
//                then 32 keys in L2) and bumps a packed (eq<<16 | lt) LDS counter; the
//                chunk histograms are summed and prefix-scanned per day -> (n_less, n_eq)
//                per sorted query position, over THIS rank's keys;
//   [multi-GPU: counts are summed over ranks with one all-reduce]
//   3. finalize — each own query looks its position up and writes the rank.
#include "../../include/mff.h"
#include "mff_internal.h"
#include "mff_sort.h"
#include "mff_group.h"
#include "mff_wave.h"

namespace mff {

constexpr int PDF_MAXM = 32767;  // queries per day (all ranks)
constexpr int PDF_ZQ = 8192;     // sorted queries per count workgroup (LDS: 16 B each)
constexpr int PDF_NBK = 2048;    // bucket table over the workgroup's query range

struct QLoader {
  const double* q;  // [R][5][D][S_loc]
  int S, D, d;
  __device__ uint64_t operator()(int i) const {
    const int s = i % S;
    const int rt = i / S;  // r*5 + t
    const double x = q[((size_t)rt * D + d) * S + s];
    return __builtin_isnan(x) ? ~0ull : ord64(x);
  }
};

__global__ __launch_bounds__(SORT_THREADS) void k_pdf_sort(const double* q_all, int R, int S, int D,
                                                           int d0, uint64_t* q_sorted, uint64_t* tmp) {
  __shared__ uint64_t sk[SORT_CAP];
  const int dd = blockIdx.x;
  const int M = R * 5 * S;
  QLoader ld{q_all, S, D, d0 + dd};
  segment_sort(ld, M, q_sorted + (size_t)dd * M, tmp + (size_t)dd * M, sk);
}

// One workgroup per (day, slice of <= PDF_ZQ consecutive sorted queries): the slice and
// its predecessor Q[P0-1] sit in LDS with a bucket table over the slice's key range, so
// a key's lower_bound is a table lookup plus a short LDS binary search.  Every key of
// the day is formed in every slice's workgroup (the slices of a day share the close
// plane through L2: their blocks are mapped onto one XCD); a key at or below Q[P0-1]
// only bumps the slice's `below` count, a key above the slice is dropped.  The slice
// then writes (n_less, n_eq) at its positions: below + exclusive scan + own lt.
__global__ __launch_bounds__(1024) void k_pdf_count(const float* close, const uint32_t* valid, int S,
                                                    int d0, int nd, const uint64_t* q_sorted, int M,
                                                    int Z, int Mz, uint32_t* counts) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t below_s;
  // XCD-aware block order: hardware dispatches block b to XCD b % 8; the Z slices of a
  // day get consecutive logical ids on one XCD
  const int nb = gridDim.x;
  const int per_xcd = nb >> 3;  // host pads the grid to a multiple of 8
  const int lid = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  const int dd = lid / Z, z = lid % Z;
  if (dd >= nd) return;
  const int d = d0 + dd;
  const uint64_t* Q = q_sorted + (size_t)dd * M;
  const int P0 = z * Mz, P1 = min(M, P0 + Mz);
  uint32_t* out = counts + ((size_t)dd * M) * 2;

  uint64_t* L = reinterpret_cast<uint64_t*>(smem);      // [Mz + 1]: Q[P0-1], Q[P0..P1)
  uint32_t* lt = reinterpret_cast<uint32_t*>(L + Mz + 1);  // [Mz]
  uint32_t* eqc = lt + Mz;                                // [Mz]
  uint16_t* T = reinterpret_cast<uint16_t*>(eqc + Mz);     // [PDF_NBK + 1]

  // valid (non-NaN) part of the slice: NaN queries sort last as ~0 and are never read
  const int nq = P1 - P0;
  for (int i = threadIdx.x; i < nq; i += blockDim.x) {
    L[1 + i] = Q[P0 + i];
    lt[i] = 0u;
    eqc[i] = 0u;
  }
  if (threadIdx.x == 0) {
    L[0] = P0 > 0 ? Q[P0 - 1] : 0ull;
    below_s = 0u;
  }
  __syncthreads();
  int nv = lower_bound_u64(L + 1, 0, nq, ~0ull);  // first sentinel
  const uint64_t qmin = nv > 0 ? L[1] : 0ull, qmax = nv > 0 ? L[nv] : 0ull;
  int sh = 0;
  while (nv > 0 && ((qmax - qmin) >> sh) >= (uint64_t)PDF_NBK) ++sh;
  for (int b = threadIdx.x; b <= PDF_NBK; b += blockDim.x) {
    int v = nv;
    if (nv > 0 && b < PDF_NBK) {
      const uint64_t edge = qmin + ((uint64_t)b << sh);
      v = (edge > qmax || edge < qmin) ? nv : lower_bound_u64(L + 1, 0, nv, edge);
    }
    T[b] = (uint16_t)v;
  }
  __syncthreads();

  if (nv > 0) {
    const int lane = lane_id();
    const int g = lane & 15;
    const int grp = (threadIdx.x >> 4);  // 64 groups of 16 lanes
    const uint64_t L0 = L[0];
    uint32_t below = 0u;
    for (int s = grp; s < S; s += 64) {  // one stock per 16-lane group
      const size_t sd = (size_t)d * S + s;
      uint32_t pb = 0u;
      if (g < 15) pb = (valid[sd * 8 + (g >> 1)] >> (16 * (g & 1))) & 0xFFFFu;
      if (g16::gmax_i((int)pb) == 0) continue;  // absent stock-day (group-uniform)
      float c[16];
      if (g < 15) {
        const float4* p4 = reinterpret_cast<const float4*>(close + sd * NBAR + 16 * g);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 t = p4[q];
          c[4 * q] = t.x; c[4 * q + 1] = t.y; c[4 * q + 2] = t.z; c[4 * q + 3] = t.w;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) c[k] = 1.f;
      }
      const int lb = g16::glast(pb);
      const double clast = (double)g16::gval(c, lb);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (!((pb >> k) & 1u)) continue;
        const uint64_t key = ord64(clast / (double)c[k]);
        if (key <= L0) { ++below; continue; }
        if (key > qmax) continue;
        int lo = 0, hi = 0;
        if (key > qmin) {
          const int b = (int)((key - qmin) >> sh);
          lo = T[b];
          hi = T[b + 1];
        }
        const int j = lower_bound_u64(L + 1, lo, hi, key);
        atomicAdd(L[1 + j] == key ? &eqc[j] : &lt[j], 1u);
      }
    }
    below = (uint32_t)__reduce_add_sync(~0ull, (int)below);
    if (lane_id() == 0) atomicAdd(&below_s, below);
  }
  __syncthreads();

  // (n_less, n_eq) at P0 + i: below + sum_{i' < i} (lt + eq) + lt[i]
  const int per = (nq + 1023) >> 10;
  const int i0 = min(nq, (int)threadIdx.x * per), i1 = min(nq, i0 + per);
  uint32_t tot = 0u;
  for (int i = i0; i < i1; ++i) tot += lt[i] + eqc[i];
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  uint32_t incl = tot;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  uint32_t run = below_s + incl - tot;
  for (int w = 0; w < wave; ++w) run += wsum[w];
  for (int i = i0; i < i1; ++i) {
    out[2 * (P0 + i)] = run + lt[i];
    out[2 * (P0 + i) + 1] = eqc[i];
    run += lt[i] + eqc[i];
  }
}

struct PdfRows {
  int r[5];
};

__global__ void k_pdf_finalize(const double* q_local, const uint64_t* q_sorted, const uint32_t* counts,
                               int S, int D, int d0, int nd, int M, PdfRows rows, double* val,
                               uint8_t* state) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long tot = 5ll * nd * S;
  if (gid >= tot) return;
  const int s = (int)(gid % S);
  const int dd = (int)((gid / S) % nd);
  const int t = (int)(gid / ((long long)S * nd));
  const int row = rows.r[t];
  if (row < 0) return;
  const int d = d0 + dd;
  const double q = q_local[((size_t)t * D + d) * S + s];
  if (__builtin_isnan(q)) return;  // no level passed (null) or absent stock-day
  const uint64_t key = ord64(q);
  const uint64_t* Q = q_sorted + (size_t)dd * M;
  const int j = lower_bound_u64(Q, 0, M, key);
  const uint32_t* cn = counts + ((size_t)dd * M + j) * 2;
  const double rank = (double)cn[0] + ((double)cn[1] + 1.0) * 0.5;
  const size_t o = (size_t)row * D * S + (size_t)d * S + s;
  val[o] = rank;
  state[o] = MFF_STATE_VALUE;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace mff

using namespace mff;

extern "C" {

size_t mff_pdf_workspace_bytes(int S_loc, int R, int nd) {
  const size_t M = (size_t)R * 5 * S_loc;
  return align256(M * nd * 8);  // merge-sort ping-pong buffer
}

int mff_pdf_sort(const double* q_all, int R, int S_loc, int D, int d0, int nd, uint64_t* q_sorted,
                 void* workspace, void* stream) {
  clear_error();
  MFF_REQUIRE(R >= 1 && S_loc > 0 && D > 0 && nd > 0 && d0 >= 0 && d0 + nd <= D,
              "mff_pdf_sort: bad sizes R=%d S=%d D=%d d0=%d nd=%d", R, S_loc, D, d0, nd);
  MFF_REQUIRE(q_all && q_sorted && workspace, "mff_pdf_sort: NULL buffer");
  uint64_t* tmp = reinterpret_cast<uint64_t*>(workspace);
  hipLaunchKernelGGL(k_pdf_sort, dim3(nd), dim3(SORT_THREADS), 0, as_stream(stream), q_all, R, S_loc, D,
                     d0, q_sorted, tmp);
  MFF_LAUNCH_CHECK();
  return 0;
}

int mff_pdf_count(const float* close, const uint32_t* valid, int S_loc, int D, int d0, int nd,
                  const uint64_t* q_sorted, int M, uint32_t* counts, void* workspace, void* stream) {
  clear_error();
  MFF_REQUIRE(S_loc > 0 && D > 0 && nd > 0 && d0 >= 0 && d0 + nd <= D && M > 0,
              "mff_pdf_count: bad sizes");
  MFF_REQUIRE(M <= PDF_MAXM, "mff_pdf_count: %d queries per day exceed %d (R*5*S_loc)", M, PDF_MAXM);
  MFF_REQUIRE(close && valid && q_sorted && counts && workspace, "mff_pdf_count: NULL buffer");
  (void)workspace;
  const int Z = (M + PDF_ZQ - 1) / PDF_ZQ;
  const int Mz = (M + Z - 1) / Z;
  const size_t lds = (size_t)(Mz + 1) * 8 + (size_t)Mz * 8 + (size_t)(PDF_NBK + 1) * 2;
  const long long nblk = ((long long)Z * nd + 7) / 8 * 8;
  MFF_REQUIRE(nblk < (1ll << 31), "mff_pdf_count: too many days in one call");
  hipLaunchKernelGGL(k_pdf_count, dim3((unsigned)nblk), dim3(1024), lds, as_stream(stream), close, valid,
                     S_loc, d0, nd, q_sorted, M, Z, Mz, counts);
  MFF_LAUNCH_CHECK();
  return 0;
}

int mff_pdf_finalize(const double* q_local, const uint64_t* q_sorted, const uint32_t* counts, int S_loc,
                     int D, int d0, int nd, int M, const int32_t* pdf_rows, double* val, uint8_t* state,
                     void* stream) {
  clear_error();
  MFF_REQUIRE(S_loc > 0 && D > 0 && nd > 0 && d0 >= 0 && d0 + nd <= D && M > 0,
              "mff_pdf_finalize: bad sizes");
  MFF_REQUIRE(q_local && q_sorted && counts && pdf_rows && val && state, "mff_pdf_finalize: NULL buffer");
  PdfRows rows;
  for (int t = 0; t < 5; ++t) rows.r[t] = pdf_rows[t];
  const long long tot = 5ll * nd * S_loc;
  const int thr = 256;
  hipLaunchKernelGGL(k_pdf_finalize, dim3((unsigned)((tot + thr - 1) / thr)), dim3(thr), 0,
                     as_stream(stream), q_local, q_sorted, counts, S_loc, D, d0, nd, M, rows, val, state);
  MFF_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
