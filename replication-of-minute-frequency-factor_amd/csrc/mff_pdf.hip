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
#include "mff_wave.h"

namespace mff {

constexpr int PDF_CHUNK = 256;  // stocks per count workgroup: <= 61,440 keys < 2^16
constexpr int PDF_SPL = 32;     // queries per LDS splitter
constexpr int PDF_MAXM = 32767; // bins (M+1) u32 must fit 128 KiB of LDS

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

__global__ __launch_bounds__(1024) void k_pdf_count(const float* close, const uint32_t* valid, int S,
                                                    int D, int d0, const uint64_t* q_sorted, int M,
                                                    uint32_t* slab) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* bins = reinterpret_cast<uint32_t*>(smem);  // [M+1]
  const int nspl = (M + PDF_SPL - 1) / PDF_SPL;
  uint64_t* spl = reinterpret_cast<uint64_t*>(smem + (((size_t)(M + 1) * 4 + 15) & ~(size_t)15));
  const int dd = blockIdx.x;
  const int chunk = blockIdx.y;
  const int nchunk = gridDim.y;
  const int d = d0 + dd;
  const uint64_t* Q = q_sorted + (size_t)dd * M;
  for (int i = threadIdx.x; i <= M; i += blockDim.x) bins[i] = 0u;
  for (int i = threadIdx.x; i < nspl; i += blockDim.x) spl[i] = Q[i * PDF_SPL];
  __syncthreads();

  const int lane = lane_id();
  const int wave = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  const bool lv = lane < 60;
  for (int j = wave; j < PDF_CHUNK; j += nw) {
    const int s = chunk * PDF_CHUNK + j;
    if (s >= S) break;
    const size_t sd = (size_t)d * S + s;
    const uint32_t mw = lv ? valid[sd * 8 + (lane >> 3)] : 0u;
    const uint32_t pb = (mw >> ((lane & 7) * 4)) & 0xFu;
    bool p[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) p[k] = (pb >> k) & 1u;
    const Bits B = ballot4(p);
    if (!any(B)) continue;
    float c[4] = {1.f, 1.f, 1.f, 1.f};
    if (lv) {
      const float4 t = reinterpret_cast<const float4*>(close + sd * NBAR)[lane];
      c[0] = t.x; c[1] = t.y; c[2] = t.z; c[3] = t.w;
    }
    const double clast = (double)elem(c, last_of(B));
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (!p[k]) continue;
      const uint64_t key = ord64(clast / (double)c[k]);
      // level 1: splitters in LDS
      int lo = 0, hi = nspl;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (spl[mid] < key) lo = mid + 1; else hi = mid;
      }
      // answer in (32(b-1), 32b]
      const int b = lo;
      int a0 = (b == 0) ? 0 : (b - 1) * PDF_SPL + 1;
      int a1 = min(b * PDF_SPL, M);
      if (b == 0) a1 = 0;
      const int jpos = lower_bound_u64(Q, a0, a1, key);
      const bool eq = jpos < M && Q[jpos] == key;
      atomicAdd(&bins[jpos], eq ? 0x10000u : 1u);
    }
  }
  __syncthreads();
  uint32_t* dst = slab + ((size_t)dd * nchunk + chunk) * (size_t)(M + 1);
  for (int i = threadIdx.x; i <= M; i += blockDim.x) dst[i] = bins[i];
}

// per day: sum chunk histograms, prefix -> (n_less, n_eq) at every query position
__global__ __launch_bounds__(1024) void k_pdf_reduce(const uint32_t* slab, int nchunk, int M,
                                                     uint32_t* counts) {
  __shared__ uint32_t part[1024];
  const int dd = blockIdx.x;
  const uint32_t* sl = slab + (size_t)dd * nchunk * (M + 1);
  const int per = (M + blockDim.x - 1) / blockDim.x;
  const int i0 = threadIdx.x * per, i1 = min(M, i0 + per);
  uint32_t tot = 0;
  for (int i = i0; i < i1; ++i) {
    uint32_t lt = 0, eq = 0;
    for (int cc = 0; cc < nchunk; ++cc) {
      const uint32_t x = sl[(size_t)cc * (M + 1) + i];
      lt += x & 0xffffu;
      eq += x >> 16;
    }
    tot += lt + eq;
  }
  part[threadIdx.x] = tot;
  __syncthreads();
  // exclusive scan of part (Hillis-Steele on 1024 entries)
  for (int o = 1; o < 1024; o <<= 1) {
    const uint32_t y = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0u;
    __syncthreads();
    part[threadIdx.x] += y;
    __syncthreads();
  }
  uint32_t run = threadIdx.x ? part[threadIdx.x - 1] : 0u;
  uint32_t* out = counts + (size_t)dd * M * 2;
  for (int i = i0; i < i1; ++i) {
    uint32_t lt = 0, eq = 0;
    for (int cc = 0; cc < nchunk; ++cc) {
      const uint32_t x = sl[(size_t)cc * (M + 1) + i];
      lt += x & 0xffffu;
      eq += x >> 16;
    }
    out[2 * i] = run + lt;  // keys below Q[i]
    out[2 * i + 1] = eq;    // keys equal to Q[i]
    run += lt + eq;
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
  const size_t nchunk = (S_loc + PDF_CHUNK - 1) / PDF_CHUNK;
  return align256(M * nd * 8) + align256(nchunk * nd * (M + 1) * 4);
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
  const int nchunk = (S_loc + PDF_CHUNK - 1) / PDF_CHUNK;
  uint32_t* slab = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(workspace) +
                                               align256((size_t)M * nd * 8));
  const int nspl = (M + PDF_SPL - 1) / PDF_SPL;
  const size_t lds = (((size_t)(M + 1) * 4 + 15) & ~(size_t)15) + (size_t)nspl * 8;
  hipLaunchKernelGGL(k_pdf_count, dim3(nd, nchunk), dim3(1024), lds, as_stream(stream), close, valid,
                     S_loc, D, d0, q_sorted, M, slab);
  MFF_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_pdf_reduce, dim3(nd), dim3(1024), 0, as_stream(stream), slab, nchunk, M, counts);
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
