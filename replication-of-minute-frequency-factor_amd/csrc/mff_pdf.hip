// mff_pdf.hip — doc_pdf60..95: the frame-wide average rank (CM:1006-1138).
//
// The reference ranks `close.last().over(code,date) / close` over ALL rows of the day
// frame (CM:1015-1017: `.rank()` is outside `.over`), then reports, per stock-day, the
// rank of the level where the cumulative volume share first exceeds p.  Stage 1 emits
// that level's key q (the "query", 5 per stock-day).  The rank of q among the day's
// keys is n_less(q) + (n_eq(q) + 1) / 2 (S6 'average'), computed here without sorting
// the day's ~240*S keys:
//   1. sort    — per day, the 5*S (x R ranks) queries as total-order u64 (mff_sort.h);
//   2. count   — per (day, slice of <= PDF_ZQ sorted queries) workgroup, every local key
//                c_last/c_b finds its position among the slice's queries (LDS bucket
//                table + fixed-depth LDS binary search) and bumps a packed
//                (n_eq << 32 | n_less) LDS counter by its weight; a scan turns the
//                counters into (n_less, n_eq) per sorted query position, over THIS
//                rank's keys.  The keys are stage 1's flat per-day level list: one key
//                per distinct close of a stock-day (rows with equal closes have equal
//                keys), weighted by its bar count, so ~L << 240 keys per stock-day;
//   [multi-GPU: per sorted position each rank writes one word 2 n_less + n_eq (the
//    average rank is linear in it); the words are summed over ranks by one all-reduce]
//   3. finalize — each own query looks its position up in its slice (LDS) and writes the
//                rank.  With one rank, 2 and 3 run as one kernel (mff_pdf_rank_local):
//                the slice's counters never leave LDS.
#include <stdlib.h>

#include <type_traits>

#include <mutex>

#include "../../include/mff.h"
#include "mff_internal.h"
#include "mff_sort.h"
#include "mff_group.h"
#include "mff_wave.h"

namespace mff {

size_t pdf_levels_split(int S, int D, size_t* off_key, size_t* off_w);  // mff_stage1g.hip

constexpr int PDF_MAXM = 1 << 24;
// The level lists are split at a key chosen per pass (pdf_split_init: the mean of the
// previous passes' per-day median queries; ord64(1.0) before any), stored in the level
// buffer's header: stage 1 writes the keys below it into list A, the others into list B.
constexpr uint64_t PDF_KSPLIT0 = 0xBFF0000000000000ull;  // ord64(1.0)
// slice capacity of the split-aligned count (LDS: 12 B per query + the bucket table,
// within 160 KiB): two slices cover 25,800 queries, a day of 5,160 stocks
constexpr int PDF_KCAP = 12900;
// learned split key, one per device: sum / count of the per-day medians seen since the
// last pass start, and the key in use
struct PdfLearn {
  double sum;
  uint32_t n;
  uint32_t pad;
  uint64_t key;
};  // queries per day (all ranks): 2 n_less + n_eq stays in u32
constexpr int PDF_ZQ = 9160;     // sorted queries per workgroup, u64 counters (LDS: 16 B each)
constexpr int PDF_ZQ32 = 12500;  // sorted queries per count workgroup, packed u32 counters (12 B)
constexpr int PDF_PAD = 64;      // ~0 sentinels after the slice's distinct values
constexpr int PDF_NBK = 4096;  // bucket table over the workgroup's distinct query values
constexpr int PDF_CT = 1024;     // threads per count / finalize workgroup (<= 1024: wsum[16])
// packed counter: n_less part in the low PDF_LB bits, n_eq part above.  Exact while a
// slice's total weight stays below 2^PDF_LB (240 bars x S_loc < 2^21: S_loc <= 8738) and
// no single value collects 2^(32 - PDF_LB) equal keys -- the latter is detected (the
// fields no longer sum to the slice's weight) and the slice recounted with u64 counters.
// The one value every stock-day holds is 1.0 (c_last / c_last: the last close's level),
// so its equal keys are counted apart, in a full u32.
constexpr int PDF_LB = 21;
// count: level-list entries per thread per chunk (8 or 16; the next chunk is loaded while
// this one is searched)
constexpr int PDF_UNR = 8;

struct QLoader {
  const double* q;  // [R][5][D][S_loc]
  int S, D, d;
  __device__ uint64_t operator()(int i) const {
    const int s = i % S;
    const int rt = i / S;  // r*5 + t
    const double x = q[((size_t)rt * D + d) * S + s];
    return __builtin_isnan(x) ? ~0ull : ord64(x);
  }
  // (row, column) view for segment_sort_binned: row r*5+t, column s
  int nrow;
  __device__ int rows() const { return nrow; }
  __device__ int cols() const { return S; }
  __device__ uint64_t at(int rt, int s) const { return key(raw(rt, s)); }
  // the load and the key conversion apart, so the sort's passes issue a batch of loads
  // before converting any of them
  __device__ double raw(int rt, int s) const { return q[((size_t)rt * D + d) * S + s]; }
  __device__ static uint64_t key(double x) {
    // branch-free: a select, not a divergent region between the loads and their use
    const uint64_t k = ord64(x);
    return __builtin_isnan(x) ? ~0ull : k;
  }
};

// 8 waves per SIMD (two 1,024-thread workgroups per CU, 64 VGPRs: 22 spilled) measured
// faster than 4 without spills (sort alone at c4: 1.37 vs 1.78 ms; bitonic ranges: 2.78)
__global__ __launch_bounds__(SORT_THREADS, 8) void k_pdf_sort(const double* q_all, int R, int S, int D,
                                                           int d0, uint64_t* q_sorted, uint64_t* tmp) {
  __shared__ uint64_t sk[SORT_CAPB];  // >= SORT_CAP for the merge fallback
  __shared__ uint32_t bins[SORT_NBIN + 1];
  __shared__ __attribute__((aligned(8))) uint32_t ctl[64];
  const int dd = blockIdx.x;
  const int M = R * 5 * S;
  QLoader ld{q_all, S, D, d0 + dd, R * 5};
  // bucketed (no merge passes) when the day's queries fit the registers and no bin
  // overflows half a chunk; otherwise chunk sort + global merges
  if (M <= SORT_REG * SORT_THREADS && segment_sort_binned(ld, M, q_sorted + (size_t)dd * M, sk, bins, ctl))
    return;
  segment_sort(ld, M, q_sorted + (size_t)dd * M, tmp + (size_t)dd * M, sk);
}

// One workgroup per (day, slice of <= PDF_ZQ consecutive sorted queries).  The slice,
// its predecessor Q[P0-1] and a bucket table over the slice's key range sit in LDS.
// Every 16-lane group walks the day's stocks (the next stock's closes are loaded while
// the current one is binned); a stock's 16x16 keys are binned together: all lookups of
// one search step are independent LDS reads issued back to back, and the step count is
// the table's worst bucket occupancy (block-uniform), so there is no divergent loop.
// A key at or below Q[P0-1] only bumps the slice's `below` count, a key above the slice
// is dropped (a later slice bins it).  Counters are one packed u64 per query position
// (n_less in the low word, n_eq in the high word): one ds_add_u64 per binned key.
// The slice then turns them into (n_less, n_eq) at its positions: below + exclusive scan.
struct PdfSlice {
  const uint64_t* L;  // LDS [nq + 1 + PDF_PAD]: Q[P0-1], Q[P0..P1), ~0 x PDF_PAD
  const uint16_t* T;  // LDS [PDF_NBK + 1]
  uint64_t L0, qmin, qmax;
  int nv, sh, steps;
  // lower_bound of `key` inside the slice (key in (L0, qmax]); position relative to P0
  __device__ __forceinline__ void range(uint64_t key, int& lo, int& hi) const {
    lo = hi = 0;
    if (key > qmin) {
      const int b = (int)((key - qmin) >> sh);
      lo = T[b];
      hi = T[b + 1];
    }
  }
};

// lower_bound of key in the sorted Q[0, M), by one wave: 64 probes per round (every
// lane of the wave calls it and gets the result)
__device__ __forceinline__ int wave_lower_bound(const uint64_t* Q, int M, uint64_t key) {
  const int lane = lane_id();
  int lo = 0, hi = M;  // the answer is in [lo, hi]
  while (hi - lo > 64) {
    const int step = (hi - lo + 63) / 64;
    const int p = lo + (lane + 1) * step - 1;
    const bool less = p < hi && Q[p] < key;
    const int c = __popcll(__ballot(less));  // Q sorted: the lanes below c are less
    const int nlo = lo + c * step;
    hi = min(hi, lo + (c + 1) * step);
    lo = nlo;
  }
  const int p = lo + lane;
  const bool less = p < hi && Q[p] < key;
  return lo + __popcll(__ballot(less));
}

// block-wide exclusive scan of one u32 per thread (wsum: 16 words of LDS); returns the
// thread's offset, *total = the block sum.  Ends synced.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* wsum, uint32_t* total) {
  const int lane = lane_id(), wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t incl = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  uint32_t off = incl - x, tot = 0u;
  for (int w = 0; w < nw; ++w) {
    if (w < wave) off += wsum[w];
    tot += wsum[w];
  }
  *total = tot;
  __syncthreads();
  return off;
}

// Load the slice, keep its DISTINCT values above Q[P0-1] (duplicated queries -- many
// stock-days share e.g. the key 1.0 -- would otherwise deepen every search), build the
// bucket table and the search depth.  Block-wide; ends synced.
//   L[0] = Q[P0-1], L[1..nv] = distinct slice values > L[0], L[nv+1 .. nv+PDF_PAD] = ~0
// The slice is copied into L coalesced, then compacted in place: each thread's contiguous
// chunk (at most PDF_SETUP_PER entries) goes through registers, and the scan's trailing
// barrier orders every read before the first write.  The bucket table T[b] = the first
// value whose bucket is >= b (lower_bound of the bucket's lower edge) is built in two
// parallel steps: each value that opens its bucket marks T[bucket] = its index, then a
// block-wide suffix minimum fills the empty buckets (round 6; the round-3 scatter wrote each
// empty run from one thread -- up to ~2,000 serial stores for the run above the last value,
// as the top bucket index lies in [2048, 4096) -- and with one workgroup per CU nothing hid
// that: the slice setup took ~20 us).
constexpr int PDF_SETUP_MAXQ = PDF_ZQ32 > PDF_ZQ ? (PDF_ZQ32 > PDF_KCAP ? PDF_ZQ32 : PDF_KCAP) : (PDF_ZQ > PDF_KCAP ? PDF_ZQ : PDF_KCAP);
constexpr int PDF_SETUP_PER = (PDF_SETUP_MAXQ + PDF_CT - 1) / PDF_CT;
template <typename CT>
__device__ __forceinline__ PdfSlice pdf_slice_setup(const uint64_t* Q, int M, int P0, int P1,
                                                    uint64_t* L, CT* C, uint16_t* T,
                                                    uint32_t* wsum, int* occ_s, uint64_t lo_floor = 0ull,
                                                    const uint32_t* cfill = nullptr) {
  // cfill (optional): per sorted position of the slice a count word; the counter of each
  // distinct value then starts from the word at its first position instead of 0
  const int nq = P1 - P0;
  // every load of the copy in flight before the first LDS store (a rolled loop waits for
  // each load in turn: ~13 global round trips per slice, with one workgroup per CU
  // nothing hides them)
  {
    uint64_t x[PDF_SETUP_PER];
#pragma unroll
    for (int k = 0; k < PDF_SETUP_PER; ++k) {
      const int i = (int)threadIdx.x + k * (int)blockDim.x;
      x[k] = i < nq ? Q[P0 + i] : 0ull;
    }
#pragma unroll
    for (int k = 0; k < PDF_SETUP_PER; ++k) {
      const int i = (int)threadIdx.x + k * (int)blockDim.x;
      if (i < nq) L[1 + i] = x[k];
    }
  }
  // lo_floor: a slice whose queries are all >= the split key counts every key below it
  // as `below` (L0 = split key - 1), so it need not read the list those keys are in
  const uint64_t Lq = P0 > 0 ? Q[P0 - 1] : 0ull;
  const uint64_t L0 = Lq > lo_floor ? Lq : lo_floor;  // (no max(): it may go through double)
  if (threadIdx.x == 0) {
    L[0] = L0;
    *occ_s = 0;
  }
  __syncthreads();
  const int per = (nq + (int)blockDim.x - 1) / (int)blockDim.x;  // <= PDF_SETUP_PER (blockDim = PDF_CT)
  const int i0 = min(nq, (int)threadIdx.x * per), i1 = min(nq, i0 + per);
  uint64_t v[PDF_SETUP_PER];
  uint32_t keep = 0u, cnt = 0u;
#pragma unroll
  for (int k = 0; k < PDF_SETUP_PER; ++k) {
    const int i = i0 + k;
    v[k] = 0ull;
    if (i < i1) {
      const uint64_t x = L[1 + i], xp = L[i];  // L[0] = Q[P0-1]
      v[k] = x;
      if (x != ~0ull && x > L0 && x != xp) {
        keep |= 1u << k;
        ++cnt;
      }
    }
  }
  uint32_t nu;
  uint32_t off = block_excl_scan(cnt, wsum, &nu);  // ends synced: every read above is done
#pragma unroll
  for (int k = 0; k < PDF_SETUP_PER; ++k)
    if ((keep >> k) & 1u) {
      if (cfill) C[off] = (CT)cfill[i0 + k];
      L[1 + off++] = v[k];
    }
  if (!cfill)
    for (int i = threadIdx.x; i < nq; i += blockDim.x) C[i] = (CT)0;
  for (int b = threadIdx.x; b <= PDF_NBK; b += blockDim.x) T[b] = 0xFFFFu;  // unmarked
  if (threadIdx.x < PDF_PAD) L[1 + nu + threadIdx.x] = ~0ull;
  __syncthreads();
  PdfSlice sl;
  sl.L = L;
  sl.T = T;
  sl.L0 = L0;
  sl.nv = (int)nu;
  sl.qmin = nu > 0 ? L[1] : 0ull;
  sl.qmax = nu > 0 ? L[nu] : 0ull;
  int sh = 0;
  while (sl.nv > 0 && ((sl.qmax - sl.qmin) >> sh) >= (uint64_t)PDF_NBK) ++sh;
  sl.sh = sh;
  const uint64_t* L1 = L + 1;
  for (int i = threadIdx.x; i < sl.nv; i += blockDim.x) {
    const int bi = (int)((L1[i] - sl.qmin) >> sh);
    const int bp = i > 0 ? (int)((L1[i - 1] - sl.qmin) >> sh) : -1;
    if (bi != bp) T[bi] = (uint16_t)i;  // the first value of bucket bi
  }
  __syncthreads();
  {
    // suffix minimum over T[0 .. NBK) with T[NBK] = nv: thread t owns buckets
    // [KB t, KB t + KB); a wave-level reverse scan, then one across the waves
    static_assert(PDF_NBK % PDF_CT == 0, "buckets per thread");
    constexpr int KB = PDF_NBK / PDF_CT;
    const int t = (int)threadIdx.x, lane = lane_id(), wv = t >> 6, nw = (int)blockDim.x >> 6;
    uint32_t m[KB];
    uint32_t run = 0xFFFFu;
#pragma unroll
    for (int k = KB - 1; k >= 0; --k) {
      m[k] = min((uint32_t)T[KB * t + k], run);
      run = m[k];
    }
    // inclusive reverse min over lanes >= lane, then exclusive (lanes > lane)
    uint32_t inc = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_down((int)inc, o, 64);
      if (lane + o < 64) inc = min(inc, y);
    }
    uint32_t after = (uint32_t)__shfl_down((int)inc, 1, 64);
    if (lane == 63) after = 0xFFFFu;
    if (lane == 0) wsum[wv] = inc;
    __syncthreads();
    uint32_t carry = (uint32_t)sl.nv;  // T[NBK]
    for (int w = wv + 1; w < nw; ++w) carry = min(carry, wsum[w]);
    carry = min(carry, after);
#pragma unroll
    for (int k = 0; k < KB; ++k) T[KB * t + k] = (uint16_t)min(m[k], carry);
    if (t == 0) T[PDF_NBK] = (uint16_t)sl.nv;
  }
  __syncthreads();
  int occ = 0;
  for (int b = threadIdx.x; b < PDF_NBK; b += blockDim.x) occ = max(occ, (int)T[b + 1] - (int)T[b]);
  occ = __reduce_max_sync(~0ull, occ);
  if (lane_id() == 0) atomicMax(occ_s, occ);
  __syncthreads();
  const int mo = *occ_s;
  sl.steps = mo > 0 ? 32 - __builtin_clz((unsigned)mo) : 0;  // ceil(log2(mo + 1))
  return sl;
}

// packed counters -> final (n_less | n_eq << 32) per distinct value (block-wide)
__device__ __forceinline__ void pdf_slice_scan(uint64_t* C, int nv, uint32_t below, uint32_t* wsum) {
  const int per = (nv + (int)blockDim.x - 1) / (int)blockDim.x;
  const int i0 = min(nv, (int)threadIdx.x * per), i1 = min(nv, i0 + per);
  uint32_t tot = 0u;
  for (int i = i0; i < i1; ++i) tot += (uint32_t)C[i] + (uint32_t)(C[i] >> 32);
  uint32_t all;
  uint32_t run = below + block_excl_scan(tot, wsum, &all);
  for (int i = i0; i < i1; ++i) {
    const uint32_t lt = (uint32_t)C[i], eq = (uint32_t)(C[i] >> 32);
    C[i] = (uint64_t)(run + lt) | ((uint64_t)eq << 32);
    run += lt + eq;
  }
  __syncthreads();
}

// own queries [5][D][S] of day d that fall in this slice -> rank (S6 average)
__device__ __forceinline__ void pdf_slice_resolve(const PdfSlice& sl, const uint64_t* C, const double* q_local,
                                                  int S, int D, int d, const int (&rows)[5], double* val,
                                                  uint8_t* state) {
  if (sl.nv == 0) return;
  const size_t plane = (size_t)D * S;
  for (int i = threadIdx.x; i < 5 * S; i += blockDim.x) {
    const int t = i / S, s = i - t * S;
    if (rows[t] < 0) continue;
    const double q = q_local[(size_t)t * plane + (size_t)d * S + s];
    if (__builtin_isnan(q)) continue;  // no level passed (null) or absent stock-day
    const uint64_t key = ord64(q);
    if (key <= sl.L0 || key > sl.qmax) continue;  // another slice owns its first copy
    int lo, hi;
    sl.range(key, lo, hi);
    const int j = lower_bound_u64(sl.L + 1, lo, hi, key);
    const uint64_t cn = C[j];
    const double rank = (double)(uint32_t)cn + ((double)(uint32_t)(cn >> 32) + 1.0) * 0.5;
    const size_t o = (size_t)rows[t] * plane + (size_t)d * S + s;
    val[o] = rank;
    state[o] = MFF_STATE_VALUE;
  }
}

struct Rows5 {
  int r[5];
};

struct PdfArgs {
  // level side channel written by stage 1 (mff_pdf_levels_bytes): per-day entry counts,
  // flat key / weight lists of capacity `cap` per day
  const uint32_t* lvl_count;
  const uint64_t* lvl_key;
  const uint8_t* lvl_w;
  size_t cap;
  const uint64_t* q_sorted;
  uint32_t* counts;       // [nd][M] 2 n_less + n_eq (count phase) or NULL (fused finalize)
  const double* q_local;  // fused finalize: own queries [5][D][S]
  double* val;
  uint8_t* state;
  int rows[5];
  int S, D, d0, nd, M, Z, Mz;
  int packed;  // count: u32 packed counters (PDF_LB), u64 recount on overflow
  int kslice;  // fused count: slices aligned at the split key (each reads one level list)
  PdfLearn* learn;  // kslice: the learned split key's state (k_pdf_learn, after the count)
  int frame;   // count: ONE sorted list [M] for every day (a multi-date frame ranked
               // frame-wide, CM:1015-1017); each day's words are atomically added to counts[M]
};

// One (day, slice [P0, P1)) count.  C32: packed u32 counters (n_less part low, n_eq part
// high); returns false -- before writing anything -- when an n_eq field overflowed, so the
// caller recounts the slice with u64 counters.
template <bool FUSED, bool C32>
__device__ __forceinline__ bool pdf_count_slice(const PdfArgs& a, int d, int dd, int P0, int P1, int mz,
                                                unsigned char* smem, uint32_t* wsum, uint32_t* below_s,
                                                uint32_t* inw_s, uint32_t* one_s, int* occ_s,
                                                uint64_t lo_floor) {
  constexpr uint64_t K1 = 0xBFF0000000000000ull;  // ord64(1.0)
  typedef typename std::conditional<C32, uint32_t, uint64_t>::type CT;
  const int S = a.S;
  const int qd = a.frame ? 0 : dd;  // the sorted list this day's keys are counted against
  const uint64_t* Q = a.q_sorted + (size_t)qd * a.M;
  const int nq = P1 - P0;
  uint64_t* L = reinterpret_cast<uint64_t*>(smem);  // [mz + 1 + PDF_PAD]
  CT* C = reinterpret_cast<CT*>(L + mz + 1 + PDF_PAD);  // [mz]
  uint16_t* T = reinterpret_cast<uint16_t*>(C + mz);
  __shared__ int nxt_s[2];  // the key loop's next chunk, per list
  if (threadIdx.x == 0) {
    *below_s = 0u;
    *inw_s = 0u;
    *one_s = 0u;
    nxt_s[0] = nxt_s[1] = 0;
  }
  const PdfSlice sl = pdf_slice_setup(Q, a.M, P0, P1, L, C, T, wsum, occ_s, lo_floor);

  uint32_t below = 0u, inw = 0u;
  if (sl.nv > 0) {
    // The day's levels are two lists split at the pass's key (stage 1 writes keys below
    // it from the front of the day's region, the others from its back): a slice reads
    // list A only if some of its keys can exceed L0, list B only if the slice reaches the
    // split key; list A skipped counts as `below` by its bars (its weight bytes only).
    const int nA = (int)a.lvl_count[2 * d], nB = (int)a.lvl_count[2 * d + 1];
    const uint64_t ksplit = pdf_split_key(a.lvl_count, a.D);
    const bool readA = sl.L0 < ksplit - 1ull, readB = sl.qmax >= ksplit;
    if (!readA) {
      // every list-A key is below this slice: their bars, from list A's weight bytes
      // (1 B per entry, 16 per load; the day's slots start 64-B aligned)
      // (four 16-B loads in flight per thread and round)
      const uint8_t* WA = a.lvl_w + (size_t)d * a.cap;
      const int step = 16 * (int)blockDim.x;
      for (int i0 = 16 * (int)threadIdx.x; i0 < nA; i0 += 4 * step) {
        uint4 q4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = i0 + r * step;
          q4[r] = i + 16 <= nA ? *reinterpret_cast<const uint4*>(WA + i) : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = i0 + r * step;
          if (i + 16 <= nA) {
            const uint32_t wq[4] = {q4[r].x, q4[r].y, q4[r].z, q4[r].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const uint32_t h = (wq[k] & 0x00FF00FFu) + ((wq[k] >> 8) & 0x00FF00FFu);
              below += (h & 0xFFFFu) + (h >> 16);
            }
          } else if (i < nA) {
            for (int k = i; k < nA; ++k) below += WA[k];
          }
        }
      }
    }
    // The day's level list is flat (stage 1 appends every stock-day's levels: key =
    // c_last / c as ord64, weight = bars at the level), so a thread simply takes chunks of
    // UNR entries (their loads in flight together, their searches interleaved).  A key at or below Q[P0-1] only adds its weight to `below`; a key
    // above the slice belongs to a later slice.  Search: binary lifting from T[b]-1
    // (L1[T[b]-1] < key <= L1[T[b+1]]), one LDS read, compare and select per step.  With
    // at most 6 steps the probes stay inside the PDF_PAD sentinels (probe <= nv + 2^steps
    // - 2), so the steps are unrolled with constant strides: j is a byte offset and each
    // probe is one ds_read_b64 with an immediate offset.
    constexpr int UNR = PDF_UNR;
    const uint64_t* L1 = L + 1;
    const char* Lb = reinterpret_cast<const char*>(L);
    const int nvc = sl.nv;
    const uint64_t* K = a.lvl_key + (size_t)d * a.cap;
    const uint8_t* Wt = a.lvl_w + (size_t)d * a.cap;
    const int steps = sl.steps;
    const bool shallow = steps <= 6;
    // software-pipelined: the next UNR entries are loaded before this UNR's searches
    // (two register sets, the loop unrolled twice: no copies between them).  A thread
    // takes UNR consecutive entries (chunk c = entries [UNR c, UNR c + UNR)): the keys as
    // four 16-B loads and the bars as one 8-B load (a wave reads 4 KB of keys
    // contiguously) instead of UNR strided key and byte loads.  Every day's list starts
    // 64-B aligned (pdf_day_cap: S x 256 entries per day), so the vector loads are
    // aligned; the last partial chunk loads entry by entry.
    static_assert(UNR == 8 || UNR == 16, "chunk loads assume 8 or 16 entries");
    int s = 0, e = 0, s8 = 0;  // the list being read: entries [s, e), chunks from s8 = s rounded down
    auto fetch = [&](uint64_t (&nkey)[UNR], uint32_t (&nw)[UNR], int c) {
      const int i0 = s8 + c * UNR;
      if (i0 >= s && i0 + UNR <= e) {
        const uint4* kp = reinterpret_cast<const uint4*>(K + i0);
#pragma unroll
        for (int q = 0; q < UNR / 2; ++q) {
          const uint4 t = kp[q];
          nkey[2 * q] = (uint64_t)t.x | ((uint64_t)t.y << 32);
          nkey[2 * q + 1] = (uint64_t)t.z | ((uint64_t)t.w << 32);
        }
        uint32_t wv[UNR / 4];
        if constexpr (UNR == 8) {
          const uint2 w2 = *reinterpret_cast<const uint2*>(Wt + i0);
          wv[0] = w2.x;
          wv[1] = w2.y;
        } else {
          const uint4 w4 = *reinterpret_cast<const uint4*>(Wt + i0);
          wv[0] = w4.x;
          wv[1] = w4.y;
          wv[2] = w4.z;
          wv[3] = w4.w;
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) nw[u] = (wv[u >> 2] >> (8 * (u & 3))) & 0xFFu;
      } else {
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          const int i = i0 + u;
          const bool v = i >= s && i < e;
          nkey[u] = v ? K[i] : 0ull;
          nw[u] = v ? (uint32_t)Wt[i] : 0u;
        }
      }
    };
    // p = the key's position among L[1..]: L1[p - 1] < key <= L1[p].  The search runs on
    // the byte offset jb = 8 p' of the probe base p' (L[p'] < key), unsigned, so every probe
    // is one ds_read_b64 at jb + an immediate offset; the bucket lookups of the UNR keys
    // are issued together (no branch around them).
    auto process = [&](const uint64_t (&key)[UNR], const uint32_t (&w)[UNR]) {
      uint32_t jb[UNR];
      bool in[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const bool bl = key[u] <= sl.L0;  // (padding entries have weight 0)
        in[u] = !bl && key[u] <= sl.qmax;
        below += bl ? w[u] : 0u;
        inw += in[u] ? w[u] : 0u;
        const bool g = in[u] && key[u] > sl.qmin;
        const uint32_t bk = g ? (uint32_t)((key[u] - sl.qmin) >> sl.sh) : 0u;
        const uint32_t t = sl.T[bk];
        jb[u] = g ? t << 3 : 0u;  // L[jb / 8] < key
      }
      if (shallow) {
        // the probe base as an LDS pointer: each probe is base register + immediate
        const char* pj[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) pj[u] = Lb + jb[u];
#pragma unroll
        for (int st = 5; st >= 0; --st) {
          if (st < steps) {
            const uint32_t bb = 8u << st;
            uint64_t x[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) x[u] = *reinterpret_cast<const uint64_t*>(pj[u] + bb);
#pragma unroll
            for (int u = 0; u < UNR; ++u) pj[u] += x[u] < key[u] ? bb : 0u;
          }
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) jb[u] = (uint32_t)(pj[u] - Lb);
      } else {
        int j[UNR];  // index into L1 of the probe base (-1: below L1[0])
#pragma unroll
        for (int u = 0; u < UNR; ++u) j[u] = (int)(jb[u] >> 3) - 1;
        for (int bb = (1 << steps) >> 1; bb > 0; bb >>= 1) {
          uint64_t x[UNR];
#pragma unroll
          for (int u = 0; u < UNR; ++u) x[u] = L1[min(j[u] + bb, nvc)];
#pragma unroll
          for (int u = 0; u < UNR; ++u) j[u] = x[u] < key[u] ? j[u] + bb : j[u];
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) jb[u] = (uint32_t)(j[u] + 1) << 3;
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const uint32_t pos = jb[u] >> 3;
        const uint64_t x = *reinterpret_cast<const uint64_t*>(Lb + jb[u] + 8);  // L1[pos]
        if (in[u]) {
          if (C32 && x == key[u] && key[u] == K1) atomicAdd(one_s, w[u]);
          else if (C32) atomicAdd(reinterpret_cast<uint32_t*>(&C[pos]), x == key[u] ? (w[u] << PDF_LB) : w[u]);
          else atomicAdd(reinterpret_cast<unsigned long long*>(&C[pos]),
                         x == key[u] ? ((uint64_t)w[u] << 32) : (uint64_t)w[u]);
        }
      }
    };
    // The chunks are handed out dynamically, 64 per wave-grab (lane l takes chunk b + l:
    // a wave still reads 4 KB of keys contiguously) from an LDS counter per list: with one
    // workgroup per CU a static round-robin split left the early waves waiting at the
    // barrier after the loop for the late ones (round 6 stamps: ~19 % of a workgroup's
    // cycles between wave 0's loop end and the scan, profiles/r06/count_stamps.log)
    const int lane = lane_id();
    auto grab = [&](int list) -> int {
      int b = 0;
      if (lane == 0) b = atomicAdd(&nxt_s[list], 64);
      return __builtin_amdgcn_readfirstlane(b);
    };
    for (int list = 0; list < 2; ++list) {
      if (list == 0 ? !readA : !readB) continue;
      s = list == 0 ? 0 : (int)a.cap - nB;
      e = list == 0 ? nA : (int)a.cap;
      s8 = s & ~(UNR - 1);  // 64-B aligned chunks (every day's region starts 64-B aligned)
      const int nch = (e - s8 + UNR - 1) / UNR;
      uint64_t ka[UNR], kb[UNR];
      uint32_t wa[UNR], wb[UNR];
      // software-pipelined over two register sets: the next grab's chunk loads before this
      // chunk's searches (a chunk past the list loads zero weights: processed as nothing)
      int b0 = grab(list);
      fetch(ka, wa, b0 + lane);
      while (b0 < nch) {  // wave-uniform
        const int b1 = grab(list);
        fetch(kb, wb, b1 + lane);
        process(ka, wa);
        if (b1 >= nch) break;
        b0 = grab(list);
        fetch(ka, wa, b0 + lane);
        process(kb, wb);
      }
    }
    below = (uint32_t)__reduce_add_sync(~0ull, (int)below);
    inw = (uint32_t)__reduce_add_sync(~0ull, (int)inw);
    if (lane_id() == 0) {
      atomicAdd(below_s, below);
      atomicAdd(inw_s, inw);
    }
  }
  __syncthreads();
  if (C32) {
    // packed fields -> 2 n_less + n_eq per distinct value; the fields must sum to the
    // slice's in-range weight (else an n_eq field wrapped: recount with u64 counters)
    uint32_t* C2 = reinterpret_cast<uint32_t*>(C);
    const int per = (sl.nv + (int)blockDim.x - 1) / (int)blockDim.x;
    const int i0 = min(sl.nv, (int)threadIdx.x * per), i1 = min(sl.nv, i0 + per);
    const uint32_t one = *one_s;
    auto eq_at = [&](int i) { return (C2[i] >> PDF_LB) + (L[1 + i] == K1 ? one : 0u); };
    uint32_t tot = 0u;
    for (int i = i0; i < i1; ++i) tot += (C2[i] & ((1u << PDF_LB) - 1u)) + eq_at(i);
    uint32_t all;
    uint32_t run = *below_s + block_excl_scan(tot, wsum, &all);
    if (all != *inw_s) return false;  // block-uniform; nothing written yet
    for (int i = i0; i < i1; ++i) {
      const uint32_t lt = C2[i] & ((1u << PDF_LB) - 1u), eq = eq_at(i);
      C2[i] = 2u * (run + lt) + eq;
      run += lt + eq;
    }
    __syncthreads();
  } else {
    pdf_slice_scan(reinterpret_cast<uint64_t*>(C), sl.nv, *below_s, wsum);
  }
  // per distinct value: 2 n_less + n_eq (C32) or n_less | n_eq << 32
  auto twice_rank = [&](int j) -> uint32_t {
    if (C32) return reinterpret_cast<const uint32_t*>(C)[j];
    const uint64_t cn = reinterpret_cast<const uint64_t*>(C)[j];
    return 2u * (uint32_t)cn + (uint32_t)(cn >> 32);
  };
  if (FUSED) {
    // own queries [5][D][S] of day d that fall in this slice -> rank (S6 average).  RB
    // queries per thread in flight: their loads issued together, then their positions
    // found together by the key loop's binary lifting (block-uniform steps, every probe one
    // ds_read_b64 at a constant stride; the PDF_PAD sentinels bound it) instead of a
    // divergent lower_bound per query (round 6: the resolve was 0.93 of the count's 3.93 ms)
    if (sl.nv > 0) {
      const size_t plane = (size_t)a.D * S;
      constexpr int RB = 4;
      const int bd = (int)blockDim.x;
      const char* Lb = reinterpret_cast<const char*>(sl.L);
      const bool shallow = sl.steps <= 6;
      for (int t = 0; t < 5; ++t) {
        if (a.rows[t] < 0) continue;  // block-uniform
        const double* qrow = a.q_local + (size_t)t * plane + (size_t)d * S;
        const size_t orow = (size_t)a.rows[t] * plane + (size_t)d * S;
        for (int s0 = threadIdx.x; s0 < S; s0 += RB * bd) {
          uint64_t key[RB];
          bool in[RB];
          uint32_t jb[RB];
#pragma unroll
          for (int k = 0; k < RB; ++k) {
            const int s = s0 + k * bd;
            const double q = s < S ? qrow[s] : __builtin_nan("");
            key[k] = ord64(q);
            // NaN: no level passed (null) or absent; outside (L0, qmax]: another slice
            // owns the value's first copy
            in[k] = !__builtin_isnan(q) && key[k] > sl.L0 && key[k] <= sl.qmax;
          }
#pragma unroll
          for (int k = 0; k < RB; ++k) {
            const bool g = in[k] && key[k] > sl.qmin;
            jb[k] = g ? (uint32_t)sl.T[(key[k] - sl.qmin) >> sl.sh] << 3 : 0u;  // L[jb / 8] < key
          }
          if (shallow) {
#pragma unroll
            for (int st = 5; st >= 0; --st) {
              if (st < sl.steps) {
                const uint32_t bb = 8u << st;
                uint64_t x[RB];
#pragma unroll
                for (int k = 0; k < RB; ++k) x[k] = *reinterpret_cast<const uint64_t*>(Lb + jb[k] + bb);
#pragma unroll
                for (int k = 0; k < RB; ++k) jb[k] += x[k] < key[k] ? bb : 0u;
              }
            }
          } else {
#pragma unroll
            for (int k = 0; k < RB; ++k) {
              if (!in[k]) continue;
              int lo, hi;
              sl.range(key[k], lo, hi);
              jb[k] = (uint32_t)lower_bound_u64(sl.L + 1, lo, hi, key[k]) << 3;
            }
          }
#pragma unroll
          for (int k = 0; k < RB; ++k) {
            if (!in[k]) continue;
            const uint32_t c2 = twice_rank((int)(jb[k] >> 3));  // L1[jb / 8] >= key
            const size_t o = orow + (size_t)(s0 + k * bd);
            a.val[o] = ((double)c2 + 1.0) * 0.5;
            a.state[o] = MFF_STATE_VALUE;
          }
        }
      }
    }
  } else {
    // per sorted position: the counts of its distinct value (positions holding Q[P0-1]
    // or NaN are never looked up); one word per position, 2 n_less + n_eq: the average
    // rank n_less + (n_eq + 1) / 2 = (2 n_less + n_eq + 1) / 2 is linear in it, so the
    // ranks' words simply add up
    uint32_t* out = a.counts + (size_t)qd * a.M + P0;
    for (int i = threadIdx.x; i < nq; i += blockDim.x) {
      const uint64_t x = Q[P0 + i];
      uint32_t c2 = 0u;
      if (x > sl.L0 && x <= sl.qmax) {
        int lo, hi;
        sl.range(x, lo, hi);
        c2 = twice_rank(lower_bound_u64(L + 1, lo, hi, x));
      }
      // frame: every day adds its keys' words to the one list's counters (the words
      // are linear in the rank, so the days' sum is the frame-wide 2 n_less + n_eq)
      if (a.frame) {
        if (c2 != 0u) atomicAdd(out + i, c2);
      } else {
        out[i] = c2;
      }
    }
  }
  __syncthreads();  // the LDS is reused by the next slice count of this workgroup
  return true;
}

// One workgroup per (day, slice of <= Mz sorted queries).  a.packed: u32 counters (the
// slice twice as long as with u64 ones: every slice re-reads the day's level list, the
// kernel's dominant traffic), a slice whose n_eq field overflowed recounted as two halves
// with u64 counters.
template <bool FUSED>
__global__ __launch_bounds__(PDF_CT) void k_pdf_count(PdfArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t below_s, inw_s, one_s;
  __shared__ int occ_s;
  // XCD-aware block order: hardware dispatches block b to XCD b % 8; the Z slices of a
  // day get consecutive logical ids on one XCD (they share the day's level list in L2)
  const int per_xcd = gridDim.x >> 3;  // host pads the grid to a multiple of 8
  const int lid = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  const int dd = lid / a.Z, z = lid % a.Z;
  if (dd >= a.nd) return;
  const int d = a.d0 + dd;
  int P0 = z * a.Mz, P1 = min(a.M, P0 + a.Mz);
  uint64_t lo_floor = 0ull;
  if (a.kslice) {
    // the queries below the split key [0, PK) and the others [PK, M), each cut into equal
    // slices of at most Mz: a slice then reads one of the day's two level lists
    __shared__ int pk_s;
    const uint64_t ksplit = pdf_split_key(a.lvl_count, a.D);
    if (threadIdx.x < 64) {
      const int pk = wave_lower_bound(a.q_sorted + (size_t)dd * a.M, a.M, ksplit);
      if (threadIdx.x == 0) pk_s = pk;
    }
    __syncthreads();
    const int PK = pk_s;
    const int zA = (PK + a.Mz - 1) / a.Mz, zB = (a.M - PK + a.Mz - 1) / a.Mz;
    if (z >= zA + zB) return;  // block-uniform
    if (z < zA) {
      const int len = (PK + zA - 1) / zA;
      P0 = z * len;
      P1 = min(PK, P0 + len);
    } else {
      const int len = (a.M - PK + zB - 1) / zB;
      P0 = PK + (z - zA) * len;
      P1 = min(a.M, P0 + len);
      lo_floor = ksplit - 1ull;
    }
  }
  if (a.packed) {
    if (!pdf_count_slice<FUSED, true>(a, d, dd, P0, P1, a.Mz, smem, wsum, &below_s, &inw_s, &one_s, &occ_s,
                                      lo_floor)) {
      __syncthreads();
      const int mid = P0 + (P1 - P0 + 1) / 2;
      pdf_count_slice<FUSED, false>(a, d, dd, P0, mid, mid - P0, smem, wsum, &below_s, &inw_s, &one_s, &occ_s,
                                    lo_floor);
      pdf_count_slice<FUSED, false>(a, d, dd, mid, P1, P1 - mid, smem, wsum, &below_s, &inw_s, &one_s, &occ_s,
                                    lo_floor);
    }
  } else {
    pdf_count_slice<FUSED, false>(a, d, dd, P0, P1, a.Mz, smem, wsum, &below_s, &inw_s, &one_s, &occ_s,
                                  lo_floor);
  }
}

// multi-rank finalize: counts summed over ranks -> per (day, slice) LDS lookup of own queries
__global__ __launch_bounds__(PDF_CT) void k_pdf_finalize(PdfArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int occ_s;
  __shared__ uint32_t wsum[16];
  const int dd = blockIdx.x / a.Z, z = blockIdx.x % a.Z;
  if (dd >= a.nd) return;
  const int d = a.d0 + dd;
  const uint64_t* Q = a.q_sorted + (size_t)dd * a.M;
  const int P0 = z * a.Mz, P1 = min(a.M, P0 + a.Mz);
  uint64_t* L = reinterpret_cast<uint64_t*>(smem);
  uint64_t* C = L + a.Mz + 1 + PDF_PAD;
  uint16_t* T = reinterpret_cast<uint16_t*>(C + a.Mz);
  const PdfSlice sl = pdf_slice_setup(Q, a.M, P0, P1, L, C, T, wsum, &occ_s);
  // counts of each distinct value, from its first sorted position
  const uint32_t* cn = a.counts + (size_t)dd * a.M + P0;
  for (int i = threadIdx.x; i < P1 - P0; i += blockDim.x) {
    const uint64_t x = Q[P0 + i];
    const uint64_t xp = i > 0 ? Q[P0 + i - 1] : sl.L0;
    if (x > sl.L0 && x <= sl.qmax && x != xp) {
      int lo, hi;
      sl.range(x, lo, hi);
      // c = 2 n_less + n_eq summed over ranks -> (c >> 1, c & 1): same average rank (c + 1) / 2
      const uint32_t c = cn[i];
      C[lower_bound_u64(L + 1, lo, hi, x)] = (uint64_t)(c >> 1) | ((uint64_t)(c & 1u) << 32);
    }
  }
  __syncthreads();
  pdf_slice_resolve(sl, C, a.q_local, a.S, a.D, d, a.rows, a.val, a.state);
}

// multi-rank, day-owner side: the counts of day d's sorted list (summed over ranks) at
// each query's first sorted position, written in the queries' origin layout
// [R][5][nd][S_all] (the all_to_all receive buffer of mff_pdf_sort), so one all_to_all
// returns every rank the counts of its own queries.  One workgroup per (day, slice of
// sorted positions), as the count: the slice's distinct values, a bucket table and their
// count words in LDS (pdf_slice_setup with cfill), then every origin query of the day
// finds its value by the binary lifting of the count's key loop (round 6; the thread per
// query with a global binary search over the day's list and 64-bit index divisions took
// 0.66 ms for one rank's 313 days at N = 8, bench extras rank_share_n8).  Slice 0 also
// writes 0 for the NaN queries (no level passed, or an absent stock-day).
__global__ __launch_bounds__(PDF_CT) void k_pdf_origin_lds(const double* q_all, int RT, int S, int D, int d0, int nd,
                                                          const uint64_t* q_sorted, const uint32_t* counts, int M,
                                                          int Z, int Mz, uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int occ_s;
  __shared__ uint32_t wsum[16];
  const int dd = blockIdx.x / Z, z = blockIdx.x % Z;
  if (dd >= nd) return;
  const uint64_t* Q = q_sorted + (size_t)dd * M;
  const int P0 = z * Mz, P1 = min(M, P0 + Mz);
  if (P0 >= P1) return;
  uint64_t* L = reinterpret_cast<uint64_t*>(smem);
  uint32_t* C = reinterpret_cast<uint32_t*>(L + Mz + 1 + PDF_PAD);
  uint16_t* T = reinterpret_cast<uint16_t*>(C + Mz);
  const PdfSlice sl = pdf_slice_setup(Q, M, P0, P1, L, C, T, wsum, &occ_s, 0ull, counts + (size_t)dd * M + P0);
  const char* Lb = reinterpret_cast<const char*>(sl.L);
  const bool shallow = sl.steps <= 6;
  constexpr int RB = 4;
  const int bd = (int)blockDim.x;
  for (int rt = 0; rt < RT; ++rt) {
    const double* qrow = q_all + ((size_t)rt * D + d0 + dd) * S;
    uint32_t* orow = out + ((size_t)rt * nd + dd) * S;
    for (int s0 = threadIdx.x; s0 < S; s0 += RB * bd) {
      uint64_t key[RB];
      bool in[RB], nan_[RB];
      uint32_t jb[RB];
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        const int s = s0 + k * bd;
        const double q = s < S ? qrow[s] : 0.0;
        nan_[k] = s < S && __builtin_isnan(q);
        key[k] = ord64(q);
        in[k] = s < S && !nan_[k] && sl.nv > 0 && key[k] > sl.L0 && key[k] <= sl.qmax;
      }
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        const bool g = in[k] && key[k] > sl.qmin;
        jb[k] = g ? (uint32_t)sl.T[(key[k] - sl.qmin) >> sl.sh] << 3 : 0u;
      }
      if (shallow) {
#pragma unroll
        for (int st = 5; st >= 0; --st) {
          if (st < sl.steps) {
            const uint32_t bb = 8u << st;
            uint64_t x[RB];
#pragma unroll
            for (int k = 0; k < RB; ++k) x[k] = *reinterpret_cast<const uint64_t*>(Lb + jb[k] + bb);
#pragma unroll
            for (int k = 0; k < RB; ++k) jb[k] += x[k] < key[k] ? bb : 0u;
          }
        }
      } else {
#pragma unroll
        for (int k = 0; k < RB; ++k) {
          if (!in[k]) continue;
          int lo, hi;
          sl.range(key[k], lo, hi);
          jb[k] = (uint32_t)lower_bound_u64(sl.L + 1, lo, hi, key[k]) << 3;
        }
      }
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        if (in[k]) orow[s0 + k * bd] = C[jb[k] >> 3];
        else if (nan_[k] && z == 0) orow[s0 + k * bd] = 0u;
      }
    }
  }
}

// own queries [5][D][S] with their counts in the same layout (2 n_less + n_eq summed over
// ranks) -> average rank (c + 1) / 2 (S6); NaN queries keep stage 1's null / absent
__global__ __launch_bounds__(256) void k_pdf_finalize_own(const double* q, const uint32_t* cnt, int S, int D,
                                                           Rows5 rows, double* val, uint8_t* state) {
  const size_t plane = (size_t)D * S;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= 5 * plane) return;
  const int t = (int)(i / plane);
  const size_t j = i - (size_t)t * plane;
  if (rows.r[t] < 0 || __builtin_isnan(q[i])) return;
  const size_t o = (size_t)rows.r[t] * plane + j;
  val[o] = ((double)cnt[i] + 1.0) * 0.5;
  state[o] = MFF_STATE_VALUE;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// the learned split key (per device, allocated on first use and cleared on the stream)
static PdfLearn* g_learn[64];
static std::mutex g_learn_mu;
static PdfLearn* pdf_learn_state(hipStream_t st) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    set_error("pdf_learn_state: no device");
    return nullptr;
  }
  std::lock_guard<std::mutex> lk(g_learn_mu);
  if (!g_learn[dev]) {
    PdfLearn* p = nullptr;
    if (hipMalloc(&p, sizeof(PdfLearn)) != hipSuccess || hipMemsetAsync(p, 0, sizeof(PdfLearn), st) != hipSuccess) {
      set_error("pdf_learn_state: allocation failed");
      return nullptr;
    }
    g_learn[dev] = p;
  }
  return g_learn[dev];
}

// every 16th day of the call: its median query (as a ratio) into the learned key's sum
// (one wave per sampled day, after the count)
__global__ __launch_bounds__(64) void k_pdf_learn(const uint64_t* q_sorted, int M, PdfLearn* s) {
  const uint64_t* Qd = q_sorted + (size_t)blockIdx.x * 16 * M;
  const int nvalid = wave_lower_bound(Qd, M, ~0ull);  // NaN queries sort last
  if (nvalid > 0 && threadIdx.x == 0) {
    atomicAdd(&s->sum, unord64(Qd[(nvalid - 1) / 2]));
    atomicAdd(&s->n, 1u);
  }
}

// one thread: this pass's split key = the mean of the medians gathered since the last
// pass start (as a ratio, then its key), or the key in use, or 1.0 before any
__global__ void k_pdf_split_init(PdfLearn* s, uint64_t* hdr_key) {
  if (s->key == 0ull) s->key = PDF_KSPLIT0;
  if (s->n != 0u) {
    s->key = ord64(s->sum / (double)s->n);
    s->sum = 0.0;
    s->n = 0u;
  }
  *hdr_key = s->key;
}

int pdf_split_init(uint32_t* lvl_count, int D, hipStream_t st) {
  PdfLearn* s = pdf_learn_state(st);
  if (!s) return -2;
  uint64_t* hdr = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(lvl_count) + pdf_koff(D));
  hipLaunchKernelGGL(k_pdf_split_init, dim3(1), dim3(1), 0, st, s, hdr);
  MFF_LAUNCH_CHECK();
  return 0;
}

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

static void pdf_slices(int M, int& Z, int& Mz, size_t& lds, bool packed) {
  Z = (M + (packed ? PDF_ZQ32 : PDF_ZQ) - 1) / (packed ? PDF_ZQ32 : PDF_ZQ);
  Mz = (M + Z - 1) / Z;
  // packed: L u64 + C u32 (the u64 recount's half slices fit the same bytes)
  lds = (size_t)(Mz + 1 + PDF_PAD) * 8 + (size_t)Mz * (packed ? 4 : 8) + (size_t)(PDF_NBK + 1) * 2;
}

static int pdf_launch(PdfArgs& a, const uint64_t* q_sorted, int M, hipStream_t st, int mode) {
  size_t lds;
  // packed counters for the count phases while a slice's weight (<= 240 bars per stock of
  // this rank) fits the n_less field (MFF_PDF_U64: the u64 counters always, a test hook)
  a.packed = mode != 2 && (long long)NBAR * a.S < (1ll << PDF_LB) && getenv("MFF_PDF_U64") == nullptr;
  pdf_slices(M, a.Z, a.Mz, lds, a.packed);
  // one rank, one day per sorted list: slices aligned at PDF_KSPLIT (one more slot per day
  // for the split)
  a.kslice = mode != 2 && a.packed && !a.frame;
  if (a.kslice) {
    a.learn = pdf_learn_state(st);
    if (!a.learn) return -2;
    a.Mz = PDF_KCAP;
    a.Z = (M + PDF_KCAP - 1) / PDF_KCAP + 1;  // + 1: the split falls inside a slice's span
    lds = (size_t)(PDF_KCAP + 1 + PDF_PAD) * 8 + (size_t)PDF_KCAP * 4 + (size_t)(PDF_NBK + 1) * 2;
  }
  a.q_sorted = q_sorted;
  a.M = M;
  if (mode == 2) {
    const long long nblk = (long long)a.Z * a.nd;
    MFF_REQUIRE(nblk < (1ll << 31), "mff_pdf_finalize: too many days in one call");
    hipLaunchKernelGGL(k_pdf_finalize, dim3((unsigned)nblk), dim3(PDF_CT), lds, st, a);
  } else {
    const long long nblk = ((long long)a.Z * a.nd + 7) / 8 * 8;
    MFF_REQUIRE(nblk < (1ll << 31), "mff_pdf_count: too many days in one call");
    if (mode == 1)
      hipLaunchKernelGGL(k_pdf_count<true>, dim3((unsigned)nblk), dim3(PDF_CT), lds, st, a);
    else
      hipLaunchKernelGGL(k_pdf_count<false>, dim3((unsigned)nblk), dim3(PDF_CT), lds, st, a);
    if (a.kslice) {  // (the sharded count of the full day lists learns the same key on every rank)
      MFF_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_pdf_learn, dim3((unsigned)((a.nd + 15) / 16)), dim3(64), 0, st, q_sorted, M, a.learn);
    }
  }
  MFF_LAUNCH_CHECK();
  return 0;
}

static void pdf_levels_args(PdfArgs& a, const void* pdf_levels, int S, int D) {
  size_t ok, ow;
  pdf_levels_split(S, D, &ok, &ow);
  const char* base = reinterpret_cast<const char*>(pdf_levels);
  a.lvl_count = reinterpret_cast<const uint32_t*>(base);
  a.lvl_key = reinterpret_cast<const uint64_t*>(base + ok);
  a.lvl_w = reinterpret_cast<const uint8_t*>(base + ow);
  a.cap = pdf_day_cap(S);
}

int mff_pdf_count(const void* pdf_levels, int S_loc, int D, int d0, int nd,
                  const uint64_t* q_sorted, int M, uint32_t* counts, void* workspace, void* stream) {
  clear_error();
  MFF_REQUIRE(S_loc > 0 && D > 0 && nd > 0 && d0 >= 0 && d0 + nd <= D && M > 0,
              "mff_pdf_count: bad sizes");
  MFF_REQUIRE(M <= PDF_MAXM, "mff_pdf_count: %d queries per day exceed %d (R*5*S_loc)", M, PDF_MAXM);
  MFF_REQUIRE(pdf_levels && q_sorted && counts && workspace, "mff_pdf_count: NULL buffer");
  PdfArgs a;
  memset(&a, 0, sizeof(a));
  pdf_levels_args(a, pdf_levels, S_loc, D);
  a.counts = counts;
  a.S = S_loc; a.D = D; a.d0 = d0; a.nd = nd;
  return pdf_launch(a, q_sorted, M, as_stream(stream), 0);
}

int mff_pdf_count_frame(const void* pdf_levels, int S, int D, const uint64_t* q_sorted, int M,
                        uint32_t* counts, void* stream) {
  clear_error();
  MFF_REQUIRE(S > 0 && D > 0 && M > 0, "mff_pdf_count_frame: bad sizes S=%d D=%d M=%d", S, D, M);
  MFF_REQUIRE(M <= PDF_MAXM, "mff_pdf_count_frame: %d queries exceed %d", M, PDF_MAXM);
  // 2 n_less + n_eq over every key of the frame (<= 240 per stock-day) must fit u32
  MFF_REQUIRE((long long)NBAR * S * D < (1ll << 31), "mff_pdf_count_frame: frame of %d x %d stock-days too large",
              D, S);
  MFF_REQUIRE(pdf_levels && q_sorted && counts, "mff_pdf_count_frame: NULL buffer");
  PdfArgs a;
  memset(&a, 0, sizeof(a));
  pdf_levels_args(a, pdf_levels, S, D);
  a.counts = counts;
  a.S = S; a.D = D; a.d0 = 0; a.nd = D;
  a.frame = 1;
  return pdf_launch(a, q_sorted, M, as_stream(stream), 0);
}

int mff_pdf_finalize(const double* q_local, const uint64_t* q_sorted, const uint32_t* counts, int S_loc,
                     int D, int d0, int nd, int M, const int32_t* pdf_rows, double* val, uint8_t* state,
                     void* stream) {
  clear_error();
  MFF_REQUIRE(S_loc > 0 && D > 0 && nd > 0 && d0 >= 0 && d0 + nd <= D && M > 0 && M <= PDF_MAXM,
              "mff_pdf_finalize: bad sizes");
  MFF_REQUIRE(q_local && q_sorted && counts && pdf_rows && val && state, "mff_pdf_finalize: NULL buffer");
  PdfArgs a;
  memset(&a, 0, sizeof(a));
  a.counts = const_cast<uint32_t*>(counts);
  a.q_local = q_local; a.val = val; a.state = state;
  for (int t = 0; t < 5; ++t) a.rows[t] = pdf_rows[t];
  a.S = S_loc; a.D = D; a.d0 = d0; a.nd = nd;
  return pdf_launch(a, q_sorted, M, as_stream(stream), 2);
}

int mff_pdf_origin_counts(const double* q_all, int R, int S_all, int D, int d0, int nd,
                          const uint64_t* q_sorted, const uint32_t* counts, int M, uint32_t* out,
                          void* stream) {
  clear_error();
  MFF_REQUIRE(R >= 1 && S_all > 0 && D > 0 && nd > 0 && d0 >= 0 && d0 + nd <= D && M > 0 && M <= PDF_MAXM,
              "mff_pdf_origin_counts: bad sizes R=%d S=%d D=%d d0=%d nd=%d M=%d", R, S_all, D, d0, nd, M);
  MFF_REQUIRE(q_all && q_sorted && counts && out, "mff_pdf_origin_counts: NULL buffer");
  int Z, Mz;
  size_t lds;
  pdf_slices(M, Z, Mz, lds, true);
  hipLaunchKernelGGL(k_pdf_origin_lds, dim3((unsigned)((long long)Z * nd)), dim3(PDF_CT), lds, as_stream(stream),
                     q_all, R * 5, S_all, D, d0, nd, q_sorted, counts, M, Z, Mz, out);
  MFF_LAUNCH_CHECK();
  return 0;
}

int mff_pdf_finalize_own(const double* q_local, const uint32_t* own_counts, int S_loc, int D,
                         const int32_t* pdf_rows, double* val, uint8_t* state, void* stream) {
  clear_error();
  MFF_REQUIRE(S_loc > 0 && D > 0, "mff_pdf_finalize_own: bad sizes S=%d D=%d", S_loc, D);
  MFF_REQUIRE(q_local && own_counts && pdf_rows && val && state, "mff_pdf_finalize_own: NULL buffer");
  Rows5 rows;
  for (int t = 0; t < 5; ++t) rows.r[t] = pdf_rows[t];
  const size_t n = (size_t)5 * D * S_loc;
  hipLaunchKernelGGL(k_pdf_finalize_own, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream),
                     q_local, own_counts, S_loc, D, rows, val, state);
  MFF_LAUNCH_CHECK();
  return 0;
}

int mff_pdf_rank_local(const void* pdf_levels, const double* q_local, int S, int D,
                       int d0, int nd, const uint64_t* q_sorted, int M, const int32_t* pdf_rows,
                       double* val, uint8_t* state, void* stream) {
  clear_error();
  MFF_REQUIRE(S > 0 && D > 0 && nd > 0 && d0 >= 0 && d0 + nd <= D && M > 0 && M <= PDF_MAXM,
              "mff_pdf_rank_local: bad sizes");
  MFF_REQUIRE(pdf_levels && q_local && q_sorted && pdf_rows && val && state,
              "mff_pdf_rank_local: NULL buffer");
  PdfArgs a;
  memset(&a, 0, sizeof(a));
  pdf_levels_args(a, pdf_levels, S, D);
  a.q_local = q_local; a.val = val; a.state = state;
  for (int t = 0; t < 5; ++t) a.rows[t] = pdf_rows[t];
  a.S = S; a.D = D; a.d0 = d0; a.nd = nd;
  return pdf_launch(a, q_sorted, M, as_stream(stream), 1);
}

}  // extern "C"
