// mff_stage1g.hip — stage 1, 16 lanes per stock-day (the default path).
//
// A wave64 computes FOUR stock-days at once, one per DPP row of 16 lanes; lane gi of a
// row owns bars 16*gi .. 16*gi+15 of every plane (four float4 loads per plane, all
// planes in flight together).  Per-lane work is a straight loop over 16 bars with
// carries (previous present bar, running prefix sums); everything that crosses lanes
// is a 4-step DPP row operation (mff_group.h).  Each group keeps its 58 results spread
// over its 16 lanes (factor f lives in lane f%16, register f/16) and the lanes store
// them in parallel at the end (val[row][d][s]: the 16 stocks a block handles per step
// are consecutive, so each 128-byte line is filled by one block within one step).
//
// Per family (reference lines CM:<n>, semantics S*/C* in DESIGN.md §4):
//  SEG   bar tests + DPP broadcasts of session endpoints             CM:10-90
//  OLS   exact shifted prefix sums; window start (t-50) fetched from lane gi-3
//        (slot k-2) or gi-4 (k<2) with one bpermute per quantity; betas through LDS
//        for the two-pass std                                          CM:93-376
//  ORD   bitonic sort of 256 volume keys (16 per lane), thresholds by index CM:379-480
//  MOM   one pass of shifted raw sums (shift = a member of the set, so identical
//        values give exact zeros, C3); up/down subsets use min == max     CM:483-729
//  SUM/TRD masked sums, one reciprocal 1/v per bar                     CM:732-831,1203-1406
//  CORR  six Pearson sums, shifts = each variant's first pair           CM:834-932
//  LVL/PDF close levels by a bitonic sort of (close descending, volume) keys: a level is
//        a run of equal closes, its volume an exact u32 segment sum; doc_pdf's
//        threshold by the exact comparison 20*cum > k*sum(v).  Stock-days that hit an
//        exact doc_pdf tie or carry non-integral volume are appended to a list that the
//        wave64 kernel (mff_stage1.hip) finishes.                       CM:935-1138
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "../../include/mff.h"
#include "mff_group.h"
#include "mff_fmath.h"
#include "mff_stats.h"
#include "mff_internal.h"

namespace mff {

int launch_w64(const float* const fld[5], const uint32_t* valid, int S, int D, const int32_t* ids, int nf,
               double* val, uint8_t* state, double* pdfq, const int* list, const int* list_count,
               uint32_t fam_mask, int list_grid, hipStream_t st, uint32_t* lvl_count = nullptr,
               uint64_t* lvl_key = nullptr, uint8_t* lvl_w = nullptr);
int launch_serial(const float* const fld[5], const uint32_t* valid, int S, int D, const int8_t* row,
                  uint32_t fam, double* val, uint8_t* state, const uint32_t* ord_th, hipStream_t st);

// 16 stock-days of one day per block iteration; kGIter iterations per block.  One:
// with a loop, everything derived from the lane ids (lane masks, offsets, the scratch
// address) is hoisted out of it and stays live across it -- the ORD + LVL launch then
// took 128 VGPRs (4 waves per SIMD) against 91 (5 waves) without; measured 15.5 against
// 16.6 ms in the pass (profiles/r05/ab_giter.txt)
constexpr int kGIter = 1;
// waves per SIMD the group kernel is built for (its LDS allows 5 at 31.7 KB per block)
constexpr int kGWaves = 5;
// blocks of the exact-list launch (grid-stride over the device-side list count)
constexpr int kExactGrid = 1024;

namespace g16 {

constexpr int NB = 256;  // OLS betas per stock-day (LDS, 8 B each)

struct GArgs {
  const float* fld[5];  // open high low close: fp32; [4] volume: u32 shares (include/mff.h)
  const uint32_t* mask;
  double* val;
  uint8_t* state;
  double* pdfq;
  // doc_pdf level side channel (mff_pdf_levels_bytes), or null: per day, a flat list of
  // (key c_last/c_level as ord64, bars at the level) over every stock-day's levels, in
  // no particular order; lvl_count[d] = entries (appended by atomic reservation)
  uint32_t* lvl_count;
  uint64_t* lvl_key;
  uint8_t* lvl_w;
  int* fb_list;
  int* fb_count;
  uint32_t fam_exact;  // families whose non-fast stock-days go to the exact list
  uint32_t* ord_th;    // ORD volume thresholds [3][D][S] (top-50 min, top-20 min, bottom-50 max)
                       // for the serial returns kernel's products, or null
  int S, D;
  uint32_t fam;
  int8_t row[NF];
};

// ---- result registers: factor f of the group lives in lane f%16, register f/16
struct Res {
  double r[4];
  uint32_t st;
  __device__ __forceinline__ void put(int f, double x, uint32_t s) {
    if (gi() == (f & 15)) {
      const int q = f >> 4;
      r[q] = x;
      st = (st & ~(0xFFu << (8 * q))) | (s << (8 * q));
    }
  }
  __device__ __forceinline__ void val(int f, double x) { put(f, x, MFF_STATE_VALUE); }
  __device__ __forceinline__ void null(int f) { put(f, 0.0, MFF_STATE_NULL); }
};

__device__ __forceinline__ double gmin_d(double x) {
  x = fmin(x, dpp_d<QP_XOR1>(x));
  x = fmin(x, dpp_d<QP_XOR2>(x));
  x = fmin(x, dpp_d<ROW_HALF_MIRROR>(x));
  x = fmin(x, dpp_d<ROW_MIRROR>(x));
  return x;
}
__device__ __forceinline__ double gmax_d(double x) {
  x = fmax(x, dpp_d<QP_XOR1>(x));
  x = fmax(x, dpp_d<QP_XOR2>(x));
  x = fmax(x, dpp_d<ROW_HALF_MIRROR>(x));
  x = fmax(x, dpp_d<ROW_MIRROR>(x));
  return x;
}

// a register value the optimiser must treat as new (no instruction emitted)
__device__ __forceinline__ void opaque(float& x) { asm("" : "+v"(x)); }
__device__ __forceinline__ void opaque(double& x) { asm("" : "+v"(x)); }
__device__ __forceinline__ void opaque(uint32_t& x) { asm("" : "+v"(x)); }
// every section starts from fresh names for the planes it reads, so the f32->f64
// conversions and quotients of one section are recomputed, not kept live (CSE) into
// the next one
template <typename T>
__device__ __forceinline__ void fresh(T (&x)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) opaque(x[k]);
}

__device__ __forceinline__ void lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t xor_lane(uint32_t x, int lj) { return (uint32_t)__shfl_xor((int)x, lj, 16); }
__device__ __forceinline__ uint64_t xor_lane(uint64_t x, int lj) {
  const uint32_t lo = xor_lane((uint32_t)x, lj), hi = xor_lane((uint32_t)(x >> 32), lj);
  return ((uint64_t)hi << 32) | lo;
}

// ascending bitonic sort of the group's 256 keys (bar order e = 16*gi + k)
template <typename T>
__device__ __forceinline__ void gsort256(T (&a)[K]) {
  const int g = gi();
#pragma unroll
  for (int size = 2; size <= 256; size <<= 1) {
#pragma unroll
    for (int j = size >> 1; j > 0; j >>= 1) {
      if (j >= 16) {
        const int lj = j >> 4;
        const bool lower = (g & lj) == 0;
        const bool up = ((16 * g) & size) == 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const T p = xor_lane(a[k], lj);
          const T mn = a[k] < p ? a[k] : p, mx = a[k] < p ? p : a[k];
          a[k] = (lower == up) ? mn : mx;
        }
      } else {
#pragma unroll
        for (int k = 0; k < K; ++k) {
          if ((k & j) == 0) {
            const bool up = ((16 * g + k) & size) == 0;
            const T x = a[k], y = a[k | j];
            const T mn = x < y ? x : y, mx = x < y ? y : x;
            a[k] = up ? mn : mx;
            a[k | j] = up ? mx : mn;
          }
        }
      }
    }
  }
}

// Family groups of the 16-lane kernel, one instantiation each: the families that need
// order statistics (sorts).  Everything else (SEG, OLS, MOM*, SUM*, CORR, TRD) runs one
// lane per stock-day in mff_stage1s.hip; G_HL (OLS, MOMH) stays instantiable here for
// the family-cost tools.  A group's registers
// are allocated for that group alone; the planes a group reads are re-read by the next
// launch, which costs little here: the stage is VALU bound.
[[maybe_unused]] constexpr uint32_t G_HL = F_OLS | F_MOMH;  // high, low
constexpr uint32_t G_ORD = F_ORD | F_ORDV;   // volume (thresholds; the products are serial)
constexpr uint32_t G_LVL = F_LVL | F_PDF;    // close, volume
constexpr uint32_t kGroups[2] = {G_ORD, G_LVL};
// both sorted groups in one launch: the volume plane is read once for the two sorts
constexpr uint32_t G_OL = G_ORD | G_LVL;

template <uint32_t SET>
// (256, 5): at most 102 VGPRs, five waves per SIMD
__global__ __launch_bounds__(256, kGWaves) void k_stage1g(GArgs a) {
  // 2 KB per group plus 64 B of padding: the four groups of a wave start 16 banks apart,
  // so a store of 16 consecutive words per group covers the 64 banks once
  // per group: the sorted families need 2 x 240 words (level cumulative volumes and
  // close words; the 256-word key / volume images fit inside), the OLS betas 256 doubles
  constexpr int SW = (SET & F_OLS) ? 2 * NB : 2 * NBAR;  // words
  __shared__ __attribute__((aligned(16))) uint64_t scratch[16][SW / 2 + 8];
  const int lane = lane_id();
  const int wave = threadIdx.x >> 6;
  const int grp = lane >> 4;
  const int g = gi();
  const int gb = gbase();
  uint64_t* scr = scratch[wave * 4 + grp];
  double* scr_d = reinterpret_cast<double*>(scr);
  const uint32_t fam = a.fam & SET;
  const int ntile = (a.S + 16 * kGIter - 1) / (16 * kGIter);
  const int d = blockIdx.x / ntile;
  const int s0 = (blockIdx.x % ntile) * (16 * kGIter);
  const size_t plane = (size_t)a.D * a.S;

  for (int it = 0; it < kGIter; ++it) {
    const int s = s0 + it * 16 + wave * 4 + grp;
    const bool act = s < a.S;
    const size_t sd = (size_t)d * a.S + (act ? s : 0);
    const bool ln = act && g < 15;  // lane holds bars

    uint32_t pb = 0;
    if (ln) {
      const uint32_t w = a.mask[sd * 8 + (g >> 1)];
      pb = (w >> (16 * (g & 1))) & 0xFFFFu;
    }
    const int n = gcount(pb);
    Res R;
    R.r[0] = R.r[1] = R.r[2] = R.r[3] = 0.0;
    R.st = 0u;
    double qv = qnan();  // lane t < 5: doc_pdf query t (the level close ratio)
    // doc_pdf level list of this group's stock-day (appended after the result stores):
    // level count, last close, close-word base (the levels themselves stay in scratch)
    uint32_t emitL = 0u, emitB = 0u;
    float emitC = 1.0f;

    if (n > 0) {
      // ---------------------------------------------------------------- loads
      float o[K], h[K], lo[K], c[K];
      uint32_t v[K];  // volume (u32 shares)
      auto load = [&](int f, float (&x)[K], float dflt) {
        if (ln) {
          const float4* p4 = reinterpret_cast<const float4*>(a.fld[f] + sd * NBAR + 16 * g);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 t = p4[q];
            x[4 * q + 0] = t.x; x[4 * q + 1] = t.y; x[4 * q + 2] = t.z; x[4 * q + 3] = t.w;
          }
        } else {
#pragma unroll
          for (int k = 0; k < K; ++k) x[k] = dflt;
        }
      };
      constexpr uint32_t needO = F_SEG | F_MOMR | F_TRD;
      constexpr uint32_t needHL = F_OLS | F_MOMH;
      constexpr uint32_t needC = F_SEG | F_MOMR | F_SUMC | F_CORR | F_LVL | F_PDF | F_TRD;
      constexpr uint32_t needV = F_ORD | F_MOMV | F_SUMC | F_SUMV | F_CORR | F_LVL | F_PDF | F_ORDV | F_TRD;
      // a field is loaded only for families the field table lists for it (mff_internal.h)
      static_assert(!(needO & ~kFieldFams[0]) && !(needHL & ~(kFieldFams[1] & kFieldFams[2])) &&
                        !(needC & ~kFieldFams[3]) && !(needV & ~kFieldFams[4]),
                    "k_stage1g loads a field for a family kFieldFams does not list");
      auto loadv = [&](uint32_t (&x)[K]) {  // volume, absent bars 0
        if (ln) {
          const uint4* p4 = reinterpret_cast<const uint4*>(a.fld[4] + sd * NBAR + 16 * g);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint4 t = p4[q];
            x[4 * q + 0] = t.x; x[4 * q + 1] = t.y; x[4 * q + 2] = t.z; x[4 * q + 3] = t.w;
          }
#pragma unroll
          for (int k = 0; k < K; ++k) x[k] &= present_bits(pb, k);
        } else {
#pragma unroll
          for (int k = 0; k < K; ++k) x[k] = 0u;
        }
      };
      auto sanitize = [&](float (&x)[K], float dflt) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
          if (dflt == 0.0f)  // x + 0 (no -0) where present, the bits of +0 elsewhere
            x[k] = bitsf(fbits(x[k] + 0.0f) & present_bits(pb, k));
          else
            x[k] = ((pb >> k) & 1u) ? x[k] + 0.0f : dflt;
        }
      };
      // phase A planes: high, low (OLS, MOMH); later phases load the others
      if (fam & needHL) {
        load(1, h, 1.0f);
        load(2, lo, 1.0f);
        sanitize(h, 1.0f);
        sanitize(lo, 1.0f);
      }
      const int fb = gfirst(pb), lb = glast(pb);

      // ================================================================ OLS CM:93-376
      if (fam & F_OLS) {
        const double x0a = (double)gval(lo, fb), y0a = (double)gval(h, fb);
        const float ln0 = dpp_f<ROW_SHL + 1>(lo[0]), hn0 = dpp_f<ROW_SHL + 1>(h[0]);
        const uint32_t pn0 = dpp_u<ROW_SHL + 1>(pb) & 1u;
        // lane totals -> carry-in of the prefix sums
        double tx = 0, ty = 0, txx = 0, tyy = 0, txy = 0, q15x = 0, q15y = 0, q15xx = 0, q15yy = 0, q15xy = 0;
        uint32_t tpk = 0, q15pk = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const bool pk = (pb >> k) & 1u;
          const bool pnx = (k < 15) ? ((pb >> (k + 1)) & 1u) : (pn0 != 0u);
          const float lnx = (k < 15) ? lo[k + 1] : ln0, hnx = (k < 15) ? h[k + 1] : hn0;
          const double dx = pk ? (double)lo[k] - x0a : 0.0, dy = pk ? (double)h[k] - y0a : 0.0;
          const uint32_t pkv = (pk ? 1u : 0u) | ((pk && pnx && lo[k] != lnx) ? 0x100u : 0u) |
                               ((pk && pnx && h[k] != hnx) ? 0x10000u : 0u);
          tx += dx; ty += dy; txx += dx * dx; tyy += dy * dy; txy += dx * dy; tpk += pkv;
          if (k == 15) { q15x = dx; q15y = dy; q15xx = dx * dx; q15yy = dy * dy; q15xy = dx * dy; q15pk = pkv; }
        }
        double Rx = gscan_excl(tx), Ry = gscan_excl(ty), Rxx = gscan_excl(txx), Ryy = gscan_excl(tyy),
               Rxy = gscan_excl(txy);
        uint32_t Rpk = gscan_excl_u(tpk);
        // prefix at slots 14 / 15 of this lane (read by lane gi+4 for its k = 0 / 1)
        const double E15x = Rx + tx, E15y = Ry + ty, E15xx = Rxx + txx, E15yy = Ryy + tyy, E15xy = Rxy + txy;
        const uint32_t E15pk = Rpk + tpk;
        // fresh SSA names for the second walk: otherwise the 16 per-bar deviations and
        // their 80 products from the first walk stay live (CSE) and the kernel spills
        double x0 = x0a, y0 = y0a;
        opaque(x0);
        opaque(y0);
#pragma unroll
        for (int k = 0; k < K; ++k) { opaque(lo[k]); opaque(h[k]); }
        double H1x = 0, H1y = 0, H1xx = 0, H1yy = 0, H1xy = 0, H2x = 0, H2y = 0, H2xx = 0, H2yy = 0, H2xy = 0;
        uint32_t H1pk = 0, H2pk = 0;
        double sq = 0, scs = 0, scr = 0, bsum = 0, blast = 0;
        int lastT = -1, wq = 0;
        uint32_t wmask = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const bool pk = (pb >> k) & 1u;
          const bool pnx = (k < 15) ? ((pb >> (k + 1)) & 1u) : (pn0 != 0u);
          const float lnx = (k < 15) ? lo[k + 1] : ln0, hnx = (k < 15) ? h[k + 1] : hn0;
          const double dx = pk ? (double)lo[k] - x0 : 0.0, dy = pk ? (double)h[k] - y0 : 0.0;
          const uint32_t chx = (pk && pnx && lo[k] != lnx) ? 1u : 0u;
          const uint32_t chy = (pk && pnx && h[k] != hnx) ? 1u : 0u;
          Rx += dx; Ry += dy; Rxx += dx * dx; Ryy += dy * dy; Rxy += dx * dy;
          Rpk += (pk ? 1u : 0u) | (chx << 8) | (chy << 16);
          // prefix at t-50: lane gi-3 slot k-2 (its H2 now) or lane gi-4 slot 14/15
          double bx, by, bxx, byy, bxy;
          uint32_t bpk;
          if (k >= 2) {
            const int src = gb + (g >= 3 ? g - 3 : 0);
            bx = bpermd(src, H2x); by = bpermd(src, H2y); bxx = bpermd(src, H2xx);
            byy = bpermd(src, H2yy); bxy = bpermd(src, H2xy); bpk = bpermu(src, H2pk);
            if (g < 3) { bx = by = bxx = byy = bxy = 0.0; bpk = 0u; }
          } else {
            const int src = gb + (g >= 4 ? g - 4 : 0);
            const double ex = (k == 0) ? E15x - q15x : E15x, ey = (k == 0) ? E15y - q15y : E15y;
            const double exx = (k == 0) ? E15xx - q15xx : E15xx, eyy = (k == 0) ? E15yy - q15yy : E15yy;
            const double exy = (k == 0) ? E15xy - q15xy : E15xy;
            const uint32_t epk = (k == 0) ? E15pk - q15pk : E15pk;
            bx = bpermd(src, ex); by = bpermd(src, ey); bxx = bpermd(src, exx);
            byy = bpermd(src, eyy); bxy = bpermd(src, exy); bpk = bpermu(src, epk);
            if (g < 4) { bx = by = bxx = byy = bxy = 0.0; bpk = 0u; }
          }
          H2x = H1x; H2y = H1y; H2xx = H1xx; H2yy = H1yy; H2xy = H1xy; H2pk = H1pk;
          H1x = Rx; H1y = Ry; H1xx = Rxx; H1yy = Ryy; H1xy = Rxy; H1pk = Rpk;
          const int t = 16 * g + k;
          const uint32_t cnt = (Rpk & 0xffu) - (bpk & 0xffu);
          const uint32_t cxw = ((Rpk >> 8) & 0xffu) - ((bpk >> 8) & 0xffu) - chx;
          const uint32_t cyw = ((Rpk >> 16) & 0xffu) - ((bpk >> 16) & 0xffu) - chy;
          const bool okw = ln && t >= 49 && cnt == 50u;
          if (okw) {
            const double Sx = Rx - bx, Sy = Ry - by, Sxx = Rxx - bxx, Syy = Ryy - byy, Sxy = Rxy - bxy;
            const bool cx = cxw == 0u, cy = cyw == 0u;
            const double vx = cx ? 0.0 : (Sxx - Sx * Sx * 0.02) * 0.02;
            const double vy = cy ? 0.0 : (Syy - Sy * Sy * 0.02) * 0.02;
            const double cv = (cx || cy) ? 0.0 : (Sxy - Sx * Sy * 0.02) * 0.02;
            double beta;
            if (vx != 0.0) beta = cv / vx;
            else beta = (y0 + Sy * 0.02) / (x0 + Sx * 0.02);  // mean_y / mean_x
            const double prod = vx * vy;
            if (prod != 0.0) {
              const double ip = 1.0 / prod;
              sq += sqrt(cv) * ip;           // cov**0.5 / (vx*vy)   CM:137
              scs += cv * cv * ip;           // cov**2 / (vx*vy)     CM:212
              scr += cv * sqrt(prod) * ip;   // cov / (vx*vy)**0.5   CM:261
              ++wq;
            }
            scr_d[t] = beta;
            bsum += beta;
            blast = beta;
            lastT = t;
            wmask |= 1u << k;
          }
          // keep the 16 steps in order: hoisting the bpermutes keeps 16 prefixes live
          __builtin_amdgcn_sched_barrier(0);
        }
        const int W = gcount(wmask);
        if (W > 0) {
          lds_fence();
          const int fT = gfirst(wmask), lT = gmax_i(lastT);
          const double b0 = scr_d[fT];
          const double bl = bpermd(gb + (lT >> 4), blast);
          double d1 = 0.0, d2 = 0.0;
#pragma unroll
          for (int k = 0; k < K; ++k)
            if ((wmask >> k) & 1u) {
              const double dd = scr_d[16 * g + k] - b0;
              d1 += dd;
              d2 += dd * dd;
            }
          d1 = gsum(d1);
          d2 = gsum(d2);
          const int Wq = gsum_i(wq);
          const double Sq = gsum(sq), Scs = gsum(scs), Scr = gsum(scr);
          const double bmean = b0 + d1 / (double)W;
          double bstd = 0.0;
          const bool has_std = W >= 2;
          if (has_std) bstd = sqrt((d2 - d1 * d1 / (double)W) / (double)(W - 1));
          (void)bsum;
          if (has_std && tot_ne(bstd, 0.0) && Wq > 0)
            R.val(5, (Sq / (double)Wq) * (bl - bmean) / bstd);  // mmt_ols_qrs CM:156-171
          else
            R.val(5, 0.0);
          R.val(6, Wq > 0 ? Scs / (double)Wq : 0.0);
          R.val(7, Wq > 0 ? Scr / (double)Wq : 0.0);
          R.val(8, bmean);
          R.val(9, (has_std && tot_gt(bstd, 0.0)) ? (bl - bmean) / bstd : bmean);
          lds_fence();
        }
      }

      __builtin_amdgcn_sched_barrier(0);
      // ================================================================ MOMH CM:499-515
      if (fam & F_MOMH) {
        fresh(h);
        fresh(lo);

        const double x0 = (double)gval(h, fb) / (double)gval(lo, fb);
        double s1 = 0, s2 = 0;
#pragma unroll
        for (int k = 0; k < K; ++k)
          if ((pb >> k) & 1u) {
            const double dd = (double)h[k] / (double)lo[k] - x0;
            s1 += dd;
            s2 += dd * dd;
          }
        RawMom m{gsum(s1), gsum(s2), 0, 0, n};
        double sdv;
        if (std1_raw(m, m.s1 == 0.0 && m.s2 == 0.0, sdv)) R.val(15, sdv); else R.null(15);
      }

      __builtin_amdgcn_sched_barrier(0);
      // phase B/C planes: volume, close, open
      double sumv = 0.0;
      if (fam & needV) {
        loadv(v);
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k) t += (double)v[k];
        sumv = gsum(t);
      }
      if (fam & needC) {
        load(3, c, 1.0f);
        // LVL / PDF read closes of present bars only (masked keys, the last present
        // close), so their absent slots need no canonical value
        if (fam & needC & ~(F_LVL | F_PDF)) sanitize(c, 1.0f);
      }
      if (fam & needO) {
        load(0, o, 1.0f);
        sanitize(o, 1.0f);
      }

      // ================================================================ ORD / ORDV sort
      if (fam & (F_ORD | F_ORDV)) {
        fresh(v);

        uint32_t key[K];
#pragma unroll
        for (int k = 0; k < K; ++k) key[k] = v[k] | absent_bits(pb, k);  // v sanitized; < 2^32 - 1
        gsort256u(key);
        // the sorted keys go through the group's LDS scratch (element e = 16 g + k at slot
        // 16 k + g: conflict-free stores), and each lane reads the one element it needs:
        // lanes 0..9 the top ten (n-1-g), lanes 10..12 the three order statistics
        uint32_t* so = reinterpret_cast<uint32_t*>(scr);
#pragma unroll
        for (int k = 0; k < K; ++k) so[16 * k + g] = key[k];
        lds_fence();
        const int e = g < 10 ? n - 1 - g
                    : g == 10 ? (n >= 50 ? n - 50 : 0)    // top_k(50).min()   CM:391-396
                    : g == 11 ? (n >= 20 ? n - 20 : 0)    // top_k(20).min()
                    : (n >= 50 ? 49 : n - 1);             // bottom_k(50).max() CM:417-422
        const uint32_t xe = (e >= 0 && g < 13) ? so[((e & 15) << 4) | (e >> 4)] : 0u;
        lds_fence();  // the LVL section reuses the scratch
        if ((fam & F_ORD) && a.ord_th && g >= 10 && g < 13 && act) {
          const size_t pl = (size_t)a.D * a.S;
          a.ord_th[(size_t)(g - 10) * pl + sd] = xe;
        }
        if (fam & F_ORDV) {
          // the top ten / five elements (fewer when n < 10: e < 0 reads nothing)
          const double t10 = gsum(g < 10 ? (double)xe : 0.0);
          const double t5 = gsum(g < 5 ? (double)xe : 0.0);
          R.val(47, t10 / sumv);  // doc_vol10_ratio
          R.val(48, t5 / sumv);   // doc_vol5_ratio
          R.val(49, t5 / sumv);   // doc_vol50_ratio: top_k(5) [sic CM:1196]
        }
      }

      // ================================================================ RET: MOMR + TRD + ORD products
      if (fam & (F_MOMR | F_TRD)) {
        fresh(c);
        fresh(o);
        fresh(v);

        const double x0 = (double)gval(c, fb) / (double)gval(o, fb) - 1.0;  // first return
        double s1 = 0, s2 = 0, s3 = 0, s4 = 0;
        double u1 = 0, u2 = 0, umn = __builtin_inf(), umx = -__builtin_inf();
        double w1 = 0, w2 = 0, wmn = __builtin_inf(), wmx = -__builtin_inf();
        uint32_t upm = 0, dnm = 0;
        double vT20 = 0, vT50 = 0, rT20 = 0, rT50 = 0, vH20 = 0, vH50 = 0, a20 = 0, n20 = 0, q20 = 0, a50 = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const bool pk = (pb >> k) & 1u;
          const int m = 16 * g + k;
          const double q = (double)c[k] / (double)o[k];  // close / open
          const double r = q - 1.0;                       // close / open - 1
          if (pk) {
            const double dd = r - x0, d2 = dd * dd;
            s1 += dd; s2 += d2; s3 += d2 * dd; s4 += d2 * d2;
            if (tot_gt(r, 0.0)) { upm |= 1u << k; u1 += dd; u2 += d2; umn = fmin(umn, r); umx = fmax(umx, r); }
            if (tot_lt(r, 0.0)) { dnm |= 1u << k; w1 += dd; w2 += d2; wmn = fmin(wmn, r); wmx = fmax(wmx, r); }
            const double vk = (double)v[k];
            if (m >= 220) { vT20 += vk; rT20 += vk * r; }
            if (m >= 190) { vT50 += vk; rT50 += vk * r; }
            if (m <= 50) {
              const double iw = 1.0 / vk;  // inf when v = 0: r/0 semantics
              const double ta = r * iw;
              vH50 += vk; a50 += ta;
              if (m <= 20) {
                vH20 += vk; a20 += ta;
                n20 += (r < 0.0 ? -r : 0.0) * iw;
                q20 += (r > 0.0 ? r : 0.0) * iw;
              }
            }
          }
        }
        if (fam & F_MOMR) {
          RawMom m{gsum(s1), gsum(s2), gsum(s3), gsum(s4), n};
          double sdr;
          const bool has_sdr = std1_raw(m, m.s1 == 0.0 && m.s2 == 0.0, sdr);
          if (has_sdr) R.val(16, sdr); else R.null(16);  // vol_return1min
          const int nu = gcount(upm), nd = gcount(dnm);
          const double U1 = gsum(u1), U2 = gsum(u2), Umn = gmin_d(umn), Umx = gmax_d(umx);
          const double D1 = gsum(w1), D2 = gsum(w2), Dmn = gmin_d(wmn), Dmx = gmax_d(wmx);
          double sup = 0.0, sdn = 0.0;  // fill_null(0)
          std1_raw(RawMom{U1, U2, 0, 0, nu}, Umn == Umx, sup);
          std1_raw(RawMom{D1, D2, 0, 0, nd}, Dmn == Dmx, sdn);
          R.val(17, sup);  // vol_upVol
          R.val(19, sdn);  // vol_downVol
          if (has_sdr) { R.val(18, sup / sdr); R.val(20, sdn / sdr); }
          else { R.null(18); R.null(20); }
          double sk, ku;
          skew_kurt(m, sk, ku);
          R.val(21, sk);
          R.val(22, ku);
          R.val(23, sk / ku);
        }
        if (fam & F_TRD) {
          if (gany((pb & rmask(220, 239)) != 0u)) R.val(50, gsum(rT20) / (gsum(vT20) + 1.0));
          if (gany((pb & rmask(190, 239)) != 0u)) {
            double den = gsum(vT50);
            if (den == 0.0) den = 1.0;
            R.val(51, gsum(rT50) / den);
          }
          const int nh20 = gcount(pb & rmask(0, 20)), nh50 = gcount(pb & rmask(0, 50));
          if (nh20 > 0) {
            const double sH = gsum(vH20);
            R.val(54, sH * gsum(a20) / (double)nh20);
            R.val(56, sH * gsum(n20) / (double)nh20);
            R.val(57, sH * gsum(q20) / (double)nh20);
          }
          if (nh50 > 0) R.val(55, gsum(vH50) * gsum(a50) / (double)nh50);
        }
      }

      // ================================================================ SEG CM:10-90
      if (fam & F_SEG) {
        fresh(c);
        fresh(o);

        auto seg = [&](int f, int ma, int mb, float ca, float cb, float oa, float ob) {
          const bool pa = gpres(pb, ma), pbb = gpres(pb, mb);
          if (!pa && !pbb) return;
          R.val(f, (double)(pbb ? cb : ca) / (double)(pa ? oa : ob));
        };
        seg(0, 120, 239, gvalc<120>(c), gvalc<239>(c), gvalc<120>(o), gvalc<239>(o));  // mmt_pm
        seg(1, 210, 239, gvalc<210>(c), gvalc<239>(c), gvalc<210>(o), gvalc<239>(o));  // mmt_last30
        seg(3, 0, 119, gvalc<0>(c), gvalc<119>(c), gvalc<0>(o), gvalc<119>(o));        // mmt_am
        seg(4, 30, 209, gvalc<30>(c), gvalc<209>(c), gvalc<30>(o), gvalc<209>(o));     // mmt_between
        // mmt_paratio CM:42-60, C1: g(PM) - g(AM); one session gives g - g
        const uint32_t am = pb & rmask(0, 119), pm = pb & rmask(120, 239);
        const int af = gfirst(am), al = glast(am), pf = gfirst(pm), pl = glast(pm);
        double gA = 0.0, gP = 0.0;
        if (af >= 0) gA = (double)gval(c, al) / (double)gval(o, af) - 1.0;
        if (pf >= 0) gP = (double)gval(c, pl) / (double)gval(o, pf) - 1.0;
        R.val(2, (af >= 0 && pf >= 0) ? gP - gA : (af >= 0 ? gA - gA : gP - gP));
      }

      // ================================================================ MOMV CM:485-496, 690-729
      if (fam & F_MOMV) {
        fresh(v);

        const double x0 = (double)gvalu(v, fb);
        double s1 = 0, s2 = 0, s3 = 0, s4 = 0;
#pragma unroll
        for (int k = 0; k < K; ++k)
          if ((pb >> k) & 1u) {
            const double dd = (double)v[k] - x0, d2 = dd * dd;
            s1 += dd; s2 += d2; s3 += d2 * dd; s4 += d2 * d2;
          }
        RawMom m{gsum(s1), gsum(s2), gsum(s3), gsum(s4), n};
        double sdv;
        if (std1_raw(m, m.s1 == 0.0 && m.s2 == 0.0, sdv)) R.val(14, sdv); else R.null(14);
        // skew/kurt of v / sum(v) == of v (scale-free); sum(v) = 0 -> shares NaN
        double sk, ku;
        skew_kurt(m, sk, ku);
        if (sumv == 0.0) sk = ku = qnan();
        R.val(24, sk);
        R.val(25, ku);
        R.val(26, sk / ku);
      }

      // ================================================================ SUMV CM:764-831, 1251-1306
      if (fam & F_SUMV) {
        fresh(v);

        const uint32_t mpre = pb & rmask(0, 236), mcls = pb & rmask(237, 239);
        const uint32_t mhead = pb & rmask(0, 30), mtail = pb & rmask(210, 239);
        double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const double vk = (double)v[k];
          if ((mpre >> k) & 1u) a0 += vk;
          if ((mcls >> k) & 1u) a1 += vk;
          if ((mhead >> k) & 1u) a2 += vk;
          if ((mtail >> k) & 1u) a3 += vk;
        }
        const double spre = gsum(a0), scls = gsum(a1), shead = gsum(a2), stail = gsum(a3);
        if (gany(mpre != 0u)) R.val(28, spre);
        if (gany(mcls != 0u)) R.val(29, scls);
        const double vfirst = (double)gvalu(v, fb);
        R.val(30, vfirst / sumv);
        R.val(31, scls / sumv);
        R.val(32, vfirst);
        R.val(52, sumv > 0.0 ? shead / sumv : 0.125);
        R.val(53, sumv > 0.0 ? stail / sumv : 0.125);
      }

      // ================================================================ SUMC + CORR CM:734-761, 834-932
      if (fam & (F_SUMC | F_CORR)) {
        fresh(c);
        fresh(v);

        // last present close / volume of this lane -> carries from the left
        float lc = 1.f, lcz = 1.f;
        uint32_t lvv = 0u, lvz = 0u;
        const uint32_t pz = pb & 0xFFFFu;
        uint32_t nzm = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          if ((pb >> k) & 1u) { lc = c[k]; lvv = v[k]; }
          if (((pb >> k) & 1u) && v[k] != 0u) { lcz = c[k]; lvz = v[k]; nzm |= 1u << k; }
        }
        (void)pz;
        float cpv, cpz;
        uint32_t vpv, vpz;
        bool hp, hz, hpv, hzv;
        carry_left(lc, pb != 0u, cpv, hp);
        carry_left(lvv, pb != 0u, vpv, hpv);
        carry_left(lcz, nzm != 0u, cpz, hz);
        carry_left(lvz, nzm != 0u, vpz, hzv);
        if (fam & F_SUMC) {
          double am = 0.0;
          float cp = cpv;
          bool h_ = hp;
#pragma unroll
          for (int k = 0; k < K; ++k)
            if ((pb >> k) & 1u) {
              if (h_ && v[k] != 0u) am += fabs((double)c[k] - (double)cp) / ((double)cp * (double)v[k]);
              cp = c[k];
              h_ = true;
            }
          R.val(27, gsum(am));  // liq_amihud_1min
        }
        if (fam & F_CORR) {
          // first two present bars f1, f2 and first two non-zero-volume bars z1, z2
          const int f1 = fb;
          uint32_t pb2 = pb;
          if (f1 >= 0 && (f1 >> 4) == g) pb2 &= ~(1u << (f1 & 15));
          const int f2 = gfirst(pb2);
          const int z1 = gfirst(nzm);
          uint32_t nz2 = nzm;
          if (z1 >= 0 && (z1 >> 4) == g) nz2 &= ~(1u << (z1 & 15));
          const int z2 = gfirst(nz2);
          const double cf1 = (double)gval(c, f1), vf1 = (double)gvalu(v, f1);
          const double cf2 = f2 >= 0 ? (double)gval(c, f2) : 0.0, vf2 = f2 >= 0 ? (double)gvalu(v, f2) : 0.0;
          const double cz1 = z1 >= 0 ? (double)gval(c, z1) : 1.0, vz1 = z1 >= 0 ? (double)gvalu(v, z1) : 1.0;
          const double cz2 = z2 >= 0 ? (double)gval(c, z2) : 1.0, vz2 = z2 >= 0 ? (double)gvalu(v, z2) : 1.0;
          // shifts = first pair of each variant (exact zeros for constant sides)
          const double x1 = (cf2 - cf1) / cf1, y1 = vf2;   // prv: (pct_change(close), volume)
          const double x2 = cf1, y2 = vf1;                 // pv
          const double x3 = cf2, y3 = vf1;                 // pvd: (close, volume.shift(1))
          const double x4 = cf1, y4 = vf2;                 // pvl: (close, volume.shift(-1))
          const double x5 = (cz2 - cz1) / cz1, y5 = (vz2 - vz1) / vz1;  // prvr
          const double x6 = cz2;                           // pvr (y shift = y5)
          const int nzc = gcount(nzm);
          auto fin = [&](int fidx, int np, double a0, double a1, double a2, double a3, double a4) {
            R.val(fidx, pearson_raw(np, gsum(a0), gsum(a1), gsum(a2), gsum(a3), gsum(a4)));
          };
          // pass 1: pv, prv, pvd (previous present bar)
          {
            double P[3][5];
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
              for (int j = 0; j < 5; ++j) P[i][j] = 0.0;
            float cp = cpv;
            uint32_t vp = vpv;
            bool h_ = hp;
#pragma unroll
            for (int k = 0; k < K; ++k) {
              if ((pb >> k) & 1u) {
                const double ck = (double)c[k], vk = (double)v[k];
                double dx = ck - x2, dy = vk - y2;
                P[0][0] += dx; P[0][1] += dy; P[0][2] += dx * dx; P[0][3] += dy * dy; P[0][4] += dx * dy;
                if (h_) {
                  const double pc = (ck - (double)cp) / (double)cp;
                  dx = pc - x1; dy = vk - y1;
                  P[1][0] += dx; P[1][1] += dy; P[1][2] += dx * dx; P[1][3] += dy * dy; P[1][4] += dx * dy;
                  dx = ck - x3; dy = (double)vp - y3;
                  P[2][0] += dx; P[2][1] += dy; P[2][2] += dx * dx; P[2][3] += dy * dy; P[2][4] += dx * dy;
                }
                cp = c[k]; vp = v[k]; h_ = true;
              }
            }
            fin(35, n, P[0][0], P[0][1], P[0][2], P[0][3], P[0][4]);          // corr_pv
            fin(33, n - 1, P[1][0], P[1][1], P[1][2], P[1][3], P[1][4]);      // corr_prv
            fin(36, n - 1, P[2][0], P[2][1], P[2][2], P[2][3], P[2][4]);      // corr_pvd
          }
          // pass 2: prvr, pvr over rows with volume != 0 (CM:855-866, 924-930)
          if (nzc > 0) {
            double P[2][5];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
              for (int j = 0; j < 5; ++j) P[i][j] = 0.0;
            float czp = cpz;
            uint32_t vzp = vpz;
            bool hz_ = hz;
#pragma unroll
            for (int k = 0; k < K; ++k) {
              if (((nzm >> k) & 1u)) {
                const double ck = (double)c[k], vk = (double)v[k];
                if (hz_) {
                  const double pcz = (ck - (double)czp) / (double)czp;
                  const double pvz = (vk - (double)vzp) / (double)vzp;
                  double dx = pcz - x5, dy = pvz - y5;
                  P[0][0] += dx; P[0][1] += dy; P[0][2] += dx * dx; P[0][3] += dy * dy; P[0][4] += dx * dy;
                  dx = ck - x6;
                  P[1][0] += dx; P[1][1] += dy; P[1][2] += dx * dx; P[1][3] += dy * dy; P[1][4] += dx * dy;
                }
                czp = c[k]; vzp = v[k]; hz_ = true;
              }
            }
            fin(34, nzc - 1, P[0][0], P[0][1], P[0][2], P[0][3], P[0][4]);  // corr_prvr
            fin(38, nzc - 1, P[1][0], P[1][1], P[1][2], P[1][3], P[1][4]);  // corr_pvr
          }
          // pass 3: pvl, right-to-left with the next present volume (CM:905-916)
          {
            double a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0;
            uint32_t fvv = 0u;
#pragma unroll
            for (int k = K - 1; k >= 0; --k)
              if ((pb >> k) & 1u) fvv = v[k];
            uint32_t vn;
            bool hn;
            carry_right(fvv, pb != 0u, vn, hn);
#pragma unroll
            for (int k = K - 1; k >= 0; --k)
              if ((pb >> k) & 1u) {
                if (hn) {
                  const double dx = (double)c[k] - x4, dy = (double)vn - y4;
                  a0 += dx; a1 += dy; a2 += dx * dx; a3 += dy * dy; a4 += dx * dy;
                }
                vn = v[k];
                hn = true;
              }
            fin(37, n - 1, a0, a1, a2, a3, a4);  // corr_pvl
          }
        }
      }

      // ================================================================ LVL / PDF: close levels
      if (fam & (F_LVL | F_PDF)) {
        fresh(c);
        fresh(v);
        // Levels (distinct closes) in descending close order: after an ascending sort,
        // element e < n is a bar with close word cw[e] (ascending = close descending,
        // close = bitsf(cbase - cw)) and volume vv[e]; a level is a run of equal cw.
        //  * narrow days (closes within 2^24 float steps, i.e. a high/low close ratio
        //    below 2: every real A-share day): u32 keys (bits(cmax) - bits(c)) << 8 | bar,
        //    the bar's volume read back from LDS after the sort;
        //  * otherwise u64 keys ~bits(close) << 32 | volume.
        // Closes are > 0, so the float order is the bit order; absent bars sort last.
        // A stock-day with a non-integral volume still sorts (volume 0) for the level
        // list, and its LVL/PDF values go to the exact path.
        uint32_t cmx = 0u, cmn = 0xffffffffu;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          cmx = max(cmx, fbits(c[k]) & present_bits(pb, k));
          cmn = min(cmn, fbits(c[k]) | absent_bits(pb, k));
        }
        // the level volumes below are exact u32 cumulative sums: a day whose volume
        // reaches 2^32 shares goes to the exact kernel (f64 sums, exact below 2^53)
        const bool ok = sumv < 4294967296.0;
        cmx = gmax_u(cmx);
        cmn = gmin_u(cmn);
        const float clastf = gval(c, lb);
        bool fast = !gany(!ok);
        const int e0 = 16 * g;
        uint32_t cw[K], vv[K], cbase = cmx;
        // a day whose closes span >= 2^24 float steps (a close ratio of 2 or more) does
        // not fit the u32 keys: the exact wave64 kernel takes it whole (values, queries
        // and its doc_pdf levels; list entry flagged by the top bit)
        const bool wide = cmx - cmn >= (1u << 24);  // uniform inside the group
        if (wide) {
          // (not a kept row-set stock-day whose LVL / PDF come from mff_stage1_rows)
          if (g == 0 && !(grid_skip(a.mask[sd * 8 + 7]) & (F_LVL | F_PDF))) {
            const int idx = atomicAdd(a.fb_count, 1);
            a.fb_list[idx] = (int)((uint32_t)sd | 0x80000000u);
          }
#pragma unroll
          for (int k = 0; k < K; ++k) { cw[k] = 0u; vv[k] = 0u; }
        } else {
          // 256 volumes of this group, bar 16g + k at slot 16k + g (the key's low byte):
          // each store instruction writes 16 consecutive words per group (conflict free)
          uint32_t* sv = reinterpret_cast<uint32_t*>(scr);
          uint32_t key[K];
#pragma unroll
          for (int k = 0; k < K; ++k) {
            const uint32_t slot = (uint32_t)(16 * k + g);
            sv[slot] = v[k];  // absent bars hold 0 (sanitized)
            key[k] = ((cmx - fbits(c[k])) << 8) | slot | absent_bits(pb, k);
          }
          gsort256u(key);
          lds_fence();
#pragma unroll
          for (int k = 0; k < K; ++k) {
            cw[k] = key[k] >> 8;
            vv[k] = sv[key[k] & 0xffu];  // elements past n: key ~0 -> slot 255 (bar 255: none, 0)
          }
          lds_fence();
        }
        // Levels = runs of equal close words among the n sorted bars.  validm: this lane's
        // elements e < n; a run ends where the next element's word differs (or at
        // e = n - 1); the element after an end starts a run.
        const int nin = min(max(n - e0, 0), K);
        const uint32_t validm = (uint32_t)((1u << nin) - 1u);
        const uint32_t nextw = dpp_u<ROW_SHL + 1>(cw[0]);
        uint32_t diffm = 0u, tv = 0u;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const uint32_t wn = k < K - 1 ? cw[k + 1] : nextw;
          diffm |= (cw[k] != wn ? 1u : 0u) << k;
          tv += vv[k];  // 0 past n
        }
        const uint32_t lastm = (n - 1 >= e0 && n - 1 < e0 + K) ? 1u << (n - 1 - e0) : 0u;
        const uint32_t endm = (diffm | lastm) & validm;
        const int L = gcount(endm);
        if (!wide && a.lvl_key) {
          emitL = (uint32_t)L;
          emitC = clastf;
          emitB = cbase;
        }
        if (!wide) {
          // Compact the levels (run ends, descending close) into LDS by level index:
          //   lv[l] = cumulative volume through level l (exact u32 when sum(v) < 2^32; a
          //   larger day is not `fast`: its values come from the exact kernel),
          //   lc[l] = cw << 8 | e, its last sorted element (cw < 2^24 on this path),
          // so level l has volume lv[l] - lv[l-1] and e_l - e_(l-1) bars, and everything
          // per level below runs over ceil(L/16) slots per lane (a lane's levels
          // contiguous) instead of the 16 sorted bars.
          uint32_t* lv = reinterpret_cast<uint32_t*>(scr);
          uint32_t* lc = lv + NBAR;  // L <= 240 levels
          uint32_t cum = gscan_excl_u(tv);
          int li = (int)gscan_excl_u((uint32_t)__builtin_popcount(endm));
#pragma unroll
          for (int k = 0; k < K; ++k) {
            cum += vv[k];
            if ((endm >> k) & 1u) {
              lv[li] = cum;
              lc[li] = (cw[k] << 8) | (uint32_t)(e0 + k);
              ++li;
            }
          }
          lds_fence();
          const uint32_t Sv = (uint32_t)sumv;
          const double inv = 1.0 / sumv;
          // level 0 (the highest close) is the member shift of the share moments
          const double x0 = (double)lv[0] * inv;
          // doc_pdf: the first level whose cumulative share exceeds k/20 is the first with
          // 20*cum > k*Sv, i.e. cum > floor(k*Sv/20) (integers); an exact tie
          // 20*cum == k*Sv at a level (only when 20 | k*Sv) is left to the exact path.
          // floor(k*Sv/20) = k*(Sv/20) + (k*(Sv%20))/20 in u32.
          double s1 = 0, s2 = 0, s3 = 0, s4 = 0;
          if (fam & F_LVL) {
            // levels interleaved over the lanes (level l from lane l % 16): each read
            // instruction touches 16 consecutive words per group
            for (int l = g; l < L; l += 16) {
              const uint32_t V = lv[l] - (l > 0 ? lv[l - 1] : 0u);
              const double dd = (double)V * inv - x0, d2 = dd * dd;
              s1 += dd; s2 += d2; s3 += d2 * dd; s4 += d2 * d2;
            }
          }
          if (fast && (fam & F_LVL)) {
            // level shares V_l / sum(v) (C7: equal volumes -> identical shares)
            RawMom m{gsum(s1), gsum(s2), gsum(s3), gsum(s4), L};
            double sk, ku;
            skew_kurt(m, sk, ku);
            if (!(sumv > 0.0)) sk = ku = qnan();
            R.val(39, ku);  // doc_kurt
            R.val(40, sk);  // doc_skew
            R.val(41, sk);  // doc_std: .skew() [sic CM:999]
          }
          if (fast && (fam & F_PDF)) {
            // lane t < 5 answers query t: levels with cum <= T come first (cum is
            // monotone), so their count e is found by binary search over lv
            const uint32_t kt = g == 0 ? 12u : g == 1 ? 14u : g == 2 ? 16u : g == 3 ? 18u : 19u;
            const uint32_t sq20 = Sv / 20u, sr20 = Sv - 20u * sq20;
            const uint32_t b = kt * sr20;  // < 380
            const uint32_t bq = b / 20u;
            const uint32_t T = kt * sq20 + bq;
            int e = 0;
#pragma unroll
            for (int st = 128; st >= 1; st >>= 1)
              if (e + st <= L && lv[e + st - 1] <= T) e += st;
            // an exact tie 20*cum == k*Sv is at the last level with cum <= T
            const bool tie = g < 5 && b == 20u * bq && e > 0 && lv[e - 1] == T;
            if (gany(tie) && Sv != 0u) fast = false;  // the reference's float order decides
            // Sv = 0: shares NaN, NaN > p (S11) -> the first level
            if (Sv == 0u) e = 0;
            if (g < 5 && e < L) qv = fdiv_f32in(clastf, bitsf(cbase - (lc[e] >> 8)));
          }
          lds_fence();
        }
        if (!fast && !wide && (fam & (a.fam_exact))) {
          if (g == 0 && !(grid_skip(a.mask[sd * 8 + 7]) & (F_LVL | F_PDF))) {
            const int idx = atomicAdd(a.fb_count, 1);
            a.fb_list[idx] = (int)sd;
          }
        }
        if (fam & F_PDF) {
          if (!fast) qv = qnan();
#pragma unroll
          for (int t = 0; t < 5; ++t) R.null(PDF0 + t);  // filled by mff_pdf_finalize (or the fallback)
        }
      }
    }

    // ---------------------------------------------------------------- doc_pdf level list
    // One reservation per wave for its four groups' levels: every stock-day of the block
    // is day d, so one returning atomic per 4 stock-days on the day's counter instead of
    // one per stock-day (5,000 serialized adds per day at c4: 1.3 ms of the kernel).  The
    // day's levels go to two lists (pdf_levels_split): list A the keys c_last / close
    // below the pass's split key, from the front of the day's region, list B the others
    // from its back; one u64 counter holds both counts (A low, B high), so the
    // reservation stays one atomic.  Levels are in descending close order (keys
    // ascending), so a group's list-A levels are its first gA.  Issued before the result stores, the reservation used after them.
    // Row set (include/mff.h): the families mff_stage1_rows computes for this stock-day
    // (mask word 7): none, or every one (its mask words are zero: n == 0 above), or for a
    // kept stock-day the families that read a field holding a null -- their stores, and
    // with doc_pdf its levels and queries, are left to mff_stage1_rows
    const uint32_t skip = act ? grid_skip(a.mask[sd * 8 + 7]) : 0u;
    if (skip & F_PDF) emitL = 0u;
    const bool emit = a.lvl_key != nullptr;  // uniform
    uint32_t lpreA = 0u, lpreB = 0u, gA = 0u;
    uint64_t lwb = 0ull;
    if (emit) {
      const uint32_t* lc = reinterpret_cast<const uint32_t*>(scr) + NBAR;
      const uint64_t ksplit = pdf_split_key(a.lvl_count, a.D);
      // keys ascend with l (closes descend): gA = lower_bound of the split key over the
      // group's levels, two rounds of 16 probes (blocks of 16 levels, then within one)
      auto key_at = [&](int l) {
        return dbits(fdiv_f32in(emitC, bitsf(emitB - (lc[l] >> 8)))) | 0x8000000000000000ull;
      };
      const int pb = 16 * g + 15;
      const bool lb1 = pb < (int)emitL && key_at(pb) < ksplit;
      const uint32_t c1 = (uint32_t)__popc((uint32_t)(__ballot(lb1) >> gbase()) & 0xFFFFu);
      const int pw = 16 * (int)c1 + g;
      const bool lb2 = pw < (int)emitL && key_at(pw) < ksplit;
      gA = 16u * c1 + (uint32_t)__popc((uint32_t)(__ballot(lb2) >> gbase()) & 0xFFFFu);
      const uint32_t nB = emitL - gA;
      const uint32_t a0 = (uint32_t)__builtin_amdgcn_readlane((int)gA, 0);
      const uint32_t a1 = (uint32_t)__builtin_amdgcn_readlane((int)gA, 16);
      const uint32_t a2 = (uint32_t)__builtin_amdgcn_readlane((int)gA, 32);
      const uint32_t a3 = (uint32_t)__builtin_amdgcn_readlane((int)gA, 48);
      const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)nB, 0);
      const uint32_t b1 = (uint32_t)__builtin_amdgcn_readlane((int)nB, 16);
      const uint32_t b2 = (uint32_t)__builtin_amdgcn_readlane((int)nB, 32);
      const uint32_t b3 = (uint32_t)__builtin_amdgcn_readlane((int)nB, 48);
      lpreA = grp == 0 ? 0u : grp == 1 ? a0 : grp == 2 ? a0 + a1 : a0 + a1 + a2;
      lpreB = grp == 0 ? 0u : grp == 1 ? b0 : grp == 2 ? b0 + b1 : b0 + b1 + b2;
      const uint64_t tot = (uint64_t)(a0 + a1 + a2 + a3) | ((uint64_t)(b0 + b1 + b2 + b3) << 32);
      if (lane == 0 && tot != 0ull)
        lwb = atomicAdd(reinterpret_cast<unsigned long long*>(a.lvl_count) + d, (unsigned long long)tot);
    }

    // ---------------------------------------------------------------- stores
    // the row set's families are stored by mff_stage1_rows alone, which may run
    // concurrently (a kept stock-day: the family test, behind a wave-uniform branch)
    if (act && skip != ~0u) {
      auto store = [&](auto kept) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int f = 16 * q + g;
          if (f < NF) {
            const int row = a.row[f];
            if (row >= 0 && (!decltype(kept)::value || !(kFamOf(f) & skip))) {
              a.val[(size_t)row * plane + sd] = R.r[q];
              a.state[(size_t)row * plane + sd] = (uint8_t)((R.st >> (8 * q)) & 0xFFu);
            }
          }
        }
      };
      if (__builtin_amdgcn_ballot_w64(skip != 0u) == 0ull) store(std::false_type());
      else store(std::true_type());
      if (a.pdfq && g < 5 && !(skip & F_PDF)) {
        a.pdfq[(size_t)g * plane + sd] = qv;
      }
    }
    if (emit) {
      // key c_last / close (correctly rounded), bars at the level; levels interleaved
      // over the group's lanes (level l from lane l % 16), so one store instruction
      // writes 16 consecutive entries per group (list B's in descending addresses; the
      // block holding the group's A / B boundary writes to both lists).  The levels are
      // still in the group's scratch (lc, from the LVL section).
      const uint64_t wb = ((uint64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(lwb >> 32)) << 32) |
                          (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)lwb);
      const uint32_t baseA = (uint32_t)wb + lpreA, baseB = (uint32_t)(wb >> 32) + lpreB;
      const uint32_t* lc = reinterpret_cast<const uint32_t*>(scr) + NBAR;
      const size_t capd = pdf_day_cap(a.S);
      uint64_t* kd = a.lvl_key + (size_t)d * capd;
      uint8_t* wd = a.lvl_w + (size_t)d * capd;
      for (int l = g; l < (int)emitL; l += 16) {
        const uint32_t cwb = lc[l];
        const uint32_t ee = cwb & 0xFFu;
        const uint32_t ep = l > 0 ? (lc[l - 1] & 0xFFu) : 0xFFFFFFFFu;  // -1 before level 0
        const size_t at = (uint32_t)l < gA ? (size_t)(baseA + (uint32_t)l)
                                          : capd - 1 - (size_t)(baseB + (uint32_t)l - gA);
        kd[at] = dbits(fdiv_f32in(emitC, bitsf(emitB - (cwb >> 8)))) | 0x8000000000000000ull;  // ord64 of a positive
        wd[at] = (uint8_t)(ee - ep);
      }
      lds_fence();  // the next iteration rewrites the scratch
    }
  }
}

}  // namespace g16
}  // namespace mff

using namespace mff;

// workspace: list count (256 B) | exact list int [S*D] | ORD volume thresholds u32 [3][S*D]
extern "C" size_t mff_stage1_workspace_bytes(int S, int D) {
  return 256 + (size_t)S * (size_t)D * (sizeof(int) + 3 * sizeof(uint32_t));
}

namespace mff {
// doc_pdf level side channel: counts u32 [D] | keys u64 [D][S*256] | bars u8 [D][S*256]
// (a day holds at most one level per bar of every stock)
// level buffer: per day the entry counts of list A and list B (u32 pairs, A first: one
// u64 counter per day) and the split key (u64, pdf_koff), then
// the keys u64 [D][S * 256] and the bars u8 [D][S * 256] (pdf_day_cap); list A (keys below
// the split key) fills a day's slots from the front, list B from the back
size_t pdf_levels_split(int S, int D, size_t* off_key, size_t* off_w) {
  const size_t cap = pdf_day_cap(S) * (size_t)D;
  *off_key = (pdf_koff(D) + 8 + 255) & ~(size_t)255;
  *off_w = *off_key + cap * 8;
  return *off_w + cap;
}
}  // namespace mff

extern "C" size_t mff_pdf_levels_bytes(int S, int D) {
  size_t a, b;
  return pdf_levels_split(S, D, &a, &b);
}

// part bit 1: the LVL/PDF group (levels + queries) and the exact list kernel — everything
// the doc_pdf rank needs; part bit 2: the ORD group and the serial families (which read
// the ORD thresholds).  mff_stage1 = both, in that order.  Bit 4: the high / low serial
// kernel (OLS, MOMH) alone — it reads nothing another launch writes, so it may run on its
// own stream from the start; bit 8 (with bit 2): part 2 without it.  Part 17 = part 1
// without the exact list kernel, part 32 = that kernel alone (it only adds LVL/PDF
// values and doc_pdf levels of the listed stock-days, so the serial families need not
// wait for it).
static int stage1_parts(const float* open, const float* high, const float* low, const float* close,
                        const uint32_t* volume, const uint32_t* valid, int S, int D, const int32_t* factor_ids,
                        int nf, double* val, uint8_t* state, double* pdf_query, void* pdf_levels,
                        void* workspace, void* stream, int part) {
  clear_error();
  MFF_REQUIRE(part == 1 || part == 2 || part == 3 || part == 4 || part == 10 || part == 11 || part == 17 ||
                  part == 32 || part == 64 || part == 129 || part == 145,
              "mff_stage1_part: part=%d must be 1, 2, 3, 4, 10, 11, 17, 32, 64, 129 or 145", part);
  MFF_REQUIRE(S > 0 && D > 0, "mff_stage1: S=%d D=%d must be positive", S, D);
  MFF_REQUIRE((long long)S * D < (1ll << 31), "mff_stage1: S*D must be < 2^31");
  MFF_REQUIRE(nf > 0 && nf <= NF, "mff_stage1: nf=%d out of range", nf);
  MFF_REQUIRE(factor_ids != nullptr, "mff_stage1: factor_ids is NULL");
  MFF_REQUIRE(valid && val && state, "mff_stage1: NULL device buffer");
  MFF_REQUIRE(workspace != nullptr, "mff_stage1: workspace is NULL (mff_stage1_workspace_bytes)");
  // the volume plane travels with the price planes (its rows are read as u32)
  const float* fld[5] = {open, high, low, close, reinterpret_cast<const float*>(volume)};
  g16::GArgs a;
  memset(&a, 0, sizeof(a));
  for (int f = 0; f < 5; ++f) a.fld[f] = fld[f];
  a.mask = valid; a.val = val; a.state = state; a.pdfq = pdf_query;
  a.S = S; a.D = D;
  a.fam_exact = ~0u;
  for (int i = 0; i < NF; ++i) a.row[i] = -1;
  for (int r = 0; r < nf; ++r) {
    const int id = factor_ids[r];
    MFF_REQUIRE(id >= 0 && id < NF, "mff_stage1: factor id %d out of range", id);
    MFF_REQUIRE(a.row[id] < 0, "mff_stage1: factor id %d requested twice", id);
    a.row[id] = (int8_t)r;
    a.fam |= kFactorFamily[id];
  }
  // a kept row-set stock-day's null field sends exactly the families that read it to
  // mff_stage1_rows (include/mff.h MFF_ROWS_KEEP; rows_fams and kFieldFams in mff_internal.h)
  static_assert(rows_fams(MFF_ROWS_KEEP | (1u << MFF_ROWS_NULL_SHIFT)) == kFieldFams[0], "open");
  static_assert(rows_fams(MFF_ROWS_KEEP | (16u << MFF_ROWS_NULL_SHIFT)) == kFieldFams[4], "volume");
  static_assert(rows_fams(MFF_ROWS_LISTED) == ~0u && grid_skip(0u) == 0u, "listed whole / not listed");
  for (int f = 0; f < 5; ++f)
    MFF_REQUIRE(!(a.fam & kFieldFams[f]) || fld[f] != nullptr, "mff_stage1: field plane %d required", f);
  MFF_REQUIRE(!(a.fam & F_PDF) || (pdf_query != nullptr && pdf_levels != nullptr),
              "mff_stage1: doc_pdf requested but pdf_query / pdf_levels is NULL");
  hipStream_t st = as_stream(stream);
  int* cnt = reinterpret_cast<int*>(workspace);
  a.fb_count = cnt;
  a.fb_list = reinterpret_cast<int*>(reinterpret_cast<char*>(workspace) + 256);
  a.ord_th = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(workspace) + 256 + (size_t)S * D * sizeof(int));
  const char* impl = getenv("MFF_STAGE1_IMPL");
  const bool w64 = impl && strcmp(impl, "w64") == 0;
  const long long nblk = (long long)((S + 16 * kGIter - 1) / (16 * kGIter)) * D;
  // one 16-lane group launch; it stores its own group's rows (and the queries) only
  auto group_launch = [&](int gi) -> int {
    const uint32_t set = gi < 2 ? g16::kGroups[gi] : g16::G_OL;
    if (!(a.fam & set)) return 0;
    g16::GArgs b = a;
    for (int i = 0; i < NF; ++i)
      if (!(kFactorFamily[i] & set)) b.row[i] = -1;
    if (!(set & F_PDF)) b.pdfq = nullptr;
    if (gi == 0) hipLaunchKernelGGL(g16::k_stage1g<g16::G_ORD>, dim3((unsigned)nblk), dim3(256), 0, st, b);
    else if (gi == 1) hipLaunchKernelGGL(g16::k_stage1g<g16::G_LVL>, dim3((unsigned)nblk), dim3(256), 0, st, b);
    else hipLaunchKernelGGL(g16::k_stage1g<g16::G_OL>, dim3((unsigned)nblk), dim3(256), 0, st, b);
    MFF_LAUNCH_CHECK();
    return 0;
  };
  if (a.fam & F_PDF) {
    size_t ok, ow;
    pdf_levels_split(S, D, &ok, &ow);
    char* base = reinterpret_cast<char*>(pdf_levels);
    a.lvl_count = reinterpret_cast<uint32_t*>(base);
    a.lvl_key = reinterpret_cast<uint64_t*>(base + ok);
    a.lvl_w = reinterpret_cast<uint8_t*>(base + ow);
  }
  if (part == 32) {  // the exact list kernel alone (after part 17, e.g. on another stream)
    if (w64 || !(a.fam & (F_LVL | F_PDF))) return 0;
    return launch_w64(fld, valid, S, D, factor_ids, nf, val, state, pdf_query, a.fb_list, cnt, F_LVL | F_PDF, kExactGrid,
                      st, a.lvl_count, a.lvl_key, a.lvl_w);
  }
  if (part & 65) {  // the prologue of part 1: level-list counts, split key, exact-list count
    if (!(part & 128)) {
      if (a.fam & F_PDF) {
        MFF_HIP(hipMemsetAsync(a.lvl_count, 0, (size_t)D * 8, st));
        if (pdf_split_init(a.lvl_count, D, st) != 0) return -2;
      }
      MFF_HIP(hipMemsetAsync(cnt, 0, sizeof(int), st));
    }
    if (part == 64) return 0;
  }
  if (part & 1) {  // LVL/PDF group + exact list: everything the doc_pdf phases read
    if (w64) {  // the wave-per-stock-day kernel for everything
      const int rc = launch_w64(fld, valid, S, D, factor_ids, nf, val, state, pdf_query, nullptr, nullptr, ~0u, 0, st);
      if (rc != 0 || !(a.fam & F_PDF)) return rc;
      g16::GArgs b = a;  // doc_pdf level lists only (no rows, no queries, no exact list)
      for (int i = 0; i < NF; ++i) b.row[i] = -1;
      b.pdfq = nullptr;
      b.fam = F_PDF;
      b.fam_exact = 0u;
      hipLaunchKernelGGL(g16::k_stage1g<g16::G_LVL>, dim3((unsigned)nblk), dim3(256), 0, st, b);
      MFF_LAUNCH_CHECK();
      // levels of the wide days (listed by the launch above)
      return launch_w64(fld, valid, S, D, factor_ids, nf, val, state, pdf_query, a.fb_list, cnt, F_PDF, kExactGrid, st,
                        a.lvl_count, a.lvl_key, a.lvl_w);
    }
    // ORD in the same launch when both sorted groups are requested (part 2 then skips it)
    int rc = group_launch((a.fam & g16::G_ORD) && (a.fam & (F_LVL | F_PDF)) ? 2 : 1);
    if (rc != 0) return rc;
    if ((a.fam & (F_LVL | F_PDF)) && !(part & 16)) {
      // exact general path for the listed stock-days (LVL + PDF only); part 17 leaves it
      // to a later part-32 call
      rc = launch_w64(fld, valid, S, D, factor_ids, nf, val, state, pdf_query, a.fb_list, cnt,
                      F_LVL | F_PDF, kExactGrid, st, a.lvl_count, a.lvl_key, a.lvl_w);
      if (rc != 0) return rc;
    }
  }
  constexpr uint32_t kHL = F_OLS | F_MOMH;  // the high / low serial kernel's families
  if (part & 4) {
    if (w64) return 0;  // the w64 path (part 1) computed every family
    return launch_serial(fld, valid, S, D, a.row, a.fam & kHL, val, state, a.ord_th, st);
  }
  if ((part & 2) && !w64) {  // the ORD sort (thresholds) before the serial kernels (products)
    if (!((a.fam & g16::G_ORD) && (a.fam & (F_LVL | F_PDF)))) {
      const int rc = group_launch(0);
      if (rc != 0) return rc;
    }
    return launch_serial(fld, valid, S, D, a.row, (part & 8) ? a.fam & ~kHL : a.fam, val, state, a.ord_th, st);
  }
  return 0;
}

extern "C" int mff_stage1(const float* open, const float* high, const float* low, const float* close,
                          const uint32_t* volume, const uint32_t* valid, int S, int D, const int32_t* factor_ids,
                          int nf, double* val, uint8_t* state, double* pdf_query, void* pdf_levels,
                          void* workspace, void* stream) {
  return stage1_parts(open, high, low, close, volume, valid, S, D, factor_ids, nf, val, state, pdf_query,
                      pdf_levels, workspace, stream, 3);
}

extern "C" int mff_stage1_part(const float* open, const float* high, const float* low, const float* close,
                               const uint32_t* volume, const uint32_t* valid, int S, int D,
                               const int32_t* factor_ids, int nf, double* val, uint8_t* state,
                               double* pdf_query, void* pdf_levels, void* workspace, void* stream, int part) {
  return stage1_parts(open, high, low, close, volume, valid, S, D, factor_ids, nf, val, state, pdf_query,
                      pdf_levels, workspace, stream, part);
}
