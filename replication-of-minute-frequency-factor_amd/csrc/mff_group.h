// mff_group.h — 16-lane group primitives for the stage-1 kernel.
//
// Layout: a wave64 holds FOUR stock-days, one per DPP row (lanes 16g..16g+15).  Lane
// gi = lane & 15 of a group owns the 16 contiguous bars m = 16*gi + k (k = 0..15) of
// every field plane; lane 15 owns bars 240..255, i.e. none.  Group reductions, scans and
// shifts are DPP row operations (quad_perm / row_mirror / row_shr / row_shl act inside a
// row of 16 lanes), so a group never touches another group's data and costs 4 steps.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mff_wave.h"

namespace mff {
namespace g16 {

__device__ __forceinline__ int gi() { return (int)(threadIdx.x & 15u); }
__device__ __forceinline__ int gbase() { return (int)(threadIdx.x & 48u); }

// DPP controls (GFX9 encoding)
constexpr int QP_XOR1 = 0xB1;   // quad_perm [1,0,3,2]
constexpr int QP_XOR2 = 0x4E;   // quad_perm [2,3,0,1]
constexpr int ROW_SHR = 0x110;  // + n
constexpr int ROW_SHL = 0x100;  // + n
constexpr int ROW_MIRROR = 0x140;
constexpr int ROW_HALF_MIRROR = 0x141;
constexpr int K = 16;  // bars per lane

template <int CTRL>
__device__ __forceinline__ int dpp_i(int x) {
  // lanes whose source is outside the row read 0 (bound_ctrl: identity for sums /
  // scans) without a register holding an `old` value to copy first
  return __builtin_amdgcn_mov_dpp(x, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t x) { return (uint32_t)dpp_i<CTRL>((int)x); }
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) { return __int_as_float(dpp_i<CTRL>(__float_as_int(x))); }
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
  const uint64_t b = dbits(x);
  const uint32_t lo = (uint32_t)dpp_i<CTRL>((int)(uint32_t)b);
  const uint32_t hi = (uint32_t)dpp_i<CTRL>((int)(uint32_t)(b >> 32));
  return bitsd(((uint64_t)hi << 32) | lo);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t b) {
  const uint32_t lo = (uint32_t)dpp_i<CTRL>((int)(uint32_t)b);
  const uint32_t hi = (uint32_t)dpp_i<CTRL>((int)(uint32_t)(b >> 32));
  return ((uint64_t)hi << 32) | lo;
}

template <int CTRL>
__device__ __forceinline__ float dppT(float x) { return dpp_f<CTRL>(x); }
template <int CTRL>
__device__ __forceinline__ double dppT(double x) { return dpp_d<CTRL>(x); }
template <int CTRL>
__device__ __forceinline__ uint32_t dppT(uint32_t x) { return dpp_u<CTRL>(x); }

// ---- all-reduce inside the group (every lane of the row gets the same bits)
__device__ __forceinline__ double gsum(double x) {
  x += dpp_d<QP_XOR1>(x);
  x += dpp_d<QP_XOR2>(x);
  x += dpp_d<ROW_HALF_MIRROR>(x);
  x += dpp_d<ROW_MIRROR>(x);
  return x;
}
__device__ __forceinline__ double gprod(double x) {
  x *= dpp_d<QP_XOR1>(x);
  x *= dpp_d<QP_XOR2>(x);
  x *= dpp_d<ROW_HALF_MIRROR>(x);
  x *= dpp_d<ROW_MIRROR>(x);
  return x;
}
__device__ __forceinline__ int gsum_i(int x) {
  x += dpp_i<QP_XOR1>(x);
  x += dpp_i<QP_XOR2>(x);
  x += dpp_i<ROW_HALF_MIRROR>(x);
  x += dpp_i<ROW_MIRROR>(x);
  return x;
}
__device__ __forceinline__ uint32_t gsum_u(uint32_t x) { return (uint32_t)gsum_i((int)x); }
__device__ __forceinline__ int gmin_i(int x) {
  x = min(x, dpp_i<QP_XOR1>(x));
  x = min(x, dpp_i<QP_XOR2>(x));
  x = min(x, dpp_i<ROW_HALF_MIRROR>(x));
  x = min(x, dpp_i<ROW_MIRROR>(x));
  return x;
}
__device__ __forceinline__ int gmax_i(int x) {
  x = max(x, dpp_i<QP_XOR1>(x));
  x = max(x, dpp_i<QP_XOR2>(x));
  x = max(x, dpp_i<ROW_HALF_MIRROR>(x));
  x = max(x, dpp_i<ROW_MIRROR>(x));
  return x;
}
__device__ __forceinline__ bool gany(bool b) { return gmax_i(b ? 1 : 0) != 0; }

// ---- scans over the lanes of the group
__device__ __forceinline__ double gscan_incl(double x) {
  x += dpp_d<ROW_SHR + 1>(x);
  x += dpp_d<ROW_SHR + 2>(x);
  x += dpp_d<ROW_SHR + 4>(x);
  x += dpp_d<ROW_SHR + 8>(x);
  return x;
}
__device__ __forceinline__ uint32_t gscan_incl_u(uint32_t x) {
  x += dpp_u<ROW_SHR + 1>(x);
  x += dpp_u<ROW_SHR + 2>(x);
  x += dpp_u<ROW_SHR + 4>(x);
  x += dpp_u<ROW_SHR + 8>(x);
  return x;
}
// exclusive: value of the lane to the left after the inclusive scan (lane 0 gets 0)
__device__ __forceinline__ double gscan_excl(double x) { return dpp_d<ROW_SHR + 1>(gscan_incl(x)); }
__device__ __forceinline__ uint32_t gscan_excl_u(uint32_t x) { return dpp_u<ROW_SHR + 1>(gscan_incl_u(x)); }

// Carry-in for a per-lane left-to-right walk: the (value, flag) of the nearest lane to
// the left whose flag is set (polars shift(1) / pct_change over present rows, S4/S5).
template <typename T>
__device__ __forceinline__ void carry_left(T v, bool h, T& cv, bool& ch) {
  uint32_t hh = h ? 1u : 0u;
#pragma unroll
  for (int step = 0; step < 4; ++step) {
    T ov;
    uint32_t oh;
    if (step == 0) { ov = dppT<ROW_SHR + 1>(v); oh = dpp_u<ROW_SHR + 1>(hh); }
    if (step == 1) { ov = dppT<ROW_SHR + 2>(v); oh = dpp_u<ROW_SHR + 2>(hh); }
    if (step == 2) { ov = dppT<ROW_SHR + 4>(v); oh = dpp_u<ROW_SHR + 4>(hh); }
    if (step == 3) { ov = dppT<ROW_SHR + 8>(v); oh = dpp_u<ROW_SHR + 8>(hh); }
    if (!hh && oh) { v = ov; hh = 1u; }
  }
  cv = dppT<ROW_SHR + 1>(v);
  ch = dpp_u<ROW_SHR + 1>(hh) != 0u;
}
// Carry-in for a right-to-left walk: nearest lane to the right with the flag set.
template <typename T>
__device__ __forceinline__ void carry_right(T v, bool h, T& cv, bool& ch) {
  uint32_t hh = h ? 1u : 0u;
#pragma unroll
  for (int step = 0; step < 4; ++step) {
    T ov;
    uint32_t oh;
    if (step == 0) { ov = dppT<ROW_SHL + 1>(v); oh = dpp_u<ROW_SHL + 1>(hh); }
    if (step == 1) { ov = dppT<ROW_SHL + 2>(v); oh = dpp_u<ROW_SHL + 2>(hh); }
    if (step == 2) { ov = dppT<ROW_SHL + 4>(v); oh = dpp_u<ROW_SHL + 4>(hh); }
    if (step == 3) { ov = dppT<ROW_SHL + 8>(v); oh = dpp_u<ROW_SHL + 8>(hh); }
    if (!hh && oh) { v = ov; hh = 1u; }
  }
  cv = dppT<ROW_SHL + 1>(v);
  ch = dpp_u<ROW_SHL + 1>(hh) != 0u;
}

// ---- value of group bar m (m group-uniform, data-dependent)
__device__ __forceinline__ int bpermi(int src_lane, int v) { return __builtin_amdgcn_ds_bpermute(src_lane << 2, v); }
__device__ __forceinline__ float bpermf(int src_lane, float v) { return __int_as_float(bpermi(src_lane, __float_as_int(v))); }
__device__ __forceinline__ uint32_t bpermu(int src_lane, uint32_t v) { return (uint32_t)bpermi(src_lane, (int)v); }
__device__ __forceinline__ double bpermd(int src_lane, double v) {
  const uint64_t b = dbits(v);
  const uint32_t lo = (uint32_t)bpermi(src_lane, (int)(uint32_t)b);
  const uint32_t hi = (uint32_t)bpermi(src_lane, (int)(uint32_t)(b >> 32));
  return bitsd(((uint64_t)hi << 32) | lo);
}

// x[k] for a lane-varying k.  Written as an integer bit blend on purpose: a chain of
// `c ? x[j] : t` selects gets folded into load(select(&x[j], ...)), which pins the array
// in private memory (scratch); the blend keeps it in registers (v_bfi / v_cndmask).
__device__ __forceinline__ uint32_t blend_u(bool c, uint32_t a, uint32_t b) {
  const uint32_t m = 0u - (uint32_t)c;
  return (a & m) | (b & ~m);
}
__device__ __forceinline__ uint32_t pick(const uint32_t (&x)[K], int k) {
  uint32_t t = x[0];
#pragma unroll
  for (int j = 1; j < K; ++j) t = blend_u(k == j, x[j], t);
  return t;
}
__device__ __forceinline__ float pick(const float (&x)[K], int k) {
  uint32_t t = __float_as_uint(x[0]);
#pragma unroll
  for (int j = 1; j < K; ++j) t = blend_u(k == j, __float_as_uint(x[j]), t);
  return __uint_as_float(t);
}
__device__ __forceinline__ uint64_t pick(const uint64_t (&x)[K], int k) {
  uint32_t lo = (uint32_t)x[0], hi = (uint32_t)(x[0] >> 32);
#pragma unroll
  for (int j = 1; j < K; ++j) {
    lo = blend_u(k == j, (uint32_t)x[j], lo);
    hi = blend_u(k == j, (uint32_t)(x[j] >> 32), hi);
  }
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ float gval(const float (&x)[K], int m) {
  return bpermf(gbase() + (m >> 4), pick(x, m & 15));
}
__device__ __forceinline__ uint32_t gvalu(const uint32_t (&x)[K], int m) {
  return bpermu(gbase() + (m >> 4), pick(x, m & 15));
}
// bar m known at compile time
template <int M>
__device__ __forceinline__ float gvalc(const float (&x)[K]) {
  return bpermf(gbase() + (M >> 4), x[M & 15]);
}
// presence bit of group bar m
__device__ __forceinline__ bool gpres(uint32_t pb, int m) {
  return (bpermu(gbase() + (m >> 4), pb) >> (m & 15)) & 1u;
}

// all-ones when bar k of the lane is present / absent (one v_bfe_i32: a mask for
// v_and / v_or instead of a compare and a select)
// (the shift form compiles to and + cmp + cndmask; __builtin_amdgcn_sbfe gives the bfe but
// the longer live ranges spilled the group kernel: measured slower)
__device__ __forceinline__ uint32_t present_bits(uint32_t pb, int k) { return (uint32_t)((int32_t)(pb << (31 - k)) >> 31); }
__device__ __forceinline__ uint32_t absent_bits(uint32_t pb, int k) { return ~present_bits(pb, k); }

// ---- bar-range masks of this lane (16-bit, bit k = bar 16*gi+k in [lo, hi])
__device__ __forceinline__ uint32_t rmask(int lo, int hi) {
  const int b0 = 16 * gi();
  int a = lo - b0, b = hi - b0;
  if (a < 0) a = 0;
  if (b > 15) b = 15;
  if (b < a) return 0u;
  return ((0xFFFFu >> (15 - b)) >> a) << a;
}
// first / last set bar of a per-lane 16-bit mask, over the group (-1 when empty)
__device__ __forceinline__ int gfirst(uint32_t m) {
  const int v = m ? 16 * gi() + (int)__builtin_ctz(m) : (1 << 20);
  const int r = gmin_i(v);
  return r == (1 << 20) ? -1 : r;
}
__device__ __forceinline__ int glast(uint32_t m) {
  return gmax_i(m ? 16 * gi() + 31 - (int)__builtin_clz(m) : -1);
}
__device__ __forceinline__ int gcount(uint32_t m) { return gsum_i(__builtin_popcount(m)); }
__device__ __forceinline__ uint32_t gmax_u(uint32_t x) {
  x = max(x, dpp_u<QP_XOR1>(x));
  x = max(x, dpp_u<QP_XOR2>(x));
  x = max(x, dpp_u<ROW_HALF_MIRROR>(x));
  x = max(x, dpp_u<ROW_MIRROR>(x));
  return x;
}
__device__ __forceinline__ uint32_t gmin_u(uint32_t x) {
  x = min(x, dpp_u<QP_XOR1>(x));
  x = min(x, dpp_u<QP_XOR2>(x));
  x = min(x, dpp_u<ROW_HALF_MIRROR>(x));
  x = min(x, dpp_u<ROW_MIRROR>(x));
  return x;
}

// ---- ascending sort of the group's 256 u32 keys (element e = 16*gi + k), bitonic with
// the "flip" merge: every merge of size s starts by comparing e with e ^ (s-1), then
// half-cleans with e ^ j; every compare-exchange is ascending, so in-lane steps are a
// bare v_min_u32 / v_max_u32 pair with compile-time register indices.  Cross-lane
// partners are DPP patterns inside the 16-lane row (xor 1, 2, 3 quad_perm; xor 7
// row_half_mirror; xor 15 row_mirror; xor 8 row_ror:8) except xor 4 (ds_swizzle).
constexpr int QP_XOR3 = 0x1B;   // quad_perm [3,2,1,0]
constexpr int ROW_ROR8 = 0x128;

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_full(uint32_t x) {
  // every source lane is inside the row, so `old` is never used
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t swz_xor4(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (4 << 10));
}
// partner value for lane xor M (M in {1,2,3,4,7,8,15}) of element register x
template <int M>
__device__ __forceinline__ uint32_t gpartner(uint32_t x) {
  // ds_swizzle (bit mode, xor M inside 32 lanes): the exchange runs on the LDS pipe and
  // leaves the VALU (the sorted kernels' limit) to the compare-exchanges
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (M << 10));
}
// one cross-lane step: lane partner g ^ M, register k paired with partner register
// FLIP ? 15-k : k; the lane whose bit LB is clear keeps the minimum
template <int M, int LB, bool FLIP>
__device__ __forceinline__ void gcross(uint32_t (&a)[K]) {
  // one v_med3_u32 per register: med3(x, p, 0) = min, med3(x, p, ~0) = max
  const uint32_t bound = (gi() & LB) == 0 ? 0u : 0xFFFFFFFFu;
  uint32_t p[K];
#pragma unroll
  for (int k = 0; k < K; ++k) p[k] = gpartner<M>(a[FLIP ? K - 1 - k : k]);
#pragma unroll
  for (int k = 0; k < K; ++k) asm("v_med3_u32 %0, %1, %2, %3" : "=v"(a[k]) : "v"(a[k]), "v"(p[k]), "v"(bound));
}
template <int J, bool FLIP>
__device__ __forceinline__ void glocal(uint32_t (&a)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int o = FLIP ? (k ^ (2 * J - 1)) : (k ^ J);
    if (o > k) {
      const uint32_t x = a[k], y = a[o];
      a[k] = min(x, y);
      a[o] = max(x, y);
    }
  }
}
__device__ __forceinline__ void glocal_tail(uint32_t (&a)[K]) {
  glocal<8, false>(a);
  glocal<4, false>(a);
  glocal<2, false>(a);
  glocal<1, false>(a);
}
// the lane's 16 keys ascending by a 60-comparator network (10 layers; checked on all 2^16
// 0-1 inputs) instead of the 80 compare-exchanges of bitonic sizes 2..16
__device__ __forceinline__ void gsort16_lane(uint32_t (&a)[K]) {
  constexpr int8_t net[60][2] = {
      {0, 13}, {1, 12}, {2, 15}, {3, 14}, {4, 8}, {5, 6}, {7, 11}, {9, 10},
      {0, 5}, {1, 7}, {2, 9}, {3, 4}, {6, 13}, {8, 14}, {10, 15}, {11, 12},
      {0, 1}, {2, 3}, {4, 5}, {6, 8}, {7, 9}, {10, 11}, {12, 13}, {14, 15},
      {0, 2}, {1, 3}, {4, 10}, {5, 11}, {6, 7}, {8, 9}, {12, 14}, {13, 15},
      {1, 2}, {3, 12}, {4, 6}, {5, 7}, {8, 10}, {9, 11}, {13, 14},
      {1, 4}, {2, 6}, {5, 8}, {7, 10}, {9, 13}, {11, 14},
      {2, 4}, {3, 6}, {9, 12}, {11, 13},
      {3, 5}, {6, 8}, {7, 9}, {10, 12},
      {3, 4}, {5, 6}, {7, 8}, {9, 10}, {11, 12},
      {6, 7}, {8, 9}};
#pragma unroll
  for (int i = 0; i < 60; ++i) {
    const uint32_t x = a[net[i][0]], y = a[net[i][1]];
    a[net[i][0]] = min(x, y);
    a[net[i][1]] = max(x, y);
  }
}
__device__ __forceinline__ void gsort256u(uint32_t (&a)[K]) {
  // sizes 2..16 inside the lane
  gsort16_lane(a);
  // size 32: flip with lane ^ 1
  gcross<1, 1, true>(a); glocal_tail(a);
  // size 64: flip lane ^ 3, then lane ^ 1
  gcross<3, 2, true>(a); gcross<1, 1, false>(a); glocal_tail(a);
  // size 128: flip lane ^ 7, then ^ 2, ^ 1
  gcross<7, 4, true>(a); gcross<2, 2, false>(a); gcross<1, 1, false>(a); glocal_tail(a);
  // size 256: flip lane ^ 15, then ^ 4, ^ 2, ^ 1
  gcross<15, 8, true>(a); gcross<4, 4, false>(a); gcross<2, 2, false>(a); gcross<1, 1, false>(a);
  glocal_tail(a);
}

}  // namespace g16
}  // namespace mff
