// mff_wave.h — wave64 primitives for one stock-day held in one wavefront.
//
// Layout ("blocked"): lane l (0..59) owns bars m = 4l+0 .. 4l+3 as four register
// slots k = 0..3; lanes 60..63 own nothing.  One float4 load per lane per field plane
// covers the 960 contiguous bytes of a stock-day.
// Presence of every bar is kept wave-uniform as four 64-bit ballots
// (Bits.b[k] bit l == bar 4l+k present), so segment endpoints, window counts and
// first/last bars are scalar bit arithmetic.
//
// Reductions broadcast their result to every lane (xor butterfly: every lane sums the
// same partial sums in mirrored order, so all lanes hold a bitwise-identical value).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mff {

constexpr int WAVE = 64;
constexpr int NBAR = 240;

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63u); }

// ---------------------------------------------------------------- bit casts
__device__ __forceinline__ uint32_t fbits(float x) { return __float_as_uint(x); }
__device__ __forceinline__ float bitsf(uint32_t b) { return __uint_as_float(b); }
__device__ __forceinline__ uint64_t dbits(double x) { return (uint64_t)__double_as_longlong(x); }
__device__ __forceinline__ double bitsd(uint64_t b) { return __longlong_as_double((long long)b); }

__device__ __forceinline__ double qnan() { return __longlong_as_double(0x7ff8000000000000ll); }

// S11: polars compares floats in total order: NaN is above every number.
__device__ __forceinline__ bool tot_gt(double a, double b) {
  return (a > b) || (__builtin_isnan(a) && !__builtin_isnan(b));
}
__device__ __forceinline__ bool tot_lt(double a, double b) { return tot_gt(b, a); }
__device__ __forceinline__ bool tot_ne(double a, double b) {
  bool an = __builtin_isnan(a), bn = __builtin_isnan(b);
  return (an || bn) ? !(an && bn) : (a != b);
}

// ---------------------------------------------------------------- cross-lane moves
__device__ __forceinline__ int bperm_i(int src, int v) {
  return __builtin_amdgcn_ds_bpermute(src << 2, v);
}
__device__ __forceinline__ uint32_t bperm(int src, uint32_t v) { return (uint32_t)bperm_i(src, (int)v); }
__device__ __forceinline__ float bperm(int src, float v) {
  return __int_as_float(bperm_i(src, __float_as_int(v)));
}
__device__ __forceinline__ double bperm(int src, double v) {
  uint64_t b = dbits(v);
  int lo = bperm_i(src, (int)(uint32_t)b), hi = bperm_i(src, (int)(uint32_t)(b >> 32));
  return bitsd(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ uint64_t bperm(int src, uint64_t v) {
  int lo = bperm_i(src, (int)(uint32_t)v), hi = bperm_i(src, (int)(uint32_t)(v >> 32));
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

// value of a wave-uniform lane
__device__ __forceinline__ float rdlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ uint32_t rdlane(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ double rdlane(double v, int l) {
  uint64_t b = dbits(v);
  uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
  uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
  return bitsd(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint64_t rdlane(uint64_t v, int l) {
  uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// 32-bit words of a lane value (DPP carries, element picks)
template <typename T> struct Words;
template <> struct Words<uint32_t> {
  static constexpr int N = 1;
  __device__ static void split(uint32_t x, uint32_t* w) { w[0] = x; }
  __device__ static uint32_t join(const uint32_t* w) { return w[0]; }
};
template <> struct Words<float> {
  static constexpr int N = 1;
  __device__ static void split(float x, uint32_t* w) { w[0] = __float_as_uint(x); }
  __device__ static float join(const uint32_t* w) { return __uint_as_float(w[0]); }
};
template <> struct Words<double> {
  static constexpr int N = 2;
  __device__ static void split(double x, uint32_t* w) {
    const uint64_t b = dbits(x);
    w[0] = (uint32_t)b;
    w[1] = (uint32_t)(b >> 32);
  }
  __device__ static double join(const uint32_t* w) { return bitsd(((uint64_t)w[1] << 32) | w[0]); }
};
template <> struct Words<uint64_t> {
  static constexpr int N = 2;
  __device__ static void split(uint64_t b, uint32_t* w) {
    w[0] = (uint32_t)b;
    w[1] = (uint32_t)(b >> 32);
  }
  __device__ static uint64_t join(const uint32_t* w) { return ((uint64_t)w[1] << 32) | w[0]; }
};
// element e (wave-uniform) of a blocked 4-slot array: the four slots of lane e / 4 read
// into scalars, then a scalar pick (a select chain on the vector slots is folded into an
// indexed load, which pins the array in private memory: scratch)
template <typename T>
__device__ __forceinline__ T elem(const T (&x)[4], int e) {
  const int k = e & 3, l = e >> 2;
  const T a0 = rdlane(x[0], l), a1 = rdlane(x[1], l), a2 = rdlane(x[2], l), a3 = rdlane(x[3], l);
  return k == 0 ? a0 : k == 1 ? a1 : k == 2 ? a2 : a3;
}

// ---------------------------------------------------------------- reductions
// (defined after the DPP helpers below)
__device__ __forceinline__ double wsum(double x);
__device__ __forceinline__ double wprod(double x);
__device__ __forceinline__ uint32_t wsum_u32(uint32_t x);

// ---------------------------------------------------------------- DPP scans / reductions
// GFX9 DPP: row_shr:1/2/4/8 inside each 16-lane row (Hillis-Steele), then row_bcast:15 into
// rows 1 and 3 and row_bcast:31 into rows 2 and 3 -- one VALU op per step, no LDS.  Lanes
// without a source (and rows outside the row mask) read `id`.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x, uint32_t id) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, CTRL, ROW_MASK, 0xF, false);
}
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_f64(double x, double id) {
  const uint64_t b = dbits(x), i = dbits(id);
  const uint32_t lo = dpp_u32<CTRL, ROW_MASK>((uint32_t)b, (uint32_t)i);
  const uint32_t hi = dpp_u32<CTRL, ROW_MASK>((uint32_t)(b >> 32), (uint32_t)(i >> 32));
  return bitsd(((uint64_t)hi << 32) | lo);
}
// inclusive prefix sum over the first 16 lanes (lanes >= 16: their row's prefix)
__device__ __forceinline__ uint32_t wscan16_dpp(uint32_t x) {
  x += dpp_u32<0x111, 0xF>(x, 0u);
  x += dpp_u32<0x112, 0xF>(x, 0u);
  x += dpp_u32<0x114, 0xF>(x, 0u);
  x += dpp_u32<0x118, 0xF>(x, 0u);
  return x;
}
// inclusive prefix sum over the 64 lanes
__device__ __forceinline__ uint32_t wscan_dpp(uint32_t x) {
  x = wscan16_dpp(x);
  x += dpp_u32<0x142, 0xA>(x, 0u);
  x += dpp_u32<0x143, 0xC>(x, 0u);
  return x;
}
// all-reduce: a DPP butterfly inside each 16-lane row (quad_perm xor 1, xor 2,
// row_half_mirror, row_mirror: every lane of a row ends with the row total, bitwise
// identical -- each step adds the same two partial sums in either order), then the four
// row totals by readlane, combined in one fixed order: every lane gets the same bits.
// A few cycles per step instead of a round trip through the LDS crossbar per step (the
// ds_bpermute of __shfl_xor).  Call in wave-uniform control flow.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_in_row(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_in_row(double x) {
  const uint64_t b = dbits(x);
  const uint32_t lo = dpp_in_row<CTRL>((uint32_t)b), hi = dpp_in_row<CTRL>((uint32_t)(b >> 32));
  return bitsd(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double wsum(double x) {
  x += dpp_in_row<0xB1>(x);
  x += dpp_in_row<0x4E>(x);
  x += dpp_in_row<0x141>(x);
  x += dpp_in_row<0x140>(x);
  const double a = rdlane(x, 0), b = rdlane(x, 16), c = rdlane(x, 32), d = rdlane(x, 48);
  return (a + b) + (c + d);
}
__device__ __forceinline__ double wprod(double x) {
  x *= dpp_in_row<0xB1>(x);
  x *= dpp_in_row<0x4E>(x);
  x *= dpp_in_row<0x141>(x);
  x *= dpp_in_row<0x140>(x);
  const double a = rdlane(x, 0), b = rdlane(x, 16), c = rdlane(x, 32), d = rdlane(x, 48);
  return (a * b) * (c * d);
}
__device__ __forceinline__ uint32_t wsum_u32(uint32_t x) {
  x += dpp_in_row<0xB1>(x);
  x += dpp_in_row<0x4E>(x);
  x += dpp_in_row<0x141>(x);
  x += dpp_in_row<0x140>(x);
  return rdlane(x, 0) + rdlane(x, 16) + rdlane(x, 32) + rdlane(x, 48);
}
// value of lane l - 1 (lane 0: id), DPP wave_shr:1
__device__ __forceinline__ uint32_t wave_shr1(uint32_t x, uint32_t id) { return dpp_u32<0x138, 0xF>(x, id); }
__device__ __forceinline__ double wave_shr1(double x, double id) { return dpp_f64<0x138, 0xF>(x, id); }
__device__ __forceinline__ float wave_shr1(float x, float id) {
  return __uint_as_float(dpp_u32<0x138, 0xF>(__float_as_uint(x), __float_as_uint(id)));
}

// wave min and max of non-NaN doubles, returned in every lane
__device__ __forceinline__ void wminmax_dpp(double& lo, double& hi) {
  const double pinf = __builtin_inf(), ninf = -__builtin_inf();
#define MFF_MINMAX_STEP(C, R)                         \
  {                                                   \
    const double a = dpp_f64<C, R>(lo, pinf);         \
    const double b = dpp_f64<C, R>(hi, ninf);         \
    lo = a < lo ? a : lo;                             \
    hi = b > hi ? b : hi;                             \
  }
  MFF_MINMAX_STEP(0x111, 0xF)
  MFF_MINMAX_STEP(0x112, 0xF)
  MFF_MINMAX_STEP(0x114, 0xF)
  MFF_MINMAX_STEP(0x118, 0xF)
  MFF_MINMAX_STEP(0x142, 0xA)
  MFF_MINMAX_STEP(0x143, 0xC)
#undef MFF_MINMAX_STEP
  lo = rdlane(lo, 63);
  hi = rdlane(hi, 63);
}

// ---------------------------------------------------------------- presence bits
struct Bits {
  uint64_t b[4];
};

__device__ __forceinline__ Bits ballot4(const bool (&p)[4]) {
  Bits r;
#pragma unroll
  for (int k = 0; k < 4; ++k) r.b[k] = __ballot(p[k]);
  return r;
}
__device__ __forceinline__ int count(const Bits& B) {
  return __popcll(B.b[0]) + __popcll(B.b[1]) + __popcll(B.b[2]) + __popcll(B.b[3]);
}
__device__ __forceinline__ bool any(const Bits& B) { return (B.b[0] | B.b[1] | B.b[2] | B.b[3]) != 0; }
// (a scalar pick of the word: an indexed B.b[m & 3] pins the four words in scratch)
__device__ __forceinline__ bool test(const Bits& B, int m) {
  const int k = m & 3;
  const uint64_t w = k == 0 ? B.b[0] : k == 1 ? B.b[1] : k == 2 ? B.b[2] : B.b[3];
  return (w >> (m >> 2)) & 1ull;
}
// first / last set element index (4l+k), -1 when empty
__device__ __forceinline__ int first_of(const Bits& B) {
  int best = 1 << 20;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (B.b[k]) best = min(best, 4 * (int)__builtin_ctzll(B.b[k]) + k);
  return best == (1 << 20) ? -1 : best;
}
__device__ __forceinline__ int last_of(const Bits& B) {
  int best = -1;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (B.b[k]) best = max(best, 4 * (63 - (int)__builtin_clzll(B.b[k])) + k);
  return best;
}
// bars in [lo, hi] (inclusive), as Bits
__device__ __forceinline__ Bits range_bits(int lo, int hi) {
  Bits R;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    int l0 = (lo - k + 3) >> 2;  // ceil((lo-k)/4), lo-k >= -3
    if (lo - k < 0) l0 = 0;
    int l1 = (hi - k) >> 2;      // floor((hi-k)/4)
    if (hi - k < 0) l1 = -1;
    uint64_t m = 0;
    if (l1 >= l0) {
      uint64_t upto = (l1 >= 63) ? ~0ull : ((1ull << (l1 + 1)) - 1);
      uint64_t below = (l0 <= 0) ? 0ull : ((1ull << l0) - 1);
      m = upto & ~below;
    }
    R.b[k] = m;
  }
  return R;
}
__device__ __forceinline__ Bits band(const Bits& A, const Bits& B) {
  Bits R;
#pragma unroll
  for (int k = 0; k < 4; ++k) R.b[k] = A.b[k] & B.b[k];
  return R;
}
// this lane's slot k membership
__device__ __forceinline__ bool mine(const Bits& B, int k) { return (B.b[k] >> lane_id()) & 1ull; }

// ---------------------------------------------------------------- scans
// inclusive prefix over all 64 lanes: DPP row_shr 1/2/4/8 inside the rows, then
// row_bcast:15 / row_bcast:31 across them (wscan_dpp's steps)
__device__ __forceinline__ double wscan_incl(double x) {
  x += dpp_f64<0x111, 0xF>(x, 0.0);
  x += dpp_f64<0x112, 0xF>(x, 0.0);
  x += dpp_f64<0x114, 0xF>(x, 0.0);
  x += dpp_f64<0x118, 0xF>(x, 0.0);
  x += dpp_f64<0x142, 0xA>(x, 0.0);
  x += dpp_f64<0x143, 0xC>(x, 0.0);
  return x;
}
__device__ __forceinline__ uint32_t wscan_incl_u32(uint32_t x) { return wscan_dpp(x); }
// inclusive prefix over the 256 blocked elements (bar order)
__device__ __forceinline__ void scan4(double (&v)[4]) {
  v[1] += v[0];
  v[2] += v[1];
  v[3] += v[2];
  const double ex = wave_shr1(wscan_incl(v[3]), 0.0);
  v[0] += ex; v[1] += ex; v[2] += ex; v[3] += ex;
}
__device__ __forceinline__ void scan4_u32(uint32_t (&v)[4]) {
  v[1] += v[0];
  v[2] += v[1];
  v[3] += v[2];
  const uint32_t ex = wave_shr1(wscan_incl_u32(v[3]), 0u);
  v[0] += ex; v[1] += ex; v[2] += ex; v[3] += ex;
}

// For each element: the value of the nearest PREVIOUS element with flag set
// (polars shift(1) / pct_change over present rows, S4/S5).
// the lane's last / first flagged slot value (slot 0 / 3 when none), by integer bit
// blends: the select chain on per-lane flags is otherwise folded into an indexed load from
// a private copy of the array (scratch)
template <typename T>
__device__ __forceinline__ T last_flagged(const T (&x)[4], const bool (&f)[4]) {
  using W = Words<T>;
  uint32_t r[W::N], w[W::N];
  W::split(x[0], r);
#pragma unroll
  for (int j = 1; j < 4; ++j) {
    W::split(x[j], w);
    const uint32_t m = 0u - (uint32_t)f[j];
#pragma unroll
    for (int i = 0; i < W::N; ++i) r[i] = (w[i] & m) | (r[i] & ~m);
  }
  return W::join(r);
}
template <typename T>
__device__ __forceinline__ T first_flagged(const T (&x)[4], const bool (&f)[4]) {
  using W = Words<T>;
  uint32_t r[W::N], w[W::N];
  W::split(x[3], r);
#pragma unroll
  for (int j = 2; j >= 0; --j) {
    W::split(x[j], w);
    const uint32_t m = 0u - (uint32_t)f[j];
#pragma unroll
    for (int i = 0; i < W::N; ++i) r[i] = (w[i] & m) | (r[i] & ~m);
  }
  return W::join(r);
}
// one carry step: take the (value, flag) of the source lane of CTRL (rows ROW_MASK) when
// this lane has no flag yet; lanes without a source read flag 0
template <int CTRL, int ROW_MASK, int N>
__device__ __forceinline__ void carry_step(uint32_t (&w)[N], uint32_t& h) {
  const uint32_t oh = dpp_u32<CTRL, ROW_MASK>(h, 0u);
  uint32_t ow[N];
#pragma unroll
  for (int i = 0; i < N; ++i) ow[i] = dpp_u32<CTRL, ROW_MASK>(w[i], 0u);
  if (!h && oh) {
#pragma unroll
    for (int i = 0; i < N; ++i) w[i] = ow[i];
    h = 1u;
  }
}
// For each element: the value of the nearest PREVIOUS element with flag set
// (polars shift(1) / pct_change over present rows, S4/S5): per lane its last flagged
// value, a DPP carry over the lanes (row_shr 1/2/4/8, row_bcast:15 / 31, then wave_shr:1
// for the lanes before), then a walk over the lane's four slots.
template <typename T>
__device__ __forceinline__ void prev_valid(const T (&x)[4], const bool (&f)[4], T (&prev)[4], bool (&has)[4]) {
  using W = Words<T>;
  constexpr int N = W::N;
  uint32_t h = (f[0] | f[1] | f[2] | f[3]) ? 1u : 0u;
  uint32_t w[N];
  W::split(last_flagged(x, f), w);
  carry_step<0x111, 0xF>(w, h);
  carry_step<0x112, 0xF>(w, h);
  carry_step<0x114, 0xF>(w, h);
  carry_step<0x118, 0xF>(w, h);
  carry_step<0x142, 0xA>(w, h);
  carry_step<0x143, 0xC>(w, h);
  uint32_t pw[N];
#pragma unroll
  for (int i = 0; i < N; ++i) pw[i] = wave_shr1(w[i], 0u);
  T cv = W::join(pw);
  bool ch = wave_shr1(h, 0u) != 0u;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    prev[k] = cv;
    has[k] = ch;
    if (f[k]) { cv = x[k]; ch = true; }
  }
}
// nearest NEXT element with flag set (polars shift(-1))
template <typename T>
__device__ __forceinline__ void next_valid(const T (&x)[4], const bool (&f)[4], T (&next)[4], bool (&has)[4]) {
  const int l = lane_id();
  bool lh = f[0] | f[1] | f[2] | f[3];
  T lv = first_flagged(x, f);
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T ov = __shfl_down(lv, o);
    int oh = __shfl_down((int)lh, o);
    if (l + o < 64 && !lh) { lv = ov; lh = oh != 0; }
  }
  T cv = __shfl_down(lv, 1);
  bool ch = __shfl_down((int)lh, 1) != 0;
  if (l == 63) ch = false;
#pragma unroll
  for (int k = 3; k >= 0; --k) {
    next[k] = cv;
    has[k] = ch;
    if (f[k]) { cv = x[k]; ch = true; }
  }
}

// ---------------------------------------------------------------- bitonic sort
// Ascending sort of the 256 blocked elements (e = 4*lane + k).
template <typename K>
__device__ __forceinline__ void cmpx_local(K& a, K& b, bool up) {
  bool sw = up ? (a > b) : (a < b);
  K t = a;
  a = sw ? b : a;
  b = sw ? t : b;
}
template <typename K>
__device__ __forceinline__ void bitonic256(K (&a)[4]) {
  const int l = lane_id();
#pragma unroll
  for (int size = 2; size <= 256; size <<= 1) {
#pragma unroll
    for (int j = size >> 1; j > 0; j >>= 1) {
      if (j >= 4) {
        const int lj = j >> 2;
        const bool lower = (l & lj) == 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int e = 4 * l + k;
          const bool up = (e & size) == 0;
          K p = __shfl_xor(a[k], lj);
          K mn = a[k] < p ? a[k] : p;
          K mx = a[k] < p ? p : a[k];
          a[k] = (lower == up) ? mn : mx;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if ((k & j) == 0) {
            const int e = 4 * l + k;
            cmpx_local(a[k], a[k | j], (e & size) == 0);
          }
        }
      }
    }
  }
}

// f64 total-order image as u64 (ascending u64 == ascending total order; -0 == +0)
__device__ __forceinline__ uint64_t ord64(double x) {
  if (x == 0.0) x = 0.0;
  uint64_t b = dbits(x);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double unord64(uint64_t k) {
  uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return bitsd(b);
}

}  // namespace mff
