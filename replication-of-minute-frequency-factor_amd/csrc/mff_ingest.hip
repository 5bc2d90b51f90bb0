// mff_ingest.hip — long day-frame rows -> dense panel in HBM.
//
// The reference reads one parquet day file per task (MinuteFrequentFactorCICC.py:22) and
// every cal_* works on its long rows (code, date, time, open, high, low, close, volume);
// minute_in_trade (MinuteFrequentFactorCalculateMethodsCICC.py:98-106) is the time ->
// minute map of the 240-bar grid 09:30-11:29, 13:00-14:59.  Here the host only encodes
// code / date to dense indices (sorted universes) and ships the numeric columns; this
// kernel maps time -> minute, casts the f64 prices to the fp32 planes and the volume to
// the u32 share plane ([5][D][S][240], 4 B a bar each),
// sets the presence bits [D][S][8] and checks the engine's input contract (include/mff.h)
// on the fly, counting violations instead of trapping.
//
// One thread per row, grid-stride over 256-row blocks.  Rows of a day file arrive in
// (code, time) order (C4), so a wave's 64 rows are 64 consecutive minutes of at most a
// few stock-days: the fp32 stores coalesce and the 64 presence bits fall in <= 3 mask
// words.  The bits are OR-combined per distinct word inside the wave (leader loop:
// ballot of the lanes sharing the leader's word, DPP/bpermute OR-reduction) and one
// atomicOr per word and wave goes to HBM; its old value exposes duplicates across waves,
// the popcount of the combined bits duplicates inside the wave.  Unsorted input stays
// correct (more leader iterations).  HBM-bound byte work: 56 B read (4+4 index, 8 time,
// 4x8 prices, 8 volume) + 20 B written per row, plus 4 B of atomics per mask word.
#include "../../include/mff.h"
#include "mff_internal.h"
#include "mff_wave.h"

namespace mff {

enum IngestErr { IE_INDEX = 0, IE_TIME = 1, IE_DUP = 2, IE_PRICE = 3, IE_VOLUME = 4 };

struct IngestArgs {
  const int32_t* stock;
  const int32_t* day;
  const int64_t* time;
  const double* px[4];  // open high low close
  const void* vol;
  int vol_kind;
  int64_t n;
  int S, D;
  float* bars;  // [5][D][S][240]
  uint32_t* mask;
  uint32_t* err;
};

// HHMMSSmmm -> 0..239, or -1 off the grid (start-labelled bars, CM:98-106)
__device__ __forceinline__ int minute_of(int64_t t) {
  if (t < 0 || t >= 240000000ll) return -1;
  const int ti = (int)t;
  const int hh = ti / 10000000, mm = (ti / 100000) % 100, rest = ti % 100000;
  const int clock = hh * 60 + mm;
  if (rest != 0 || mm >= 60) return -1;
  if (clock >= 570 && clock < 690) return clock - 570;
  if (clock >= 780 && clock < 900) return clock - 660;
  return -1;
}

__device__ __forceinline__ double load_volume(const void* p, int kind, int64_t i) {
  switch (kind) {
    case MFF_VOLUME_F64: return reinterpret_cast<const double*>(p)[i];
    case MFF_VOLUME_I64: return (double)reinterpret_cast<const int64_t*>(p)[i];
    case MFF_VOLUME_F32: return (double)reinterpret_cast<const float*>(p)[i];
    default: return (double)reinterpret_cast<const int32_t*>(p)[i];
  }
}

__device__ __forceinline__ uint32_t wave_or(uint32_t x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x |= (uint32_t)__shfl_xor((int)x, o, 64);
  return x;
}

__global__ __launch_bounds__(256) void k_ingest(IngestArgs a) {
  const int lane = lane_id();
  const size_t plane = (size_t)a.D * a.S * 240;
  uint32_t e_idx = 0, e_time = 0, e_dup = 0, e_px = 0, e_vol = 0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t base = (int64_t)blockIdx.x * 256; base < a.n; base += stride) {
    const int64_t i = base + threadIdx.x;
    bool ok = i < a.n;
    size_t sd = 0;
    int m = 0;
    if (ok) {
      const int s = a.stock[i], d = a.day[i];
      m = minute_of(a.time[i]);
      const bool in = s >= 0 && s < a.S && d >= 0 && d < a.D;
      e_idx += in ? 0u : 1u;
      e_time += (in && m < 0) ? 1u : 0u;
      ok = in && m >= 0;
      if (ok) {
        sd = (size_t)d * a.S + s;
        const size_t cell = sd * 240 + m;
        bool bad = false;
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const double x = a.px[f][i];
          bad |= !(x > 0.0 && x <= 3.4028234663852886e38);  // finite > 0, fp32-representable
          a.bars[f * plane + cell] = (float)x;
        }
        const double v = load_volume(a.vol, a.vol_kind, i);
        e_px += bad ? 1u : 0u;
        const bool vok = v >= 0.0 && v <= (double)MFF_VOLUME_MAX && v == rint(v);
        e_vol += vok ? 0u : 1u;
        reinterpret_cast<uint32_t*>(a.bars)[4 * plane + cell] = vok ? (uint32_t)v : 0u;
      }
    }
    // presence bits: one atomicOr per distinct mask word of this wave
    const size_t word = sd * 8 + (m >> 5);  // mask [D][S][8]
    const uint32_t bit = ok ? (1u << (m & 31)) : 0u;
    uint64_t todo = __ballot(ok);
    while (todo) {
      const int leader = __ffsll((long long)todo) - 1;
      const size_t wl = ((size_t)(uint32_t)__shfl((int)(uint32_t)(word >> 32), leader, 64) << 32) |
                        (uint32_t)__shfl((int)(uint32_t)word, leader, 64);
      const bool mine = ok && word == wl;
      const uint64_t grp = __ballot(mine);
      const uint32_t orv = wave_or(mine ? bit : 0u);
      if (lane == leader) {
        const uint32_t old = atomicOr(a.mask + wl, orv);
        e_dup += (uint32_t)(__popcll(grp) - __popc(orv)) + (uint32_t)__popc(old & orv);
      }
      todo &= ~grp;
    }
  }
  const uint32_t cnt[5] = {e_idx, e_time, e_dup, e_px, e_vol};
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const uint32_t t = wsum_u32(cnt[k]);
    if (lane == 0 && t != 0u) atomicAdd(a.err + k, t);
  }
}

}  // namespace mff

extern "C" {

int mff_ingest_rows(const int32_t* stock, const int32_t* day, const int64_t* time,
                    const double* open, const double* high, const double* low,
                    const double* close, const void* volume, int volume_kind, int64_t nrows,
                    int S, int D, float* bars, uint32_t* valid, uint32_t* errors, void* stream) {
  using namespace mff;
  clear_error();
  MFF_REQUIRE(nrows >= 0 && S > 0 && D > 0, "mff_ingest_rows: bad sizes (nrows=%lld S=%d D=%d)",
              (long long)nrows, S, D);
  MFF_REQUIRE(volume_kind >= MFF_VOLUME_F64 && volume_kind <= MFF_VOLUME_I32,
              "mff_ingest_rows: unknown volume_kind %d", volume_kind);
  MFF_REQUIRE(bars && valid && errors, "mff_ingest_rows: null output pointer");
  if (nrows == 0) return 0;
  MFF_REQUIRE(stock && day && time && open && high && low && close && volume,
              "mff_ingest_rows: null input pointer");
  IngestArgs a{stock, day, time, {open, high, low, close}, volume, volume_kind, nrows, S, D,
               bars, valid, errors};
  const int64_t blocks = (nrows + 255) / 256;
  const int grid = (int)(blocks < 8192 ? blocks : 8192);  // 32 blocks per CU, grid-stride
  hipLaunchKernelGGL(k_ingest, dim3(grid), dim3(256), 0, as_stream(stream), a);
  MFF_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
