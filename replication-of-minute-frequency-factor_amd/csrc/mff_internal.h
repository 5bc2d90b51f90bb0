// mff_internal.h — shared host-side plumbing of libmff.so (error slot, launch checks).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/mff.h"

namespace mff {

// thread-local last error (mff_last_error)
void set_error(const char* fmt, ...);
void clear_error();

#define MFF_REQUIRE(cond, ...)          \
  do {                                  \
    if (!(cond)) {                      \
      ::mff::set_error(__VA_ARGS__);    \
      return -1;                        \
    }                                   \
  } while (0)

#define MFF_HIP(call)                                                        \
  do {                                                                       \
    hipError_t e_ = (call);                                                  \
    if (e_ != hipSuccess) {                                                  \
      ::mff::set_error("%s failed: %s", #call, hipGetErrorString(e_));       \
      return -2;                                                             \
    }                                                                        \
  } while (0)

#define MFF_LAUNCH_CHECK()                                                   \
  do {                                                                       \
    hipError_t e_ = hipGetLastError();                                       \
    if (e_ != hipSuccess) {                                                  \
      ::mff::set_error("kernel launch failed: %s", hipGetErrorString(e_));   \
      return -2;                                                             \
    }                                                                        \
  } while (0)

// doc_pdf level buffer header (pdf_levels_split in mff_stage1g.hip): per day a u64
// counter (list A count low, list B high), then the u64 split key of this pass's lists
// at pdf_koff(D) (keys below it in list A)
__host__ __device__ inline size_t pdf_koff(int D) { return (size_t)8 * (size_t)D; }
// level-list slots per day: one level per distinct close of a stock-day, at most its rows
// -- 240 grid bars, or MFF_ROWS_MAX = 255 rows of a row-set stock-day (the host rejects
// more) -- so S x 256 slots hold lists A and B of any day; a multiple of 16 entries, so
// every day's keys start 128-B and its weight bytes 16-B aligned (the count's vector loads)
__host__ __device__ inline size_t pdf_day_cap(int S) { return (size_t)S * 256; }
static_assert(MFF_ROWS_MAX <= 256, "pdf_day_cap holds MFF_ROWS_MAX levels per stock-day");
__device__ inline uint64_t pdf_split_key(const uint32_t* lvl_count, int D) {
  return *reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(lvl_count) + pdf_koff(D));
}
// sets this pass's split key in the header (mff_pdf.hip): the key learned from the
// previous passes' doc_pdf queries (their per-day median), 1.0 before any
int pdf_split_init(uint32_t* lvl_count, int D, hipStream_t st);

// factor families (the kernel section that computes a factor); bit per family
enum Fam : uint32_t {
  F_SEG = 1u << 0,
  F_OLS = 1u << 1,
  F_ORD = 1u << 2,
  F_MOMV = 1u << 3,
  F_MOMH = 1u << 4,
  F_MOMR = 1u << 5,
  F_SUMC = 1u << 6,
  F_SUMV = 1u << 7,
  F_CORR = 1u << 8,
  F_LVL = 1u << 9,
  F_PDF = 1u << 10,
  F_ORDV = 1u << 11,
  F_TRD = 1u << 12,
};

constexpr int NF = 58;
extern const char* const kFactorNames[NF];
// first catalogue id of doc_pdf60..95
constexpr int PDF0 = 42;
inline constexpr uint32_t kFactorFamily[NF] = {
    F_SEG, F_SEG, F_SEG, F_SEG, F_SEG,
    F_OLS, F_OLS, F_OLS, F_OLS, F_OLS,
    F_ORD, F_ORD, F_ORD, F_ORD,
    F_MOMV, F_MOMH, F_MOMR, F_MOMR, F_MOMR, F_MOMR, F_MOMR,
    F_MOMR, F_MOMR, F_MOMR, F_MOMV, F_MOMV, F_MOMV,
    F_SUMC, F_SUMV, F_SUMV, F_SUMV, F_SUMV, F_SUMV,
    F_CORR, F_CORR, F_CORR, F_CORR, F_CORR, F_CORR,
    F_LVL, F_LVL, F_LVL, F_PDF, F_PDF, F_PDF, F_PDF, F_PDF,
    F_ORDV, F_ORDV, F_ORDV,
    F_TRD, F_TRD, F_SUMV, F_SUMV, F_TRD, F_TRD, F_TRD, F_TRD,
};
// kFactorFamily[f] as a constant expression for device code (catalogue order, CM:12-1381)
__host__ __device__ constexpr uint32_t kFamOf(int f) {
  return f < 5 ? F_SEG : f < 10 ? F_OLS : f < 14 ? F_ORD : f == 14 ? F_MOMV : f == 15 ? F_MOMH
       : f < 24 ? F_MOMR : f < 27 ? F_MOMV : f == 27 ? F_SUMC : f < 33 ? F_SUMV : f < 39 ? F_CORR
       : f < 42 ? F_LVL : f < 47 ? F_PDF : f < 50 ? F_ORDV : f < 52 ? F_TRD : f < 54 ? F_SUMV : F_TRD;
}

// The one field -> families table: kFieldFams[p] = the families whose values read field p
// (open, high, low, close, volume).  Every grid kernel loads a field only for families
// listed here (the serial kernels' planes kPlanes derive from it; the group kernel's load
// predicates are checked against it), and a kept row-set stock-day's null field sends
// exactly these families to mff_stage1_rows (rows_fams): a family the table misses for a
// field would be stored by a grid kernel from that field's fill values under a null.
inline constexpr uint32_t kFieldFams[5] = {
    F_SEG | F_ORD | F_MOMR | F_TRD,                                              // open
    F_OLS | F_MOMH,                                                              // high
    F_OLS | F_MOMH,                                                              // low
    F_SEG | F_ORD | F_MOMR | F_SUMC | F_CORR | F_LVL | F_PDF | F_TRD,            // close
    F_ORD | F_MOMV | F_SUMC | F_SUMV | F_CORR | F_LVL | F_PDF | F_ORDV | F_TRD,   // volume
};
// the fields (bit p) the families of `set` read
__host__ __device__ constexpr uint32_t fields_of(uint32_t set) {
  return ((set & kFieldFams[0]) ? 1u : 0u) | ((set & kFieldFams[1]) ? 2u : 0u) | ((set & kFieldFams[2]) ? 4u : 0u) |
         ((set & kFieldFams[3]) ? 8u : 0u) | ((set & kFieldFams[4]) ? 16u : 0u);
}

// Row set (include/mff.h): the families mff_stage1_rows computes for a stock-day with
// row-set flags `fl` (valid word 7, or its first row's `reserved`): every family, unless
// the grid bars are kept (MFF_ROWS_KEEP) -- then those reading a field that holds a null
// (kFieldFams)
__host__ __device__ constexpr uint32_t rows_fams(uint32_t fl) {
  const uint32_t nb = (fl >> MFF_ROWS_NULL_SHIFT) & 31u;
  return !(fl & MFF_ROWS_KEEP) ? ~0u
         : ((nb & 1u) ? kFieldFams[0] : 0u) | ((nb & 2u) ? kFieldFams[1] : 0u) | ((nb & 4u) ? kFieldFams[2] : 0u) |
           ((nb & 8u) ? kFieldFams[3] : 0u) | ((nb & 16u) ? kFieldFams[4] : 0u);
}
// the families a grid kernel must not store for a stock-day whose valid word 7 is w7
__host__ __device__ constexpr uint32_t grid_skip(uint32_t w7) { return (w7 & MFF_ROWS_LISTED) ? rows_fams(w7) : 0u; }

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace mff
