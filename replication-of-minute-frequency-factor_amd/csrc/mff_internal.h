// mff_internal.h — shared host-side plumbing of libmff.so (error slot, launch checks).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

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
extern const uint32_t kFactorFamily[NF];
// first catalogue id of doc_pdf60..95
constexpr int PDF0 = 42;

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace mff
