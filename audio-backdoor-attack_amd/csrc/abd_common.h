// Shared helpers for the libabd HIP sources (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../../include/abd.h"

namespace abd {

void set_last_error(const char* fmt, ...);

#define ABD_HIP(expr)                                                                 \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess) {                                                           \
      ::abd::set_last_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr,              \
                            hipGetErrorString(e_));                                   \
      return (int)e_;                                                                 \
    }                                                                                 \
  } while (0)

#define ABD_CHECK(cond, code, ...)                                                    \
  do {                                                                                \
    if (!(cond)) {                                                                    \
      ::abd::set_last_error(__VA_ARGS__);                                             \
      return (code);                                                                  \
    }                                                                                 \
  } while (0)

// Launch check: hipGetLastError after an async launch (no sync, graph-capture safe).
#ifdef ABD_DEBUG_SYNC  // measurement builds only: every launch completes before the next is issued
#define ABD_LAUNCH_CHECK() \
  do {                     \
    ABD_HIP(hipGetLastError()); \
    ABD_HIP(hipDeviceSynchronize()); \
  } while (0)
#else
#define ABD_LAUNCH_CHECK() ABD_HIP(hipGetLastError())
#endif

constexpr int kWave = 64;

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Bijective XCD-aware remap (cdna_hip_programming.md T1): blocks that share an XCD
// (b % 8 equal) get contiguous logical ids, so neighbouring work shares an L2.
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int xcd = bid & 7;
  const int q = nblocks >> 3, r = nblocks & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

}  // namespace abd
