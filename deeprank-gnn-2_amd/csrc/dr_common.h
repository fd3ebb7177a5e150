// Shared device helpers for the deeprank2_amd HIP kernels (gfx950, wave64).
#pragma once

#include <hip/hip_runtime.h>

#include <mutex>

#define DR_CHECK(expr)                 \
  do {                                 \
    const int _e = (int)(expr);        \
    if (_e != 0) return _e;            \
  } while (0)

// Sum over the 64 lanes of a wave (butterfly; every lane gets the total).
__device__ __forceinline__ float dr_wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Allow up to the full 160 KiB of LDS for a kernel; done once per kernel
// (hipFuncSetAttribute is not a stream operation, so it stays out of capture).
inline int dr_allow_big_lds(const void* fn) {
  static std::mutex mu;
  static const void* done[64] = {nullptr};
  static int n_done = 0;
  std::lock_guard<std::mutex> lock(mu);
  for (int i = 0; i < n_done; ++i)
    if (done[i] == fn) return 0;
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e != hipSuccess) return (int)e;
  if (n_done < 64) done[n_done++] = fn;
  return 0;
}
