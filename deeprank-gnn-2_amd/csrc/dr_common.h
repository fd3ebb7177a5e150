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

// threadIdx.x, opaque to the optimiser when OPAQUE: a kernel that loops a
// body over several work items (ginet_acc_kernel) would otherwise get the
// body's thread-index arithmetic hoisted out of the loop and kept live across
// it, past the register budget (spills).
template <bool OPAQUE>
__device__ __forceinline__ int dr_tid() {
  int t = threadIdx.x;
  if (OPAQUE) {
    asm volatile("; dr_tid" : "+v"(t));
    __builtin_assume(t >= 0 && t < 1024);  // (the range threadIdx.x has under any launch bound here)
  }
  return t;
}

// the wave index of thread tid, wave-uniform (an SGPR) also when tid came
// from dr_tid<true> (the optimiser no longer sees it derive from threadIdx.x)
template <bool OPAQUE>
__device__ __forceinline__ int dr_wave(int tid) {
  return OPAQUE ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6;
}

// Lane permutations on the DPP path (a VALU operand modifier, no LDS round
// trip as ds_bpermute has): CTRL is the gfx9 dpp_ctrl (0xB1 quad_perm
// [1,0,3,2] = lane^1, 0x4E quad_perm [2,3,0,1] = lane^2, 0x141
// row_half_mirror = 7-i within 8 lanes, 0x140 row_mirror = 15-i within 16).
template <int CTRL>
__device__ __forceinline__ float dr_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Sum over each aligned group of 8 lanes, in every lane of the group: the
// same pairs, in the same order, as the __shfl_xor 1, 2, 4 butterfly (after
// the quad steps all four lanes of a quad hold its sum, so the mirrored lane
// of the other quad holds the other quad's), bit for bit.
__device__ __forceinline__ float dr_sum8(float v) {
  v += dr_dpp<0xB1>(v);
  v += dr_dpp<0x4E>(v);
  v += dr_dpp<0x141>(v);
  return v;
}

// Sum over the 64 lanes, wave-uniform result: 8-lane groups and rows by DPP,
// then the four row sums by readlane ((r0 + r1) + (r2 + r3)).  A different
// association than dr_wave_sum's butterfly; a few tens of cycles instead of
// six dependent LDS round trips.
__device__ __forceinline__ float dr_wave_sum_dpp(float v) {
  v = dr_sum8(v);
  v += dr_dpp<0x140>(v);
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return (r0 + r1) + (r2 + r3);
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

// Counter-based uniform in [0,1) for dropout (splitmix64 finaliser, 24 bits):
// u(seed, offset, idx) is a pure function, so the forward and the backward
// pass regenerate the same keep mask without storing it.  The host replica
// (dr_dropout_mask) calls the same code.
__host__ __device__ inline uint64_t dr_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

__host__ __device__ inline float dr_uniform(uint64_t seed, uint64_t offset, uint32_t idx) {
  uint64_t z = dr_mix64(seed + 0x9E3779B97F4A7C15ULL * (offset + 1));
  z = dr_mix64(z ^ (0xD1B54A32D192ED03ULL * ((uint64_t)idx + 1)));
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

// Host-side description of an LDS carve for the carve tests
// (tests/test_lds_carves.py): "name=value;" pairs, region offsets in 4-byte
// words, "total" the words the carve reserves, "$name" a layout parameter.
#include <cstdio>
struct DrCarveDesc {
  char* buf;
  int len, pos;
};
inline void dr_carve_put(DrCarveDesc& d, const char* name, long long v) {
  const int room = d.len - d.pos;
  const int n = std::snprintf(d.buf + (room > 0 ? d.pos : 0), room > 0 ? room : 0, "%s=%lld;", name, v);
  d.pos += n > 0 ? n : 0;
}
#define DR_DESC(d, c, f) dr_carve_put(d, #f, (long long)(c).f)
#define DR_DESC_P(d, c, f) dr_carve_put(d, "$" #f, (long long)(c).f)
