// Device helpers shared by the per-graph fused kernels (gfx950, wave64).
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/deeprank2_amd.h"
#include "dr_common.h"

#ifndef DR_GATHER_IMM
#define DR_GATHER_IMM 1  // per-graph gathers: index reads as one base + immediate offsets (0: compiler-formed addresses)
#endif

#ifndef DR_Z_ARGS
#define DR_Z_ARGS 1  // large-graph tile kernels: Z rows stored only at the tile's depth-0 pooling arg candidates (0: every row)
#endif
#ifndef DR_TILE_XCD
#define DR_TILE_XCD 1  // tile kernels: consecutive tiles on one XCD (0: tile = blockIdx.x)
#endif

namespace drk {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr float LOWEST = -3.402823466e+38f;

__host__ __device__ inline int r4(int v) { return (v + 3) & ~3; }
__host__ __device__ inline int r16(int v) { return (v + 15) & ~15; }
__host__ __device__ inline int imax(int a, int b) { return a > b ? a : b; }

// torch relu keeps NaN (clamp_min propagates it); its backward masks where the
// output is <= 0 (threshold_backward), so a NaN output passes the gradient.
__device__ __forceinline__ float relu_keepnan(float v) { return (v <= 0.f) ? 0.f : v; }
__device__ __forceinline__ float relu_bwd(float out, float g) { return (out <= 0.f) ? 0.f : g; }

#define DRK_AS1(p) ((const __attribute__((address_space(1))) void*)(p))
#define DRK_AS3(p) ((__attribute__((address_space(3))) void*)(p))

// Asynchronous global->LDS copy of n 4-byte words (global_load_lds_dword: one
// wave instruction moves 256 contiguous bytes).  M0 (the LDS base) is
// wave-uniform; lane l lands at base + 4l.
template <int NT>
__device__ __forceinline__ void dma_words(void* lds_dst, const void* gsrc, int n) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t* src = reinterpret_cast<const uint32_t*>(gsrc);
  uint32_t* dst = reinterpret_cast<uint32_t*>(lds_dst);
  for (int base = wave * 64; base < n; base += NT)
    if (base + lane < n) __builtin_amdgcn_global_load_lds(DRK_AS1(src + base + lane), DRK_AS3(dst + base), 4, 0, 0);
}

// 16-byte lanes (global_load_lds_dwordx4, 1 KiB per wave instruction); source
// and destination 16-byte aligned; n4 = number of 16-byte units.
template <int NT>
__device__ __forceinline__ void dma_x4(void* lds_dst, const void* gsrc, int n4) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint4* src = reinterpret_cast<const uint4*>(gsrc);
  uint4* dst = reinterpret_cast<uint4*>(lds_dst);
  for (int base = wave * 64; base < n4; base += NT)
    if (base + lane < n4) __builtin_amdgcn_global_load_lds(DRK_AS1(src + base + lane), DRK_AS3(dst + base), 16, 0, 0);
}

// The tile a tile-kernel workgroup runs.  Workgroups are dispatched to the 8
// XCDs round-robin (block b to XCD group b % 8), so with tile = blockIdx.x a
// graph's consecutive tiles land on 8 different L2s and each fetches the
// graph's halo rows itself.  The bijective remap gives XCD group x the
// contiguous tiles [x*per + min(x, rem), ...) (cdna_hip_programming.md T1).
__host__ __device__ inline int xcd_tile_of(int b, int n) {
  if (!DR_TILE_XCD) return b;
  const int x = b & 7, q = b >> 3, per = n >> 3, rem = n & 7;
  return x * per + (x < rem ? x : rem) + q;
}
__device__ __forceinline__ int xcd_tile() { return xcd_tile_of(blockIdx.x, gridDim.x); }

__device__ __forceinline__ float4 f4add(float4 a, float4 v) {
  return make_float4(a.x + v.x, a.y + v.y, a.z + v.z, a.w + v.w);
}

// acc = sum over CSR row [eb, ee) of X[col[e], c4..c4+3] in edge order (the
// order torch_scatter's CPU scatter_add_ visits them).  Four index reads, then
// four row reads in flight per step.  The empty asm keeps the four 16-bit
// index reads separate: hipcc would otherwise merge them into a ds_read_b64
// that is misaligned for 3 of 4 row starts (LDS replays those at ~64 cycles).
__device__ __forceinline__ float4 gather_row_chunk(const uint16_t* col, int eb, int ee, const float* X, int XS,
                                                   int c4) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int e = eb;
  for (; e + 4 <= ee; e += 4) {
    int e1 = e + 1, e2 = e + 2, e3 = e + 3;
    asm volatile("" : "+v"(e1), "+v"(e2), "+v"(e3));
    const int j0 = col[e], j1 = col[e1], j2 = col[e2], j3 = col[e3];
    const float4 v0 = *reinterpret_cast<const float4*>(&X[__umul24(j0, XS) + c4]);
    const float4 v1 = *reinterpret_cast<const float4*>(&X[__umul24(j1, XS) + c4]);
    const float4 v2 = *reinterpret_cast<const float4*>(&X[__umul24(j2, XS) + c4]);
    const float4 v3 = *reinterpret_cast<const float4*>(&X[__umul24(j3, XS) + c4]);
    acc = f4add(f4add(f4add(f4add(acc, v0), v1), v2), v3);
  }
  if (e < ee) {  // the last 1-3 edges: their index and row reads in flight together, adds predicated
    const int l = ee - 1;
    const int j0 = col[e], j1 = col[min(e + 1, l)], j2 = col[min(e + 2, l)];
    const float4 v0 = *reinterpret_cast<const float4*>(&X[__umul24(j0, XS) + c4]);
    const float4 v1 = *reinterpret_cast<const float4*>(&X[__umul24(j1, XS) + c4]);
    const float4 v2 = *reinterpret_cast<const float4*>(&X[__umul24(j2, XS) + c4]);
    acc = f4add(acc, v0);
    acc = e + 1 < ee ? f4add(acc, v1) : acc;
    acc = e + 2 < ee ? f4add(acc, v2) : acc;
  }
  return acc;
}

// One CSR row's sums of two 16-byte X chunks (c4a, c4b) at once: one index
// read per edge feeds both chunks' row reads, four edges per step; each chunk
// summed in edge order (same sums as gather_row_chunk)
__device__ __forceinline__ void gather_row_two_chunks(const uint16_t* col, int eb, int ee, const float* X, int XS,
                                                      int c4a, int c4b, float4& outa, float4& outb) {
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
  int e = eb;
  for (; e + 4 <= ee; e += 4) {
    int e1 = e + 1, e2 = e + 2, e3 = e + 3;
    asm volatile("" : "+v"(e1), "+v"(e2), "+v"(e3));
    const int r0 = __umul24((int)col[e], XS), r1 = __umul24((int)col[e1], XS);
    const int r2 = __umul24((int)col[e2], XS), r3 = __umul24((int)col[e3], XS);
    const float4 v0 = *reinterpret_cast<const float4*>(&X[r0 + c4a]);
    const float4 v1 = *reinterpret_cast<const float4*>(&X[r1 + c4a]);
    const float4 v2 = *reinterpret_cast<const float4*>(&X[r2 + c4a]);
    const float4 v3 = *reinterpret_cast<const float4*>(&X[r3 + c4a]);
    const float4 w0 = *reinterpret_cast<const float4*>(&X[r0 + c4b]);
    const float4 w1 = *reinterpret_cast<const float4*>(&X[r1 + c4b]);
    const float4 w2 = *reinterpret_cast<const float4*>(&X[r2 + c4b]);
    const float4 w3 = *reinterpret_cast<const float4*>(&X[r3 + c4b]);
    a = f4add(f4add(f4add(f4add(a, v0), v1), v2), v3);
    b = f4add(f4add(f4add(f4add(b, w0), w1), w2), w3);
  }
  for (; e < ee; ++e) {
    const int r = __umul24((int)col[e], XS);
    a = f4add(a, *reinterpret_cast<const float4*>(&X[r + c4a]));
    b = f4add(b, *reinterpret_cast<const float4*>(&X[r + c4b]));
  }
  outa = a;
  outb = b;
}

// The four index reads of a gather step from an LDS column array: one base
// address and immediate offsets, waited for inside the statement (the
// compiler does not track inline-asm LDS reads).  col must point into LDS.
__device__ __forceinline__ void lds_index4(const uint16_t* col, int& j0, int& j1, int& j2, int& j3) {
  const uint32_t ad = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) uint16_t*)col);
  asm volatile(
      "ds_read_u16 %0, %4\n\t"
      "ds_read_u16 %1, %4 offset:2\n\t"
      "ds_read_u16 %2, %4 offset:4\n\t"
      "ds_read_u16 %3, %4 offset:6\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(j0), "=&v"(j1), "=&v"(j2), "=&v"(j3)
      : "v"(ad));
}

// gather_row_chunk for an LDS column array, with the index reads of
// lds_index4 and each row read addressed by one v_mad_u32_u24 (xc: LDS byte
// pointer of this lane's chunk in row 0; rb: bytes per X row).  Same sums,
// same edge order.
__device__ __forceinline__ float4 gather_row_chunk_imm(const uint16_t* col, int eb, int ee, const char* xc, int rb) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int e = eb;
  for (; e + 4 <= ee; e += 4) {
    int j0, j1, j2, j3;
    lds_index4(col + e, j0, j1, j2, j3);
    const float4 v0 = *reinterpret_cast<const float4*>(xc + __umul24(j0, rb));
    const float4 v1 = *reinterpret_cast<const float4*>(xc + __umul24(j1, rb));
    const float4 v2 = *reinterpret_cast<const float4*>(xc + __umul24(j2, rb));
    const float4 v3 = *reinterpret_cast<const float4*>(xc + __umul24(j3, rb));
    acc = f4add(f4add(f4add(f4add(acc, v0), v1), v2), v3);
  }
  if (e < ee) {  // the last 1-3 edges: their index and row reads in flight together, adds predicated
    const int l = ee - 1;
    const int j0 = col[e], j1 = col[min(e + 1, l)], j2 = col[min(e + 2, l)];
    const float4 v0 = *reinterpret_cast<const float4*>(xc + __umul24(j0, rb));
    const float4 v1 = *reinterpret_cast<const float4*>(xc + __umul24(j1, rb));
    const float4 v2 = *reinterpret_cast<const float4*>(xc + __umul24(j2, rb));
    acc = f4add(acc, v0);
    acc = e + 1 < ee ? f4add(acc, v1) : acc;
    acc = e + 2 < ee ? f4add(acc, v2) : acc;
  }
  return acc;
}

// gather_row_chunk for LDS column arrays: the _imm form unless built with
// DR_GATHER_IMM=0 (A/B)
__device__ __forceinline__ float4 gather_row_chunk_lds(const uint16_t* col, int eb, int ee, const float* X, int XS, int c4) {
#if DR_GATHER_IMM
  return gather_row_chunk_imm(col, eb, ee, reinterpret_cast<const char*>(X + c4), XS * 4);
#else
  return gather_row_chunk(col, eb, ee, X, XS, c4);
#endif
}

// gather_row_two_chunks with fewer VALU instructions per edge, for the
// per-graph kernels, whose gathers run 16 waves on 4 SIMDs and are VALU-issue
// bound (a wave64 VALU op holds its SIMD 4 cycles): the four index reads of
// a step are one base address and immediate offsets (inline asm, waited for
// inside the same statement -- the compiler does not track them), and each
// edge's two 16-byte reads are one v_mad_u32_u24 (row base) and a lane
// constant byte delta.  xa: LDS byte pointer of this lane's first chunk in
// row 0; db: the second chunk's byte distance from the first; rb: bytes per X
// row.  Same sums, same edge order as gather_row_chunk.
__device__ __forceinline__ void gather_row_two_chunks_imm(const uint16_t* col, int eb, int ee, const char* xa, int db,
                                                          int rb, float4& outa, float4& outb) {
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
  int e = eb;
  for (; e + 4 <= ee; e += 4) {
    int j0, j1, j2, j3;
    lds_index4(col + e, j0, j1, j2, j3);
    const char* p0 = xa + __umul24(j0, rb);
    const char* p1 = xa + __umul24(j1, rb);
    const char* p2 = xa + __umul24(j2, rb);
    const char* p3 = xa + __umul24(j3, rb);
    const float4 v0 = *reinterpret_cast<const float4*>(p0), w0 = *reinterpret_cast<const float4*>(p0 + db);
    const float4 v1 = *reinterpret_cast<const float4*>(p1), w1 = *reinterpret_cast<const float4*>(p1 + db);
    const float4 v2 = *reinterpret_cast<const float4*>(p2), w2 = *reinterpret_cast<const float4*>(p2 + db);
    const float4 v3 = *reinterpret_cast<const float4*>(p3), w3 = *reinterpret_cast<const float4*>(p3 + db);
    a = f4add(f4add(f4add(f4add(a, v0), v1), v2), v3);
    b = f4add(f4add(f4add(f4add(b, w0), w1), w2), w3);
  }
  for (; e < ee; ++e) {
    const char* p = xa + __umul24((int)col[e], rb);
    a = f4add(a, *reinterpret_cast<const float4*>(p));
    b = f4add(b, *reinterpret_cast<const float4*>(p + db));
  }
  outa = a;
  outb = b;
}

// Two CSR rows' sums of X chunks at once (one lane, two rows): each row in
// its own edge order (same sums as gather_row_chunk), four edges of each row
// per step, so eight index reads and then eight row reads are in flight.
__device__ __forceinline__ void gather_two_row_chunks(const uint16_t* col, int eb0, int ee0, int eb1, int ee1,
                                                      const float* X, int XS, int c4, float4& out0, float4& out1) {
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0;
  int e0 = eb0, e1 = eb1;
  for (; e0 + 4 <= ee0 && e1 + 4 <= ee1; e0 += 4, e1 += 4) {
    int f1 = e0 + 1, f2 = e0 + 2, f3 = e0 + 3, g1 = e1 + 1, g2 = e1 + 2, g3 = e1 + 3;
    asm volatile("" : "+v"(f1), "+v"(f2), "+v"(f3), "+v"(g1), "+v"(g2), "+v"(g3));
    const int j0 = col[e0], j1 = col[f1], j2 = col[f2], j3 = col[f3];
    const int k0 = col[e1], k1 = col[g1], k2 = col[g2], k3 = col[g3];
    const float4 v0 = *reinterpret_cast<const float4*>(&X[__umul24(j0, XS) + c4]);
    const float4 v1 = *reinterpret_cast<const float4*>(&X[__umul24(j1, XS) + c4]);
    const float4 v2 = *reinterpret_cast<const float4*>(&X[__umul24(j2, XS) + c4]);
    const float4 v3 = *reinterpret_cast<const float4*>(&X[__umul24(j3, XS) + c4]);
    const float4 w0 = *reinterpret_cast<const float4*>(&X[__umul24(k0, XS) + c4]);
    const float4 w1 = *reinterpret_cast<const float4*>(&X[__umul24(k1, XS) + c4]);
    const float4 w2 = *reinterpret_cast<const float4*>(&X[__umul24(k2, XS) + c4]);
    const float4 w3 = *reinterpret_cast<const float4*>(&X[__umul24(k3, XS) + c4]);
    a0 = f4add(f4add(f4add(f4add(a0, v0), v1), v2), v3);
    a1 = f4add(f4add(f4add(f4add(a1, w0), w1), w2), w3);
  }
  // the rest of each row on its own (4 edges in flight, then singles)
  for (; e0 + 4 <= ee0; e0 += 4) {
    int f1 = e0 + 1, f2 = e0 + 2, f3 = e0 + 3;
    asm volatile("" : "+v"(f1), "+v"(f2), "+v"(f3));
    const int j0 = col[e0], j1 = col[f1], j2 = col[f2], j3 = col[f3];
    const float4 v0 = *reinterpret_cast<const float4*>(&X[__umul24(j0, XS) + c4]);
    const float4 v1 = *reinterpret_cast<const float4*>(&X[__umul24(j1, XS) + c4]);
    const float4 v2 = *reinterpret_cast<const float4*>(&X[__umul24(j2, XS) + c4]);
    const float4 v3 = *reinterpret_cast<const float4*>(&X[__umul24(j3, XS) + c4]);
    a0 = f4add(f4add(f4add(f4add(a0, v0), v1), v2), v3);
  }
  for (; e1 + 4 <= ee1; e1 += 4) {
    int g1 = e1 + 1, g2 = e1 + 2, g3 = e1 + 3;
    asm volatile("" : "+v"(g1), "+v"(g2), "+v"(g3));
    const int k0 = col[e1], k1 = col[g1], k2 = col[g2], k3 = col[g3];
    const float4 w0 = *reinterpret_cast<const float4*>(&X[__umul24(k0, XS) + c4]);
    const float4 w1 = *reinterpret_cast<const float4*>(&X[__umul24(k1, XS) + c4]);
    const float4 w2 = *reinterpret_cast<const float4*>(&X[__umul24(k2, XS) + c4]);
    const float4 w3 = *reinterpret_cast<const float4*>(&X[__umul24(k3, XS) + c4]);
    a1 = f4add(f4add(f4add(f4add(a1, w0), w1), w2), w3);
  }
  for (; e0 < ee0; ++e0) a0 = f4add(a0, *reinterpret_cast<const float4*>(&X[__umul24((int)col[e0], XS) + c4]));
  for (; e1 < ee1; ++e1) a1 = f4add(a1, *reinterpret_cast<const float4*>(&X[__umul24((int)col[e1], XS) + c4]));
  out0 = a0;
  out1 = a1;
}

// As gather_two_row_chunks with the column ids pre-scaled to byte offsets of
// X rows (col[e] = j * XS * 4, so rows up to 64 KiB into X): one add per edge
// and lane forms the address (same sums, same order).
__device__ __forceinline__ void gather_two_row_chunks_boff(const uint16_t* col, int eb0, int ee0, int eb1, int ee1,
                                                           const char* Xc, float4& out0, float4& out1) {
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0;
  int e0 = eb0, e1 = eb1;
#define DRK_XR(off) (*reinterpret_cast<const float4*>(Xc + (off)))
  for (; e0 + 4 <= ee0 && e1 + 4 <= ee1; e0 += 4, e1 += 4) {
    int f1 = e0 + 1, f2 = e0 + 2, f3 = e0 + 3, g1 = e1 + 1, g2 = e1 + 2, g3 = e1 + 3;
    asm volatile("" : "+v"(f1), "+v"(f2), "+v"(f3), "+v"(g1), "+v"(g2), "+v"(g3));
    const uint32_t j0 = col[e0], j1 = col[f1], j2 = col[f2], j3 = col[f3];
    const uint32_t k0 = col[e1], k1 = col[g1], k2 = col[g2], k3 = col[g3];
    const float4 v0 = DRK_XR(j0), v1 = DRK_XR(j1), v2 = DRK_XR(j2), v3 = DRK_XR(j3);
    const float4 w0 = DRK_XR(k0), w1 = DRK_XR(k1), w2 = DRK_XR(k2), w3 = DRK_XR(k3);
    a0 = f4add(f4add(f4add(f4add(a0, v0), v1), v2), v3);
    a1 = f4add(f4add(f4add(f4add(a1, w0), w1), w2), w3);
  }
  for (; e0 + 4 <= ee0; e0 += 4) {
    int f1 = e0 + 1, f2 = e0 + 2, f3 = e0 + 3;
    asm volatile("" : "+v"(f1), "+v"(f2), "+v"(f3));
    const uint32_t j0 = col[e0], j1 = col[f1], j2 = col[f2], j3 = col[f3];
    const float4 v0 = DRK_XR(j0), v1 = DRK_XR(j1), v2 = DRK_XR(j2), v3 = DRK_XR(j3);
    a0 = f4add(f4add(f4add(f4add(a0, v0), v1), v2), v3);
  }
  for (; e1 + 4 <= ee1; e1 += 4) {
    int g1 = e1 + 1, g2 = e1 + 2, g3 = e1 + 3;
    asm volatile("" : "+v"(g1), "+v"(g2), "+v"(g3));
    const uint32_t k0 = col[e1], k1 = col[g1], k2 = col[g2], k3 = col[g3];
    const float4 w0 = DRK_XR(k0), w1 = DRK_XR(k1), w2 = DRK_XR(k2), w3 = DRK_XR(k3);
    a1 = f4add(f4add(f4add(f4add(a1, w0), w1), w2), w3);
  }
  for (; e0 < ee0; ++e0) a0 = f4add(a0, DRK_XR((uint32_t)col[e0]));
  for (; e1 < ee1; ++e1) a1 = f4add(a1, DRK_XR((uint32_t)col[e1]));
#undef DRK_XR
  out0 = a0;
  out1 = a1;
}

}  // namespace drk

#ifdef DR_STAMPS
#define DRK_STAMP(i)                                                                              \
  do {                                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    if (tid == 0 && a.p.stamps) a.p.stamps[(int64_t)b * 32 + (i)] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                            \
  } while (0)
#else
#define DRK_STAMP(i) \
  do {               \
  } while (0)
#endif
