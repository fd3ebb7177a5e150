// GINet training step, one workgroup per graph, everything resident in LDS.
//
// Replaces (deeprank2 v3.1.0):
//   GINetConvLayer.forward        deeprank2/neuralnets/gnn/ginet.py:40-60
//   GINet.forward                 ginet.py:90-125
//   get_preloaded_cluster         deeprank2/utils/community_pooling.py:23-27
//   community_pooling             community_pooling.py:165-242
//   max_pool_x / scatter_mean     ginet.py:103,114,117-118
//   autograd backward + loss      deeprank2/trainer.py:686-689
//
// Algebra used (all exact):
//   * the attention of ginet.py:48-55 is softmax over a size-1 dim, i.e. 1 for
//     every finite logit, so conv(x) = A·(x Wᵀ) with A[i,j] = #edges (i→j);
//     its parameters get exact-zero gradients (done by the reduce kernel);
//   * both branches see the same graph (data.clone(), ginet.py:92), so conv1
//     and conv1_ext are one GEMM with W = [W1; W1e] (32 outputs);
//   * per-batch cluster offsetting + consecutive_cluster is, graph by graph, a
//     dense relabelling of that graph's ids (precomputed into the store), and
//     pool_edge's coalesced pooled graph is precomputed as a CSR too.
//
// Execution: 1024 threads (16 waves) per graph; the graph and the weights are
// staged by global->LDS DMA (16-byte lanes where the store layout allows);
// conv1 aggregates first, Z = A·X, then H = relu(Z·Wᵀ) on the f32 MFMA
// (v_mfma_f32_16x16x4_f32: an exact k-ordered fmaf chain).  Because the
// depth-0 max pool routes each channel's gradient to one member per cluster,
// the conv1 weight gradient is sum_k v_k·Z[arg_k] and the backward needs no
// gather over the edges at all.
// Roofline: HBM-bound on the compulsory inputs (x, CSR, clusters) and the
// per-graph partial writes — see DESIGN.md §Roofline.

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdlib>
#include <cstring>

#include "../../include/deeprank2_amd.h"
#include "dr_common.h"
#include "graph_common.h"
#include "ginet_head.h"

namespace {

#ifndef DR_GATHER_ROW2
#define DR_GATHER_ROW2 1  // GINet gather: one row, two chunks per lane (0: two rows, one chunk)
#endif
#ifndef DR_CONV2_KEYS
#define DR_CONV2_KEYS 0  // 1: conv2 reads the pooled rows from the depth-0 keys, no barrier after their decode (measured 0.1 us slower, r05)
#endif
#ifndef DR_TILE_STORE_WAIT
#define DR_TILE_STORE_WAIT 0  // 1: the tile kernels wait for their Z stores before the MFMA phase (r05 form, A/B)
#endif
#ifndef DR_DMA_ROT
#define DR_DMA_ROT 0  // 1: spread starting waves (measured 0.1 us slower per pass, r05)
#endif
constexpr int NT = 1024;     // 16 waves
constexpr int NW = NT / 64;
constexpr int HEADW = 672;   // G64 hpre128 hh128 hd128 dh128 dG64 dout16 spare16
constexpr float LOWEST = -3.402823466e+38f;

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;

__host__ __device__ inline int r4(int v) { return (v + 3) & ~3; }
__host__ __device__ inline int r16(int v) { return (v + 15) & ~15; }

struct Carve {
  int KP, LDW, XS;
  int w1, w2, fc2, x, z, rp, col, cl0, key, p1, a1, dp1, y2, h2, p1rp, p1c, p1trp, p1tc, m1p, m1i, p2, nt, cl1,
      head, dgp, keep, total;
};

// LDS carve (4-byte words, every region 16-byte aligned).  X keeps the HBM
// row stride XS = r4(F) (16-byte rows for the DMA and the float4 gather);
// Z = A·X uses the stride KP+2 so the MFMA column reads are bank-conflict
// free.
__host__ __device__ inline Carve carve(int N, int E, int F, int K0, int P1, int K1, int alias, int OUT) {
  Carve c;
  // K padded to the kernel's KPT (32 for F <= 32, else 64: the MFMA steps it
  // runs; zeros past F).  (Until r05 KP was r16(F), shorter than KPT for F <= 16
  // and 33..48: the padding zeroed to KPT then ran 14 words past Z into the
  // row pointers being DMA'd beside it, and the last k steps read other
  // waves' rows.)
  c.KP = F <= 32 ? 32 : 64;
  c.LDW = c.KP + 2;   // rows 2 words apart: lanes (row li, k+kq) hit 32 distinct banks
  c.XS = r4(F);
  int o = 0;
#define TAKE(field, words) \
  c.field = o;             \
  o += r4(words);
  TAKE(w1, 32 * F)           // [W1; W1e] (conv1 / conv1_ext .fc.weight), rows of F
  TAKE(w2, 1024)             // [W2 | W2e] (conv2 / conv2_ext .fc.weight)
  TAKE(fc2, OUT * 128 + OUT) // fc2.weight rows, then fc2.bias
  TAKE(x, N * c.XS)
  TAKE(z, N * c.LDW)
  TAKE(rp, N + 1)
  TAKE(col, (E + 1) / 2)     // uint16 column ids
  TAKE(cl0, N)               // depth-0 cluster of each node
  TAKE(key, 2 * K0 * 32)     // depth-0 pooling keys (uint64)
  TAKE(p1, K0 * 32)
  TAKE(a1, K0 * 32)
  TAKE(dp1, K0 * 32)
  TAKE(y2, K0 * 64)
  TAKE(h2, K0 * 64)
  TAKE(p1rp, K0 + 1)
  TAKE(p1c, P1)
  if (alias) {
    c.p1trp = c.p1rp;
    c.p1tc = c.p1c;
  } else {
    TAKE(p1trp, K0 + 1)
    TAKE(p1tc, P1)
  }
  TAKE(m1p, K1 + 1)
  TAKE(m1i, K0)
  TAKE(p2, K1 * 64)
  TAKE(nt, K1 * 64)
  TAKE(cl1, K0)  // depth-1 cluster of each depth-0 cluster
  TAKE(head, HEADW)
  TAKE(dgp, NW * 64)
  TAKE(keep, 32)  // 128 dropout keep bytes
#undef TAKE
  c.total = o;
  return c;
}

// The accumulating pass's prefetch layout (dr_ginet_acc_pass with the batch's
// maximum sizes): the weights stay put across a workgroup's graphs, and the
// inputs of graph k+1 are DMA'd by the waves that have no tile in graph k's
// front half (N <= 240), into the other of two input buffers:
//   [W1 | W2 | fc2] [inputs, parity 0: x rp col cl0 p1rp p1c p1trp p1tc m1p
//   m1i] [inputs, parity 1] [scratch: z key p1 a1 dp1 y2 h2 p2 nt cl1 head
//   dgp keep]
// (word offsets from the carve base; each region sized for the batch maxima).
struct AccLayout {
  int in0, in1, scr, total;
};

__host__ __device__ inline Carve carve_acc(int N, int E, int F, int K0, int P1, int K1, int alias, int OUT,
                                           const AccLayout& L, int par) {
  Carve c;
  c.KP = F <= 32 ? 32 : 64;  // as carve()
  c.LDW = c.KP + 2;
  c.XS = r4(F);
  int o = 0;
#define TAKE(field, words) \
  c.field = o;             \
  o += r4(words);
  TAKE(w1, 32 * F)
  TAKE(w2, 1024)
  TAKE(fc2, OUT * 128 + OUT)
  o = par ? L.in1 : L.in0;
  TAKE(x, N * c.XS)
  TAKE(rp, N + 1)
  TAKE(col, (E + 1) / 2)
  TAKE(cl0, N)
  TAKE(p1rp, K0 + 1)
  TAKE(p1c, P1)
  if (alias) {
    c.p1trp = c.p1rp;
    c.p1tc = c.p1c;
  } else {
    TAKE(p1trp, K0 + 1)
    TAKE(p1tc, P1)
  }
  TAKE(m1p, K1 + 1)
  TAKE(m1i, K0)
  o = L.scr;
  TAKE(z, N * c.LDW)
  TAKE(key, 2 * K0 * 32)
  TAKE(p1, K0 * 32)
  TAKE(a1, K0 * 32)
  TAKE(dp1, K0 * 32)
  TAKE(y2, K0 * 64)
  TAKE(h2, K0 * 64)
  TAKE(p2, K1 * 64)
  TAKE(nt, K1 * 64)
  TAKE(cl1, K0)
  TAKE(head, HEADW)
  TAKE(dgp, NW * 64)
  TAKE(keep, 32)
#undef TAKE
  c.total = o;
  return c;
}

// the layout for the batch maxima (every graph's carve_acc fits inside it)
__host__ __device__ inline AccLayout acc_layout(int Nm, int Em, int F, int K0m, int P1m, int K1m, int alias, int OUT) {
  AccLayout L;
  L.in0 = r4(32 * F) + 1024 + r4(OUT * 128 + OUT);
  const int XS = r4(F), LDW = (F <= 32 ? 32 : 64) + 2;
  const int in = r4(Nm * XS) + r4(Nm + 1) + r4((Em + 1) / 2) + r4(Nm) + r4(K0m + 1) + r4(P1m) +
                 (alias ? 0 : r4(K0m + 1) + r4(P1m)) + r4(K1m + 1) + r4(K0m);
  L.in1 = L.in0 + in;
  L.scr = L.in1 + in;
  L.total = L.scr + r4(Nm * LDW) + r4(2 * K0m * 32) + 3 * r4(K0m * 32) + 2 * r4(K0m * 64) + 2 * r4(K1m * 64) + r4(K0m) +
            r4(HEADW) + r4(NW * 64) + r4(32);
  return L;
}

struct GinetArgs {
  dr_graph_store s;
  dr_ginet_weights w;
  dr_pass p;
  const dr_graph_desc* descs;
  int32_t B;
};

// torch relu keeps NaN (clamp_min propagates it); its backward masks where
// the output is <= 0 (threshold_backward), so a NaN output passes the grad.
__device__ __forceinline__ float relu_keepnan(float v) { return (v <= 0.f) ? 0.f : v; }
__device__ __forceinline__ float relu_bwd(float out, float g) { return (out <= 0.f) ? 0.f : g; }


#define AS1(p) ((const __attribute__((address_space(1))) void*)(p))
#define AS3(p) ((__attribute__((address_space(3))) void*)(p))

// Asynchronous global->LDS copy of n 4-byte words (global_load_lds_dword: one
// wave instruction moves 256 contiguous bytes, no VGPR round trip).  The LDS
// base handed to the instruction (M0) is wave-uniform; lane l lands at base+4l.
// w0: the wave that takes the first 64 lanes (the copies of a staging
// sequence start on different waves, so the short ones do not all queue on
// wave 0: an LDS DMA instruction holds its wave ~a few hundred cycles at issue)
__device__ __forceinline__ void dma_words(void* lds_dst, const void* gsrc, int n, int tid = threadIdx.x, int w0 = 0) {
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(((tid >> 6) - w0) & (NW - 1));
  const uint32_t* src = reinterpret_cast<const uint32_t*>(gsrc);
  uint32_t* dst = reinterpret_cast<uint32_t*>(lds_dst);
  for (int base = wave * 64; base < n; base += NT)
    if (base + lane < n) __builtin_amdgcn_global_load_lds(AS1(src + base + lane), AS3(dst + base), 4, 0, 0);
}

// Same with 16-byte lanes (global_load_lds_dwordx4, 1 KiB per wave
// instruction).  Source and destination 16-byte aligned; n4 = 16-byte units.
__device__ __forceinline__ void dma_x4(void* lds_dst, const void* gsrc, int n4, int tid = threadIdx.x, int w0 = 0) {
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(((tid >> 6) - w0) & (NW - 1));
  const uint4* src = reinterpret_cast<const uint4*>(gsrc);
  uint4* dst = reinterpret_cast<uint4*>(lds_dst);
  for (int base = wave * 64; base < n4; base += NT)
    if (base + lane < n4) __builtin_amdgcn_global_load_lds(AS1(src + base + lane), AS3(dst + base), 16, 0, 0);
}

// One LDS-DMA instruction from inline asm (M0 = the wave's LDS destination,
// saved and restored around it: M0 is a reserved register the compiler may be
// using)
__device__ __forceinline__ void lds_dma_dword(uint32_t m0, const void* src) {
  uint32_t saved;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %2, off\n\ts_mov_b32 m0, %0"
               : "=&s"(saved)
               : "s"(m0), "v"(src));
}
__device__ __forceinline__ void lds_dma_x4(uint32_t m0, const void* src) {
  uint32_t saved;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\ts_mov_b32 m0, %0"
               : "=&s"(saved)
               : "s"(m0), "v"(src));
}

// The same copies issued from inline asm: the compiler does not know they
// write LDS, so it inserts no wait for them before later LDS reads (with the
// builtin it waits for the DMA before the next LDS access), and (no memory
// clobber) reloads nothing around them.  For copies into
// LDS no one reads until an explicit s_waitcnt vmcnt(0) + barrier: the
// accumulating pass's prefetch of the next graph's inputs under this graph's
// tail.
__device__ __forceinline__ void dma_words_async(void* lds_dst, const void* gsrc, int n, int tid, int w0 = 0) {
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(((tid >> 6) - w0) & (NW - 1));
  const uint32_t* src = reinterpret_cast<const uint32_t*>(gsrc);
  const uint32_t dst = (uint32_t)(size_t)AS3(lds_dst);
  for (int base = wave * 64; base < n; base += NT)
    if (base + lane < n)
      lds_dma_dword(__builtin_amdgcn_readfirstlane(dst + 4 * base), src + base + lane);
}

// the same over waves [wf, wf + nw) only (the others skip)
__device__ __forceinline__ void dma_words_async_sub(void* lds_dst, const void* gsrc, int n, int tid, int wf, int nw) {
  const int lane = tid & 63, rw = __builtin_amdgcn_readfirstlane((tid >> 6) - wf);
  const uint32_t* src = reinterpret_cast<const uint32_t*>(gsrc);
  const uint32_t dst = (uint32_t)(size_t)AS3(lds_dst);
  if (rw < 0) return;
  for (int base = rw * 64; base < n; base += nw * 64)
    if (base + lane < n)
      lds_dma_dword(__builtin_amdgcn_readfirstlane(dst + 4 * base), src + base + lane);
}
__device__ __forceinline__ void dma_x4_async_sub(void* lds_dst, const void* gsrc, int n4, int tid, int wf, int nw) {
  const int lane = tid & 63, rw = __builtin_amdgcn_readfirstlane((tid >> 6) - wf);
  const uint4* src = reinterpret_cast<const uint4*>(gsrc);
  const uint32_t dst = (uint32_t)(size_t)AS3(lds_dst);
  if (rw < 0) return;
  for (int base = rw * 64; base < n4; base += nw * 64)
    if (base + lane < n4)
      lds_dma_x4(__builtin_amdgcn_readfirstlane(dst + 16 * base), src + base + lane);
}

__device__ __forceinline__ void dma_x4_async(void* lds_dst, const void* gsrc, int n4, int tid, int w0 = 0) {
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(((tid >> 6) - w0) & (NW - 1));
  const uint4* src = reinterpret_cast<const uint4*>(gsrc);
  const uint32_t dst = (uint32_t)(size_t)AS3(lds_dst);
  for (int base = wave * 64; base < n4; base += NT)
    if (base + lane < n4)
      lds_dma_x4(__builtin_amdgcn_readfirstlane(dst + 16 * base), src + base + lane);
}

__device__ __forceinline__ float4 f4add(float4 a, float4 v) {
  return make_float4(a.x + v.x, a.y + v.y, a.z + v.z, a.w + v.w);
}

// Z[i, :XS] = sum over CSR row i of X[col[e], :XS] (edges in CSR order, i.e.
// the order torch_scatter's CPU scatter_add_ visits them).  8 lanes per row,
// one float4 chunk each (a 16-lane ds_read_b128 group then touches 2 rows, not
// 4); edges unrolled by 4 so 4 index reads and then their row reads are in
// flight together.  Z rows have the stride ldz of the MFMA operand layout.
__device__ __forceinline__ void gather_rows(const int* rp, const uint16_t* col, const float* X, int XS, float* Z,
                                            int ldz, int n, int tid = threadIdx.x) {
  const int nch = XS >> 2;
  const int sub = tid & 7;
  for (int i = tid >> 3; i < n; i += NT / 8) {
    const int eb = rp[i], ee = rp[i + 1];
    for (int ch = sub; ch < nch; ch += 8) {
      const int c4 = ch * 4;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      int e = eb;
      for (; e + 4 <= ee; e += 4) {
        // Keep four separate 16-bit reads: hipcc would otherwise merge them
        // into one ds_read_b64 that is misaligned for 3 of 4 row starts (LDS
        // replays those at ~64 cycles).  The empty asm hides the contiguity.
        int e1 = e + 1, e2 = e + 2, e3 = e + 3;
        asm volatile("" : "+v"(e1), "+v"(e2), "+v"(e3));
        const int j0 = col[e], j1 = col[e1], j2 = col[e2], j3 = col[e3];
        const float4 v0 = *reinterpret_cast<const float4*>(&X[__umul24(j0, XS) + c4]);
        const float4 v1 = *reinterpret_cast<const float4*>(&X[__umul24(j1, XS) + c4]);
        const float4 v2 = *reinterpret_cast<const float4*>(&X[__umul24(j2, XS) + c4]);
        const float4 v3 = *reinterpret_cast<const float4*>(&X[__umul24(j3, XS) + c4]);
        acc = f4add(f4add(f4add(f4add(acc, v0), v1), v2), v3);
      }
      for (; e < ee; ++e) acc = f4add(acc, *reinterpret_cast<const float4*>(&X[__umul24((int)col[e], XS) + c4]));
      float* zr = Z + i * ldz + c4;
      zr[0] = acc.x;
      zr[1] = acc.y;
      zr[2] = acc.z;
      zr[3] = acc.w;
    }
  }
}

#ifdef DR_STAMPS
#define STAMP(i)                                                                                  \
  do {                                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    if (tid == 0 && a.p.stamps) a.p.stamps[(int64_t)b * 32 + (i)] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                            \
  } while (0)
#define SSTAMP(i)                                                                                   \
  do {                                                                                              \
    __builtin_amdgcn_sched_barrier(0);                                                              \
    if (tid == 0 && ga.p.stamps) ga.p.stamps[(int64_t)b * 32 + (i)] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                              \
  } while (0)
// cross-workgroup timeline (s_memrealtime: one 100 MHz clock for the whole chip)
#define RSTAMP(row, i)                                                                                  \
  do {                                                                                                  \
    __builtin_amdgcn_sched_barrier(0);                                                                  \
    if (threadIdx.x == 0 && a.g.p.stamps) a.g.p.stamps[(int64_t)(row) * 32 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                                  \
  } while (0)
#else
#define RSTAMP(row, i) \
  do {                 \
  } while (0)
#define STAMP(i) \
  do {           \
  } while (0)
#define SSTAMP(i) \
  do {            \
  } while (0)
#endif

// sum over a pooled CSR row [eb, ee) of v[col[e] * 64 + o], in edge order;
// four index reads, then four value reads in flight per step (same sum order
// as the plain loop).
__device__ __forceinline__ float pooled_row_sum(const int* col, int eb, int ee, const float* v, int o) {
  float acc = 0.f;
  int e = eb;
  for (; e + 4 <= ee; e += 4) {
    const int c0 = col[e], c1 = col[e + 1], c2 = col[e + 2], c3 = col[e + 3];
    const float v0 = v[c0 * 64 + o], v1 = v[c1 * 64 + o], v2 = v[c2 * 64 + o], v3 = v[c3 * 64 + o];
    acc = (((acc + v0) + v1) + v2) + v3;
  }
  for (; e < ee; ++e) acc += v[col[e] * 64 + o];
  return acc;
}

// Everything after the depth-0 pooling (P1 / A1 in LDS): conv2 on the pooled
// graph, depth-1 pooling, mean, head, loss and the whole backward.  Shared by
// the single-workgroup kernel and the large-graph tail kernel; zat(i, kk)
// reads Z = A·X at node i (LDS or the large path's HBM workspace).
struct TailLds {
  float *w2, *fc2, *p1, *dp1, *y2, *h2, *p2, *nt, *dgp;
  float *g, *hpre, *hh, *hd, *dh, *dg, *dout;
  int *a1, *p1rp, *p1c, *p1trp, *p1tc, *m1p, *m1i, *cl1;
  const uint8_t* keep = nullptr;  // prefetched dropout keep flags, or null (hash in the head)
  // accumulating pass (dr_ginet_acc_pass): the workgroup's running sums
  // [dW1cat 32F | dW2cat 1024 | the head's, GinetHeadLds::acc], or null
  float* acc = nullptr;
  float* accf = nullptr;  // GinetHeadLds::accf
  // or null: the depth-0 pooling keys, P1 not yet decoded (conv2 decodes the
  // rows it reads; the decode runs beside it in the same step)
  const unsigned long long* key = nullptr;
  // p2's first row zeroed by the caller before its last barrier: with one
  // depth-1 cluster (K1 = 1, K0 < 16) conv2 folds the depth-1 max into it by
  // LDS atomic max, and the pooling and mean steps go
  bool p2_zeroed = false;
};

template <class C>
__device__ __forceinline__ TailLds tail_lds(const C& c, float* lds) {
  TailLds t;
  t.w2 = lds + c.w2;
  t.fc2 = lds + c.fc2;
  t.p1 = lds + c.p1;
  t.a1 = reinterpret_cast<int*>(lds + c.a1);
  t.dp1 = lds + c.dp1;
  t.y2 = lds + c.y2;
  t.h2 = lds + c.h2;
  t.p1rp = reinterpret_cast<int*>(lds + c.p1rp);
  t.p1c = reinterpret_cast<int*>(lds + c.p1c);
  t.p1trp = reinterpret_cast<int*>(lds + c.p1trp);
  t.p1tc = reinterpret_cast<int*>(lds + c.p1tc);
  t.m1p = reinterpret_cast<int*>(lds + c.m1p);
  t.m1i = reinterpret_cast<int*>(lds + c.m1i);
  t.p2 = lds + c.p2;
  t.nt = lds + c.nt;
  t.cl1 = reinterpret_cast<int*>(lds + c.cl1);
  t.g = lds + c.head;
  t.hpre = t.g + 64;
  t.hh = t.hpre + 128;
  t.hd = t.hh + 128;
  t.dh = t.hd + 128;
  t.dg = t.dh + 128;
  t.dout = t.dg + 64;
  t.dgp = lds + c.dgp;
  return t;
}

template <class ZAt, bool WT = false, bool ACC = false>
__device__ __forceinline__ void ginet_tail(const GinetArgs& a, const TailLds& t, const float (&fc1_row)[8],
                                           const float (&fc1_col)[8], float fc1_bias, int b, int N, int K0, int K1,
                                           int F, int OUT, float y_g, uint64_t drop_offset, ZAt zat, int pb) {
  if (pb < 0) pb = b;  // the partials' row (slab, head vectors, loss term)
  const int tid = dr_tid<ACC>();
  STAMP(4);
  // one depth-1 cluster: its max over the K0 pooled rows per channel by LDS
  // atomic max on the bits as conv2 produces the rows (H2 >= +0 or NaN, so
  // the unsigned order of the bits is the value order; NaN wins, as the
  // reference's NaN-propagating amax), the tie counts in the pooling backward
  const bool one_cl = t.p2_zeroed && K1 == 1 && K0 < 16;
  // ---------------- conv2 on the pooled graph (ginet.py:101,112) ------------
  // H2[k][o] = relu(sum over pooled row k, in edge order, of Y2[j][o]) with
  // Y2[j][o] = P1[j] . W2[o] (16-term fmaf chain) formed per neighbour in
  // registers: no Y2 array and no barrier between the GEMM and the sum
  for (int p = tid; p < K0 * 64; p += NT) {
    const int k = p >> 6, o = p & 63, br = o >> 5;
    float wr[16];  // rows 0..31 = W2, 32..63 = W2e
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 v = *reinterpret_cast<const float4*>(t.w2 + o * 16 + 4 * q);
      wr[4 * q] = v.x;
      wr[4 * q + 1] = v.y;
      wr[4 * q + 2] = v.z;
      wr[4 * q + 3] = v.w;
    }
    float acc = 0.f;
    for (int e = t.p1rp[k]; e < t.p1rp[k + 1]; ++e) {
      float y = 0.f;
      if (t.key) {  // P1 = the key's value half, 0 for an empty (cluster, channel)
        const unsigned long long* kr = t.key + t.p1c[e] * 32 + br * 16;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const ulonglong2 kv = *reinterpret_cast<const ulonglong2*>(kr + 2 * q);
          const float v0 = kv.x ? __uint_as_float((uint32_t)(kv.x >> 32)) : 0.f;
          const float v1 = kv.y ? __uint_as_float((uint32_t)(kv.y >> 32)) : 0.f;
          y = fmaf(v0, wr[2 * q], y);
          y = fmaf(v1, wr[2 * q + 1], y);
        }
      } else {
        const float* pr = t.p1 + t.p1c[e] * 32 + br * 16;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 v = *reinterpret_cast<const float4*>(pr + 4 * q);
          y = fmaf(v.x, wr[4 * q], y);
          y = fmaf(v.y, wr[4 * q + 1], y);
          y = fmaf(v.z, wr[4 * q + 2], y);
          y = fmaf(v.w, wr[4 * q + 3], y);
        }
      }
      acc += y;
    }
    const float h2v = relu_keepnan(acc);
    t.h2[p] = h2v;
    if (one_cl) __hip_atomic_fetch_max(reinterpret_cast<uint32_t*>(t.p2) + o, __float_as_uint(h2v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __syncthreads();

  if (one_cl) {
    STAMP(5);  // (no pooling or mean step: stamps 5, 6 mark the same point)
    STAMP(6);
  } else {
    STAMP(5);
    // ---------------- depth-1 max_pool_x: scatter_reduce amax (ginet.py:103) --
    // NaN propagates; remember the tie count for the even-split backward.
    // Members are split into S slices per (cluster, channel): each slice's
    // max (NaN-propagating) and its count of members equal to it, combined per
    // pair (max is order-free here: H2 >= +0 or NaN).  Also record each
    // depth-0 cluster's depth-1 cluster for the backward.
    // (by the last wave, idle here unless K1 >= 15: the pooling pairs start at
    // wave 0; m counts the member offsets at or below q, all reads in flight)
    for (int q = tid - (NT - 64); q >= 0 && q < K0; q += 64) {
      int m = 0;
      if (K1 <= 16) {
#pragma unroll
        for (int j = 1; j < 16; ++j) m += (j < K1 && t.m1p[j < K1 ? j : 0] <= q) ? 1 : 0;
      } else {
        while (q >= t.m1p[m + 1]) ++m;
      }
      t.cl1[t.m1i[q]] = m;
    }
    if (K0 < 16) {  // few members per pair: one pass
      for (int p = tid; p < K1 * 64; p += NT) {
        const int m = p >> 6, o = p & 63;
        const int mb = t.m1p[m], me = t.m1p[m + 1];
        // members' values gathered once (<= 15): all index reads, then all
        // value reads in flight (predicated); max and tie count are order-free
        float v[16];
        int q[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) q[u] = t.m1i[(mb + u < me) ? mb + u : mb];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = t.h2[q[u] * 64 + o];
        float mx = v[0];
#pragma unroll
        for (int u = 1; u < 16; ++u)
          if (mb + u < me) mx = (mx != mx || v[u] != v[u]) ? __int_as_float(0x7fc00000) : fmaxf(mx, v[u]);
        float ties = 0.f;
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (mb + u < me) ties += (v[u] == mx) ? 1.f : 0.f;
        t.p2[p] = mx;
        t.nt[p] = ties;
        if (K1 == 1) t.g[o] = (0.f + mx) / (float)K1;  // the mean below, for one cluster (same ops)
      }
    } else {
      const int pairs = K1 * 64;
      const int LS = pairs <= 32 ? 4 : pairs <= 64 ? 3 : pairs <= 128 ? 2 : pairs <= 256 ? 1 : 0;  // pairs*S <= 512
      const int S = 1 << LS;
      float* smx = t.dgp;            // [pairs*S] (dgp is free until the head)
      float* scnt = t.dgp + 512;
      const float NEG = -__builtin_inff();
      for (int p = tid; p < pairs * S; p += NT) {
        const int sl = p & (S - 1), pr = p >> LS, m = pr >> 6, o = pr & 63;
        const int mb = t.m1p[m], cnt = t.m1p[m + 1] - mb;
        const int qb = mb + ((cnt * sl) >> LS), qe = mb + ((cnt * (sl + 1)) >> LS);
        float mx = NEG;
        for (int q = qb; q < qe; ++q) {
          const float v = t.h2[t.m1i[q] * 64 + o];
          mx = (mx != mx || v != v) ? __int_as_float(0x7fc00000) : fmaxf(mx, v);
        }
        float ties = 0.f;
        for (int q = qb; q < qe; ++q) ties += (t.h2[t.m1i[q] * 64 + o] == mx) ? 1.f : 0.f;
        smx[p] = mx;
        scnt[p] = ties;
      }
      __syncthreads();
      for (int p = tid; p < pairs; p += NT) {
        float mx = NEG;
        bool nan = false;
        for (int sl = 0; sl < S; ++sl) {
          const float v = smx[(p << LS) + sl];
          if (v != v) nan = true;
          else mx = fmaxf(mx, v);
        }
        float ties = 0.f;
        if (nan) mx = __int_as_float(0x7fc00000);
        else
          for (int sl = 0; sl < S; ++sl) ties += (smx[(p << LS) + sl] == mx) ? scnt[(p << LS) + sl] : 0.f;
        t.p2[p] = mx;
        t.nt[p] = ties;
      }
    }
    __syncthreads();

    STAMP(6);
    // ---------------- per-graph mean (scatter_mean, ginet.py:117-118) ----------
    // (K1 = 1 with K0 < 16: written by the pooling above)
    if (!(K1 == 1 && K0 < 16)) {
      if (tid < 64) {
        float acc = 0.f;
        for (int m = 0; m < K1; ++m) acc += t.p2[m * 64 + tid];
        t.g[tid] = acc / (float)K1;
      }
      __syncthreads();
    }
  }

  STAMP(7);
  {
    drk::GinetHeadLds hl;
    hl.fc2 = t.fc2;
    hl.g = one_cl ? t.p2 : t.g;  // (one cluster: the mean (0 + max) / 1 is the max itself)
    hl.hpre = t.hpre;
    hl.hh = t.hh;
    hl.hd = t.hd;
    hl.dh = t.dh;
    hl.dg = t.dg;
    hl.dout = t.dout;
    hl.dgp = t.dgp;
    hl.keep = t.keep;
    hl.acc = ACC ? t.acc + 32 * F + 1024 : nullptr;
    hl.accf = ACC ? t.accf : nullptr;
    hl.dg_deferred = true;  // summed from dgp by the pooling backward below
    if (!drk::ginet_head<NT, WT, ACC>(a.p, hl, fc1_row, fc1_col, fc1_bias, b, OUT, y_g, drop_offset, 8, pb)) return;
  }  // stamps 8 (forward head done) and 9 (loss gradient done) are taken inside

  STAMP(10);
  // ---------------- depth-1 pooling + mean backward -------------------------
  // scatter_mean: grad/count; scatter_reduce amax: grad split evenly over the
  // members equal to the max ((src==max) * grad/ties, so NaN stays NaN).
  // dS2[k][o] (the gradient at H2's pre-activation) is formed per neighbour
  // inside dY2 = A1^T dS2 (pooled graph, transposed CSR, edge order): no dS2
  // array and no barrier between the two
  for (int p = tid; p < K0 * 64; p += NT) {
    const int j = p >> 6, o = p & 63;
    float dgs = 0.f;  // dG[o]: the head's 16 per-wave partials in order (ginet_head, dg_deferred)
#pragma unroll
    for (int rc = 0; rc < NW; ++rc) dgs += t.dgp[rc * 64 + o];
    const float dgo = dgs / (float)K1;
    float acc = 0.f;
    if (one_cl) {  // the one cluster's tie count per channel, here instead of in the pooling step
      const float mx = t.p2[o];
      float ties = 0.f;
      for (int q = 0; q < K0; ++q) ties += (t.h2[q * 64 + o] == mx) ? 1.f : 0.f;
      for (int e = t.p1trp[j]; e < t.p1trp[j + 1]; ++e) {
        const float h = t.h2[t.p1tc[e] * 64 + o];
        acc += relu_bwd(h, (h == mx ? 1.f : 0.f) * (dgo / ties));
      }
    } else {
      for (int e = t.p1trp[j]; e < t.p1trp[j + 1]; ++e) {
        const int k = t.p1tc[e], mo = t.cl1[k] * 64 + o;
        const float h = t.h2[k * 64 + o];
        acc += relu_bwd(h, (h == t.p2[mo] ? 1.f : 0.f) * (dgo / t.nt[mo]));
      }
    }
    t.y2[p] = acc;
  }
  __syncthreads();
  STAMP(11);
  STAMP(12);
  // conv2 weight-gradient partials, and the gradient reaching each depth-0
  // arg member through relu (v = relu'(H1[arg]) * dP1); with many clusters on MFMA:
  // dW2 = dY2^T P1 per branch (4 tiles of 16 x 16, K = K0) and
  // dP1 = dY2 W2 per branch (ceil(K0/16) row tiles, K = 32); one wave per tile
  if (K0 < 12) {  // few clusters: direct loops
    float* slab = a.p.slab + (int64_t)pb * DR_SLAB_STRIDE(F) + 32 * F;
    for (int p = tid; p < 1024; p += NT) {
      const int br = p >> 9, o = ((p >> 4) & 31) + br * 32, j = p & 15;
      float acc = 0.f;
      int k = 0;
      for (; k + 4 <= K0; k += 4) {  // 8 independent reads, then the fmaf chain in k order
        float yv[4], pv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          yv[u] = t.y2[(k + u) * 64 + o];
          pv[u] = t.p1[(k + u) * 32 + br * 16 + j];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = fmaf(yv[u], pv[u], acc);
      }
      for (; k < K0; ++k) acc = fmaf(t.y2[k * 64 + o], t.p1[k * 32 + br * 16 + j], acc);
      if (ACC) t.acc[32 * F + p] += acc;
      else drk::st_part<WT>(slab + p, acc);
    }
    for (int p = tid; p < K0 * 32; p += NT) {
      const int k = p >> 5, ch = p & 31, br = ch >> 4, j = ch & 15;
      const float* wb = t.w2 + br * 512;
      float acc = 0.f;
#pragma unroll 8
      for (int o = 0; o < 32; ++o) acc = fmaf(t.y2[k * 64 + br * 32 + o], wb[o * 16 + j], acc);
      const int i = t.a1[p];
      t.dp1[p] = (i < N) ? relu_bwd(t.p1[p], acc) : 0.f;  // P1 = H1[arg] exactly
    }
  } else
  {
    const int lane = tid & 63, wave = dr_wave<ACC>(tid), li = lane & 15, kq = lane >> 4;
    float* slab = a.p.slab + (int64_t)pb * DR_SLAB_STRIDE(F) + 32 * F;
    const int nrt = (K0 + 15) >> 4;
    for (int job = wave; job < 4 + 2 * nrt; job += NW) {
      if (job < 4) {
        const int br = job >> 1, ot = job & 1;
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int k0 = 0; k0 < K0; k0 += 4) {
          const int k = k0 + kq;
          const float av = k < K0 ? t.y2[k * 64 + br * 32 + ot * 16 + li] : 0.f;
          const float bv = k < K0 ? t.p1[k * 32 + br * 16 + li] : 0.f;
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
        }
        if (ACC) {  // the four sums read first, then written (no read-after-write chain)
          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = t.acc[32 * F + br * 512 + (ot * 16 + kq * 4 + r) * 16 + li];
#pragma unroll
          for (int r = 0; r < 4; ++r) t.acc[32 * F + br * 512 + (ot * 16 + kq * 4 + r) * 16 + li] = o[r] + acc[r];
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) drk::st_part<WT>(slab + br * 512 + (ot * 16 + kq * 4 + r) * 16 + li, acc[r]);
        }
      } else {
        const int q = job - 4, br = q & 1, r0 = (q >> 1) * 16;
        const int kr = min(r0 + li, K0 - 1);
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int o = 4 * u + kq;
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(t.y2[kr * 64 + br * 32 + o], t.w2[br * 512 + o * 16 + li], acc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int k = r0 + kq * 4 + r;
          if (k < K0) {
            const int p = k * 32 + br * 16 + li;
            const int i = t.a1[p];
            t.dp1[p] = (i < N) ? relu_bwd(t.p1[p], acc[r]) : 0.f;  // P1 = H1[arg] exactly
          }
        }
      }
    }
  }
  __syncthreads();

  STAMP(13);
  // ---------------- dW1cat[c, :] = sum_k v[k, c] * Z[arg(k, c), :] ---------
  // (dH1 is non-zero only at the depth-0 arg members, so dS1^T (A X) needs
  // K0 rows of Z per channel instead of a backward gather over all edges.)
  {
    const int SS = DR_SLAB_STRIDE(F);
    float* slab = a.p.slab + (int64_t)pb * SS;
    // G clusters at a time, the last group predicated (clusters past K0 and
    // empty ones contribute nothing): every Z read of a group in flight (HBM on
    // the large path: with many clusters, groups of 16 halve the round trips),
    // then accumulated in cluster order (same fmaf chain)
    auto dw1 = [&](auto g_t) {
      constexpr int G = decltype(g_t)::value;
      for (int p = tid; p < 32 * F; p += NT) {
        const int ch = p / F, kk = p - ch * F;
        float acc = 0.f;
        for (int k = 0; k < K0; k += G) {
          float zv[G], dv[G];
          bool ok[G];
#pragma unroll
          for (int u = 0; u < G; ++u) {
            const bool in = k + u < K0;
            const int i = in ? t.a1[(k + u) * 32 + ch] : N;
            ok[u] = i < N;
            dv[u] = in ? t.dp1[(k + u) * 32 + ch] : 0.f;
            zv[u] = zat(ok[u] ? i : 0, kk);
          }
#pragma unroll
          for (int u = 0; u < G; ++u)
            if (ok[u]) acc = fmaf(dv[u], zv[u], acc);
        }
        if (ACC) t.acc[p] += acc;
        else drk::st_part<WT>(slab + p, acc);
      }
    };
    if (K0 > 8) dw1(std::integral_constant<int, 16>());  // (all of K0 <= 32 in flight at once: +0.6 us atom, not kept)
    else dw1(std::integral_constant<int, 8>());
  }
  STAMP(14);
}

// A graph descriptor by one s_load_dwordx16 (the pointer is wave-uniform);
// `touch` (optional): one dword of another descriptor loaded beside it and
// dropped, so that line is in the scalar cache when its graph starts
__device__ __forceinline__ uint64_t uniform_ptr(const void* p) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(u >> 32)) << 32) | (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)u);
}
__device__ __forceinline__ dr_graph_desc desc_scalar(const dr_graph_desc* p, const dr_graph_desc* touch = nullptr) {
  typedef int v16i __attribute__((ext_vector_type(16)));
  v16i r;
  if (touch) {
    int dropped;
    asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dword %1, %3, 0x0\n\ts_waitcnt lgkmcnt(0)"
                 : "=s"(r), "=s"(dropped)
                 : "s"(uniform_ptr(p)), "s"(uniform_ptr(touch)));
  } else {
    asm volatile("s_load_dwordx16 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(uniform_ptr(p)));
  }
  dr_graph_desc d;
  __builtin_memcpy(&d, &r, sizeof(d));
  return d;
}

// Accumulating pass (dr_ginet_acc_pass): a workgroup runs graphs gi, gi + R,
// ... one after another and adds each graph's gradients to running sums (LDS
// region acc at the front of its LDS, fc1.weight's in the caller's registers)
// instead of writing per-graph partials; the graph carve starts acc_words in.
struct AccCtx {
  int gi = -1;           // the graph (batch position) this call runs
  float* acc = nullptr;  // [dW1cat 32F | dW2cat 1024 | GinetHeadLds::acc's block]
  float* accf = nullptr;  // fc1.weight's sums in the kernel's registers (null: in acc)
  int acc_words = 0;
  // prefetch layout (graph_body<..., PF = true>): this graph's tail-input
  // buffer (parity), whether its inputs and W1 still need staging (the
  // workgroup's first graph), and the next graph's batch position (-1: none)
  AccLayout lay;
  int par = 0, next = -1;
  bool first = true;
  int64_t step = 0;  // dr_pass.step_counter[0] (constant for the launch)
  // PF: LDS word set to 1 by the graph whose idle waves staged the next
  // graph's inputs (read by that next graph before its staging)
  uint32_t* staged = nullptr;
};

// KPT: conv1's K (F) padded to whole 16-deep MFMA steps, 32 (F <= 32) or 64.
// ACC / PF: the accumulating pass (AccCtx) and its prefetch layout.  Returns
// the step counter value the pass used (its dropout offset).
template <int KPT, bool ACC = false, bool PF = false>
__device__ __forceinline__ uint64_t graph_body(const GinetArgs& a, const AccCtx& ac) {
  extern __shared__ __attribute__((aligned(16))) float lds_raw[];
  float* lds = lds_raw + (ACC ? ac.acc_words : 0);
  const int tid = dr_tid<ACC>();
  const int lane = tid & 63;
  const int wave = dr_wave<ACC>(tid);
  const int b = ACC ? ac.gi : (int)blockIdx.x;
  const dr_graph_store& s = a.s;
  // one 64-byte scalar load (ACC: spelled out — in the accumulating kernel's
  // loop hipcc cannot prove the descriptors unwritten and reads them with
  // vector loads and readfirstlanes, ~1 K cycles)
  const dr_graph_desc d = ACC ? desc_scalar(a.descs + b, ac.next >= 0 ? a.descs + ac.next : nullptr) : a.descs[b];
  const int g = d.gid;
  const int64_t n0 = d.node0, ec0 = d.col0, k00 = d.k0, q0 = d.p1, k10 = d.k1;
  const int N = d.n_nodes, E = d.n_edges, K0 = d.n_k0, P1 = d.n_p1, K1 = d.n_k1;
  const int F = s.n_feat;
  const int alias = s.transpose_aliased;
  const int OUT = a.p.out_dim;
  // Fetch every kernel-argument field the staging needs, and the descriptor,
  // in one scalar round trip each (hipcc would otherwise load them lazily
  // with a wait before each DMA).
  asm volatile("" ::"s"(s.x), "s"(s.col), "s"(s.rowptr), "s"(s.cl0), "s"(s.p1_rowptr), "s"(s.p1_col),
               "s"(s.p1t_rowptr), "s"(s.p1t_col), "s"(s.m1_ptr), "s"(s.m1_idx), "s"(s.y), "s"(F), "s"(alias),
               "s"(OUT), "s"(n0), "s"(ec0), "s"(k00), "s"(q0), "s"(k10), "s"(N), "s"(E), "s"(K0), "s"(P1), "s"(K1),
               "s"(g));
  const Carve c = PF ? carve_acc(N, E, F, K0, P1, K1, alias, OUT, ac.lay, ac.par) : carve(N, E, F, K0, P1, K1, alias, OUT);
  const int LDW = c.LDW, XS = c.XS;

  float* sW1 = lds + c.w1;
  float* sW2 = lds + c.w2;
  float* sFc2 = lds + c.fc2;
  float* sX = lds + c.x;
  float* sZ = lds + c.z;
  int* srp = reinterpret_cast<int*>(lds + c.rp);
  uint16_t* scol = reinterpret_cast<uint16_t*>(lds + c.col);
  int* scl0 = reinterpret_cast<int*>(lds + c.cl0);
  unsigned long long* skey = reinterpret_cast<unsigned long long*>(lds + c.key);
  float* sP1 = lds + c.p1;
  int* sA1 = reinterpret_cast<int*>(lds + c.a1);
  int* sp1rp = reinterpret_cast<int*>(lds + c.p1rp);
  int* sp1c = reinterpret_cast<int*>(lds + c.p1c);
  int* sp1trp = reinterpret_cast<int*>(lds + c.p1trp);
  int* sp1tc = reinterpret_cast<int*>(lds + c.p1tc);
  int* sm1p = reinterpret_cast<int*>(lds + c.m1p);
  int* sm1i = reinterpret_cast<int*>(lds + c.m1i);
  uint8_t* skeep = reinterpret_cast<uint8_t*>(lds + c.keep);

  STAMP(0);
  // ---------------- stage the graph into LDS --------------------------------
  // Only the graph and conv1's weights are staged (DMA'd straight into LDS):
  // one CU pulls ~11-30 B/cycle, so the staging time is its bytes, and the
  // head's 64 KB of fc1 registers (row and column layouts) are loaded after
  // the staging barrier instead, under the LDS-bound front half.
  float fc1_row[8], fc1_col[8], fc1_bias;
  auto load_fc1 = [&]() {
    const int r = tid >> 3, part = tid & 7;
    const float4 u0 = *reinterpret_cast<const float4*>(a.w.fc1w + r * 64 + part * 8);
    const float4 u1 = *reinterpret_cast<const float4*>(a.w.fc1w + r * 64 + part * 8 + 4);
    fc1_row[0] = u0.x; fc1_row[1] = u0.y; fc1_row[2] = u0.z; fc1_row[3] = u0.w;
    fc1_row[4] = u1.x; fc1_row[5] = u1.y; fc1_row[6] = u1.z; fc1_row[7] = u1.w;
    fc1_bias = a.w.fc1b[r];
    const int o = tid & 63, rcc = dr_wave<ACC>(tid);
#pragma unroll
    for (int j = 0; j < 8; ++j) fc1_col[j] = a.w.fc1w[(rcc * 8 + j) * 64 + o];
  };
  // (ACC: scalar loads through the constant address space — read-only for the
  // launch; hipcc cannot prove that in the accumulating loop and would use a
  // vector load, waited for by the staging's vmcnt(0))
  typedef const __attribute__((address_space(4))) float* CF32;
  const float y_g = ACC ? *(CF32)(s.y + g) : s.y[g];
  uint64_t drop_offset = a.p.drop_offset;
  // the graph's inputs (PF: graph k+1's are DMA'd during graph k's tail)
  // (asm-issued: waited for by the s_waitcnt vmcnt(0) before the staging barrier)
  auto stage_inputs = [&](const dr_graph_desc& dd, const Carve& cc) {
    const int64_t dn0 = dd.node0, dk00 = dd.k0;
    const int dg = dd.gid, dN = dd.n_nodes, dK0 = dd.n_k0;
    dma_x4_async(lds + cc.x, s.x + dn0 * (int64_t)XS, dN * XS / 4, tid);
    dma_x4_async(lds + cc.col, s.col + dd.col0, (dd.n_edges + 7) / 8, tid, 7);
    dma_words_async(lds + cc.rp, s.rowptr + dn0 + dg, dN + 1, tid, 13);
    dma_words_async(lds + cc.cl0, s.cl0 + dn0, dN, tid, 3);
    dma_words_async(lds + cc.p1rp, s.p1_rowptr + dk00 + dg, dK0 + 1, tid, 10);
    dma_words_async(lds + cc.p1c, s.p1_col + dd.p1, dd.n_p1, tid, 11);
    if (!alias) {
      dma_words_async(lds + cc.p1trp, s.p1t_rowptr + dk00 + dg, dK0 + 1, tid, 12);
      dma_words_async(lds + cc.p1tc, s.p1t_col + dd.p1, dd.n_p1, tid, 9);
    }
    dma_words_async(lds + cc.m1p, s.m1_ptr + dd.k1 + dg, dd.n_k1 + 1, tid, 8);
    dma_words_async(lds + cc.m1i, s.m1_idx + dk00, dK0, tid, 1);
  };
  if (!PF) {  // (DR_DMA_ROT = 1: starting waves spread over the copies; measured slower)
    dma_x4(sX, s.x + n0 * (int64_t)XS, N * XS / 4, tid);
    dma_x4(scol, s.col + ec0, (E + 7) / 8, tid, DR_DMA_ROT * 7);
    dma_words(srp, s.rowptr + n0 + g, N + 1, tid, DR_DMA_ROT * 13);
    dma_words(scl0, s.cl0 + n0, N, tid, DR_DMA_ROT * 3);
    dma_words(sp1rp, s.p1_rowptr + k00 + g, K0 + 1, tid, DR_DMA_ROT * 10);
    dma_words(sp1c, s.p1_col + q0, P1, tid, DR_DMA_ROT * 11);
    if (!alias) {
      dma_words(sp1trp, s.p1t_rowptr + k00 + g, K0 + 1, tid, DR_DMA_ROT * 12);
      dma_words(sp1tc, s.p1t_col + q0, P1, tid, DR_DMA_ROT * 9);
    }
    dma_words(sm1p, s.m1_ptr + k10 + g, K1 + 1, tid, DR_DMA_ROT * 8);
    dma_words(sm1i, s.m1_idx + k00, K0, tid, DR_DMA_ROT * 1);
  } else if (ac.first || *ac.staged == 0u) {
    stage_inputs(d, c);
  }
  if (!PF || ac.first) {
    dma_words(sW1, a.w.w1, 16 * F, tid, DR_DMA_ROT * 5);  // [W1; W1e] rows of F, packed
    dma_words(sW1 + 16 * F, a.w.w1e, 16 * F, tid, DR_DMA_ROT * 14);
  }
  {  // zero Z's K padding (cols XS..KPT; X's own pad is zero) and the pooling keys
    const int padz = KPT - XS;  // (rows are KP = KPT wide, carve)
    for (int p = tid; p < N * padz; p += NT) {
      const int i = p / padz;
      sZ[i * LDW + XS + (p - i * padz)] = 0.f;
    }
    for (int p = tid; p < K0 * 32; p += NT) skey[p] = 0ull;
    if (tid < 64) lds[c.p2 + tid] = 0.f;  // (TailLds::p2_zeroed)
  }
  // loaded late: no early wait (ACC: read once per launch by the kernel)
  if (a.p.step_counter) drop_offset = ACC ? (uint64_t)ac.step : (uint64_t)a.p.step_counter[0];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // snapshot for dr_reduce_update, stored only now so that no wait for the
  // counter load sits between the descriptor and the graph DMA
  if (a.p.step_counter && b == 0 && tid == 0) a.p.step_counter[1] = (int64_t)drop_offset;
  __syncthreads();

  STAMP(1);
  // The conv2 / head weights are not needed before the tail: load them into
  // VGPRs now and store them to LDS after the front half, so their latency
  // overlaps it.  (An LDS DMA here would make hipcc wait for it before every
  // LDS read.)
  float wv2, wfc[3];
  auto load_head_weights = [&]() {
    wv2 = (tid < 512) ? a.w.w2[tid] : a.w.w2e[tid - 512];
    const int nf = OUT * 128;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int p = tid + u * NT;
      wfc[u] = 0.f;
      if (p < nf) wfc[u] = a.w.fc2w[p];
      else if (p < nf + OUT) wfc[u] = a.w.fc2b[p - nf];
    }
    // fc1 last: the wait for W2 / fc2 before their LDS stores (end of the
    // front half) then leaves these 11 loads in flight (vmcnt counts in order)
    load_fc1();
  };
  load_head_weights();
  // ---------------- conv1 + depth-0 pooling, one 16-row tile per wave -------
  // Each wave runs its rows through the whole front half with no workgroup
  // barrier in between:
  //   Z = A X  (ginet.py:45,58 aggregated first: A (X W^T) = (A X) W^T), 8
  //     lanes per row, edges in CSR order (torch_scatter's scatter_add_ order),
  //     two rows per lane in flight;
  //   H = relu(Z [W1;W1e]^T) on v_mfma_f32_16x16x4_f32 (exact k-ordered fmaf
  //     chain), B operands in registers;
  //   depth-0 max pool (torch_scatter scatter_max, community_pooling.py:209):
  //     a 64-bit LDS atomic max of (H bits << 32 | ~node) per (cluster,
  //     channel): H >= +0 after relu so the bit order is the value order, and
  //     among equal values the smallest node wins — the first max of the
  //     reference's node-ordered strict '>' scan; NaN never enters; an empty
  //     (cluster, channel) keeps key 0 -> value 0, no arg.  H itself is never
  //     stored: the backward needs only P1 = H[arg] and Z[arg].
  {
    const int li = lane & 15, kq = lane >> 4;
    // gather lanes -> (row slot, 16-byte chunk): ds_read_b128 serves a wave in
    // four 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, and the same
    // +32; MI355X_MICROARCH.md §LDS), so each group takes both halves of two
    // slots' rows: with 128-byte rows it then waits an extra cycle only when
    // those two rows share a bank half, not when either of two half-row pairs does
    const int q4 = (lane & 31) >> 2;
    const int slot = ((lane >> 5) << 2) + ((0x31130220u >> (4 * q4)) & 3);
    const int sub = (((0xCCu >> q4) & 1) << 2) | (lane & 3), nch = XS >> 2;
    // conv1 B operand of v_mfma_f32_16x16x4_f32: lane (li, kq) holds
    // W[li][k + 4u + kq] (wa: conv1 rows, wb: conv1_ext rows), zero past F
    constexpr int NKV = KPT / 4;
    float wa[NKV], wb[NKV];
#pragma unroll
    for (int j = 0; j < NKV; ++j) {
      const int kk = 16 * (j >> 2) + 4 * (j & 3) + kq;
      wa[j] = kk < F ? sW1[li * F + kk] : 0.f;
      wb[j] = kk < F ? sW1[(16 + li) * F + kk] : 0.f;
    }
    if (PF) {  // the waves with no tile stage the next graph's inputs into the other buffer
      const int busy = (N + 15) >> 4;
      if (ac.next >= 0 && busy < NW && wave >= busy) {
        const dr_graph_desc dn = desc_scalar(a.descs + ac.next);
        const Carve cn = carve_acc(dn.n_nodes, dn.n_edges, F, dn.n_k0, dn.n_p1, dn.n_k1, alias, OUT, ac.lay, ac.par ^ 1);
        const int nw = NW - busy;
        const int64_t dn0 = dn.node0, dk00 = dn.k0;
        const int dg = dn.gid, dN = dn.n_nodes, dK0 = dn.n_k0;
        dma_x4_async_sub(lds + cn.x, s.x + dn0 * (int64_t)XS, dN * XS / 4, tid, busy, nw);
        dma_x4_async_sub(lds + cn.col, s.col + dn.col0, (dn.n_edges + 7) / 8, tid, busy, nw);
        dma_words_async_sub(lds + cn.rp, s.rowptr + dn0 + dg, dN + 1, tid, busy, nw);
        dma_words_async_sub(lds + cn.cl0, s.cl0 + dn0, dN, tid, busy, nw);
        dma_words_async_sub(lds + cn.p1rp, s.p1_rowptr + dk00 + dg, dK0 + 1, tid, busy, nw);
        dma_words_async_sub(lds + cn.p1c, s.p1_col + dn.p1, dn.n_p1, tid, busy, nw);
        if (!alias) {
          dma_words_async_sub(lds + cn.p1trp, s.p1t_rowptr + dk00 + dg, dK0 + 1, tid, busy, nw);
          dma_words_async_sub(lds + cn.p1tc, s.p1t_col + dn.p1, dn.n_p1, tid, busy, nw);
        }
        dma_words_async_sub(lds + cn.m1p, s.m1_ptr + dn.k1 + dg, dn.n_k1 + 1, tid, busy, nw);
        dma_words_async_sub(lds + cn.m1i, s.m1_idx + dk00, dK0, tid, busy, nw);
      }
      if (tid == 0) *ac.staged = (ac.next >= 0 && busy < NW) ? 1u : 0u;
    }
    for (int tt = wave; tt * 16 < N; tt += NW) {
      const int r0 = tt * 16;
#if DR_GATHER_ROW2
      if (nch <= 8) {  // one row per lane (r0 + lane/4), chunks q and q ^ 4 (q = lane%4, or +4 on odd rows)
        const int i = r0 + (lane >> 2);
        const int ca = (lane & 3) | ((lane & 4)), cb = ca ^ 4;
        const int eb = i < N ? srp[i] : 0, ee = i < N ? srp[i + 1] : 0;
        float4 za, zb;
#if DR_GATHER_IMM
        drk::gather_row_two_chunks_imm(scol, eb, ee, reinterpret_cast<const char*>(sX + ca * 4), (cb - ca) * 16, XS * 4, za, zb);
#else
        drk::gather_row_two_chunks(scol, eb, ee, sX, XS, ca * 4, cb * 4, za, zb);
#endif
        if (i < N) {
          // (rows LDW = KP + 2 words apart: 8-byte aligned, two 64-bit stores per chunk)
          if (ca < nch) {
            float2* zr = reinterpret_cast<float2*>(sZ + i * LDW + ca * 4);
            zr[0] = make_float2(za.x, za.y);
            zr[1] = make_float2(za.z, za.w);
          }
          if (cb < nch) {
            float2* zr = reinterpret_cast<float2*>(sZ + i * LDW + cb * 4);
            zr[0] = make_float2(zb.x, zb.y);
            zr[1] = make_float2(zb.z, zb.w);
          }
        }
      } else
#endif
      {  // rows r0+slot and r0+8+slot together: two independent edge chains per lane
        const int i0 = r0 + slot, i1 = r0 + 8 + slot;
        const int eb0 = i0 < N ? srp[i0] : 0, ee0 = i0 < N ? srp[i0 + 1] : 0;
        const int eb1 = i1 < N ? srp[i1] : 0, ee1 = i1 < N ? srp[i1 + 1] : 0;
        for (int ch = sub; ch < nch; ch += 8) {
          float4 z0, z1;
          drk::gather_two_row_chunks(scol, eb0, ee0, eb1, ee1, sX, XS, ch * 4, z0, z1);
          if (i0 < N) {
            float* zr = sZ + i0 * LDW + ch * 4;
            zr[0] = z0.x;
            zr[1] = z0.y;
            zr[2] = z0.z;
            zr[3] = z0.w;
          }
          if (i1 < N) {
            float* zr = sZ + i1 * LDW + ch * 4;
            zr[0] = z1.x;
            zr[1] = z1.y;
            zr[2] = z1.z;
            zr[3] = z1.w;
          }
        }
      }
      // this wave's Z rows are complete in LDS before its own MFMA reads them
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (tt == 0) STAMP(20);  // (wave 0's first tile: gather done)
      const int ar = min(r0 + li, N - 1);  // rows past N compute garbage that is never pooled
      floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KPT / 16; ++ks) {
        float av[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) av[u] = sZ[ar * LDW + ks * 16 + 4 * u + kq];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], wa[4 * ks + u], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], wb[4 * ks + u], acc1, 0, 0, 0);
        }
      }
      if (tt == 0) STAMP(21);  // (MFMA issued)
      // the four rows' clusters in one 16-byte read (rows past N: unused)
      const int4 kk4 = *reinterpret_cast<const int4*>(scl0 + r0 + kq * 4);
      const int kk[4] = {kk4.x, kk4.y, kk4.z, kk4.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + kq * 4 + r;
        if (row < N) {
          const int k = kk[r];
          const unsigned long long low = 0xffffffffull - (unsigned long long)(uint32_t)row;
          const float v0 = relu_keepnan(acc0[r]), v1 = relu_keepnan(acc1[r]);
          if (v0 == v0)
            __hip_atomic_fetch_max(skey + k * 32 + li, ((unsigned long long)__float_as_uint(v0) << 32) | low,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (v1 == v1)
            __hip_atomic_fetch_max(skey + k * 32 + 16 + li, ((unsigned long long)__float_as_uint(v1) << 32) | low,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      if (tt == 0) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        STAMP(22);  // (pool atomics done)
      }
    }
  }
  // the head's dropout keep flags, by the last two waves (idle in the front
  // half up to N = 224): off the tail's critical path
  if (tid >= NT - 128) {
    const int r = tid - (NT - 128);
    if (a.p.use_dropout) skeep[r] = drk::keep_unit(a.p, drop_offset, a.p.slot ? a.p.slot[b] : b, r) ? 1 : 0;
  }
  sW2[tid] = wv2;
  {
    const int nf = OUT * 128 + OUT;
#pragma unroll
    for (int u = 0; u < 3; ++u)
      if (tid + u * NT < nf) sFc2[tid + u * NT] = wfc[u];
  }
  STAMP(2);
  __syncthreads();
  STAMP(3);
  // (no barrier after the decode: conv2, the tail's first step, reads the
  // pooled rows from the keys themselves — TailLds::key)
  for (int p = tid; p < K0 * 32; p += NT) {
    const unsigned long long key = skey[p];
    sP1[p] = key ? __uint_as_float((uint32_t)(key >> 32)) : 0.f;
    sA1[p] = key ? (int)(0xffffffffu - (uint32_t)key) : N;
  }
  if (!DR_CONV2_KEYS) __syncthreads();

  TailLds t = tail_lds(c, lds);
  t.key = !DR_CONV2_KEYS ? nullptr : skey;
  t.p2_zeroed = true;
  t.keep = skeep;
  t.acc = ACC ? ac.acc : nullptr;
  t.accf = ACC ? ac.accf : nullptr;
  auto zat = [&](int i, int kk) { return sZ[i * LDW + kk]; };
  // (dr_pass.slot: the graph's rows of the batch when it is split over launches)
  const int orow = a.p.slot ? a.p.slot[b] : b;
  ginet_tail<decltype(zat), false, ACC>(a, t, fc1_row, fc1_col, fc1_bias, orow, N, K0, K1, F, OUT, y_g, drop_offset, zat, orow);
  return drop_offset;
}

template <int KPT>
__global__ void __launch_bounds__(NT) ginet_graph_kernel(GinetArgs a) {
#ifdef DR_STAMPS  // cross-kernel timeline (s_memrealtime, 100 MHz chip clock): slots 30 / 31 = entry / exit
  if (threadIdx.x == 0 && a.p.stamps) a.p.stamps[(int64_t)blockIdx.x * 32 + 30] = __builtin_amdgcn_s_memrealtime();
#endif
  graph_body<KPT>(a, AccCtx{});
#ifdef DR_STAMPS
  if (threadIdx.x == 0 && a.p.stamps) a.p.stamps[(int64_t)blockIdx.x * 32 + 31] = __builtin_amdgcn_s_memrealtime();
#endif
}

// ---------------------------------------------------------------------------
// Accumulating pass (dr_ginet_acc_pass; batches past the CU count): R
// workgroups, workgroup w runs graphs w, w + R, w + 2R, ... in that order and
// sums their gradients on chip — the conv weights' and the head's in an LDS
// region ahead of the graph carve, fc1.weight's (dh (x) g, 128 x 64) in
// registers — then writes ONE row [dW1cat | dW2cat | fc1.weight | fc1.bias |
// fc2.weight | fc2.bias] (dr_ginet_acc_row_floats) and its loss sum to
// loss_per_graph[w].  The reduce then sums R rows instead of B per-graph
// partials (and no outer products): the per-graph slab, B x (32F + 1024 +
// 320) floats written and read back per step, becomes R x ~10 K.  The graph
// -> workgroup map and each workgroup's order are fixed, so the sums are
// deterministic (another fp32 association than the per-graph partials: the
// tests compare the two at fp32 tolerance).
// ---------------------------------------------------------------------------
// The accumulators (LDS, ahead of the graph carve): [dW1cat 32F | dW2cat 1024
// | fc1.bias 128 | fc2.weight OUT x 128 | fc2.bias OUT | loss | pad | fc1.weight
// 128 x 64 unless it is summed in registers (F <= 32)].  The row written per
// workgroup: [dW1cat | dW2cat | fc1.weight | fc1.bias | fc2.weight | fc2.bias].
__host__ __device__ inline int acc_row_floats(int F, int OUT) { return r4(32 * F + 1024 + 128 * 64 + 128 + 128 * OUT + OUT); }
__host__ __device__ inline int acc_head_words(int OUT) { return r4(128 + 128 * OUT + OUT + 1); }
__host__ __device__ inline int acc_words(int F, int OUT, bool fc1_in_lds) {
  return 32 * F + 1024 + acc_head_words(OUT) + (fc1_in_lds ? 128 * 64 : 0);
}

template <int KPT, bool PF>
__global__ void __launch_bounds__(NT) ginet_acc_kernel(GinetArgs a, const int32_t* plan, AccLayout lay) {
  extern __shared__ __attribute__((aligned(16))) float lds_raw[];
  const int F = a.s.n_feat, OUT = a.p.out_dim, tid = threadIdx.x;
  constexpr bool REG = KPT == 32;  // fc1.weight's sums in registers where the kernel has them to spare
  AccCtx ac;
  ac.acc = lds_raw;
  ac.acc_words = acc_words(F, OUT, !REG) + 4;  // + the staged flag (16 bytes)
  ac.staged = reinterpret_cast<uint32_t*>(lds_raw + ac.acc_words - 4);
  ac.lay = lay;
  typedef const __attribute__((address_space(4))) int64_t* CI64K;
  ac.step = a.p.step_counter ? *(CI64K)a.p.step_counter : 0;
  float accf[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  ac.accf = REG ? accf : nullptr;
  for (int p = tid; p < ac.acc_words; p += NT) lds_raw[p] = 0.f;
  __syncthreads();
  // plan: [R + 1 starts | the batch positions, workgroup by workgroup], or
  // null: every R-th position from blockIdx.x
  const int R = gridDim.x, w = blockIdx.x;
  typedef const __attribute__((address_space(4))) int32_t* CPlan;  // scalar loads (read-only for the launch)
  const CPlan cp = (CPlan)plan;
  const int k0 = plan ? cp[w] : 0, k1 = plan ? cp[w + 1] : (a.B - w + R - 1) / R;
  for (int k = k0; k < k1; ++k) {
    ac.gi = plan ? cp[R + 1 + k] : w + k * R;
    ac.first = k == k0;
    ac.par = (k - k0) & 1;
    ac.next = k + 1 < k1 ? (plan ? cp[R + 2 + k] : w + (k + 1) * R) : -1;
    // the body reads the arguments from the kernarg segment through a pointer
    // the optimiser cannot follow across iterations: each graph reloads what it
    // uses (scalar loads) instead of every argument being held in SGPRs over the
    // whole loop (spilled to VGPR lanes: ~650 readlane/writelane)
    typedef const __attribute__((address_space(4))) GinetArgs* KArgs;
    KArgs ka = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("; dr_kargs" : "+s"(ka));
    graph_body<KPT, true, PF>(*(const GinetArgs*)ka, ac);
    __syncthreads();  // the graph carve is restaged by the next graph
  }
  // the workgroup's row, then its loss sum
  const int c0 = 32 * F + 1024, HW = 128 + 128 * OUT + OUT;
  float* row = a.p.slab + (int64_t)blockIdx.x * acc_row_floats(F, OUT);
  for (int p = tid; p < c0 / 4; p += NT) reinterpret_cast<float4*>(row)[p] = reinterpret_cast<const float4*>(lds_raw)[p];
  float4* rw = reinterpret_cast<float4*>(row + c0 + tid * 8);
  if (REG) {
    rw[0] = make_float4(accf[0], accf[1], accf[2], accf[3]);
    rw[1] = make_float4(accf[4], accf[5], accf[6], accf[7]);
  } else {
    const float4* src = reinterpret_cast<const float4*>(lds_raw + c0 + acc_head_words(OUT) + tid * 8);
    rw[0] = src[0];
    rw[1] = src[1];
  }
  for (int p = tid; p < HW; p += NT) row[c0 + 128 * 64 + p] = lds_raw[c0 + p];
  if (tid == 0) a.p.loss_per_graph[blockIdx.x] = lds_raw[c0 + HW];
}

// =========================================================================
// Graphs larger than one workgroup's LDS (atom-level: N ~ 3e3, E ~ 5e4).
// =========================================================================

constexpr int NTA = 512;  // conv1 tile kernel: 8 waves
constexpr int TR = DR_LARGE_TILE;

struct LargeArgs {
  GinetArgs g;
  dr_large_plan plan;
};

struct ConvCarve {
  int KP, LDW, XS, w1, z, h, m0i, m0p, rng, flg, xh, hid, lcol, trp, total;
};

// HM / EM: halo rows and edges of the largest tile (0: no halo staging)
__host__ __device__ inline ConvCarve conv_carve(int N, int F, int K0, int HM, int EM) {
  ConvCarve c;
  c.KP = r16(F);
  c.LDW = c.KP + 2;
  c.XS = r4(F);
  int o = 0;
  c.w1 = o;
  o += r4(32 * c.LDW);
  c.z = o;
  o += r4(TR * c.LDW);
  // with halos (HM > 0): H lives in the halo-X region (dead after the
  // gather) and the tile's own member lists replace the graph's
  c.h = o;
  o += HM ? 0 : TR * 32;
  c.m0i = o;
  o += r4(HM ? TR : N);
  c.m0p = o;
  o += r4(K0 + 1);
  c.rng = o;
  o += r4(2 * K0);
  c.flg = o;  // per tile row: a depth-0 pooling arg candidate (its Z row is stored)
  o += r4(TR);
  c.xh = o;  // halo X rows (XS stride, 16-byte rows), then H
  o += HM ? r4(drk::imax(HM * c.XS, TR * 32)) : 0;
  if (HM) c.h = c.xh;
  c.hid = o;
  o += r4(HM);
  c.trp = o;  // the tile's rowptr slice
  o += HM ? r4(TR + 1) : 0;
  c.lcol = o;  // the tile's edges as halo indices (uint16); last, so its size moves nothing
  o += HM ? r4((EM + 8) / 2) : 0;
  c.total = o;
  return c;
}

// first position in the ascending run v[lo, hi) whose value is >= key
__device__ __forceinline__ int lower_bound_lds(const int* v, int lo, int hi, int key) {
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (v[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Global-address-space views for in-launch hand-offs (MI355X_MICROARCH.md
// §inter-workgroup visibility): agent-scope relaxed atomics lower to sc1
// global loads/stores, which bypass the per-CU L1 and write through the
// per-XCD L2, so a payload stored this way, drained (s_waitcnt vmcnt(0)) and
// signalled by an agent-scope counter add is read correctly by the workgroup
// whose add came last with sc1 loads, wherever the two sit.

template <bool INL>
__device__ __forceinline__ void store_u64(void* p, uint64_t v) {
  if (INL) __hip_atomic_store((gu64*)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *reinterpret_cast<uint64_t*>(p) = v;
}
template <bool INL>
__device__ __forceinline__ void store_z4(float* p, float4 v) {
  if (INL) {
    store_u64<true>(p, (uint64_t)__float_as_uint(v.x) | ((uint64_t)__float_as_uint(v.y) << 32));
    store_u64<true>(p + 2, (uint64_t)__float_as_uint(v.z) | ((uint64_t)__float_as_uint(v.w) << 32));
  } else {
    *reinterpret_cast<float4*>(p) = v;
  }
}
__device__ __forceinline__ uint32_t load_sc1_u32(const void* p) {
  return __hip_atomic_load((const gu32*)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The tile's partial depth-0 max per (cluster, channel) of H (LDS, stride
// 32, rows r0..r0+nrows-1): strict '>' in node order, first max wins, NaN never
// enters (torch_scatter scatter_max, community_pooling.py:209).  Published by
// 64-bit atomic max keys or per-tile partials (dr_large_plan).
template <int NTT, bool INL>
__device__ __forceinline__ void tile_partial_max(const dr_large_plan& pl, const float* sH, const int* sm0i,
                                                 const int* sm0p, int* srng, bool compact, int tile, int b, int K0,
                                                 int N, int r0, int nrows, int* sflag = nullptr) {
  const int tid = threadIdx.x;
  // each cluster's members inside this tile: a sub-run of its ascending list
  for (int k = tid; k < K0; k += NTT) {
    const int mb = sm0p[k], me = sm0p[k + 1];
    srng[2 * k] = compact ? mb : lower_bound_lds(sm0i, mb, me, r0);
    srng[2 * k + 1] = compact ? me : lower_bound_lds(sm0i, mb, me, r0 + nrows);
  }
  __syncthreads();
  for (int p = tid; p < K0 * 32; p += NTT) {
    const int k = p >> 5, ch = p & 31;
    float best = LOWEST;
    int arg = N;
    for (int m = srng[2 * k]; m < srng[2 * k + 1]; ++m) {
      const int i = sm0i[m];
      const float v = sH[(i - r0) * 32 + ch];
      if (v > best) {
        best = v;
        arg = i;
      }
    }
    if (sflag && arg < N) sflag[arg - r0] = 1;  // (benign race: every writer stores 1)
    if (pl.part_key) {  // order-free combine over the graph's tiles (see dr_large_plan.part_key)
      if (best > LOWEST)
        __hip_atomic_fetch_max((gu64*)(pl.part_key) + ((int64_t)b * pl.k0_max + k) * 32 + ch,
                               ((unsigned long long)__float_as_uint(best) << 32) | (unsigned long long)(0xffffffffu - (uint32_t)arg),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const int64_t o = ((int64_t)tile * pl.k0_max + k) * 32 + ch;
      pl.part_val[o] = best;
      pl.part_arg[o] = arg;
    }
  }
}

// One tile of TR nodes: Z rows (CSR gather over HBM/L2), H = relu(Z W^T) on
// MFMA, and the tile's partial depth-0 max per (cluster, channel).
template <int NTT, bool INL>
__device__ __forceinline__ void conv_tile_f32(const LargeArgs& la, float* lds) {
  const GinetArgs& a = la.g;
  const dr_large_plan& pl = la.plan;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tile = drk::xcd_tile();
  const int b = pl.tile_slot[tile];
  const int t = tile - pl.tile_first[b];
  const dr_graph_desc d = a.descs[b];
  const dr_graph_store& s = a.s;
  const int g = d.gid;
  const int64_t n0 = d.node0, ec0 = d.col0, k00 = d.k0;
  const int N = d.n_nodes, K0 = d.n_k0, F = s.n_feat;
  const int TRr = pl.tile_rows;
  const int r0 = t * TRr, nrows = min(TRr, N - r0);
  const ConvCarve c = conv_carve(N, F, K0, pl.halo_max, 0);
  const int KP = c.KP, LDW = c.LDW, XS = c.XS;
  float* sW1 = lds + c.w1;
  float* sZ = lds + c.z;
  float* sH = lds + c.h;
  int* sm0i = reinterpret_cast<int*>(lds + c.m0i);
  int* sm0p = reinterpret_cast<int*>(lds + c.m0p);
  int* srng = reinterpret_cast<int*>(lds + c.rng);

  const bool compact = pl.tile_members != nullptr;
  if (compact) {  // this tile's members by cluster (host-built), runs from tile_mptr
    drk::dma_words<NTT>(sm0i, pl.tile_members + (int64_t)tile * TRr, nrows);
    drk::dma_words<NTT>(sm0p, pl.tile_mptr + (int64_t)tile * (pl.k0_max + 1), K0 + 1);
  } else {
    drk::dma_words<NTT>(sm0i, s.m0_idx + n0, N);
    drk::dma_words<NTT>(sm0p, s.m0_ptr + k00 + g, K0 + 1);
  }
  for (int p = tid; p < 32 * KP; p += NTT) {  // [W1; W1e] zero-padded to KP
    const int r = p / KP, k = p - r * KP;
    float v = 0.f;
    if (k < F) v = (r < 16) ? a.w.w1[r * F + k] : a.w.w1e[(r - 16) * F + k];
    sW1[r * LDW + k] = v;
  }
  for (int p = tid; p < TRr * (KP - XS); p += NTT) {  // Z pad columns
    const int r = p / (KP - XS);
    sZ[r * LDW + XS + (p - r * (KP - XS))] = 0.f;
  }
  // Z rows go to global memory only at the tile's depth-0 pooling arg
  // candidates (the tail reads Z at the final args, which are tile args)
  constexpr bool ZARGS = DR_Z_ARGS && !INL;
  int* sflag = reinterpret_cast<int*>(lds + c.flg);
  if (ZARGS)
    for (int p = tid; p < TRr; p += NTT) sflag[p] = 0;
  if (pl.halo_ids) {
    // Halo path: stage the tile's rowptr slice, its halo ids, then the halo X
    // rows and the tile's edges (as halo indices) into LDS; gather from LDS.
    int* strp = reinterpret_cast<int*>(lds + c.trp);
    int* shid = reinterpret_cast<int*>(lds + c.hid);
    uint16_t* slcol = reinterpret_cast<uint16_t*>(lds + c.lcol);
    float* sXh = lds + c.xh;
    const int h0 = pl.halo_off[tile], H = pl.halo_off[tile + 1] - h0;
    const int l0 = pl.lcol_off[tile];
    drk::dma_words<NTT>(strp, s.rowptr + n0 + g + r0, nrows + 1);
    drk::dma_words<NTT>(shid, pl.halo_ids + h0, H);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int ebase = strp[0];
    drk::dma_x4<NTT>(slcol, pl.lcol + l0, (strp[nrows] - ebase + 7) / 8);
    {
      const float* X = s.x + n0 * (int64_t)XS;
      const int nch = XS >> 2, tot = H * nch;
      const int wv = __builtin_amdgcn_readfirstlane(wave);
      for (int base = wv * 64; base < tot; base += NTT)
        if (base + lane < tot) {
          const int hr = (base + lane) / nch, ch = base + lane - hr * nch;
          __builtin_amdgcn_global_load_lds(DRK_AS1(X + (int64_t)shid[hr] * XS + ch * 4), DRK_AS3(sXh + base * 4), 16, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    float* zg = pl.z + (int64_t)pl.z_row0[b] * XS;
    const int nch = XS >> 2, sub = tid & 7;
    for (int r = tid >> 3; r < nrows; r += NTT / 8) {
      const int eb = strp[r] - ebase, ee = strp[r + 1] - ebase;
      for (int ch = sub; ch < nch; ch += 8) {
        const int c4 = ch * 4;
        const float4 acc = drk::gather_row_chunk(slcol, eb, ee, sXh, XS, c4);  // (the _imm form measured +0.4 us here)
        float* zr = sZ + r * LDW + c4;
        zr[0] = acc.x;
        zr[1] = acc.y;
        zr[2] = acc.z;
        zr[3] = acc.w;
        if (!ZARGS) store_z4<INL>(zg + (int64_t)(r0 + r) * XS + c4, acc);
      }
    }
  } else {
  // Z = A X for the tile's rows: 8 lanes per row, 16-byte chunks of X rows.
  {
    const int* rp = s.rowptr + n0 + g;
    const uint16_t* col = s.col + ec0;
    const float* X = s.x + n0 * (int64_t)XS;
    float* zg = pl.z + (int64_t)pl.z_row0[b] * XS;
    const int nch = XS >> 2, sub = tid & 7;
    for (int r = tid >> 3; r < nrows; r += NTT / 8) {
      const int i = r0 + r;
      const int eb = rp[i], ee = rp[i + 1];
      for (int ch = sub; ch < nch; ch += 8) {
        const int c4 = ch * 4;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        int e = eb;
        for (; e + 4 <= ee; e += 4) {
          const int j0 = col[e], j1 = col[e + 1], j2 = col[e + 2], j3 = col[e + 3];
          const float4 v0 = *reinterpret_cast<const float4*>(X + (int64_t)j0 * XS + c4);
          const float4 v1 = *reinterpret_cast<const float4*>(X + (int64_t)j1 * XS + c4);
          const float4 v2 = *reinterpret_cast<const float4*>(X + (int64_t)j2 * XS + c4);
          const float4 v3 = *reinterpret_cast<const float4*>(X + (int64_t)j3 * XS + c4);
          acc = f4add(f4add(f4add(f4add(acc, v0), v1), v2), v3);
        }
        for (; e < ee; ++e) acc = f4add(acc, *reinterpret_cast<const float4*>(X + (int64_t)col[e] * XS + c4));
        float* zr = sZ + r * LDW + c4;
        zr[0] = acc.x;
        zr[1] = acc.y;
        zr[2] = acc.z;
        zr[3] = acc.w;
        if (!ZARGS) store_z4<INL>(zg + (int64_t)i * XS + c4, acc);
      }
    }
  }
  }
  // (no s_waitcnt vmcnt(0) here: the MFMA phase reads Z from LDS, and the Z
  // stores to global memory need not land before it -- the tail reads them in
  // the next launch.  DR_TILE_STORE_WAIT = 1 restores the wait, A/B)
  if (DR_TILE_STORE_WAIT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // H = relu(Z [W1; W1e]^T), one 16-row MFMA tile per wave
  {
    const int li = lane & 15, kq = lane >> 4;
    for (int tt = wave; tt * 16 < nrows; tt += NTT / 64) {
      const int q0 = tt * 16;
      const int ar = min(q0 + li, nrows - 1);
      floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < KP; k += 16) {
        float av[4], b0[4], b1[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int kk = k + 4 * u + kq;
          av[u] = sZ[ar * LDW + kk];
          b0[u] = sW1[li * LDW + kk];
          b1[u] = sW1[(16 + li) * LDW + kk];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], b0[u], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], b1[u], acc1, 0, 0, 0);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = q0 + kq * 4 + r;
        if (row < nrows) {
          sH[row * 32 + li] = relu_keepnan(acc0[r]);
          sH[row * 32 + 16 + li] = relu_keepnan(acc1[r]);
        }
      }
    }
  }
  tile_partial_max<NTT, INL>(pl, sH, sm0i, sm0p, srng, compact, tile, b, K0, N, r0, nrows, ZARGS ? sflag : nullptr);
  if (ZARGS) {
    __syncthreads();
    float* zg = pl.z + (int64_t)pl.z_row0[b] * XS;
    const int nch = XS >> 2;
    for (int p = tid; p < nrows * nch; p += NTT) {
      const int r = p / nch, c4 = (p - r * nch) * 4;
      if (sflag[r]) {
        const float2* zr = reinterpret_cast<const float2*>(sZ + r * LDW + c4);  // (rows 8-byte aligned)
        const float2 lo = zr[0], hi = zr[1];
        *reinterpret_cast<float4*>(zg + (int64_t)(r0 + r) * XS + c4) = make_float4(lo.x, lo.y, hi.x, hi.y);
      }
    }
  }
}

__global__ void __launch_bounds__(NTA) ginet_large_conv1_kernel(LargeArgs la) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  conv_tile_f32<NTA, false>(la, lds);
}

// ---- bf16 compute (dr_pass.compute_dtype == DR_DTYPE_BF16, BASELINE configs[3]) ----
// Same tile as ginet_large_conv1_kernel with the node GEMM on bf16 operands:
// X rows come from the store's bf16 copy (half the bytes of the halo staging
// and of the gather's LDS reads), Z = A X is accumulated in fp32 and rounded
// to bf16 (its LDS operand copy and the HBM workspace the tail reads for
// dW1), W1 is rounded to bf16, and H = relu(Z W1^T) comes from
// v_mfma_f32_16x16x32_bf16 with fp32 accumulation (one MFMA per 16x16 output
// tile and 32 of K).  H, the pooling and everything after it stay fp32.

typedef short bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {  // round to nearest even (torch's .to(bfloat16))
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
__device__ __forceinline__ uint2 pack4bf(float a, float b, float c, float d) {
  return make_uint2((uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16), (uint32_t)f2bf(c) | ((uint32_t)f2bf(d) << 16));
}
__device__ __forceinline__ float4 unpack4bf(uint2 v) {
  return make_float4(__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u), __uint_as_float(v.y << 16),
                     __uint_as_float(v.y & 0xffff0000u));
}

struct ConvCarveB {  // offsets in 4-byte words; bf16 row strides in bf16 elements
  int KPB, ZSB, XSB, w1, z, h, m0i, m0p, rng, flg, xh, hid, lcol, trp, total;
};

__host__ __device__ inline ConvCarveB conv_carve_bf16(int N, int F, int K0, int HM, int EM) {
  ConvCarveB c;
  c.KPB = (F + 31) & ~31;  // K padded to whole 32-deep MFMA steps (zeros)
  c.ZSB = c.KPB + 8;       // 16-byte row shift: the 16 rows of an operand read start on distinct bank quads
  c.XSB = (F + 7) & ~7;    // the store's x_bf16_stride (16-byte rows)
  int o = 0;
  c.w1 = o;
  o += r4(32 * c.ZSB / 2);
  c.z = o;
  o += r4(TR * c.ZSB / 2);
  c.h = o;
  o += TR * 32;  // fp32 H
  c.m0i = o;
  o += r4(HM ? TR : N);
  c.m0p = o;
  o += r4(K0 + 1);
  c.rng = o;
  o += r4(2 * K0);
  c.flg = o;  // per tile row: a depth-0 pooling arg candidate (as conv_carve)
  o += r4(TR);
  c.xh = o;  // halo X rows, bf16, XSB stride
  o += HM ? r4(HM * c.XSB / 2) : 0;
  c.hid = o;
  o += r4(HM);
  c.trp = o;
  o += HM ? r4(TR + 1) : 0;
  c.lcol = o;
  o += HM ? r4((EM + 8) / 2) : 0;
  c.total = o;
  return c;
}

template <int NTT, bool INL>
__device__ __forceinline__ void conv_tile_bf16(const LargeArgs& la, float* lds) {
  const GinetArgs& a = la.g;
  const dr_large_plan& pl = la.plan;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tile = drk::xcd_tile();
  const int b = pl.tile_slot[tile];
  const int t = tile - pl.tile_first[b];
  const dr_graph_desc d = a.descs[b];
  const dr_graph_store& s = a.s;
  const int g = d.gid;
  const int64_t n0 = d.node0, ec0 = d.col0, k00 = d.k0;
  const int N = d.n_nodes, K0 = d.n_k0, F = s.n_feat;
  const int TRr = pl.tile_rows;
  const int r0 = t * TRr, nrows = min(TRr, N - r0);
  const ConvCarveB c = conv_carve_bf16(N, F, K0, pl.halo_max, 0);
  const int KPB = c.KPB, ZSB = c.ZSB, XSB = s.x_bf16_stride;
  uint16_t* sW = reinterpret_cast<uint16_t*>(lds + c.w1);
  uint16_t* sZ = reinterpret_cast<uint16_t*>(lds + c.z);
  float* sH = lds + c.h;
  int* sm0i = reinterpret_cast<int*>(lds + c.m0i);
  int* sm0p = reinterpret_cast<int*>(lds + c.m0p);
  int* srng = reinterpret_cast<int*>(lds + c.rng);
  const uint16_t* X = s.x_bf16 + n0 * (int64_t)XSB;
  uint16_t* zg = reinterpret_cast<uint16_t*>(pl.z) + (int64_t)pl.z_row0[b] * XSB;

  const bool compact = pl.tile_members != nullptr;
  if (compact) {
    drk::dma_words<NTT>(sm0i, pl.tile_members + (int64_t)tile * TRr, nrows);
    drk::dma_words<NTT>(sm0p, pl.tile_mptr + (int64_t)tile * (pl.k0_max + 1), K0 + 1);
  } else {
    drk::dma_words<NTT>(sm0i, s.m0_idx + n0, N);
    drk::dma_words<NTT>(sm0p, s.m0_ptr + k00 + g, K0 + 1);
  }
  for (int p = tid; p < 32 * KPB; p += NTT) {  // [W1; W1e] in bf16, K zero-padded to KPB
    const int r = p / KPB, k = p - r * KPB;
    float v = 0.f;
    if (k < F) v = (r < 16) ? a.w.w1[r * F + k] : a.w.w1e[(r - 16) * F + k];
    sW[r * ZSB + k] = f2bf(v);
  }
  for (int p = tid; p < TRr * (KPB - XSB); p += NTT) {  // Z pad columns (X's own pad is zero)
    const int r = p / (KPB - XSB);
    sZ[r * ZSB + XSB + (p - r * (KPB - XSB))] = 0;
  }
  constexpr bool ZARGS = DR_Z_ARGS && !INL;  // (as conv_tile_f32)
  int* sflag = reinterpret_cast<int*>(lds + c.flg);
  if (ZARGS)
    for (int p = tid; p < TRr; p += NTT) sflag[p] = 0;
  // Z = A X for the tile's rows: 8 lanes per row, 4 bf16 (8 bytes) per lane
  // and edge, summed in fp32 in CSR order; rounded to bf16 once per row.
  const int nch = XSB >> 2, sub = tid & 7;
  if (pl.halo_ids) {
    int* strp = reinterpret_cast<int*>(lds + c.trp);
    int* shid = reinterpret_cast<int*>(lds + c.hid);
    uint16_t* slcol = reinterpret_cast<uint16_t*>(lds + c.lcol);
    uint16_t* sXh = reinterpret_cast<uint16_t*>(lds + c.xh);
    const int h0 = pl.halo_off[tile], H = pl.halo_off[tile + 1] - h0;
    const int l0 = pl.lcol_off[tile];
    drk::dma_words<NTT>(strp, s.rowptr + n0 + g + r0, nrows + 1);
    drk::dma_words<NTT>(shid, pl.halo_ids + h0, H);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int ebase = strp[0];
    drk::dma_x4<NTT>(slcol, pl.lcol + l0, (strp[nrows] - ebase + 7) / 8);
    {  // halo rows: 16-byte DMA lanes, XSB/8 per row
      const int n16 = XSB >> 3, tot = H * n16;
      const int wv = __builtin_amdgcn_readfirstlane(wave);
      for (int base = wv * 64; base < tot; base += NTT)
        if (base + lane < tot) {
          const int hr = (base + lane) / n16, q = base + lane - hr * n16;
          __builtin_amdgcn_global_load_lds(DRK_AS1(X + (int64_t)shid[hr] * XSB + q * 8), DRK_AS3(sXh + base * 8), 16, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int r = tid >> 3; r < nrows; r += NTT / 8) {
      const int eb = strp[r] - ebase, ee = strp[r + 1] - ebase;
      for (int ch = sub; ch < nch; ch += 8) {
        const int c4 = ch * 4;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        int e = eb;
        for (; e + 4 <= ee; e += 4) {
          int e1 = e + 1, e2 = e + 2, e3 = e + 3;
          asm volatile("" : "+v"(e1), "+v"(e2), "+v"(e3));
          const int j0 = slcol[e], j1 = slcol[e1], j2 = slcol[e2], j3 = slcol[e3];
          const uint2 v0 = *reinterpret_cast<const uint2*>(&sXh[__umul24(j0, XSB) + c4]);
          const uint2 v1 = *reinterpret_cast<const uint2*>(&sXh[__umul24(j1, XSB) + c4]);
          const uint2 v2 = *reinterpret_cast<const uint2*>(&sXh[__umul24(j2, XSB) + c4]);
          const uint2 v3 = *reinterpret_cast<const uint2*>(&sXh[__umul24(j3, XSB) + c4]);
          acc = f4add(f4add(f4add(f4add(acc, unpack4bf(v0)), unpack4bf(v1)), unpack4bf(v2)), unpack4bf(v3));
        }
        for (; e < ee; ++e) acc = f4add(acc, unpack4bf(*reinterpret_cast<const uint2*>(&sXh[__umul24((int)slcol[e], XSB) + c4])));
        const uint2 zb = pack4bf(acc.x, acc.y, acc.z, acc.w);
        *reinterpret_cast<uint2*>(&sZ[r * ZSB + c4]) = zb;
        if (!ZARGS) store_u64<INL>(zg + (int64_t)(r0 + r) * XSB + c4, (uint64_t)zb.x | ((uint64_t)zb.y << 32));
      }
    }
  } else {
    const int* rp = s.rowptr + n0 + g;
    const uint16_t* col = s.col + ec0;
    for (int r = tid >> 3; r < nrows; r += NTT / 8) {
      const int i = r0 + r;
      const int eb = rp[i], ee = rp[i + 1];
      for (int ch = sub; ch < nch; ch += 8) {
        const int c4 = ch * 4;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        int e = eb;
        for (; e + 4 <= ee; e += 4) {
          const int j0 = col[e], j1 = col[e + 1], j2 = col[e + 2], j3 = col[e + 3];
          const uint2 v0 = *reinterpret_cast<const uint2*>(X + (int64_t)j0 * XSB + c4);
          const uint2 v1 = *reinterpret_cast<const uint2*>(X + (int64_t)j1 * XSB + c4);
          const uint2 v2 = *reinterpret_cast<const uint2*>(X + (int64_t)j2 * XSB + c4);
          const uint2 v3 = *reinterpret_cast<const uint2*>(X + (int64_t)j3 * XSB + c4);
          acc = f4add(f4add(f4add(f4add(acc, unpack4bf(v0)), unpack4bf(v1)), unpack4bf(v2)), unpack4bf(v3));
        }
        for (; e < ee; ++e) acc = f4add(acc, unpack4bf(*reinterpret_cast<const uint2*>(X + (int64_t)col[e] * XSB + c4)));
        const uint2 zb = pack4bf(acc.x, acc.y, acc.z, acc.w);
        *reinterpret_cast<uint2*>(&sZ[r * ZSB + c4]) = zb;
        if (!ZARGS) store_u64<INL>(zg + (int64_t)i * XSB + c4, (uint64_t)zb.x | ((uint64_t)zb.y << 32));
      }
    }
  }
  if (DR_TILE_STORE_WAIT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (as in conv_tile_f32)
  __syncthreads();
  // H = relu(Z [W1; W1e]^T): lane l holds Z[row l&15][k 8(l>>4)..+7] and
  // W[col l&15][same k] (16-byte LDS reads); C row (l>>4)*4+r, col l&15.
  {
    const int li = lane & 15, kq = lane >> 4;
    for (int tt = wave; tt * 16 < nrows; tt += NTT / 64) {
      const int q0 = tt * 16;
      const int ar = min(q0 + li, nrows - 1);
      floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < KPB; k += 32) {
        const bf16x8 av = *reinterpret_cast<const bf16x8*>(&sZ[ar * ZSB + k + 8 * kq]);
        const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(&sW[li * ZSB + k + 8 * kq]);
        const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(&sW[(16 + li) * ZSB + k + 8 * kq]);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b0, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b1, acc1, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = q0 + kq * 4 + r;
        if (row < nrows) {
          sH[row * 32 + li] = relu_keepnan(acc0[r]);
          sH[row * 32 + 16 + li] = relu_keepnan(acc1[r]);
        }
      }
    }
  }
  tile_partial_max<NTT, INL>(pl, sH, sm0i, sm0p, srng, compact, tile, b, K0, N, r0, nrows, ZARGS ? sflag : nullptr);
  if (ZARGS) {
    __syncthreads();
    const int nch = XSB >> 2;
    for (int p = tid; p < nrows * nch; p += NTT) {
      const int r = p / nch, c4 = (p - r * nch) * 4;
      if (sflag[r]) *reinterpret_cast<uint2*>(zg + (int64_t)(r0 + r) * XSB + c4) = *reinterpret_cast<const uint2*>(&sZ[r * ZSB + c4]);
    }
  }
}

__global__ void __launch_bounds__(NTA) ginet_large_conv1_bf16_kernel(LargeArgs la) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  conv_tile_bf16<NTA, false>(la, lds);
}

struct TailCarve {
  int w2, fc2, p1, a1, dp1, y2, h2, p1rp, p1c, p1trp, p1tc, m1p, m1i, p2, nt, cl1, head, dgp, total;
};

__host__ __device__ inline TailCarve tail_carve(int K0, int P1, int K1, int alias, int OUT) {
  TailCarve c;
  int o = 0;
#define TAKE(field, words) \
  c.field = o;             \
  o += r4(words);
  TAKE(w2, 1024)
  TAKE(fc2, OUT * 128 + OUT)
  TAKE(p1, K0 * 32)
  TAKE(a1, K0 * 32)
  TAKE(dp1, K0 * 32)
  TAKE(y2, K0 * 64)
  TAKE(h2, K0 * 64)
  TAKE(p1rp, K0 + 1)
  TAKE(p1c, P1)
  if (alias) {
    c.p1trp = c.p1rp;
    c.p1tc = c.p1c;
  } else {
    TAKE(p1trp, K0 + 1)
    TAKE(p1tc, P1)
  }
  TAKE(m1p, K1 + 1)
  TAKE(m1i, K0)
  TAKE(p2, K1 * 64)
  TAKE(nt, K1 * 64)
  TAKE(cl1, K0)  // depth-1 cluster of each depth-0 cluster
  TAKE(head, HEADW)
  TAKE(dgp, NW * 64)
#undef TAKE
  c.total = o;
  return c;
}

// One workgroup per graph: combine the tiles' partial maxima, then the tail.
// The per-graph tail of the large path: combine the tiles' partial maxima,
// then ginet_tail.  INL: run by the last-arriving tile workgroup of graph b
// inside the one-launch kernel, so the tiles' hand-off (part_key atomics, Z
// rows) is read with agent-scope (sc1) loads.
template <bool INL>
__device__ __forceinline__ void tail_body(const LargeArgs& la, int b, float* lds) {
  const GinetArgs& a = la.g;
  const dr_large_plan& pl = la.plan;
  const int tid = threadIdx.x;
  const dr_graph_store& s = a.s;
  const dr_graph_desc d = a.descs[b];
  const int g = d.gid;
  const int64_t k00 = d.k0, q0 = d.p1, k10 = d.k1;
  const int N = d.n_nodes, K0 = d.n_k0, P1 = d.n_p1, K1 = d.n_k1;
  const int F = s.n_feat, alias = s.transpose_aliased, OUT = a.p.out_dim;
  const TailCarve c = tail_carve(K0, P1, K1, alias, OUT);
  const TailLds t = tail_lds(c, lds);
  const int row = a.p.slot ? a.p.slot[b] : b;  // the graph's rows of the batch (dr_pass.slot)
  STAMP(0);

  float fc1_row[8], fc1_col[8], fc1_bias;
  {
    const int r = tid >> 3, part = tid & 7;
#pragma unroll
    for (int j = 0; j < 8; ++j) fc1_row[j] = a.w.fc1w[r * 64 + part * 8 + j];
    fc1_bias = a.w.fc1b[r];
    const int o = tid & 63, rc = tid >> 6;
#pragma unroll
    for (int j = 0; j < 8; ++j) fc1_col[j] = a.w.fc1w[(rc * 8 + j) * 64 + o];
  }
  const float y_g = s.y[g];
  uint64_t drop_offset = a.p.drop_offset;
  drk::dma_words<NT>(t.p1rp, s.p1_rowptr + k00 + g, K0 + 1);
  drk::dma_words<NT>(t.p1c, s.p1_col + q0, P1);
  if (!alias) {
    drk::dma_words<NT>(t.p1trp, s.p1t_rowptr + k00 + g, K0 + 1);
    drk::dma_words<NT>(t.p1tc, s.p1t_col + q0, P1);
  }
  drk::dma_words<NT>(t.m1p, s.m1_ptr + k10 + g, K1 + 1);
  drk::dma_words<NT>(t.m1i, s.m1_idx + k00, K0);
  t.w2[tid] = (tid < 512) ? a.w.w2[tid] : a.w.w2e[tid - 512];
  for (int p = tid; p < OUT * 129; p += NT) t.fc2[p] = (p < OUT * 128) ? a.w.fc2w[p] : a.w.fc2b[p - OUT * 128];
  STAMP(1);
  // tiles in node order, strict '>': the first maximum over the whole graph
  const int tb = pl.tile_first[b], te = pl.tile_first[b + 1];
  if (pl.part_key) {
    for (int p = tid; p < K0 * 32; p += NT) {
      unsigned long long* kp = reinterpret_cast<unsigned long long*>(pl.part_key) + (int64_t)b * pl.k0_max * 32 + p;
      unsigned long long key;
      if (INL) {
        key = __hip_atomic_load((gu64*)(kp), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store((gu64*)(kp), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        key = *kp;
        *kp = 0ull;  // ready for the next pass
      }
      t.p1[p] = key ? __uint_as_float((uint32_t)(key >> 32)) : 0.f;
      t.a1[p] = key ? (int)(0xffffffffu - (uint32_t)key) : N;
    }
  } else
  for (int p = tid; p < K0 * 32; p += NT) {
    float best = LOWEST;
    int arg = N;
    int tl = tb;
    for (; tl + 8 <= te; tl += 8) {  // 8 tiles' partials loaded together, combined in tile order
      float v[8];
      int ag[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int64_t o = ((int64_t)(tl + u) * pl.k0_max) * 32 + p;
        v[u] = pl.part_val[o];
        ag[u] = pl.part_arg[o];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (v[u] > best) {
          best = v[u];
          arg = ag[u];
        }
    }
    for (; tl < te; ++tl) {
      const int64_t o = ((int64_t)tl * pl.k0_max) * 32 + p;
      const float v = pl.part_val[o];
      if (v > best) {
        best = v;
        arg = pl.part_arg[o];
      }
    }
    t.p1[p] = (best == LOWEST) ? 0.f : best;
    t.a1[p] = arg;
  }
  if (a.p.step_counter) drop_offset = (uint64_t)a.p.step_counter[0];  // loaded late: no early wait
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // snapshot for dr_reduce_update, stored only now so that no wait for the
  // counter load sits between the descriptor and the graph DMA
  if (a.p.step_counter && b == 0 && tid == 0) a.p.step_counter[1] = (int64_t)drop_offset;
  __syncthreads();
  STAMP(2);
  STAMP(3);
  if (a.p.compute_dtype == DR_DTYPE_BF16) {  // the bf16 Z the conv1 GEMM consumed
    const int XSB = s.x_bf16_stride;
    const uint16_t* zb = reinterpret_cast<const uint16_t*>(pl.z) + (int64_t)pl.z_row0[b] * XSB;
    if (INL)
      ginet_tail(a, t, fc1_row, fc1_col, fc1_bias, row, N, K0, K1, F, OUT, y_g, drop_offset, [&](int i, int kk) {
        const int64_t o = (int64_t)i * XSB + kk;  // the 4-byte word holding the bf16 value
        const uint32_t w = load_sc1_u32(zb + (o & ~(int64_t)1));
        return __uint_as_float((o & 1) ? (w & 0xffff0000u) : (w << 16));
      }, -1);
    else
      ginet_tail(a, t, fc1_row, fc1_col, fc1_bias, row, N, K0, K1, F, OUT, y_g, drop_offset,
                 [&](int i, int kk) { return bf2f(zb[(int64_t)i * XSB + kk]); }, -1);
    return;
  }
  const float* z = pl.z + (int64_t)pl.z_row0[b] * r4(F);
  const int XS = r4(F);
  if (INL)
    ginet_tail(a, t, fc1_row, fc1_col, fc1_bias, row, N, K0, K1, F, OUT, y_g, drop_offset,
               [&](int i, int kk) { return __uint_as_float(load_sc1_u32(z + (int64_t)i * XS + kk)); }, -1);
  else
    ginet_tail(a, t, fc1_row, fc1_col, fc1_bias, row, N, K0, K1, F, OUT, y_g, drop_offset,
               [&](int i, int kk) { return z[(int64_t)i * XS + kk]; }, -1);
}

__global__ void __launch_bounds__(NT) ginet_large_tail_kernel(LargeArgs la) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  tail_body<false>(la, blockIdx.x, lds);
}

}  // namespace

extern "C" int64_t dr_ginet_lds_bytes(int32_t n_nodes, int32_t n_edges, int32_t n_feat, int32_t k0, int32_t p1_edges,
                                      int32_t k1, int32_t transpose_aliased, int32_t out_dim) {
  return 4LL * carve(n_nodes, n_edges, n_feat, k0, p1_edges, k1, transpose_aliased, out_dim).total;
}

extern "C" int dr_ginet_graph_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                                   const dr_ginet_weights* w, const dr_pass* pass, int32_t lds_bytes,
                                   void* stream) {
  if (!store || !descs || !w || !pass || n_batch < 0) return DR_E_ARG;
  if (pass->out_dim < 1 || pass->out_dim > DR_MAX_OUT) return DR_E_UNSUPPORTED;
  if (store->n_feat < 1 || 32 * store->n_feat > 2 * NT) return DR_E_UNSUPPORTED;  // F <= 64
  if (lds_bytes > 160 * 1024) return DR_E_LDS;
  if (pass->compute_dtype != DR_DTYPE_F32) return DR_E_UNSUPPORTED;  // bf16 runs dr_ginet_large_pass
  if ((pass->flags & DR_PASS_BACKWARD) && (!pass->slab || !pass->head)) return DR_E_ARG;
  if ((pass->flags & DR_PASS_BACKWARD) && pass->loss_kind == DR_LOSS_NONE && !pass->dout) return DR_E_ARG;
  if ((pass->flags & DR_PASS_FORWARD) && !pass->out) return DR_E_ARG;
  if (pass->use_dropout == DR_DROPOUT_MASK && !pass->mask) return DR_E_ARG;
  if (pass->use_dropout < DR_DROPOUT_OFF || pass->use_dropout > DR_DROPOUT_HASH) return DR_E_ARG;
  if (n_batch == 0) return DR_OK;
  if (!store->cl0) return DR_E_ARG;
  GinetArgs args;
  args.s = *store;
  args.w = *w;
  args.p = *pass;
  args.descs = descs;
  args.B = n_batch;
  if (store->n_feat <= 32) {
    DR_CHECK(dr_allow_big_lds(reinterpret_cast<const void*>(&ginet_graph_kernel<32>)));
    hipLaunchKernelGGL(ginet_graph_kernel<32>, dim3(n_batch), dim3(NT), lds_bytes, (hipStream_t)stream, args);
  } else {
    DR_CHECK(dr_allow_big_lds(reinterpret_cast<const void*>(&ginet_graph_kernel<64>)));
    hipLaunchKernelGGL(ginet_graph_kernel<64>, dim3(n_batch), dim3(NT), lds_bytes, (hipStream_t)stream, args);
  }
  return (int)hipGetLastError();
}

// Accumulating pass: n_groups workgroups, graph gi on workgroup gi % n_groups
// (or as plan lists them); each writes one row of dr_ginet_acc_row_floats
// floats to pass->slab and its loss sum to pass->loss_per_graph[w].
// max_sizes (host, optional): the batch's largest N, E, K0, P1, K1 — the
// prefetch layout when it fits, else lds_bytes (the largest graph's carve, as
// for dr_ginet_graph_pass) plus the accumulators.
extern "C" int32_t dr_ginet_acc_row_floats(int32_t n_feat, int32_t out_dim) { return acc_row_floats(n_feat, out_dim); }

extern "C" int64_t dr_ginet_acc_lds_bytes(const int32_t* max_sizes, int32_t n_feat, int32_t transpose_aliased, int32_t out_dim) {
  if (!max_sizes) return -1;
  const AccLayout L = acc_layout(max_sizes[0], max_sizes[1], n_feat, max_sizes[2], max_sizes[3], max_sizes[4],
                                 transpose_aliased, out_dim);
  return 4LL * (acc_words(n_feat, out_dim, n_feat > 32) + 4 + L.total);
}

extern "C" int dr_ginet_acc_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                                 const dr_ginet_weights* w, const dr_pass* pass, int32_t lds_bytes, int32_t n_groups,
                                 const int32_t* plan, const int32_t* max_sizes, void* stream) {
  if (!store || !descs || !w || !pass || n_batch < 0 || n_groups < 1) return DR_E_ARG;
  if (pass->out_dim < 1 || pass->out_dim > DR_MAX_OUT) return DR_E_UNSUPPORTED;
  if (store->n_feat < 1 || 32 * store->n_feat > 2 * NT) return DR_E_UNSUPPORTED;  // F <= 64
  if (pass->compute_dtype != DR_DTYPE_F32) return DR_E_UNSUPPORTED;
  // training passes only (the sums are gradients), with the fused loss
  if (!(pass->flags & DR_PASS_BACKWARD) || !pass->slab || !pass->loss_per_graph) return DR_E_ARG;
  if (pass->loss_kind == DR_LOSS_NONE || pass->slot) return DR_E_UNSUPPORTED;
  if ((pass->flags & DR_PASS_FORWARD) && !pass->out) return DR_E_ARG;
  if (pass->use_dropout == DR_DROPOUT_MASK && !pass->mask) return DR_E_ARG;
  if (pass->use_dropout < DR_DROPOUT_OFF || pass->use_dropout > DR_DROPOUT_HASH) return DR_E_ARG;
  const int F = store->n_feat, OUT = pass->out_dim;
  const int64_t lds = (int64_t)lds_bytes + 4LL * (acc_words(F, OUT, F > 32) + 4);
  AccLayout L{};
  int64_t lds_pf = -1;
  if (max_sizes) {
    L = acc_layout(max_sizes[0], max_sizes[1], F, max_sizes[2], max_sizes[3], max_sizes[4], store->transpose_aliased, OUT);
    lds_pf = dr_ginet_acc_lds_bytes(max_sizes, F, store->transpose_aliased, OUT);
  }
  const bool pf = lds_pf > 0 && lds_pf <= 160 * 1024;
  if (!pf && lds > 160 * 1024) return DR_E_LDS;
  if (n_batch == 0) return DR_OK;
  if (!store->cl0) return DR_E_ARG;
  if (n_groups > n_batch && !plan) n_groups = n_batch;
  GinetArgs args;
  args.s = *store;
  args.w = *w;
  args.p = *pass;
  args.descs = descs;
  args.B = n_batch;
  const hipStream_t st = (hipStream_t)stream;
#define DR_ACC_LAUNCH(KPT, PF, BYTES)                                                                   \
  do {                                                                                                \
    DR_CHECK(dr_allow_big_lds(reinterpret_cast<const void*>(&ginet_acc_kernel<KPT, PF>)));            \
    hipLaunchKernelGGL((ginet_acc_kernel<KPT, PF>), dim3(n_groups), dim3(NT), (int)(BYTES), st, args, plan, L); \
  } while (0)
  if (F <= 32) {
    if (pf) DR_ACC_LAUNCH(32, true, lds_pf);
    else DR_ACC_LAUNCH(32, false, lds);
  } else {
    if (pf) DR_ACC_LAUNCH(64, true, lds_pf);
    else DR_ACC_LAUNCH(64, false, lds);
  }
#undef DR_ACC_LAUNCH
  return (int)hipGetLastError();
}

extern "C" int64_t dr_ginet_large_conv_lds_bytes(int32_t n_nodes, int32_t n_feat, int32_t k0, int32_t halo_max,
                                                 int32_t tile_edges_max) {
  return 4LL * conv_carve(n_nodes, n_feat, k0, halo_max, tile_edges_max).total;
}

extern "C" int64_t dr_ginet_large_conv_lds_bytes_bf16(int32_t n_nodes, int32_t n_feat, int32_t k0, int32_t halo_max,
                                                      int32_t tile_edges_max) {
  return 4LL * conv_carve_bf16(n_nodes, n_feat, k0, halo_max, tile_edges_max).total;
}

extern "C" int64_t dr_ginet_tail_lds_bytes(int32_t k0, int32_t p1_edges, int32_t k1, int32_t transpose_aliased,
                                           int32_t out_dim) {
  return 4LL * tail_carve(k0, p1_edges, k1, transpose_aliased, out_dim).total;
}

extern "C" int dr_ginet_large_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                                   const dr_large_plan* plan, const dr_ginet_weights* w, const dr_pass* pass,
                                   int32_t conv_lds_bytes, int32_t tail_lds_bytes, void* stream) {
  if (!store || !descs || !w || !pass || !plan || n_batch < 0) return DR_E_ARG;
  if (pass->out_dim < 1 || pass->out_dim > DR_MAX_OUT) return DR_E_UNSUPPORTED;
  if (store->n_feat < 1 || store->n_feat > 64) return DR_E_UNSUPPORTED;
  if (conv_lds_bytes > 160 * 1024 || tail_lds_bytes > 160 * 1024) return DR_E_LDS;
  if (!plan->tile_first || !plan->z_row0 || !plan->tile_slot || !plan->z || !plan->part_val || !plan->part_arg)
    return DR_E_ARG;
  if (plan->n_tiles < n_batch || plan->k0_max < 1 || plan->k0_max > 64) return DR_E_ARG;
  if (plan->tile_rows < 16 || plan->tile_rows > TR || plan->tile_rows % 16) return DR_E_ARG;
  if (plan->halo_ids && (plan->halo_max < 1 || plan->halo_max > 65535 || !plan->halo_off || !plan->lcol_off ||
                         !plan->lcol || !plan->tile_members || !plan->tile_mptr))
    return DR_E_ARG;
  if (!plan->halo_ids && plan->halo_max) return DR_E_ARG;
  if (plan->arrive) return DR_E_ARG;  // (the one-launch form was removed in r06)
  if ((pass->flags & DR_PASS_BACKWARD) && (!pass->slab || !pass->head)) return DR_E_ARG;
  if ((pass->flags & DR_PASS_BACKWARD) && pass->loss_kind == DR_LOSS_NONE && !pass->dout) return DR_E_ARG;
  if ((pass->flags & DR_PASS_FORWARD) && !pass->out) return DR_E_ARG;
  if (pass->use_dropout == DR_DROPOUT_MASK && !pass->mask) return DR_E_ARG;
  if (pass->use_dropout < DR_DROPOUT_OFF || pass->use_dropout > DR_DROPOUT_HASH) return DR_E_ARG;
  const bool bf16 = pass->compute_dtype == DR_DTYPE_BF16;
  if (pass->compute_dtype != DR_DTYPE_F32 && !bf16) return DR_E_ARG;
  if (bf16 && (!store->x_bf16 || store->x_bf16_stride < store->n_feat || store->x_bf16_stride % 8)) return DR_E_ARG;
  if (n_batch == 0) return DR_OK;
  DR_CHECK(dr_allow_big_lds(reinterpret_cast<const void*>(&ginet_large_conv1_kernel)));
  DR_CHECK(dr_allow_big_lds(reinterpret_cast<const void*>(&ginet_large_conv1_bf16_kernel)));
  DR_CHECK(dr_allow_big_lds(reinterpret_cast<const void*>(&ginet_large_tail_kernel)));
  LargeArgs la;
  la.g.s = *store;
  la.g.w = *w;
  la.g.p = *pass;
  la.g.descs = descs;
  la.g.B = n_batch;
  la.plan = *plan;
  hipStream_t st = (hipStream_t)stream;
  if (bf16)
    hipLaunchKernelGGL(ginet_large_conv1_bf16_kernel, dim3(plan->n_tiles), dim3(NTA), conv_lds_bytes, st, la);
  else
    hipLaunchKernelGGL(ginet_large_conv1_kernel, dim3(plan->n_tiles), dim3(NTA), conv_lds_bytes, st, la);
  hipLaunchKernelGGL(ginet_large_tail_kernel, dim3(n_batch), dim3(NT), tail_lds_bytes, st, la);
  return (int)hipGetLastError();
}

extern "C" int dr_dropout_mask(uint64_t seed, uint64_t offset, int32_t n, float p, uint8_t* keep_host) {
  if (n < 0 || (n > 0 && !keep_host)) return DR_E_ARG;
  for (int i = 0; i < n; ++i) keep_host[i] = dr_uniform(seed, offset, (uint32_t)i) >= p ? 1 : 0;
  return DR_OK;
}

// ---- carve descriptions for the host-side carve tests (tests/test_lds_carves.py)
extern "C" int dr_debug_carve_ginet(const int32_t* q, char* buf, int32_t len) {
  const Carve c = carve(q[0], q[1], q[2], q[3], q[4], q[5], q[6], q[7]);
  DrCarveDesc d{buf, len, 0};
  DR_DESC_P(d, c, KP);
  DR_DESC_P(d, c, LDW);
  DR_DESC_P(d, c, XS);
  DR_DESC(d, c, w1);
  DR_DESC(d, c, w2);
  DR_DESC(d, c, fc2);
  DR_DESC(d, c, x);
  DR_DESC(d, c, z);
  DR_DESC(d, c, rp);
  DR_DESC(d, c, col);
  DR_DESC(d, c, cl0);
  DR_DESC(d, c, key);
  DR_DESC(d, c, p1);
  DR_DESC(d, c, a1);
  DR_DESC(d, c, dp1);
  DR_DESC(d, c, y2);
  DR_DESC(d, c, h2);
  DR_DESC(d, c, p1rp);
  DR_DESC(d, c, p1c);
  DR_DESC(d, c, p1trp);
  DR_DESC(d, c, p1tc);
  DR_DESC(d, c, m1p);
  DR_DESC(d, c, m1i);
  DR_DESC(d, c, p2);
  DR_DESC(d, c, nt);
  DR_DESC(d, c, cl1);
  DR_DESC(d, c, head);
  DR_DESC(d, c, dgp);
  DR_DESC(d, c, keep);
  DR_DESC(d, c, total);
  return d.pos;
}

extern "C" int dr_debug_xcd_tile(int32_t n_blocks, int32_t* tiles) {
  if (n_blocks < 0 || (n_blocks > 0 && !tiles)) return DR_E_ARG;
  for (int b = 0; b < n_blocks; ++b) tiles[b] = drk::xcd_tile_of(b, n_blocks);
  return DR_OK;
}

extern "C" int dr_debug_carve_ginet_conv(const int32_t* q, char* buf, int32_t len) {
  const ConvCarve c = conv_carve(q[0], q[1], q[2], q[3], q[4]);
  DrCarveDesc d{buf, len, 0};
  DR_DESC_P(d, c, KP);
  DR_DESC_P(d, c, LDW);
  DR_DESC_P(d, c, XS);
  DR_DESC(d, c, w1);
  DR_DESC(d, c, z);
  DR_DESC(d, c, h);
  DR_DESC(d, c, m0i);
  DR_DESC(d, c, m0p);
  DR_DESC(d, c, rng);
  DR_DESC(d, c, flg);
  DR_DESC(d, c, xh);
  DR_DESC(d, c, hid);
  DR_DESC(d, c, lcol);
  DR_DESC(d, c, trp);
  DR_DESC(d, c, total);
  return d.pos;
}

extern "C" int dr_debug_carve_ginet_conv_bf16(const int32_t* q, char* buf, int32_t len) {
  const ConvCarveB c = conv_carve_bf16(q[0], q[1], q[2], q[3], q[4]);
  DrCarveDesc d{buf, len, 0};
  DR_DESC_P(d, c, KPB);
  DR_DESC_P(d, c, ZSB);
  DR_DESC_P(d, c, XSB);
  DR_DESC(d, c, w1);
  DR_DESC(d, c, z);
  DR_DESC(d, c, h);
  DR_DESC(d, c, m0i);
  DR_DESC(d, c, m0p);
  DR_DESC(d, c, rng);
  DR_DESC(d, c, flg);
  DR_DESC(d, c, xh);
  DR_DESC(d, c, hid);
  DR_DESC(d, c, lcol);
  DR_DESC(d, c, trp);
  DR_DESC(d, c, total);
  return d.pos;
}

extern "C" int dr_debug_carve_ginet_tail(const int32_t* q, char* buf, int32_t len) {
  const TailCarve c = tail_carve(q[0], q[1], q[2], q[3], q[4]);
  DrCarveDesc d{buf, len, 0};
  DR_DESC(d, c, w2);
  DR_DESC(d, c, fc2);
  DR_DESC(d, c, p1);
  DR_DESC(d, c, a1);
  DR_DESC(d, c, dp1);
  DR_DESC(d, c, y2);
  DR_DESC(d, c, h2);
  DR_DESC(d, c, p1rp);
  DR_DESC(d, c, p1c);
  DR_DESC(d, c, p1trp);
  DR_DESC(d, c, p1tc);
  DR_DESC(d, c, m1p);
  DR_DESC(d, c, m1i);
  DR_DESC(d, c, p2);
  DR_DESC(d, c, nt);
  DR_DESC(d, c, cl1);
  DR_DESC(d, c, head);
  DR_DESC(d, c, dgp);
  DR_DESC(d, c, total);
  return d.pos;
}

