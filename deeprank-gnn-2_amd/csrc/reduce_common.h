// Gradient reduction over the batch + Adam for one block of parameter
// elements (the stand-alone reduce kernel, reduce_adam.hip; the r03-r05
// one-launch GINet steps that also ran it are gone).  r06 measured and did
// not keep blocks that stage their partials in LDS first (outer products and
// row sums): 3.9 vs 3.5 us per launch, the load -> LDS -> barrier -> sum
// chain is longer than the direct loads (profiles/r06/not_kept/).
//
// Replaces loss_.backward()'s accumulation over the batch and
// optimizer.step() of Trainer._epoch (deeprank2/trainer.py:689-690; Adam
// configured at trainer.py:419).
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>

#include "../../include/deeprank2_amd.h"
#include "dr_common.h"

namespace drr {

#ifndef DR_RP
#define DR_RP 64
#endif
#ifndef DR_RC
#define DR_RC 8
#endif
constexpr int RP = DR_RP;  // parameter elements per block
constexpr int RC = DR_RC;  // batch chunks per block
constexpr int RU = 8;   // batch rows per chunk issued together (predicated)
constexpr int RU2 = 24; // then the rest of a chunk, this many at a time
constexpr int RT = RP * RC;  // threads per block

// One 64-byte kernel-argument line per parameter: a block fetches everything
// it needs about its parameter with one scalar load.
struct alignas(64) ParamRec {
  float* param;
  float* grad;
  float* m;
  float* v;
  int32_t numel, kind, off1, off2;
  int32_t cols, mbase, pad1, pad2;  // mbase: flat index of element 0 (dr_adam.mirror_idx)
};

struct alignas(64) ReduceHdr {
  const float* slab;
  const float* head;
  const float* lpg;
  float* loss_out;
  int64_t* step_counter;
  const float* grad_div;
  const uint32_t* fault;  // dr_adam.fault: nonzero -> NaN loss / gradients, no update
  int32_t B, slab_stride, head_stride, adam_enabled;
  float loss_scale, pad0;
  float lr, beta1, beta2, eps, weight_decay, bias_c1, bias_c2_sqrt, pad1;
  float log2_beta1, log2_beta2;  // beta^t = exp2(t log2 beta): one v_exp_f32, not powf
  int32_t n_params, n_blocks;
  int16_t blk0[DR_MAX_PARAMS + 1];  // first block of each parameter (prefix sums of ceil(numel / RP)), blk0[n_params] = n_blocks
  int32_t slab_rows;  // slab rows per graph (>= 1): a slab-kind gradient sums B * slab_rows rows
  float* mirror;            // dr_adam.mirror / mirror_idx: packed copies of updated elements
  const int4* mirror_idx;
  uint32_t* fault_clear;    // dr_adam.fault_clear / ticket (stand-alone reduce kernel only)
  uint32_t* ticket;
};

typedef __attribute__((address_space(1))) unsigned int gu32r;

// Diagnostic timeline (stamps build only, dr_debug_reduce_stamps): thread 0
// of block j writes s_memrealtime (100 MHz chip clock) at point i to
// g_reduce_stamps[j * 8 + i]: 0 entry, 5 kernel-argument record in, 1 its
// partials summed, 2 past the barrier, 3 stores issued, 4 stores done.
#ifdef DR_STAMPS
__device__ int64_t g_reduce_stamps[4096 * 8];
#define RDSTAMP(i)                                                                                      \
  do {                                                                                                  \
    __builtin_amdgcn_sched_barrier(0);                                                                  \
    if (threadIdx.x == 0) drr::g_reduce_stamps[(int64_t)blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                                  \
  } while (0)
#else
#define RDSTAMP(i) \
  do {             \
  } while (0)
#endif

// LD: how the partials are read.  0: plain loads (written by an earlier
// launch).  1: agent-scope relaxed atomic loads (sc1: past this CU's L1) and
// 2: system-scope ones, for partials published inside the same launch by
// write-through stores of other workgroups (MI355X_MICROARCH.md
// §inter-workgroup visibility).
template <int LD>
__device__ __forceinline__ float ld_part(const float* p) {
  if (LD == 1) return __uint_as_float(__hip_atomic_load((const gu32r*)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  if (LD == 2) return __uint_as_float(__hip_atomic_load((const gu32r*)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  return *p;
}

// One block = RP consecutive elements (from elem_block * RP) of parameter r,
// RC batch chunks per element; t = thread index within the block's RT
// threads, part = the block's [RC][RP] LDS scratch.  first: the block that
// also sums the loss and advances the step counter.  tstep: the Adam step
// (counter[1] + 1) when h.step_counter is set.  Every load of the block is
// issued in one straight-line group (clamped indices, zero weights past the
// batch), so one wait covers the partials and the Adam state.  The caller
// synchronises the workgroup between two calls that share `part`.
// WTP: the updated parameters are stored write-through (agent scope), for a
// launch whose other workgroups read them after a grid-wide hand-off (the
// reduce-at-start GINet step, ginet_fused.hip).
// row_off: the partials of graph b sit at row row_off + b (slab: (row_off + b)
// * slab_rows): the half of the pipelined step's double buffer.
template <int LD, bool LEAN = false, bool WTP = false>
__device__ __forceinline__ void reduce_block(const ReduceHdr& h, const ParamRec& r, int elem_block, bool first, int t,
                                             float (*part)[RP], int64_t tstep, int64_t row_off = 0) {
  // LEAN: partials always given, Adam always on (the one-launch step): the
  // gradients-supplied path is compiled out (less code to fetch cold)
  const int lp = t % RP, ch = t / RP;
  const int e = elem_block * RP + lp;
  const bool live = e < r.numel;
  // a graph pass whose in-launch hand-off gave up (dr_pass.fault): its
  // partials are wrong, so the step reports NaN and changes no state
  const uint32_t fv = (!LEAN && h.fault) ? *h.fault : 0u;
  const bool bad = fv != 0u;
  if (first && t < 64 && h.lpg && h.loss_out) {
    float acc = 0.f;  // lane-strided partial sums, then a fixed-order wave reduction
    for (int b = t; b < h.B; b += 64) acc += ld_part<LD>(h.lpg + row_off + b);
    acc = dr_wave_sum(acc);
    if (t == 0) h.loss_out[0] = bad ? __builtin_nanf("") : acc * h.loss_scale;
  } else if (bad && first && t == 0 && h.loss_out) {
    h.loss_out[0] = __builtin_nanf("");
  }
  const int ec = live ? e : 0;
  const bool slab_kind = r.kind == DR_GRAD_SLAB, outer = r.kind == DR_GRAD_OUTER;
  const bool has_src = h.slab && (slab_kind || outer || r.kind == DR_GRAD_HEAD);
  const int64_t st = slab_kind ? h.slab_stride : h.head_stride;
  const float* base = (slab_kind ? h.slab : h.head) + row_off * (slab_kind ? h.slab_rows : 1) * st;
  const int col1 = outer ? r.off1 + ec / r.cols : r.off1 + ec;
  const int col2 = outer ? r.off2 + ec % r.cols : 0;
  const int nb = slab_kind ? h.B * h.slab_rows : h.B;  // rows of this gradient's partials
  const int b0 = (nb * ch) / RC, b1 = (nb * (ch + 1)) / RC;
  float u[RU], w[RU];
  if (has_src && b0 < b1) {
#pragma unroll
    for (int k = 0; k < RU; ++k) {
      const int64_t row = min(b0 + k, b1 - 1);
      u[k] = ld_part<LD>(base + row * st + col1);
      w[k] = outer ? ld_part<LD>(base + row * st + col2) : 1.f;
    }
  }
  const bool upd = live && ch == 0 && (LEAN || h.adam_enabled) && !bad;
  float p0 = 0.f, m0 = 0.f, v0 = 0.f, gin = 0.f;
  int4 mi = make_int4(-1, -1, -1, -1);  // dr_adam.mirror slots of this element, loaded with the state
  if (ch == 0 && (LEAN || h.adam_enabled) && r.numel > 0) {  // numel 0: an empty record (no pointers)
    p0 = r.param[ec];
    m0 = r.m[ec];
    v0 = r.v[ec];
    if (!LEAN && h.mirror) mi = h.mirror_idx[r.mbase + ec];
  }
  float div = 1.f;
  if (!LEAN && ch == 0 && !h.slab && r.grad) {
    gin = r.grad[ec];
    if (h.grad_div) div = *h.grad_div;
  }
  if (h.slab) {
    float acc = 0.f;
    if (has_src && b0 < b1) {
#pragma unroll
      for (int k = 0; k < RU; ++k)
        if (b0 + k < b1) acc = outer ? fmaf(u[k], w[k], acc) : acc + u[k];
      // more than RU rows per chunk (e.g. split partial rows): the rest, RU2
      // rows' loads in flight at a time (same rows, same order)
      for (int bb = b0 + RU; bb < b1; bb += RU2) {
        float u2[RU2], w2[RU2];
#pragma unroll
        for (int k = 0; k < RU2; ++k) {
          const int64_t row = min(bb + k, b1 - 1);
          u2[k] = ld_part<LD>(base + row * st + col1);
          w2[k] = outer ? ld_part<LD>(base + row * st + col2) : 1.f;
        }
#pragma unroll
        for (int k = 0; k < RU2; ++k)
          if (bb + k < b1) acc = outer ? fmaf(u2[k], w2[k], acc) : acc + u2[k];
      }
    }
    part[ch][lp] = acc;
  }
  RDSTAMP(1);
  __syncthreads();
  RDSTAMP(2);
  if (ch != 0 || !live) return;
  // dr_adam.fault_clear: lane 0 of each block takes a ticket once its read of
  // the flag has returned; the last block's lane 0 clears the flag (every
  // block has read it by then) for the next graph pass
  const bool tick = !LEAN && h.fault_clear && lp == 0;
  uint32_t tk = 0u;
  if (tick) {
    asm volatile("" ::"v"(fv) : "memory");
    tk = __hip_atomic_fetch_add(h.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  float gsum;
  if (LEAN || h.slab) {
    gsum = 0.f;
#pragma unroll
    for (int k = 0; k < RC; ++k) gsum += part[k][lp];
    if (bad) gsum = __builtin_nanf("");
    if (r.grad) r.grad[e] = gsum;
  } else {  // gradients supplied (e.g. after an RCCL all-reduce): Adam only
    gsum = gin;
    if (h.grad_div) {
      gsum = gin / div;
      r.grad[e] = gsum;
      if (first && lp == 0 && h.loss_out) h.loss_out[0] = h.loss_out[0] / div;
    }
    if (bad) r.grad[e] = __builtin_nanf("");
  }
  if (upd) {
    float bc1 = h.bias_c1, bc2s = h.bias_c2_sqrt;
    if (h.step_counter) {  // step and bias corrections from the device counter
      bc1 = 1.f - exp2f((float)tstep * h.log2_beta1);
      bc2s = sqrtf(1.f - exp2f((float)tstep * h.log2_beta2));
      if (!LEAN && first && lp == 0) h.step_counter[0] = tstep;  // LEAN: the caller advances it
    }
    float gr = gsum;
    if (h.weight_decay != 0.f) gr = fmaf(h.weight_decay, p0, gr);
    // torch.optim.Adam: exp_avg.lerp_(g, 1-b1); exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
    // every product-sum spelled out (fmaf / __fmul_rn / __fadd_rn): contraction
    // is then the same in every kernel that inlines this block
    const float mv = fmaf(1.f - h.beta1, __fsub_rn(gr, m0), m0);
    const float vv = fmaf(__fmul_rn(1.f - h.beta2, gr), gr, __fmul_rn(v0, h.beta2));
    r.m[e] = mv;
    r.v[e] = vv;
    const float denom = __fadd_rn(__fdiv_rn(sqrtf(vv), bc2s), h.eps);
    const float pn = fmaf(-(h.lr / bc1), __fdiv_rn(mv, denom), p0);
    if (WTP) __hip_atomic_store((__attribute__((address_space(1))) unsigned int*)(r.param + e), __float_as_uint(pn), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else r.param[e] = pn;
    if (!LEAN && h.mirror) {
      if (mi.x >= 0) h.mirror[mi.x] = pn;
      if (mi.y >= 0) h.mirror[mi.y] = pn;
      if (mi.z >= 0) h.mirror[mi.z] = pn;
      if (mi.w >= 0) h.mirror[mi.w] = pn;
    }
  }
  if (tick && tk == (uint32_t)h.n_blocks - 1u) {
    *h.fault_clear = 0u;
    *h.ticket = 0u;
  }
  RDSTAMP(3);
#ifdef DR_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  RDSTAMP(4);
}

// Host: header + records from the C-ABI table and Adam settings; returns the
// number of RP-element blocks, or a negative DR_E_* code.
inline int build_reduce(const dr_param_table* t, const float* slab, const float* head, int32_t n_batch,
                        const dr_adam* adam, const float* loss_per_graph, float loss_scale, float* loss_out,
                        ReduceHdr& h, ParamRec* rec) {
  if (!t || !adam || n_batch < 0) return DR_E_ARG;
  if ((slab == nullptr) != (head == nullptr)) return DR_E_ARG;
  if (t->n_params < 1 || t->n_params > DR_MAX_PARAMS) return DR_E_ARG;
  std::memset(&h, 0, sizeof(h));
  h.slab = slab;
  h.head = head;
  h.lpg = loss_per_graph;
  h.loss_out = loss_out;
  h.step_counter = adam->step_counter;
  h.grad_div = adam->grad_div;
  h.fault = adam->fault;
  h.B = n_batch;
  h.slab_stride = t->slab_stride;
  h.head_stride = t->head_stride;
  h.adam_enabled = adam->enabled;
  h.loss_scale = loss_scale;
  h.lr = adam->lr;
  h.beta1 = adam->beta1;
  h.beta2 = adam->beta2;
  h.eps = adam->eps;
  h.weight_decay = adam->weight_decay;
  h.bias_c1 = adam->bias_c1;
  h.bias_c2_sqrt = adam->bias_c2_sqrt;
  h.log2_beta1 = (float)std::log2((double)adam->beta1);
  h.log2_beta2 = (float)std::log2((double)adam->beta2);
  if ((adam->mirror == nullptr) != (adam->mirror_idx == nullptr)) return DR_E_ARG;
  if (adam->mirror_idx && (reinterpret_cast<uintptr_t>(adam->mirror_idx) & 15)) return DR_E_ARG;
  if (adam->fault_clear && !adam->ticket) return DR_E_ARG;
  h.mirror = adam->mirror;
  h.mirror_idx = reinterpret_cast<const int4*>(adam->mirror_idx);
  h.fault_clear = adam->fault_clear;
  h.ticket = adam->ticket;
  int blocks = 0, mbase = 0;
  for (int i = 0; i < t->n_params; ++i) {
    if (t->numel[i] < 0 || !t->param[i]) return DR_E_ARG;
    if (adam->enabled && (!t->exp_avg[i] || !t->exp_avg_sq[i])) return DR_E_ARG;
    if (!slab && !t->grad[i]) return DR_E_ARG;
    const dr_grad_recipe r = t->recipe[i];
    if (r.kind < DR_GRAD_ZERO || r.kind > DR_GRAD_HEAD || (r.kind == DR_GRAD_OUTER && r.cols <= 0)) return DR_E_ARG;
    ParamRec& pr = rec[i];
    std::memset(&pr, 0, sizeof(pr));
    pr.param = t->param[i];
    pr.grad = t->grad[i];
    pr.m = t->exp_avg[i];
    pr.v = t->exp_avg_sq[i];
    pr.numel = t->numel[i];
    pr.kind = r.kind;
    pr.off1 = r.off1;
    pr.off2 = r.off2;
    pr.cols = r.cols;
    pr.mbase = mbase;
    mbase += t->numel[i];
    h.blk0[i] = (int16_t)blocks;
    blocks += (t->numel[i] + RP - 1) / RP;
  }
  if (blocks > 32767) return DR_E_UNSUPPORTED;
  for (int i = t->n_params; i <= DR_MAX_PARAMS; ++i) h.blk0[i] = (int16_t)blocks;
  h.n_params = t->n_params;
  h.n_blocks = blocks;
  if (t->slab_rows < 0 || t->slab_rows > 64) return DR_E_ARG;
  h.slab_rows = t->slab_rows > 0 ? t->slab_rows : 1;
  return blocks;
}

}  // namespace drr
