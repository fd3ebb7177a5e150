// Gradient reduction over the batch + Adam for one block of parameter
// elements (the stand-alone reduce kernel, reduce_adam.hip).
//
// Replaces loss_.backward()'s accumulation over the batch and
// optimizer.step() of Trainer._epoch (deeprank2/trainer.py:689-690; Adam
// configured at trainer.py:419).  Every gradient element is a sum over the
// per-graph partials in a fixed order — RC chunks of consecutive batch rows,
// each summed in row order from zero, then the chunks in order — so the
// result is deterministic (no float atomics) and the same whichever block
// form below computes it.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>

#include "../../include/deeprank2_amd.h"
#include "dr_common.h"

namespace drr {

constexpr int RP = 64;  // parameter elements per block (row-partial blocks)
constexpr int RC = 8;   // batch chunks per element
constexpr int RU = 8;   // batch rows per chunk issued together (predicated)
constexpr int RU2 = 24; // then the rest of a chunk, this many at a time
constexpr int RT = RP * RC;  // threads per block
// Outer-product blocks (DR_GRAD_OUTER, e.g. fc1.weight = sum_b dh_b g_b^T)
// stage the head slices they read in LDS first (reduce_outer_block): at B =
// 64 GINet's fc1.weight took 1 M dword loads from 128 blocks (16 K
// wave-level loads, 128 per CU: the reduce's critical path, ~1.5 us of
// address processing, tools/step_timeline.py).  Up to this many LDS floats:
constexpr int OUTER_LDS_FLOATS = 12288;
constexpr uint8_t BLK_OUTER = 0x80;  // blk_param flag: the block is an outer-product block

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
  int16_t blk0[DR_MAX_PARAMS + 1];  // first block of each parameter, blk0[n_params] = n_blocks
  int32_t slab_rows;  // slab rows per graph (>= 1): a slab-kind gradient sums B * slab_rows rows
  float* mirror;            // dr_adam.mirror / mirror_idx: packed copies of updated elements
  const int4* mirror_idx;
  uint32_t* fault_clear;    // dr_adam.fault_clear / ticket
  uint32_t* ticket;
};

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

// The loss: loss_out[0] = loss_scale * sum(loss_per_graph) (lane-strided
// partial sums, then a fixed-order wave reduction), by the first 64 threads
// of block 0; NaN after a faulted pass.
__device__ __forceinline__ void reduce_loss(const ReduceHdr& h, bool first, int t, bool bad) {
  if (first && t < 64 && h.lpg && h.loss_out) {
    float acc = 0.f;
    for (int b = t; b < h.B; b += 64) acc += h.lpg[b];
    acc = dr_wave_sum(acc);
    if (t == 0) h.loss_out[0] = bad ? __builtin_nanf("") : acc * h.loss_scale;
  } else if (bad && first && t == 0 && h.loss_out) {
    h.loss_out[0] = __builtin_nanf("");
  }
}

// Element e's Adam state (and its dr_adam.mirror slots), loaded up front so
// the loads leave ahead of the partials'
struct ElemState {
  float p0 = 0.f, m0 = 0.f, v0 = 0.f;
  int4 mi = make_int4(-1, -1, -1, -1);
};
__device__ __forceinline__ ElemState load_state(const ReduceHdr& h, const ParamRec& r, int ec, bool want) {
  ElemState s;
  if (want && h.adam_enabled && r.numel > 0) {  // numel 0: an empty record (no pointers)
    s.p0 = r.param[ec];
    s.m0 = r.m[ec];
    s.v0 = r.v[ec];
    if (h.mirror) s.mi = h.mirror_idx[r.mbase + ec];
  }
  return s;
}

// Element e with its gradient gsum (from the partials): the gradient store,
// then torch.optim.Adam's update
__device__ __forceinline__ void adam_element(const ReduceHdr& h, const ParamRec& r, int e, float gsum, const ElemState& s,
                                             bool upd, bool counter_lane, int64_t tstep) {
  if (!upd) return;
  float bc1 = h.bias_c1, bc2s = h.bias_c2_sqrt;
  if (h.step_counter) {  // step and bias corrections from the device counter
    bc1 = 1.f - exp2f((float)tstep * h.log2_beta1);
    bc2s = sqrtf(1.f - exp2f((float)tstep * h.log2_beta2));
    if (counter_lane) h.step_counter[0] = tstep;
  }
  float gr = gsum;
  if (h.weight_decay != 0.f) gr = fmaf(h.weight_decay, s.p0, gr);
  // torch.optim.Adam: exp_avg.lerp_(g, 1-b1); exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
  // every product-sum spelled out (fmaf / __fmul_rn / __fadd_rn): contraction
  // is then the same in every block form that inlines this
  const float mv = fmaf(1.f - h.beta1, __fsub_rn(gr, s.m0), s.m0);
  const float vv = fmaf(__fmul_rn(1.f - h.beta2, gr), gr, __fmul_rn(s.v0, h.beta2));
  r.m[e] = mv;
  r.v[e] = vv;
  const float denom = __fadd_rn(__fdiv_rn(sqrtf(vv), bc2s), h.eps);
  const float pn = fmaf(-(h.lr / bc1), __fdiv_rn(mv, denom), s.p0);
  r.param[e] = pn;
  if (h.mirror) {
    if (s.mi.x >= 0) h.mirror[s.mi.x] = pn;
    if (s.mi.y >= 0) h.mirror[s.mi.y] = pn;
    if (s.mi.z >= 0) h.mirror[s.mi.z] = pn;
    if (s.mi.w >= 0) h.mirror[s.mi.w] = pn;
  }
}

// dr_adam.fault_clear: one lane of each block takes a ticket once its read of
// the flag has returned; the last block's lane clears the flag (every block
// has read it by then) for the next graph pass
__device__ __forceinline__ uint32_t take_ticket(const ReduceHdr& h, bool lane, uint32_t fv) {
  if (!(lane && h.fault_clear)) return 0u;
  asm volatile("" ::"v"(fv) : "memory");
  return __hip_atomic_fetch_add(h.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void last_ticket(const ReduceHdr& h, bool lane, uint32_t tk) {
  if (lane && h.fault_clear && tk == (uint32_t)h.n_blocks - 1u) {
    *h.fault_clear = 0u;
    *h.ticket = 0u;
  }
}

// One block = RP consecutive elements (from elem_block * RP) of parameter r,
// RC batch chunks per element; t = thread index within the block's RT
// threads, part = the block's [RC][RP] LDS scratch.  first: the block that
// also sums the loss and advances the step counter.  tstep: the Adam step
// (counter[1] + 1) when h.step_counter is set.  Every load of the block is
// issued in one straight-line group (clamped indices, zero weights past the
// batch), the Adam state first, so one wait covers them.
__device__ __forceinline__ void reduce_block(const ReduceHdr& h, const ParamRec& r, int elem_block, bool first, int t,
                                             float (*part)[RP], int64_t tstep) {
  const int lp = t % RP, ch = t / RP;
  const int e = elem_block * RP + lp;
  const bool live = e < r.numel;
  // a graph pass whose in-launch hand-off gave up (dr_pass.fault): its
  // partials are wrong, so the step reports NaN and changes no state
  const uint32_t fv = h.fault ? *h.fault : 0u;
  const bool bad = fv != 0u;
  const int ec = live ? e : 0;
  const ElemState s = load_state(h, r, ec, ch == 0);
  float gin = 0.f, div = 1.f;
  if (ch == 0 && !h.slab && r.grad) {
    gin = r.grad[ec];
    if (h.grad_div) div = *h.grad_div;
  }
  reduce_loss(h, first, t, bad);
  const bool slab_kind = r.kind == DR_GRAD_SLAB, outer = r.kind == DR_GRAD_OUTER;
  const bool has_src = h.slab && (slab_kind || outer || r.kind == DR_GRAD_HEAD);
  const int64_t st = slab_kind ? h.slab_stride : h.head_stride;
  const float* base = slab_kind ? h.slab : h.head;
  const int col1 = outer ? r.off1 + ec / r.cols : r.off1 + ec;
  const int col2 = outer ? r.off2 + ec % r.cols : 0;
  const int nb = slab_kind ? h.B * h.slab_rows : h.B;  // rows of this gradient's partials
  const int b0 = (nb * ch) / RC, b1 = (nb * (ch + 1)) / RC;
  float u[RU], w[RU];
  if (has_src && b0 < b1) {
#pragma unroll
    for (int k = 0; k < RU; ++k) {
      const int64_t row = min(b0 + k, b1 - 1);
      u[k] = base[row * st + col1];
      w[k] = outer ? base[row * st + col2] : 1.f;
    }
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
          u2[k] = base[row * st + col1];
          w2[k] = outer ? base[row * st + col2] : 1.f;
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
  const uint32_t tk = take_ticket(h, lp == 0, fv);
  float gsum;
  if (h.slab) {
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
  adam_element(h, r, e, gsum, s, h.adam_enabled && !bad, first && lp == 0, tstep);
  last_ticket(h, lp == 0, tk);
  RDSTAMP(3);
#ifdef DR_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  RDSTAMP(4);
}

// One outer-product block: RP consecutive elements from e0 of a
// DR_GRAD_OUTER parameter (grad[i][j] = sum_b head[b][off1 + i] head[b][off2 + j]),
// RC batch chunks per element as in reduce_block.  The block first stages the
// head slices its elements read — U = head[:, off1 + rows of the block]
// ([rows][B]) and W = head[:, off2 + columns of the block] ([B][cols]),
// 16-byte loads where aligned — in LDS (sm) with a few loads per thread,
// instead of every thread loading 2 x B/RC scattered partials: the same
// products, sums and order as reduce_block, so the same bits.  Needs partials
// (h.slab set) and B * (columns + rows) <= OUTER_LDS_FLOATS - RC * RP.
__device__ __forceinline__ void reduce_outer_block(const ReduceHdr& h, const ParamRec& r, int e0, bool first, int t,
                                                   float* sm, int64_t tstep) {
  const int lp = t % RP, ch = t / RP;
  const int cols = r.cols, e = e0 + lp;
  const int elast = min(e0 + RP, r.numel) - 1;
  const bool live = e < r.numel;
  const uint32_t fv = h.fault ? *h.fault : 0u;
  const bool bad = fv != 0u;
  const ElemState s = load_state(h, r, live ? e : e0, ch == 0 && live);
  reduce_loss(h, first, t, bad);
  const int ir0 = e0 / cols, ir1 = elast / cols;  // the block's rows
  const int jlo = ir0 == ir1 ? e0 - ir0 * cols : 0, jn = ir0 == ir1 ? elast - e0 + 1 : cols;  // its columns
  const int nr = ir1 - ir0 + 1, nb = h.B;
  const int64_t st = h.head_stride;
  float* part = sm;                  // [RC][RP]
  float* sU = sm + RC * RP;          // [nr][nb]
  float* sW = sU + nr * nb;          // [nb][jn]
  const float* wsrc = h.head + r.off2 + jlo;
  if (((r.off2 + jlo) & 3) == 0 && (jn & 3) == 0 && (st & 3) == 0) {
    const int q = jn >> 2;
    for (int p = t; p < nb * q; p += RT) {
      const int b = p / q, c4 = p - b * q;
      *reinterpret_cast<float4*>(sW + b * jn + 4 * c4) = *reinterpret_cast<const float4*>(wsrc + b * st + 4 * c4);
    }
  } else {
    for (int p = t; p < nb * jn; p += RT) {
      const int b = p / jn, jj = p - b * jn;
      sW[p] = wsrc[b * st + jj];
    }
  }
  for (int p = t; p < nr * nb; p += RT) {
    const int ii = p / nb, b = p - ii * nb;
    sU[p] = h.head[b * st + r.off1 + ir0 + ii];
  }
  __syncthreads();
  {
    const int ec = live ? e : e0;
    const int ii = ec / cols - ir0, jj = ec % cols - jlo;
    const int b0 = (nb * ch) / RC, b1 = (nb * (ch + 1)) / RC;
    float acc = 0.f;
    for (int b = b0; b < b1; ++b) acc = fmaf(sU[ii * nb + b], sW[b * jn + jj], acc);
    part[ch * RP + lp] = acc;
  }
  RDSTAMP(1);
  __syncthreads();
  RDSTAMP(2);
  if (ch != 0 || !live) return;
  const uint32_t tk = take_ticket(h, lp == 0, fv);
  float gsum = 0.f;
#pragma unroll
  for (int k = 0; k < RC; ++k) gsum += part[k * RP + lp];
  if (bad) gsum = __builtin_nanf("");
  if (r.grad) r.grad[e] = gsum;
  adam_element(h, r, e, gsum, s, h.adam_enabled && !bad, first && lp == 0, tstep);
  last_ticket(h, lp == 0, tk);
  RDSTAMP(3);
#ifdef DR_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  RDSTAMP(4);
}

// Host: whether parameter i of the table reduces in outer-product blocks
inline bool outer_blocks(const dr_param_table* t, int i, const float* slab, int32_t n_batch) {
  const dr_grad_recipe r = t->recipe[i];
  if (r.kind != DR_GRAD_OUTER || !slab || r.cols <= 0) return false;
  // the widest block: RP columns of one row, or every column of RP / cols + 2 rows
  const int64_t cols = r.cols >= RP ? RP : r.cols, rows = r.cols >= RP ? 2 : RP / r.cols + 2;
  return (int64_t)n_batch * (cols + rows) <= OUTER_LDS_FLOATS - RC * RP;
}

// Host: header + records from the C-ABI table and Adam settings; the block
// list goes to blk_param / blk_elem (each block's parameter, BLK_OUTER for an
// outer-product block, and its first element); returns the number of blocks,
// or a negative DR_E_* code.
inline int build_reduce(const dr_param_table* t, const float* slab, const float* head, int32_t n_batch,
                        const dr_adam* adam, const float* loss_per_graph, float loss_scale, float* loss_out,
                        ReduceHdr& h, ParamRec* rec, uint8_t* blk_param, uint16_t* blk_elem, int max_blocks) {
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
    if (t->numel[i] < 0 || t->numel[i] > 65535 || !t->param[i]) return t->numel[i] > 65535 ? DR_E_UNSUPPORTED : DR_E_ARG;
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
    const bool ob = outer_blocks(t, i, slab, n_batch);
    for (int e0 = 0; e0 < t->numel[i]; e0 += RP, ++blocks) {
      if (blocks >= max_blocks) return DR_E_UNSUPPORTED;
      blk_param[blocks] = (uint8_t)(i | (ob ? BLK_OUTER : 0));
      blk_elem[blocks] = (uint16_t)e0;
    }
  }
  for (int i = t->n_params; i <= DR_MAX_PARAMS; ++i) h.blk0[i] = (int16_t)blocks;
  h.n_params = t->n_params;
  h.n_blocks = blocks;
  if (t->slab_rows < 0 || t->slab_rows > 64) return DR_E_ARG;
  h.slab_rows = t->slab_rows > 0 ? t->slab_rows : 1;
  return blocks;
}

}  // namespace drr
