// Gradient reduction over the batch + Adam, shared by every fused model.
//
// Replaces loss_.backward()'s accumulation over the batch and
// optimizer.step() of Trainer._epoch (deeprank2/trainer.py:689-690; Adam
// configured at trainer.py:419).  Each parameter element's gradient is a sum
// over the per-graph partials the graph pass wrote (slab rows, or outer
// products of per-graph head vectors), taken in a fixed order: deterministic,
// no float atomics.  HBM-bound on the partials (~0.6 MB per GINet step at B=64).

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>

#include "../../include/deeprank2_amd.h"
#include "dr_common.h"

namespace {

constexpr int RP = 64;  // parameter elements per block
constexpr int RC = 8;   // batch chunks per block
constexpr int RU = 8;   // batch rows per chunk issued together (predicated)
#define DR_REDUCE_MAX_BLOCKS 512  // 32 K parameter elements (GINet at F=64: ~11.5 K)

// One 64-byte kernel-argument line per parameter: a block (blockIdx.y = the
// parameter) fetches everything it needs about its parameter with one scalar
// load that does not depend on any other load.
struct alignas(64) ParamRec {
  float* param;
  float* grad;
  float* m;
  float* v;
  int32_t numel, kind, off1, off2;
  int32_t cols, pad0, pad1, pad2;
};

struct alignas(64) ReduceArgs {
  const float* slab;
  const float* head;
  const float* lpg;
  float* loss_out;
  int64_t* step_counter;
  const float* grad_div;
  int32_t B, slab_stride, head_stride, adam_enabled;
  float loss_scale, pad0;
  float lr, beta1, beta2, eps, weight_decay, bias_c1, bias_c2_sqrt, pad1;
  float log2_beta1, log2_beta2;  // beta^t = exp2(t log2 beta): one v_exp_f32, not powf
  int32_t pad2[12];
  ParamRec rec[DR_MAX_PARAMS];
  // 1-D grid: block -> (parameter, first element); blocks never straddle two parameters
  uint8_t blk_param[DR_REDUCE_MAX_BLOCKS];
  uint16_t blk_elem[DR_REDUCE_MAX_BLOCKS];  // first element / RP
};

// 1-D grid over sum_p ceil(numel_p / RP) blocks: block j reduces RP
// consecutive elements of parameter blk_param[j].  Its record and the header
// are scalar loads from the kernel arguments; the partials, the Adam state
// and the step counter are fetched in one vector round trip.
__global__ void __launch_bounds__(RP* RC) reduce_adam_kernel(ReduceArgs a) {
  __shared__ float part[RC][RP];
  const int pi = a.blk_param[blockIdx.x];
  const ParamRec r = a.rec[pi];
  // Pull every kernel-argument line this block uses in one scalar round trip
  // (hipcc would otherwise issue them lazily, one wait each).
  {
    const float *slab = a.slab, *head = a.head;
    const int32_t B = a.B, ss = a.slab_stride, hs = a.head_stride, en = a.adam_enabled;
    asm volatile("" ::"s"(slab), "s"(head), "s"(B), "s"(ss), "s"(hs), "s"(en), "s"(r.param), "s"(r.grad), "s"(r.m),
                 "s"(r.v), "s"(r.numel), "s"(r.kind), "s"(r.off1), "s"(r.off2), "s"(r.cols));
  }
  const int lp = threadIdx.x % RP, ch = threadIdx.x / RP;
  const int e = a.blk_elem[blockIdx.x] * RP + lp;
  const bool live = e < r.numel;
  const bool first = blockIdx.x == 0;
  if (first && threadIdx.x < 64 && a.lpg && a.loss_out) {
    float acc = 0.f;  // lane-strided partial sums, then a fixed-order wave reduction
    for (int b = threadIdx.x; b < a.B; b += 64) acc += a.lpg[b];
    acc = dr_wave_sum(acc);
    if (threadIdx.x == 0) a.loss_out[0] = acc * a.loss_scale;
  }
  // Every load of the block is issued in one straight-line group (no
  // branches, clamped indices, zero weights for rows past the batch), so a
  // single wait covers the partials, the Adam state and the step counter.
  const int ec = live ? e : 0;
  const bool slab_kind = r.kind == DR_GRAD_SLAB, outer = r.kind == DR_GRAD_OUTER;
  const bool has_src = a.slab && (slab_kind || outer || r.kind == DR_GRAD_HEAD);
  const float* base = slab_kind ? a.slab : a.head;
  const int64_t st = slab_kind ? a.slab_stride : a.head_stride;
  const int col1 = outer ? r.off1 + ec / r.cols : r.off1 + ec;
  const int col2 = outer ? r.off2 + ec % r.cols : 0;
  const int b0 = (a.B * ch) / RC, b1 = (a.B * (ch + 1)) / RC;
  float u[RU], w[RU];
  if (has_src && b0 < b1) {
#pragma unroll
    for (int k = 0; k < RU; ++k) {
      const int64_t row = min(b0 + k, b1 - 1);
      u[k] = base[row * st + col1];
      w[k] = outer ? base[row * st + col2] : 1.f;
    }
  }
  const bool upd = live && ch == 0 && a.adam_enabled;
  float p0 = 0.f, m0 = 0.f, v0 = 0.f, gin = 0.f;
  int64_t tstep = 0;
  if (ch == 0 && a.adam_enabled) {
    p0 = r.param[ec];
    m0 = r.m[ec];
    v0 = r.v[ec];
    if (a.step_counter) tstep = a.step_counter[1] + 1;
  }
  float div = 1.f;
  if (ch == 0 && !a.slab && r.grad) {
    gin = r.grad[ec];
    if (a.grad_div) div = *a.grad_div;
  }
  if (a.slab) {
    float acc = 0.f;
    if (has_src && b0 < b1) {
#pragma unroll
      for (int k = 0; k < RU; ++k)
        if (b0 + k < b1) acc = outer ? fmaf(u[k], w[k], acc) : acc + u[k];
      // batches larger than RC*RU rows per block: the rest, RU rows at a time
      for (int bb = b0 + RU; bb < b1; bb += RU) {
#pragma unroll
        for (int k = 0; k < RU; ++k) {
          const int64_t row = min(bb + k, b1 - 1);
          u[k] = base[row * st + col1];
          w[k] = outer ? base[row * st + col2] : 1.f;
        }
#pragma unroll
        for (int k = 0; k < RU; ++k)
          if (bb + k < b1) acc = outer ? fmaf(u[k], w[k], acc) : acc + u[k];
      }
    }
    part[ch][lp] = acc;
  }
  __syncthreads();
  if (ch != 0 || !live) return;
  float gsum;
  if (a.slab) {
    gsum = 0.f;
#pragma unroll
    for (int k = 0; k < RC; ++k) gsum += part[k][lp];
    if (r.grad) r.grad[e] = gsum;
  } else {  // gradients supplied (e.g. after an RCCL all-reduce): Adam only
    gsum = gin;
    if (a.grad_div) {
      gsum = gin / div;
      r.grad[e] = gsum;
      if (first && lp == 0 && a.loss_out) a.loss_out[0] = a.loss_out[0] / div;
    }
  }
  if (upd) {
    float bc1 = a.bias_c1, bc2s = a.bias_c2_sqrt;
    if (a.step_counter) {  // step and bias corrections from the device counter
      bc1 = 1.f - exp2f((float)tstep * a.log2_beta1);
      bc2s = sqrtf(1.f - exp2f((float)tstep * a.log2_beta2));
      if (first && lp == 0) a.step_counter[0] = tstep;
    }
    float gr = gsum;
    if (a.weight_decay != 0.f) gr = fmaf(a.weight_decay, p0, gr);
    // torch.optim.Adam: exp_avg.lerp_(g, 1-b1); exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
    const float mv = m0 + (1.f - a.beta1) * (gr - m0);
    const float vv = fmaf((1.f - a.beta2) * gr, gr, v0 * a.beta2);
    r.m[e] = mv;
    r.v[e] = vv;
    const float denom = sqrtf(vv) / bc2s + a.eps;
    r.param[e] = p0 - (a.lr / bc1) * (mv / denom);
  }
}

}  // namespace

extern "C" int dr_reduce_update(const dr_param_table* t, const float* slab, const float* head, int32_t n_batch,
                                const dr_adam* adam, const float* loss_per_graph, float loss_scale, float* loss_out,
                                void* stream) {
  if (!t || !adam || n_batch < 0) return DR_E_ARG;
  if ((slab == nullptr) != (head == nullptr)) return DR_E_ARG;
  if (t->n_params < 1 || t->n_params > DR_MAX_PARAMS) return DR_E_ARG;
  ReduceArgs a;
  std::memset(&a, 0, sizeof(a));
  a.slab = slab;
  a.head = head;
  a.lpg = loss_per_graph;
  a.loss_out = loss_out;
  a.step_counter = adam->step_counter;
  a.grad_div = adam->grad_div;
  a.B = n_batch;
  a.slab_stride = t->slab_stride;
  a.head_stride = t->head_stride;
  a.adam_enabled = adam->enabled;
  a.loss_scale = loss_scale;
  a.lr = adam->lr;
  a.beta1 = adam->beta1;
  a.beta2 = adam->beta2;
  a.eps = adam->eps;
  a.weight_decay = adam->weight_decay;
  a.bias_c1 = adam->bias_c1;
  a.bias_c2_sqrt = adam->bias_c2_sqrt;
  a.log2_beta1 = (float)std::log2((double)adam->beta1);
  a.log2_beta2 = (float)std::log2((double)adam->beta2);
  int blocks = 0;
  for (int i = 0; i < t->n_params; ++i) {
    if (t->numel[i] < 0 || !t->param[i]) return DR_E_ARG;
    if (adam->enabled && (!t->exp_avg[i] || !t->exp_avg_sq[i])) return DR_E_ARG;
    if (!slab && !t->grad[i]) return DR_E_ARG;
    const dr_grad_recipe r = t->recipe[i];
    if (r.kind < DR_GRAD_ZERO || r.kind > DR_GRAD_HEAD || (r.kind == DR_GRAD_OUTER && r.cols <= 0)) return DR_E_ARG;
    ParamRec& pr = a.rec[i];
    pr.param = t->param[i];
    pr.grad = t->grad[i];
    pr.m = t->exp_avg[i];
    pr.v = t->exp_avg_sq[i];
    pr.numel = t->numel[i];
    pr.kind = r.kind;
    pr.off1 = r.off1;
    pr.off2 = r.off2;
    pr.cols = r.cols;
    for (int x = 0; x * RP < t->numel[i]; ++x) {
      if (blocks == DR_REDUCE_MAX_BLOCKS) return DR_E_UNSUPPORTED;
      a.blk_param[blocks] = (uint8_t)i;
      a.blk_elem[blocks] = (uint16_t)x;
      ++blocks;
    }
  }
  if (blocks == 0) return DR_OK;
  hipLaunchKernelGGL(reduce_adam_kernel, dim3(blocks), dim3(RP * RC), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}
