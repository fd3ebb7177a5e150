// Gradient reduction over the batch + Adam, shared by every fused model.
//
// Replaces loss_.backward()'s accumulation over the batch and
// optimizer.step() of Trainer._epoch (deeprank2/trainer.py:689-690; Adam
// configured at trainer.py:419).  Each parameter element's gradient is a sum
// over the per-graph partials the graph pass wrote (slab rows, or outer
// products of per-graph head vectors), taken in a fixed order: deterministic,
// no float atomics.  HBM-bound on the partials (~0.6 MB per GINet step at B=64).

#include <hip/hip_runtime.h>

#include <cstring>

#include "../../include/deeprank2_amd.h"
#include "dr_common.h"

namespace {

constexpr int RP = 64;  // parameter elements per block
constexpr int RC = 8;   // batch chunks per block
constexpr int RU = 8;   // batch rows per chunk issued together (predicated)

struct ReduceArgs {
  dr_param_table t;
  dr_adam adam;
  const float* slab;
  const float* head;
  const float* lpg;
  float* loss_out;
  float loss_scale;
  int32_t B;
  int32_t off[DR_MAX_PARAMS + 1];
};

struct GradSrc {
  const float* p1;
  const float* p2;
  int64_t st;
};

__device__ __forceinline__ GradSrc grad_src(const ReduceArgs& a, int pi, int e) {
  const dr_grad_recipe r = a.t.recipe[pi];
  switch (r.kind) {
    case DR_GRAD_SLAB:
      return {a.slab + r.off1 + e, nullptr, a.t.slab_stride};
    case DR_GRAD_OUTER:
      return {a.head + r.off1 + e / r.cols, a.head + r.off2 + e % r.cols, a.t.head_stride};
    case DR_GRAD_HEAD:
      return {a.head + r.off1 + e, nullptr, a.t.head_stride};
    default:
      return {nullptr, nullptr, 0};
  }
}

__global__ void __launch_bounds__(RP* RC) reduce_adam_kernel(ReduceArgs a) {
  __shared__ float part[RC][RP];
  const int lp = threadIdx.x % RP, ch = threadIdx.x / RP;
  const int gi = blockIdx.x * RP + lp;
  if (blockIdx.x == 0 && threadIdx.x < 64 && a.lpg && a.loss_out) {
    float acc = 0.f;  // lane-strided partial sums, then a fixed-order wave reduction
    for (int b = threadIdx.x; b < a.B; b += 64) acc += a.lpg[b];
    acc = dr_wave_sum(acc);
    if (threadIdx.x == 0) a.loss_out[0] = acc * a.loss_scale;
  }
  const int np = a.t.n_params;
  const bool live = gi < a.off[np];
  int pi = 0;
  if (live)
    while (gi >= a.off[pi + 1]) ++pi;
  const int e = live ? gi - a.off[pi] : 0;
  // Adam state loads are issued together with the partial-sum loads: one
  // memory round trip per element instead of two.
  const bool upd = live && ch == 0 && a.adam.enabled;
  float p0 = 0.f, m0 = 0.f, v0 = 0.f, gin = 0.f;
  if (upd) {
    p0 = a.t.param[pi][e];
    m0 = a.t.exp_avg[pi][e];
    v0 = a.t.exp_avg_sq[pi][e];
  }
  if (live && ch == 0 && !a.slab && a.t.grad[pi]) gin = a.t.grad[pi][e];
  if (a.slab) {
    float acc = 0.f;
    const GradSrc src = live ? grad_src(a, pi, e) : GradSrc{nullptr, nullptr, 0};
    if (src.p1) {
      const int b0 = (a.B * ch) / RC, b1 = (a.B * (ch + 1)) / RC;
      const float* q1 = src.p1 + (int64_t)b0 * src.st;
      const float* q2 = src.p2 ? src.p2 + (int64_t)b0 * src.st : nullptr;
      for (int bb = b0; bb < b1; bb += RU) {
        float u[RU], v[RU];
#pragma unroll
        for (int k = 0; k < RU; ++k) {
          const bool ok = bb + k < b1;
          u[k] = ok ? q1[k * src.st] : 0.f;
          v[k] = (ok && q2) ? q2[k * src.st] : 1.f;
        }
#pragma unroll
        for (int k = 0; k < RU; ++k) acc = q2 ? fmaf(u[k], v[k], acc) : acc + u[k];
        q1 += RU * src.st;
        if (q2) q2 += RU * src.st;
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
    if (a.t.grad[pi]) a.t.grad[pi][e] = gsum;
  } else {  // gradients supplied (e.g. after an RCCL all-reduce): Adam only
    gsum = gin;
  }
  if (upd) {
    float bc1 = a.adam.bias_c1, bc2s = a.adam.bias_c2_sqrt;
    if (a.adam.step_counter) {  // step and bias corrections from the device counter
      const int64_t t = a.adam.step_counter[1] + 1;
      bc1 = 1.f - powf(a.adam.beta1, (float)t);
      bc2s = sqrtf(1.f - powf(a.adam.beta2, (float)t));
      if (gi == 0) a.adam.step_counter[0] = t;
    }
    float gr = gsum;
    if (a.adam.weight_decay != 0.f) gr = fmaf(a.adam.weight_decay, p0, gr);
    // torch.optim.Adam: exp_avg.lerp_(g, 1-b1); exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
    const float mv = m0 + (1.f - a.adam.beta1) * (gr - m0);
    const float vv = fmaf((1.f - a.adam.beta2) * gr, gr, v0 * a.adam.beta2);
    a.t.exp_avg[pi][e] = mv;
    a.t.exp_avg_sq[pi][e] = vv;
    const float denom = sqrtf(vv) / bc2s + a.adam.eps;
    a.t.param[pi][e] = p0 - (a.adam.lr / bc1) * (mv / denom);
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
  a.t = *t;
  a.adam = *adam;
  a.slab = slab;
  a.head = head;
  a.lpg = loss_per_graph;
  a.loss_out = loss_out;
  a.loss_scale = loss_scale;
  a.B = n_batch;
  a.off[0] = 0;
  for (int i = 0; i < t->n_params; ++i) {
    if (t->numel[i] < 0 || !t->param[i]) return DR_E_ARG;
    if (adam->enabled && (!t->exp_avg[i] || !t->exp_avg_sq[i])) return DR_E_ARG;
    if (!slab && !t->grad[i]) return DR_E_ARG;
    const dr_grad_recipe r = t->recipe[i];
    if (r.kind < DR_GRAD_ZERO || r.kind > DR_GRAD_HEAD || (r.kind == DR_GRAD_OUTER && r.cols <= 0)) return DR_E_ARG;
    a.off[i + 1] = a.off[i] + t->numel[i];
  }
  const int total = a.off[t->n_params];
  if (total == 0) return DR_OK;
  hipLaunchKernelGGL(reduce_adam_kernel, dim3((total + RP - 1) / RP), dim3(RP * RC), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}
