// Gradient reduction over the batch + Adam, shared by every fused model.
//
// Replaces loss_.backward()'s accumulation over the batch and
// optimizer.step() of Trainer._epoch (deeprank2/trainer.py:689-690; Adam
// configured at trainer.py:419).  Each parameter element's gradient is a sum
// over the per-graph partials the graph pass wrote (slab rows, or outer
// products of per-graph head vectors), taken in a fixed order: deterministic,
// no float atomics.  HBM-bound on the partials (~0.6 MB per GINet step at B=64).
// The per-block arithmetic lives in reduce_common.h.

#include <hip/hip_runtime.h>

#include "reduce_common.h"

namespace {

using drr::RP;
using drr::RT;
#define DR_REDUCE_MAX_BLOCKS 512  // 32 K parameter elements (GINet at F=64: ~11.5 K)

struct alignas(64) ReduceArgs {
  drr::ReduceHdr h;
  drr::ParamRec rec[DR_MAX_PARAMS];
  // 1-D grid: block -> (parameter, first element); blocks never straddle two parameters
  uint8_t blk_param[DR_REDUCE_MAX_BLOCKS];
  uint16_t blk_elem[DR_REDUCE_MAX_BLOCKS];  // first element / RP
};

// 1-D grid over sum_p ceil(numel_p / RP) blocks: block j reduces RP
// consecutive elements of parameter blk_param[j].  Its record and the header
// are scalar loads from the kernel arguments.
__global__ void __launch_bounds__(RT) reduce_adam_kernel(ReduceArgs a) {
  __shared__ float part[drr::RC][RP];
  RDSTAMP(0);
  const int pi = a.blk_param[blockIdx.x];
  const drr::ParamRec r = a.rec[pi];
  // Pull every kernel-argument line this block uses in one scalar round trip
  // (hipcc would otherwise issue them lazily, one wait each).
  {
    const float *slab = a.h.slab, *head = a.h.head;
    const int32_t B = a.h.B, ss = a.h.slab_stride, hs = a.h.head_stride, en = a.h.adam_enabled;
    asm volatile("" ::"s"(slab), "s"(head), "s"(B), "s"(ss), "s"(hs), "s"(en), "s"(r.param), "s"(r.grad), "s"(r.m),
                 "s"(r.v), "s"(r.numel), "s"(r.kind), "s"(r.off1), "s"(r.off2), "s"(r.cols));
  }
  RDSTAMP(5);  // (stamps build: the block's kernel-argument record is in)
  const int64_t tstep = (a.h.step_counter && a.h.adam_enabled) ? a.h.step_counter[1] + 1 : 0;
  drr::reduce_block<0>(a.h, r, a.blk_elem[blockIdx.x], blockIdx.x == 0, threadIdx.x, part, tstep);
}

}  // namespace

extern "C" int dr_reduce_update(const dr_param_table* t, const float* slab, const float* head, int32_t n_batch,
                                const dr_adam* adam, const float* loss_per_graph, float loss_scale, float* loss_out,
                                void* stream) {
  ReduceArgs a;
  std::memset(&a, 0, sizeof(a));
  const int blocks = drr::build_reduce(t, slab, head, n_batch, adam, loss_per_graph, loss_scale, loss_out, a.h, a.rec);
  if (blocks < 0) return blocks;
  if (blocks > DR_REDUCE_MAX_BLOCKS) return DR_E_UNSUPPORTED;
  int j = 0;
  for (int i = 0; i < t->n_params; ++i)
    for (int x = 0; x * RP < t->numel[i]; ++x, ++j) {
      a.blk_param[j] = (uint8_t)i;
      a.blk_elem[j] = (uint16_t)x;
    }
  if (blocks == 0) return DR_OK;
  hipLaunchKernelGGL(reduce_adam_kernel, dim3(blocks), dim3(RT), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

#ifdef DR_STAMPS
// stamps build only: the reduce kernel's timeline stamps (drr::g_reduce_stamps)
extern "C" int dr_debug_reduce_stamps(int64_t* host, int32_t n) {
  if (!host || n < 0 || n > 4096 * 8) return DR_E_ARG;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(drr::g_reduce_stamps), (size_t)n * sizeof(int64_t), 0, hipMemcpyDeviceToHost);
}
#endif
