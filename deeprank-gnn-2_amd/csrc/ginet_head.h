// The GINet head shared by the GINet kernels (ginet.py:117-123 and
// ginet_nocluster.py:103-109): fc1 -> relu -> dropout -> fc2, the loss
// gradient of Trainer._epoch (trainer.py:686-689) and the head backward down
// to dG, with the per-graph head vectors (g, hd, dh, dout) for
// dr_reduce_update.  Expects g [64] in LDS; returns false after a
// forward-only pass.
#pragma once

#include "graph_common.h"

namespace drk {

__device__ __forceinline__ bool keep_unit(const dr_pass& p, uint64_t offset, int b, int r) {
  if (p.use_dropout == DR_DROPOUT_MASK) return p.mask[(int64_t)b * 128 + r] != 0;
  return dr_uniform(p.drop_seed, offset, (uint32_t)(b * 128 + r)) >= p.drop_p;
}

struct GinetHeadLds {
  float *fc2, *g, *hpre, *hh, *hd, *dh, *dg, *dout, *dgp;
  const uint8_t* keep = nullptr;  // optional [128] dropout keep flags computed ahead (head_keep_prefetch)
  // accumulating pass (dr_ginet_acc_pass): the workgroup's running sums of the
  // head gradients over its graphs, [fc1.bias 128 | fc2.weight OUT x 128 |
  // fc2.bias OUT | loss 1 | pad to 16 B | fc1.weight 128 x 64 unless accf],
  // instead of per-graph head vectors (16-byte aligned)
  float* acc = nullptr;
  float* accf = nullptr;  // or: fc1.weight's sums of this thread (row tid/8, columns 8 (tid%8) ..) in registers
  // the caller sums dG from the 16 per-wave partials (dgp) itself, in the
  // same order, where it first needs it: no dG step and no closing barrier
  bool dg_deferred = false;
};

// The fc1-output dropout keep flags of graph b, written to LDS by the first
// 128 threads while the graph is still being staged: the counter hash (or the
// mask read) leaves the head's critical path.
__device__ __forceinline__ void head_keep_prefetch(const dr_pass& p, uint64_t offset, int b, uint8_t* keep) {
  const int r = threadIdx.x;
  if (r < 128 && p.use_dropout) keep[r] = keep_unit(p, offset, b, r) ? 1 : 0;
}

// Diagnostic stamps (stamps build only): s_memtime at two points inside the head.
__device__ __forceinline__ void head_stamp(int64_t* row, int i) {
#ifdef DR_STAMPS
  __builtin_amdgcn_sched_barrier(0);
  if (threadIdx.x == 0 && row) row[i] = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
#else
  (void)row;
  (void)i;
#endif
}

// Per-graph partial stores: plain, or write-through (sc1: agent-scope relaxed
// atomic stores) when other workgroups of the same launch read them
// (dr_ginet_train_step's in-launch reduction; MI355X_MICROARCH.md
// §inter-workgroup visibility).
template <bool WT>
__device__ __forceinline__ void st_part(float* p, float v) {
  if (WT)
    __hip_atomic_store((__attribute__((address_space(1))) unsigned int*)(p), __float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = v;
}

template <int NT, bool WT = false, bool ACC = false>
__device__ __forceinline__ bool ginet_head(const dr_pass& p, const GinetHeadLds& t, const float (&fc1_row)[8],
                                           const float (&fc1_col)[8], float fc1_bias, int b, int OUT, float y_g,
                                           uint64_t drop_offset, int stamp0 = -1, int pb = -1) {
  // pb: the row of the per-graph partials (loss term, head vectors) when it
  // differs from the output row b (dr_ginet_piped_step's double buffer)
  if (pb < 0) pb = b;
  int64_t* srow = (stamp0 >= 0 && p.stamps) ? p.stamps + (int64_t)b * 32 : nullptr;
  constexpr int NW = NT / 64;
  const int tid = dr_tid<ACC>();
  const int lane = tid & 63;
  const int wave = dr_wave<ACC>(tid);
  // ---------------- head: fc1 -> relu -> dropout -> fc2 (ginet.py:120-123) --
  {
    const int r = tid >> 3, part = tid & 7;  // 8 lanes per fc1 row
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = fmaf(t.g[part * 8 + j], fc1_row[j], acc);
    acc = dr_sum8(acc);  // the xor-1,2,4 butterfly sums, on the DPP path
    if (part == 0) {
      acc += fc1_bias;
      t.hpre[r] = acc;
      const float hh = relu_keepnan(acc);
      t.hh[r] = hh;
      float hd = hh;
      if (p.use_dropout) hd = ((t.keep ? t.keep[r] != 0 : keep_unit(p, drop_offset, b, r)) ? hh : 0.f) * p.drop_scale;
      t.hd[r] = hd;
    }
  }
  __syncthreads();
  if (OUT == 1 && p.loss_kind == DR_LOSS_MSE && (p.flags & DR_PASS_BACKWARD)) {
    // one MSE logit (the headline): waves 0 and 1 each form the logit (the
    // same sums), the loss gradient and their 64 rows of dh, so the logit,
    // loss and dh steps need no workgroup barrier between them
    if (tid < 128) {
      float v = fmaf(t.hd[lane], t.fc2[lane], t.hd[lane + 64] * t.fc2[lane + 64]);
      v = dr_wave_sum_dpp(v);
      const float logit = v + t.fc2[128];
      const float d = logit - y_g;
      const float dout0 = 2.f * d * p.loss_scale;
      if (tid == 0) {
        if (p.flags & DR_PASS_FORWARD) p.out[b] = logit;
        if (ACC) t.acc[128 + 128 + 1] += d * d;
        else if (p.loss_per_graph) st_part<WT>(p.loss_per_graph + pb, d * d);
        t.dout[0] = dout0;
      }
      head_stamp(srow, stamp0);
      head_stamp(srow, stamp0 + 1);
      float acc = fmaf(t.fc2[tid], dout0, 0.f);
      if (p.use_dropout) acc = ((t.keep ? t.keep[tid] != 0 : keep_unit(p, drop_offset, b, tid)) ? acc : 0.f) * p.drop_scale;
      t.dh[tid] = relu_bwd(t.hh[tid], acc);
    }
  } else {
    for (int q = wave; q < OUT; q += NW) {
      const float* wr = t.fc2 + q * 128;
      float v = fmaf(t.hd[lane], wr[lane], t.hd[lane + 64] * wr[lane + 64]);
      v = dr_wave_sum_dpp(v);
      if (lane == 0) t.dout[q] = v + t.fc2[OUT * 128 + q];  // logits parked in t.dout
    }
    __syncthreads();
    if ((p.flags & DR_PASS_FORWARD) && tid < OUT) p.out[(int64_t)b * OUT + tid] = t.dout[tid];
    if (!(p.flags & DR_PASS_BACKWARD)) return false;
    // (the loss below is taken by thread 0, which read its logits above in
    // program order; the other logits' readers are lanes of the same wave 0
    // while OUT <= 64: no barrier needed between the output stores and the loss)
    if (OUT > 64) __syncthreads();
    head_stamp(srow, stamp0);

    // ---------------- loss gradient (trainer.py:688-689) ----------------------
    if (tid == 0) {
      if (p.loss_kind == DR_LOSS_MSE) {
        const float d = t.dout[0] - y_g;
        if (ACC) t.acc[128 + 128 * OUT + OUT] += d * d;
        else if (p.loss_per_graph) st_part<WT>(p.loss_per_graph + pb, d * d);
        t.dout[0] = 2.f * d * p.loss_scale;
        for (int q = 1; q < OUT; ++q) t.dout[q] = 0.f;  // the loss reads column 0 only (engine's layer path alike)
      } else if (p.loss_kind == DR_LOSS_CE) {
        const int yi = (int)y_g;
        float mx = t.dout[0];
        for (int q = 1; q < OUT; ++q) mx = fmaxf(mx, t.dout[q]);
        float se = 0.f;
        for (int q = 0; q < OUT; ++q) se += expf(t.dout[q] - mx);
        const float lse = mx + logf(se);
        const float wy = p.class_w ? p.class_w[yi] : 1.f;
        if (ACC) t.acc[128 + 128 * OUT + OUT] += wy * (lse - t.dout[yi]);
        else if (p.loss_per_graph) st_part<WT>(p.loss_per_graph + pb, wy * (lse - t.dout[yi]));
        for (int q = 0; q < OUT; ++q) t.dout[q] = wy * (expf(t.dout[q] - lse) - (q == yi ? 1.f : 0.f)) * p.loss_scale;
      } else {
        for (int q = 0; q < OUT; ++q) t.dout[q] = p.dout[(int64_t)b * OUT + q];
      }
    }
    __syncthreads();

    head_stamp(srow, stamp0 + 1);
    // ---------------- head backward -------------------------------------------
    if (tid < 128) {
      float acc = 0.f;
      for (int q = 0; q < OUT; ++q) acc = fmaf(t.fc2[q * 128 + tid], t.dout[q], acc);
      if (p.use_dropout) acc = ((t.keep ? t.keep[tid] != 0 : keep_unit(p, drop_offset, b, tid)) ? acc : 0.f) * p.drop_scale;
      t.dh[tid] = relu_bwd(t.hh[tid], acc);
    }
  }
  __syncthreads();
  {
    const int o = tid & 63, rc = dr_wave<ACC>(tid);  // 16 chunks of 8 fc1 rows
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = fmaf(fc1_col[j], t.dh[rc * 8 + j], acc);
    t.dgp[rc * 64 + o] = acc;
  }
  __syncthreads();
  if (!t.dg_deferred && tid < 64) {
    float acc = 0.f;
    for (int rc = 0; rc < NW; ++rc) acc += t.dgp[rc * 64 + tid];
    t.dg[tid] = acc;
  }
  if (ACC) {
    // this graph's head gradients added to the workgroup's sums: fc1.weight
    // += dh (x) g (thread (r, part): row r, columns 8 part ..), fc1.bias +=
    // dh, fc2.weight += dout (x) hd, fc2.bias += dout
    const int r = tid >> 3, part = tid & 7;
    const float dhr = t.dh[r];
    const float4* gv = reinterpret_cast<const float4*>(t.g + part * 8);
    const float4 x0 = gv[0], x1 = gv[1];
    if (t.accf) {  // in the caller's registers
      float* f = t.accf;
      f[0] = fmaf(dhr, x0.x, f[0]); f[1] = fmaf(dhr, x0.y, f[1]); f[2] = fmaf(dhr, x0.z, f[2]); f[3] = fmaf(dhr, x0.w, f[3]);
      f[4] = fmaf(dhr, x1.x, f[4]); f[5] = fmaf(dhr, x1.y, f[5]); f[6] = fmaf(dhr, x1.z, f[6]); f[7] = fmaf(dhr, x1.w, f[7]);
    } else {  // in LDS (the row's fc1.weight block)
      float4* w = reinterpret_cast<float4*>(t.acc + ((128 + 128 * OUT + OUT + 1 + 3) & ~3) + r * 64 + part * 8);
      float4 v0 = w[0], v1 = w[1];
      v0.x = fmaf(dhr, x0.x, v0.x); v0.y = fmaf(dhr, x0.y, v0.y); v0.z = fmaf(dhr, x0.z, v0.z); v0.w = fmaf(dhr, x0.w, v0.w);
      v1.x = fmaf(dhr, x1.x, v1.x); v1.y = fmaf(dhr, x1.y, v1.y); v1.z = fmaf(dhr, x1.z, v1.z); v1.w = fmaf(dhr, x1.w, v1.w);
      w[0] = v0;
      w[1] = v1;
    }
    float* hacc = t.acc;
    if (tid < 128) {
      hacc[tid] += t.dh[tid];
      for (int q = 0; q < OUT; ++q) hacc[128 + q * 128 + tid] = fmaf(t.dout[q], t.hd[tid], hacc[128 + q * 128 + tid]);
    }
    if (tid < OUT) hacc[128 + 128 * OUT + tid] += t.dout[tid];
  } else {
    const int HS = DR_HEAD_STRIDE(OUT);
    float* hg = p.head + (int64_t)pb * HS;
    if (tid < 64) st_part<WT>(hg + tid, t.g[tid]);
    if (tid < 128) {
      st_part<WT>(hg + 64 + tid, t.hd[tid]);
      st_part<WT>(hg + 192 + tid, t.dh[tid]);
    }
    if (tid < OUT) st_part<WT>(hg + 320 + tid, t.dout[tid]);
  }
  if (!t.dg_deferred) __syncthreads();

  return true;
}

}  // namespace drk
