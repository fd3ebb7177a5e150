// Diagnostic: dr_reduce_update alone inside a hipGraph (GINet residue step
// shapes: F=30, out=1, B=64), to separate its own cost from the step's.
//   hipcc --offload-arch=gfx950 -O3 tools/reduce_bench.cpp -Iinclude \
//     -Ldeeprank-gnn-2_amd/deeprank2_amd -ldeeprank2_amd -o tools/reduce_bench.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "deeprank2_amd.h"

int main() {
  const int F = 30, OUT = 1, B = 64;
  const int SS = DR_SLAB_STRIDE(F), HS = DR_HEAD_STRIDE(OUT);
  // GINet recipe (deeprank2_amd/neuralnets/gnn/ginet.py: recipe)
  struct P { int numel, kind, off1, off2, cols; };
  std::vector<P> ps = {
      {16 * F, DR_GRAD_SLAB, 0, 0, 0}, {1, DR_GRAD_ZERO, 0, 0, 0}, {33, DR_GRAD_ZERO, 0, 0, 0},
      {512, DR_GRAD_SLAB, 32 * F, 0, 0}, {1, DR_GRAD_ZERO, 0, 0, 0}, {65, DR_GRAD_ZERO, 0, 0, 0},
      {16 * F, DR_GRAD_SLAB, 16 * F, 0, 0}, {1, DR_GRAD_ZERO, 0, 0, 0}, {33, DR_GRAD_ZERO, 0, 0, 0},
      {512, DR_GRAD_SLAB, 32 * F + 512, 0, 0}, {1, DR_GRAD_ZERO, 0, 0, 0}, {65, DR_GRAD_ZERO, 0, 0, 0},
      {128 * 64, DR_GRAD_OUTER, 192, 0, 64}, {128, DR_GRAD_HEAD, 192, 0, 0},
      {OUT * 128, DR_GRAD_OUTER, 320, 64, 128}, {OUT, DR_GRAD_HEAD, 320, 0, 0}};
  dr_param_table t;
  std::memset(&t, 0, sizeof(t));
  t.n_params = (int)ps.size();
  t.slab_stride = SS;
  t.head_stride = HS;
  for (size_t i = 0; i < ps.size(); ++i) {
    float* buf;
    hipMalloc(&buf, 4 * ps[i].numel * sizeof(float));
    hipMemset(buf, 0, 4 * ps[i].numel * sizeof(float));
    t.param[i] = buf;
    t.grad[i] = buf + ps[i].numel;
    t.exp_avg[i] = buf + 2 * ps[i].numel;
    t.exp_avg_sq[i] = buf + 3 * ps[i].numel;
    t.numel[i] = ps[i].numel;
    t.recipe[i] = {ps[i].kind, ps[i].off1, ps[i].off2, ps[i].cols};
  }
  float *slab, *head, *lpg, *lout;
  int64_t* counter;
  hipMalloc(&slab, (size_t)B * SS * 4);
  hipMalloc(&head, (size_t)B * HS * 4);
  hipMalloc(&lpg, B * 4);
  hipMalloc(&lout, 4);
  hipMalloc(&counter, 16);
  hipMemset(slab, 0, (size_t)B * SS * 4);
  hipMemset(head, 0, (size_t)B * HS * 4);
  hipMemset(lpg, 0, B * 4);
  hipMemset(counter, 0, 16);
  dr_adam adam{1e-3f, 0.9f, 0.999f, 1e-8f, 1e-5f, 0.1f, 0.03f, 1, counter};
  dr_adam adam_off = adam;
  adam_off.enabled = 0;
  hipStream_t s;
  hipStreamCreate(&s);
  auto time = [&](const char* name, auto fn) {
    const int reps = 200;
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int i = 0; i < reps; ++i) fn();
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphLaunch(ge, s);
    hipStreamSynchronize(s);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a, s);
    for (int k = 0; k < 10; ++k) hipGraphLaunch(ge, s);
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    std::printf("  %-34s %6.2f us\n", name, ms * 1e3f / (10 * reps));
  };
  time("reduce+Adam (GINet, B=64)", [&] { dr_reduce_update(&t, slab, head, B, &adam, lpg, 1.f / B, lout, s); });
  time("reduce, Adam off", [&] { dr_reduce_update(&t, slab, head, B, &adam_off, lpg, 1.f / B, lout, s); });
  time("reduce, Adam off, B=8, no loss", [&] { dr_reduce_update(&t, slab, head, 8, &adam_off, nullptr, 1.f, nullptr, s); });
  dr_adam adam_nocnt = adam;
  adam_nocnt.step_counter = nullptr;
  time("reduce+Adam, host bias corrections", [&] { dr_reduce_update(&t, slab, head, B, &adam_nocnt, lpg, 1.f / B, lout, s); });
  dr_param_table tng = t;
  for (int i = 0; i < tng.n_params; ++i) tng.grad[i] = nullptr;
  time("reduce+Adam, grads not written", [&] { dr_reduce_update(&tng, slab, head, B, &adam, lpg, 1.f / B, lout, s); });
  dr_param_table t1 = t;
  t1.n_params = 1;
  time("one SLAB param (480), Adam off", [&] { dr_reduce_update(&t1, slab, head, B, &adam_off, nullptr, 1.f, nullptr, s); });
  dr_param_table t13 = t;
  t13.n_params = 13;
  time("13 params (no fc1 bias/fc2), Adam off", [&] { dr_reduce_update(&t13, slab, head, B, &adam_off, nullptr, 1.f, nullptr, s); });
  return 0;
}
