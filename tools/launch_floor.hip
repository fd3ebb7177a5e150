// Diagnostic: the per-kernel floor on this GPU inside a hipGraph (what a
// step pays per launch), versus how much a kernel writes.  Build + run:
//   hipcc --offload-arch=gfx950 -O3 tools/launch_floor.hip -o /tmp/launch_floor && /tmp/launch_floor
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));           \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__global__ void empty_kernel() {}

__global__ void write_kernel(float* p, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = (float)i;
}

__global__ void rw_kernel(const float* a, float* p, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = a[i] + 1.f;
}

// graph-pass-like producer: 64 blocks, block b writes row b (stride floats)
__global__ void produce_rows(float* slab, int stride, float v) {
  float* row = slab + (size_t)blockIdx.x * stride;
  for (int i = threadIdx.x; i < stride; i += blockDim.x) row[i] = v + (float)i;
}

// reduce-like consumer: block j sums 64 rows for 64 consecutive columns (8 chunks x 64 lanes)
__global__ void reduce_rows(const float* slab, int stride, int rows, float* out, int cols) {
  __shared__ float part[8][64];
  const int lp = threadIdx.x & 63, ch = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lp;
  float acc = 0.f;
  if (c < cols) {
    const int r0 = rows * ch / 8, r1 = rows * (ch + 1) / 8;
    float u[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) u[k] = (r0 + k < r1) ? slab[(size_t)(r0 + k) * stride + c] : 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += u[k];
  }
  part[ch][lp] = acc;
  __syncthreads();
  if (ch == 0 && c < cols) {
    float s = 0.f;
    for (int k = 0; k < 8; ++k) s += part[k][lp];
    out[c] = s;
  }
}

// fused alternative: every block atomically adds its row into acc; the last
// block to arrive (ticket) applies an update over all columns and re-zeroes acc
__global__ void produce_atomic_last(float* acc, int cols, float* params, unsigned* ticket, int nblocks) {
  __shared__ bool last;
  for (int i = threadIdx.x; i < cols; i += blockDim.x) atomicAdd(&acc[i], 1.f + (float)blockIdx.x);
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) last = (atomicAdd(ticket, 1u) == (unsigned)nblocks - 1);
  __syncthreads();
  if (!last) return;
  __threadfence();
  for (int i = threadIdx.x; i < cols; i += blockDim.x) {
    const float g = __hip_atomic_load(&acc[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    params[i] -= 1e-3f * g;
    acc[i] = 0.f;
  }
  if (threadIdx.x == 0) *ticket = 0u;
}

template <int W>
struct BigArg {
  int v[W];
};

template <int W>
__global__ void bigarg_kernel(BigArg<W> a, float* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = (float)a.v[W - 1];
}

template <class F>
float graph_us(hipStream_t s, int reps, F launch) {
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < reps; ++i) launch();
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
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  hipGraphExecDestroy(ge);
  hipGraphDestroy(g);
  return ms * 1e3f / (10.f * reps);
}

int main() {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  float *p, *q;
  const int n = 1 << 22;
  CK(hipMalloc(&p, n * sizeof(float)));
  CK(hipMalloc(&q, n * sizeof(float)));
  CK(hipMemset(q, 0, n * sizeof(float)));
  const int reps = 200;
  std::printf("per-launch time inside a hipGraph of %d launches:\n", reps);
  std::printf("  empty 1x64            : %6.2f us\n", graph_us(s, reps, [&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s); }));
  std::printf("  empty 64x1024         : %6.2f us\n", graph_us(s, reps, [&] { hipLaunchKernelGGL(empty_kernel, dim3(64), dim3(1024), 0, s); }));
  std::printf("  empty 256x1024        : %6.2f us\n", graph_us(s, reps, [&] { hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(1024), 0, s); }));
  for (int m : {1, 1 << 10, 1 << 15, 1 << 17, 1 << 20}) {
    const int blocks = (m + 255) / 256 < 1024 ? (m + 255) / 256 : 1024;
    std::printf("  write %8d floats   : %6.2f us\n", m, graph_us(s, reps, [&] { hipLaunchKernelGGL(write_kernel, dim3(blocks), dim3(256), 0, s, p, m); }));
  }
  for (int m : {1 << 15, 1 << 17}) {
    const int blocks = (m + 255) / 256;
    std::printf("  read+write %6d     : %6.2f us\n", m, graph_us(s, reps, [&] { hipLaunchKernelGGL(rw_kernel, dim3(blocks), dim3(256), 0, s, q, p, m); }));
  }
  {  // the step's pattern: 64-row producer then a column reduce of its fresh output
    const int stride = 2308, cols = 2308;
    float* out = q;
    std::printf("  producer 64 rows only : %6.2f us\n", graph_us(s, reps, [&] { hipLaunchKernelGGL(produce_rows, dim3(64), dim3(1024), 0, s, p, stride, 1.f); }));
    std::printf("  reduce stale rows only: %6.2f us\n", graph_us(s, reps, [&] { hipLaunchKernelGGL(reduce_rows, dim3((cols + 63) / 64), dim3(512), 0, s, p, stride, 64, out, cols); }));
    std::printf("  producer + reduce     : %6.2f us per pair\n", 2.f * graph_us(s, reps, [&] {
                  static int k = 0;
                  if ((k++ & 1) == 0) hipLaunchKernelGGL(produce_rows, dim3(64), dim3(1024), 0, s, p, stride, 1.f);
                  else hipLaunchKernelGGL(reduce_rows, dim3((cols + 63) / 64), dim3(512), 0, s, p, stride, 64, out, cols);
                }));
  }
  {
    float* acc = p;
    float* params = q;
    unsigned* ticket;
    CK(hipMalloc(&ticket, sizeof(unsigned)));
    CK(hipMemset(ticket, 0, sizeof(unsigned)));
    CK(hipMemset(acc, 0, 16384 * sizeof(float)));
    for (int cols : {2048, 10496}) {
      std::printf("  fused atomics+last %5d: %6.2f us\n", cols, graph_us(s, reps, [&] {
                    hipLaunchKernelGGL(produce_atomic_last, dim3(64), dim3(1024), 0, s, acc, cols, params, ticket, 64);
                  }));
    }
    CK(hipFree(ticket));
  }
  {
    BigArg<4> a4{};
    BigArg<128> a128{};
    BigArg<384> a384{};
    BigArg<900> a900{};
    std::printf("  kernarg   16 B        : %6.2f us\n", graph_us(s, reps, [&] { hipLaunchKernelGGL(bigarg_kernel<4>, dim3(180), dim3(512), 0, s, a4, q); }));
    std::printf("  kernarg  512 B        : %6.2f us\n", graph_us(s, reps, [&] { hipLaunchKernelGGL(bigarg_kernel<128>, dim3(180), dim3(512), 0, s, a128, q); }));
    std::printf("  kernarg 1536 B        : %6.2f us\n", graph_us(s, reps, [&] { hipLaunchKernelGGL(bigarg_kernel<384>, dim3(180), dim3(512), 0, s, a384, q); }));
    std::printf("  kernarg 3600 B        : %6.2f us\n", graph_us(s, reps, [&] { hipLaunchKernelGGL(bigarg_kernel<900>, dim3(180), dim3(512), 0, s, a900, q); }));
  }
  // two dependent kernels per "step" (graph-pass-like + reduce-like)
  std::printf("  pair empty+empty      : %6.2f us per pair\n", 2.f * graph_us(s, reps, [&] {
                hipLaunchKernelGGL(empty_kernel, dim3(64), dim3(1024), 0, s);
              }));
  CK(hipFree(p));
  CK(hipFree(q));
  return 0;
}
