// Generic (any edge list, any graph size) kernels behind the layer-level API
// GINetConvLayer.forward(x, edge_index, edge_attr) (ginet.py:40-60) and its
// backward.  The whole-model fast path is ginet_fused.hip; these handle
// arbitrary COO inputs: asymmetric edges, self loops, duplicates, graphs too
// large for one workgroup's LDS.
//
//   dr_csr_from_coo : stable CSR by row (the order torch_scatter's CPU
//                     scatter_add_ visits edges in), fully on the device
//   dr_spmm_csr     : out[i] = sum_{e in row i} y[col[e]]       (ginet.py:58)
//                     or the row mean (foutnet.py:56-58; 0/0 = NaN on empty rows);
//                     dr_spmm_csr_w adds edge weights and scatter_mean's
//                     clamped mean (sgat.py:74-80)
//   dr_linear_*     : fc(x) = x W^T (ginet.py:45) and its two gradients
//   dr_edge_mlp_scatter[_bwd] : the vanilla edge MLP + scatter_sum (vanilla_gnn.py:29-35)
//
// All are HBM/L2-bound gathers; deterministic (no float atomics).

#include <hip/hip_runtime.h>

#include "../../include/deeprank2_amd.h"
#include "dr_common.h"

namespace {

__global__ void count_rows_kernel(const int64_t* __restrict__ row, int64_t n, int32_t* __restrict__ cnt) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&cnt[row[e]], 1);
}

// Exclusive scan of cnt[0..n) into out[0..n] (out[n] = total), one workgroup
// of 1024 threads walking the array in chunks with a running carry.
__global__ void __launch_bounds__(1024) scan_kernel(const int32_t* __restrict__ cnt, int32_t n, int32_t* __restrict__ out) {
  __shared__ int32_t part[1024];
  __shared__ int32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < n; base += 1024) {
    const int i = base + threadIdx.x;
    const int v = (i < n) ? cnt[i] : 0;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const int t = (threadIdx.x >= off) ? part[threadIdx.x - off] : 0;
      __syncthreads();
      part[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < n) out[i] = carry + part[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[n] = carry;
}

__global__ void place_kernel(const int64_t* __restrict__ row, int64_t n, int32_t* __restrict__ cursor,
                             int32_t* __restrict__ perm) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int pos = atomicAdd(&cursor[row[e]], 1);
    perm[pos] = (int32_t)e;
  }
}

// Atomic placement scrambles the order inside a row; restore edge order
// (stable CSR) with a per-row insertion sort, then gather the columns.
__global__ void sort_rows_kernel(const int32_t* __restrict__ rowptr, int32_t n_rows, int32_t* __restrict__ perm,
                                 const int64_t* __restrict__ col, int32_t* __restrict__ col_sorted) {
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < n_rows; r += gridDim.x * blockDim.x) {
    const int b = rowptr[r], e = rowptr[r + 1];
    for (int i = b + 1; i < e; ++i) {
      const int v = perm[i];
      int j = i - 1;
      while (j >= b && perm[j] > v) {
        perm[j + 1] = perm[j];
        --j;
      }
      perm[j + 1] = v;
    }
    for (int i = b; i < e; ++i) col_sorted[i] = (int32_t)col[perm[i]];
  }
}

__global__ void spmm_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                            const float* __restrict__ w, const float* __restrict__ y, int32_t n_rows, int32_t C,
                            int32_t mode, float* __restrict__ out) {
  const int64_t total = (int64_t)n_rows * C;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < total; p += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(p / C);
    const int c = (int)(p - (int64_t)i * C);
    float acc = 0.f;
    const int eb = rowptr[i], ee = rowptr[i + 1];
    if (w)
      for (int e = eb; e < ee; ++e) acc = fmaf(w[e], y[(int64_t)col[e] * C + c], acc);
    else
      for (int e = eb; e < ee; ++e) acc += y[(int64_t)col[e] * C + c];
    if (mode & DR_SPMM_MEAN) acc /= (float)(ee - eb);
    if (mode & DR_SPMM_MEAN_CLAMP) acc /= (float)(ee > eb ? ee - eb : 1);
    out[p] = ((mode & DR_SPMM_RELU) && acc <= 0.f) ? 0.f : acc;
  }
}

__global__ void xwT_kernel(const float* __restrict__ x, const float* __restrict__ w, int32_t M, int32_t K, int32_t N,
                           float* __restrict__ y) {
  const int64_t total = (int64_t)M * N;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < total; p += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = p / N;
    const int n = (int)(p - m * N);
    const float* xr = x + m * K;
    const float* wr = w + (int64_t)n * K;
    float acc = 0.f;
    for (int k = 0; k < K; ++k) acc = fmaf(xr[k], wr[k], acc);
    y[p] = acc;
  }
}

__global__ void xw_kernel(const float* __restrict__ dy, const float* __restrict__ w, int32_t M, int32_t N, int32_t K,
                          float* __restrict__ dx) {
  const int64_t total = (int64_t)M * K;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < total; p += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = p / K;
    const int k = (int)(p - m * K);
    const float* dr = dy + m * N;
    float acc = 0.f;
    for (int n = 0; n < N; ++n) acc = fmaf(dr[n], w[(int64_t)n * K + k], acc);
    dx[p] = acc;
  }
}

__global__ void dw_partial_kernel(const float* __restrict__ dy, const float* __restrict__ x, int32_t M, int32_t N,
                                  int32_t K, int32_t n_split, float* __restrict__ scratch) {
  const int64_t plane = (int64_t)N * K;
  const int64_t total = plane * n_split;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < total; p += (int64_t)gridDim.x * blockDim.x) {
    const int s = (int)(p / plane);
    const int64_t q = p - (int64_t)s * plane;
    const int n = (int)(q / K);
    const int k = (int)(q - (int64_t)n * K);
    const int64_t mb = ((int64_t)M * s) / n_split, me = ((int64_t)M * (s + 1)) / n_split;
    float acc = 0.f;
    for (int64_t m = mb; m < me; ++m) acc = fmaf(dy[m * N + n], x[m * K + k], acc);
    scratch[p] = acc;
  }
}

__global__ void dw_sum_kernel(const float* __restrict__ scratch, int64_t plane, int32_t n_split, float* __restrict__ dw) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < plane; p += (int64_t)gridDim.x * blockDim.x) {
    float acc = 0.f;
    for (int s = 0; s < n_split; ++s) acc += scratch[s * plane + p];
    dw[p] = acc;
  }
}

// Vanilla edge MLP fused into the CSR gather (vanilla_gnn.py:29-35), 32 channels:
// S[i,c] = sum_{e in row i} relu(A[i,c] + B[col e, c] + Wc[c,:] ea_e + be[c]).
__device__ __forceinline__ float edge_pre(const float* we, int ld_we, int c, const float* ea, int Fe, float base) {
  float v = 0.f;
  for (int f = 0; f < Fe; ++f) v = fmaf(we[c * ld_we + f], ea[f], v);
  return base + v;
}

__global__ void edge_mlp_scatter_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                        int32_t n_rows, const float* __restrict__ A, const float* __restrict__ B,
                                        const float* __restrict__ ea, int32_t Fe, const float* __restrict__ wc,
                                        int32_t ld_we, const float* __restrict__ be, float* __restrict__ S) {
  const int64_t total = (int64_t)n_rows * 32;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < total; p += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(p >> 5), c = (int)(p & 31);
    const float a = A[p], bc = be[c];
    float acc = 0.f;
    for (int e = rowptr[i]; e < rowptr[i + 1]; ++e) {
      const float pre = edge_pre(wc, ld_we, c, ea + (int64_t)e * Fe, Fe, a + B[(int64_t)col[e] * 32 + c]) + bc;
      acc += (pre <= 0.f) ? 0.f : pre;
    }
    S[p] = acc;
  }
}

// Its backward given ds = dL/dS: D[i] = sum_{e in row i} relu'(pre_e) ds_i,
// D'[j] = sum_{e: dst j} relu'(pre_e) ds_src (transposed CSR + slot map),
// EAP[i, c, f] = sum_{e in row i} relu'(pre_e) ds_i ea_e[f].
__global__ void edge_mlp_scatter_bwd_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                            const int32_t* __restrict__ trowptr, const int32_t* __restrict__ tcol,
                                            const int32_t* __restrict__ teid, int32_t n_rows,
                                            const float* __restrict__ A, const float* __restrict__ B,
                                            const float* __restrict__ ea, int32_t Fe, const float* __restrict__ wc,
                                            int32_t ld_we, const float* __restrict__ be, const float* __restrict__ DS,
                                            float* __restrict__ D, float* __restrict__ DP, float* __restrict__ EAP) {
  const int64_t total = (int64_t)n_rows * 32;
  const int FeS = Fe > 0 ? Fe : 1;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < total; p += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(p >> 5), c = (int)(p & 31);
    const float a = A[p], bi = B[p], bc = be[c], dsi = DS[p];
    int cnt = 0;
    float eap[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int e = rowptr[i]; e < rowptr[i + 1]; ++e) {
      const float* ev = ea + (int64_t)e * Fe;
      const float pre = edge_pre(wc, ld_we, c, ev, Fe, a + B[(int64_t)col[e] * 32 + c]) + bc;
      if (!(pre <= 0.f)) {
        ++cnt;
        for (int f = 0; f < Fe && f < 8; ++f) eap[f] += ev[f];
      }
    }
    D[p] = cnt ? dsi * (float)cnt : 0.f;
    for (int f = 0; f < Fe && f < 8; ++f) EAP[p * FeS + f] = cnt ? dsi * eap[f] : 0.f;
    float acc = 0.f;
    for (int q = trowptr[i]; q < trowptr[i + 1]; ++q) {
      const int src = tcol[q], e = teid[q];
      const float pre = edge_pre(wc, ld_we, c, ea + (int64_t)e * Fe, Fe, A[(int64_t)src * 32 + c] + bi) + bc;
      if (!(pre <= 0.f)) acc += DS[(int64_t)src * 32 + c];
    }
    DP[p] = acc;
  }
}

// Segment max over member lists (segptr/members: CSR of a cluster vector,
// members ascending within a segment).
//   mode 0 = torch_scatter.scatter_max (community_pooling.py:209): strict '>'
//            from the lowest float, first max wins, NaN never enters, empty
//            segment -> 0 with arg = n_rows;
//   mode 1 = scatter_reduce('amax', include_self=False) as PyG's max_pool_x
//            (ginet.py:103): NaN propagates, empty -> 0; arg = first max.
__global__ void segment_max_kernel(const int32_t* __restrict__ segptr, const int32_t* __restrict__ members,
                                   const float* __restrict__ x, int32_t n_seg, int32_t C, int32_t n_rows,
                                   int32_t mode, float* __restrict__ out, int32_t* __restrict__ arg) {
  const int64_t total = (int64_t)n_seg * C;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < total; p += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(p / C), c = (int)(p - (int64_t)k * C);
    const int mb = segptr[k], me = segptr[k + 1];
    float best = -3.402823466e+38f, amax = -__builtin_inff();
    int a = n_rows;
    bool nan = false;
    for (int m = mb; m < me; ++m) {
      const int i = members[m];
      const float v = x[(int64_t)i * C + c];
      nan |= (v != v);
      amax = fmaxf(amax, v);
      if (v > best) {  // false for NaN: scatter_max never takes it
        best = v;
        a = i;
      }
    }
    float r;
    if (mode == 0) r = (a == n_rows) ? 0.f : best;
    else r = (me == mb) ? 0.f : (nan ? __int_as_float(0x7fc00000) : amax);
    out[p] = r;
    if (arg) arg[p] = a;
  }
}

// Backward: mode 0 routes dout to the arg member; mode 1 splits it evenly
// over the members equal to the max ((x == max) * dout / ties).
__global__ void segment_max_bwd_kernel(const int32_t* __restrict__ segptr, const int32_t* __restrict__ members,
                                       const float* __restrict__ x, const float* __restrict__ out,
                                       const int32_t* __restrict__ arg, const float* __restrict__ dout,
                                       int32_t n_seg, int32_t C, int32_t n_rows, int32_t mode,
                                       float* __restrict__ dx) {
  const int64_t total = (int64_t)n_seg * C;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < total; p += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(p / C), c = (int)(p - (int64_t)k * C);
    const int mb = segptr[k], me = segptr[k + 1];
    if (mode == 0) {
      for (int m = mb; m < me; ++m) dx[(int64_t)members[m] * C + c] = 0.f;
      const int a = arg[p];
      if (a < n_rows) dx[(int64_t)a * C + c] = dout[p];
    } else {
      const float mx = out[p];
      // torch's scatter_reduce amax backward counts the zero-initialised
      // output as one more tie when the max is +-0, even with include_self=False
      float ties = (mx == 0.f) ? 1.f : 0.f;
      for (int m = mb; m < me; ++m) ties += (x[(int64_t)members[m] * C + c] == mx) ? 1.f : 0.f;
      const float gsh = dout[p] / ties;
      for (int m = mb; m < me; ++m) {
        const int64_t q = (int64_t)members[m] * C + c;
        dx[q] = (x[q] == mx ? 1.f : 0.f) * gsh;
      }
    }
  }
}

// Segment mean (torch_scatter.scatter_mean: count clamped to 1), in member order.
__global__ void segment_mean_kernel(const int32_t* __restrict__ segptr, const int32_t* __restrict__ members,
                                    const float* __restrict__ x, int32_t n_seg, int32_t C,
                                    float* __restrict__ out) {
  const int64_t total = (int64_t)n_seg * C;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < total; p += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(p / C), c = (int)(p - (int64_t)k * C);
    const int mb = segptr[k], me = segptr[k + 1];
    float acc = 0.f;
    for (int m = mb; m < me; ++m) acc += x[(int64_t)members[m] * C + c];
    out[p] = acc / (float)(me - mb > 0 ? me - mb : 1);
  }
}

inline int grid_for(int64_t work, int block = 256) {
  int64_t g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > 8192) g = 8192;
  return (int)g;
}

}  // namespace

extern "C" int dr_csr_from_coo(const int64_t* row, const int64_t* col, int64_t n_edges, int32_t n_rows, int32_t* rowptr,
                               int32_t* perm, int32_t* col_sorted, int32_t* scratch, void* stream) {
  if (n_edges < 0 || n_rows < 0 || !rowptr || !scratch) return DR_E_ARG;
  if (n_edges > 0 && (!row || !col || !perm || !col_sorted)) return DR_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  DR_CHECK(hipMemsetAsync(scratch, 0, sizeof(int32_t) * (size_t)(n_rows + 1), st));
  if (n_edges > 0) hipLaunchKernelGGL(count_rows_kernel, dim3(grid_for(n_edges)), dim3(256), 0, st, row, n_edges, scratch);
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, st, scratch, n_rows, rowptr);
  if (n_edges > 0) {
    DR_CHECK(hipMemcpyAsync(scratch, rowptr, sizeof(int32_t) * (size_t)n_rows, hipMemcpyDeviceToDevice, st));
    hipLaunchKernelGGL(place_kernel, dim3(grid_for(n_edges)), dim3(256), 0, st, row, n_edges, scratch, perm);
    hipLaunchKernelGGL(sort_rows_kernel, dim3(grid_for(n_rows)), dim3(256), 0, st, rowptr, n_rows, perm, col, col_sorted);
  }
  return (int)hipGetLastError();
}

extern "C" int dr_spmm_csr_w(const int32_t* rowptr, const int32_t* col, const float* w, const float* y, int32_t n_rows,
                             int32_t n_chan, int32_t mode, float* out, void* stream) {
  if (!rowptr || !out || n_rows < 0 || n_chan < 0) return DR_E_ARG;
  if ((mode & DR_SPMM_MEAN) && (mode & DR_SPMM_MEAN_CLAMP)) return DR_E_ARG;
  const int64_t work = (int64_t)n_rows * n_chan;
  if (work == 0) return DR_OK;
  hipLaunchKernelGGL(spmm_kernel, dim3(grid_for(work)), dim3(256), 0, (hipStream_t)stream, rowptr, col, w, y, n_rows,
                     n_chan, mode, out);
  return (int)hipGetLastError();
}

extern "C" int dr_spmm_csr(const int32_t* rowptr, const int32_t* col, const float* y, int32_t n_rows, int32_t n_chan,
                           int32_t mode, float* out, void* stream) {
  return dr_spmm_csr_w(rowptr, col, nullptr, y, n_rows, n_chan, mode, out, stream);
}

extern "C" int dr_linear_xwT(const float* x, const float* w, int32_t m, int32_t k, int32_t n, float* y, void* stream) {
  if (!y || m < 0 || k < 0 || n < 0) return DR_E_ARG;
  const int64_t work = (int64_t)m * n;
  if (work == 0) return DR_OK;
  hipLaunchKernelGGL(xwT_kernel, dim3(grid_for(work)), dim3(256), 0, (hipStream_t)stream, x, w, m, k, n, y);
  return (int)hipGetLastError();
}

extern "C" int dr_linear_xw(const float* dy, const float* w, int32_t m, int32_t n, int32_t k, float* dx, void* stream) {
  if (!dx || m < 0 || k < 0 || n < 0) return DR_E_ARG;
  const int64_t work = (int64_t)m * k;
  if (work == 0) return DR_OK;
  hipLaunchKernelGGL(xw_kernel, dim3(grid_for(work)), dim3(256), 0, (hipStream_t)stream, dy, w, m, n, k, dx);
  return (int)hipGetLastError();
}

extern "C" int dr_linear_dw(const float* dy, const float* x, int32_t m, int32_t n, int32_t k, float* dw, float* scratch,
                            int32_t n_split, void* stream) {
  if (!dw || !scratch || m < 0 || n < 0 || k < 0 || n_split < 1) return DR_E_ARG;
  const int64_t plane = (int64_t)n * k;
  if (plane == 0) return DR_OK;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(dw_partial_kernel, dim3(grid_for(plane * n_split)), dim3(256), 0, st, dy, x, m, n, k, n_split, scratch);
  hipLaunchKernelGGL(dw_sum_kernel, dim3(grid_for(plane)), dim3(256), 0, st, scratch, plane, n_split, dw);
  return (int)hipGetLastError();
}

extern "C" int dr_edge_mlp_scatter(const int32_t* rowptr, const int32_t* col, int32_t n_rows, const float* A,
                                   const float* B, const float* ea, int32_t n_edge_feat, const float* wc,
                                   int32_t ld_we, const float* be, float* S, void* stream) {
  if (!rowptr || !A || !B || !wc || !be || !S || n_rows < 0 || n_edge_feat < 0 || n_edge_feat > 8) return DR_E_ARG;
  if (n_rows == 0) return DR_OK;
  hipLaunchKernelGGL(edge_mlp_scatter_kernel, dim3(grid_for((int64_t)n_rows * 32)), dim3(256), 0, (hipStream_t)stream,
                     rowptr, col, n_rows, A, B, ea, n_edge_feat, wc, ld_we, be, S);
  return (int)hipGetLastError();
}

extern "C" int dr_edge_mlp_scatter_bwd(const int32_t* rowptr, const int32_t* col, const int32_t* trowptr,
                                       const int32_t* tcol, const int32_t* teid, int32_t n_rows, const float* A,
                                       const float* B, const float* ea, int32_t n_edge_feat, const float* wc,
                                       int32_t ld_we, const float* be, const float* DS, float* D, float* DP,
                                       float* EAP, void* stream) {
  if (!rowptr || !trowptr || !A || !B || !wc || !be || !DS || !D || !DP || !EAP || n_rows < 0 || n_edge_feat < 0 ||
      n_edge_feat > 8)
    return DR_E_ARG;
  if (n_rows == 0) return DR_OK;
  hipLaunchKernelGGL(edge_mlp_scatter_bwd_kernel, dim3(grid_for((int64_t)n_rows * 32)), dim3(256), 0,
                     (hipStream_t)stream, rowptr, col, trowptr, tcol, teid, n_rows, A, B, ea, n_edge_feat, wc, ld_we,
                     be, DS, D, DP, EAP);
  return (int)hipGetLastError();
}

extern "C" int dr_segment_max(const int32_t* segptr, const int32_t* members, const float* x, int32_t n_seg,
                              int32_t n_chan, int32_t n_rows, int32_t mode, float* out, int32_t* arg, void* stream) {
  if (!segptr || !x || !out || n_seg < 0 || n_chan < 0 || n_rows < 0 || mode < 0 || mode > 1) return DR_E_ARG;
  const int64_t work = (int64_t)n_seg * n_chan;
  if (work == 0) return DR_OK;
  hipLaunchKernelGGL(segment_max_kernel, dim3(grid_for(work)), dim3(256), 0, (hipStream_t)stream, segptr, members, x,
                     n_seg, n_chan, n_rows, mode, out, arg);
  return (int)hipGetLastError();
}

extern "C" int dr_segment_max_bwd(const int32_t* segptr, const int32_t* members, const float* x, const float* out,
                                  const int32_t* arg, const float* dout, int32_t n_seg, int32_t n_chan,
                                  int32_t n_rows, int32_t mode, float* dx, void* stream) {
  if (!segptr || !x || !dout || !dx || n_seg < 0 || n_chan < 0 || mode < 0 || mode > 1) return DR_E_ARG;
  if (mode == 0 && !arg) return DR_E_ARG;
  if (mode == 1 && !out) return DR_E_ARG;
  const int64_t work = (int64_t)n_seg * n_chan;
  if (work == 0) return DR_OK;
  hipLaunchKernelGGL(segment_max_bwd_kernel, dim3(grid_for(work)), dim3(256), 0, (hipStream_t)stream, segptr, members,
                     x, out, arg, dout, n_seg, n_chan, n_rows, mode, dx);
  return (int)hipGetLastError();
}

extern "C" int dr_segment_mean(const int32_t* segptr, const int32_t* members, const float* x, int32_t n_seg,
                               int32_t n_chan, float* out, void* stream) {
  if (!segptr || !x || !out || n_seg < 0 || n_chan < 0) return DR_E_ARG;
  const int64_t work = (int64_t)n_seg * n_chan;
  if (work == 0) return DR_OK;
  hipLaunchKernelGGL(segment_mean_kernel, dim3(grid_for(work)), dim3(256), 0, (hipStream_t)stream, segptr, members, x,
                     n_seg, n_chan, out);
  return (int)hipGetLastError();
}
