// Markov clustering (MCL) of many graphs at once, one workgroup per graph.
//
// Replaces community_detection(method="mcl") (deeprank2/utils/community_pooling.py
// :96-162) as Trainer._precluster runs it (deeprank2/trainer.py:319-348):
// networkx's 0/1 adjacency of the undirected simple graph, then
// markov_clustering 0.0.6 run_mcl defaults — diagonal set to 1, column (l1)
// normalisation, then per iteration: expansion M <- M·M, inflation
// M <- normalize(M∘M), pruning (entries < 1e-3 zeroed, each column's first
// maximum kept) and convergence np.allclose(new, last) — all in float64 like
// the reference.  The converged support is written as a 0/1 pattern;
// dr_mcl_assign (host) turns it into cluster ids exactly as get_clusters does.
//
// The matrices (NP x NP doubles, NP = N rounded up to 64, two buffers) live in
// an HBM workspace; the expansion is an LDS-tiled fp64 GEMM (the fp64 vector
// and matrix rates are equal on MI355X, so plain FMAs), everything else is
// column-parallel.  Bound: fp64 FMA throughput (2·NP^3 flops per iteration).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <set>
#include <vector>

#include "../../include/deeprank2_amd.h"

namespace {

constexpr int MT = 256;  // threads per graph
constexpr int TB = 64;   // output tile
constexpr int TK = 16;   // k step

struct MclArgs {
  dr_mcl_graphs g;
  int32_t max_iter;
  double threshold;
};

__device__ __forceinline__ void gemm(const double* M, double* T, int NP, double* As, double* Bs) {
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  for (int r0 = 0; r0 < NP; r0 += TB)
    for (int c0 = 0; c0 < NP; c0 += TB) {
      double acc[4][4];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = 0.0;
      for (int k0 = 0; k0 < NP; k0 += TK) {
        for (int p = tid; p < TB * TK; p += MT) {
          const int r = p / TK, k = p % TK;  // A tile, stored [k][r]
          As[k * (TB + 1) + r] = M[(int64_t)(r0 + r) * NP + k0 + k];
          const int kb = p / TB, c = p % TB;  // B tile [k][c]
          Bs[kb * (TB + 1) + c] = M[(int64_t)(k0 + kb) * NP + c0 + c];
        }
        __syncthreads();
#pragma unroll 4
        for (int k = 0; k < TK; ++k) {
          double av[4], bv[4];
#pragma unroll
          for (int a = 0; a < 4; ++a) av[a] = As[k * (TB + 1) + ty * 4 + a];
#pragma unroll
          for (int b = 0; b < 4; ++b) bv[b] = Bs[k * (TB + 1) + tx * 4 + b];
#pragma unroll
          for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) acc[a][b] = fma(av[a], bv[b], acc[a][b]);
        }
        __syncthreads();
      }
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) T[(int64_t)(r0 + ty * 4 + a) * NP + c0 + tx * 4 + b] = acc[a][b];
    }
}

// sklearn normalize(norm="l1", axis=0): column sums in row order; zero columns stay zero
__device__ __forceinline__ void normalize_cols(double* M, int N, int NP, bool square_first) {
  for (int j = threadIdx.x; j < N; j += MT) {
    double s = 0.0;
    for (int i = 0; i < N; ++i) {
      double v = M[(int64_t)i * NP + j];
      if (square_first) {
        v = v * v;
        M[(int64_t)i * NP + j] = v;
      }
      s += fabs(v);
    }
    if (s == 0.0) s = 1.0;
    for (int i = 0; i < N; ++i) M[(int64_t)i * NP + j] /= s;
  }
}

__global__ void __launch_bounds__(MT) mcl_kernel(MclArgs a) {
  __shared__ double As[TK * (TB + 1)], Bs[TK * (TB + 1)];
  __shared__ int conv;
  const int g = blockIdx.x, tid = threadIdx.x;
  const dr_mcl_graphs& G = a.g;
  const int64_t n0 = G.node_off[g];
  const int N = (int)(G.node_off[g + 1] - n0);
  const int NP = (N + TB - 1) / TB * TB;
  double* M = G.ws + G.ws_off[g];
  double* T = M + (int64_t)NP * NP;
  const int* rp = G.rowptr + n0 + g;
  const int* col = G.col + G.edge_off[g];
  for (int64_t p = tid; p < (int64_t)NP * NP; p += MT) M[p] = 0.0;
  __syncthreads();
  const double* w = G.weight ? G.weight + G.edge_off[g] : nullptr;
  for (int i = tid; i < N; i += MT)  // undirected simple graph: both directions, duplicates merge
    for (int e = rp[i]; e < rp[i + 1]; ++e) {
      const int j = col[e];
      const double v = w ? w[e] : 1.0;  // weighted: the host hands a symmetric coalesced list
      M[(int64_t)i * NP + j] = v;
      M[(int64_t)j * NP + i] = v;
    }
  __syncthreads();
  for (int i = tid; i < N; i += MT) M[(int64_t)i * NP + i] = 1.0;  // add_self_loops(loop_value=1)
  __syncthreads();
  normalize_cols(M, N, NP, false);
  __syncthreads();
  int it = 0;
  for (; it < a.max_iter; ++it) {
    gemm(M, T, NP, As, Bs);  // expansion (power 2)
    __syncthreads();
    normalize_cols(T, N, NP, true);  // inflation (power 2) + normalize
    __syncthreads();
    if (tid == 0) conv = 1;
    for (int j = tid; j < N; j += MT) {  // prune: < threshold -> 0, keep the column's first maximum
      double mx = T[j];
      int am = 0;
      for (int i = 1; i < N; ++i) {
        const double v = T[(int64_t)i * NP + j];
        if (v > mx) {
          mx = v;
          am = i;
        }
      }
      for (int i = 0; i < N; ++i) {
        double& v = T[(int64_t)i * NP + j];
        if (v < a.threshold && i != am) v = 0.0;
      }
    }
    __syncthreads();
    bool ok = true;  // np.allclose(new, last): |new - last| <= 1e-8 + 1e-5 |last|
    for (int64_t p = tid; p < (int64_t)NP * NP; p += MT) {
      const double nv = T[p], lv = M[p];
      if (!(fabs(nv - lv) <= 1e-8 + 1e-5 * fabs(lv))) ok = false;
    }
    if (!ok) conv = 0;
    __syncthreads();
    double* tmp = M;
    M = T;
    T = tmp;
    if (conv) break;
    __syncthreads();
  }
  uint8_t* pat = G.pattern + G.pat_off[g];
  for (int64_t p = tid; p < (int64_t)N * N; p += MT) {
    const int i = (int)(p / N), j = (int)(p - (int64_t)i * N);
    pat[p] = M[(int64_t)i * NP + j] != 0.0 ? 1 : 0;
  }
  if (tid == 0 && G.iters) G.iters[g] = it + (it < a.max_iter ? 1 : 0);
}

}  // namespace

extern "C" int64_t dr_mcl_workspace_doubles(int32_t n_nodes) {
  const int64_t NP = (n_nodes + TB - 1) / TB * TB;
  return 2 * NP * NP;
}

extern "C" int dr_mcl(const dr_mcl_graphs* graphs, int32_t n_graphs, int32_t max_iter, double pruning_threshold,
                      void* stream) {
  if (!graphs || n_graphs < 0 || max_iter < 0) return DR_E_ARG;
  if (!graphs->node_off || !graphs->rowptr || !graphs->edge_off || !graphs->ws_off || !graphs->ws ||
      !graphs->pattern || !graphs->pat_off)
    return DR_E_ARG;
  if (n_graphs == 0) return DR_OK;
  MclArgs a;
  a.g = *graphs;
  a.max_iter = max_iter;
  a.threshold = pruning_threshold;
  hipLaunchKernelGGL(mcl_kernel, dim3(n_graphs), dim3(MT), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

// get_clusters + the reference's index assignment (host): attractors = rows
// with a non-zero diagonal; each attractor row's support is a cluster; unique
// clusters sorted lexicographically; index[c] = position (later clusters win).
extern "C" int dr_mcl_assign(const uint8_t* pattern, const int64_t* pat_off, const int64_t* node_off,
                             int32_t n_graphs, int32_t* cluster_out, int32_t* n_clusters) {
  if (!pattern || !pat_off || !node_off || !cluster_out || n_graphs < 0) return DR_E_ARG;
  for (int g = 0; g < n_graphs; ++g) {
    const int64_t n0 = node_off[g];
    const int N = (int)(node_off[g + 1] - n0);
    const uint8_t* P = pattern + pat_off[g];
    std::set<std::vector<int32_t>> uniq;
    for (int i = 0; i < N; ++i) {
      if (!P[(int64_t)i * N + i]) continue;
      std::vector<int32_t> c;
      for (int j = 0; j < N; ++j)
        if (P[(int64_t)i * N + j]) c.push_back(j);
      uniq.insert(c);
    }
    std::vector<std::vector<int32_t>> cl(uniq.begin(), uniq.end());  // std::set order == sorted tuples
    for (int i = 0; i < N; ++i) cluster_out[n0 + i] = 0;
    for (size_t ic = 0; ic < cl.size(); ++ic)
      for (int32_t j : cl[ic]) cluster_out[n0 + j] = (int32_t)ic;
    if (n_clusters) n_clusters[g] = (int32_t)cl.size();
  }
  return DR_OK;
}
