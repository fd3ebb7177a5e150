// VanillaNetwork training step as a pipeline of batch-wide row-parallel kernels.
//
// Replaces (deeprank2 v3.1.0):
//   VanillaConvolutionalLayer.forward  deeprank2/neuralnets/gnn/vanilla_gnn.py:26-38
//   VanillaNetwork.forward             vanilla_gnn.py:59-65
//   autograd backward + loss           deeprank2/trainer.py:686-689
//
// Per layer:  m_e = relu(We [x_i | x_j | ea_e] + be)  for each edge e = (i -> j),
//             s_i = sum_{e: src i} m_e,   x'_i = relu(Wn [x_i | s_i] + bn).
// The edge GEMM is never formed: We = [Wa | Wb | Wc] splits it into two node
// GEMMs, A = X Wa^T and B = X Wb^T, and pre_e = A_i + B_j + Wc ea_e + be is
// rebuilt on the fly inside the CSR gather (the fused gather + edge MLP +
// scatter).  The backward needs no per-edge storage either: with
// dpre_e = relu'(pre_e) ds_i,
//   D_i  = sum_{e: src i} dpre_e,   D'_j = sum_{e: dst j} dpre_e  (transposed CSR),
//   dWa = D^T X,  dWb = D'^T X,  dWc = sum_e dpre_e ea_e^T,  dx = ... + D Wa + D' Wb.
// Unlike GINet/FoutNet, a residue graph's E x 32 edge work does not fit one
// workgroup's LDS, so every node-level stage is a kernel over ALL rows of the
// batch (every CU busy, latency hidden by occupancy), intermediates in an HBM
// scratch (L2/MALL resident), weights staged in LDS per workgroup; only the
// mean/graph-MLP and the weight-gradient reductions are per graph.

#include <hip/hip_runtime.h>

#include <algorithm>

#include <type_traits>

#include "graph_common.h"

namespace {

using namespace drk;

constexpr int MAXFE = 8;
constexpr int RB = 256;  // row-kernel workgroup size

struct Scratch {
  int64_t x1, x2, du, dx1, s1, s2, a1, b1, a2, b2, ds, d, dp, eap, total;
};

__host__ __device__ inline Scratch scratch_layout(int64_t rows, int F, int Fe) {
  Scratch c;
  const int64_t XS = r4(F);
  int64_t o = 0;
  c.x1 = o; o += rows * XS;
  c.x2 = o; o += rows * XS;
  c.du = o; o += rows * XS;
  c.dx1 = o; o += rows * XS;
  c.s1 = o; o += rows * 32;
  c.s2 = o; o += rows * 32;
  c.a1 = o; o += rows * 32;
  c.b1 = o; o += rows * 32;
  c.a2 = o; o += rows * 32;
  c.b2 = o; o += rows * 32;
  c.ds = o; o += rows * 32;
  c.d = o; o += rows * 32;
  c.dp = o; o += rows * 32;
  c.eap = o; o += rows * 32 * (Fe > 0 ? Fe : 1);
  c.total = o;
  return c;
}

struct VA {
  dr_graph_store s;
  dr_vanilla_weights w;
  dr_pass p;
  dr_vanilla_scratch ws;
  const dr_graph_desc* descs;
  int32_t B, F, Fe, XS, KE, KN;
  Scratch L;
};

struct Layer {
  const float *we, *be, *wn, *bn;
  const float* xin;  // scratch input rows (layer 2) or nullptr = the store's x (layer 1)
  float *a, *bm, *s, *xout;
};

__host__ __device__ inline Layer layer_of(const VA& a, int l) {
  Layer L;
  float* ws = a.ws.base;
  if (l == 1) {
    L.we = a.w.we1; L.be = a.w.be1; L.wn = a.w.wn1; L.bn = a.w.bn1;
    L.xin = nullptr;
    L.a = ws + a.L.a1; L.bm = ws + a.L.b1; L.s = ws + a.L.s1; L.xout = ws + a.L.x1;
  } else {
    L.we = a.w.we2; L.be = a.w.be2; L.wn = a.w.wn2; L.bn = a.w.bn2;
    L.xin = ws + a.L.x1;
    L.a = ws + a.L.a2; L.bm = ws + a.L.b2; L.s = ws + a.L.s2; L.xout = ws + a.L.x2;
  }
  return L;
}

// node row r's input features (layer 1 reads the HBM-resident store)
__device__ __forceinline__ const float* xin_row(const VA& a, const Layer& L, int64_t r) {
  if (L.xin) return L.xin + r * a.XS;
  const int b = a.ws.row_slot[r];
  const dr_graph_desc& d = a.descs[b];
  return a.s.x + (d.node0 + (r - a.ws.row0[b])) * a.XS;
}

struct RowGraph {
  const int* rp;
  const uint16_t* col;
  const int* trp;
  const uint16_t* tcol;
  const int* teid;
  const float* ea;  // CSR slot order, row stride FeS
  int i;            // local row
  int64_t r0;       // batch row of local node 0
};

__device__ __forceinline__ RowGraph row_graph(const VA& a, int64_t r) {
  const int b = a.ws.row_slot[r];
  const dr_graph_desc& d = a.descs[b];
  RowGraph g;
  g.r0 = a.ws.row0[b];
  g.i = (int)(r - g.r0);
  g.rp = a.s.rowptr + d.node0 + d.gid;
  g.col = a.s.col + d.col0;
  g.trp = a.s.t_rowptr + d.node0 + d.gid;
  g.tcol = a.s.t_col + d.col0;
  g.teid = a.s.t_eid + d.col0;
  g.ea = a.s.ea + d.col0 * (a.Fe > 0 ? a.Fe : 1);
  return g;
}

// pre_e = (A_i + be) + B_j, then + Wc ea_e by a k-ordered fmaf chain (ab =
// A_i + be once per row; the per-graph kernel's order, vanilla_graph.hip)
__device__ __forceinline__ float edge_pre(float ab, float q, const float* wc, const float* ea, int Fe) {
  float v = ab + q;
  for (int f = 0; f < Fe; ++f) v = fmaf(wc[f], ea[f], v);
  return v;
}

// an edge's bit of channel c as 0 / 1 (the backward's counts and attribute
// sums: fmaf(bit, ea, sum) adds ea exactly when the bit is set; 0 * ea for an
// inactive edge, as in the reference's dpre^T ea product)
__device__ __forceinline__ float edge_bit(uint32_t w, int c) { return (float)((w >> c) & 1u); }

// relu'(pre) as torch's threshold_backward on relu(pre): 0 where relu(pre) <= 0
__device__ __forceinline__ bool active(float pre) { return !(pre <= 0.f); }

// ---- forward ------------------------------------------------------------------

// S_i = sum_{e in row i} relu(A_i + B_j + Wc ea_e + be): 32 threads per row
__global__ void __launch_bounds__(RB) vb_edge_fwd(VA a, int l) {
  __shared__ float swc[32 * MAXFE + 32];
  const Layer L = layer_of(a, l);
  const int F = a.F, Fe = a.Fe, KE = a.KE, FeS = Fe > 0 ? Fe : 1;
  for (int p = threadIdx.x; p < 32 * Fe; p += RB) swc[p] = L.we[(p / Fe) * KE + 2 * F + p % Fe];
  if (threadIdx.x < 32) swc[32 * MAXFE + threadIdx.x] = L.be[threadIdx.x];
  __syncthreads();
  const int c = threadIdx.x & 31;
  const float* wc = swc + c * Fe;
  const float bc = swc[32 * MAXFE + c];
  // per-edge ReLU words for the backward (a 64-lane ballot holds the two rows
  // of the wave: lanes 0-31 and 32-63)
  uint32_t* words = a.ws.relu_words ? a.ws.relu_words + (int64_t)(l - 1) * a.ws.edge0[a.B] : nullptr;
  const int hs = threadIdx.x & 32;
  for (int64_t r = blockIdx.x * (RB / 32) + (threadIdx.x >> 5); r < a.ws.n_rows; r += (int64_t)gridDim.x * (RB / 32)) {
    const RowGraph g = row_graph(a, r);
    const float ab = L.a[r * 32 + c] + bc;
    const float* Bg = L.bm + g.r0 * 32 + c;
    uint32_t* wr = words ? words + a.ws.edge0[a.ws.row_slot[r]] : nullptr;
    float acc = 0.f;
    const int eb = g.rp[g.i], ee = g.rp[g.i + 1];
    int e = eb;
    for (; e + 4 <= ee; e += 4) {  // four independent gathers in flight, summed in edge order
      const int j0 = g.col[e], j1 = g.col[e + 1], j2 = g.col[e + 2], j3 = g.col[e + 3];
      const float q[4] = {Bg[(int64_t)j0 * 32], Bg[(int64_t)j1 * 32], Bg[(int64_t)j2 * 32], Bg[(int64_t)j3 * 32]};
      const float* ea = g.ea + (int64_t)e * FeS;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float pre = edge_pre(ab, q[u], wc, ea + u * FeS, Fe);
        acc += relu_keepnan(pre);
        if (wr) {
          const uint64_t m = __ballot(active(pre));
          if (c == 0) wr[e + u] = (uint32_t)(m >> hs);
        }
      }
    }
    for (; e < ee; ++e) {
      const float pre = edge_pre(ab, Bg[(int64_t)g.col[e] * 32], wc, g.ea + (int64_t)e * FeS, Fe);
      acc += relu_keepnan(pre);
      if (wr) {
        const uint64_t m = __ballot(active(pre));
        if (c == 0) wr[e] = (uint32_t)(m >> hs);
      }
    }
    L.s[r * 32 + c] = acc;
  }
}

// vb_edge_fwd with the edge-attribute width FE fixed at compile time and 8
// edges in flight per row (the column ids, edge attributes and B rows of a
// group are all requested before the first is used); same sums, same order.
template <int FE, int U>
__device__ __forceinline__ void fwd_group(const RowGraph& g, int e, const float* Bg, const float (&wcr)[FE > 0 ? FE : 1],
                                          float ab, int FeS, int c, int hs, uint32_t* wr, float& acc) {
  constexpr int FA = FE > 0 ? FE : 1;
  int j[U];
  float ev[U][FA], q[U];
#pragma unroll
  for (int u = 0; u < U; ++u) j[u] = g.col[e + u];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int f = 0; f < FE; ++f) ev[u][f] = g.ea[(int64_t)(e + u) * FeS + f];
#pragma unroll
  for (int u = 0; u < U; ++u) q[u] = Bg[(int64_t)j[u] * 32];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    float pre = ab + q[u];
#pragma unroll
    for (int f = 0; f < FE; ++f) pre = fmaf(wcr[f], ev[u][f], pre);
    acc += relu_keepnan(pre);
    if (wr) {
      const uint64_t m = __ballot(active(pre));
      if (c == 0) wr[e + u] = (uint32_t)(m >> hs);
    }
  }
}

template <int FE>
__global__ void __launch_bounds__(RB) vb_edge_fwd8(VA a, int l) {
  constexpr int FA = FE > 0 ? FE : 1;
  const Layer L = layer_of(a, l);
  const int F = a.F, KE = a.KE, FeS = FE > 0 ? FE : 1;
  const int c = threadIdx.x & 31;
  float wcr[FA];
#pragma unroll
  for (int f = 0; f < FE; ++f) wcr[f] = L.we[c * KE + 2 * F + f];
  const float bc = L.be[c];
  uint32_t* words = a.ws.relu_words ? a.ws.relu_words + (int64_t)(l - 1) * a.ws.edge0[a.B] : nullptr;
  const int hs = threadIdx.x & 32;
  for (int64_t r = blockIdx.x * (RB / 32) + (threadIdx.x >> 5); r < a.ws.n_rows; r += (int64_t)gridDim.x * (RB / 32)) {
    const RowGraph g = row_graph(a, r);
    const float ab = L.a[r * 32 + c] + bc;
    const float* Bg = L.bm + g.r0 * 32 + c;
    uint32_t* wr = words ? words + a.ws.edge0[a.ws.row_slot[r]] : nullptr;
    float acc = 0.f;
    const int eb = g.rp[g.i], ee = g.rp[g.i + 1];
    int e = eb;
    for (; e + 8 <= ee; e += 8) fwd_group<FE, 8>(g, e, Bg, wcr, ab, FeS, c, hs, wr, acc);
    for (; e + 4 <= ee; e += 4) fwd_group<FE, 4>(g, e, Bg, wcr, ab, FeS, c, hs, wr, acc);
    for (; e < ee; ++e) fwd_group<FE, 1>(g, e, Bg, wcr, ab, FeS, c, hs, wr, acc);
    L.s[r * 32 + c] = acc;
  }
}

// vb_edge_bwd's ReLU-word form with FE fixed and 8 edges in flight (same
// counts, sums and order).
template <int FE>
__global__ void __launch_bounds__(RB) vb_edge_bwd8(VA a, int l) {
  constexpr int FA = FE > 0 ? FE : 1;
  const int FeS = FE > 0 ? FE : 1;
  float* ws = a.ws.base;
  const float* DS = ws + a.L.ds;
  float *D = ws + a.L.d, *DP = ws + a.L.dp, *EAP = ws + a.L.eap;
  const int c = threadIdx.x & 31;
  const uint32_t* words = a.ws.relu_words + (int64_t)(l - 1) * a.ws.edge0[a.B];
  for (int64_t r = blockIdx.x * (RB / 32) + (threadIdx.x >> 5); r < a.ws.n_rows; r += (int64_t)gridDim.x * (RB / 32)) {
    const RowGraph g = row_graph(a, r);
    const uint32_t* wr = words + a.ws.edge0[a.ws.row_slot[r]];
    const float dsi = DS[r * 32 + c];
    const float* DSg = DS + g.r0 * 32 + c;
    float cnt = 0.f;
    float eap[FA];
#pragma unroll
    for (int f = 0; f < FA; ++f) eap[f] = 0.f;
    const int eb = g.rp[g.i], ee = g.rp[g.i + 1];
    int e = eb;
    for (; e + 8 <= ee; e += 8) {
      uint32_t wv[8];
      float ev[8][FA];
#pragma unroll
      for (int u = 0; u < 8; ++u) wv[u] = wr[e + u];
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int f = 0; f < FE; ++f) ev[u][f] = g.ea[(int64_t)(e + u) * FeS + f];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float bit = edge_bit(wv[u], c);
        cnt += bit;
#pragma unroll
        for (int f = 0; f < FE; ++f) eap[f] = fmaf(bit, ev[u][f], eap[f]);
      }
    }
    for (; e < ee; ++e) {
      const float bit = edge_bit(wr[e], c);
      cnt += bit;
#pragma unroll
      for (int f = 0; f < FE; ++f) eap[f] = fmaf(bit, g.ea[(int64_t)e * FeS + f], eap[f]);
    }
    D[r * 32 + c] = cnt != 0.f ? dsi * cnt : 0.f;
#pragma unroll
    for (int f = 0; f < FE; ++f) EAP[(r * 32 + c) * FeS + f] = cnt != 0.f ? dsi * eap[f] : 0.f;
    float acc = 0.f;
    const int qb = g.trp[g.i], qe = g.trp[g.i + 1];
    int q = qb;
    for (; q + 8 <= qe; q += 8) {
      int src[8], ed[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        src[u] = g.tcol[q + u];
        ed[u] = g.teid[q + u];
      }
      uint32_t wv[8];
      float dv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        wv[u] = wr[ed[u]];
        dv[u] = DSg[(int64_t)src[u] * 32];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if ((wv[u] >> c) & 1u) acc += dv[u];
    }
    for (; q < qe; ++q)
      if ((wr[g.teid[q]] >> c) & 1u) acc += DSg[(int64_t)g.tcol[q] * 32];
    DP[r * 32 + c] = acc;
  }
}

// ---- tiled edge kernels (dr_vanilla_scratch tile plan) -----------------------
// One workgroup per tile of consecutive rows of one graph.  The tile's halo --
// the distinct neighbours of its rows, out- and in-edges -- is staged in LDS
// once (B rows in the forward, dS rows in the backward: one 128-byte row each,
// coalesced), together with one record per edge, so the per-edge work of
// vb_edge_fwd8 / vb_edge_bwd8 reads LDS instead of gathering a 128-byte row
// from L2/HBM per edge, and an edge's scalars are ONE broadcast LDS read:
//   forward CSR record   {halo-local column, ea[0..3)}      (16 bytes; Fe = 4: 32)
//   backward CSR record  {ReLU word, ea[0..3)}              (16 bytes; Fe = 4: 32)
//   backward transposed  {halo-local column, ReLU word}     (8 bytes)
// Rows are taken in the same lane layout (32 channels per row, eight rows per
// workgroup) and every sum runs in the same order: results are bit-identical
// to the untiled kernels.  LDS (floats): halo rows [halo_max][32] | CSR
// records [edges][RS] | (backward) transposed records [tedges][2].
template <int FE>
struct TileRec {
  static constexpr int RS = FE <= 3 ? 4 : 8;  // floats per CSR record
};
struct TileCarve {
  int rows, rec, trec, total;
};
__host__ __device__ inline TileCarve tile_carve(int hmax, int emax, int tmax, int Fe, bool bwd) {
  TileCarve c;
  const int RS = Fe <= 3 ? 4 : 8;
  c.rows = 0;
  c.rec = hmax * 32;
  c.trec = c.rec + emax * RS;
  c.total = c.trec + (bwd ? 2 * tmax : 0);
  return c;
}

// the tile's halo rows of a node-level [rows][32] array (graph block at g32) -> LDS
__device__ __forceinline__ void stage_halo(float* dst, const float* g32, const int* ids, int H) {
  for (int p = threadIdx.x; p < H * 8; p += RB) {
    const int h = p >> 3, q = (p & 7) * 4;
    *reinterpret_cast<float4*>(dst + h * 32 + q) = *reinterpret_cast<const float4*>(g32 + (int64_t)ids[h] * 32 + q);
  }
}

// edge e's record {head, ea[0..FE)} -> LDS (RS floats); head: a column id or a word
template <int FE>
__device__ __forceinline__ void put_rec(float* rec, int e, uint32_t head, const float* ea_e) {
  constexpr int RS = TileRec<FE>::RS;
  float v[4] = {__uint_as_float(head), 0.f, 0.f, 0.f};
#pragma unroll
  for (int f = 0; f < (FE < 3 ? FE : 3); ++f) v[1 + f] = ea_e[f];
  *reinterpret_cast<float4*>(rec + e * RS) = make_float4(v[0], v[1], v[2], v[3]);
  if (FE > 3) rec[e * RS + 4] = ea_e[3];
}
template <int FE>
__device__ __forceinline__ uint32_t get_rec(const float* rec, int e, float (&ev)[FE > 0 ? FE : 1]) {
  constexpr int RS = TileRec<FE>::RS;
  const float4 r = *reinterpret_cast<const float4*>(rec + e * RS);
  if (FE > 0) ev[0] = r.y;
  if (FE > 1) ev[1 < FE ? 1 : 0] = r.z;
  if (FE > 2) ev[2 < FE ? 2 : 0] = r.w;
  if (FE > 3) ev[3 < FE ? 3 : 0] = rec[e * RS + 4];
  return __float_as_uint(r.x);
}

template <int FE>
__global__ void __launch_bounds__(RB) vb_edge_fwd_tile(VA a, int l) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int FA = FE > 0 ? FE : 1, FeS = FA;
  const Layer L = layer_of(a, l);
  const int F = a.F, KE = a.KE;
  const int t = blockIdx.x, tid = threadIdx.x, c = tid & 31, hs = tid & 32;
  const int64_t rt0 = a.ws.tile_row0[t], rt1 = a.ws.tile_row0[t + 1];
  const int b = a.ws.row_slot[rt0];
  const dr_graph_desc& d = a.descs[b];
  const int64_t g0 = a.ws.row0[b];
  const int* rp = a.s.rowptr + d.node0 + d.gid;
  const int i0 = (int)(rt0 - g0), e0 = rp[i0], ne = rp[(int)(rt1 - g0)] - e0;
  const int h0 = a.ws.halo_off[t], H = a.ws.halo_off[t + 1] - h0;
  const TileCarve tc = tile_carve(a.ws.halo_max, a.ws.tile_edges_max, 0, FE, false);
  float* sB = lds + tc.rows;
  float* sR = lds + tc.rec;
  stage_halo(sB, L.bm + g0 * 32, a.ws.halo_ids + h0, H);
  {
    const float* ea = a.s.ea + (d.col0 + e0) * FeS;
    const uint16_t* lc = a.ws.lcol + a.ws.lcol_off[t];
    for (int p = tid; p < ne; p += RB) put_rec<FE>(sR, p, lc[p], ea + (int64_t)p * FeS);
  }
  float wcr[FA];
#pragma unroll
  for (int f = 0; f < FE; ++f) wcr[f] = L.we[c * KE + 2 * F + f];
  const float bc = L.be[c];
  uint32_t* wr = a.ws.relu_words + (int64_t)(l - 1) * a.ws.edge0[a.B] + a.ws.edge0[b] + e0;
  __syncthreads();
  for (int64_t r = rt0 + (tid >> 5); r < rt1; r += RB / 32) {
    const int i = (int)(r - g0);
    const float ab = L.a[r * 32 + c] + bc;
    float acc = 0.f;
    const int eb = rp[i] - e0, ee = rp[i + 1] - e0;
    int e = eb;
    auto group = [&](auto un) {
      constexpr int U = decltype(un)::value;
      uint32_t j[U];
      float ev[U][FA], q[U];
#pragma unroll
      for (int u = 0; u < U; ++u) j[u] = get_rec<FE>(sR, e + u, ev[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) q[u] = sB[j[u] * 32 + c];
      uint32_t mine = 0u;  // lane c < U keeps word c: one contiguous store per group
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float pre = ab + q[u];
#pragma unroll
        for (int f = 0; f < FE; ++f) pre = fmaf(wcr[f], ev[u][f], pre);
        acc += relu_keepnan(pre);
        const uint64_t m = __ballot(active(pre));
        if (c == u) mine = (uint32_t)(m >> hs);
      }
      if (c < U) wr[e + c] = mine;
    };
    for (; e + 8 <= ee; e += 8) group(std::integral_constant<int, 8>());
    for (; e + 4 <= ee; e += 4) group(std::integral_constant<int, 4>());
    for (; e < ee; ++e) group(std::integral_constant<int, 1>());
    L.s[r * 32 + c] = acc;
  }
}

template <int FE>
__global__ void __launch_bounds__(RB) vb_edge_bwd_tile(VA a, int l) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int FA = FE > 0 ? FE : 1, FeS = FA;
  float* ws = a.ws.base;
  const float* DS = ws + a.L.ds;
  float *D = ws + a.L.d, *DP = ws + a.L.dp, *EAP = ws + a.L.eap;
  const int t = blockIdx.x, tid = threadIdx.x, c = tid & 31;
  const int64_t rt0 = a.ws.tile_row0[t], rt1 = a.ws.tile_row0[t + 1];
  const int b = a.ws.row_slot[rt0];
  const dr_graph_desc& d = a.descs[b];
  const int64_t g0 = a.ws.row0[b];
  const int* rp = a.s.rowptr + d.node0 + d.gid;
  const int* trp = a.s.t_rowptr + d.node0 + d.gid;
  const int i0 = (int)(rt0 - g0), i1 = (int)(rt1 - g0);
  const int e0 = rp[i0], ne = rp[i1] - e0, q0 = trp[i0], nq = trp[i1] - q0;
  const int h0 = a.ws.halo_off[t], H = a.ws.halo_off[t + 1] - h0;
  const TileCarve tc = tile_carve(a.ws.halo_max, a.ws.tile_edges_max, a.ws.tile_tedges_max, FE, true);
  float* sD = lds + tc.rows;
  float* sR = lds + tc.rec;
  uint2* sTR = reinterpret_cast<uint2*>(lds + tc.trec);
  const uint32_t* words = a.ws.relu_words + (int64_t)(l - 1) * a.ws.edge0[a.B] + a.ws.edge0[b];
  stage_halo(sD, DS + g0 * 32, a.ws.halo_ids + h0, H);
  {
    const float* ea = a.s.ea + (d.col0 + e0) * FeS;
    for (int p = tid; p < ne; p += RB) put_rec<FE>(sR, p, words[e0 + p], ea + (int64_t)p * FeS);
    const uint16_t* lt = a.ws.ltcol + a.ws.ltcol_off[t];
    const int* teid = a.s.t_eid + d.col0;  // transposed slot -> CSR slot
    for (int p = tid; p < nq; p += RB)
      sTR[p] = make_uint2(lt[p], words[teid[q0 + p]]);  // gathered while staging: no dependent loads in the row loop
  }
  __syncthreads();
  const bool twc = a.ws.tile_wc != nullptr;  // the tile's dWc share instead of per-row eap
  float wsum[FA];
#pragma unroll
  for (int f = 0; f < FA; ++f) wsum[f] = 0.f;
  for (int64_t r = rt0 + (tid >> 5); r < rt1; r += RB / 32) {
    const int i = (int)(r - g0);
    const float dsi = DS[r * 32 + c];
    float cnt = 0.f;
    float eap[FA];
#pragma unroll
    for (int f = 0; f < FA; ++f) eap[f] = 0.f;
    const int eb = rp[i] - e0, ee = rp[i + 1] - e0;
    int e = eb;
    for (; e + 8 <= ee; e += 8) {
      uint32_t wv[8];
      float ev[8][FA];
#pragma unroll
      for (int u = 0; u < 8; ++u) wv[u] = get_rec<FE>(sR, e + u, ev[u]);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float bit = edge_bit(wv[u], c);
        cnt += bit;
#pragma unroll
        for (int f = 0; f < FE; ++f) eap[f] = fmaf(bit, ev[u][f], eap[f]);
      }
    }
    for (; e < ee; ++e) {
      float ev[FA];
      const float bit = edge_bit(get_rec<FE>(sR, e, ev), c);
      cnt += bit;
#pragma unroll
      for (int f = 0; f < FE; ++f) eap[f] = fmaf(bit, ev[f], eap[f]);
    }
    D[r * 32 + c] = cnt != 0.f ? dsi * cnt : 0.f;
    if (twc) {
#pragma unroll
      for (int f = 0; f < FE; ++f) wsum[f] += cnt != 0.f ? dsi * eap[f] : 0.f;
    } else {
#pragma unroll
      for (int f = 0; f < FE; ++f) EAP[(r * 32 + c) * FeS + f] = cnt != 0.f ? dsi * eap[f] : 0.f;
    }
    float acc = 0.f;
    const int qb = trp[i] - q0, qe = trp[i + 1] - q0;
    int q = qb;
    for (; q + 8 <= qe; q += 8) {
      uint2 tr[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) tr[u] = sTR[q + u];
      float dv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) dv[u] = sD[tr[u].x * 32 + c];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if ((tr[u].y >> c) & 1u) acc += dv[u];
    }
    for (; q < qe; ++q) {
      const uint2 tr = sTR[q];
      if ((tr.y >> c) & 1u) acc += sD[tr.x * 32 + c];
    }
    DP[r * 32 + c] = acc;
  }
  if (twc && FE > 0) {  // the 8 row groups' shares, combined in group order (sD is dead)
    __syncthreads();
    const int rg = tid >> 5;
#pragma unroll
    for (int f = 0; f < FE; ++f) sD[(rg * 32 + c) * FeS + f] = wsum[f];
    __syncthreads();
    if (tid < 32 * FeS) {
      float v = 0.f;
      for (int g = 0; g < RB / 32; ++g) v += sD[g * 32 * FeS + tid];
      a.ws.tile_wc[(int64_t)t * 32 * FeS + tid] = v;
    }
  }
}

// per graph: scatter_mean -> graph MLP -> loss -> head backward (one workgroup)
constexpr int HT = 1024;  // vb_head threads: 32 row chunks at a time for the mean over ~3k-node graphs
__global__ void __launch_bounds__(HT) vb_head(VA a) {
  __shared__ float sG[64], sH[128], sDh[128], sDout[16], sRed[HT];
  __shared__ float sW1[128 * 65];  // fc1.weight [128][F] at row stride F + 1 (conflict-free both ways)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x;
  const int F = a.F, XS = a.XS, OUT = a.p.out_dim;
  const int LW = F + 1;
  {  // fc1.weight into LDS first: its loads overlap the mean's (the MLP and its
     // backward then read LDS instead of 128-long chains of global loads)
    float w[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int p = tid + u * HT;
      w[u] = p < 128 * F ? a.w.g1w[p] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int p = tid + u * HT;
      if (p < 128 * F) sW1[(p / F) * LW + p % F] = w[u];
    }
  }
  const int64_t r0 = a.ws.row0[b];
  const int N = a.ws.row0[b + 1] - (int)r0;
  const float* X2 = a.ws.base + a.L.x2 + r0 * XS;
  const float y_g = a.s.y[a.descs[b].gid];
  if (a.p.step_counter && b == 0 && tid == 0) a.p.step_counter[1] = a.p.step_counter[0];
  {  // the mean: column sums over the graph's DR_VANILLA_CHUNK-row chunks (rows
     // in order within a chunk), the chunks summed in groups of 8 (in order),
     // then the groups in order.  The chunk-fused forward leaves its tiles'
     // sums in part_mean; otherwise they are summed here from X2.  (Groups, not
     // one running sum: a group's 8 loads are in flight together.)
    constexpr int CR = DR_VANILLA_CHUNK, GS = 8, NG = HT / 32;  // NG groups of GS chunks per round
    const int nch = (N + CR - 1) / CR;
    const int n = tid & 31, gq = tid >> 5;
    float t = 0.f;  // thread n < F: the ordered sum over the groups
    for (int g0 = 0; g0 * GS < nch; g0 += NG) {
      const int c0 = (g0 + gq) * GS;
      float gs = 0.f;
      if (n < F && c0 < nch) {
        const int c1 = min(nch, c0 + GS);
        float v[GS];
        if (a.ws.part_mean) {
          const float* pm = a.ws.part_mean + ((int64_t)a.ws.chunk_first[b] + c0) * 32 + n;
#pragma unroll
          for (int u = 0; u < GS; ++u) v[u] = c0 + u < c1 ? pm[(int64_t)u * 32] : 0.f;
        } else {
#pragma unroll 1
          for (int u = 0; u < GS; ++u) {  // the chunk's rows in order
            float acc = 0.f;
            if (c0 + u < c1) {
              const int i1 = min(N, (c0 + u + 1) * CR);
              int i = (c0 + u) * CR;
              for (; i + 16 <= i1; i += 16) {  // 16 rows' loads in flight, summed in row order
                float w[16];
#pragma unroll
                for (int q = 0; q < 16; ++q) w[q] = X2[(int64_t)(i + q) * XS + n];
#pragma unroll
                for (int q = 0; q < 16; ++q) acc += w[q];
              }
              for (; i < i1; ++i) acc += X2[(int64_t)i * XS + n];
            }
            v[u] = acc;
          }
        }
#pragma unroll
        for (int u = 0; u < GS; ++u)
          if (c0 + u < c1) gs += v[u];
      }
      sRed[tid] = gs;
      __syncthreads();
      if (tid < F)
        for (int q = 0; q < NG && (g0 + q) * GS < nch; ++q) t += sRed[q * 32 + tid];
      __syncthreads();
    }
    if (tid < F) sG[tid] = t / (float)N;
  }
  __syncthreads();
  if (tid < 128) {
    float acc = 0.f;
    for (int n = 0; n < F; ++n) acc = fmaf(sG[n], sW1[tid * LW + n], acc);
    sH[tid] = relu_keepnan(acc + a.w.g1b[tid]);
  }
  __syncthreads();
  for (int q = wave; q < OUT; q += HT / 64) {
    float v = fmaf(sH[lane], a.w.g2w[q * 128 + lane], sH[lane + 64] * a.w.g2w[q * 128 + lane + 64]);
    v = dr_wave_sum(v);
    if (lane == 0) sDout[q] = v + a.w.g2b[q];
  }
  __syncthreads();
  const int row = a.p.slot ? a.p.slot[b] : b;  // the graph's rows of the batch (dr_pass.slot)
  if ((a.p.flags & DR_PASS_FORWARD) && tid < OUT) a.p.out[(int64_t)row * OUT + tid] = sDout[tid];
  if (!(a.p.flags & DR_PASS_BACKWARD)) return;
  __syncthreads();
  if (tid == 0) {  // loss gradient (trainer.py:688-689)
    if (a.p.loss_kind == DR_LOSS_MSE) {
      const float dl = sDout[0] - y_g;
      if (a.p.loss_per_graph) a.p.loss_per_graph[row] = dl * dl;
      sDout[0] = 2.f * dl * a.p.loss_scale;
    } else if (a.p.loss_kind == DR_LOSS_CE) {
      const int yi = (int)y_g;
      float mx = sDout[0];
      for (int q = 1; q < OUT; ++q) mx = fmaxf(mx, sDout[q]);
      float se = 0.f;
      for (int q = 0; q < OUT; ++q) se += expf(sDout[q] - mx);
      const float lse = mx + logf(se);
      const float wy = a.p.class_w ? a.p.class_w[yi] : 1.f;
      if (a.p.loss_per_graph) a.p.loss_per_graph[row] = wy * (lse - sDout[yi]);
      for (int q = 0; q < OUT; ++q) sDout[q] = wy * (expf(sDout[q] - lse) - (q == yi ? 1.f : 0.f)) * a.p.loss_scale;
    } else {
      for (int q = 0; q < OUT; ++q) sDout[q] = a.p.dout[(int64_t)row * OUT + q];
    }
  }
  __syncthreads();
  if (tid < 128) {
    float acc = 0.f;
    for (int q = 0; q < OUT; ++q) acc = fmaf(a.w.g2w[q * 128 + tid], sDout[q], acc);
    sDh[tid] = relu_bwd(sH[tid], acc);
  }
  __syncthreads();
  float* hg = a.p.head + (int64_t)row * DR_VANILLA_HEAD_STRIDE(F, OUT);
  const int HD = XS + 256 + r4(OUT);  // d mean, consumed by vb_du2
  if (tid < F) {
    float acc = 0.f;
    for (int r = 0; r < 128; ++r) acc = fmaf(sW1[r * LW + tid], sDh[r], acc);
    hg[HD + tid] = acc / (float)N;  // scatter_mean backward: grad / count
  }
  if (tid < XS) hg[tid] = tid < F ? sG[tid] : 0.f;
  if (tid < 128) {
    hg[XS + tid] = sH[tid];
    hg[XS + 128 + tid] = sDh[tid];
  }
  if (tid < OUT) hg[XS + 256 + tid] = sDout[tid];
}

// ---- backward -----------------------------------------------------------------

// DU = relu'(X2) * dmean[graph]  (layer 2)   or   relu'(X1) * DX1  (layer 1)
__global__ void __launch_bounds__(RB) vb_du(VA a, int l) {
  const int F = a.F, XS = a.XS;
  const float* xo = a.ws.base + (l == 2 ? a.L.x2 : a.L.x1);
  const float* dx1 = a.ws.base + a.L.dx1;
  float* du = a.ws.base + a.L.du;
  const int HS = DR_VANILLA_HEAD_STRIDE(F, a.p.out_dim), HD = XS + 256 + r4(a.p.out_dim);
  // four consecutive columns of one row per thread (XS is a multiple of 4)
  const int64_t total4 = a.ws.n_rows * XS / 4;
  for (int64_t p4 = blockIdx.x * (int64_t)RB + threadIdx.x; p4 < total4; p4 += (int64_t)gridDim.x * RB) {
    const int64_t p = p4 * 4, r = p / XS;
    const int n = (int)(p - r * XS);
    const float4 x4 = *reinterpret_cast<const float4*>(xo + p);
    float4 g4;
    if (l == 2) {
      const float* hg = a.p.head + (int64_t)(a.p.slot ? a.p.slot[a.ws.row_slot[r]] : a.ws.row_slot[r]) * HS + HD + n;
      g4 = make_float4(n < F ? hg[0] : 0.f, n + 1 < F ? hg[1] : 0.f, n + 2 < F ? hg[2] : 0.f, n + 3 < F ? hg[3] : 0.f);
    } else {
      g4 = *reinterpret_cast<const float4*>(dx1 + p);
    }
    float4 o;
    o.x = n < F ? relu_bwd(x4.x, g4.x) : 0.f;
    o.y = n + 1 < F ? relu_bwd(x4.y, g4.y) : 0.f;
    o.z = n + 2 < F ? relu_bwd(x4.z, g4.z) : 0.f;
    o.w = n + 3 < F ? relu_bwd(x4.w, g4.w) : 0.f;
    *reinterpret_cast<float4*>(du + p) = o;
  }
}

// D, D' and the edge-attribute partials of one layer: 32 threads per row
__global__ void __launch_bounds__(RB) vb_edge_bwd(VA a, int l) {
  __shared__ float swc[32 * MAXFE + 32];
  const Layer L = layer_of(a, l);
  const int F = a.F, Fe = a.Fe, KE = a.KE, FeS = Fe > 0 ? Fe : 1;
  for (int p = threadIdx.x; p < 32 * Fe; p += RB) swc[p] = L.we[(p / Fe) * KE + 2 * F + p % Fe];
  if (threadIdx.x < 32) swc[32 * MAXFE + threadIdx.x] = L.be[threadIdx.x];
  __syncthreads();
  float* ws = a.ws.base;
  const float* DS = ws + a.L.ds;
  float *D = ws + a.L.d, *DP = ws + a.L.dp, *EAP = ws + a.L.eap;
  const int c = threadIdx.x & 31;
  const float* wc = swc + c * Fe;
  const float bc = swc[32 * MAXFE + c];
  const uint32_t* words = a.ws.relu_words ? a.ws.relu_words + (int64_t)(l - 1) * a.ws.edge0[a.B] : nullptr;
  if (words) {  // the forward's ReLU words: no B_j / A_i gathers, no edge_attr for the transposed sum
    for (int64_t r = blockIdx.x * (RB / 32) + (threadIdx.x >> 5); r < a.ws.n_rows; r += (int64_t)gridDim.x * (RB / 32)) {
      const RowGraph g = row_graph(a, r);
      const uint32_t* wr = words + a.ws.edge0[a.ws.row_slot[r]];
      const float dsi = DS[r * 32 + c];
      const float* DSg = DS + g.r0 * 32 + c;
      float cnt = 0.f;
      float eap[MAXFE];
#pragma unroll
      for (int f = 0; f < MAXFE; ++f) eap[f] = 0.f;
      const int eb = g.rp[g.i], ee = g.rp[g.i + 1];
      for (int e = eb; e < ee; ++e) {
        const float bit = edge_bit(wr[e], c);
        cnt += bit;
#pragma unroll
        for (int f = 0; f < MAXFE; ++f)
          if (f < Fe) eap[f] = fmaf(bit, g.ea[(int64_t)e * FeS + f], eap[f]);
      }
      D[r * 32 + c] = cnt != 0.f ? dsi * cnt : 0.f;
      for (int f = 0; f < Fe; ++f) EAP[(r * 32 + c) * FeS + f] = cnt != 0.f ? dsi * eap[f] : 0.f;
      float acc = 0.f;  // D'_i over edges (src -> i), in transposed (original edge) order
      const int qb = g.trp[g.i], qe = g.trp[g.i + 1];
      int q = qb;
      for (; q + 4 <= qe; q += 4) {
        int src[4], ed[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          src[u] = g.tcol[q + u];
          ed[u] = g.teid[q + u];
        }
        uint32_t wv[4];
        float dv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          wv[u] = wr[ed[u]];
          dv[u] = DSg[(int64_t)src[u] * 32];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if ((wv[u] >> c) & 1u) acc += dv[u];
      }
      for (; q < qe; ++q)
        if ((wr[g.teid[q]] >> c) & 1u) acc += DSg[(int64_t)g.tcol[q] * 32];
      DP[r * 32 + c] = acc;
    }
    return;
  }
  for (int64_t r = blockIdx.x * (RB / 32) + (threadIdx.x >> 5); r < a.ws.n_rows; r += (int64_t)gridDim.x * (RB / 32)) {
    const RowGraph g = row_graph(a, r);
    const float ab = L.a[r * 32 + c] + bc, bi = L.bm[r * 32 + c], dsi = DS[r * 32 + c];
    const float* Bg = L.bm + g.r0 * 32 + c;
    const float* Ag = L.a + g.r0 * 32 + c;
    const float* DSg = DS + g.r0 * 32 + c;
    float cnt = 0.f;
    float eap[MAXFE];
#pragma unroll
    for (int f = 0; f < MAXFE; ++f) eap[f] = 0.f;
    const int eb = g.rp[g.i], ee = g.rp[g.i + 1];
    for (int e = eb; e < ee; ++e) {
      const float* ea = g.ea + (int64_t)e * FeS;
      const float bit = active(edge_pre(ab, Bg[(int64_t)g.col[e] * 32], wc, ea, Fe)) ? 1.f : 0.f;
      cnt += bit;
#pragma unroll
      for (int f = 0; f < MAXFE; ++f)
        if (f < Fe) eap[f] = fmaf(bit, ea[f], eap[f]);
    }
    D[r * 32 + c] = cnt != 0.f ? dsi * cnt : 0.f;
    for (int f = 0; f < Fe; ++f) EAP[(r * 32 + c) * FeS + f] = cnt != 0.f ? dsi * eap[f] : 0.f;
    float acc = 0.f;  // D'_i over edges (src -> i): pre = A_src + B_i + Wc ea_e + be
    const int qb = g.trp[g.i], qe = g.trp[g.i + 1];
    int q = qb;
    for (; q + 4 <= qe; q += 4) {
      int src[4], ed[4];
      float av[4], dv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        src[u] = g.tcol[q + u];
        ed[u] = g.teid[q + u];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        av[u] = Ag[(int64_t)src[u] * 32];
        dv[u] = DSg[(int64_t)src[u] * 32];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (active(edge_pre(av[u] + bc, bi, wc, g.ea + (int64_t)ed[u] * FeS, Fe))) acc += dv[u];
    }
    for (; q < qe; ++q) {
      const int src = g.tcol[q], e = g.teid[q];
      if (active(edge_pre(Ag[(int64_t)src * 32] + bc, bi, wc, g.ea + (int64_t)e * FeS, Fe))) acc += DSg[(int64_t)src * 32];
    }
    DP[r * 32 + c] = acc;
  }
}

// ---- node GEMMs on MFMA -----------------------------------------------------
// out(r, n) = init(r, n) + sum_{k < K} A(r, k) W(k, n) for every batch row r,
// n < NO, on v_mfma_f32_16x16x4_f32 (k in order).  A workgroup (4 waves)
// stages W [KP][NOP] in LDS once, then takes 64-row tiles: the A tile
// [64][KP] comes in as 16-byte loads (one row base per tile row, looked up
// once) into LDS at stride KP + 4 (the 16 rows of an operand read hit
// distinct banks), each wave runs 16 rows x all NO columns.  A's k axis is
// 16-byte aligned pieces: a feature row takes XS = r4(F) columns (its pad
// columns read as 0, W rows there are 0).  Modes (vanilla_gnn.py:29-37 and
// their gradients):
//   GM_HALVES: [A | B] = Xin [Wa; Wb]^T            (K = XS,      NO = 64)
//   GM_NODE:   Xout = relu([Xin | S] Wn^T + bn)    (K = XS + 32, NO = F)
//   GM_DXS:    [dX1 | DS] = DU Wn                  (K = XS,      NO = F + 32)
//   GM_DX1:    dX1 += [D | D'] [Wa2; Wb2]          (K = 64,      NO = F)
enum GemmMode { GM_HALVES = 0, GM_NODE = 1, GM_DXS = 2, GM_DX1 = 3 };
constexpr int GT = 64;  // rows per tile

__host__ __device__ inline void gemm_dims(int mode, int F, int& K, int& NO) {
  const int XS = r4(F);
  K = mode == GM_NODE ? XS + 32 : (mode == GM_DX1 ? 64 : XS);
  NO = mode == GM_HALVES ? 64 : (mode == GM_DXS ? F + 32 : F);
}
__host__ __device__ inline int gemm_lds_floats(int mode, int F) {
  int K, NO;
  gemm_dims(mode, F, K, NO);
  const int NOP = (NO + 15) & ~15;
  return K * NOP + GT * (K + 4) + GT * 2;  // W | A tile | row bases (64-bit)
}

template <int MODE>
__global__ void __launch_bounds__(RB) vb_gemm(VA a, int l) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const Layer L = layer_of(a, l);
  const int F = a.F, KE = a.KE, KN = a.KN, XS = a.XS;
  int KP, NO;
  gemm_dims(MODE, F, KP, NO);
  const int NOP = (NO + 15) & ~15, LA = KP + 4, CH = KP / 4;
  float* Ws = lds;              // [KP][NOP]
  float* As = lds + KP * NOP;   // [GT][LA]
  const float** rowp = reinterpret_cast<const float**>(As + GT * LA);  // [GT] feature-row bases
  const float* wn = l == 2 ? a.w.wn2 : a.w.wn1;
  for (int p = threadIdx.x; p < KP * NOP; p += RB) {
    const int k = p / NOP, n = p - k * NOP;
    float v = 0.f;
    if (n < NO) {
      if (MODE == GM_HALVES) v = k < F ? L.we[(n & 31) * KE + (n < 32 ? 0 : F) + k] : 0.f;
      else if (MODE == GM_NODE) v = k < F ? L.wn[n * KN + k] : (k < XS ? 0.f : L.wn[n * KN + F + k - XS]);
      else if (MODE == GM_DXS) v = k < F ? wn[k * KN + n] : 0.f;
      else v = a.w.we2[(k & 31) * KE + (k < 32 ? 0 : F) + n];
    }
    Ws[p] = v;
  }
  float* ws = a.ws.base;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, kq = lane >> 4;
  const int64_t R = a.ws.n_rows;
  for (int64_t t0 = (int64_t)blockIdx.x * GT; t0 < R; t0 += (int64_t)gridDim.x * GT) {
    __syncthreads();  // W staged / the previous tile's A reads done
    if ((MODE == GM_HALVES || MODE == GM_NODE) && threadIdx.x < GT) {
      const int64_t r = t0 + threadIdx.x;
      rowp[threadIdx.x] = r < R ? xin_row(a, L, r) : nullptr;
    }
    if (MODE == GM_HALVES || MODE == GM_NODE) __syncthreads();
    for (int p = threadIdx.x; p < GT * CH; p += RB) {
      const int i = p / CH, c4 = (p - i * CH) * 4;
      const int64_t r = t0 + i;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < R) {
        if (MODE == GM_HALVES || MODE == GM_NODE) {
          if (c4 < XS) {
            v = *reinterpret_cast<const float4*>(rowp[i] + c4);
            if (c4 + 4 > F) {  // the row's pad columns (scratch rows leave them unwritten)
              v.y = c4 + 1 < F ? v.y : 0.f;
              v.z = c4 + 2 < F ? v.z : 0.f;
              v.w = c4 + 3 < F ? v.w : 0.f;
              v.x = c4 < F ? v.x : 0.f;
            }
          } else {
            v = *reinterpret_cast<const float4*>(L.s + r * 32 + c4 - XS);
          }
        } else if (MODE == GM_DXS) {
          v = *reinterpret_cast<const float4*>(ws + a.L.du + r * XS + c4);
        } else {
          v = *reinterpret_cast<const float4*>(c4 < 32 ? ws + a.L.d + r * 32 + c4 : ws + a.L.dp + r * 32 + c4 - 32);
        }
      }
      *reinterpret_cast<float4*>(As + i * LA + c4) = v;
    }
    __syncthreads();
    const int i0 = wave * 16;
    for (int n0 = 0; n0 < NO; n0 += 16) {
      const int n = n0 + li;
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
      if (MODE == GM_DX1) {  // the accumulation starts from dX1 (the DU Wn part, GM_DXS)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int64_t r = t0 + i0 + kq * 4 + q;
          acc[q] = (r < R && n < NO) ? ws[a.L.dx1 + r * XS + n] : 0.f;
        }
      }
      for (int k0 = 0; k0 < KP; k0 += 4)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(As[(i0 + li) * LA + k0 + kq], Ws[(k0 + kq) * NOP + n], acc, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t r = t0 + i0 + kq * 4 + q;
        if (r >= R || n >= NO) continue;
        const float v = acc[q];
        if (MODE == GM_HALVES) (n < 32 ? L.a : L.bm)[r * 32 + (n & 31)] = v;
        else if (MODE == GM_NODE) L.xout[r * XS + n] = relu_keepnan(v + L.bn[n]);
        else if (MODE == GM_DXS) {
          if (n < F) {
            if (l == 2) ws[a.L.dx1 + r * XS + n] = v;
          } else {
            ws[a.L.ds + r * 32 + n - F] = v;
          }
        } else {
          ws[a.L.dx1 + r * XS + n] = v;
        }
      }
    }
  }
}

// Weight-gradient partials of one layer per chunk of DR_VANILLA_CHUNK rows
// (all CUs busy), rows staged through LDS; vb_wgrad_combine then sums each
// graph's chunks in order into its slab (deterministic).  The three GEMMs
// (dWa = D^T X, dWb = D'^T X, dWn = DU^T [X | S]: K = the chunk's rows,
// zero-padded to WR) run on MFMA, one 16x16 output tile per job, jobs over
// the 4 waves; the bias / edge-attribute sums stay scalar.
constexpr int WR = DR_VANILLA_CHUNK;

__host__ __device__ inline int layer_grad_size(int F, int Fe) { return 32 * (2 * F + Fe) + 32 + F * (F + 32) + F; }

__global__ void __launch_bounds__(RB) vb_wgrad_mfma(VA a, int l) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int ch = blockIdx.x;
  const int b = a.ws.chunk_slot[ch];
  const int F = a.F, Fe = a.Fe, KE = a.KE, KN = a.KN, XS = a.XS, FeS = Fe > 0 ? Fe : 1;
  const Layer L = layer_of(a, l);
  const int64_t r0 = a.ws.row0[b];
  const int N = a.ws.row0[b + 1] - (int)r0;
  const int i0 = (ch - a.ws.chunk_first[b]) * WR, nr = min(WR, N - i0);
  const int64_t g0 = r0 + i0;
  float* ws = a.ws.base;
  const float* X = L.xin ? L.xin + g0 * XS : a.s.x + (a.descs[b].node0 + i0) * XS;
  float* cX = lds;
  float* cS = cX + WR * XS;
  float* cD = cS + WR * 32;
  float* cDP = cD + WR * 32;
  float* cDU = cDP + WR * 32;
  // the chunk's rows (contiguous in every array) by 16-byte loads; rows past the chunk: zeros
  auto stage4 = [&](float* dst, const float* src, int n4, int valid4) {
    for (int p = threadIdx.x; p < n4; p += RB)
      reinterpret_cast<float4*>(dst)[p] = p < valid4 ? reinterpret_cast<const float4*>(src)[p] : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  stage4(cX, X, WR * XS / 4, nr * XS / 4);
  stage4(cDU, ws + a.L.du + g0 * XS, WR * XS / 4, nr * XS / 4);
  stage4(cS, L.s + g0 * 32, WR * 8, nr * 8);
  stage4(cD, ws + a.L.d + g0 * 32, WR * 8, nr * 8);
  stage4(cDP, ws + a.L.dp + g0 * 32, WR * 8, nr * 8);
  __syncthreads();
  const int nwe = 32 * KE, nwn = F * KN, total = nwe + 32 + nwn + F;
  float* out = a.ws.part + (int64_t)ch * total;
  // scalar sums: dWc (edge-attribute partials, read from HBM), dbe, dbn: four
  // lanes per output (16 rows each, loads issued together), combined in order
  const float* eap = ws + a.L.eap + g0 * 32 * FeS;
  for (int p0 = threadIdx.x; p0 < 4 * (32 * Fe + 32 + F); p0 += RB) {
    const int p = p0 >> 2, qr = p0 & 3, ib = qr * (WR / 4);
    float v = 0.f;
    if (p < 32 * Fe && a.ws.tile_wc) {  // the chunk's tiles' shares (the backward edge kernel), in tile order
      const int c = p / Fe, f = p - c * Fe;
      const int TR = a.ws.tile_rows, t0 = a.ws.tile_first[b] + i0 / TR, nt = (nr + TR - 1) / TR;
      if (qr == 0)
        for (int q = 0; q < nt; ++q) v += a.ws.tile_wc[(int64_t)(t0 + q) * 32 * FeS + c * FeS + f];
    } else if (p < 32 * Fe) {
      const int c = p / Fe, f = p - c * Fe;
      float t[WR / 4];
#pragma unroll
      for (int u = 0; u < WR / 4; ++u) t[u] = ib + u < nr ? eap[((ib + u) * 32 + c) * FeS + f] : 0.f;
#pragma unroll
      for (int u = 0; u < WR / 4; ++u) v += t[u];
    } else if (p < 32 * Fe + 32) {
      const int c = p - 32 * Fe;
#pragma unroll
      for (int u = 0; u < WR / 4; ++u) v += cD[(ib + u) * 32 + c];  // rows past the chunk are 0
    } else {
      const int n = p - 32 * Fe - 32;
#pragma unroll
      for (int u = 0; u < WR / 4; ++u) v += cDU[(ib + u) * XS + n];
    }
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    if (qr == 0) {
      if (p < 32 * Fe) out[(p / Fe) * KE + 2 * F + p % Fe] = v;
      else if (p < 32 * Fe + 32) out[nwe + p - 32 * Fe] = v;
      else out[nwe + 32 + nwn + p - 32 * Fe - 32] = v;
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, kq = lane >> 4;
  const int KT = (F + 15) >> 4, QT = (KN + 15) >> 4;
  const int jw = 2 * 2 * KT, jobs = jw + KT * QT;
  for (int job = wave; job < jobs; job += RB / 64) {
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    if (job < jw) {  // dWa (w = 0) / dWb (w = 1): rows c of the tile, columns k
      const int w = job / (2 * KT), rem = job - w * 2 * KT, ct = rem / KT, kt = rem - ct * KT;
      const float* Dm = w ? cDP : cD;
      const int cc = ct * 16 + li, kc = kt * 16 + li;
      for (int i = 0; i < WR; i += 4)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(Dm[(i + kq) * 32 + cc], kc < XS ? cX[(i + kq) * XS + kc] : 0.f, acc, 0, 0, 0);
      if (kc < F) {
#pragma unroll
        for (int q = 0; q < 4; ++q) out[(ct * 16 + kq * 4 + q) * KE + w * F + kc] = acc[q];
      }
    } else {  // dWn: rows n, columns q of [X | S]
      const int jj = job - jw, nt = jj / QT, qt = jj - nt * QT;
      const int nn = nt * 16 + li, qc = qt * 16 + li;
      for (int i = 0; i < WR; i += 4) {
        const float av = nn < XS ? cDU[(i + kq) * XS + nn] : 0.f;
        const float bv = qc < F ? cX[(i + kq) * XS + qc] : (qc < KN ? cS[(i + kq) * 32 + qc - F] : 0.f);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
      }
      if (qc < KN) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int n = nt * 16 + kq * 4 + q;
          if (n < F) out[nwe + 32 + n * KN + qc] = acc[q];
        }
      }
    }
  }
}

__global__ void __launch_bounds__(RB) vb_wgrad_combine(VA a, int l) {
  const int total = layer_grad_size(a.F, a.Fe);
  const int64_t work = (int64_t)a.B * total;
  for (int64_t q = blockIdx.x * (int64_t)RB + threadIdx.x; q < work; q += (int64_t)gridDim.x * RB) {
    const int b = (int)(q / total), p = (int)(q - (int64_t)b * total);
    // chunks in order, 8 chunks' loads in flight (an atom graph has ~50: one
    // dependent load per chunk made this a latency chain)
    const float* part = a.ws.part + p;
    const int ce = a.ws.chunk_first[b + 1];
    float v = 0.f;
    int ch = a.ws.chunk_first[b];
    for (; ch + 8 <= ce; ch += 8) {
      float u[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) u[k] = part[(int64_t)(ch + k) * total];
#pragma unroll
      for (int k = 0; k < 8; ++k) v += u[k];
    }
    for (; ch < ce; ++ch) v += part[(int64_t)ch * total];
    a.p.slab[(int64_t)(a.p.slot ? a.p.slot[b] : b) * DR_VANILLA_SLAB_STRIDE(a.F, a.Fe) + (l == 2 ? total : 0) + p] = v;
  }
}

// the FE-specialised 8-in-flight edge kernels (Fe <= 4; the backward needs the
// forward's ReLU words), tiled when the scratch carries a tile plan.  Returns
// 0: not launched, 1: untiled, 2: tiled (the backward then wrote tile_wc)
inline int launch_edge8(bool fwd, const VA& a, int l, dim3 grid, hipStream_t st) {
  if (a.Fe > 4 || (!fwd && !a.ws.relu_words)) return 0;
  if (a.ws.tile_row0 && a.ws.relu_words && a.ws.n_tiles > 0) {
    const int FeS = a.Fe > 0 ? a.Fe : 1;
    size_t lds = 4 * (size_t)tile_carve(a.ws.halo_max, a.ws.tile_edges_max, a.ws.tile_tedges_max, FeS, !fwd).total;
    if (!fwd && a.ws.tile_wc) lds = std::max(lds, (size_t)4 * (RB / 32) * 32 * 4);  // the tile's dWc shares, combined in LDS
    const dim3 tg((unsigned)a.ws.n_tiles);
#define DR_ET(FE)                                                                              \
  if (fwd) {                                                                                   \
    if (dr_allow_big_lds(reinterpret_cast<const void*>(&vb_edge_fwd_tile<FE>))) return 0;      \
    hipLaunchKernelGGL(vb_edge_fwd_tile<FE>, tg, dim3(RB), lds, st, a, l);                     \
  } else {                                                                                     \
    if (dr_allow_big_lds(reinterpret_cast<const void*>(&vb_edge_bwd_tile<FE>))) return 0;      \
    hipLaunchKernelGGL(vb_edge_bwd_tile<FE>, tg, dim3(RB), lds, st, a, l);                     \
  }
    switch (a.Fe) {
      case 0: DR_ET(0) break;
      case 1: DR_ET(1) break;
      case 2: DR_ET(2) break;
      case 3: DR_ET(3) break;
      default: DR_ET(4) break;
    }
#undef DR_ET
    return 2;
  }
#define DR_E8(FE)                                                                   \
  if (fwd) hipLaunchKernelGGL(vb_edge_fwd8<FE>, grid, dim3(RB), 0, st, a, l);      \
  else hipLaunchKernelGGL(vb_edge_bwd8<FE>, grid, dim3(RB), 0, st, a, l);
  switch (a.Fe) {
    case 0: DR_E8(0) break;
    case 1: DR_E8(1) break;
    case 2: DR_E8(2) break;
    case 3: DR_E8(3) break;
    default: DR_E8(4) break;
  }
#undef DR_E8
  return 1;
}

inline int rows_grid(int64_t rows, int rows_per_block) {
  int64_t g = (rows + rows_per_block - 1) / rows_per_block;
  if (g < 1) g = 1;
  if (g > 2048) g = 2048;  // grid-stride beyond 8 workgroups per CU
  return (int)g;
}

// ---- chunk-fused pipeline: tile == weight-gradient chunk == 64 rows ---------
// With a tile plan of DR_VANILLA_CHUNK rows (Fe <= 4, F <= 32), one
// 1024-thread workgroup per chunk runs every row-local stage of its rows
// around the halo edge work, so the node-level intermediates between them
// stay in LDS:
//   vc_fwd<l>  [A | B] = X [Wa; Wb]^T of its own rows and of its halo rows
//              (MFMA), edge gather -> S_l, node MLP X_l = relu([X | S_l] Wn^T
//              + bn) (vb_gemm<GM_HALVES> + vb_edge_fwd_tile + vb_gemm<GM_NODE>);
//   vc_nb2     DU2 = relu'(X2) dmean, [dX1 | DS2] = DU2 Wn2, dWn2 / dbn2
//              (vb_du + vb_gemm<GM_DXS> + vb_wgrad_mfma's Wn part);
//   vc_eb2n1   D2, D2' from the DS2 halo, dWa2 / dWb2 / dbe2 / dWc2,
//              dX1 += [D2 | D2'] [Wa2; Wb2], DU1 = relu'(X1) dX1, DS1 = DU1 Wn1,
//              dWn1 / dbn1 (vb_edge_bwd_tile + vb_gemm<GM_DX1> + vb_du +
//              vb_gemm<GM_DXS> + vb_wgrad_mfma, two layers);
//   vc_eb1     D1, D1' from the DS1 halo, dWa1 / dWb1 / dbe1 / dWc1;
//   vc_combine every graph's chunk partials of both layers, in chunk order.
// 7 launches per step instead of 17.  Every GEMM takes the operands and the k
// order of the kernel it replaces, and the sums run in the same order, so the
// outputs, slabs, head vectors and ReLU words are bit-identical to the untiled
// pipeline; only dWc sums its rows' shares in another order (as the 16-row
// tiles already did).
constexpr int CT = 1024;      // threads of the chunk kernels
__device__ __forceinline__ int vc_tile() { return xcd_tile(); }  // (graph_common.h)

constexpr int CW = CT / 64;   // waves
constexpr int CRG = CT / 32;  // row groups (32 lanes = the 32 channels of one row)

// diagnostic builds (-DDR_STAMPS): thread 0's s_memtime at phase i of chunk
// kernel k (0 vc_fwd<1>, 1 vc_fwd<2>, 2 vc_nb2, 3 vc_eb2n1, 4 vc_eb1) in
// dr_pass.stamps [5][n_tiles][16]
#ifdef DR_STAMPS
#define CSTAMP(k, i)                                                                                            \
  do {                                                                                                          \
    if (threadIdx.x == 0 && a.p.stamps)                                                                         \
      a.p.stamps[((int64_t)(k) * gridDim.x + blockIdx.x) * 16 + (i)] = (int64_t)__builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define CSTAMP(k, i) \
  do {               \
  } while (0)
#endif

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
}

// The chunk kernels' prologues issue every global load before the first LDS
// store (the tile's offsets come from one dr_vanilla_tile record), so staging
// costs about the halo's id -> row chain instead of one memory latency per
// array and per dependent index (measured: 35-48 % of a chunk workgroup's
// lifetime, profiles/r04/stamps_vchunk_atom.txt).  KPT items per thread go
// through registers; anything beyond (graphs past the measured sizes) takes a
// tail loop.
constexpr int KPT = 2;

// KPT (= 2) values per thread as two named registers: an array member indexed
// in an unrolled loop was left in scratch memory (and its store waited for the
// load it was meant to overlap)
template <class T>
struct P2 {
  T a, b;
  __device__ __forceinline__ T& operator[](int k) { return k ? b : a; }
  __device__ __forceinline__ const T& operator[](int k) const { return k ? b : a; }
};
__device__ __forceinline__ float& f4at(float4& v, int f) { return f == 0 ? v.x : (f == 1 ? v.y : (f == 2 ? v.z : v.w)); }

// A bounds-checked view of one tile's slice of an array (buffer resource,
// built from wave-uniform values): loads past `bytes` return 0 without
// touching memory, so the prologue's guarded loads need no branches -- the
// compiler then issues them all before the first wait instead of waiting
// at each branch join.
constexpr int OOB = 0x7ffffff0;  // a byte offset past every view
struct Buf {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ Buf(const void* base, int64_t bytes) {
    const uint64_t p = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p), hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    const int nb = __builtin_amdgcn_readfirstlane((int)(bytes < OOB ? bytes : OOB));
    r = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, nb, 0x00020000);
  }
  __device__ __forceinline__ float f32(int off) const { return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0)); }
  __device__ __forceinline__ uint32_t u32(int off) const { return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0); }
  __device__ __forceinline__ uint32_t u16(int off) const { return __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0); }
  __device__ __forceinline__ float4 f4(int off) const {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
  }
};

// a record {head, ea[0..FE)} from registers (put_rec's layout; FE <= 4)
template <int FE>
__device__ __forceinline__ void put_rec_v(float* rec, int e, uint32_t head, float4 ev) {
  constexpr int RS = TileRec<FE>::RS;
  *reinterpret_cast<float4*>(rec + e * RS) =
      make_float4(__uint_as_float(head), FE > 0 ? ev.x : 0.f, FE > 1 ? ev.y : 0.f, FE > 2 ? ev.z : 0.f);
  if (FE > 3) rec[e * RS + 4] = ev.w;
}
// edge p's FE attributes (zero past the view and past FE)
template <int FE>
__device__ __forceinline__ float4 ea_v(const Buf& ea, int p) {
  constexpr int FeS = FE > 0 ? FE : 1;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int f = 0; f < FE; ++f) f4at(v, f) = ea.f32((p * FeS + f) * 4);
  return v;
}

// rows [0, WR) of a row-major [rows][XS] array (XS <= 64: one float4 per
// thread of CT), rows >= nr zero; columns >= mask_f zeroed when mask_f > 0
struct RowsV {
  float4 v;
  int i, c4;
  __device__ __forceinline__ void load(const float* src, int XS, int nr, int mask_f) {
    const int CH = XS / 4;
    i = threadIdx.x / CH;
    c4 = (threadIdx.x - i * CH) * 4;
    const Buf b(src, (int64_t)nr * XS * 4);
    v = b.f4(i < WR ? (i * XS + c4) * 4 : OOB);
    mf = mask_f;
  }
  int mf;
  // (the mask is applied here, not at the load: a branch on the loaded value
  // there made the compiler wait for every load issued before it)
  __device__ __forceinline__ void store(float* dst, int LD) const {
    float4 w = v;
    if (mf > 0) {
      w.x = c4 < mf ? w.x : 0.f;
      w.y = c4 + 1 < mf ? w.y : 0.f;
      w.z = c4 + 2 < mf ? w.z : 0.f;
      w.w = c4 + 3 < mf ? w.w : 0.f;
    }
    if (i < WR) *reinterpret_cast<float4*>(dst + i * LD + c4) = w;
  }
};

// n entries of a staged weight layout: `off(p)` = the source element's float
// offset into the weight array (or -1: zero); KPT per thread in registers,
// the rest by a tail loop at store time
template <class Off, int NT = CT>
struct MapV {
  P2<float> v;
  __device__ __forceinline__ void load(const Buf& w, int n, Off off) {
#pragma unroll
    for (int k = 0; k < KPT; ++k) {
      const int p = threadIdx.x + k * NT;
      const int o = p < n ? off(p) : -1;
      v[k] = w.f32(o >= 0 ? o * 4 : OOB);
    }
  }
  __device__ __forceinline__ void store(float* dst, const Buf& w, int n, Off off) const {
#pragma unroll
    for (int k = 0; k < KPT; ++k) {
      const int p = threadIdx.x + k * NT;
      if (p < n) dst[p] = v[k];
    }
    #pragma unroll 1
    for (int p = threadIdx.x + KPT * NT; p < n; p += NT) {
      const int o = off(p);
      dst[p] = w.f32(o >= 0 ? o * 4 : OOB);
    }
  }
};
template <int NT = CT, class Off>
__device__ __forceinline__ MapV<Off, NT> map_load(const Buf& w, int n, Off off) {
  MapV<Off, NT> m;
  m.load(w, n, off);
  return m;
}

// a tile's halo rows of a node-level [rows][32] array (its graph's block g32,
// ng rows): the ids first (load_ids), the rows once they are in (load_rows),
// then store
struct HaloV {
  Buf ids, rows;
  const float* g32;
  int H;
  P2<int> id;
  P2<float4> v;
  __device__ __forceinline__ HaloV(const int* ids_, int H_, const float* g32_, int ng)
      : ids(ids_, (int64_t)H_ * 4), rows(g32_, (int64_t)ng * 128), g32(g32_), H(H_) {}
  // the rows straight into LDS (global_load_lds: no registers; the caller
  // waits vmcnt(0) before its barrier)
  __device__ __forceinline__ void dma(float* dst) const {
    const int wb = __builtin_amdgcn_readfirstlane(threadIdx.x & ~63);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
#pragma unroll
    for (int k = 0; k < KPT; ++k) {
      const int p = threadIdx.x + k * CT;
      if (p < H * 8)
        __builtin_amdgcn_global_load_lds(DRK_AS1(g32 + (int64_t)id[k] * 32 + (p & 7) * 4), DRK_AS3(d4 + wb + k * CT), 16, 0, 0);
    }
    for (int base = wb + KPT * CT; base < H * 8; base += CT) {
      const int p = base + (threadIdx.x & 63);
      if (p < H * 8)
        __builtin_amdgcn_global_load_lds(DRK_AS1(g32 + (int64_t)ids.u32((p >> 3) * 4) * 32 + (p & 7) * 4), DRK_AS3(d4 + base), 16, 0, 0);
    }
  }
  __device__ __forceinline__ void load_ids() {
#pragma unroll
    for (int k = 0; k < KPT; ++k) id[k] = (int)ids.u32(((threadIdx.x + k * CT) >> 3) * 4);
  }
  __device__ __forceinline__ void load_rows() {
#pragma unroll
    for (int k = 0; k < KPT; ++k) {
      const int p = threadIdx.x + k * CT;
      v[k] = rows.f4(p < H * 8 ? id[k] * 128 + (p & 7) * 16 : OOB);
    }
  }
  __device__ __forceinline__ void store(float* dst) const {
#pragma unroll
    for (int k = 0; k < KPT; ++k) {
      const int p = threadIdx.x + k * CT;
      if (p < H * 8) *reinterpret_cast<float4*>(dst + p * 4) = v[k];
    }
    #pragma unroll 1
    for (int p = threadIdx.x + KPT * CT; p < H * 8; p += CT)
      *reinterpret_cast<float4*>(dst + p * 4) = rows.f4((int)ids.u32((p >> 3) * 4) * 128 + (p & 7) * 16);
  }
};

struct BwdCarve {
  int LDD, LU, NOP3, d, w3, du, sh, halo, trec, x1, dx, x0, s1, w1, total;
};
// [D | D'] rows, (vc_eb2n1) [Wa2; Wb2] and DU1, the waves' dWc shares, then
// the edge phase's halo dS rows and transposed records {column, word} (the
// CSR records stay in registers).  After the edges the same space holds
// (vc_eb2n1) X1 / dX1 / X0 / S1 rows and Wn1[:, F:]^T, (vc_eb1) X0 rows.
__host__ __device__ inline BwdCarve bwd_carve(int F, int hmax, int emax, int tmax, int Fe, bool two_layers) {
  (void)emax;
  BwdCarve c;
  const int XS = r4(F), FeS = Fe > 0 ? Fe : 1;
  c.LDD = 64 + 4;  // [D | D'] rows
  c.LU = XS + 4;
  c.NOP3 = r16(F);
  int o = 0;
  c.d = o;  o += WR * c.LDD;
  c.w3 = o; o += two_layers ? 64 * c.NOP3 : 0;   // [Wa2; Wb2] [64][NOP3]
  c.du = o; o += two_layers ? WR * c.LU : 0;     // DU1
  c.sh = o; o += CW * 32 * FeS;                  // the waves' dWc shares
  c.halo = o;
  c.trec = o + hmax * 32;
  const int edge = hmax * 32 + 2 * tmax;
  c.x0 = o;
  c.x1 = c.x0 + WR * XS;  // vc_eb2n1 only, as the rest (vc_eb1: empty, at the end of X0)
  c.dx = two_layers ? c.x1 + WR * XS : c.x1;
  c.s1 = two_layers ? c.dx + WR * XS : c.x1;
  c.w1 = two_layers ? c.s1 + WR * 32 : c.x1;
  const int late = two_layers ? 3 * WR * XS + WR * 32 + XS * 32 : WR * XS;
  o += edge > late ? edge : late;
  c.total = o;
  return c;
}

struct FwdCarve {
  int HS, KP, LA, NOP, hp, xo, wab, halo, rec, a, wn, bn, x2, total;
};
// Edge phase: the halo's X rows (then, in place, their B = X Wb^T), the tile's
// own X rows (then, in place, A = X Wa^T), [Wa; Wb]^T and the CSR records.
// Once the edges are done the same space holds the node MLP's [X | S] rows,
// Wn^T and bn.  Rows at stride HS = 36 (the MFMA A-operand reads of 16 rows
// at stride 32 would hit two banks).
__host__ __device__ inline FwdCarve fwd_carve(int F, int hmax, int emax, int Fe) {
  FwdCarve c;
  const int XS = r4(F);
  c.HS = 36;
  c.KP = XS + 32;  // [X | S]
  c.LA = c.KP + 4;
  c.NOP = r16(F);
  c.hp = r16(hmax);  // halo rows rounded up to the MFMA's 16-row blocks
  int o = 0;
  c.xo = o;   o += WR * c.HS;       // own X rows -> A
  c.wab = o;  o += XS * 64;         // [Wa; Wb]^T [XS][64]
  c.halo = o; o += c.hp * c.HS;     // halo X rows -> B
  c.rec = o;  o += emax * (Fe <= 3 ? 4 : 8);  // CSR records {halo column, ea}
  const int edge = o;
  c.a = 0;                          // after the edges: [X | S] rows (node MLP A operand)
  c.wn = WR * c.LA;                 // Wn^T [KP][NOP]
  c.bn = c.wn + c.KP * c.NOP;       // bn, zero past F
  c.x2 = c.bn + c.NOP;              // layer 2: the output rows [64][33] for the tile's column sums
  const int late = c.x2 + WR * 33;
  c.total = edge > late ? edge : late;
  return c;
}

// [A | B] rows = X [Wa; Wb]^T in place over X rows at stride HS (vb_gemm<GM_HALVES>'s
// operands and k order; half 0 = A, 1 = B): rows [0, nrows) in 16-row blocks, a
// block's two 16-column tiles on one wave (its reads finish before its writes)
__device__ __forceinline__ void halves_in_place(float* sX, int HS, int nrows, const float* sW, int XS, int half, int job0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, kq = lane >> 4;
  const int nb = (nrows + 15) >> 4;
  for (int jb = (wave + CW - job0 % CW) % CW; jb < nb; jb += CW) {
    const int ib = jb * 16;
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    const int n0 = half * 32 + li, n1 = n0 + 16;
    for (int k0 = 0; k0 < XS; k0 += 4) {
      const float av = sX[(ib + li) * HS + k0 + kq];
      acc0 = mfma4(av, sW[(k0 + kq) * 64 + n0], acc0);
      acc1 = mfma4(av, sW[(k0 + kq) * 64 + n1], acc1);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = ib + kq * 4 + q;
      if (i < nrows) {
        sX[i * HS + li] = acc0[q];
        sX[i * HS + 16 + li] = acc1[q];
      }
    }
  }
}

// Layer l of the chunk-fused forward: [A | B] of the tile's rows and halo
// rows (MFMA, in LDS: the node-level A / B arrays and their GEMM launch are
// gone), the edge gather S_i = sum_e relu(A_i + B_j + Wc ea_e + be) with the
// ReLU words, then the node MLP X_l = relu([X | S_l] Wn^T + bn).
template <int FE, int LAYER>
__global__ void __launch_bounds__(CT, 8) vc_fwd(VA a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int FA = FE > 0 ? FE : 1, FeS = FA;
  const Layer L = layer_of(a, LAYER);
  const int F = a.F, KE = a.KE, KN = a.KN, XS = a.XS;
  const int tid = threadIdx.x, c = tid & 31, hs = tid & 32, g = tid >> 5;
  CSTAMP(LAYER - 1, 0);
  const int tile = vc_tile();
  const dr_vanilla_tile m = a.ws.tile_meta[tile];
  const int nr = m.nr, ne = m.ne, H = m.n_halo;
  const int64_t rt0 = m.rt0;
  const FwdCarve fc = fwd_carve(F, a.ws.halo_max, a.ws.tile_edges_max, FE);
  const int HS = fc.HS;
  float* sXo = lds + fc.xo;
  float* sWab = lds + fc.wab;
  float* sB = lds + fc.halo;
  float* sR = lds + fc.rec;
  // the layer's input rows: the store's x (layer 1) or X1 (layer 2); graph block xg
  const float* xg = LAYER == 1 ? a.s.x + (m.xrow - m.i0) * XS : L.xin + m.g0 * XS;
  // ---- prologue: every global load (bounds-checked views, no branches), the
  // halo ids first ----
  const Buf idv(a.ws.halo_ids + m.h0, (int64_t)H * 4);
  const Buf xgv(xg, (int64_t)m.n_graph * XS * 4);
  P2<int> hid;
#pragma unroll
  for (int k = 0; k < KPT; ++k) hid[k] = (int)idv.u32(((tid + k * CT) >> 3) * 4);
  const Buf rpv(a.s.rowptr + m.rp0 + m.i0, (int64_t)(nr + 1) * 4);  // the tile's rows' CSR bounds
  P2<int> rb, re;
#pragma unroll
  for (int k = 0; k < 2; ++k) {  // CRG == 32: row group g owns tile rows g and g + 32
    const int i = g + CRG * k;
    rb[k] = (int)rpv.u32(i * 4);
    re[k] = (int)rpv.u32((i + 1) * 4);
  }
  float wcr[FA];
#pragma unroll
  for (int f = 0; f < FE; ++f) wcr[f] = L.we[c * KE + 2 * F + f];
  const float bc = L.be[c];
  const int n_words = a.ws.edge0[a.B];
  const uint16_t* lc = a.ws.lcol + m.lcol_off;
  const float* ea = a.s.ea + (m.col0 + m.e0) * FeS;
  const Buf lcv(lc, (int64_t)ne * 2), eav(ea, (int64_t)ne * FeS * 4);
  P2<uint32_t> rh;
  P2<float4> rv;
#pragma unroll
  for (int k = 0; k < KPT; ++k) {
    const int p = tid + k * CT;
    rh[k] = lcv.u16(p * 2);
    rv[k] = ea_v<FE>(eav, p);
  }
  // own X rows: one float4 per thread (XS <= 32: WR * 8 pieces of 4 columns)
  const int oi = tid >> 3, oc = (tid & 7) * 4;
  const float4 xo = xgv.f4(oi < nr && oc < XS ? ((m.i0 + oi) * XS + oc) * 4 : OOB);
  const Buf wabv(L.we, (int64_t)32 * KE * 4);
  auto wab_off = [&](int p) -> int {  // vb_gemm<GM_HALVES>'s W staging
    const int k = p >> 6, n = p & 63;
    return k < F ? (n & 31) * KE + (n < 32 ? 0 : F) + k : -1;
  };
  const auto wab = map_load(wabv, XS * 64, wab_off);
  // halo X rows (8 pieces of 4 columns per row; the ids are in by now)
  P2<float4> hx;
#pragma unroll
  for (int k = 0; k < KPT; ++k) {
    const int p = tid + k * CT, q4 = (p & 7) * 4;
    hx[k] = xgv.f4(p < H * 8 && q4 < XS ? (hid[k] * XS + q4) * 4 : OOB);
  }
  // X rows' pad columns (>= F) read as zero (scratch rows leave them unwritten)
  auto mask4 = [&](float4 v, int c4) {
    if (c4 + 4 > F) {
      v.x = c4 < F ? v.x : 0.f;
      v.y = c4 + 1 < F ? v.y : 0.f;
      v.z = c4 + 2 < F ? v.z : 0.f;
      v.w = c4 + 3 < F ? v.w : 0.f;
    }
    return v;
  };
  // ---- LDS stores, in the order of the loads ----
#pragma unroll
  for (int k = 0; k < KPT; ++k) {
    const int p = tid + k * CT;
    if (p < ne) put_rec_v<FE>(sR, p, rh[k] * (HS * 4), rv[k]);  // the halo row's byte offset
  }
  if (oi < WR) *reinterpret_cast<float4*>(sXo + oi * HS + oc) = mask4(xo, oc);
  wab.store(sWab, wabv, XS * 64, wab_off);
#pragma unroll
  for (int k = 0; k < KPT; ++k) {
    const int p = tid + k * CT;
    if (p < H * 8) *reinterpret_cast<float4*>(sB + (p >> 3) * HS + (p & 7) * 4) = mask4(hx[k], (p & 7) * 4);
  }
  #pragma unroll 1
  for (int p = tid + KPT * CT; p < H * 8; p += CT) {
    const int q4 = (p & 7) * 4;
    const float4 v = xgv.f4(q4 < XS ? ((int)idv.u32((p >> 3) * 4) * XS + q4) * 4 : OOB);
    *reinterpret_cast<float4*>(sB + (p >> 3) * HS + q4) = mask4(v, q4);
  }
  #pragma unroll 1
  for (int p = tid + KPT * CT; p < ne; p += CT) put_rec<FE>(sR, p, lc[p] * (HS * 4), ea + (int64_t)p * FeS);
  __syncthreads();
  CSTAMP(LAYER - 1, 1);
  // ---- [A | B]: A of the own rows, B of the halo rows, in place ----
  halves_in_place(sXo, HS, WR, sWab, XS, 0, 0);
  halves_in_place(sB, HS, H, sWab, XS, 1, WR / 16);
  // (the node MLP's operands, loaded now: they land during the edge phase)
  const float4 xa = mask4(xo, oc);
  const Buf wnv(L.wn, (int64_t)F * KN * 4);
  const int KP = fc.KP, NOP = fc.NOP;
  auto wn_off = [&](int p) -> int {  // vb_gemm<GM_NODE>'s W staging
    const int k = p / NOP, n = p - k * NOP;
    if (n >= F || (k >= F && k < XS)) return -1;
    return n * KN + (k < F ? k : F + k - XS);
  };
  const auto wn = map_load(wnv, KP * NOP, wn_off);
  const Buf bnb(L.bn, (int64_t)F * 4);
  const float bnv = bnb.f32(tid < F ? tid * 4 : OOB);
  __syncthreads();
  CSTAMP(LAYER - 1, 2);
  // ---- edge gather ----
  uint32_t* wr = a.ws.relu_words + (int64_t)(LAYER - 1) * n_words + m.word0 + m.e0;
  P2<float> sacc{0.f, 0.f};
  const char* sBc = reinterpret_cast<const char*>(sB + c);  // + a record's byte offset = B[j][c]
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = g + CRG * k;
    if (i >= nr) break;
    const float abk = sXo[i * HS + c] + bc;
    float acc = 0.f;
    const int ee = re[k] - m.e0;
    int e = rb[k] - m.e0;
    auto group = [&](auto un) {
      constexpr int U = decltype(un)::value;
      uint32_t j[U];
      float ev[U][FA], q[U];
#pragma unroll
      for (int u = 0; u < U; ++u) j[u] = get_rec<FE>(sR, e + u, ev[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) q[u] = *reinterpret_cast<const float*>(sBc + j[u]);
      uint32_t mine = 0u;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float pre = abk + q[u];
#pragma unroll
        for (int f = 0; f < FE; ++f) pre = fmaf(wcr[f], ev[u][f], pre);
        acc += relu_keepnan(pre);
        const uint64_t mm = __ballot(active(pre));
        if (c == u) mine = (uint32_t)(mm >> hs);
      }
      if (c < U) wr[e + c] = mine;
    };
    // (8 edges in flight for FE <= 1; 4 above, within the 64 VGPRs of two
    // workgroups per CU)
    if (FE <= 1)
      for (; e + 8 <= ee; e += 8) group(std::integral_constant<int, 8>());
    for (; e + 4 <= ee; e += 4) group(std::integral_constant<int, 4>());
    for (; e < ee; ++e) group(std::integral_constant<int, 1>());
    L.s[(rt0 + i) * 32 + c] = acc;
    sacc[k] = acc;
  }
  __syncthreads();
  CSTAMP(LAYER - 1, 3);
  // ---- node MLP: [X | S] rows, Wn^T and bn into the dead edge space ----
  float* sA = lds + fc.a;
  float* sWn = lds + fc.wn;
  float* sBn = lds + fc.bn;
  if (oi < WR && oc < XS) *reinterpret_cast<float4*>(sA + oi * fc.LA + oc) = xa;
#pragma unroll
  for (int k = 0; k < 2; ++k) sA[(g + CRG * k) * fc.LA + XS + c] = g + CRG * k < nr ? sacc[k] : 0.f;
  wn.store(sWn, wnv, KP * NOP, wn_off);
  if (tid < NOP) sBn[tid] = bnv;
  __syncthreads();
  // vb_gemm<GM_NODE>'s operands and k order
  const int lane = tid & 63, wave = tid >> 6, li = lane & 15, kq = lane >> 4;
  const int nct = NOP / 16;
  for (int job = wave; job < 4 * nct; job += CW) {
    const int ib = (job / nct) * 16, n = (job % nct) * 16 + li;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < KP; k0 += 4) acc = mfma4(sA[(ib + li) * fc.LA + k0 + kq], sWn[(k0 + kq) * NOP + n], acc);
    const float bn = sBn[n];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = ib + kq * 4 + q;
      const float v = relu_keepnan(acc[q] + bn);
      if (i < nr && n < F) L.xout[(rt0 + i) * XS + n] = v;
      if (LAYER == 2 && n < F) lds[fc.x2 + i * 33 + n] = v;
    }
  }
  if (LAYER == 2 && a.ws.part_mean) {  // the tile's column sums for the mean (vb_head's order)
    __syncthreads();
    if (tid < F) {
      float t = 0.f;
      for (int i = 0; i < nr; ++i) t += lds[fc.x2 + i * 33 + tid];
      a.ws.part_mean[(int64_t)tile * 32 + tid] = t;
    }
  }
  CSTAMP(LAYER - 1, 4);
}

// weight-gradient partial row of a layer for a chunk (both layers' rows live together)
__device__ __forceinline__ float* part_row(const VA& a, int l, int ch) {
  return a.ws.part + ((int64_t)(l - 1) * a.ws.n_chunks + ch) * r4(layer_grad_size(a.F, a.Fe));  // rows at 16 bytes (vc_combine)
}

// dWn = DU^T [X | S] (K = the chunk's 64 rows, zero past it) and dbn = sum DU:
// vb_wgrad_mfma's jobs and order.  DU at stride LU, X at stride XS, S at 32.
template <int NT>
__device__ __forceinline__ void node_wgrad(const VA& a, float* out, const float* sDU, int LU, const float* sX, const float* sS, int job0) {
  const int F = a.F, XS = a.XS, KN = a.KN, KE = a.KE;
  const int nwe = 32 * KE, nwn = F * KN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, kq = lane >> 4;
  const int KT = (F + 15) >> 4, QT = (KN + 15) >> 4;
  for (int jj = (wave + NT / 64 - job0 % (NT / 64)) % (NT / 64); jj < KT * QT; jj += NT / 64) {
    const int nt = jj / QT, qt = jj - nt * QT;
    const int nn = nt * 16 + li, qc = qt * 16 + li;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < WR; i += 4) {
      const float av = nn < XS ? sDU[(i + kq) * LU + nn] : 0.f;
      const float bv = qc < F ? sX[(i + kq) * XS + qc] : (qc < KN ? sS[(i + kq) * 32 + qc - F] : 0.f);
      acc = mfma4(av, bv, acc);
    }
    if (qc < KN) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = nt * 16 + kq * 4 + q;
        if (n < F) out[nwe + 32 + n * KN + qc] = acc[q];
      }
    }
  }
  for (int p0 = threadIdx.x; p0 < 4 * F; p0 += NT) {  // dbn: four lanes of 16 rows, combined in order
    const int p = p0 >> 2, ib = (p0 & 3) * (WR / 4);
    float v = 0.f;
#pragma unroll
    for (int u = 0; u < WR / 4; ++u) v += sDU[(ib + u) * LU + p];
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    if ((p0 & 3) == 0) out[nwe + 32 + nwn + p] = v;
  }
}

constexpr int NB2 = 512;  // vc_nb2 threads: 4 workgroups per CU

__global__ void __launch_bounds__(NB2, 8) vc_nb2(VA a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int F = a.F, XS = a.XS, KN = a.KN;
  const int tid = threadIdx.x;
  CSTAMP(2, 0);
  const int tile = vc_tile();
  const dr_vanilla_tile m = a.ws.tile_meta[tile];
  const int64_t rt0 = m.rt0;
  const int nr = m.nr;
  const int LU = XS + 4, NOPD = r16(F + 32);
  float* sDU = lds;
  float* sX1 = sDU + WR * LU;
  float* sS = sX1 + WR * XS;
  float* sW = sS + WR * 32;
  float* ws = a.ws.base;
  const int hrow = a.p.slot ? a.p.slot[m.slot] : m.slot;
  RowsV x2, x1, s2;
  x2.load(ws + a.L.x2 + rt0 * XS, XS, nr, 0);
  x1.load(ws + a.L.x1 + rt0 * XS, XS, nr, 0);
  s2.load(ws + a.L.s2 + rt0 * 32, 32, nr, 0);
  const Buf wb(a.w.wn2, (int64_t)F * KN * 4);
  auto w_off = [&](int p) -> int {  // vb_gemm<GM_DXS>'s W staging (Wn2)
    const int k = p / NOPD, n = p - k * NOPD;
    return (k < F && n < F + 32) ? k * KN + n : -1;
  };
  // XS * NOPD <= 2048 weights (F <= 32): two register batches of 2 x NB2
  const auto w = map_load<NB2>(wb, XS * NOPD, w_off);
  auto w_off2 = [&](int p) -> int { return w_off(p + 2 * NB2); };
  const auto w2 = map_load<NB2>(wb, XS * NOPD - 2 * NB2, w_off2);
  const int HD = XS + 256 + r4(a.p.out_dim);
  const Buf dmb(a.p.head + (int64_t)hrow * DR_VANILLA_HEAD_STRIDE(F, a.p.out_dim) + HD, (int64_t)F * 4);
  float dm[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) dm[q] = dmb.f32((x2.c4 + q) * 4);
  // DU2 = relu'(X2) dmean (vb_du, layer 2): zero past the tile's rows and past F
  float4 du = make_float4(0.f, 0.f, 0.f, 0.f);
  if (x2.i < nr) {
    du.x = x2.c4 < F ? relu_bwd(x2.v.x, dm[0]) : 0.f;
    du.y = x2.c4 + 1 < F ? relu_bwd(x2.v.y, dm[1]) : 0.f;
    du.z = x2.c4 + 2 < F ? relu_bwd(x2.v.z, dm[2]) : 0.f;
    du.w = x2.c4 + 3 < F ? relu_bwd(x2.v.w, dm[3]) : 0.f;
  }
  if (x2.i < WR) *reinterpret_cast<float4*>(sDU + x2.i * LU + x2.c4) = du;
  x1.store(sX1, XS);
  s2.store(sS, 32);
  w.store(sW, wb, min(XS * NOPD, 2 * NB2), w_off);
  w2.store(sW + 2 * NB2, wb, XS * NOPD - 2 * NB2, w_off2);
  __syncthreads();
  CSTAMP(2, 1);
  const int lane = tid & 63, wave = tid >> 6, li = lane & 15, kq = lane >> 4;
  const int nct = NOPD / 16;
  for (int job = wave; job < 4 * nct; job += NB2 / 64) {  // [dX1 | DS2] = DU2 Wn2
    const int ib = (job / nct) * 16, n = (job % nct) * 16 + li;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < XS; k0 += 4) acc = mfma4(sDU[(ib + li) * LU + k0 + kq], sW[(k0 + kq) * NOPD + n], acc);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = ib + kq * 4 + q;
      if (i >= nr) continue;
      if (n < F) ws[a.L.dx1 + (rt0 + i) * XS + n] = acc[q];
      else if (n < F + 32) ws[a.L.ds + (rt0 + i) * 32 + n - F] = acc[q];
    }
  }
  node_wgrad<NB2>(a, part_row(a, 2, tile), sDU, LU, sX1, sS, 4 * nct);
  CSTAMP(2, 2);
}

// A chunk's D_i = relu'-count x dS_i, D'_i (transposed) and its rows' dWc
// shares from the halo of dS rows (vb_edge_bwd_tile's sums and order).  A
// row's CSR records {word, ea} go straight to registers (lane c of its row
// group holds edge c of the row; ds_bpermute hands edge u to the group), so
// only the halo rows and the transposed records take LDS.  The caller
// interleaves: load1 (ids, row bounds), its own loads, load2 (halo rows,
// records), load3 (transposed words), store, its stores, a barrier, run.
template <int FE>
struct EdgeBwd {
  static constexpr int FA = FE > 0 ? FE : 1, FeS = FA;
  static constexpr bool MF = FE <= 3;  // cnt / eap on MFMA (part1_mfma) in half the waves; FE = 4: the VALU pass
  // The MFMA pass is bound by the fp32 MFMA pipe and the VALU pass by VALU /
  // LDS issue, so the waves split: on every SIMD (waves w, w + 4, w + 8,
  // w + 12) two take each pass, and the two pipes work side by side
  __device__ __forceinline__ static bool mf_wave() { return MF && ((threadIdx.x >> 8) & 1); }
  const dr_vanilla_tile& m;
  const uint32_t* words;  // the graph's ReLU words of layer l
  const float* ea;
  const uint16_t* lt;
  const int* teid;
  HaloV halo;
  Buf wv, eav, ltv, tev, wgv, rpv, trpv, dsv;
  P2<uint32_t> tc, tw;
  P2<int> te;
  P2<int> rb, re, qb, qe;
  P2<float> dsi;
  P2<uint32_t> rw;  // row k's edge c (the first 32 of the row)
  P2<float4> rv;

  __device__ __forceinline__ EdgeBwd(const VA& a, const dr_vanilla_tile& mm, int l, const float* ds)
      : m(mm),
        words(a.ws.relu_words + (int64_t)(l - 1) * a.ws.edge0[a.B] + mm.word0),
        ea(a.s.ea + (mm.col0 + mm.e0) * FeS),
        lt(a.ws.ltcol + mm.ltcol_off),
        teid(a.s.t_eid + mm.col0 + mm.q0),
        halo(a.ws.halo_ids + mm.h0, mm.n_halo, ds + mm.g0 * 32, mm.n_graph),
        wv(words + mm.e0, (int64_t)mm.ne * 4),
        eav(ea, (int64_t)mm.ne * FeS * 4),
        ltv(lt, (int64_t)mm.nq * 2),
        tev(teid, (int64_t)mm.nq * 4),
        wgv(words, (int64_t)mm.e_graph * 4),
        rpv(a.s.rowptr + mm.rp0 + mm.i0, (int64_t)(mm.nr + 1) * 4),
        trpv(a.s.t_rowptr + mm.rp0 + mm.i0, (int64_t)(mm.nr + 1) * 4),
        dsv(ds + mm.rt0 * 32, (int64_t)mm.nr * 128) {}

  // edge p's (tile-local CSR slot) record, or zeros when !ok
  __device__ __forceinline__ void rec_at(int p, bool ok, uint32_t& w, float4& v) const {
    const int o = ok ? p * 4 : OOB;
    w = wv.u32(o);
    const int oe = ok ? p * FeS * 4 : OOB;
    v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int f = 0; f < FE; ++f) f4at(v, f) = eav.f32(oe + 4 * f);
  }

  __device__ __forceinline__ void load1() {
    const int tid = threadIdx.x, c = tid & 31, g = tid >> 5;
    halo.load_ids();
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = g + CRG * k;
      rb[k] = (int)rpv.u32(i * 4);
      re[k] = (int)rpv.u32((i + 1) * 4);
      qb[k] = (int)trpv.u32(i * 4);
      qe[k] = (int)trpv.u32((i + 1) * 4);
      dsi[k] = dsv.f32((i * 32 + c) * 4);
    }
#pragma unroll
    for (int k = 0; k < KPT; ++k) {
      const int p = tid + k * CT;
      tc[k] = ltv.u16(p * 2);
      te[k] = (int)tev.u32(p * 4);
    }
  }
  __device__ __forceinline__ void load2(float* sDS) {
    const int c = threadIdx.x & 31;
    halo.dma(sDS);
    if (!mf_wave()) {
#pragma unroll
      for (int k = 0; k < 2; ++k) rec_at(rb[k] - m.e0 + c, c < re[k] - rb[k], rw[k], rv[k]);
    }
  }
  // cnt_i and eap_i of the wave's four rows (2w, 2w + 1, 2w + 32, 2w + 33) on
  // MFMA: C[c][4r + s] = sum over row r's edges e of bit_c(w_e) * [ea_e | 1][s]
  // (A = the edges' ReLU bits, 16 channels x 4 edges per step; B = each
  // edge's attributes and a one in its row's four columns), so a step takes 4
  // edges for all 32 channels instead of one edge per row group.  The counts
  // are exact (sums of ones); D_i = dS_i cnt_i as in the VALU pass, and the
  // dWc share sum_i dS_i eap_i in another order (fp32 tolerance, like the
  // tiles' dWc).  Then D rows into sD and the wave's dWc share into sSh.
  __device__ __forceinline__ void part1_mfma(float* sD, int LDD, float* sSh) const {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, chl = lane & 15, kq = lane >> 4;
    const int sn = lane & 3, rn = (lane >> 2) & 3;  // this lane's B / C column: row rn, slot sn (3: the count)
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int rowA = 2 * wave + CRG * kk;
      if (rowA >= m.nr) break;
      // rows A = rowA and rowA + 1 are consecutive CSR rows: [sA, mA), [mA, eB)
      const int sA = __builtin_amdgcn_readlane(rb[kk], 0), mA = __builtin_amdgcn_readlane(re[kk], 0);
      const int eB = rowA + 1 < m.nr ? __builtin_amdgcn_readlane(re[kk], 32) : mA;
      // two steps (8 edges) per iteration, their loads issued together; a
      // step past the rows reads zeros and adds nothing
      for (int j0 = sA; j0 < eB; j0 += 8) {
        uint32_t w[2];
        float ev[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int jj = j0 + 4 * u + kq, p = jj - m.e0;
          const bool ok = jj < eB;
          w[u] = wv.u32(ok ? p * 4 : OOB);
          ev[u] = eav.f32(ok && sn < FE ? (p * FeS + sn) * 4 : OOB);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int jj = j0 + 4 * u + kq;
          const int r = 2 * kk + (jj < mA ? 0 : 1);
          const float bv = (jj < eB && r == rn) ? (sn == 3 ? 1.f : ev[u]) : 0.f;
          acc0 = mfma4(edge_bit(w[u], chl), bv, acc0);
          acc1 = mfma4(edge_bit(w[u], chl + 16), bv, acc1);
        }
      }
    }
    // lane: C[channel kq * 4 + q (+ 16)][row rn, slot sn]
    const int li = 2 * wave + (rn & 1) + CRG * (rn >> 1);  // the tile row of column group rn
    float ds[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int q = 0; q < 4; ++q) ds[h][q] = dsv.f32(li < m.nr ? (li * 32 + kq * 4 + q + 16 * h) * 4 : OOB);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ch = kq * 4 + q + 16 * h;
        const float v = h ? acc1[q] : acc0[q];
        // the row's count, from the quad's slot-3 lane
        const float cnt = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xFF, 0xF, 0xF, false));
        if (sn == 3) sD[li * LDD + ch] = cnt != 0.f ? ds[h][q] * cnt : 0.f;
        if constexpr (FE > 0) {
          float sh = (sn < FE && cnt != 0.f) ? ds[h][q] * v : 0.f;
          sh += __shfl_xor(sh, 4, 64);  // the wave's four rows
          sh += __shfl_xor(sh, 8, 64);
          if (rn == 0 && sn < FE) sSh[(wave * 32 + ch) * FeS + sn] = sh;
        }
      }
  }
  __device__ __forceinline__ void load3() {
#pragma unroll
    for (int k = 0; k < KPT; ++k) tw[k] = wgv.u32(threadIdx.x + k * CT < m.nq ? te[k] * 4 : OOB);
  }
  __device__ __forceinline__ void store(uint2* sTR, float* sD, int LDD) const {
    const int tid = threadIdx.x;
    #pragma unroll 1
    for (int p = tid; p < (WR - m.nr) * 64; p += CT) sD[(m.nr + (p >> 6)) * LDD + (p & 63)] = 0.f;
#pragma unroll
    for (int k = 0; k < KPT; ++k) {
      const int p = tid + k * CT;
      if (p < m.nq) sTR[p] = make_uint2(tc[k] * 128, tw[k]);  // the halo row's byte offset
    }
    #pragma unroll 1
    for (int p = tid + KPT * CT; p < m.nq; p += CT) sTR[p] = make_uint2(lt[p] * 128u, words[teid[p]]);
  }
  __device__ __forceinline__ void run(const VA& a, int sk, float* sD, int LDD, const float* sDS, const uint2* sTR, float* sSh) const {
    (void)a;
    (void)sk;
    const int tid = threadIdx.x, c = tid & 31, g = tid >> 5, hs = tid & 32;
    const bool mfw = mf_wave();
    if (mfw) part1_mfma(sD, LDD, sSh);
    CSTAMP(sk, 8);  // (stamps build: the end of the counts pass)
    float wsum[FA];
#pragma unroll
    for (int f = 0; f < FA; ++f) wsum[f] = 0.f;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int li = g + CRG * k;
      if (li >= m.nr) break;
      if (!mfw) {
      float cnt = 0.f;
      float eap[FA];
#pragma unroll
      for (int f = 0; f < FA; ++f) eap[f] = 0.f;
      const int deg = re[k] - rb[k];
      uint32_t w_r = rw[k];
      float4 v_r = rv[k];
      // the row's edges in order, 32 at a time from the lanes of the row group
      auto edge = [&](int u) {
        const int src = (hs + u) << 2;
        const uint32_t w = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)w_r);
        float ev[FA];
#pragma unroll
        for (int f = 0; f < FE; ++f) ev[f] = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(f4at(v_r, f))));
        const float bit = edge_bit(w, c);
        cnt += bit;
#pragma unroll
        for (int f = 0; f < FE; ++f) eap[f] = fmaf(bit, ev[f], eap[f]);
      };
      for (int base = 0; base < deg; base += 32) {
        if (base > 0) rec_at(rb[k] - m.e0 + base + c, base + c < deg, w_r, v_r);  // degree > 32
        const int n = min(32, deg - base);
        for (int u = 0; u < n; ++u) edge(u);
      }
      sD[li * LDD + c] = cnt != 0.f ? dsi[k] * cnt : 0.f;
#pragma unroll
      for (int f = 0; f < FE; ++f) wsum[f] += cnt != 0.f ? dsi[k] * eap[f] : 0.f;
      }
      float acc = 0.f;
      const char* sDSc = reinterpret_cast<const char*>(sDS + c);  // + a record's byte offset = dS[j][c]
      const int qe_ = qe[k] - m.q0;
      int q = qb[k] - m.q0;
      for (; q + 4 <= qe_; q += 4) {
        uint2 tr[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) tr[u] = sTR[q + u];
        float dv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) dv[u] = *reinterpret_cast<const float*>(sDSc + tr[u].x);
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if ((tr[u].y >> c) & 1u) acc += dv[u];
      }
      for (; q < qe_; ++q) {
        const uint2 tr = sTR[q];
        if ((tr.y >> c) & 1u) acc += *reinterpret_cast<const float*>(sDSc + tr.x);
      }
      sD[li * LDD + 32 + c] = acc;
    }
    // each wave's share of dWc (its two row groups summed), combined over the
    // waves in order by the caller
    if (!mfw)
#pragma unroll
    for (int f = 0; f < FE; ++f) {
      const float v = wsum[f] + __shfl_xor(wsum[f], 32, 64);
      if (tid < 64 * CW && (tid & 63) < 32) sSh[((tid >> 6) * 32 + c) * FeS + f] = v;
    }
  }
};

// dWa = D^T X, dWb = D'^T X, dbe = sum D, dWc = the waves' shares in order
// (vb_wgrad_mfma's jobs and order for the first three)
template <int FE>
__device__ __forceinline__ void edge_wgrad(const VA& a, float* out, const float* sD, int LDD, const float* sX, const float* sSh) {
  constexpr int FeS = FE > 0 ? FE : 1;
  const int F = a.F, XS = a.XS, KE = a.KE;
  const int nwe = 32 * KE;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, kq = lane >> 4;
  const int KT = (F + 15) >> 4, jw = 2 * 2 * KT;
  for (int job = wave; job < jw; job += CW) {
    const int w = job / (2 * KT), rem = job - w * 2 * KT, ct = rem / KT, kt = rem - ct * KT;
    const int cc = ct * 16 + li, kc = kt * 16 + li;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < WR; i += 4) acc = mfma4(sD[(i + kq) * LDD + w * 32 + cc], kc < XS ? sX[(i + kq) * XS + kc] : 0.f, acc);
    if (kc < F) {
#pragma unroll
      for (int q = 0; q < 4; ++q) out[(ct * 16 + kq * 4 + q) * KE + w * F + kc] = acc[q];
    }
  }
  const int tid = threadIdx.x;
  const int p0 = tid - (CT - 4 * 32);  // the last 128 threads: dbe, four lanes of 16 rows each
  if (p0 >= 0) {
    const int cch = p0 >> 2, ib = (p0 & 3) * (WR / 4);
    float v = 0.f;
#pragma unroll
    for (int u = 0; u < WR / 4; ++u) v += sD[(ib + u) * LDD + cch];
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    if ((p0 & 3) == 0) out[nwe + cch] = v;
  }
  if (tid < 32 * FE) {  // dWc [32][Fe]
    const int cch = tid / FeS, f = tid - cch * FeS;
    float v = 0.f;
    for (int w = 0; w < CW; ++w) v += sSh[(w * 32 + cch) * FeS + f];
    out[cch * KE + 2 * F + f] = v;
  }
}

template <int FE>
__global__ void __launch_bounds__(CT, 8) vc_eb2n1(VA a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int F = a.F, XS = a.XS, KE = a.KE, KN = a.KN;
  const int t = vc_tile(), tid = threadIdx.x;
  CSTAMP(3, 0);
  const dr_vanilla_tile m = a.ws.tile_meta[t];
  const int64_t rt0 = m.rt0;
  const int nr = m.nr;
  const BwdCarve bc = bwd_carve(F, a.ws.halo_max, a.ws.tile_edges_max, a.ws.tile_tedges_max, FE, true);
  float* sD = lds + bc.d;
  float* sW3 = lds + bc.w3;
  float* sDU = lds + bc.du;
  float* sSh = lds + bc.sh;
  float* ws = a.ws.base;
  EdgeBwd<FE> eb(a, m, 2, ws + a.L.ds);
  eb.load1();
  const int NOP3 = bc.NOP3;
  const Buf w3b(a.w.we2, (int64_t)32 * KE * 4);
  auto w3_off = [&](int p) -> int {  // vb_gemm<GM_DX1>'s W staging
    const int k = p / NOP3, n = p - k * NOP3;
    return n < F ? (k & 31) * KE + (k < 32 ? 0 : F) + n : -1;
  };
  const auto w3 = map_load(w3b, 64 * NOP3, w3_off);
  eb.load2(lds + bc.halo);
  eb.load3();
  w3.store(sW3, w3b, 64 * NOP3, w3_off);
  eb.store(reinterpret_cast<uint2*>(lds + bc.trec), sD, bc.LDD);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the halo DMA
  __syncthreads();
  CSTAMP(3, 1);
  eb.run(a, 3, sD, bc.LDD, lds + bc.halo, reinterpret_cast<const uint2*>(lds + bc.trec), sSh);
  __syncthreads();
  CSTAMP(3, 2);
  // X1 / dX1 / X0 / S1 rows (DMA) and Wn1's DS columns into the dead edge space
  float* sX1 = lds + bc.x1;
  float* sDX = lds + bc.dx;
  float* sX0 = lds + bc.x0;
  float* sS1 = lds + bc.s1;
  float* sW1 = lds + bc.w1;
  dma_x4<CT>(sX1, ws + a.L.x1 + rt0 * XS, nr * XS / 4);
  dma_x4<CT>(sDX, ws + a.L.dx1 + rt0 * XS, nr * XS / 4);
  dma_x4<CT>(sX0, a.s.x + m.xrow * XS, nr * XS / 4);
  dma_x4<CT>(sS1, ws + a.L.s1 + rt0 * 32, nr * 8);
  const Buf w1b(a.w.wn1, (int64_t)F * KN * 4);
  auto w1_off = [&](int p) -> int {  // vb_gemm<GM_DXS>'s W staging (Wn1), the DS columns
    const int k = p >> 5, n = p & 31;
    return k < F ? k * KN + F + n : -1;
  };
  const auto w1 = map_load(w1b, XS * 32, w1_off);
  #pragma unroll 1
  for (int p = tid; p < (WR - nr) * XS; p += CT) {
    sX1[nr * XS + p] = 0.f;
    sDX[nr * XS + p] = 0.f;
    sX0[nr * XS + p] = 0.f;
  }
  #pragma unroll 1
  for (int p = tid; p < (WR - nr) * 32; p += CT) sS1[nr * 32 + p] = 0.f;
  w1.store(sW1, w1b, XS * 32, w1_off);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  CSTAMP(3, 3);
  edge_wgrad<FE>(a, part_row(a, 2, t), sD, bc.LDD, sX1, sSh);
  // dX1 = dX1 + [D | D'] [Wa2; Wb2] (vb_gemm<GM_DX1>), then DU1 = relu'(X1) dX1 (vb_du)
  const int lane = tid & 63, wave = tid >> 6, li = lane & 15, kq = lane >> 4;
  const int nct = NOP3 / 16;
  for (int job = (wave + CW - 8 % CW) % CW; job < 4 * nct; job += CW) {
    const int ib = (job / nct) * 16, n = (job % nct) * 16 + li;
    floatx4 acc;
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = n < F ? sDX[(ib + kq * 4 + q) * XS + n] : 0.f;
    for (int k0 = 0; k0 < 64; k0 += 4) acc = mfma4(sD[(ib + li) * bc.LDD + k0 + kq], sW3[(k0 + kq) * NOP3 + n], acc);
    if (n < XS) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = ib + kq * 4 + q;
        sDU[i * bc.LU + n] = n < F ? relu_bwd(sX1[i * XS + n], acc[q]) : 0.f;
      }
    }
  }
  __syncthreads();
  CSTAMP(3, 4);
  // DS1 = DU1 Wn1[:, F:] (vb_gemm<GM_DXS> layer 1) and layer 1's dWn / dbn
  for (int job = wave; job < 8; job += CW) {
    const int ib = (job >> 1) * 16, n = (job & 1) * 16 + li;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < XS; k0 += 4) acc = mfma4(sDU[(ib + li) * bc.LU + k0 + kq], sW1[(k0 + kq) * 32 + n], acc);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = ib + kq * 4 + q;
      if (i < nr) ws[a.L.d + (rt0 + i) * 32 + n] = acc[q];
    }
  }
  node_wgrad<CT>(a, part_row(a, 1, t), sDU, bc.LU, sX0, sS1, 8);
  CSTAMP(3, 5);
}

template <int FE>
__global__ void __launch_bounds__(CT, 8) vc_eb1(VA a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int F = a.F, XS = a.XS;
  const int t = vc_tile(), tid = threadIdx.x;
  CSTAMP(4, 0);
  const dr_vanilla_tile m = a.ws.tile_meta[t];
  const int nr = m.nr;
  const BwdCarve bc = bwd_carve(F, a.ws.halo_max, a.ws.tile_edges_max, a.ws.tile_tedges_max, FE, false);
  float* sD = lds + bc.d;
  EdgeBwd<FE> eb(a, m, 1, a.ws.base + a.L.d);
  eb.load1();
  eb.load2(lds + bc.halo);
  eb.load3();
  eb.store(reinterpret_cast<uint2*>(lds + bc.trec), sD, bc.LDD);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the halo DMA
  __syncthreads();
  CSTAMP(4, 1);
  eb.run(a, 4, sD, bc.LDD, lds + bc.halo, reinterpret_cast<const uint2*>(lds + bc.trec), lds + bc.sh);
  __syncthreads();
  CSTAMP(4, 2);
  float* sX0 = lds + bc.x0;  // X0 rows into the dead edge space
  dma_x4<CT>(sX0, a.s.x + m.xrow * XS, nr * XS / 4);
  #pragma unroll 1
  for (int p = tid; p < (WR - nr) * XS; p += CT) sX0[nr * XS + p] = 0.f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  edge_wgrad<FE>(a, part_row(a, 1, t), sD, bc.LDD, sX0, lds + bc.sh);
  CSTAMP(4, 3);
}

// both layers' chunk partials per graph, in chunk order (vb_wgrad_combine x 2):
// four consecutive entries per thread (16-byte loads; part rows at stride
// r4(total)), 16 chunks' loads in flight
__global__ void __launch_bounds__(RB) vc_combine(VA a) {
  const int total = layer_grad_size(a.F, a.Fe), PS = r4(total), P4 = PS / 4;
  const int64_t work = (int64_t)a.B * 2 * P4;
  for (int64_t q = blockIdx.x * (int64_t)RB + threadIdx.x; q < work; q += (int64_t)gridDim.x * RB) {
    const int b = (int)(q / (2 * P4)), rem = (int)(q - (int64_t)b * 2 * P4), lay = rem / P4, p = (rem - lay * P4) * 4;
    const float* part = a.ws.part + (int64_t)lay * a.ws.n_chunks * PS + p;
    const int ce = a.ws.chunk_first[b + 1];
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    int ch = a.ws.chunk_first[b];
    for (; ch + 16 <= ce; ch += 16) {
      float4 u[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) u[k] = *reinterpret_cast<const float4*>(part + (int64_t)(ch + k) * PS);
#pragma unroll
      for (int k = 0; k < 16; ++k) v = f4add(v, u[k]);
    }
    for (; ch + 4 <= ce; ch += 4) {
      float4 u[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) u[k] = *reinterpret_cast<const float4*>(part + (int64_t)(ch + k) * PS);
#pragma unroll
      for (int k = 0; k < 4; ++k) v = f4add(v, u[k]);
    }
    for (; ch < ce; ++ch) v = f4add(v, *reinterpret_cast<const float4*>(part + (int64_t)ch * PS));
    float* dst = a.p.slab + (int64_t)(a.p.slot ? a.p.slot[b] : b) * DR_VANILLA_SLAB_STRIDE(a.F, a.Fe) + (int64_t)lay * total + p;
    if (p < total) dst[0] = v.x;
    if (p + 1 < total) dst[1] = v.y;
    if (p + 2 < total) dst[2] = v.z;
    if (p + 3 < total) dst[3] = v.w;
  }
}

inline bool chunk_carves(const dr_vanilla_scratch* sc, int F, int Fe, int64_t* fwd1, int64_t* fwd2, int64_t* eb2, int64_t* eb1) {
  *fwd1 = *fwd2 = 4LL * fwd_carve(F, sc->halo_max, sc->tile_edges_max, Fe).total;
  *eb2 = 4LL * bwd_carve(F, sc->halo_max, sc->tile_edges_max, sc->tile_tedges_max, Fe, true).total;
  *eb1 = 4LL * bwd_carve(F, sc->halo_max, sc->tile_edges_max, sc->tile_tedges_max, Fe, false).total;
  const int64_t lim = 160 * 1024;
  return *fwd1 <= lim && *fwd2 <= lim && *eb2 <= lim && *eb1 <= lim;
}

// the chunk-fused kernels run when the tile plan cuts graphs into the 64-row
// weight-gradient chunks, the partial buffer holds both layers, Fe <= 4 and
// every carve fits one workgroup's LDS
inline bool chunk_fused(const dr_vanilla_scratch* sc, int F, int Fe) {
  if (!sc->tile_row0 || !sc->tile_meta || !sc->relu_words || sc->tile_rows != WR || sc->part_layers != 2 || Fe > 4 || F > 32 ||
      sc->n_tiles != sc->n_chunks)
    return false;
  int64_t f1, f2, e2, e1;
  return chunk_carves(sc, F, Fe, &f1, &f2, &e2, &e1);
}

inline int64_t nb2_lds(int F) { return 4LL * (WR * (r4(F) + 4) + WR * r4(F) + WR * 32 + r4(F) * r16(F + 32)); }

// the chunk-fused step (vb_gemm<GM_HALVES> for layer 1, then the vc_* kernels)
template <int FE>
int launch_chunk_fused(const VA& a, const dr_vanilla_scratch* sc, hipStream_t st, int gg, size_t glds_halves) {
  int64_t f1, f2, e2, e1;
  chunk_carves(sc, a.F, a.Fe, &f1, &f2, &e2, &e1);
  const dim3 tg((unsigned)sc->n_tiles);
  DR_CHECK(dr_allow_big_lds(reinterpret_cast<const void*>(&vc_fwd<FE, 1>)));
  DR_CHECK(dr_allow_big_lds(reinterpret_cast<const void*>(&vc_fwd<FE, 2>)));
  DR_CHECK(dr_allow_big_lds(reinterpret_cast<const void*>(&vc_eb2n1<FE>)));
  DR_CHECK(dr_allow_big_lds(reinterpret_cast<const void*>(&vc_eb1<FE>)));
  DR_CHECK(dr_allow_big_lds(reinterpret_cast<const void*>(&vc_nb2)));
  (void)gg;
  (void)glds_halves;
  hipLaunchKernelGGL((vc_fwd<FE, 1>), tg, dim3(CT), (size_t)f1, st, a);
  hipLaunchKernelGGL((vc_fwd<FE, 2>), tg, dim3(CT), (size_t)f2, st, a);
  hipLaunchKernelGGL(vb_head, dim3(a.B), dim3(HT), 0, st, a);
  if (a.p.flags & DR_PASS_BACKWARD) {
    hipLaunchKernelGGL(vc_nb2, tg, dim3(NB2), (size_t)nb2_lds(a.F), st, a);
    hipLaunchKernelGGL(vc_eb2n1<FE>, tg, dim3(CT), (size_t)e2, st, a);
    hipLaunchKernelGGL(vc_eb1<FE>, tg, dim3(CT), (size_t)e1, st, a);
    hipLaunchKernelGGL(vc_combine, dim3(rows_grid((int64_t)a.B * 2 * (r4(layer_grad_size(a.F, a.Fe)) / 4), RB)), dim3(RB), 0, st, a);
  }
  return (int)hipGetLastError();
}

}  // namespace

extern "C" int64_t dr_vanilla_scratch_floats(int64_t n_rows, int32_t n_feat, int32_t n_edge_feat) {
  return scratch_layout(n_rows, n_feat, n_edge_feat).total;
}

extern "C" int64_t dr_vanilla_lds_bytes(int32_t n_feat, int32_t n_edge_feat, int32_t out_dim) {
  (void)out_dim;
  const int XS = r4(n_feat), FeS = n_edge_feat > 0 ? n_edge_feat : 1;
  (void)FeS;
  return 4LL * WR * (2 * XS + 3 * 32);  // the largest dynamic LDS of the pipeline (vb_wgrad_mfma)
}

extern "C" int64_t dr_vanilla_part_floats(int32_t n_feat, int32_t n_edge_feat) {
  return r4(layer_grad_size(n_feat, n_edge_feat));  // (the chunk-fused rows are 16-byte aligned)
}

extern "C" int dr_vanilla_graph_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                                     const dr_vanilla_weights* w, const dr_pass* pass,
                                     const dr_vanilla_scratch* scratch, int32_t lds_bytes, void* stream) {
  (void)lds_bytes;
  if (!store || !descs || !w || !pass || !scratch || n_batch < 0) return DR_E_ARG;
  if (pass->out_dim < 1 || pass->out_dim > DR_MAX_OUT) return DR_E_UNSUPPORTED;
  if (store->n_feat < 1 || store->n_feat > 64 || store->n_edge_feat < 0 || store->n_edge_feat > MAXFE)
    return DR_E_UNSUPPORTED;
  if (!scratch->base || !scratch->row0 || !scratch->row_slot) return DR_E_ARG;
  if ((pass->flags & DR_PASS_BACKWARD) && (!pass->slab || !pass->head)) return DR_E_ARG;
  if ((pass->flags & DR_PASS_BACKWARD) && pass->loss_kind == DR_LOSS_NONE && !pass->dout) return DR_E_ARG;
  if ((pass->flags & DR_PASS_FORWARD) && !pass->out) return DR_E_ARG;
  if ((pass->flags & DR_PASS_BACKWARD) && (!scratch->part || !scratch->chunk_first || !scratch->chunk_slot))
    return DR_E_ARG;
  if (scratch->tile_row0) {  // the tile plan: complete, and its LDS within one workgroup's 160 KiB
    if (!scratch->relu_words || !scratch->halo_off || !scratch->halo_ids || !scratch->lcol_off || !scratch->lcol ||
        !scratch->ltcol_off || !scratch->ltcol || scratch->n_tiles < 1 || scratch->halo_max < 1 ||
        scratch->halo_max > 65535 || scratch->tile_edges_max < 0 || scratch->tile_tedges_max < 0)
      return DR_E_ARG;
    const int FeS = store->n_edge_feat > 0 ? store->n_edge_feat : 1;
    if (4LL * tile_carve(scratch->halo_max, scratch->tile_edges_max, scratch->tile_tedges_max, FeS, true).total > 160 * 1024 ||
        4LL * tile_carve(scratch->halo_max, scratch->tile_edges_max, scratch->tile_tedges_max, FeS, false).total > 160 * 1024)
      return DR_E_LDS;
  }
  if (scratch->tile_wc && (!scratch->tile_row0 || !scratch->tile_first || scratch->tile_rows < 1 || WR % scratch->tile_rows))
    return DR_E_ARG;
  if (pass->use_dropout != DR_DROPOUT_OFF) return DR_E_UNSUPPORTED;
  // no in-launch hand-offs here: the pass never faults, but it clears the
  // caller's per-launch flag like every pass that takes one (dr_pass.fault)
  if (pass->fault) DR_CHECK(hipMemsetAsync(pass->fault, 0, sizeof(uint32_t), (hipStream_t)stream));
  if (n_batch == 0) return DR_OK;
  VA a;
  a.s = *store;
  a.w = *w;
  a.p = *pass;
  a.ws = *scratch;
  a.descs = descs;
  a.B = n_batch;
  a.F = store->n_feat;
  a.Fe = store->n_edge_feat;
  a.XS = r4(a.F);
  a.KE = 2 * a.F + a.Fe;
  a.KN = a.F + 32;
  a.L = scratch_layout(scratch->n_rows, a.F, a.Fe);
  hipStream_t st = (hipStream_t)stream;
  const int64_t R = scratch->n_rows;
  const size_t lds_wg = (size_t)dr_vanilla_lds_bytes(a.F, a.Fe, pass->out_dim);
  const int gg = rows_grid(R, GT) < 1024 ? rows_grid(R, GT) : 1024;
  auto glds = [&](int mode) { return (size_t)4 * gemm_lds_floats(mode, a.F); };
  if (!chunk_fused(scratch, a.F, a.Fe)) a.ws.part_mean = nullptr;  // (only the chunk-fused forward writes it)
  if (chunk_fused(scratch, a.F, a.Fe)) {
    switch (a.Fe) {
      case 0: return launch_chunk_fused<0>(a, scratch, st, gg, glds(GM_HALVES));
      case 1: return launch_chunk_fused<1>(a, scratch, st, gg, glds(GM_HALVES));
      case 2: return launch_chunk_fused<2>(a, scratch, st, gg, glds(GM_HALVES));
      case 3: return launch_chunk_fused<3>(a, scratch, st, gg, glds(GM_HALVES));
      default: return launch_chunk_fused<4>(a, scratch, st, gg, glds(GM_HALVES));
    }
  }
  for (int l = 1; l <= 2; ++l) {
    hipLaunchKernelGGL(vb_gemm<GM_HALVES>, dim3(gg), dim3(RB), glds(GM_HALVES), st, a, l);
    if (!launch_edge8(true, a, l, dim3(rows_grid(R, RB / 32)), st))
      hipLaunchKernelGGL(vb_edge_fwd, dim3(rows_grid(R, RB / 32)), dim3(RB), 0, st, a, l);
    hipLaunchKernelGGL(vb_gemm<GM_NODE>, dim3(gg), dim3(RB), glds(GM_NODE), st, a, l);
  }
  hipLaunchKernelGGL(vb_head, dim3(n_batch), dim3(HT), 0, st, a);
  if (pass->flags & DR_PASS_BACKWARD) {
    hipLaunchKernelGGL(vb_du, dim3(rows_grid(R * a.XS / 4, RB)), dim3(RB), 0, st, a, 2);
    hipLaunchKernelGGL(vb_gemm<GM_DXS>, dim3(gg), dim3(RB), glds(GM_DXS), st, a, 2);
    // the weight-gradient chunks read tile_wc only after the tiled backward wrote it
    VA aw = a;
    int eb = launch_edge8(false, a, 2, dim3(rows_grid(R, RB / 32)), st);
    if (!eb) hipLaunchKernelGGL(vb_edge_bwd, dim3(rows_grid(R, RB / 32)), dim3(RB), 0, st, a, 2);
    if (eb != 2) aw.ws.tile_wc = nullptr;
    hipLaunchKernelGGL(vb_gemm<GM_DX1>, dim3(gg), dim3(RB), glds(GM_DX1), st, a, 2);
    hipLaunchKernelGGL(vb_wgrad_mfma, dim3(scratch->n_chunks), dim3(RB), lds_wg, st, aw, 2);
    hipLaunchKernelGGL(vb_wgrad_combine, dim3(rows_grid((int64_t)n_batch * layer_grad_size(a.F, a.Fe), RB)), dim3(RB), 0, st, a, 2);
    hipLaunchKernelGGL(vb_du, dim3(rows_grid(R * a.XS / 4, RB)), dim3(RB), 0, st, a, 1);
    hipLaunchKernelGGL(vb_gemm<GM_DXS>, dim3(gg), dim3(RB), glds(GM_DXS), st, a, 1);
    aw = a;
    eb = launch_edge8(false, a, 1, dim3(rows_grid(R, RB / 32)), st);
    if (!eb) hipLaunchKernelGGL(vb_edge_bwd, dim3(rows_grid(R, RB / 32)), dim3(RB), 0, st, a, 1);
    if (eb != 2) aw.ws.tile_wc = nullptr;
    hipLaunchKernelGGL(vb_wgrad_mfma, dim3(scratch->n_chunks), dim3(RB), lds_wg, st, aw, 1);
    hipLaunchKernelGGL(vb_wgrad_combine, dim3(rows_grid((int64_t)n_batch * layer_grad_size(a.F, a.Fe), RB)), dim3(RB), 0, st, a, 1);
  }
  return (int)hipGetLastError();
}

// ---- carve descriptions for the host-side carve tests (tests/test_lds_carves.py)
extern "C" int dr_debug_carve_vanilla_tile(const int32_t* q, char* buf, int32_t len) {
  const TileCarve c = tile_carve(q[0], q[1], q[2], q[3], q[4] != 0);
  DrCarveDesc d{buf, len, 0};
  DR_DESC(d, c, rows);
  DR_DESC(d, c, rec);
  DR_DESC(d, c, trec);
  DR_DESC(d, c, total);
  return d.pos;
}

extern "C" int dr_debug_carve_vanilla_chunk_fwd(const int32_t* q, char* buf, int32_t len) {
  const FwdCarve c = fwd_carve(q[0], q[1], q[2], q[3]);
  DrCarveDesc d{buf, len, 0};
  DR_DESC_P(d, c, HS);
  DR_DESC_P(d, c, KP);
  DR_DESC_P(d, c, LA);
  DR_DESC_P(d, c, NOP);
  DR_DESC_P(d, c, hp);
  DR_DESC(d, c, xo);
  DR_DESC(d, c, wab);
  DR_DESC(d, c, halo);
  DR_DESC(d, c, rec);
  DR_DESC(d, c, a);
  DR_DESC(d, c, wn);
  DR_DESC(d, c, bn);
  DR_DESC(d, c, x2);
  DR_DESC(d, c, total);
  return d.pos;
}

extern "C" int dr_debug_carve_vanilla_chunk_bwd(const int32_t* q, char* buf, int32_t len) {
  const BwdCarve c = bwd_carve(q[0], q[1], q[2], q[3], q[4], q[5] != 0);
  DrCarveDesc d{buf, len, 0};
  DR_DESC_P(d, c, LDD);
  DR_DESC_P(d, c, LU);
  DR_DESC_P(d, c, NOP3);
  DR_DESC(d, c, d);
  DR_DESC(d, c, w3);
  DR_DESC(d, c, du);
  DR_DESC(d, c, sh);
  DR_DESC(d, c, halo);
  DR_DESC(d, c, trec);
  DR_DESC(d, c, x0);
  DR_DESC(d, c, x1);
  DR_DESC(d, c, dx);
  DR_DESC(d, c, s1);
  DR_DESC(d, c, w1);
  DR_DESC(d, c, total);
  return d.pos;
}

