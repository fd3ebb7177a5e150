// FoutNet and SGAT training steps, one workgroup per graph, everything
// resident in LDS.
//
// Replaces (deeprank2 v3.1.0):
//   FoutLayer.forward      deeprank2/neuralnets/gnn/foutnet.py:48-66
//   FoutNet.forward        foutnet.py:99-118
//   get_preloaded_cluster / community_pooling / max_pool_x / scatter_mean
//                          (community_pooling.py:23-27,165-242; foutnet.py:105-114)
//   autograd backward + loss (deeprank2/trainer.py:686-689)
//
// FoutLayer: out_i = x_i Wc + mean_{e=(i->j)} (x_j Wn) + b, NaN when node i has
// no out-edge (mean over an empty set, foutnet.py:58).  By linearity this is
// [x_i | mean_j x_j] [Wc; Wn] + b: the reference's O(N·E) Python loop becomes a
// CSR gather of X (Zm = D^-1 A X, 0/0 = NaN on empty rows) and one MFMA GEMM
// whose A operand reads X for k < F and Zm for F <= k < 2F.
// Backward: the depth-0 max pool routes each channel's gradient to one
// member per cluster, so dWc = sum_k v_k x[arg_k], dWn = sum_k v_k Zm[arg_k]
// and db = sum_k v_k — no gather over the edges.  The pooled conv2 backward
// scatters through the transposed pooled CSR.
//
// SGAT (template flag SG; deeprank2/neuralnets/gnn/sgat.py:56-133) has the same
// shape: SGraphAttentionLayer is z_i = mean_{e=(i->j)} a_e [x_i | x_j] W + b
// with torch_scatter's scatter_mean (count clamped to 1, so an edge-less row
// is 0, not NaN), i.e. [c_i x_i | Zw_i] [W_top; W_bot] + b with
// c_i = sum_e a_e / max(deg_i, 1) and Zw_i = sum_e a_e x_j / max(deg_i, 1).
// conv2 runs on the pooled graph with the pooled edge_attr (PyG pool_edge
// coalesce sums, precomputed in the store as p1_ea).  Needs Fe == 1 (sgat.py:71
// broadcasts edge_attr [E, Fe] over the output channels).

#include <hip/hip_runtime.h>

#include <cstring>

#include "graph_common.h"

#ifndef DR_FOUT_FRONT
#define DR_FOUT_FRONT 1  // FoutNet per-graph kernel: Zm, conv1 and depth-0 pooling fused per wave (0: three barrier phases)
#endif
#ifndef DR_FOUT_MSE_HEAD
#define DR_FOUT_MSE_HEAD 1  // FoutNet tail: one MSE logit's logit / loss / dh on wave 0 without barriers (0: the general head)
#endif
#ifndef DR_TILE_STORE_WAIT
#define DR_TILE_STORE_WAIT 0  // 1: the tile kernel waits for its Zm stores before the MFMA phase (r05 form, A/B)
#endif

namespace {

using namespace drk;

constexpr int NT = 1024;
constexpr int NW = NT / 64;
constexpr int HEADW = 512;  // G32 hpre64 hh64 dh64 dG32 dout16 spare

struct Carve {
  int KP, XS, LDZ;
  bool wide;  // zm rows hold [x_i | Zm_i] (conv1 A operand at a conflict-free stride)
  int ea, c1, p1w, p1tid, c2;  // SGAT only (0 words otherwise)
  int wc1, w2, fc1, fc2, x, zm, h1, rp, col, m0p, m0i, p1, a1, dp1, zm2, s2, h2, d2, dz2, p1rp, p1c, p1trp, p1tc,
      m1p, m1i, p2, nt, head, dgp, red, total;
};

// X keeps the HBM row stride XS = r4(F) (16-byte rows: DMA + float4 gather);
// when the graph fits, the zm rows hold [x_i | Zm_i] (the own row copied in the
// gather phase; SGAT: [x_i | Zw_i]) with stride LDZ = 2 r4(F) + 2, an odd
// multiple of 2: the conv1 MFMA operand reads of lanes (row li, k+kq) hit
// distinct banks (X's stride of 32 words puts 16 rows on one bank).  Otherwise
// zm holds Zm alone (LDZ = r4(F) + 2) and conv1 reads x_i from X.
__host__ __device__ inline Carve carve_at(int N, int E, int F, int K0, int P1, int K1, int alias, int OUT, bool sg, bool wide) {
  Carve c;
  c.KP = r16(2 * F);
  c.XS = r4(F);
  c.wide = wide;
  c.LDZ = wide ? 2 * c.XS + 2 : c.XS + 2;
  int o = 0;
#define TAKE(field, words) \
  c.field = o;             \
  o += r4(words);
  TAKE(wc1, c.KP * 16)                 // [Wc; Wn; 0] [KP, 16] (k-major, as stored)
  TAKE(w2, 16 * 32 * 2 + 32 + 16)      // Wc2 [16,32], Wn2 [16,32], b2 [32], b1 [16]
  TAKE(fc1, 64 * 32 + 64)              // fc1.weight [64,32], fc1.bias
  TAKE(fc2, OUT * 64 + OUT)            // fc2.weight [out,64], fc2.bias
  TAKE(x, N * c.XS)
  TAKE(zm, N * c.LDZ)
  TAKE(h1, N * 16)
  TAKE(rp, N + 1)
  TAKE(col, (E + 1) / 2)
  TAKE(m0p, K0 + 1)
  TAKE(m0i, N)
  TAKE(p1, K0 * 16)
  TAKE(a1, K0 * 16)
  TAKE(dp1, K0 * 16)
  TAKE(zm2, K0 * 16)
  TAKE(s2, K0 * 32)
  TAKE(h2, K0 * 32)
  TAKE(d2, K0 * 32)
  TAKE(dz2, K0 * 16)
  TAKE(p1rp, K0 + 1)
  TAKE(p1c, P1)
  if (alias) {
    c.p1trp = c.p1rp;
    c.p1tc = c.p1c;
  } else {
    TAKE(p1trp, K0 + 1)
    TAKE(p1tc, P1)
  }
  TAKE(m1p, K1 + 1)
  TAKE(m1i, K0)
  TAKE(p2, K1 * 32)
  TAKE(nt, K1 * 32)
  TAKE(head, HEADW)
  TAKE(dgp, NT)                        // the head backward's [NT / 32 chunks][32] partials
  TAKE(red, 2 * NT)
  if (sg) {
    TAKE(ea, E)
    TAKE(c1, N)
    TAKE(p1w, P1)
    TAKE(p1tid, P1)
    TAKE(c2, K0)
  } else {
    c.ea = c.c1 = c.p1w = c.p1tid = c.c2 = 0;
  }
#undef TAKE
  c.total = o;
  return c;
}

// The wide layout when it fits one workgroup's LDS, else the narrow one
// (the conv1 A operand then reads x_i from the X rows; same sums either way).
// `limit` = the bytes of LDS available: 160 KiB when the host sizes a launch
// (for the batch's elementwise-largest graph), the launch's dynamic LDS inside
// the kernel, so a graph never takes a layout its launch did not reserve.
__host__ __device__ inline Carve carve(int N, int E, int F, int K0, int P1, int K1, int alias, int OUT, bool sg,
                                       int64_t limit = 160 * 1024) {
  // decide first, then carve once: selecting between two Carve values makes
  // hipcc build them in scratch (44 B per lane, ~3 MB of writes per launch)
  const bool wide = 4LL * carve_at(N, E, F, K0, P1, K1, alias, OUT, sg, true).total <= limit;
  return carve_at(N, E, F, K0, P1, K1, alias, OUT, sg, wide);
}

struct FoutArgs {
  dr_graph_store s;
  dr_fout_weights w;
  dr_pass p;
  const dr_graph_desc* descs;
  int32_t B;
  int32_t lds_bytes;  // the launch's dynamic LDS: a graph takes the wide layout only if it fits this
};

// gather_row_chunk with edge weights: acc = sum_e w[e] X[col[e], c4..c4+3];
// sw = sum_e w[e] in edge order (the weights are loaded anyway)
__device__ __forceinline__ float4 gather_row_chunk_w(const uint16_t* col, const float* w, int eb, int ee,
                                                     const float* X, int XS, int c4, float& sw) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  sw = 0.f;
  for (int e = eb; e < ee; ++e) {
    const float we = w[e];
    sw += we;
    const float4 v = *reinterpret_cast<const float4*>(&X[__umul24((int)col[e], XS) + c4]);
    acc = make_float4(fmaf(we, v.x, acc.x), fmaf(we, v.y, acc.y), fmaf(we, v.z, acc.z), fmaf(we, v.w, acc.w));
  }
  return acc;
}

// gather_row_chunk_w for LDS col / w (the per-graph kernel): four edges per
// step, their index reads as lds_index4 and their row reads in flight
// together; the fmaf chain and the weight sum in edge order as above
__device__ __forceinline__ float4 gather_row_chunk_w_lds(const uint16_t* col, const float* w, int eb, int ee,
                                                         const float* X, int XS, int c4, float& sw) {
#if DR_GATHER_IMM
  const char* xc = reinterpret_cast<const char*>(X + c4);
  const int rb = XS * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  float s = 0.f;
  int e = eb;
  for (; e + 4 <= ee; e += 4) {
    int j[4];
    lds_index4(col + e, j[0], j[1], j[2], j[3]);
    float we[4];
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      we[u] = w[e + u];
      v[u] = *reinterpret_cast<const float4*>(xc + __umul24(j[u], rb));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      s += we[u];
      acc = make_float4(fmaf(we[u], v[u].x, acc.x), fmaf(we[u], v[u].y, acc.y), fmaf(we[u], v[u].z, acc.z), fmaf(we[u], v[u].w, acc.w));
    }
  }
  for (; e < ee; ++e) {
    const float we = w[e];
    s += we;
    const float4 v = *reinterpret_cast<const float4*>(xc + __umul24((int)col[e], rb));
    acc = make_float4(fmaf(we, v.x, acc.x), fmaf(we, v.y, acc.y), fmaf(we, v.z, acc.z), fmaf(we, v.w, acc.w));
  }
  sw = s;
  return acc;
#else
  return gather_row_chunk_w(col, w, eb, ee, X, XS, c4, sw);
#endif
}

// gather_row_chunk_w_lds for two 16-byte chunks of a row at once (the fused
// front's lane layout): one index and one weight read per edge feed both
// chunks; each chunk's fmaf chain and the weight sum in edge order, as above
__device__ __forceinline__ void gather_row_two_chunks_w_lds(const uint16_t* col, const float* w, int eb, int ee, const char* xa,
                                                            int db, int rb, float4& outa, float4& outb, float& sw) {
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
  float s = 0.f;
  int e = eb;
  for (; e + 4 <= ee; e += 4) {
    int j[4];
    lds_index4(col + e, j[0], j[1], j[2], j[3]);
    float we[4];
    float4 v[4], x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      we[u] = w[e + u];
      const char* pr = xa + __umul24(j[u], rb);
      v[u] = *reinterpret_cast<const float4*>(pr);
      x[u] = *reinterpret_cast<const float4*>(pr + db);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      s += we[u];
      a = make_float4(fmaf(we[u], v[u].x, a.x), fmaf(we[u], v[u].y, a.y), fmaf(we[u], v[u].z, a.z), fmaf(we[u], v[u].w, a.w));
      b = make_float4(fmaf(we[u], x[u].x, b.x), fmaf(we[u], x[u].y, b.y), fmaf(we[u], x[u].z, b.z), fmaf(we[u], x[u].w, b.w));
    }
  }
  for (; e < ee; ++e) {
    const float we = w[e];
    s += we;
    const char* pr = xa + __umul24((int)col[e], rb);
    const float4 v = *reinterpret_cast<const float4*>(pr), x = *reinterpret_cast<const float4*>(pr + db);
    a = make_float4(fmaf(we, v.x, a.x), fmaf(we, v.y, a.y), fmaf(we, v.z, a.z), fmaf(we, v.w, a.w));
    b = make_float4(fmaf(we, x.x, b.x), fmaf(we, x.y, b.y), fmaf(we, x.z, b.z), fmaf(we, x.w, b.w));
  }
  outa = a;
  outb = b;
  sw = s;
}

// The per-graph tail shared by fout_graph_kernel and the large-graph tail
// kernel: conv2 on the pooled graph, depth-1 max pool, mean, head, loss and
// the whole backward down to the conv1 weight partials.  Needs the depth-0
// pool (P1, A1: value and first arg per (cluster, channel)) and the pooled
// graph / weights in LDS (FoutTail); xarg(i, k) = [c1 x]_{i,k} (SGAT: c1_i x_ik)
// and zarg(i, k) = Zm_{i,k} at the pooling args, wherever they live.
struct FoutTail {
  float *P1, *dP1, *Zm2, *S2, *H2, *D2, *Dz2, *P2, *NTie, *G, *Hpre, *Hh, *Dh, *DG, *Dout, *DGp, *P1w, *C2;
  int *A1, *p1rp, *p1c, *p1trp, *p1tc, *m1p, *m1i, *P1tid;
  const float *Wc2, *Wn2, *B2, *Fc1, *Fc1b, *Fc2;
};

#define FT_STAMP(i)                                                                             \
  do {                                                                                          \
    if (DR_STAMPS_ON && tid == 0 && p.stamps) p.stamps[(int64_t)b * 32 + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#ifdef DR_STAMPS
#define DR_STAMPS_ON 1
#else
#define DR_STAMPS_ON 0
#endif

template <bool SG, class XF, class ZF>
__device__ __forceinline__ void fout_tail(const dr_pass& p, const FoutTail t, int b, int N, int K0, int K1, int F, int OUT,
                                          float y_g, XF xarg, ZF zarg) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  FT_STAMP(4);
  // ---------------- conv2 on the pooled graph: FoutLayer(16, 32) ----------
  // (SGAT: SGraphAttentionLayer(16, 32) with the pooled edge weights)
  for (int p = tid; p < K0 * 16; p += NT) {  // Zm2 = mean over pooled out-neighbours
    const int k = p >> 4, j = p & 15;
    const int eb = t.p1rp[k], ee = t.p1rp[k + 1];
    float acc = 0.f;
    if (SG) {
      float sw = 0.f;
      for (int e = eb; e < ee; ++e) {
        acc = fmaf(t.P1w[e], t.P1[t.p1c[e] * 16 + j], acc);
        sw += t.P1w[e];
      }
      const float deg = (float)imax(ee - eb, 1);
      t.Zm2[p] = acc / deg;
      if (j == 0) t.C2[k] = sw / deg;
    } else {
      for (int e = eb; e < ee; ++e) acc += t.P1[t.p1c[e] * 16 + j];
      t.Zm2[p] = acc / (float)(ee - eb);
    }
  }
  __syncthreads();
  for (int p = tid; p < K0 * 32; p += NT) {
    const int k = p >> 5, o = p & 31;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) acc = fmaf(t.P1[k * 16 + j], t.Wc2[j * 32 + o], acc);
    if (SG) acc *= t.C2[k];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc = fmaf(t.Zm2[k * 16 + j], t.Wn2[j * 32 + o], acc);
    const float sv = acc + t.B2[o];
    t.S2[p] = sv;
    t.H2[p] = relu_keepnan(sv);
  }
  __syncthreads();

  FT_STAMP(5);
  // ---------------- depth-1 max_pool_x (amax: NaN propagates) + mean -------
  for (int p = tid; p < K1 * 32; p += NT) {
    const int m = p >> 5, o = p & 31;
    const int mb = t.m1p[m], me = t.m1p[m + 1];
    float mx = t.H2[t.m1i[mb] * 32 + o];
    for (int q = mb + 1; q < me; ++q) {
      const float v = t.H2[t.m1i[q] * 32 + o];
      mx = (mx != mx || v != v) ? __int_as_float(0x7fc00000) : fmaxf(mx, v);
    }
    float ties = 0.f;
    for (int q = mb; q < me; ++q) ties += (t.H2[t.m1i[q] * 32 + o] == mx) ? 1.f : 0.f;
    t.P2[p] = mx;
    t.NTie[p] = ties;
  }
  __syncthreads();
  if (tid < 32) {
    float acc = 0.f;
    for (int m = 0; m < K1; ++m) acc += t.P2[m * 32 + tid];
    t.G[tid] = acc / (float)K1;
  }
  __syncthreads();

  FT_STAMP(6);
  // ---------------- head: fc1 (32->64) -> relu -> fc2 (foutnet.py:115-117) --
  {
    const int r = tid >> 3, part = tid & 7;  // 8 lanes per fc1 row, 4 inputs each
    float acc = 0.f;
    if (r < 64) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = fmaf(t.G[part * 4 + j], t.Fc1[r * 32 + part * 4 + j], acc);
    }
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    acc += __shfl_xor(acc, 4, 64);
    if (r < 64 && part == 0) {
      acc += t.Fc1b[r];
      t.Hpre[r] = acc;
      t.Hh[r] = relu_keepnan(acc);
    }
  }
  __syncthreads();
  if (DR_FOUT_MSE_HEAD && OUT == 1 && p.loss_kind == DR_LOSS_MSE && (p.flags & DR_PASS_BACKWARD)) {
    // one MSE logit (configs[2]): wave 0 forms the logit (the same wave sum),
    // the loss gradient and dh for the 64 hidden units, with no workgroup
    // barrier between them (as ginet_head.h's MSE path)
    if (wave == 0) {
      const float v = dr_wave_sum(t.Hh[lane] * t.Fc2[lane]);
      const float logit = v + t.Fc2[64];
      const float dlt = logit - y_g;
      const float dout0 = 2.f * dlt * p.loss_scale;
      if (lane == 0) {
        if (p.flags & DR_PASS_FORWARD) p.out[b] = logit;
        if (p.loss_per_graph) p.loss_per_graph[b] = dlt * dlt;
        t.Dout[0] = dout0;
      }
      t.Dh[lane] = relu_bwd(t.Hh[lane], fmaf(t.Fc2[lane], dout0, 0.f));
    }
    FT_STAMP(7);
    __syncthreads();
  } else {
  for (int q = wave; q < OUT; q += NW) {
    float v = t.Hh[lane] * t.Fc2[q * 64 + lane];
    v = dr_wave_sum(v);
    if (lane == 0) t.Dout[q] = v + t.Fc2[OUT * 64 + q];
  }
  __syncthreads();
  if ((p.flags & DR_PASS_FORWARD) && tid < OUT) p.out[(int64_t)b * OUT + tid] = t.Dout[tid];
  if (!(p.flags & DR_PASS_BACKWARD)) return;
  __syncthreads();

  FT_STAMP(7);
  // ---------------- loss gradient (trainer.py:688-689) ----------------------
  if (tid == 0) {
    if (p.loss_kind == DR_LOSS_MSE) {
      const float dlt = t.Dout[0] - y_g;
      if (p.loss_per_graph) p.loss_per_graph[b] = dlt * dlt;
      t.Dout[0] = 2.f * dlt * p.loss_scale;
    } else if (p.loss_kind == DR_LOSS_CE) {
      const int yi = (int)y_g;
      float mx = t.Dout[0];
      for (int q = 1; q < OUT; ++q) mx = fmaxf(mx, t.Dout[q]);
      float se = 0.f;
      for (int q = 0; q < OUT; ++q) se += expf(t.Dout[q] - mx);
      const float lse = mx + logf(se);
      const float wy = p.class_w ? p.class_w[yi] : 1.f;
      if (p.loss_per_graph) p.loss_per_graph[b] = wy * (lse - t.Dout[yi]);
      for (int q = 0; q < OUT; ++q) t.Dout[q] = wy * (expf(t.Dout[q] - lse) - (q == yi ? 1.f : 0.f)) * p.loss_scale;
    } else {
      for (int q = 0; q < OUT; ++q) t.Dout[q] = p.dout[(int64_t)b * OUT + q];
    }
  }
  __syncthreads();

  // ---------------- head backward -------------------------------------------
  if (tid < 64) {
    float acc = 0.f;
    for (int q = 0; q < OUT; ++q) acc = fmaf(t.Fc2[q * 64 + tid], t.Dout[q], acc);
    t.Dh[tid] = relu_bwd(t.Hh[tid], acc);
  }
  __syncthreads();
  }
  {
    const int o = tid & 31, rc = tid >> 5;  // 32 chunks of 2 fc1 rows
    float acc = fmaf(t.Fc1[(rc * 2) * 32 + o], t.Dh[rc * 2], t.Fc1[(rc * 2 + 1) * 32 + o] * t.Dh[rc * 2 + 1]);
    t.DGp[rc * 32 + o] = acc;
  }
  __syncthreads();
  if (tid < 32) {
    float acc = 0.f;
    for (int rc = 0; rc < NT / 32; ++rc) acc += t.DGp[rc * 32 + tid];
    t.DG[tid] = acc;
  }
  {
    const int HS = DR_FOUT_HEAD_STRIDE(OUT);
    float* hg = p.head + (int64_t)b * HS;
    if (tid < 32) hg[tid] = t.G[tid];
    if (tid < 64) {
      hg[32 + tid] = t.Hh[tid];
      hg[96 + tid] = t.Dh[tid];
    }
    if (tid < OUT) hg[160 + tid] = t.Dout[tid];
  }
  __syncthreads();

  FT_STAMP(8);
  // ---------------- depth-1 pooling + mean backward -------------------------
  for (int p = tid; p < K1 * 32; p += NT) {
    const int m = p >> 5, o = p & 31;
    const float gm = (t.DG[o] / (float)K1) / t.NTie[p];
    const float mx = t.P2[p];
    for (int q = t.m1p[m]; q < t.m1p[m + 1]; ++q) {
      const int k = t.m1i[q];
      const float h = t.H2[k * 32 + o];
      t.D2[k * 32 + o] = relu_bwd(h, (h == mx ? 1.f : 0.f) * gm);
    }
  }
  __syncthreads();
  // conv2 weight partials; gradient into the mean term (dZm2 = dS2 Wn2^T)
  {
    const int SS = DR_FOUT_SLAB_STRIDE(F);
    float* slab = p.slab + (int64_t)b * SS + 32 * F + 16;
    for (int p = tid; p < 1024 + 32; p += NT) {
      float acc = 0.f;
      if (p < 512) {  // dWc2[j][o] = sum_k (c2_k) P1[k][j] dS2[k][o]
        const int j = p >> 5, o = p & 31;
        for (int k = 0; k < K0; ++k) acc = fmaf((SG ? t.C2[k] : 1.f) * t.P1[k * 16 + j], t.D2[k * 32 + o], acc);
      } else if (p < 1024) {  // dWn2[j][o] = sum_{k: deg>0} Zm2[k][j] dS2[k][o]
        const int q = p - 512, j = q >> 5, o = q & 31;
        for (int k = 0; k < K0; ++k)
          if (SG || t.p1rp[k + 1] > t.p1rp[k]) acc = fmaf(t.Zm2[k * 16 + j], t.D2[k * 32 + o], acc);
      } else {  // db2[o]
        const int o = p - 1024;
        for (int k = 0; k < K0; ++k) acc += t.D2[k * 32 + o];
      }
      slab[p] = acc;
    }
  }
  for (int p = tid; p < K0 * 16; p += NT) {
    const int k = p >> 4, j = p & 15;
    float dz = 0.f, dp = 0.f;
#pragma unroll 8
    for (int o = 0; o < 32; ++o) {
      const float ds = t.D2[k * 32 + o];
      dz = fmaf(ds, t.Wn2[j * 32 + o], dz);
      dp = fmaf(ds, t.Wc2[j * 32 + o], dp);
    }
    const int deg = t.p1rp[k + 1] - t.p1rp[k];
    t.Dz2[p] = deg > 0 ? dz / (float)deg : 0.f;
    t.dP1[p] = SG ? t.C2[k] * dp : dp;
  }
  __syncthreads();
  // dP1[j] += sum_{i: j in N(i)} dZm2[i] / deg_i  (transposed pooled CSR), then
  // route to the depth-0 arg member through relu: v = relu'(H1[arg]) dP1
  for (int p = tid; p < K0 * 16; p += NT) {
    const int k = p >> 4, j = p & 15;
    float acc = t.dP1[p];
    if (SG) {
      for (int e = t.p1trp[k]; e < t.p1trp[k + 1]; ++e) acc = fmaf(t.P1w[t.P1tid[e]], t.Dz2[t.p1tc[e] * 16 + j], acc);
    } else {
      for (int e = t.p1trp[k]; e < t.p1trp[k + 1]; ++e) acc += t.Dz2[t.p1tc[e] * 16 + j];
    }
    const int i = t.A1[p];
    t.dP1[p] = (i < N) ? relu_bwd(t.P1[p], acc) : 0.f;  // H1[arg] is the pooled value itself
  }
  __syncthreads();

  FT_STAMP(9);
  // ---------------- conv1 weight partials: sum_k v_k [x | Zm][arg_k] -------
  {
    const int SS = DR_FOUT_SLAB_STRIDE(F);
    float* slab = p.slab + (int64_t)b * SS;
    for (int p = tid; p < 32 * F + 16; p += NT) {
      float acc = 0.f;
      if (p < 32 * F) {
        const int half = p >= 16 * F;  // 0: dWc [F,16], 1: dWn [F,16]
        const int q = p - half * 16 * F, kk = q >> 4, ch = q & 15;
        for (int k = 0; k < K0; ++k) {
          const int i = t.A1[k * 16 + ch];
          if (i < N) acc = fmaf(t.dP1[k * 16 + ch], half ? zarg(i, kk) : xarg(i, kk), acc);
        }
      } else {
        const int ch = p - 32 * F;
        for (int k = 0; k < K0; ++k) acc += t.dP1[k * 16 + ch];
      }
      slab[p] = acc;
    }
  }
}

template <bool SG>
__global__ void __launch_bounds__(NT) fout_graph_kernel(FoutArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int b = blockIdx.x;
  const dr_graph_store& s = a.s;
  const dr_graph_desc d = a.descs[b];
  const int g = d.gid;
  const int64_t n0 = d.node0, ec0 = d.col0, k00 = d.k0, q0 = d.p1, k10 = d.k1;
  const int N = d.n_nodes, E = d.n_edges, K0 = d.n_k0, P1 = d.n_p1, K1 = d.n_k1;
  const int F = s.n_feat;
  const int alias = s.transpose_aliased;
  const int OUT = a.p.out_dim;
  const Carve c = carve(N, E, F, K0, P1, K1, alias, OUT, SG, a.lds_bytes);
  const int KP = c.KP, XS = c.XS, LDZ = c.LDZ;
  const bool WIDE = c.wide;
  const int ZO = WIDE ? XS : 0;  // column of Zm_0 in a zm row
  float* sEa = lds + c.ea;
  float* sC1 = lds + c.c1;
  float* sP1w = lds + c.p1w;
  int* sP1tid = reinterpret_cast<int*>(lds + c.p1tid);
  float* sC2 = lds + c.c2;

  float* sWc1 = lds + c.wc1;
  float* sWc2 = lds + c.w2;
  float* sWn2 = sWc2 + 512;
  float* sB2 = sWn2 + 512;
  float* sB1 = sB2 + 32;
  float* sFc1 = lds + c.fc1;
  float* sFc1b = sFc1 + 2048;
  float* sFc2 = lds + c.fc2;
  float* sX = lds + c.x;
  float* sZm = lds + c.zm;
  float* sH1 = lds + c.h1;
  int* srp = reinterpret_cast<int*>(lds + c.rp);
  uint16_t* scol = reinterpret_cast<uint16_t*>(lds + c.col);
  int* sm0p = reinterpret_cast<int*>(lds + c.m0p);
  int* sm0i = reinterpret_cast<int*>(lds + c.m0i);
  float* sP1 = lds + c.p1;
  int* sA1 = reinterpret_cast<int*>(lds + c.a1);
  float* sdP1 = lds + c.dp1;
  float* sZm2 = lds + c.zm2;
  float* sS2 = lds + c.s2;
  float* sH2 = lds + c.h2;
  float* sD2 = lds + c.d2;
  float* sDz2 = lds + c.dz2;
  int* sp1rp = reinterpret_cast<int*>(lds + c.p1rp);
  int* sp1c = reinterpret_cast<int*>(lds + c.p1c);
  int* sp1trp = reinterpret_cast<int*>(lds + c.p1trp);
  int* sp1tc = reinterpret_cast<int*>(lds + c.p1tc);
  int* sm1p = reinterpret_cast<int*>(lds + c.m1p);
  int* sm1i = reinterpret_cast<int*>(lds + c.m1i);
  float* sP2 = lds + c.p2;
  float* sNT = lds + c.nt;
  float* sG = lds + c.head;
  float* sHpre = sG + 32;
  float* sHh = sHpre + 64;
  float* sDh = sHh + 64;
  float* sDG = sDh + 64;
  float* sDout = sDG + 32;
  float* sDGp = lds + c.dgp;
  float* sRed = lds + c.red;

  DRK_STAMP(0);
  // ---------------- stage: graph by DMA, weights through VGPRs --------------
  const float y_g = s.y[g];
  // no dropout here, but the step counter contract holds: snapshot for
  // dr_reduce_update (stored after the staging wait below)
  dma_x4<NT>(sX, s.x + n0 * (int64_t)XS, N * XS / 4);
  dma_x4<NT>(scol, s.col + ec0, (E + 7) / 8);
  dma_words<NT>(srp, s.rowptr + n0 + g, N + 1);
  dma_words<NT>(sm0p, s.m0_ptr + k00 + g, K0 + 1);
  dma_words<NT>(sm0i, s.m0_idx + n0, N);
  dma_words<NT>(sp1rp, s.p1_rowptr + k00 + g, K0 + 1);
  dma_words<NT>(sp1c, s.p1_col + q0, P1);
  if (!alias) {
    dma_words<NT>(sp1trp, s.p1t_rowptr + k00 + g, K0 + 1);
    dma_words<NT>(sp1tc, s.p1t_col + q0, P1);
  }
  dma_words<NT>(sm1p, s.m1_ptr + k10 + g, K1 + 1);
  dma_words<NT>(sm1i, s.m1_idx + k00, K0);
  if (SG) {  // Fe == 1: edge weights are contiguous at col_off, pooled ones at p1_off
    dma_words<NT>(sEa, s.ea + ec0, E);
    dma_words<NT>(sP1w, s.p1_ea + q0, P1);
    dma_words<NT>(sP1tid, s.p1t_pid + q0, P1);
  }
  // The fused front (FoutNet, F <= 32, K0 <= 64): each wave gathers its 16-row
  // tile's Zm, runs conv1 on it and pools it by 64-bit LDS atomic max keys
  // (ginet_fused.hip's front half), so conv1's weights and the node clusters
  // are staged here, the keys live in the reduction scratch and the H1 rows
  // are never formed (the tail reads P1 / A1 and [x | Zm] at the args only).
  const bool FRONT = DR_FOUT_FRONT && XS <= 32 && K0 * 32 <= 2 * NT;
  int* scl0 = reinterpret_cast<int*>(sH1);
  unsigned long long* skey = reinterpret_cast<unsigned long long*>(sRed);
  if (FRONT) {
    dma_words<NT>(scl0, s.cl0 + n0, N);
    dma_words<NT>(sWc1, a.w.wc1, F * 16);  // [Wc; Wn] k-major, as the weight image below
    dma_words<NT>(sWc1 + F * 16, a.w.wn1, F * 16);
    dma_words<NT>(sB1, a.w.b1, 16);
    for (int p = 2 * F * 16 + tid; p < KP * 16; p += NT) sWc1[p] = 0.f;  // K padding rows
    for (int p = tid; p < K0 * 16; p += NT) skey[p] = 0ull;
  }
  const int64_t counter0 = (a.p.step_counter && b == 0) ? a.p.step_counter[0] : 0;  // loaded late: no early wait
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (a.p.step_counter && b == 0 && tid == 0) a.p.step_counter[1] = counter0;
  __syncthreads();

  DRK_STAMP(1);
  // Weights (needed after the gather) via VGPRs: their latency overlaps it.
  // Flat weight image: [Wc;Wn] (2F*16) | Wc2 Wn2 b2 b1 (1072) | fc1 (2048+64) | fc2 (OUT*65)
  constexpr int WREG = 6;
  float wr[WREG];
  const int nw1 = 2 * F * 16, nw2 = 1072, nf1 = 2048 + 64, nf2 = OUT * 64 + OUT;
  const int ntot = nw1 + nw2 + nf1 + nf2;
#pragma unroll
  for (int u = 0; u < WREG; ++u) {
    const int p = tid + u * NT;
    float v = 0.f;
    if (p < nw1) v = (p < F * 16) ? a.w.wc1[p] : a.w.wn1[p - F * 16];
    else if (p < nw1 + nw2) {
      const int q = p - nw1;
      v = q < 512 ? a.w.wc2[q] : q < 1024 ? a.w.wn2[q - 512] : q < 1056 ? a.w.b2[q - 1024] : a.w.b1[q - 1056];
    } else if (p < nw1 + nw2 + nf1) {
      const int q = p - nw1 - nw2;
      v = q < 2048 ? a.w.fc1w[q] : a.w.fc1b[q - 2048];
    } else if (p < ntot) {
      const int q = p - nw1 - nw2 - nf1;
      v = q < OUT * 64 ? a.w.fc2w[q] : a.w.fc2b[q - OUT * 64];
    }
    wr[u] = v;
  }
  if (FRONT) {
    // ------ fused front: Zm rows, conv1, depth-0 pooling keys, per wave ------
    // Zm = D^-1 A X (foutnet.py:55-58; 0/0 = NaN on empty rows): one row per
    // four lanes, 16-byte chunks q and q ^ 4 (same sums and order as the
    // 8-lanes-per-row gather); H1 = relu([X | Zm] [Wc; Wn] + b) on MFMA; the
    // max per (cluster, channel) as (H bits << 32 | ~node): H >= +0 or NaN
    // (never pooled), the first max in node order wins (scatter_max).
    const int li = lane & 15, kq = lane >> 4, nch = XS >> 2;
    const int ca = (lane & 3) | (lane & 4), cb = ca ^ 4;
    for (int tt = wave; tt * 16 < N; tt += NW) {
      const int r0 = tt * 16, i = r0 + (lane >> 2);
      const int eb = i < N ? srp[i] : 0, ee = i < N ? srp[i + 1] : 0;
      const float deg = SG ? (float)imax(ee - eb, 1) : (float)(ee - eb);
      float4 za, zb;
      if (SG) {  // SGAT: Zw = D^-1 A_w X, c1 = D^-1 A_w 1 (D clamped to 1, sgat.py:74-76)
        float sw;
        gather_row_two_chunks_w_lds(scol, sEa, eb, ee, reinterpret_cast<const char*>(sX + ca * 4), (cb - ca) * 16, XS * 4, za, zb, sw);
        if (i < N && (lane & 3) == 0) sC1[i] = sw / deg;
      } else {
        gather_row_two_chunks_imm(scol, eb, ee, reinterpret_cast<const char*>(sX + ca * 4), (cb - ca) * 16, XS * 4, za, zb);
      }
      if (i < N) {
        if (ca < nch) {
          if (WIDE) {
            const float4 xv = *reinterpret_cast<const float4*>(sX + i * XS + ca * 4);
            float2* xr = reinterpret_cast<float2*>(sZm + i * LDZ + ca * 4);
            xr[0] = make_float2(xv.x, xv.y);
            xr[1] = make_float2(xv.z, xv.w);
          }
          float2* zr = reinterpret_cast<float2*>(sZm + i * LDZ + ZO + ca * 4);
          zr[0] = make_float2(za.x / deg, za.y / deg);
          zr[1] = make_float2(za.z / deg, za.w / deg);
        }
        if (cb < nch) {
          if (WIDE) {
            const float4 xv = *reinterpret_cast<const float4*>(sX + i * XS + cb * 4);
            float2* xr = reinterpret_cast<float2*>(sZm + i * LDZ + cb * 4);
            xr[0] = make_float2(xv.x, xv.y);
            xr[1] = make_float2(xv.z, xv.w);
          }
          float2* zr = reinterpret_cast<float2*>(sZm + i * LDZ + ZO + cb * 4);
          zr[0] = make_float2(zb.x / deg, zb.y / deg);
          zr[1] = make_float2(zb.z / deg, zb.w / deg);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's Zm rows are in LDS before its MFMA reads them
      const int ar = min(r0 + li, N - 1);
      const float cx = SG ? sC1[ar] : 1.f;
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < KP; k += 16) {  // (B from LDS: a register-resident B measured +1.2 us per pass)
        float av[4], bv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int kk = k + 4 * u + kq;
          av[u] = kk < F ? cx * (WIDE ? sZm[ar * LDZ + kk] : sX[ar * XS + kk]) : (kk < 2 * F ? sZm[ar * LDZ + ZO + kk - F] : 0.f);
          bv[u] = sWc1[kk * 16 + li];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], acc, 0, 0, 0);
      }
      const float b1 = sB1[li];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + kq * 4 + r;
        if (row < N) {
          const float v = relu_keepnan(acc[r] + b1);
          if (v == v)
            __hip_atomic_fetch_max(skey + scl0[row] * 16 + li,
                                   ((unsigned long long)__float_as_uint(v) << 32) | (0xffffffffull - (unsigned long long)(uint32_t)row),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < WREG; ++u) {  // the other weights ([Wc; Wn] and b1 were staged)
      const int p = tid + u * NT;
      if (p < nw1) continue;
      if (p < nw1 + nw2) {
        if (p - nw1 < 1056) sWc2[p - nw1] = wr[u];
      } else if (p < nw1 + nw2 + nf1) sFc1[p - nw1 - nw2] = wr[u];
      else if (p < ntot) sFc2[p - nw1 - nw2 - nf1] = wr[u];
    }
    __syncthreads();
    DRK_STAMP(2);
    DRK_STAMP(3);
    for (int p = tid; p < K0 * 16; p += NT) {  // the keys decoded: P1 = H1[arg] exactly; empty: 0, arg N
      const unsigned long long key = skey[p];
      sP1[p] = key ? __uint_as_float((uint32_t)(key >> 32)) : 0.f;
      sA1[p] = key ? (int)(0xffffffffu - (uint32_t)key) : N;
    }
    __syncthreads();
  } else {
  // ---------------- Zm = D^-1 A X (foutnet.py:55-58; NaN on empty rows) ----
  // SGAT: Zw = D^-1 A_w X and c = D^-1 A_w 1 with D clamped to 1 (sgat.py:74-76)
  {
    const int nch = XS >> 2;
    const int sub = tid & 7;
    for (int i = tid >> 3; i < N; i += NT / 8) {
      const int eb = srp[i], ee = srp[i + 1];
      const float deg = SG ? (float)imax(ee - eb, 1) : (float)(ee - eb);
      for (int ch = sub; ch < nch; ch += 8) {
        const int c4 = ch * 4;
        float sw;
        const float4 acc = SG ? gather_row_chunk_w_lds(scol, sEa, eb, ee, sX, XS, c4, sw)
                              : gather_row_chunk_lds(scol, eb, ee, sX, XS, c4);
        if (SG && ch == 0) sC1[i] = sw / deg;
        // Rows are 8-byte aligned (LDZ even): two 64-bit stores per chunk; the
        // pad columns F..XS-1 they also fill are never read.
        if (WIDE) {  // own row x_i next to Zm_i (the conv1 A operand at a conflict-free stride)
          float2* xr = reinterpret_cast<float2*>(sZm + i * LDZ + c4);
          const float4 xv = *reinterpret_cast<const float4*>(sX + i * XS + c4);
          xr[0] = make_float2(xv.x, xv.y);
          xr[1] = make_float2(xv.z, xv.w);
        }
        float2* zr = reinterpret_cast<float2*>(sZm + i * LDZ + ZO + c4);
        // mean over the out-neighbours; 0/0 = NaN exactly as torch.mean(empty)
        zr[0] = make_float2(acc.x / deg, acc.y / deg);
        zr[1] = make_float2(acc.z / deg, acc.w / deg);
      }
    }
  }
#pragma unroll
  for (int u = 0; u < WREG; ++u) {
    const int p = tid + u * NT;
    if (p < nw1) sWc1[p] = wr[u];  // rows 0..F-1 = Wc, F..2F-1 = Wn
    else if (p < nw1 + nw2) sWc2[p - nw1] = wr[u];
    else if (p < nw1 + nw2 + nf1) sFc1[p - nw1 - nw2] = wr[u];
    else if (p < ntot) sFc2[p - nw1 - nw2 - nf1] = wr[u];
  }
  for (int p = nw1 + tid; p < KP * 16; p += NT) sWc1[p] = 0.f;  // K padding rows
  __syncthreads();

  DRK_STAMP(2);
  // ---------------- conv1 on MFMA: H1 = relu([X | Zm] [Wc; Wn] + b) -------
  {
    const int li = lane & 15, kq = lane >> 4;
    for (int t = wave; t * 16 < N; t += NW) {
      const int r0 = t * 16;
      const int ar = min(r0 + li, N - 1);
      const float cx = SG ? sC1[ar] : 1.f;
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < KP; k += 16) {
        float av[4], bv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int kk = k + 4 * u + kq;
          av[u] = kk < F ? cx * (WIDE ? sZm[ar * LDZ + kk] : sX[ar * XS + kk])
                         : (kk < 2 * F ? sZm[ar * LDZ + ZO + kk - F] : 0.f);
          bv[u] = sWc1[kk * 16 + li];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + kq * 4 + r;
        if (row < N) sH1[row * 16 + li] = relu_keepnan(acc[r] + sB1[li]);
      }
    }
  }
  __syncthreads();

  DRK_STAMP(3);
  // ---------------- depth-0 community pooling (torch_scatter scatter_max) ---
  {
    const int pairs = K0 * 16;
    const int LS = pairs <= NT / 8 ? 3 : pairs <= NT / 4 ? 2 : pairs <= NT / 2 ? 1 : 0;
    const int S1 = 1 << LS;
    float* tb = sRed;
    int* ta = reinterpret_cast<int*>(sRed + NT);
    for (int p = tid; p < pairs * S1; p += NT) {
      const int sl = p & (S1 - 1), pr = p >> LS;
      const int k = pr >> 4, ch = pr & 15;
      const int mb = sm0p[k], cnt = sm0p[k + 1] - mb;
      const int qb = mb + ((cnt * sl) >> LS), qe = mb + ((cnt * (sl + 1)) >> LS);
      float best = LOWEST;
      int arg = N;
      for (int m = qb; m < qe; ++m) {
        const int i = sm0i[m];
        const float v = sH1[i * 16 + ch];
        if (v > best) {
          best = v;
          arg = i;
        }
      }
      tb[p] = best;
      ta[p] = arg;
    }
    __syncthreads();
    for (int p = tid; p < pairs; p += NT) {
      float best = LOWEST;
      int arg = N;
      for (int sl = 0; sl < S1; ++sl) {
        const float v = tb[(p << LS) + sl];
        if (v > best) {
          best = v;
          arg = ta[(p << LS) + sl];
        }
      }
      sP1[p] = (best == LOWEST) ? 0.f : best;
      sA1[p] = arg;
    }
  }
  __syncthreads();
  }

  FoutTail t;
  t.P1 = sP1; t.A1 = sA1; t.dP1 = sdP1; t.Zm2 = sZm2; t.S2 = sS2; t.H2 = sH2; t.D2 = sD2; t.Dz2 = sDz2;
  t.p1rp = sp1rp; t.p1c = sp1c; t.p1trp = sp1trp; t.p1tc = sp1tc; t.m1p = sm1p; t.m1i = sm1i;
  t.P2 = sP2; t.NTie = sNT; t.G = sG; t.Hpre = sHpre; t.Hh = sHh; t.Dh = sDh; t.DG = sDG; t.Dout = sDout; t.DGp = sDGp;
  t.Wc2 = sWc2; t.Wn2 = sWn2; t.B2 = sB2; t.Fc1 = sFc1; t.Fc1b = sFc1b; t.Fc2 = sFc2;
  t.P1w = sP1w; t.P1tid = sP1tid; t.C2 = sC2;
  // conv1 weight partials read [c1 x | Zm] at the pooling args from LDS
  fout_tail<SG>(a.p, t, a.p.slot ? a.p.slot[b] : b, N, K0, K1, F, OUT, y_g,
                [=](int i, int kk) { return (SG ? sC1[i] : 1.f) * (WIDE ? sZm[i * LDZ + kk] : sX[i * XS + kk]); },
                [=](int i, int kk) { return sZm[i * LDZ + ZO + kk]; });
  DRK_STAMP(10);
}

// ---- graphs beyond one workgroup's LDS (atom-level): tile kernel + tail kernel ----
// Same arithmetic as fout_graph_kernel, split like dr_ginet_large_pass and on
// its plan (dr_large_plan: tiles of tile_rows nodes, optional LDS halos, the
// depth-0 pool combined over tiles by 64-bit atomic max keys):
//   1. one 512-thread workgroup per tile: the tile's Zm rows (the mean over
//      out-neighbours, from halo-staged X rows), conv1 on MFMA with the same
//      operand order and bias add, relu, and the tile's share of the depth-0
//      max per (cluster, channel) as key (H bits << 32 | ~node) -- first max in
//      node order, NaN never enters, exactly the strict '>' scan; the Zm rows
//      (and SGAT's c1 in column XS) go to plan->z for the tail;
//   2. one 1024-thread workgroup per graph: decode the keys into P1 / A1 and
//      run fout_tail, reading x at the pooling args from the store and Zm / c1
//      from plan->z.  Bit-identical to fout_graph_kernel on graphs both run.
constexpr int NTA = 512;
constexpr int TRF = DR_LARGE_TILE;

struct FoutLargeArgs {
  FoutArgs f;
  dr_large_plan plan;
  int32_t zs;  // plan->z row stride: r4(F) (FoutNet) or r4(F) + 4 (SGAT: c1 in column r4(F))
};

struct FConvCarve {
  int KP, LDA, XS, w, b1, a, h, c1, m0i, m0p, flg, xh, hid, trp, ew, lcol, total;
};
__host__ __device__ inline FConvCarve fconv_carve(int N, int F, int K0, int HM, int EM, bool sg) {
  FConvCarve c;
  c.KP = r16(2 * F);
  c.LDA = c.KP + 4;  // lanes (row li, k + kq) of an operand read: banks 4 li + kq, distinct
  c.XS = r4(F);
  int o = 0;
#define TAKE(field, words) \
  c.field = o;             \
  o += r4(words);
  TAKE(w, c.KP * 16)
  TAKE(b1, 16)
  TAKE(a, TRF * c.LDA)  // [x_i | Zm_i | 0] per tile row
  TAKE(h, TRF * 16)
  TAKE(c1, sg ? TRF : 0)
  TAKE(m0i, HM ? TRF : N)
  TAKE(m0p, K0 + 1)
  TAKE(flg, TRF)  // per tile row: a depth-0 pooling arg candidate (its Zm row is stored)
  TAKE(xh, HM * c.XS)
  TAKE(hid, HM)
  TAKE(trp, HM ? TRF + 1 : 0)
  // last: the tile's edges as halo indices (uint16), then (SGAT) their weights
  // at lcol + r4((ne + 8) / 2) for the tile's ne edges -- so the kernel, which
  // carves with EM = 0, places them by its own tile's edge count
  TAKE(lcol, HM ? (EM + 8) / 2 : 0)
  TAKE(ew, (HM && sg) ? EM + 8 : 0)
#undef TAKE
  c.total = o;
  return c;
}

template <bool SG>
__global__ void __launch_bounds__(NTA) fout_large_conv1_kernel(FoutLargeArgs la) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const FoutArgs& a = la.f;
  const dr_large_plan& pl = la.plan;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tile = xcd_tile();
  const int b = pl.tile_slot[tile];
  const int t = tile - pl.tile_first[b];
  const dr_graph_desc d = a.descs[b];
  const dr_graph_store& s = a.s;
  const int g = d.gid;
  const int64_t n0 = d.node0, ec0 = d.col0, k00 = d.k0;
  const int N = d.n_nodes, K0 = d.n_k0, F = s.n_feat;
  const int TRr = pl.tile_rows;
  const int r0 = t * TRr, nrows = min(TRr, N - r0);
  const FConvCarve c = fconv_carve(N, F, K0, pl.halo_max, 0, SG);
  const int KP = c.KP, LDA = c.LDA, XS = c.XS, ZS = la.zs;
  float* sW = lds + c.w;
  float* sB1 = lds + c.b1;
  float* sA = lds + c.a;
  float* sH = lds + c.h;
  float* sC1 = lds + c.c1;
  int* sm0i = reinterpret_cast<int*>(lds + c.m0i);
  int* sm0p = reinterpret_cast<int*>(lds + c.m0p);
  // Zm (and SGAT's c1) go to global memory only at the tile's depth-0 pooling
  // arg candidates: the tail reads them only at the final args, tile args
  constexpr bool ZARGS = DR_Z_ARGS;
  int* sflag = reinterpret_cast<int*>(lds + c.flg);
  if (ZARGS)
    for (int p = tid; p < TRr; p += NTA) sflag[p] = 0;
  const bool compact = pl.tile_members != nullptr;
  if (compact) {  // this tile's members by cluster (host-built), runs from tile_mptr
    dma_words<NTA>(sm0i, pl.tile_members + (int64_t)tile * TRr, nrows);
    dma_words<NTA>(sm0p, pl.tile_mptr + (int64_t)tile * (pl.k0_max + 1), K0 + 1);
  } else {
    dma_words<NTA>(sm0i, s.m0_idx + n0, N);
    dma_words<NTA>(sm0p, s.m0_ptr + k00 + g, K0 + 1);
  }
  for (int p = tid; p < KP * 16; p += NTA) {  // [Wc; Wn; 0], k-major as stored
    const int k = p >> 4, o = p & 15;
    sW[p] = k < F ? a.w.wc1[k * 16 + o] : (k < 2 * F ? a.w.wn1[(k - F) * 16 + o] : 0.f);
  }
  if (tid < 16) sB1[tid] = a.w.b1[tid];
  // own rows x_i into the A tile (columns 0..F-1); pad columns past 2F: 0
  const float* X = s.x + n0 * (int64_t)XS;
  for (int p = tid; p < nrows * LDA; p += NTA) {
    const int r = p / LDA, k = p - r * LDA;
    if (k < F) sA[p] = X[(int64_t)(r0 + r) * XS + k];
    else if (k >= 2 * F) sA[p] = 0.f;
  }
  float* zg = pl.z + (int64_t)pl.z_row0[b] * ZS;
  // Zm = D^-1 A X for the tile's rows (SGAT: Zw, c1): 8 lanes per row, 16-byte chunks
  auto gather_rows = [&](const uint16_t* col, const float* ew, const float* Xs, const int* rowp, int ebase) {
    const int nch = XS >> 2, sub = tid & 7;
    for (int r = tid >> 3; r < nrows; r += NTA / 8) {
      const int eb = rowp[r] - ebase, ee = rowp[r + 1] - ebase;
      const float deg = SG ? (float)imax(ee - eb, 1) : (float)(ee - eb);
      for (int ch = sub; ch < nch; ch += 8) {
        const int c4 = ch * 4;
        float sw = 0.f;
        const float4 acc = SG ? gather_row_chunk_w(col, ew, eb, ee, Xs, XS, c4, sw) : gather_row_chunk(col, eb, ee, Xs, XS, c4);
        const float4 zm = make_float4(acc.x / deg, acc.y / deg, acc.z / deg, acc.w / deg);  // 0/0 = NaN (torch.mean(empty))
        const float zv[4] = {zm.x, zm.y, zm.z, zm.w};
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (c4 + q < F) sA[r * LDA + F + c4 + q] = zv[q];
        if (!ZARGS) *reinterpret_cast<float4*>(zg + (int64_t)(r0 + r) * ZS + c4) = zm;
        if (SG && ch == 0) {
          sC1[r] = sw / deg;
          if (!ZARGS) zg[(int64_t)(r0 + r) * ZS + XS] = sw / deg;
        }
      }
    }
  };
  if (pl.halo_ids) {  // halo path: the tile's neighbour X rows, edges and (SGAT) weights in LDS
    int* strp = reinterpret_cast<int*>(lds + c.trp);
    int* shid = reinterpret_cast<int*>(lds + c.hid);
    uint16_t* slcol = reinterpret_cast<uint16_t*>(lds + c.lcol);
    float* sXh = lds + c.xh;
    float* sEw;
    const int h0 = pl.halo_off[tile], H = pl.halo_off[tile + 1] - h0;
    dma_words<NTA>(strp, s.rowptr + n0 + g + r0, nrows + 1);
    dma_words<NTA>(shid, pl.halo_ids + h0, H);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int ebase = strp[0], ne = strp[nrows] - ebase;
    sEw = lds + c.lcol + r4((ne + 8) / 2);
    dma_x4<NTA>(slcol, pl.lcol + pl.lcol_off[tile], (ne + 7) / 8);
    if (SG) dma_words<NTA>(sEw, s.ea + ec0 + ebase, ne);  // Fe == 1: weights contiguous in CSR order
    {
      const int nch = XS >> 2, tot = H * nch;
      const int wv = __builtin_amdgcn_readfirstlane(wave);
      for (int base = wv * 64; base < tot; base += NTA)
        if (base + lane < tot) {
          const int hr = (base + lane) / nch, ch = base + lane - hr * nch;
          __builtin_amdgcn_global_load_lds(DRK_AS1(X + (int64_t)shid[hr] * XS + ch * 4), DRK_AS3(sXh + base * 4), 16, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    gather_rows(slcol, sEw, sXh, strp, ebase);
  } else {  // per-edge gather of X rows from HBM / L2
    gather_rows(s.col + ec0, SG ? s.ea + ec0 : nullptr, X, s.rowptr + n0 + g + r0, 0);
  }
  // (no wait for the Zm stores: the MFMA reads LDS; the tail reads Zm next launch)
  if (DR_TILE_STORE_WAIT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // conv1 on MFMA: H1 = relu([c1 x | Zm] [Wc; Wn] + b) -- fout_graph_kernel's operand order
  {
    const int li = lane & 15, kq = lane >> 4;
    for (int tt = wave; tt * 16 < nrows; tt += NTA / 64) {
      const int q0 = tt * 16;
      const int ar = min(q0 + li, nrows - 1);
      const float cx = SG ? sC1[ar] : 1.f;
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < KP; k += 16) {
        float av[4], bv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int kk = k + 4 * u + kq;
          av[u] = kk < F ? cx * sA[ar * LDA + kk] : sA[ar * LDA + kk];
          bv[u] = sW[kk * 16 + li];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = q0 + kq * 4 + r;
        if (row < nrows) sH[row * 16 + li] = relu_keepnan(acc[r] + sB1[li]);
      }
    }
  }
  __syncthreads();
  // the tile's share of the depth-0 max: members of each cluster inside the tile (a sub-run of its ascending list)
  for (int p = tid; p < K0 * 16; p += NTA) {
    const int k = p >> 4, ch = p & 15;
    int mb = sm0p[k], me = sm0p[k + 1];
    if (!compact) {
      int lo = mb, hi = me;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sm0i[mid] < r0) lo = mid + 1;
        else hi = mid;
      }
      mb = lo;
      hi = me;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sm0i[mid] < r0 + nrows) lo = mid + 1;
        else hi = mid;
      }
      me = lo;
    }
    float best = LOWEST;
    int arg = N;
    for (int m = mb; m < me; ++m) {
      const int i = sm0i[m];
      const float v = sH[(i - r0) * 16 + ch];
      if (v > best) {
        best = v;
        arg = i;
      }
    }
    if (ZARGS && arg < N) sflag[arg - r0] = 1;  // (benign race: every writer stores 1)
    if (best > LOWEST)
      __hip_atomic_fetch_max((__attribute__((address_space(1))) unsigned long long*)(pl.part_key) + ((int64_t)b * pl.k0_max + k) * 32 + ch,
                             ((unsigned long long)__float_as_uint(best) << 32) | (unsigned long long)(0xffffffffu - (uint32_t)arg),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (ZARGS) {  // the flagged rows' Zm (from the A tile's columns F..2F-1) and c1
    __syncthreads();
    const int nch = XS >> 2;
    for (int p = tid; p < nrows * nch; p += NTA) {
      const int r = p / nch, c4 = (p - r * nch) * 4;
      if (sflag[r]) {
        const float* zr = sA + r * LDA + F + c4;
        *reinterpret_cast<float4*>(zg + (int64_t)(r0 + r) * ZS + c4) =
            make_float4(zr[0], c4 + 1 < F ? zr[1] : 0.f, c4 + 2 < F ? zr[2] : 0.f, c4 + 3 < F ? zr[3] : 0.f);
        if (SG && c4 == 0) zg[(int64_t)(r0 + r) * ZS + XS] = sC1[r];
      }
    }
  }
}

struct FTailCarve {
  int w2, fc1, fc2, p1, a1, dp1, zm2, s2, h2, d2, dz2, p1rp, p1c, p1trp, p1tc, m1p, m1i, p2, nt, head, dgp, p1w, p1tid, c2, total;
};
__host__ __device__ inline FTailCarve ftail_carve(int K0, int P1, int K1, int alias, int OUT, bool sg) {
  FTailCarve c;
  int o = 0;
#define TAKE(field, words) \
  c.field = o;             \
  o += r4(words);
  TAKE(w2, 16 * 32 * 2 + 32 + 16)
  TAKE(fc1, 64 * 32 + 64)
  TAKE(fc2, OUT * 64 + OUT)
  TAKE(p1, K0 * 16)
  TAKE(a1, K0 * 16)
  TAKE(dp1, K0 * 16)
  TAKE(zm2, K0 * 16)
  TAKE(s2, K0 * 32)
  TAKE(h2, K0 * 32)
  TAKE(d2, K0 * 32)
  TAKE(dz2, K0 * 16)
  TAKE(p1rp, K0 + 1)
  TAKE(p1c, P1)
  if (alias) {
    c.p1trp = c.p1rp;
    c.p1tc = c.p1c;
  } else {
    TAKE(p1trp, K0 + 1)
    TAKE(p1tc, P1)
  }
  TAKE(m1p, K1 + 1)
  TAKE(m1i, K0)
  TAKE(p2, K1 * 32)
  TAKE(nt, K1 * 32)
  TAKE(head, HEADW)
  TAKE(dgp, NW * 64)
  TAKE(p1w, sg ? P1 : 0)
  TAKE(p1tid, sg ? P1 : 0)
  TAKE(c2, sg ? K0 : 0)
#undef TAKE
  c.total = o;
  return c;
}

template <bool SG>
__global__ void __launch_bounds__(NT) fout_large_tail_kernel(FoutLargeArgs la) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const FoutArgs& a = la.f;
  const dr_large_plan& pl = la.plan;
  const int tid = threadIdx.x;
  const int b = blockIdx.x;
  const dr_graph_store& s = a.s;
  const dr_graph_desc d = a.descs[b];
  const int g = d.gid;
  const int64_t n0 = d.node0, k00 = d.k0, q0 = d.p1, k10 = d.k1;
  const int N = d.n_nodes, K0 = d.n_k0, P1 = d.n_p1, K1 = d.n_k1;
  const int F = s.n_feat, alias = s.transpose_aliased, OUT = a.p.out_dim, XS = r4(F), ZS = la.zs;
  const FTailCarve c = ftail_carve(K0, P1, K1, alias, OUT, SG);
  FoutTail t;
  float* w2 = lds + c.w2;
  t.Wc2 = w2;
  t.Wn2 = w2 + 512;
  t.B2 = w2 + 1024;
  t.Fc1 = lds + c.fc1;
  t.Fc1b = lds + c.fc1 + 2048;
  t.Fc2 = lds + c.fc2;
  t.P1 = lds + c.p1;
  t.A1 = reinterpret_cast<int*>(lds + c.a1);
  t.dP1 = lds + c.dp1;
  t.Zm2 = lds + c.zm2;
  t.S2 = lds + c.s2;
  t.H2 = lds + c.h2;
  t.D2 = lds + c.d2;
  t.Dz2 = lds + c.dz2;
  t.p1rp = reinterpret_cast<int*>(lds + c.p1rp);
  t.p1c = reinterpret_cast<int*>(lds + c.p1c);
  t.p1trp = reinterpret_cast<int*>(lds + c.p1trp);
  t.p1tc = reinterpret_cast<int*>(lds + c.p1tc);
  t.m1p = reinterpret_cast<int*>(lds + c.m1p);
  t.m1i = reinterpret_cast<int*>(lds + c.m1i);
  t.P2 = lds + c.p2;
  t.NTie = lds + c.nt;
  t.G = lds + c.head;
  t.Hpre = t.G + 32;
  t.Hh = t.Hpre + 64;
  t.Dh = t.Hh + 64;
  t.DG = t.Dh + 64;
  t.Dout = t.DG + 32;
  t.DGp = lds + c.dgp;
  t.P1w = lds + c.p1w;
  t.P1tid = reinterpret_cast<int*>(lds + c.p1tid);
  t.C2 = lds + c.c2;
  const float y_g = s.y[g];
  dma_words<NT>(t.p1rp, s.p1_rowptr + k00 + g, K0 + 1);
  dma_words<NT>(t.p1c, s.p1_col + q0, P1);
  if (!alias) {
    dma_words<NT>(t.p1trp, s.p1t_rowptr + k00 + g, K0 + 1);
    dma_words<NT>(t.p1tc, s.p1t_col + q0, P1);
  }
  dma_words<NT>(t.m1p, s.m1_ptr + k10 + g, K1 + 1);
  dma_words<NT>(t.m1i, s.m1_idx + k00, K0);
  if (SG) {
    dma_words<NT>(t.P1w, s.p1_ea + q0, P1);
    dma_words<NT>(t.P1tid, s.p1t_pid + q0, P1);
  }
  for (int p = tid; p < 1072; p += NT) {
    const int q = p;
    w2[p] = q < 512 ? a.w.wc2[q] : q < 1024 ? a.w.wn2[q - 512] : q < 1056 ? a.w.b2[q - 1024] : a.w.b1[q - 1056];
  }
  for (int p = tid; p < 2048 + 64; p += NT) lds[c.fc1 + p] = p < 2048 ? a.w.fc1w[p] : a.w.fc1b[p - 2048];
  for (int p = tid; p < OUT * 65; p += NT) lds[c.fc2 + p] = p < OUT * 64 ? a.w.fc2w[p] : a.w.fc2b[p - OUT * 64];
  for (int p = tid; p < K0 * 16; p += NT) {  // the depth-0 pool from the tiles' keys (and the keys back to zero)
    unsigned long long* kp = reinterpret_cast<unsigned long long*>(pl.part_key) + ((int64_t)b * pl.k0_max + (p >> 4)) * 32 + (p & 15);
    const unsigned long long key = *kp;
    *kp = 0ull;
    t.P1[p] = key ? __uint_as_float((uint32_t)(key >> 32)) : 0.f;
    t.A1[p] = key ? (int)(0xffffffffu - (uint32_t)key) : N;
  }
  const int64_t counter0 = (a.p.step_counter && b == 0) ? a.p.step_counter[0] : 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (a.p.step_counter && b == 0 && tid == 0) a.p.step_counter[1] = counter0;  // snapshot for dr_reduce_update
  __syncthreads();
  const float* X = s.x + n0 * (int64_t)XS;
  const float* z = pl.z + (int64_t)pl.z_row0[b] * ZS;
  fout_tail<SG>(a.p, t, a.p.slot ? a.p.slot[b] : b, N, K0, K1, F, OUT, y_g,
                [=](int i, int kk) { return (SG ? z[(int64_t)i * ZS + XS] : 1.f) * X[(int64_t)i * XS + kk]; },
                [=](int i, int kk) { return z[(int64_t)i * ZS + kk]; });
}

}  // namespace

namespace {

int fout_family_pass(bool sg, const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                     const dr_fout_weights* w, const dr_pass* pass, int32_t lds_bytes, void* stream) {
  if (!store || !descs || !w || !pass || n_batch < 0) return DR_E_ARG;
  if (sg && (store->n_edge_feat != 1 || !store->ea || !store->p1_ea || !store->p1t_pid)) return DR_E_UNSUPPORTED;
  if (pass->out_dim < 1 || pass->out_dim > DR_MAX_OUT) return DR_E_UNSUPPORTED;
  if (store->n_feat < 1 || 2 * 16 * store->n_feat + 1072 + 2112 + 65 * pass->out_dim > 6 * NT) return DR_E_UNSUPPORTED;
  if (lds_bytes > 160 * 1024) return DR_E_LDS;
  if ((pass->flags & DR_PASS_BACKWARD) && (!pass->slab || !pass->head)) return DR_E_ARG;
  if ((pass->flags & DR_PASS_BACKWARD) && pass->loss_kind == DR_LOSS_NONE && !pass->dout) return DR_E_ARG;
  if ((pass->flags & DR_PASS_FORWARD) && !pass->out) return DR_E_ARG;
  if (pass->use_dropout != DR_DROPOUT_OFF) return DR_E_UNSUPPORTED;  // FoutNet / SGAT have no dropout
  if (n_batch == 0) return DR_OK;
  const void* fn = sg ? reinterpret_cast<const void*>(&fout_graph_kernel<true>)
                      : reinterpret_cast<const void*>(&fout_graph_kernel<false>);
  DR_CHECK(dr_allow_big_lds(fn));
  FoutArgs args;
  args.s = *store;
  args.w = *w;
  args.p = *pass;
  args.descs = descs;
  args.B = n_batch;
  args.lds_bytes = lds_bytes;
  if (sg)
    hipLaunchKernelGGL(fout_graph_kernel<true>, dim3(n_batch), dim3(NT), lds_bytes, (hipStream_t)stream, args);
  else
    hipLaunchKernelGGL(fout_graph_kernel<false>, dim3(n_batch), dim3(NT), lds_bytes, (hipStream_t)stream, args);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" int64_t dr_fout_lds_bytes(int32_t n_nodes, int32_t n_edges, int32_t n_feat, int32_t k0, int32_t p1_edges,
                                     int32_t k1, int32_t transpose_aliased, int32_t out_dim) {
  return 4LL * carve(n_nodes, n_edges, n_feat, k0, p1_edges, k1, transpose_aliased, out_dim, false).total;
}

extern "C" int64_t dr_sgat_lds_bytes(int32_t n_nodes, int32_t n_edges, int32_t n_feat, int32_t k0, int32_t p1_edges,
                                     int32_t k1, int32_t transpose_aliased, int32_t out_dim) {
  return 4LL * carve(n_nodes, n_edges, n_feat, k0, p1_edges, k1, transpose_aliased, out_dim, true).total;
}

extern "C" int dr_fout_graph_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                                  const dr_fout_weights* w, const dr_pass* pass, int32_t lds_bytes, void* stream) {
  return fout_family_pass(false, store, descs, n_batch, w, pass, lds_bytes, stream);
}

extern "C" int dr_sgat_graph_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                                  const dr_fout_weights* w, const dr_pass* pass, int32_t lds_bytes, void* stream) {
  return fout_family_pass(true, store, descs, n_batch, w, pass, lds_bytes, stream);
}

extern "C" int64_t dr_fout_large_conv_lds_bytes(int32_t n_nodes, int32_t n_feat, int32_t k0, int32_t halo_max,
                                                int32_t tile_edges_max, int32_t sgat) {
  return 4LL * fconv_carve(n_nodes, n_feat, k0, halo_max, tile_edges_max, sgat != 0).total;
}

extern "C" int64_t dr_fout_tail_lds_bytes(int32_t k0, int32_t p1_edges, int32_t k1, int32_t transpose_aliased,
                                          int32_t out_dim, int32_t sgat) {
  return 4LL * ftail_carve(k0, p1_edges, k1, transpose_aliased, out_dim, sgat != 0).total;
}

namespace {
int fout_large_family(bool sg, const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                      const dr_large_plan* plan, const dr_fout_weights* w, const dr_pass* pass, int32_t z_stride,
                      int32_t conv_lds_bytes, int32_t tail_lds_bytes, void* stream) {
  if (!store || !descs || !w || !pass || !plan || n_batch < 0) return DR_E_ARG;
  if (sg && (store->n_edge_feat != 1 || !store->ea || !store->p1_ea || !store->p1t_pid)) return DR_E_UNSUPPORTED;
  if (pass->out_dim < 1 || pass->out_dim > DR_MAX_OUT) return DR_E_UNSUPPORTED;
  if (store->n_feat < 1 || store->n_feat > 64) return DR_E_UNSUPPORTED;
  const int XS = (store->n_feat + 3) & ~3;
  if (z_stride != (sg ? XS + 4 : XS)) return DR_E_ARG;
  if (conv_lds_bytes > 160 * 1024 || tail_lds_bytes > 160 * 1024) return DR_E_LDS;
  if (!plan->tile_first || !plan->z_row0 || !plan->tile_slot || !plan->z || !plan->part_key) return DR_E_ARG;
  if (plan->n_tiles < n_batch || plan->k0_max < 1 || plan->k0_max > 64 || plan->arrive) return DR_E_ARG;
  if (plan->tile_rows < 16 || plan->tile_rows > TRF || plan->tile_rows % 16) return DR_E_ARG;
  if (plan->halo_ids && (plan->halo_max < 1 || plan->halo_max > 65535 || !plan->halo_off || !plan->lcol_off ||
                         !plan->lcol || !plan->tile_members || !plan->tile_mptr))
    return DR_E_ARG;
  if (!plan->halo_ids && plan->halo_max) return DR_E_ARG;
  if ((pass->flags & DR_PASS_BACKWARD) && (!pass->slab || !pass->head)) return DR_E_ARG;
  if ((pass->flags & DR_PASS_BACKWARD) && pass->loss_kind == DR_LOSS_NONE && !pass->dout) return DR_E_ARG;
  if ((pass->flags & DR_PASS_FORWARD) && !pass->out) return DR_E_ARG;
  if (pass->use_dropout != DR_DROPOUT_OFF || pass->compute_dtype != DR_DTYPE_F32) return DR_E_UNSUPPORTED;
  if (n_batch == 0) return DR_OK;
  const void* conv = sg ? reinterpret_cast<const void*>(&fout_large_conv1_kernel<true>) : reinterpret_cast<const void*>(&fout_large_conv1_kernel<false>);
  const void* tail = sg ? reinterpret_cast<const void*>(&fout_large_tail_kernel<true>) : reinterpret_cast<const void*>(&fout_large_tail_kernel<false>);
  DR_CHECK(dr_allow_big_lds(conv));
  DR_CHECK(dr_allow_big_lds(tail));
  FoutLargeArgs la;
  la.f.s = *store;
  la.f.w = *w;
  la.f.p = *pass;
  la.f.descs = descs;
  la.f.B = n_batch;
  la.f.lds_bytes = tail_lds_bytes;
  la.plan = *plan;
  la.zs = z_stride;
  hipStream_t st = (hipStream_t)stream;
  if (sg) {
    hipLaunchKernelGGL(fout_large_conv1_kernel<true>, dim3(plan->n_tiles), dim3(NTA), conv_lds_bytes, st, la);
    hipLaunchKernelGGL(fout_large_tail_kernel<true>, dim3(n_batch), dim3(NT), tail_lds_bytes, st, la);
  } else {
    hipLaunchKernelGGL(fout_large_conv1_kernel<false>, dim3(plan->n_tiles), dim3(NTA), conv_lds_bytes, st, la);
    hipLaunchKernelGGL(fout_large_tail_kernel<false>, dim3(n_batch), dim3(NT), tail_lds_bytes, st, la);
  }
  return (int)hipGetLastError();
}
}  // namespace

extern "C" int dr_fout_large_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                                  const dr_large_plan* plan, const dr_fout_weights* w, const dr_pass* pass,
                                  int32_t z_stride, int32_t conv_lds_bytes, int32_t tail_lds_bytes, void* stream) {
  return fout_large_family(false, store, descs, n_batch, plan, w, pass, z_stride, conv_lds_bytes, tail_lds_bytes, stream);
}

extern "C" int dr_sgat_large_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                                  const dr_large_plan* plan, const dr_fout_weights* w, const dr_pass* pass,
                                  int32_t z_stride, int32_t conv_lds_bytes, int32_t tail_lds_bytes, void* stream) {
  return fout_large_family(true, store, descs, n_batch, plan, w, pass, z_stride, conv_lds_bytes, tail_lds_bytes, stream);
}

// ---- carve descriptions for the host-side carve tests (tests/test_lds_carves.py)
extern "C" int dr_debug_carve_fout(const int32_t* q, char* buf, int32_t len) {
  const Carve c = carve(q[0], q[1], q[2], q[3], q[4], q[5], q[6], q[7], q[8] != 0, q[9]);
  DrCarveDesc d{buf, len, 0};
  DR_DESC_P(d, c, KP);
  DR_DESC_P(d, c, XS);
  DR_DESC_P(d, c, LDZ);
  DR_DESC_P(d, c, wide);
  DR_DESC(d, c, ea);
  DR_DESC(d, c, c1);
  DR_DESC(d, c, p1w);
  DR_DESC(d, c, p1tid);
  DR_DESC(d, c, c2);
  DR_DESC(d, c, wc1);
  DR_DESC(d, c, w2);
  DR_DESC(d, c, fc1);
  DR_DESC(d, c, fc2);
  DR_DESC(d, c, x);
  DR_DESC(d, c, zm);
  DR_DESC(d, c, h1);
  DR_DESC(d, c, rp);
  DR_DESC(d, c, col);
  DR_DESC(d, c, m0p);
  DR_DESC(d, c, m0i);
  DR_DESC(d, c, p1);
  DR_DESC(d, c, a1);
  DR_DESC(d, c, dp1);
  DR_DESC(d, c, zm2);
  DR_DESC(d, c, s2);
  DR_DESC(d, c, h2);
  DR_DESC(d, c, d2);
  DR_DESC(d, c, dz2);
  DR_DESC(d, c, p1rp);
  DR_DESC(d, c, p1c);
  DR_DESC(d, c, p1trp);
  DR_DESC(d, c, p1tc);
  DR_DESC(d, c, m1p);
  DR_DESC(d, c, m1i);
  DR_DESC(d, c, p2);
  DR_DESC(d, c, nt);
  DR_DESC(d, c, head);
  DR_DESC(d, c, dgp);
  DR_DESC(d, c, red);
  DR_DESC(d, c, total);
  return d.pos;
}

extern "C" int dr_debug_carve_fout_conv(const int32_t* q, char* buf, int32_t len) {
  const FConvCarve c = fconv_carve(q[0], q[1], q[2], q[3], q[4], q[5] != 0);
  DrCarveDesc d{buf, len, 0};
  DR_DESC_P(d, c, KP);
  DR_DESC_P(d, c, LDA);
  DR_DESC_P(d, c, XS);
  DR_DESC(d, c, w);
  DR_DESC(d, c, b1);
  DR_DESC(d, c, a);
  DR_DESC(d, c, h);
  DR_DESC(d, c, c1);
  DR_DESC(d, c, m0i);
  DR_DESC(d, c, m0p);
  DR_DESC(d, c, flg);
  DR_DESC(d, c, xh);
  DR_DESC(d, c, hid);
  DR_DESC(d, c, trp);
  DR_DESC(d, c, ew);
  DR_DESC(d, c, lcol);
  DR_DESC(d, c, total);
  return d.pos;
}

extern "C" int dr_debug_carve_fout_tail(const int32_t* q, char* buf, int32_t len) {
  const FTailCarve c = ftail_carve(q[0], q[1], q[2], q[3], q[4], q[5] != 0);
  DrCarveDesc d{buf, len, 0};
  DR_DESC(d, c, w2);
  DR_DESC(d, c, fc1);
  DR_DESC(d, c, fc2);
  DR_DESC(d, c, p1);
  DR_DESC(d, c, a1);
  DR_DESC(d, c, dp1);
  DR_DESC(d, c, zm2);
  DR_DESC(d, c, s2);
  DR_DESC(d, c, h2);
  DR_DESC(d, c, d2);
  DR_DESC(d, c, dz2);
  DR_DESC(d, c, p1rp);
  DR_DESC(d, c, p1c);
  DR_DESC(d, c, p1trp);
  DR_DESC(d, c, p1tc);
  DR_DESC(d, c, m1p);
  DR_DESC(d, c, m1i);
  DR_DESC(d, c, p2);
  DR_DESC(d, c, nt);
  DR_DESC(d, c, head);
  DR_DESC(d, c, dgp);
  DR_DESC(d, c, p1w);
  DR_DESC(d, c, p1tid);
  DR_DESC(d, c, c2);
  DR_DESC(d, c, total);
  return d.pos;
}

