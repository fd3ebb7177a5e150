// GINet training step, one workgroup per graph, everything resident in LDS.
//
// Replaces (deeprank2 v3.1.0):
//   GINetConvLayer.forward        deeprank2/neuralnets/gnn/ginet.py:40-60
//   GINet.forward                 ginet.py:90-125
//   get_preloaded_cluster         deeprank2/utils/community_pooling.py:23-27
//   community_pooling             community_pooling.py:165-242
//   max_pool_x / scatter_mean     ginet.py:103,114,117-118
//   autograd backward + loss      deeprank2/trainer.py:686-689
//
// Algebra used (all exact):
//   * the attention of ginet.py:48-55 is softmax over a size-1 dim, i.e. 1 for
//     every finite logit, so conv(x) = A·(x Wᵀ) with A[i,j] = #edges (i→j);
//     its parameters get exact-zero gradients (done by the reduce kernel);
//   * both branches see the same graph (data.clone(), ginet.py:92), so conv1
//     and conv1_ext are one GEMM with W = [W1; W1e] (32 outputs);
//   * per-batch cluster offsetting + consecutive_cluster is, graph by graph, a
//     dense relabelling of that graph's ids (precomputed into the store), and
//     pool_edge's coalesced pooled graph is precomputed as a CSR too.
//
// LDS holds X, Y=XWᵀ, H=relu(AY), the CSR, cluster member lists, the pooled
// graph and the head; the backward re-uses the Y/H regions for dY/dS.
// Roofline: HBM-bound on the compulsory inputs (x, CSR, clusters) — see
// DESIGN.md §Kernels for the algorithmic bytes per graph.

#include <hip/hip_runtime.h>

#include "../../include/deeprank2_amd.h"
#include "dr_common.h"

namespace {

constexpr int NT = 256;      // 4 waves
constexpr int HEADW = 672;   // G64 hpre128 hh128 hd128 dh128 dG64 dout16 spare16

struct Carve {
  int wt, x, y, h, rp, col, trp, tcol, m0p, m0i, p1, a1, dp1, y2, h2, d2, p1rp, p1c, p1trp, p1tc, m1p, m1i, p2,
      nt, head, red, total;
};

__host__ __device__ inline int r4(int v) { return (v + 3) & ~3; }

__host__ __device__ inline Carve carve(int N, int E, int F, int K0, int P1, int K1, int alias) {
  const int LDX = r4(F);
  Carve c;
  int o = 0;
#define TAKE(field, words) \
  c.field = o;             \
  o += r4(words);
  TAKE(wt, LDX * 32)
  TAKE(x, N * LDX)
  TAKE(y, N * 32)
  TAKE(h, N * 32)
  TAKE(rp, N + 1)
  TAKE(col, E)
  if (alias) {
    c.trp = c.rp;
    c.tcol = c.col;
  } else {
    TAKE(trp, N + 1)
    TAKE(tcol, E)
  }
  TAKE(m0p, K0 + 1)
  TAKE(m0i, N)
  TAKE(p1, K0 * 32)
  TAKE(a1, K0 * 32)
  TAKE(dp1, K0 * 32)
  TAKE(y2, K0 * 64)
  TAKE(h2, K0 * 64)
  TAKE(d2, K0 * 64)
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
  TAKE(p2, K1 * 64)
  TAKE(nt, K1 * 64)
  TAKE(head, HEADW)
  TAKE(red, 4 * 32 * LDX)
#undef TAKE
  c.total = o;
  return c;
}

struct GinetArgs {
  dr_graph_store s;
  dr_ginet_weights w;
  dr_ginet_pass p;
  const int32_t* gids;
  int32_t B;
};

// torch relu keeps NaN (clamp_min propagates it); its backward masks where
// the output is <= 0 (threshold_backward), so a NaN output passes the grad.
__device__ __forceinline__ float relu_keepnan(float v) { return (v <= 0.f) ? 0.f : v; }
__device__ __forceinline__ float relu_bwd(float out, float g) { return (out <= 0.f) ? 0.f : g; }

template <typename T>
__device__ __forceinline__ void copy_in(T* dst, const T* __restrict__ src, int n) {
  for (int i = threadIdx.x; i < n; i += NT) dst[i] = src[i];
}

__global__ void __launch_bounds__(NT) ginet_graph_kernel(GinetArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x;
  const int b = blockIdx.x;
  const dr_graph_store& s = a.s;
  const int g = a.gids[b];
  const int64_t n0 = s.node_off[g];
  const int N = (int)(s.node_off[g + 1] - n0);
  const int64_t e0 = s.edge_off[g];
  const int E = (int)(s.edge_off[g + 1] - e0);
  const int64_t k00 = s.k0_off[g];
  const int K0 = (int)(s.k0_off[g + 1] - k00);
  const int64_t q0 = s.p1_off[g];
  const int P1 = (int)(s.p1_off[g + 1] - q0);
  const int64_t k10 = s.k1_off[g];
  const int K1 = (int)(s.k1_off[g + 1] - k10);
  const int F = s.n_feat;
  const int LDX = r4(F);
  const int alias = s.transpose_aliased;
  const Carve c = carve(N, E, F, K0, P1, K1, alias);
  const int OUT = a.p.out_dim;

  float* sWT = lds + c.wt;
  float* sX = lds + c.x;
  float* sY = lds + c.y;
  float* sH = lds + c.h;
  int* srp = reinterpret_cast<int*>(lds + c.rp);
  int* scol = reinterpret_cast<int*>(lds + c.col);
  int* strp = reinterpret_cast<int*>(lds + c.trp);
  int* stcol = reinterpret_cast<int*>(lds + c.tcol);
  int* sm0p = reinterpret_cast<int*>(lds + c.m0p);
  int* sm0i = reinterpret_cast<int*>(lds + c.m0i);
  float* sP1 = lds + c.p1;
  int* sA1 = reinterpret_cast<int*>(lds + c.a1);
  float* sdP1 = lds + c.dp1;
  float* sY2 = lds + c.y2;
  float* sH2 = lds + c.h2;
  float* sD2 = lds + c.d2;
  int* sp1rp = reinterpret_cast<int*>(lds + c.p1rp);
  int* sp1c = reinterpret_cast<int*>(lds + c.p1c);
  int* sp1trp = reinterpret_cast<int*>(lds + c.p1trp);
  int* sp1tc = reinterpret_cast<int*>(lds + c.p1tc);
  int* sm1p = reinterpret_cast<int*>(lds + c.m1p);
  int* sm1i = reinterpret_cast<int*>(lds + c.m1i);
  float* sP2 = lds + c.p2;
  float* sNT = lds + c.nt;
  float* sG = lds + c.head;
  float* sHpre = sG + 64;
  float* sHh = sHpre + 128;
  float* sHd = sHh + 128;
  float* sDh = sHd + 128;
  float* sDG = sDh + 128;
  float* sDout = sDG + 64;
  float* sRed = lds + c.red;

  // ---------------- stage the graph into LDS --------------------------------
  for (int p = tid; p < LDX * 32; p += NT) {
    const int k = p >> 5, ch = p & 31;
    float v = 0.f;
    if (k < F) v = (ch < 16) ? a.w.w1[ch * F + k] : a.w.w1e[(ch - 16) * F + k];
    sWT[p] = v;
  }
  {
    const float* __restrict__ xg = s.x + n0 * (int64_t)F;
    for (int p = tid; p < N * F; p += NT) {
      const int i = p / F;
      const int k = p - i * F;
      sX[i * LDX + k] = xg[p];
    }
    const int padw = LDX - F;
    if (padw > 0)
      for (int p = tid; p < N * padw; p += NT) {
        const int i = p / padw;
        sX[i * LDX + F + (p - i * padw)] = 0.f;
      }
  }
  copy_in(srp, s.rowptr + n0 + g, N + 1);
  copy_in(scol, s.col + e0, E);
  if (!alias) {
    copy_in(strp, s.t_rowptr + n0 + g, N + 1);
    copy_in(stcol, s.t_col + e0, E);
  }
  copy_in(sm0p, s.m0_ptr + k00 + g, K0 + 1);
  copy_in(sm0i, s.m0_idx + n0, N);
  copy_in(sp1rp, s.p1_rowptr + k00 + g, K0 + 1);
  copy_in(sp1c, s.p1_col + q0, P1);
  if (!alias) {
    copy_in(sp1trp, s.p1t_rowptr + k00 + g, K0 + 1);
    copy_in(sp1tc, s.p1t_col + q0, P1);
  }
  copy_in(sm1p, s.m1_ptr + k10 + g, K1 + 1);
  copy_in(sm1i, s.m1_idx + k00, K0);
  __syncthreads();

  // ---------------- conv1 node GEMM: Y = X [W1;W1e]^T  (ginet.py:45) --------
  {
    const int ch = tid & 31, rg = tid >> 5;
    for (int base = 0; base < N; base += 32) {
      const int r0 = base + rg * 4;
      const int ra = min(r0, N - 1), rb = min(r0 + 1, N - 1), rc = min(r0 + 2, N - 1), rd = min(r0 + 3, N - 1);
      float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
      for (int k = 0; k < LDX; k += 4) {
        const float w0 = sWT[(k + 0) * 32 + ch], w1 = sWT[(k + 1) * 32 + ch];
        const float w2 = sWT[(k + 2) * 32 + ch], w3 = sWT[(k + 3) * 32 + ch];
        const float4 xa = *reinterpret_cast<const float4*>(&sX[ra * LDX + k]);
        const float4 xb = *reinterpret_cast<const float4*>(&sX[rb * LDX + k]);
        const float4 xc = *reinterpret_cast<const float4*>(&sX[rc * LDX + k]);
        const float4 xd = *reinterpret_cast<const float4*>(&sX[rd * LDX + k]);
        acc0 = fmaf(xa.x, w0, acc0); acc0 = fmaf(xa.y, w1, acc0); acc0 = fmaf(xa.z, w2, acc0); acc0 = fmaf(xa.w, w3, acc0);
        acc1 = fmaf(xb.x, w0, acc1); acc1 = fmaf(xb.y, w1, acc1); acc1 = fmaf(xb.z, w2, acc1); acc1 = fmaf(xb.w, w3, acc1);
        acc2 = fmaf(xc.x, w0, acc2); acc2 = fmaf(xc.y, w1, acc2); acc2 = fmaf(xc.z, w2, acc2); acc2 = fmaf(xc.w, w3, acc2);
        acc3 = fmaf(xd.x, w0, acc3); acc3 = fmaf(xd.y, w1, acc3); acc3 = fmaf(xd.z, w2, acc3); acc3 = fmaf(xd.w, w3, acc3);
      }
      if (r0 < N) sY[r0 * 32 + ch] = acc0;
      if (r0 + 1 < N) sY[(r0 + 1) * 32 + ch] = acc1;
      if (r0 + 2 < N) sY[(r0 + 2) * 32 + ch] = acc2;
      if (r0 + 3 < N) sY[(r0 + 3) * 32 + ch] = acc3;
    }
  }
  __syncthreads();

  // ---------------- conv1 aggregation + relu: H = relu(A Y)  (ginet.py:58,96)
  {
    const int c4 = (tid & 7) * 4;
    for (int i = tid >> 3; i < N; i += NT / 8) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      const int eb = srp[i], ee = srp[i + 1];
      for (int e = eb; e < ee; ++e) {
        const float4 v = *reinterpret_cast<const float4*>(&sY[scol[e] * 32 + c4]);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
      float4 o;
      o.x = relu_keepnan(acc.x); o.y = relu_keepnan(acc.y); o.z = relu_keepnan(acc.z); o.w = relu_keepnan(acc.w);
      *reinterpret_cast<float4*>(&sH[i * 32 + c4]) = o;
    }
  }
  __syncthreads();

  // ---------------- depth-0 community pooling: torch_scatter scatter_max ----
  // (community_pooling.py:209): strict '>' from lowest(), members in node
  // order => first max wins, NaN never enters, empty -> 0 with no arg.
  for (int p = tid; p < K0 * 32; p += NT) {
    const int k = p >> 5, ch = p & 31;
    float best = -3.402823466e+38f;
    int arg = N;
    for (int m = sm0p[k]; m < sm0p[k + 1]; ++m) {
      const int i = sm0i[m];
      const float v = sH[i * 32 + ch];
      if (v > best) {
        best = v;
        arg = i;
      }
    }
    if (best == -3.402823466e+38f) best = 0.f;
    sP1[p] = best;
    sA1[p] = arg;
  }
  __syncthreads();

  // ---------------- conv2 node GEMM on the pooled graph (ginet.py:101,112) --
  for (int p = tid; p < K0 * 64; p += NT) {
    const int k = p >> 6, o = p & 63, br = o >> 5;
    const float* __restrict__ wr = br ? (a.w.w2e + (o - 32) * 16) : (a.w.w2 + o * 16);
    const float* pr = sP1 + k * 32 + br * 16;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) acc = fmaf(pr[j], wr[j], acc);
    sY2[p] = acc;
  }
  __syncthreads();
  for (int p = tid; p < K0 * 64; p += NT) {
    const int k = p >> 6, o = p & 63;
    float acc = 0.f;
    for (int e = sp1rp[k]; e < sp1rp[k + 1]; ++e) acc += sY2[sp1c[e] * 64 + o];
    sH2[p] = relu_keepnan(acc);
  }
  __syncthreads();

  // ---------------- depth-1 max_pool_x: scatter_reduce amax (ginet.py:103) --
  // NaN propagates; remember the tie count for the even-split backward.
  for (int p = tid; p < K1 * 64; p += NT) {
    const int m = p >> 6, o = p & 63;
    const int mb = sm1p[m], me = sm1p[m + 1];
    float mx = sH2[sm1i[mb] * 64 + o];
    for (int q = mb + 1; q < me; ++q) {
      const float v = sH2[sm1i[q] * 64 + o];
      mx = (mx != mx || v != v) ? __int_as_float(0x7fc00000) : fmaxf(mx, v);
    }
    float ties = 0.f;
    for (int q = mb; q < me; ++q) ties += (sH2[sm1i[q] * 64 + o] == mx) ? 1.f : 0.f;
    sP2[p] = mx;
    sNT[p] = ties;
  }
  __syncthreads();

  // ---------------- per-graph mean (scatter_mean, ginet.py:117-118) ----------
  if (tid < 64) {
    float acc = 0.f;
    for (int m = 0; m < K1; ++m) acc += sP2[m * 64 + tid];
    sG[tid] = acc / (float)K1;
  }
  __syncthreads();

  // ---------------- head: fc1 -> relu -> dropout -> fc2 (ginet.py:120-123) --
  if (tid < 128) {
    const float* __restrict__ wr = a.w.fc1w + tid * 64;
    float acc = 0.f;
    for (int o = 0; o < 64; ++o) acc = fmaf(sG[o], wr[o], acc);
    acc += a.w.fc1b[tid];
    sHpre[tid] = acc;
    const float hh = relu_keepnan(acc);
    sHh[tid] = hh;
    float hd = hh;
    if (a.p.use_dropout) hd = (a.p.mask[(int64_t)b * 128 + tid] ? hh : 0.f) * a.p.drop_scale;
    sHd[tid] = hd;
  }
  __syncthreads();
  {
    const int wave = tid >> 6, lane = tid & 63;
    for (int q = wave; q < OUT; q += NT / 64) {
      const float* __restrict__ wr = a.w.fc2w + q * 128;
      float v = fmaf(sHd[lane], wr[lane], sHd[lane + 64] * wr[lane + 64]);
      v = dr_wave_sum(v);
      if (lane == 0) sDout[q] = v + a.w.fc2b[q];  // logits parked in sDout
    }
  }
  __syncthreads();
  if ((a.p.flags & DR_PASS_FORWARD) && tid < OUT) a.p.out[(int64_t)b * OUT + tid] = sDout[tid];
  if (!(a.p.flags & DR_PASS_BACKWARD)) return;
  __syncthreads();

  // ---------------- loss gradient (trainer.py:688-689) ----------------------
  if (tid == 0) {
    const int yrow = g;
    if (a.p.loss_kind == DR_LOSS_MSE) {
      const float d = sDout[0] - s.y[yrow];
      if (a.p.loss_per_graph) a.p.loss_per_graph[b] = d * d;
      sDout[0] = 2.f * d * a.p.loss_scale;
    } else if (a.p.loss_kind == DR_LOSS_CE) {
      const int yi = (int)s.y[yrow];
      float mx = sDout[0];
      for (int q = 1; q < OUT; ++q) mx = fmaxf(mx, sDout[q]);
      float se = 0.f;
      for (int q = 0; q < OUT; ++q) se += expf(sDout[q] - mx);
      const float lse = mx + logf(se);
      const float wy = a.p.class_w ? a.p.class_w[yi] : 1.f;
      if (a.p.loss_per_graph) a.p.loss_per_graph[b] = wy * (lse - sDout[yi]);
      for (int q = 0; q < OUT; ++q) sDout[q] = wy * (expf(sDout[q] - lse) - (q == yi ? 1.f : 0.f)) * a.p.loss_scale;
    } else {
      for (int q = 0; q < OUT; ++q) sDout[q] = a.p.dout[(int64_t)b * OUT + q];
    }
  }
  __syncthreads();

  // ---------------- head backward -------------------------------------------
  if (tid < 128) {
    float acc = 0.f;
    for (int q = 0; q < OUT; ++q) acc = fmaf(a.w.fc2w[q * 128 + tid], sDout[q], acc);
    if (a.p.use_dropout) acc = (a.p.mask[(int64_t)b * 128 + tid] ? acc : 0.f) * a.p.drop_scale;
    sDh[tid] = relu_bwd(sHh[tid], acc);
  }
  __syncthreads();
  if (tid < 64) {
    float acc = 0.f;
    for (int r = 0; r < 128; ++r) acc = fmaf(a.w.fc1w[r * 64 + tid], sDh[r], acc);
    sDG[tid] = acc;
  }
  {
    const int HS = DR_HEAD_STRIDE(OUT);
    float* hg = a.p.head + (int64_t)b * HS;
    if (tid < 64) hg[tid] = sG[tid];
    if (tid < 128) {
      hg[64 + tid] = sHd[tid];
      hg[192 + tid] = sDh[tid];
    }
    if (tid < OUT) hg[320 + tid] = sDout[tid];
  }
  __syncthreads();

  // ---------------- depth-1 pooling + mean backward -------------------------
  // scatter_mean: grad/count; scatter_reduce amax: grad split evenly over the
  // members equal to the max ((src==max) * grad/ties, so NaN stays NaN).
  for (int p = tid; p < K1 * 64; p += NT) {
    const int m = p >> 6, o = p & 63;
    const float gm = (sDG[o] / (float)K1) / sNT[p];
    const float mx = sP2[p];
    for (int q = sm1p[m]; q < sm1p[m + 1]; ++q) {
      const int k = sm1i[q];
      const float h = sH2[k * 64 + o];
      sD2[k * 64 + o] = relu_bwd(h, (h == mx ? 1.f : 0.f) * gm);
    }
  }
  __syncthreads();
  // dY2 = A1^T dS2 (pooled graph, transposed CSR)  -> reuse sY2
  for (int p = tid; p < K0 * 64; p += NT) {
    const int j = p >> 6, o = p & 63;
    float acc = 0.f;
    for (int e = sp1trp[j]; e < sp1trp[j + 1]; ++e) acc += sD2[sp1tc[e] * 64 + o];
    sY2[p] = acc;
  }
  __syncthreads();
  // conv2 weight-gradient partials and dP1
  {
    const int SS = DR_SLAB_STRIDE(F);
    float* slab = a.p.slab + (int64_t)b * SS + 32 * F;
    for (int p = tid; p < 1024; p += NT) {
      const int br = p >> 9, o = ((p >> 4) & 31) + br * 32, j = p & 15;
      float acc = 0.f;
      for (int k = 0; k < K0; ++k) acc = fmaf(sY2[k * 64 + o], sP1[k * 32 + br * 16 + j], acc);
      slab[p] = acc;
    }
  }
  for (int p = tid; p < K0 * 32; p += NT) {
    const int k = p >> 5, ch = p & 31, br = ch >> 4, j = ch & 15;
    const float* __restrict__ wb = br ? a.w.w2e : a.w.w2;
    float acc = 0.f;
    for (int o = 0; o < 32; ++o) acc = fmaf(sY2[k * 64 + br * 32 + o], wb[o * 16 + j], acc);
    // depth-0 scatter_max backward goes to the arg member only; fold the
    // conv1 relu backward in here (needs H1 at that member).
    const int i = sA1[p];
    sdP1[p] = (i < N) ? relu_bwd(sH[i * 32 + ch], acc) : 0.f;
  }
  __syncthreads();
  for (int p = tid; p < N * 32; p += NT) sH[p] = 0.f;
  __syncthreads();
  for (int p = tid; p < K0 * 32; p += NT) {
    const int i = sA1[p];
    if (i < N) sH[i * 32 + (p & 31)] = sdP1[p];
  }
  __syncthreads();

  // ---------------- conv1 backward: dY = A^T dS  -> reuse sY ---------------
  {
    const int c4 = (tid & 7) * 4;
    for (int j = tid >> 3; j < N; j += NT / 8) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int e = strp[j]; e < strp[j + 1]; ++e) {
        const float4 v = *reinterpret_cast<const float4*>(&sH[stcol[e] * 32 + c4]);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
      *reinterpret_cast<float4*>(&sY[j * 32 + c4]) = acc;
    }
  }
  __syncthreads();

  // ---------------- dW1cat = dY^T X  (4 row-quarters, 4x4 register blocks) --
  {
    const int q = tid >> 6, t64 = tid & 63;
    const int nblk = 8 * (LDX / 4);
    const int ib = (q * N) / 4, ie = ((q + 1) * N) / 4;
    for (int blk = t64; blk < nblk; blk += 64) {
      const int cb = (blk & 7) * 4, kb = (blk >> 3) * 4;
      float acc[4][4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[u][v] = 0.f;
      for (int i = ib; i < ie; ++i) {
        const float4 dy = *reinterpret_cast<const float4*>(&sY[i * 32 + cb]);
        const float4 xv = *reinterpret_cast<const float4*>(&sX[i * LDX + kb]);
        const float dyv[4] = {dy.x, dy.y, dy.z, dy.w};
        const float xvv[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int v = 0; v < 4; ++v) acc[u][v] = fmaf(dyv[u], xvv[v], acc[u][v]);
      }
      float* red = sRed + q * 32 * LDX;
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) red[(cb + u) * LDX + kb + v] = acc[u][v];
    }
  }
  __syncthreads();
  {
    const int SS = DR_SLAB_STRIDE(F);
    float* slab = a.p.slab + (int64_t)b * SS;
    const int plane = 32 * LDX;
    for (int p = tid; p < 32 * F; p += NT) {
      const int ch = p / F, k = p - ch * F;
      const int o = ch * LDX + k;
      slab[p] = (sRed[o] + sRed[plane + o]) + (sRed[2 * plane + o] + sRed[3 * plane + o]);
    }
  }
}

// ---------------------------------------------------------------------------
// Reduce the per-graph partials into the 16 GINet gradients, then Adam.
// ---------------------------------------------------------------------------
struct ReduceArgs {
  dr_param_table t;
  dr_adam adam;
  const float* slab;
  const float* head;
  const float* lpg;
  float* loss_out;
  float loss_scale;
  int32_t F, OUT, B;
  int32_t off[DR_GINET_NPARAM + 1];
};

__global__ void __launch_bounds__(256) ginet_reduce_kernel(ReduceArgs a) {
  const int gi = blockIdx.x * 256 + threadIdx.x;
  if (gi == 0 && a.lpg && a.loss_out) {
    float acc = 0.f;
    for (int b = 0; b < a.B; ++b) acc += a.lpg[b];
    a.loss_out[0] = acc * a.loss_scale;
  }
  if (gi >= a.off[DR_GINET_NPARAM]) return;
  int pi = 0;
  while (gi >= a.off[pi + 1]) ++pi;
  const int e = gi - a.off[pi];
  const int F = a.F;
  const int SS = DR_SLAB_STRIDE(F);
  const int HS = DR_HEAD_STRIDE(a.OUT);
  float gsum = 0.f;
  if (!a.slab) {  // gradients supplied (e.g. after an RCCL all-reduce): Adam only
    gsum = a.t.grad[pi] ? a.t.grad[pi][e] : 0.f;
  } else switch (pi) {
    case 0:  // conv1.fc.weight [16,F] = rows 0..15 of the slab's [32][F]
      for (int b = 0; b < a.B; ++b) gsum += a.slab[(int64_t)b * SS + e];
      break;
    case 6:  // conv1_ext.fc.weight = rows 16..31
      for (int b = 0; b < a.B; ++b) gsum += a.slab[(int64_t)b * SS + 16 * F + e];
      break;
    case 3:  // conv2.fc.weight [32,16]
      for (int b = 0; b < a.B; ++b) gsum += a.slab[(int64_t)b * SS + 32 * F + e];
      break;
    case 9:  // conv2_ext.fc.weight
      for (int b = 0; b < a.B; ++b) gsum += a.slab[(int64_t)b * SS + 32 * F + 512 + e];
      break;
    case 12: {  // fc1.weight [128,64] = sum_b dh ⊗ g
      const int r = e >> 6, o = e & 63;
      for (int b = 0; b < a.B; ++b) gsum = fmaf(a.head[(int64_t)b * HS + 192 + r], a.head[(int64_t)b * HS + o], gsum);
    } break;
    case 13:  // fc1.bias
      for (int b = 0; b < a.B; ++b) gsum += a.head[(int64_t)b * HS + 192 + e];
      break;
    case 14: {  // fc2.weight [out,128] = sum_b dout ⊗ hd
      const int q = e >> 7, r = e & 127;
      for (int b = 0; b < a.B; ++b) gsum = fmaf(a.head[(int64_t)b * HS + 320 + q], a.head[(int64_t)b * HS + 64 + r], gsum);
    } break;
    case 15:
      for (int b = 0; b < a.B; ++b) gsum += a.head[(int64_t)b * HS + 320 + e];
      break;
    default:  // fc_edge_attr / fc_attention: exact zeros (softmax over size-1 dim)
      gsum = 0.f;
  }
  if (a.slab && a.t.grad[pi]) a.t.grad[pi][e] = gsum;
  if (a.adam.enabled) {
    float* p = a.t.param[pi] + e;
    float* m = a.t.exp_avg[pi] + e;
    float* v = a.t.exp_avg_sq[pi] + e;
    float gr = gsum;
    if (a.adam.weight_decay != 0.f) gr = fmaf(a.adam.weight_decay, *p, gr);
    // torch.optim.Adam: exp_avg.lerp_(g, 1-b1); exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
    const float mv = *m + (1.f - a.adam.beta1) * (gr - *m);
    const float vv = fmaf((1.f - a.adam.beta2) * gr, gr, *v * a.adam.beta2);
    *m = mv;
    *v = vv;
    const float denom = sqrtf(vv) / a.adam.bias_c2_sqrt + a.adam.eps;
    *p = *p - (a.adam.lr / a.adam.bias_c1) * (mv / denom);
  }
}

}  // namespace

extern "C" int64_t dr_ginet_lds_bytes(int32_t n_nodes, int32_t n_edges, int32_t n_feat, int32_t k0, int32_t p1_edges,
                                      int32_t k1, int32_t transpose_aliased) {
  return 4LL * carve(n_nodes, n_edges, n_feat, k0, p1_edges, k1, transpose_aliased).total;
}

extern "C" int dr_ginet_graph_pass(const dr_graph_store* store, const int32_t* gids, int32_t n_batch,
                                   const dr_ginet_weights* w, const dr_ginet_pass* pass, int32_t lds_bytes,
                                   void* stream) {
  if (!store || !gids || !w || !pass || n_batch < 0) return DR_E_ARG;
  if (pass->out_dim < 1 || pass->out_dim > DR_MAX_OUT) return DR_E_UNSUPPORTED;
  if (lds_bytes > 160 * 1024) return DR_E_LDS;
  if ((pass->flags & DR_PASS_BACKWARD) && (!pass->slab || !pass->head)) return DR_E_ARG;
  if ((pass->flags & DR_PASS_BACKWARD) && pass->loss_kind == DR_LOSS_NONE && !pass->dout) return DR_E_ARG;
  if ((pass->flags & DR_PASS_FORWARD) && !pass->out) return DR_E_ARG;
  if (pass->use_dropout && !pass->mask) return DR_E_ARG;
  if (n_batch == 0) return DR_OK;
  DR_CHECK(dr_allow_big_lds(reinterpret_cast<const void*>(&ginet_graph_kernel)));
  GinetArgs args;
  args.s = *store;
  args.w = *w;
  args.p = *pass;
  args.gids = gids;
  args.B = n_batch;
  hipLaunchKernelGGL(ginet_graph_kernel, dim3(n_batch), dim3(NT), lds_bytes, (hipStream_t)stream, args);
  return (int)hipGetLastError();
}

extern "C" int dr_ginet_reduce_update(const dr_param_table* t, int32_t n_feat, int32_t out_dim, const float* slab,
                                      const float* head, int32_t n_batch, const dr_adam* adam,
                                      const float* loss_per_graph, float loss_scale, float* loss_out, void* stream) {
  if (!t || !adam || n_batch < 0) return DR_E_ARG;
  if ((slab == nullptr) != (head == nullptr)) return DR_E_ARG;
  if (!slab)
    for (int i = 0; i < DR_GINET_NPARAM; ++i)
      if (!t->grad[i]) return DR_E_ARG;
  ReduceArgs a;
  a.t = *t;
  a.adam = *adam;
  a.slab = slab;
  a.head = head;
  a.lpg = loss_per_graph;
  a.loss_out = loss_out;
  a.loss_scale = loss_scale;
  a.F = n_feat;
  a.OUT = out_dim;
  a.B = n_batch;
  a.off[0] = 0;
  for (int i = 0; i < DR_GINET_NPARAM; ++i) {
    if (t->numel[i] < 0 || !t->param[i]) return DR_E_ARG;
    if (adam->enabled && (!t->exp_avg[i] || !t->exp_avg_sq[i])) return DR_E_ARG;
    a.off[i + 1] = a.off[i] + t->numel[i];
  }
  const int total = a.off[DR_GINET_NPARAM];
  hipLaunchKernelGGL(ginet_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}
