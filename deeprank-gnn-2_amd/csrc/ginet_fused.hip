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
// Execution: 1024 threads (16 waves) per graph so the LDS-latency-bound
// gather phases have 4 waves per SIMD in flight; the two node GEMMs
// (X·Wᵀ forward, dYᵀ·X for the weight gradient) run on the f32 MFMA
// (v_mfma_f32_16x16x4_f32: an exact k-ordered fmaf chain, the same numerics as
// the VALU loop).  X is stored with an odd row stride so MFMA column reads are
// bank-conflict free.  The backward re-uses the Y/H regions for dY/dS.
// Roofline: HBM-bound on the compulsory inputs (x, CSR, clusters) and the
// per-graph partial writes — see DESIGN.md §Roofline.

#include <hip/hip_runtime.h>

#include <cstring>

#include "../../include/deeprank2_amd.h"
#include "dr_common.h"

namespace {

constexpr int NT = 1024;     // 16 waves
constexpr int NW = NT / 64;
constexpr int HEADW = 672;   // G64 hpre128 hh128 hd128 dh128 dG64 dout16 spare16
constexpr float LOWEST = -3.402823466e+38f;

typedef float floatx4 __attribute__((ext_vector_type(4)));

__host__ __device__ inline int r4(int v) { return (v + 3) & ~3; }
__host__ __device__ inline int r16(int v) { return (v + 15) & ~15; }
__host__ __device__ inline int imax(int a, int b) { return a > b ? a : b; }

struct Carve {
  int KP, LDX, ntile, S;
  int wt, x, y, h, rp, col, trp, tcol, m0p, m0i, p1, a1, dp1, y2, h2, d2, p1rp, p1c, p1trp, p1tc, m1p, m1i, p2,
      nt, head, dgp, red, total;
};

__host__ __device__ inline Carve carve(int N, int E, int F, int K0, int P1, int K1, int alias) {
  Carve c;
  c.KP = r16(F);          // K padded for 16-wide MFMA tiles (zeros)
  c.LDX = c.KP + 1;       // odd stride: conflict-free MFMA column reads of X
  c.ntile = 2 * (c.KP / 16);
  c.S = imax(1, NW / c.ntile);
  int o = 0;
#define TAKE(field, words) \
  c.field = o;             \
  o += r4(words);
  TAKE(wt, c.KP * 32)
  TAKE(x, N * c.LDX)
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
  TAKE(dgp, NW * 64)
  TAKE(red, imax(c.S * 32 * c.KP, 2 * NT))
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

__device__ __forceinline__ bool keep_unit(const dr_ginet_pass& p, int b, int r) {
  if (p.use_dropout == DR_DROPOUT_MASK) return p.mask[(int64_t)b * 128 + r] != 0;
  return dr_uniform(p.drop_seed, p.drop_offset, (uint32_t)(b * 128 + r)) >= p.drop_p;
}

// dst[i,:32] = sum over CSR row i of src[col[e],:32]; 8 lanes per row, float4 each.
__device__ __forceinline__ void csr_gather32(const int* rp, const int* col, const float* src, float* dst, int n,
                                             bool relu) {
  const int c4 = (threadIdx.x & 7) * 4;
  for (int i = threadIdx.x >> 3; i < n; i += NT / 8) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const int eb = rp[i], ee = rp[i + 1];
    for (int e = eb; e < ee; ++e) {
      const float4 v = *reinterpret_cast<const float4*>(&src[col[e] * 32 + c4]);
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    if (relu) {
      acc.x = relu_keepnan(acc.x);
      acc.y = relu_keepnan(acc.y);
      acc.z = relu_keepnan(acc.z);
      acc.w = relu_keepnan(acc.w);
    }
    *reinterpret_cast<float4*>(&dst[i * 32 + c4]) = acc;
  }
}

__global__ void __launch_bounds__(NT) ginet_graph_kernel(GinetArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
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
  const int alias = s.transpose_aliased;
  const Carve c = carve(N, E, F, K0, P1, K1, alias);
  const int KP = c.KP, LDX = c.LDX;
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
  float* sDGp = lds + c.dgp;
  float* sRed = lds + c.red;

  // ---------------- stage the graph into LDS --------------------------------
  for (int p = tid; p < KP * 32; p += NT) {
    const int k = p >> 5, ch = p & 31;
    float v = 0.f;
    if (k < F) v = (ch < 16) ? a.w.w1[ch * F + k] : a.w.w1e[(ch - 16) * F + k];
    sWT[p] = v;
  }
  {
    const float* __restrict__ xg = s.x + n0 * (int64_t)F;
    for (int p = tid; p < N * F; p += NT) {
      const int i = p / F;
      sX[i * LDX + (p - i * F)] = xg[p];
    }
    const int padw = KP - F;
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

  // ---------------- conv1 node GEMM on MFMA: Y = X [W1;W1e]^T (ginet.py:45) -
  {
    const int li = lane & 15, kq = lane >> 4;
    for (int t = wave; t * 16 < N; t += NW) {
      const int r0 = t * 16;
      const int ar = r0 + li;
      floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < KP; k += 4) {
        const float av = (ar < N) ? sX[ar * LDX + k + kq] : 0.f;
        const float b0 = sWT[(k + kq) * 32 + li];
        const float b1 = sWT[(k + kq) * 32 + 16 + li];
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b0, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b1, acc1, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + kq * 4 + r;
        if (row < N) {
          sY[row * 32 + li] = acc0[r];
          sY[row * 32 + 16 + li] = acc1[r];
        }
      }
    }
  }
  __syncthreads();

  // ---------------- conv1 aggregation + relu: H = relu(A Y)  (ginet.py:58,96)
  csr_gather32(srp, scol, sY, sH, N, true);
  __syncthreads();

  // ---------------- depth-0 community pooling: torch_scatter scatter_max ----
  // (community_pooling.py:209): strict '>' from lowest(), members in node
  // order => first max wins, NaN never enters, empty -> 0 with no arg.
  // Members are split into S1 contiguous slices combined in slice order.
  {
    const int pairs = K0 * 32;
    const int S1 = pairs > 0 ? max(1, min(8, NT / pairs)) : 1;
    float* tb = sRed;
    int* ta = reinterpret_cast<int*>(sRed + NT);
    for (int p = tid; p < pairs * S1; p += NT) {
      const int sl = p / pairs, pr = p - sl * pairs;
      const int k = pr >> 5, ch = pr & 31;
      const int mb = sm0p[k], cnt = sm0p[k + 1] - mb;
      const int qb = mb + (cnt * sl) / S1, qe = mb + (cnt * (sl + 1)) / S1;
      float best = LOWEST;
      int arg = N;
      for (int m = qb; m < qe; ++m) {
        const int i = sm0i[m];
        const float v = sH[i * 32 + ch];
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
        const float v = tb[sl * pairs + p];
        if (v > best) {
          best = v;
          arg = ta[sl * pairs + p];
        }
      }
      sP1[p] = (best == LOWEST) ? 0.f : best;
      sA1[p] = arg;
    }
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
  {
    const int r = tid >> 3, part = tid & 7;  // 8 lanes per fc1 row
    const float* __restrict__ wr = a.w.fc1w + r * 64 + part * 8;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = fmaf(sG[part * 8 + j], wr[j], acc);
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    acc += __shfl_xor(acc, 4, 64);
    if (part == 0) {
      acc += a.w.fc1b[r];
      sHpre[r] = acc;
      const float hh = relu_keepnan(acc);
      sHh[r] = hh;
      float hd = hh;
      if (a.p.use_dropout) hd = (keep_unit(a.p, b, r) ? hh : 0.f) * a.p.drop_scale;
      sHd[r] = hd;
    }
  }
  __syncthreads();
  for (int q = wave; q < OUT; q += NW) {
    const float* __restrict__ wr = a.w.fc2w + q * 128;
    float v = fmaf(sHd[lane], wr[lane], sHd[lane + 64] * wr[lane + 64]);
    v = dr_wave_sum(v);
    if (lane == 0) sDout[q] = v + a.w.fc2b[q];  // logits parked in sDout
  }
  __syncthreads();
  if ((a.p.flags & DR_PASS_FORWARD) && tid < OUT) a.p.out[(int64_t)b * OUT + tid] = sDout[tid];
  if (!(a.p.flags & DR_PASS_BACKWARD)) return;
  __syncthreads();

  // ---------------- loss gradient (trainer.py:688-689) ----------------------
  if (tid == 0) {
    if (a.p.loss_kind == DR_LOSS_MSE) {
      const float d = sDout[0] - s.y[g];
      if (a.p.loss_per_graph) a.p.loss_per_graph[b] = d * d;
      sDout[0] = 2.f * d * a.p.loss_scale;
    } else if (a.p.loss_kind == DR_LOSS_CE) {
      const int yi = (int)s.y[g];
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
    if (a.p.use_dropout) acc = (keep_unit(a.p, b, tid) ? acc : 0.f) * a.p.drop_scale;
    sDh[tid] = relu_bwd(sHh[tid], acc);
  }
  __syncthreads();
  {
    const int o = tid & 63, rc = tid >> 6;  // 16 chunks of 8 fc1 rows
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = fmaf(a.w.fc1w[(rc * 8 + j) * 64 + o], sDh[rc * 8 + j], acc);
    sDGp[rc * 64 + o] = acc;
  }
  __syncthreads();
  if (tid < 64) {
    float acc = 0.f;
    for (int rc = 0; rc < NW; ++rc) acc += sDGp[rc * 64 + tid];
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
  csr_gather32(strp, stcol, sH, sY, N, false);
  __syncthreads();

  // ---------------- dW1cat = dY^T X on MFMA, node range split in S slices ---
  {
    const int li = lane & 15, kq = lane >> 4;
    const int tile = wave % c.ntile, sl = wave / c.ntile;
    if (sl < c.S) {
      const int ct = tile & 1, kt = tile >> 1;
      const int nb = (N * sl) / c.S, ne = (N * (sl + 1)) / c.S;
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int n = nb; n < ne; n += 4) {
        const int node = n + kq;
        const bool ok = node < ne;
        const float av = ok ? sY[node * 32 + ct * 16 + li] : 0.f;
        const float bv = ok ? sX[node * LDX + kt * 16 + li] : 0.f;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
      }
      float* red = sRed + sl * 32 * KP;
#pragma unroll
      for (int r = 0; r < 4; ++r) red[(ct * 16 + kq * 4 + r) * KP + kt * 16 + li] = acc[r];
    }
  }
  __syncthreads();
  {
    const int SS = DR_SLAB_STRIDE(F);
    float* slab = a.p.slab + (int64_t)b * SS;
    const int plane = 32 * KP;
    for (int p = tid; p < 32 * F; p += NT) {
      const int ch = p / F, k = p - ch * F;
      float acc = 0.f;
      for (int sl = 0; sl < c.S; ++sl) acc += sRed[sl * plane + ch * KP + k];
      slab[p] = acc;
    }
  }
}

// ---------------------------------------------------------------------------
// Reduce the per-graph partials into the 16 GINet gradients, then Adam.
// Block = 32 parameter elements x 8 batch chunks; the chunk partials are
// combined in chunk order (deterministic).
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

constexpr int RP = 32;  // parameter elements per block
constexpr int RC = 8;   // batch chunks per block

__device__ float grad_partial(const ReduceArgs& a, int pi, int e, int b0, int b1) {
  const int F = a.F;
  const int64_t SS = DR_SLAB_STRIDE(F);
  const int64_t HS = DR_HEAD_STRIDE(a.OUT);
  float acc = 0.f;
  switch (pi) {
    case 0:  // conv1.fc.weight [16,F] = rows 0..15 of the slab's [32][F]
      for (int b = b0; b < b1; ++b) acc += a.slab[b * SS + e];
      break;
    case 6:  // conv1_ext.fc.weight = rows 16..31
      for (int b = b0; b < b1; ++b) acc += a.slab[b * SS + 16 * F + e];
      break;
    case 3:  // conv2.fc.weight [32,16]
      for (int b = b0; b < b1; ++b) acc += a.slab[b * SS + 32 * F + e];
      break;
    case 9:  // conv2_ext.fc.weight
      for (int b = b0; b < b1; ++b) acc += a.slab[b * SS + 32 * F + 512 + e];
      break;
    case 12: {  // fc1.weight [128,64] = sum_b dh ⊗ g
      const int r = e >> 6, o = e & 63;
      for (int b = b0; b < b1; ++b) acc = fmaf(a.head[b * HS + 192 + r], a.head[b * HS + o], acc);
    } break;
    case 13:  // fc1.bias
      for (int b = b0; b < b1; ++b) acc += a.head[b * HS + 192 + e];
      break;
    case 14: {  // fc2.weight [out,128] = sum_b dout ⊗ hd
      const int q = e >> 7, r = e & 127;
      for (int b = b0; b < b1; ++b) acc = fmaf(a.head[b * HS + 320 + q], a.head[b * HS + 64 + r], acc);
    } break;
    case 15:
      for (int b = b0; b < b1; ++b) acc += a.head[b * HS + 320 + e];
      break;
    default:  // fc_edge_attr / fc_attention: exact zeros (softmax over size-1 dim)
      break;
  }
  return acc;
}

__global__ void __launch_bounds__(RP* RC) ginet_reduce_kernel(ReduceArgs a) {
  __shared__ float part[RC][RP];
  const int lp = threadIdx.x % RP, ch = threadIdx.x / RP;
  const int gi = blockIdx.x * RP + lp;
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.lpg && a.loss_out) {
    float acc = 0.f;
    for (int b = 0; b < a.B; ++b) acc += a.lpg[b];
    a.loss_out[0] = acc * a.loss_scale;
  }
  const bool live = gi < a.off[DR_GINET_NPARAM];
  int pi = 0;
  if (live)
    while (gi >= a.off[pi + 1]) ++pi;
  const int e = live ? gi - a.off[pi] : 0;
  if (a.slab) {
    float v = 0.f;
    if (live) v = grad_partial(a, pi, e, (a.B * ch) / RC, (a.B * (ch + 1)) / RC);
    part[ch][lp] = v;
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
    gsum = a.t.grad[pi] ? a.t.grad[pi][e] : 0.f;
  }
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
  if (pass->use_dropout == DR_DROPOUT_MASK && !pass->mask) return DR_E_ARG;
  if (pass->use_dropout < DR_DROPOUT_OFF || pass->use_dropout > DR_DROPOUT_HASH) return DR_E_ARG;
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
  ReduceArgs a;
  std::memset(&a, 0, sizeof(a));
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
    if (!slab && !t->grad[i]) return DR_E_ARG;
    a.off[i + 1] = a.off[i] + t->numel[i];
  }
  const int total = a.off[DR_GINET_NPARAM];
  hipLaunchKernelGGL(ginet_reduce_kernel, dim3((total + RP - 1) / RP), dim3(RP * RC), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

extern "C" int dr_dropout_mask(uint64_t seed, uint64_t offset, int32_t n, float p, uint8_t* keep_host) {
  if (n < 0 || (n > 0 && !keep_host)) return DR_E_ARG;
  for (int i = 0; i < n; ++i) keep_host[i] = dr_uniform(seed, offset, (uint32_t)i) >= p ? 1 : 0;
  return DR_OK;
}
