// VanillaNetwork training step, one workgroup per graph.
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
// rebuilt on the fly in a CSR gather (the fused gather + edge MLP + scatter).
// The backward needs no per-edge storage either: with dpre_e = relu'(pre_e) ds_i
//   D_i  = sum_{e: src i} dpre_e,   D'_j = sum_{e: dst j} dpre_e  (transposed CSR),
//   dWa = D^T X,  dWb = D'^T X,  dWc = sum_e dpre_e ea_e^T,  dx = ... + D Wa + D' Wb,
// all row-wise gathers and node-level products.
// Node-level intermediates (E x 32 messages never exist) live in an HBM
// scratch laid out per batch row (L2 / MALL resident); weights live in LDS.

#include <hip/hip_runtime.h>

#include "graph_common.h"

namespace {

using namespace drk;

constexpr int NT = 1024;
constexpr int NW = NT / 64;
constexpr int MAXFE = 8;

struct VArgs {
  dr_graph_store s;
  dr_vanilla_weights w;
  dr_pass p;
  dr_vanilla_scratch ws;
  const dr_graph_desc* descs;
  int32_t B;
};

// scratch arrays (batch rows x width), array-major
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

struct VCarve {
  int KE, KN, we1, be1, wn1, bn1, we2, be2, wn2, bn2, g1w, g1b, g2w, g2b, head, red, total;
};

__host__ __device__ inline VCarve vcarve(int F, int Fe, int OUT) {
  VCarve c;
  c.KE = 2 * F + Fe;
  c.KN = F + 32;
  int o = 0;
#define TAKE(field, words) \
  c.field = o;             \
  o += r4(words);
  TAKE(we1, 32 * c.KE)
  TAKE(be1, 32)
  TAKE(wn1, F * c.KN)
  TAKE(bn1, F)
  TAKE(we2, 32 * c.KE)
  TAKE(be2, 32)
  TAKE(wn2, F * c.KN)
  TAKE(bn2, F)
  TAKE(g1w, 128 * F)
  TAKE(g1b, 128)
  TAKE(g2w, OUT * 128)
  TAKE(g2b, OUT)
  TAKE(head, 2 * r4(F) + 3 * 128 + 16)
  TAKE(red, NT)
#undef TAKE
  c.total = o;
  return c;
}

__device__ __forceinline__ void copy_w(float* dst, const float* src, int n) {
  for (int p = threadIdx.x; p < n; p += NT) dst[p] = src[p];
}

// A = Xin Wa^T, B = Xin Wb^T (pre-activation halves of the edge MLP)
__device__ __forceinline__ void edge_halves(const float* Xin, int ldx, int N, int F, const float* We, int KE, float* A,
                                            float* Bm) {
  for (int p = threadIdx.x; p < N * 64; p += NT) {
    const int i = p >> 6, c = p & 63;
    const float* w = We + (c & 31) * KE + (c < 32 ? 0 : F);
    const float* x = Xin + (int64_t)i * ldx;
    float acc = 0.f;
    for (int k = 0; k < F; ++k) acc = fmaf(x[k], w[k], acc);
    (c < 32 ? A : Bm)[(int64_t)i * 32 + (c & 31)] = acc;
  }
}

__device__ __forceinline__ float edge_const(const float* wc, const float* ea, int Fe) {
  float v = 0.f;
  for (int f = 0; f < Fe; ++f) v = fmaf(wc[f], ea[f], v);
  return v;
}

// relu'(pre) as torch's threshold_backward on relu(pre): 0 where relu(pre) <= 0
__device__ __forceinline__ bool active(float pre) { return !(pre <= 0.f); }

struct Graph {
  const int* rp;      // CSR (by edge_index[0]) row pointers, local
  const uint16_t* col;
  const int* trp;     // transposed CSR (by edge_index[1])
  const uint16_t* tcol;
  const int* teid;    // transposed slot -> CSR slot
  const float* ea;    // [slot, FeS] in CSR slot order
  int FeS;
};

// s_i = sum_{e in row i} relu(A_i + B_j + Wc ea_e + be)
__device__ __forceinline__ void edge_forward(const Graph& G, int N, int Fe, const float* A, const float* Bm,
                                             const float* We, int KE, int F, const float* be, float* S) {
  for (int p = threadIdx.x; p < N * 32; p += NT) {
    const int i = p >> 5, c = p & 31;
    const float a = A[(int64_t)i * 32 + c], bc = be[c];
    const float* wc = We + c * KE + 2 * F;
    float acc = 0.f;
    for (int e = G.rp[i]; e < G.rp[i + 1]; ++e) {
      const int j = G.col[e];
      const float pre = a + Bm[(int64_t)j * 32 + c] + edge_const(wc, G.ea + (int64_t)e * G.FeS, Fe) + bc;
      acc += relu_keepnan(pre);
    }
    S[(int64_t)i * 32 + c] = acc;
  }
}

// Xout = relu([Xin | S] Wn^T + bn)
__device__ __forceinline__ void node_update(const float* Xin, int ldx, const float* S, int N, int F, const float* Wn,
                                            int KN, const float* bn, float* Xout, int ldo) {
  for (int p = threadIdx.x; p < N * F; p += NT) {
    const int i = p / F, n = p - i * F;
    const float* w = Wn + n * KN;
    const float* x = Xin + (int64_t)i * ldx;
    const float* sv = S + (int64_t)i * 32;
    float acc = 0.f;
    for (int k = 0; k < F; ++k) acc = fmaf(x[k], w[k], acc);
    for (int k = 0; k < 32; ++k) acc = fmaf(sv[k], w[F + k], acc);
    Xout[(int64_t)i * ldo + n] = relu_keepnan(acc + bn[n]);
  }
}

// D, D' and the edge-attribute partials of one layer (see header comment)
__device__ __forceinline__ void edge_backward(const Graph& G, int N, int Fe, const float* A, const float* Bm,
                                              const float* We, int KE, int F, const float* be, const float* DS,
                                              float* D, float* DP, float* EAP) {
  for (int p = threadIdx.x; p < N * 32; p += NT) {
    const int i = p >> 5, c = p & 31;
    const float a = A[(int64_t)i * 32 + c], bi = Bm[(int64_t)i * 32 + c], bc = be[c];
    const float dsi = DS[(int64_t)i * 32 + c];
    const float* wc = We + c * KE + 2 * F;
    int cnt = 0;
    float eap[MAXFE];
#pragma unroll
    for (int f = 0; f < MAXFE; ++f) eap[f] = 0.f;
    for (int e = G.rp[i]; e < G.rp[i + 1]; ++e) {
      const int j = G.col[e];
      const float* ea = G.ea + (int64_t)e * G.FeS;
      const float pre = a + Bm[(int64_t)j * 32 + c] + edge_const(wc, ea, Fe) + bc;
      if (active(pre)) {
        ++cnt;
#pragma unroll
        for (int f = 0; f < MAXFE; ++f)
          if (f < Fe) eap[f] += ea[f];
      }
    }
    D[(int64_t)i * 32 + c] = cnt ? dsi * (float)cnt : 0.f;
    float* ep = EAP + ((int64_t)i * 32 + c) * (Fe > 0 ? Fe : 1);
    for (int f = 0; f < Fe; ++f) ep[f] = cnt ? dsi * eap[f] : 0.f;
    // D'_i: edges e = (src -> i), pre_e = A_src + B_i + Wc ea_e + be
    float acc = 0.f;
    for (int q = G.trp[i]; q < G.trp[i + 1]; ++q) {
      const int src = G.tcol[q], e = G.teid[q];
      const float pre = A[(int64_t)src * 32 + c] + bi + edge_const(wc, G.ea + (int64_t)e * G.FeS, Fe) + bc;
      if (active(pre)) acc += DS[(int64_t)src * 32 + c];
    }
    DP[(int64_t)i * 32 + c] = acc;
  }
}

// per-graph weight-gradient partials of one layer into the slab
__device__ __forceinline__ void layer_wgrad(int N, int F, int Fe, int KE, int KN, const float* Xin, int ldx,
                                            const float* S, const float* DU, const float* D, const float* DP,
                                            const float* EAP, float* slab) {
  const int nwe = 32 * KE, nwn = F * KN;
  const int total = nwe + 32 + nwn + F;
  const int FeS = Fe > 0 ? Fe : 1;
  for (int p = threadIdx.x; p < total; p += NT) {
    float acc = 0.f;
    if (p < nwe) {
      const int c = p / KE, k = p - c * KE;
      if (k < F) {
        for (int i = 0; i < N; ++i) acc = fmaf(D[(int64_t)i * 32 + c], Xin[(int64_t)i * ldx + k], acc);
      } else if (k < 2 * F) {
        for (int i = 0; i < N; ++i) acc = fmaf(DP[(int64_t)i * 32 + c], Xin[(int64_t)i * ldx + k - F], acc);
      } else {
        for (int i = 0; i < N; ++i) acc += EAP[((int64_t)i * 32 + c) * FeS + (k - 2 * F)];
      }
    } else if (p < nwe + 32) {
      const int c = p - nwe;
      for (int i = 0; i < N; ++i) acc += D[(int64_t)i * 32 + c];
    } else if (p < nwe + 32 + nwn) {
      const int q = p - nwe - 32, n = q / KN, k = q - n * KN;
      if (k < F) {
        for (int i = 0; i < N; ++i) acc = fmaf(DU[(int64_t)i * r4(F) + n], Xin[(int64_t)i * ldx + k], acc);
      } else {
        for (int i = 0; i < N; ++i) acc = fmaf(DU[(int64_t)i * r4(F) + n], S[(int64_t)i * 32 + k - F], acc);
      }
    } else {
      const int n = p - nwe - 32 - nwn;
      for (int i = 0; i < N; ++i) acc += DU[(int64_t)i * r4(F) + n];
    }
    slab[p] = acc;
  }
}

__global__ void __launch_bounds__(NT) vanilla_graph_kernel(VArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x;
  const dr_graph_store& s = a.s;
  const dr_graph_desc d = a.descs[b];
  const int g = d.gid;
  const int64_t n0 = d.node0, ec0 = d.col0;
  const int N = d.n_nodes, F = s.n_feat, Fe = s.n_edge_feat, OUT = a.p.out_dim;
  const int XS = r4(F);
  const VCarve c = vcarve(F, Fe, OUT);
  const int KE = c.KE, KN = c.KN;
  float *sWe1 = lds + c.we1, *sBe1 = lds + c.be1, *sWn1 = lds + c.wn1, *sBn1 = lds + c.bn1;
  float *sWe2 = lds + c.we2, *sBe2 = lds + c.be2, *sWn2 = lds + c.wn2, *sBn2 = lds + c.bn2;
  float *sG1w = lds + c.g1w, *sG1b = lds + c.g1b, *sG2w = lds + c.g2w, *sG2b = lds + c.g2b;
  float* sG = lds + c.head;  // mean over nodes [XS]
  float* sHh = sG + XS;      // relu(fc1)   [128]
  float* sDh = sHh + 128;    // its grad    [128]
  float* sDg = sDh + 128;    // d mean     [XS]
  float* sDout = sDg + XS;   // logits / dout [16]
  float* sHpre = sDout + 16; // [128]
  float* sRed = lds + c.red;

  const float y_g = s.y[g];
  if (a.p.step_counter && b == 0 && tid == 0) a.p.step_counter[1] = a.p.step_counter[0];
  copy_w(sWe1, a.w.we1, 32 * KE);
  copy_w(sBe1, a.w.be1, 32);
  copy_w(sWn1, a.w.wn1, F * KN);
  copy_w(sBn1, a.w.bn1, F);
  copy_w(sWe2, a.w.we2, 32 * KE);
  copy_w(sBe2, a.w.be2, 32);
  copy_w(sWn2, a.w.wn2, F * KN);
  copy_w(sBn2, a.w.bn2, F);
  copy_w(sG1w, a.w.g1w, 128 * F);
  copy_w(sG1b, a.w.g1b, 128);
  copy_w(sG2w, a.w.g2w, OUT * 128);
  copy_w(sG2b, a.w.g2b, OUT);

  const Scratch L = scratch_layout(a.ws.n_rows, F, Fe);
  const int64_t R0 = a.ws.row0[b];
  float* ws = a.ws.base;
  float *X1 = ws + L.x1 + R0 * XS, *X2 = ws + L.x2 + R0 * XS, *DU = ws + L.du + R0 * XS, *DX1 = ws + L.dx1 + R0 * XS;
  float *S1 = ws + L.s1 + R0 * 32, *S2 = ws + L.s2 + R0 * 32, *A1 = ws + L.a1 + R0 * 32, *B1 = ws + L.b1 + R0 * 32;
  float *A2 = ws + L.a2 + R0 * 32, *B2 = ws + L.b2 + R0 * 32, *DS = ws + L.ds + R0 * 32, *D = ws + L.d + R0 * 32;
  float *DP = ws + L.dp + R0 * 32, *EAP = ws + L.eap + R0 * 32 * (Fe > 0 ? Fe : 1);
  const float* X0 = s.x + n0 * XS;
  Graph G;
  G.rp = s.rowptr + n0 + g;
  G.col = s.col + ec0;
  G.trp = s.t_rowptr + n0 + g;
  G.tcol = s.t_col + ec0;
  G.teid = s.t_eid + ec0;
  G.FeS = Fe > 0 ? Fe : 1;
  G.ea = s.ea + ec0 * G.FeS;
  __syncthreads();

  DRK_STAMP(0);
  // ---------------- layer 1 (vanilla_gnn.py:26-38) ----------------------------
  edge_halves(X0, XS, N, F, sWe1, KE, A1, B1);
  __syncthreads();
  edge_forward(G, N, Fe, A1, B1, sWe1, KE, F, sBe1, S1);
  __syncthreads();
  node_update(X0, XS, S1, N, F, sWn1, KN, sBn1, X1, XS);
  __syncthreads();
  DRK_STAMP(1);
  // ---------------- layer 2 ---------------------------------------------------
  edge_halves(X1, XS, N, F, sWe2, KE, A2, B2);
  __syncthreads();
  edge_forward(G, N, Fe, A2, B2, sWe2, KE, F, sBe2, S2);
  __syncthreads();
  node_update(X1, XS, S2, N, F, sWn2, KN, sBn2, X2, XS);
  __syncthreads();
  DRK_STAMP(2);
  // ---------------- scatter_mean over the graph (vanilla_gnn.py:62) ----------
  {
    const int CH = NT / XS;  // row chunks, combined in order
    const int n = tid % XS, ch = tid / XS;
    float acc = 0.f;
    if (n < F && ch < CH) {
      const int i0 = (N * ch) / CH, i1 = (N * (ch + 1)) / CH;
      for (int i = i0; i < i1; ++i) acc += X2[(int64_t)i * XS + n];
    }
    sRed[tid] = acc;
    __syncthreads();
    if (tid < F) {
      float t = 0.f;
      for (int q = 0; q < CH; ++q) t += sRed[q * XS + tid];
      sG[tid] = t / (float)N;
    }
  }
  __syncthreads();
  // ---------------- graph MLP: Linear(F,128) -> relu -> Linear(128,out) -------
  if (tid < 128) {
    float acc = 0.f;
    for (int n = 0; n < F; ++n) acc = fmaf(sG[n], sG1w[tid * F + n], acc);
    acc += sG1b[tid];
    sHpre[tid] = acc;
    sHh[tid] = relu_keepnan(acc);
  }
  __syncthreads();
  for (int q = wave; q < OUT; q += NW) {
    float v = fmaf(sHh[lane], sG2w[q * 128 + lane], sHh[lane + 64] * sG2w[q * 128 + lane + 64]);
    v = dr_wave_sum(v);
    if (lane == 0) sDout[q] = v + sG2b[q];
  }
  __syncthreads();
  if ((a.p.flags & DR_PASS_FORWARD) && tid < OUT) a.p.out[(int64_t)b * OUT + tid] = sDout[tid];
  if (!(a.p.flags & DR_PASS_BACKWARD)) return;
  __syncthreads();
  DRK_STAMP(3);
  // ---------------- loss gradient (trainer.py:688-689) ------------------------
  if (tid == 0) {
    if (a.p.loss_kind == DR_LOSS_MSE) {
      const float dl = sDout[0] - y_g;
      if (a.p.loss_per_graph) a.p.loss_per_graph[b] = dl * dl;
      sDout[0] = 2.f * dl * a.p.loss_scale;
    } else if (a.p.loss_kind == DR_LOSS_CE) {
      const int yi = (int)y_g;
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
  if (tid < 128) {
    float acc = 0.f;
    for (int q = 0; q < OUT; ++q) acc = fmaf(sG2w[q * 128 + tid], sDout[q], acc);
    sDh[tid] = relu_bwd(sHh[tid], acc);
  }
  __syncthreads();
  if (tid < F) {
    float acc = 0.f;
    for (int r = 0; r < 128; ++r) acc = fmaf(sG1w[r * F + tid], sDh[r], acc);
    sDg[tid] = acc / (float)N;  // scatter_mean backward: grad / count
  }
  {
    const int HS = DR_VANILLA_HEAD_STRIDE(F, OUT);
    float* hg = a.p.head + (int64_t)b * HS;
    if (tid < XS) hg[tid] = tid < F ? sG[tid] : 0.f;
    if (tid < 128) {
      hg[XS + tid] = sHh[tid];
      hg[XS + 128 + tid] = sDh[tid];
    }
    if (tid < OUT) hg[XS + 256 + tid] = sDout[tid];
  }
  __syncthreads();
  DRK_STAMP(4);
  const int SS1 = 32 * KE + 32 + F * KN + F;
  float* slab = a.p.slab + (int64_t)b * DR_VANILLA_SLAB_STRIDE(F, Fe);
  // ---------------- layer 2 backward -------------------------------------------
  for (int p = tid; p < N * F; p += NT) {
    const int i = p / F, n = p - i * F;
    DU[(int64_t)i * XS + n] = relu_bwd(X2[(int64_t)i * XS + n], sDg[n]);
  }
  __syncthreads();
  for (int p = tid; p < N * KN; p += NT) {  // [dX1_direct | ds2] = du2 Wn2
    const int i = p / KN, k = p - i * KN;
    float acc = 0.f;
    for (int n = 0; n < F; ++n) acc = fmaf(DU[(int64_t)i * XS + n], sWn2[n * KN + k], acc);
    if (k < F) DX1[(int64_t)i * XS + k] = acc;
    else DS[(int64_t)i * 32 + k - F] = acc;
  }
  __syncthreads();
  edge_backward(G, N, Fe, A2, B2, sWe2, KE, F, sBe2, DS, D, DP, EAP);
  __syncthreads();
  DRK_STAMP(5);
  for (int p = tid; p < N * F; p += NT) {  // dX1 += D Wa2 + D' Wb2
    const int i = p / F, k = p - i * F;
    float acc = DX1[(int64_t)i * XS + k];
    for (int cc = 0; cc < 32; ++cc) acc = fmaf(D[(int64_t)i * 32 + cc], sWe2[cc * KE + k], acc);
    for (int cc = 0; cc < 32; ++cc) acc = fmaf(DP[(int64_t)i * 32 + cc], sWe2[cc * KE + F + k], acc);
    DX1[(int64_t)i * XS + k] = acc;
  }
  layer_wgrad(N, F, Fe, KE, KN, X1, XS, S2, DU, D, DP, EAP, slab + SS1);
  __syncthreads();
  DRK_STAMP(6);
  // ---------------- layer 1 backward -------------------------------------------
  for (int p = tid; p < N * F; p += NT) {
    const int i = p / F, n = p - i * F;
    DU[(int64_t)i * XS + n] = relu_bwd(X1[(int64_t)i * XS + n], DX1[(int64_t)i * XS + n]);
  }
  __syncthreads();
  for (int p = tid; p < N * 32; p += NT) {  // ds1 = du1 Wn1[:, F:]
    const int i = p >> 5, k = p & 31;
    float acc = 0.f;
    for (int n = 0; n < F; ++n) acc = fmaf(DU[(int64_t)i * XS + n], sWn1[n * KN + F + k], acc);
    DS[(int64_t)i * 32 + k] = acc;
  }
  __syncthreads();
  edge_backward(G, N, Fe, A1, B1, sWe1, KE, F, sBe1, DS, D, DP, EAP);
  __syncthreads();
  layer_wgrad(N, F, Fe, KE, KN, X0, XS, S1, DU, D, DP, EAP, slab);
  DRK_STAMP(7);
}

}  // namespace

extern "C" int64_t dr_vanilla_scratch_floats(int64_t n_rows, int32_t n_feat, int32_t n_edge_feat) {
  return scratch_layout(n_rows, n_feat, n_edge_feat).total;
}

extern "C" int64_t dr_vanilla_lds_bytes(int32_t n_feat, int32_t n_edge_feat, int32_t out_dim) {
  return 4LL * vcarve(n_feat, n_edge_feat, out_dim).total;
}

extern "C" int dr_vanilla_graph_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                                     const dr_vanilla_weights* w, const dr_pass* pass,
                                     const dr_vanilla_scratch* scratch, int32_t lds_bytes, void* stream) {
  if (!store || !descs || !w || !pass || !scratch || n_batch < 0) return DR_E_ARG;
  if (pass->out_dim < 1 || pass->out_dim > DR_MAX_OUT) return DR_E_UNSUPPORTED;
  if (store->n_feat < 1 || r4(store->n_feat) > NT / 16 || store->n_edge_feat < 0 || store->n_edge_feat > MAXFE)
    return DR_E_UNSUPPORTED;
  if (lds_bytes > 160 * 1024) return DR_E_LDS;
  if (!scratch->base || !scratch->row0) return DR_E_ARG;
  if ((pass->flags & DR_PASS_BACKWARD) && (!pass->slab || !pass->head)) return DR_E_ARG;
  if ((pass->flags & DR_PASS_BACKWARD) && pass->loss_kind == DR_LOSS_NONE && !pass->dout) return DR_E_ARG;
  if ((pass->flags & DR_PASS_FORWARD) && !pass->out) return DR_E_ARG;
  if (pass->use_dropout != DR_DROPOUT_OFF) return DR_E_UNSUPPORTED;
  if (n_batch == 0) return DR_OK;
  DR_CHECK(dr_allow_big_lds(reinterpret_cast<const void*>(&vanilla_graph_kernel)));
  VArgs args;
  args.s = *store;
  args.w = *w;
  args.p = *pass;
  args.ws = *scratch;
  args.descs = descs;
  args.B = n_batch;
  hipLaunchKernelGGL(vanilla_graph_kernel, dim3(n_batch), dim3(NT), lds_bytes, (hipStream_t)stream, args);
  return (int)hipGetLastError();
}
