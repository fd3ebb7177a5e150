// VanillaNetwork training step, one workgroup per graph (residue-size graphs).
//
// Replaces (deeprank2 v3.1.0):
//   VanillaConvolutionalLayer.forward  deeprank2/neuralnets/gnn/vanilla_gnn.py:26-38
//   VanillaNetwork.forward             vanilla_gnn.py:59-65
//   autograd backward + loss           deeprank2/trainer.py:686-689
//
// Per layer:  m_e = relu(We [x_i | x_j | ea_e] + be)  for each edge e = (i -> j),
//             s_i = sum_{e: src i} m_e,   x'_i = relu(Wn [x_i | s_i] + bn).
// As in the batch-wide pipeline (vanilla_fused.hip) the edge GEMM is split,
// We = [Wa | Wb | Wc]:  A = X Wa^T + be,  B = X Wb^T  (node GEMMs on MFMA) and
// pre_e = A_i + B_j + Wc ea_e is rebuilt inside the CSR gather, so the E x 32
// messages never exist.  Here the whole graph stays on one CU: A|B, S, X1 and
// the CSR (+ transpose) live in LDS, the gather reads B_j from LDS, and the
// forward records the ReLU pattern of every edge as one 32-bit word (bit c =
// channel c active) in CSR order and in transposed order.  The backward then
// needs neither A nor B again:
//   D_i  = dS_i * #active(i, c)                       (CSR row pass on the bits)
//   D'_j = sum_{e=(i->j) active} dS_i                 (transposed pass on the bits)
//   dWc  = sum_i dS_i * sum_{e in row i, active} ea_e,  dbe = sum_i D_i
//   dWa = D^T X, dWb = D'^T X, dX = DU Wn[:, :F] + D Wa + D' Wb   (MFMA)
// and relu'(X2) is kept as one bit word per node, so dWn2 = dmean * (mask^T [X1|S2]).
// Intermediates that are written once and read back much later by the same
// workgroup (S1, the edge bit words, the transposed slot map) go to a per-graph
// global scratch (L2-resident); everything gathered stays in LDS.
// Bound: HBM on the compulsory inputs (x, CSR + transpose, edge_attr) and the
// per-graph gradient partials; in practice the per-graph critical path (edge
// passes on the VALU, ~5.7 M f32 MACs of node GEMMs on MFMA) — DESIGN.md §5.

#include <hip/hip_runtime.h>

#include "../../include/deeprank2_amd.h"
#include "graph_common.h"

namespace {

using namespace drk;

constexpr int NT = 1024;  // 16 waves
constexpr int NW = NT / 64;
constexpr int MAXFE = 4;   // edge features handled by this kernel (more: the pipeline)
constexpr int LAB = 64;    // [A+be | B] per node; backward: [dS | D or D']
constexpr int LS = 34;     // S / dX / X1 row stride (F <= 32, 2 words of skew for the MFMA reads)
constexpr int REDW = 160;  // per-wave partials: 32 (dbe) + 32 * MAXFE (dWc)

struct VCarve {
  int rp, col, trp, tcol, x1, ab, s, xb, head, red, total;
};

__host__ __device__ inline VCarve vcarve(int N, int E) {
  VCarve c;
  int o = 0;
#define TAKE(field, words) \
  c.field = o;             \
  o += r4(words);
  TAKE(rp, N + 1)
  TAKE(col, (E + 1) / 2)  // uint16 column ids (16-byte DMA units)
  TAKE(trp, N + 1)
  TAKE(tcol, (E + 1) / 2)
  TAKE(x1, N * LS)
  TAKE(ab, N * LAB)
  TAKE(s, N * LS)
  TAKE(xb, N)
  TAKE(head, 512)  // g 32 | h 128 | dh 128 | dout 16 | dmean 32 | spare
  TAKE(red, NW * REDW)
#undef TAKE
  c.total = o;
  return c;
}

// per-graph global scratch (floats): S1 [N*32] | bits1 csr [E] | bits1 t [E] | bits2 csr [E] | bits2 t [E] | tpos [E]
__host__ __device__ inline int64_t vscratch_floats(int N, int E) { return (int64_t)r4(N * 32) + 5LL * r4(E); }

struct VGArgs {
  dr_graph_store s;
  dr_vanilla_weights w;
  dr_pass p;
  const dr_graph_desc* descs;
  float* scr;
  const int64_t* scr_off;
  int32_t B;
};

// C[m, n] = sum_k A(m, k) B(k, n) on v_mfma_f32_16x16x4_f32, 16x16 output tiles
// spread over the 16 waves (job j on wave (start + j) % NW, so two GEMMs of a
// phase can share the waves).  A / B must return 0 for k >= the true K
// (K4 = K rounded up to 8 here: two accumulator chains).  epi(m, n, v) for
// m < M, n < Nn.
template <class AF, class BF, class EF>
__device__ __forceinline__ void mm16(int M, int Nn, int K, int start, AF A, BF Bf, EF epi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, kq = lane >> 4;
  const int ntl = (Nn + 15) >> 4, jobs = ((M + 15) >> 4) * ntl;
  for (int job = (wave - start % NW + NW) % NW; job < jobs; job += NW) {
    const int m0 = (job / ntl) << 4, n0 = (job % ntl) << 4;
    const int am = min(m0 + li, M - 1), bn = min(n0 + li, Nn - 1);
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < K; k += 8) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(A(am, k + kq), Bf(k + kq, bn), acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(A(am, k + 4 + kq), Bf(k + 4 + kq, bn), acc1, 0, 0, 0);
    }
    if (n0 + li < Nn) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + kq * 4 + r;
        if (row < M) epi(row, n0 + li, acc0[r] + acc1[r]);
      }
    }
  }
}

__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Forward CSR row pass of one layer: S_i = sum_{e in row i} relu(A_i + B_j + Wc ea_e)
// (A already carries be), one wave per row, lane = (channel c, edge parity h).
// The ReLU pattern of each edge (ballot over the 32 channel lanes) goes to
// bc[e] (CSR order) and bt[tpos[e]] (transposed order).
__device__ void row_fwd(const int* srp, const uint16_t* scol, const float* AB, float* S, float* S1g, const float* ea,
                        int Fe, int FeS, const float* we, int KE, int F, const int* tpos, uint32_t* bc, uint32_t* bt,
                        int N) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;
  float wc[MAXFE];
#pragma unroll
  for (int f = 0; f < MAXFE; ++f) wc[f] = f < Fe ? we[c * KE + 2 * F + f] : 0.f;
  for (int i = wave; i < N; i += NW) {
    const int eb = srp[i], ee = srp[i + 1];
    const float ai = AB[i * LAB + c];
    float acc = 0.f;
    for (int e0 = eb; e0 < ee; e0 += 16) {
      const int nch = min(16, ee - e0);
      float ev[8][MAXFE];
      int tp[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int t = 2 * u + h;
        const int e = e0 + (t < nch ? t : 0);
#pragma unroll
        for (int f = 0; f < MAXFE; ++f) ev[u][f] = f < Fe ? ea[(int64_t)e * FeS + f] : 0.f;
        tp[u] = tpos[e];
      }
      float bj[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int t = 2 * u + h;
        const int j = scol[e0 + (t < nch ? t : 0)];
        bj[u] = AB[j * LAB + 32 + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int t = 2 * u + h;
        const bool ok = t < nch;
        float ce = 0.f;
#pragma unroll
        for (int f = 0; f < MAXFE; ++f) ce = fmaf(wc[f], ev[u][f], ce);
        const float pre = ai + bj[u] + ce;
        if (ok) acc += relu_keepnan(pre);
        const uint64_t m = __ballot(ok && !(pre <= 0.f));
        if ((lane & 31) == 0 && ok) {
          const uint32_t word = h ? (uint32_t)(m >> 32) : (uint32_t)m;
          bc[e0 + t] = word;
          bt[tp[u]] = word;
        }
      }
    }
    acc += __shfl_xor(acc, 32, 64);
    if (h == 0) {
      S[i * LS + c] = acc;
      if (S1g) S1g[i * 32 + c] = acc;
    }
  }
}

// Backward CSR row pass: D_i = dS_i * #active(i, c) (0 when none) into AB[:, 32:],
// and per-wave partials of dbe = sum D and dWc[c][f] = sum_i dS_i * sum_{active} ea_e[f].
__device__ void row_bwd(const int* srp, float* AB, const float* ea, int Fe, int FeS, const uint32_t* bc, float* red,
                        int N) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;
  float pbe = 0.f, pwc[MAXFE];
#pragma unroll
  for (int f = 0; f < MAXFE; ++f) pwc[f] = 0.f;
  for (int i = wave; i < N; i += NW) {
    const int eb = srp[i], ee = srp[i + 1];
    float cnt = 0.f, eap[MAXFE];
#pragma unroll
    for (int f = 0; f < MAXFE; ++f) eap[f] = 0.f;
    for (int e0 = eb; e0 < ee; e0 += 16) {
      const int nch = min(16, ee - e0);
      uint32_t wd[8];
      float ev[8][MAXFE];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int t = 2 * u + h;
        const int e = e0 + (t < nch ? t : 0);
        wd[u] = t < nch ? bc[e] : 0u;
#pragma unroll
        for (int f = 0; f < MAXFE; ++f) ev[u][f] = f < Fe ? ea[(int64_t)e * FeS + f] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if ((wd[u] >> c) & 1u) {
          cnt += 1.f;
#pragma unroll
          for (int f = 0; f < MAXFE; ++f) eap[f] += ev[u][f];
        }
      }
    }
    cnt += __shfl_xor(cnt, 32, 64);
#pragma unroll
    for (int f = 0; f < MAXFE; ++f) eap[f] += __shfl_xor(eap[f], 32, 64);
    const float ds = AB[i * LAB + c];
    const float D = cnt != 0.f ? ds * cnt : 0.f;
    if (h == 0) AB[i * LAB + 32 + c] = D;
    pbe += D;
#pragma unroll
    for (int f = 0; f < MAXFE; ++f) pwc[f] += cnt != 0.f ? ds * eap[f] : 0.f;
  }
  if (h == 0) {
    red[wave * REDW + c] = pbe;
#pragma unroll
    for (int f = 0; f < MAXFE; ++f) red[wave * REDW + 32 + c * MAXFE + f] = pwc[f];
  }
}

// Transposed pass: D'_j = sum over in-edges (i -> j) that are active in channel c of dS_i, into AB[:, 32:].
__device__ void row_t(const int* strp, const uint16_t* stcol, float* AB, const uint32_t* bt, int N) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;
  for (int j = wave; j < N; j += NW) {
    const int qb = strp[j], qe = strp[j + 1];
    float acc = 0.f;
    for (int q0 = qb; q0 < qe; q0 += 16) {
      const int nch = min(16, qe - q0);
      uint32_t wd[8];
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int t = 2 * u + h;
        wd[u] = t < nch ? bt[q0 + t] : 0u;
        const int src = stcol[q0 + (t < nch ? t : 0)];
        v[u] = AB[src * LAB + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if ((wd[u] >> c) & 1u) acc += v[u];
    }
    acc += __shfl_xor(acc, 32, 64);
    if (h == 0) AB[j * LAB + 32 + c] = acc;
  }
}

#ifdef DR_STAMPS
#define VSTAMP(i)                                                                                 \
  do {                                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    if (tid == 0 && a.p.stamps) a.p.stamps[(int64_t)b * 32 + (i)] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                            \
  } while (0)
#else
#define VSTAMP(i) \
  do {            \
  } while (0)
#endif

__global__ void __launch_bounds__(NT) vanilla_graph_kernel(VGArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x;
  const dr_graph_store& s = a.s;
  const dr_vanilla_weights& w = a.w;
  const dr_pass& p = a.p;
  const dr_graph_desc d = a.descs[b];
  const int g = d.gid, N = d.n_nodes, E = d.n_edges;
  const int F = s.n_feat, Fe = s.n_edge_feat, FeS = Fe > 0 ? Fe : 1, XS = s.x_stride;
  const int KE = 2 * F + Fe, KN = F + 32, OUT = p.out_dim;
  const int F4 = r4(F);
  const VCarve cv = vcarve(N, E);
  int* srp = reinterpret_cast<int*>(lds + cv.rp);
  uint16_t* scol = reinterpret_cast<uint16_t*>(lds + cv.col);
  int* strp = reinterpret_cast<int*>(lds + cv.trp);
  uint16_t* stcol = reinterpret_cast<uint16_t*>(lds + cv.tcol);
  float* X1 = lds + cv.x1;
  float* AB = lds + cv.ab;
  float* S = lds + cv.s;
  uint32_t* xb = reinterpret_cast<uint32_t*>(lds + cv.xb);
  float* sg = lds + cv.head;
  float* sh = sg + 32;
  float* sdh = sh + 128;
  float* sdout = sdh + 128;
  float* sdm = sdout + 16;
  float* red = lds + cv.red;

  const float* X0 = s.x + d.node0 * (int64_t)XS;
  const float* ea = s.ea + d.col0 * (int64_t)FeS;
  float* scr = a.scr + a.scr_off[b];
  float* S1g = scr;
  uint32_t* b1c = reinterpret_cast<uint32_t*>(scr + r4(N * 32));
  uint32_t* b1t = b1c + r4(E);
  uint32_t* b2c = b1t + r4(E);
  uint32_t* b2t = b2c + r4(E);
  int* tpos = reinterpret_cast<int*>(b2t + r4(E));
  const int LG = 32 * KE + 32 + F * KN + F;  // one layer's gradient entries in the slab
  float* slab = p.slab ? p.slab + (int64_t)b * DR_VANILLA_SLAB_STRIDE(F, Fe) : nullptr;

  VSTAMP(0);
  // ---------------- stage: CSR + transpose into LDS, transposed slot map ----
  dma_words<NT>(srp, s.rowptr + d.node0 + g, N + 1);
  dma_x4<NT>(scol, s.col + d.col0, (E + 7) / 8);
  dma_words<NT>(strp, s.t_rowptr + d.node0 + g, N + 1);
  dma_x4<NT>(stcol, s.t_col + d.col0, (E + 7) / 8);
  {
    const int* teid = s.t_eid + d.col0;
    for (int q = tid; q < E; q += NT) tpos[teid[q]] = q;  // CSR slot -> transposed slot
  }
  for (int p2 = tid; p2 < N * (LS - F); p2 += NT) {  // zero the pad columns of X1 and S (MFMA K padding)
    const int i = p2 / (LS - F), k = F + p2 - i * (LS - F);
    X1[i * LS + k] = 0.f;
    S[i * LS + k] = 0.f;
  }
  const float y_g = s.y[g];
  if (p.step_counter && b == 0 && tid == 0) p.step_counter[1] = p.step_counter[0];
  wait_vm();
  __syncthreads();

  VSTAMP(1);
  // ---------------- layer 1: [A | B] = X0 [Wa; Wb]^T, A += be -------------
  mm16(N, 64, F, 0, [&](int i, int k) { return k < F ? X0[(int64_t)i * XS + k] : 0.f; },
       [&](int k, int n) { return k < F ? w.we1[(n & 31) * KE + (n < 32 ? 0 : F) + k] : 0.f; },
       [&](int i, int n, float v) { AB[i * LAB + n] = v + (n < 32 ? w.be1[n] : 0.f); });
  __syncthreads();
  VSTAMP(2);
  row_fwd(srp, scol, AB, S, S1g, ea, Fe, FeS, w.we1, KE, F, tpos, b1c, b1t, N);
  wait_vm();
  __syncthreads();
  VSTAMP(3);
  // X1 = relu([X0 | S1] Wn1^T + bn1)
  mm16(N, F, F4 + 32, 0,
       [&](int i, int k) { return k < F ? X0[(int64_t)i * XS + k] : (k < F4 ? 0.f : (k < F4 + 32 ? S[i * LS + k - F4] : 0.f)); },
       [&](int k, int n) { return k < F ? w.wn1[n * KN + k] : (k < F4 ? 0.f : (k < F4 + 32 ? w.wn1[n * KN + F + k - F4] : 0.f)); },
       [&](int i, int n, float v) { X1[i * LS + n] = relu_keepnan(v + w.bn1[n]); });
  __syncthreads();
  VSTAMP(4);
  // ---------------- layer 2 ------------------------------------------------
  mm16(N, 64, F, 0, [&](int i, int k) { return k < F ? X1[i * LS + k] : 0.f; },
       [&](int k, int n) { return k < F ? w.we2[(n & 31) * KE + (n < 32 ? 0 : F) + k] : 0.f; },
       [&](int i, int n, float v) { AB[i * LAB + n] = v + (n < 32 ? w.be2[n] : 0.f); });
  __syncthreads();
  VSTAMP(5);
  row_fwd(srp, scol, AB, S, nullptr, ea, Fe, FeS, w.we2, KE, F, tpos, b2c, b2t, N);
  wait_vm();
  __syncthreads();
  VSTAMP(6);
  // X2 = relu([X1 | S2] Wn2^T + bn2) into AB (A|B of layer 2 are dead)
  mm16(N, F, F4 + 32, 0,
       [&](int i, int k) { return k < F ? X1[i * LS + k] : (k < F4 ? 0.f : (k < F4 + 32 ? S[i * LS + k - F4] : 0.f)); },
       [&](int k, int n) { return k < F ? w.wn2[n * KN + k] : (k < F4 ? 0.f : (k < F4 + 32 ? w.wn2[n * KN + F + k - F4] : 0.f)); },
       [&](int i, int n, float v) { AB[i * LAB + n] = relu_keepnan(v + w.bn2[n]); });
  __syncthreads();
  VSTAMP(7);
  // per-graph mean (scatter_mean, vanilla_gnn.py:62): 32 row slices per column, combined in order;
  // relu'(X2) as one bit word per node
  {
    const int n = tid & 31, sl = tid >> 5;
    float acc = 0.f;
    if (n < F) {
      const int i0 = (N * sl) >> 5, i1 = (N * (sl + 1)) >> 5;
      for (int i = i0; i < i1; ++i) acc += AB[i * LAB + n];
    }
    red[sl * 32 + n] = acc;
    for (int i = wave * 2 + (lane >> 5); i < N; i += 2 * NW) {
      const int c = lane & 31;
      const uint64_t m = __ballot(c < F && !(AB[i * LAB + c] <= 0.f));
      if (c == 0) xb[i] = (lane >> 5) ? (uint32_t)(m >> 32) : (uint32_t)m;
    }
  }
  __syncthreads();
  if (tid < 32) {
    float t = 0.f;
    for (int sl = 0; sl < 32; ++sl) t += red[sl * 32 + tid];
    sg[tid] = tid < F ? t / (float)N : 0.f;
  }
  __syncthreads();
  VSTAMP(8);
  // ---------------- graph MLP, loss, head backward (vanilla_gnn.py:63-64, trainer.py:686-689)
  if (tid < 128) {
    float acc = 0.f;
    for (int n = 0; n < F; ++n) acc = fmaf(sg[n], w.g1w[tid * F + n], acc);
    sh[tid] = relu_keepnan(acc + w.g1b[tid]);
  }
  __syncthreads();
  for (int q = wave; q < OUT; q += NW) {
    float v = fmaf(sh[lane], w.g2w[q * 128 + lane], sh[lane + 64] * w.g2w[q * 128 + lane + 64]);
    v = dr_wave_sum(v);
    if (lane == 0) sdout[q] = v + w.g2b[q];
  }
  __syncthreads();
  if ((p.flags & DR_PASS_FORWARD) && tid < OUT) p.out[(int64_t)b * OUT + tid] = sdout[tid];
  if (!(p.flags & DR_PASS_BACKWARD)) return;
  __syncthreads();
  if (tid == 0) {
    if (p.loss_kind == DR_LOSS_MSE) {
      const float dl = sdout[0] - y_g;
      if (p.loss_per_graph) p.loss_per_graph[b] = dl * dl;
      sdout[0] = 2.f * dl * p.loss_scale;
    } else if (p.loss_kind == DR_LOSS_CE) {
      const int yi = (int)y_g;
      float mx = sdout[0];
      for (int q = 1; q < OUT; ++q) mx = fmaxf(mx, sdout[q]);
      float se = 0.f;
      for (int q = 0; q < OUT; ++q) se += expf(sdout[q] - mx);
      const float lse = mx + logf(se);
      const float wy = p.class_w ? p.class_w[yi] : 1.f;
      if (p.loss_per_graph) p.loss_per_graph[b] = wy * (lse - sdout[yi]);
      for (int q = 0; q < OUT; ++q) sdout[q] = wy * (expf(sdout[q] - lse) - (q == yi ? 1.f : 0.f)) * p.loss_scale;
    } else {
      for (int q = 0; q < OUT; ++q) sdout[q] = p.dout[(int64_t)b * OUT + q];
    }
  }
  __syncthreads();
  if (tid < 128) {
    float acc = 0.f;
    for (int q = 0; q < OUT; ++q) acc = fmaf(w.g2w[q * 128 + tid], sdout[q], acc);
    sdh[tid] = relu_bwd(sh[tid], acc);
  }
  __syncthreads();
  {
    float* hg = p.head + (int64_t)b * DR_VANILLA_HEAD_STRIDE(F, OUT);
    const int XSH = r4(F), HD = XSH + 256 + r4(OUT);
    if (tid < F) {
      float acc = 0.f;
      for (int r = 0; r < 128; ++r) acc = fmaf(w.g1w[r * F + tid], sdh[r], acc);
      const float dm = acc / (float)N;  // scatter_mean backward: grad / count
      sdm[tid] = dm;
      hg[HD + tid] = dm;
    }
    if (tid < XSH) hg[tid] = tid < F ? sg[tid] : 0.f;
    if (tid < 128) {
      hg[XSH + tid] = sh[tid];
      hg[XSH + 128 + tid] = sdh[tid];
    }
    if (tid < OUT) hg[XSH + 256 + tid] = sdout[tid];
  }
  __syncthreads();
  VSTAMP(9);

  // ---------------- layer 2 backward ---------------------------------------
  // DU2 = relu'(X2) * dmean (one bit word per node).  dWn2 = DU2^T [X1 | S2],
  // dbn2 = sum DU2 (extra column of ones).
  {
    float* gw = slab + LG;  // layer 2
    mm16(F, KN + 1, N, 0, [&](int n, int i) { return (i < N && ((xb[i] >> n) & 1u)) ? 1.f : 0.f; },
         [&](int i, int q) { return i < N ? (q < F ? X1[i * LS + q] : (q < KN ? S[i * LS + q - F] : 1.f)) : 0.f; },
         [&](int n, int q, float v) {
           if (q < KN) gw[32 * KE + 32 + n * KN + q] = sdm[n] * v;
           else gw[32 * KE + 32 + F * KN + n] = sdm[n] * v;
         });
  }
  __syncthreads();
  // [dX1 | dS2] = DU2 [Wn2[:, :F] | Wn2[:, F:]]  -> dX1 into S's region, dS2 into AB[:, :32]
  mm16(N, 64, F, 0, [&](int i, int n) { return (n < F && ((xb[i] >> n) & 1u)) ? sdm[n] : 0.f; },
       [&](int n, int q) { return n < F ? (q < F ? w.wn2[n * KN + q] : (q >= 32 ? w.wn2[n * KN + F + q - 32] : 0.f)) : 0.f; },
       [&](int i, int q, float v) {
         if (q < 32) {
           if (q < F) S[i * LS + q] = v;
         } else {
           AB[i * LAB + q - 32] = v;
         }
       });
  __syncthreads();
  VSTAMP(10);
  row_bwd(srp, AB, ea, Fe, FeS, b2c, red, N);
  __syncthreads();
  {
    float* gw = slab + LG;
    if (tid < 32 * (1 + MAXFE)) {  // dbe2, dWc2 (fixed wave order)
      float t = 0.f;
      for (int wv = 0; wv < NW; ++wv) t += red[wv * REDW + tid];
      if (tid < 32) gw[32 * KE + tid] = t;
      else {
        const int c = (tid - 32) / MAXFE, f = (tid - 32) % MAXFE;
        if (f < Fe) gw[c * KE + 2 * F + f] = t;
      }
    }
    // dWa2 = D2^T X1,  dX1 += D2 Wa2
    mm16(32, F, N, 0, [&](int c, int i) { return i < N ? AB[i * LAB + 32 + c] : 0.f; },
         [&](int i, int k) { return i < N && k < F ? X1[i * LS + k] : 0.f; },
         [&](int c, int k, float v) { gw[c * KE + k] = v; });
    mm16(N, F, 32, 4, [&](int i, int c) { return c < 32 ? AB[i * LAB + 32 + c] : 0.f; },
         [&](int c, int k) { return c < 32 && k < F ? w.we2[c * KE + k] : 0.f; },
         [&](int i, int k, float v) { S[i * LS + k] += v; });
  }
  __syncthreads();
  VSTAMP(11);
  row_t(strp, stcol, AB, b2t, N);
  __syncthreads();
  {
    float* gw = slab + LG;
    // dWb2 = D'2^T X1,  dX1 += D'2 Wb2
    mm16(32, F, N, 0, [&](int c, int i) { return i < N ? AB[i * LAB + 32 + c] : 0.f; },
         [&](int i, int k) { return i < N && k < F ? X1[i * LS + k] : 0.f; },
         [&](int c, int k, float v) { gw[c * KE + F + k] = v; });
    mm16(N, F, 32, 4, [&](int i, int c) { return c < 32 ? AB[i * LAB + 32 + c] : 0.f; },
         [&](int c, int k) { return c < 32 && k < F ? w.we2[c * KE + F + k] : 0.f; },
         [&](int i, int k, float v) { S[i * LS + k] += v; });
  }
  __syncthreads();
  VSTAMP(12);
  // ---------------- layer 1 backward ---------------------------------------
  // DU1 = relu'(X1) * dX1 (in place)
  for (int q = tid; q < N * 32; q += NT) {
    const int i = q >> 5, n = q & 31;
    if (n < F) S[i * LS + n] = relu_bwd(X1[i * LS + n], S[i * LS + n]);
  }
  __syncthreads();
  {
    float* gw = slab;  // layer 1
    // dS1 = DU1 Wn1[:, F:] into AB[:, :32];  dWn1 = DU1^T [X0 | S1], dbn1 = sum DU1
    mm16(N, 32, F, 0, [&](int i, int n) { return n < F ? S[i * LS + n] : 0.f; },
         [&](int n, int c) { return n < F ? w.wn1[n * KN + F + c] : 0.f; },
         [&](int i, int c, float v) { AB[i * LAB + c] = v; });
    mm16(F, KN + 1, N, 8, [&](int n, int i) { return i < N ? S[i * LS + n] : 0.f; },
         [&](int i, int q) {
           return i < N ? (q < F ? X0[(int64_t)i * XS + q] : (q < KN ? S1g[i * 32 + q - F] : 1.f)) : 0.f;
         },
         [&](int n, int q, float v) {
           if (q < KN) gw[32 * KE + 32 + n * KN + q] = v;
           else gw[32 * KE + 32 + F * KN + n] = v;
         });
  }
  __syncthreads();
  VSTAMP(13);
  row_bwd(srp, AB, ea, Fe, FeS, b1c, red, N);
  __syncthreads();
  {
    float* gw = slab;
    if (tid < 32 * (1 + MAXFE)) {
      float t = 0.f;
      for (int wv = 0; wv < NW; ++wv) t += red[wv * REDW + tid];
      if (tid < 32) gw[32 * KE + tid] = t;
      else {
        const int c = (tid - 32) / MAXFE, f = (tid - 32) % MAXFE;
        if (f < Fe) gw[c * KE + 2 * F + f] = t;
      }
    }
    // dWa1 = D1^T X0
    mm16(32, F, N, 0, [&](int c, int i) { return i < N ? AB[i * LAB + 32 + c] : 0.f; },
         [&](int i, int k) { return i < N && k < F ? X0[(int64_t)i * XS + k] : 0.f; },
         [&](int c, int k, float v) { gw[c * KE + k] = v; });
  }
  __syncthreads();
  VSTAMP(14);
  row_t(strp, stcol, AB, b1t, N);
  __syncthreads();
  {
    float* gw = slab;
    // dWb1 = D'1^T X0
    mm16(32, F, N, 0, [&](int c, int i) { return i < N ? AB[i * LAB + 32 + c] : 0.f; },
         [&](int i, int k) { return i < N && k < F ? X0[(int64_t)i * XS + k] : 0.f; },
         [&](int c, int k, float v) { gw[c * KE + F + k] = v; });
  }
  VSTAMP(15);
}

}  // namespace

extern "C" int64_t dr_vanilla_fused_lds_bytes(int32_t n_nodes, int32_t n_edges) {
  return 4LL * vcarve(n_nodes, n_edges).total;
}

extern "C" int64_t dr_vanilla_fused_scratch_floats(int32_t n_nodes, int32_t n_edges) {
  return vscratch_floats(n_nodes, n_edges);
}

extern "C" int dr_vanilla_fused_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                                     const dr_vanilla_weights* w, const dr_pass* pass, float* scratch,
                                     const int64_t* scratch_off, int32_t lds_bytes, void* stream) {
  if (!store || !descs || !w || !pass || n_batch < 0) return DR_E_ARG;
  if (pass->out_dim < 1 || pass->out_dim > DR_MAX_OUT) return DR_E_UNSUPPORTED;
  if (store->n_feat < 1 || store->n_feat > 32 || store->x_stride > 32 || store->n_edge_feat < 0 ||
      store->n_edge_feat > MAXFE)
    return DR_E_UNSUPPORTED;
  if (!store->t_eid || !store->t_rowptr || !store->t_col || (store->n_edge_feat > 0 && !store->ea)) return DR_E_ARG;
  if (lds_bytes > 160 * 1024) return DR_E_LDS;
  if (!scratch || !scratch_off) return DR_E_ARG;
  if ((pass->flags & DR_PASS_BACKWARD) && (!pass->slab || !pass->head)) return DR_E_ARG;
  if ((pass->flags & DR_PASS_BACKWARD) && pass->loss_kind == DR_LOSS_NONE && !pass->dout) return DR_E_ARG;
  if ((pass->flags & DR_PASS_FORWARD) && !pass->out) return DR_E_ARG;
  if (pass->use_dropout != DR_DROPOUT_OFF) return DR_E_UNSUPPORTED;
  if (n_batch == 0) return DR_OK;
  DR_CHECK(dr_allow_big_lds(reinterpret_cast<const void*>(&vanilla_graph_kernel)));
  VGArgs a;
  a.s = *store;
  a.w = *w;
  a.p = *pass;
  a.descs = descs;
  a.scr = scratch;
  a.scr_off = scratch_off;
  a.B = n_batch;
  hipLaunchKernelGGL(vanilla_graph_kernel, dim3(n_batch), dim3(NT), lds_bytes, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}
