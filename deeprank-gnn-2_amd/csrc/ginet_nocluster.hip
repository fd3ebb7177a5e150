// ginet_nocluster.GINet training step, one workgroup per graph, in LDS.
//
// Replaces (deeprank2 v3.1.0):
//   GINet.forward (no clustering)   deeprank2/neuralnets/gnn/ginet_nocluster.py:84-111
//   GINetConvLayer.forward          ginet_nocluster.py:39-60 (same layer as ginet.py)
//   autograd backward + loss        deeprank2/trainer.py:686-689
//
// Both branches run conv1 -> relu -> conv2 -> relu on the full graph, then a
// per-graph scatter_mean, fc1 -> relu -> dropout -> fc2.  As in the pooled
// GINet the attention is identically 1, so conv(x) = A (x W^T) = (A x) W^T:
//   Z1 = A X, H1 = relu(Z1 [W1; W1e]^T)                  (N x 32, one MFMA GEMM)
//   Z2 = A H1, H2 = relu(Z2_b W2_b^T) per branch b       (N x 64, MFMA)
//   g  = mean_i H2_i                                      (column sums in the GEMM epilogue)
// H2 itself is never stored: the mean only needs its column sums, and the
// backward only needs relu'(H2), kept as 64 mask bits per node.  Backward:
//   dS2_i = relu'(H2_i) dG / N          (mean pooling: the same dG for every node)
//   dW2_b = sum_i dS2_i (x) Z2_i,  dZ2 = dS2 W2_b,  dS1 = relu'(H1) (A^T dZ2),
//   dW1   = sum_i dS1_i (x) Z1_i
// The per-graph partials use the pooled GINet's slab/head layout, so the same
// dr_reduce_update recipe turns them into gradients + Adam.
// Roofline: HBM-bound on the compulsory graph bytes (x, CSR + transpose) and
// the partial writes, like ginet_graph_kernel.

#include <hip/hip_runtime.h>

#include "ginet_head.h"

namespace {

using namespace drk;

constexpr int NT = 1024;
constexpr int NW = NT / 64;
constexpr int HEADW = 672;  // g64 hpre128 hh128 hd128 dh128 dg64 dout16 spare16
constexpr int LZ = 36;      // Z2 row stride: 16-byte rows (float4 gathers in the backward)

constexpr int SCRATCH = 3 * 1024;  // K-split partial tiles of the backward reductions

struct NcCarve {
  int KP, LDW, XS;
  int w1, dgp, w2, fc2, xz2, z1, h1, mask, rp, trp, col, tcol, head, dgn, total;
};

__host__ __device__ inline NcCarve nc_carve(int N, int E, int F, int OUT) {
  NcCarve c;
  c.KP = r16(F);
  c.LDW = c.KP + 2;
  c.XS = r4(F);
  int o = 0;
#define TAKE(field, words) \
  c.field = o;             \
  o += r4(words);
  // w1 and dgp are dead in the backward: together with the pad up to SCRATCH
  // words they hold the K-split partial tiles of dW2 / dW1
  TAKE(w1, 32 * c.LDW)             // [W1; W1e] row-major, zero-padded to KP
  TAKE(dgp, imax(NW * 64, SCRATCH - r4(32 * c.LDW)))  // column-sum partials of H2, then the head's dG partials
  TAKE(w2, 1024)                   // [W2 | W2e] (conv2 / conv2_ext .fc.weight)
  TAKE(fc2, OUT * 128 + OUT)
  TAKE(xz2, N * imax(c.XS, LZ))    // X, then Z2 = A H1 (X is dead after the conv1 gather), then dZ2
  TAKE(z1, N * c.LDW)              // Z1 = A X (kept for dW1)
  TAKE(h1, N * 32)                 // H1, then dS1 in place
  TAKE(mask, N * 2)                // relu'(H2) bits: word 2i+b, bit o of branch b
  TAKE(rp, N + 1)
  TAKE(trp, N + 1)
  TAKE(col, (E + 1) / 2)
  TAKE(tcol, (E + 1) / 2)
  TAKE(head, HEADW)
  TAKE(dgn, 64)                    // dG / N
#undef TAKE
  c.total = o;
  return c;
}

struct NcArgs {
  dr_graph_store s;
  dr_ginet_weights w;
  dr_pass p;
  const dr_graph_desc* descs;
  int32_t B;
};

// out[i, c4..c4+3] over rows [0, n): sum over CSR row i of Y[col[e], c4..]
// (8 lanes per row, one float4 chunk each), written with row stride ldo.
__device__ __forceinline__ void gather_rows(const int* rp, const uint16_t* col, const float* Y, int ys, int nch,
                                            float* out, int ldo, int n) {
  const int sub = threadIdx.x & 7;
  for (int i = threadIdx.x >> 3; i < n; i += NT / 8) {
    const int eb = rp[i], ee = rp[i + 1];
    for (int ch = sub; ch < nch; ch += 8) {
      const int c4 = ch * 4;
      const float4 acc = gather_row_chunk_lds(col, eb, ee, Y, ys, c4);
      float* o = out + i * ldo + c4;
      o[0] = acc.x;
      o[1] = acc.y;
      o[2] = acc.z;
      o[3] = acc.w;
    }
  }
}

__global__ void __launch_bounds__(NT) ginet_nocluster_kernel(NcArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int b = blockIdx.x;
  const dr_graph_store& s = a.s;
  const dr_graph_desc d = a.descs[b];
  const int g = d.gid;
  const int64_t n0 = d.node0, ec0 = d.col0;
  const int N = d.n_nodes, E = d.n_edges;
  const int F = s.n_feat;
  const int OUT = a.p.out_dim;
  const NcCarve c = nc_carve(N, E, F, OUT);
  const int KP = c.KP, LDW = c.LDW, XS = c.XS;

  float* sW1 = lds + c.w1;
  float* sW2 = lds + c.w2;
  float* sFc2 = lds + c.fc2;
  float* sX = lds + c.xz2;
  float* sZ2 = lds + c.xz2;
  float* sZ1 = lds + c.z1;
  float* sH1 = lds + c.h1;
  uint32_t* sMask = reinterpret_cast<uint32_t*>(lds + c.mask);
  int* srp = reinterpret_cast<int*>(lds + c.rp);
  int* strp = reinterpret_cast<int*>(lds + c.trp);
  uint16_t* scol = reinterpret_cast<uint16_t*>(lds + c.col);
  uint16_t* stcol = reinterpret_cast<uint16_t*>(lds + c.tcol);
  float* sDgp = lds + c.dgp;
  float* sScr = lds + c.w1;  // backward scratch (w1 + dgp, >= SCRATCH words)
  float* sDgN = lds + c.dgn;
  GinetHeadLds hl;
  hl.fc2 = sFc2;
  hl.g = lds + c.head;
  hl.hpre = hl.g + 64;
  hl.hh = hl.hpre + 128;
  hl.hd = hl.hh + 128;
  hl.dh = hl.hd + 128;
  hl.dg = hl.dh + 128;
  hl.dout = hl.dg + 64;
  hl.dgp = sDgp;

  DRK_STAMP(0);
  // ---------------- stage ---------------------------------------------------
  float fc1_row[8], fc1_col[8], fc1_bias;
  {
    const int r = tid >> 3, part = tid & 7;
    const float4 u0 = *reinterpret_cast<const float4*>(a.w.fc1w + r * 64 + part * 8);
    const float4 u1 = *reinterpret_cast<const float4*>(a.w.fc1w + r * 64 + part * 8 + 4);
    fc1_row[0] = u0.x; fc1_row[1] = u0.y; fc1_row[2] = u0.z; fc1_row[3] = u0.w;
    fc1_row[4] = u1.x; fc1_row[5] = u1.y; fc1_row[6] = u1.z; fc1_row[7] = u1.w;
    fc1_bias = a.w.fc1b[r];
    const int o = tid & 63, rc = tid >> 6;
#pragma unroll
    for (int j = 0; j < 8; ++j) fc1_col[j] = a.w.fc1w[(rc * 8 + j) * 64 + o];
  }
  const float y_g = s.y[g];
  uint64_t drop_offset = a.p.drop_offset;
  dma_x4<NT>(sX, s.x + n0 * (int64_t)XS, N * XS / 4);
  dma_x4<NT>(scol, s.col + ec0, (E + 7) / 8);
  dma_x4<NT>(stcol, s.t_col + ec0, (E + 7) / 8);
  dma_words<NT>(srp, s.rowptr + n0 + g, N + 1);
  dma_words<NT>(strp, s.t_rowptr + n0 + g, N + 1);
  {
    const int padw = KP - F;
    for (int p = tid; p < 32 * padw; p += NT) {
      const int i = p / padw;
      sW1[i * LDW + F + (p - i * padw)] = 0.f;
    }
    const int padz = KP - XS;
    for (int p = tid; p < N * padz; p += NT) {
      const int i = p / padz;
      sZ1[i * LDW + XS + (p - i * padz)] = 0.f;
    }
    for (int p = tid; p < 2 * N; p += NT) sMask[p] = 0u;
  }
  if (a.p.step_counter) drop_offset = (uint64_t)a.p.step_counter[0];  // loaded late: no early wait
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (a.p.step_counter && b == 0 && tid == 0) a.p.step_counter[1] = (int64_t)drop_offset;  // snapshot for dr_reduce_update
  __syncthreads();
  DRK_STAMP(1);

  float wv1[2], wv2, wfc[3];
  {
    const int n1 = 32 * F;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int p = tid + u * NT;
      wv1[u] = 0.f;
      if (p < n1) wv1[u] = (p < 16 * F) ? a.w.w1[p] : a.w.w1e[p - 16 * F];
    }
    wv2 = (tid < 512) ? a.w.w2[tid] : a.w.w2e[tid - 512];
    const int nf = OUT * 128;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int p = tid + u * NT;
      wfc[u] = 0.f;
      if (p < nf) wfc[u] = a.w.fc2w[p];
      else if (p < nf + OUT) wfc[u] = a.w.fc2b[p - nf];
    }
  }
  // ---------------- Z1 = A X (ginet_nocluster.py:45,58 reassociated) --------
  gather_rows(srp, scol, sX, XS, XS >> 2, sZ1, LDW, N);
  {
    const int n1 = 32 * F;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int p = tid + u * NT;
      if (p < n1) {
        const int r = p / F;
        sW1[r * LDW + (p - r * F)] = wv1[u];
      }
    }
    sW2[tid] = wv2;
    const int nf = OUT * 128 + OUT;
#pragma unroll
    for (int u = 0; u < 3; ++u)
      if (tid + u * NT < nf) sFc2[tid + u * NT] = wfc[u];
  }
  __syncthreads();
  DRK_STAMP(2);

  // ---------------- H1 = relu(Z1 [W1; W1e]^T) on MFMA ----------------------
  const int li = lane & 15, kq = lane >> 4;
  for (int t = wave; t * 16 < N; t += NW) {
    const int r0 = t * 16;
    const int ar = min(r0 + li, N - 1);
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < KP; k += 16) {
      float av[4], b0[4], b1[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int kk = k + 4 * u + kq;
        av[u] = sZ1[ar * LDW + kk];
        b0[u] = sW1[li * LDW + kk];
        b1[u] = sW1[(16 + li) * LDW + kk];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], b0[u], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], b1[u], acc1, 0, 0, 0);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + kq * 4 + r;
      if (row < N) {
        sH1[row * 32 + li] = relu_keepnan(acc0[r]);
        sH1[row * 32 + 16 + li] = relu_keepnan(acc1[r]);
      }
    }
  }
  __syncthreads();
  DRK_STAMP(3);

  // ---------------- Z2 = A H1 (X is dead: Z2 takes its place) ---------------
  gather_rows(srp, scol, sH1, 32, 8, sZ2, LZ, N);
  __syncthreads();
  DRK_STAMP(4);

  // ---------------- H2 = relu(Z2_b W2_b^T): column sums + relu' bits -------
  {
    float cs[4] = {0.f, 0.f, 0.f, 0.f};  // (branch, half) column partial sums of this lane
    for (int t = wave; t * 16 < N; t += NW) {
      const int r0 = t * 16;
      const int ar = min(r0 + li, N - 1);
#pragma unroll
      for (int br = 0; br < 2; ++br) {
        floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int kk = 4 * u + kq;
          const float av = sZ2[ar * LZ + br * 16 + kk];
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, sW2[(br * 32 + li) * 16 + kk], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, sW2[(br * 32 + 16 + li) * 16 + kk], acc1, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = r0 + kq * 4 + r;
          const bool live = row < N;
          if (live) {
            cs[br * 2] += relu_keepnan(acc0[r]);
            cs[br * 2 + 1] += relu_keepnan(acc1[r]);
          }
          // relu_bwd passes the gradient unless the output is <= 0 (NaN passes).
          // Lane kq*16+li holds channel li of row r0+kq*4+r: one ballot per half.
          const uint64_t lo = __ballot(live && !(acc0[r] <= 0.f));
          const uint64_t hi = __ballot(live && !(acc1[r] <= 0.f));
          if (li == 0 && live)
            sMask[row * 2 + br] = (uint32_t)((lo >> (kq * 16)) & 0xffffu) | ((uint32_t)((hi >> (kq * 16)) & 0xffffu) << 16);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // rows of a column live in lanes li, li+16, li+32, li+48
      cs[q] += __shfl_xor(cs[q], 16, 64);
      cs[q] += __shfl_xor(cs[q], 32, 64);
    }
    if (kq == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) sDgp[wave * 64 + (q >> 1) * 32 + (q & 1) * 16 + li] = cs[q];
    }
  }
  __syncthreads();
  DRK_STAMP(5);
  if (tid < 64) {  // per-graph scatter_mean (ginet_nocluster.py:103-104)
    float acc = 0.f;
    for (int w = 0; w < NW; ++w) acc += sDgp[w * 64 + tid];
    hl.g[tid] = acc / (float)N;
  }
  __syncthreads();

  // ---------------- head, loss, head backward (shared with GINet) -----------
  DRK_STAMP(6);
  if (!ginet_head<NT>(a.p, hl, fc1_row, fc1_col, fc1_bias, b, OUT, y_g, drop_offset)) return;
  DRK_STAMP(7);

  // ---------------- conv2 backward -----------------------------------------
  if (tid < 64) sDgN[tid] = hl.dg[tid] / (float)N;
  __syncthreads();
  // dW2cat[o][j] = (dG[o]/N) sum_{i: bit(i,o)} Z2[i][br*16+j]: a [64 x N] x [N x 16]
  // MFMA product with the 0/1 bit matrix as A; 4 output tiles x 4 node splits
  // (one per wave), splits combined in fixed order (deterministic)
  {
    const int ot = wave & 3, sp = wave >> 2, br = ot >> 1, sh = (ot & 1) * 16 + li;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int i0 = sp * 4; i0 < N; i0 += 16) {
      const int i = i0 + kq;
      float av = 0.f, bv = 0.f;
      if (i < N) {
        av = ((sMask[i * 2 + br] >> sh) & 1u) ? 1.f : 0.f;
        bv = sZ2[i * LZ + br * 16 + li];
      }
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
    }
    if (sp > 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) sScr[((ot * 3 + sp - 1) * 16 + kq * 4 + r) * 16 + li] = acc[r];
    }
    __syncthreads();
    if (sp == 0) {
      float* slab = a.p.slab + (int64_t)b * DR_SLAB_STRIDE(F) + 32 * F;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[r];
#pragma unroll
        for (int q = 0; q < 3; ++q) v += sScr[((ot * 3 + q) * 16 + kq * 4 + r) * 16 + li];
        const int o = ot * 16 + kq * 4 + r;
        slab[o * 16 + li] = v * sDgN[o];
      }
    }
  }
  __syncthreads();
  DRK_STAMP(8);
  // dZ2_b = dS2_b W2_b (N x 32 by 32 x 16 per branch, MFMA), in place of Z2:
  // each (row tile, branch) job reads only bits and W2 and writes its own block
  for (int job = wave; job < ((N + 15) >> 4) * 2; job += NW) {
    const int r0 = (job >> 1) * 16, br = job & 1;
    const uint32_t m = sMask[min(r0 + li, N - 1) * 2 + br];
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int ol = 4 * u + kq;
      const float av = ((m >> ol) & 1u) ? sDgN[br * 32 + ol] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, sW2[(br * 32 + ol) * 16 + li], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + kq * 4 + r;
      if (row < N) sZ2[row * LZ + br * 16 + li] = acc[r];
    }
  }
  __syncthreads();
  DRK_STAMP(9);
  // dS1 = relu'(H1) (A^T dZ2), in place of H1 (transposed CSR, true edge order)
  {
    const int sub = tid & 7;
    for (int jn = tid >> 3; jn < N; jn += NT / 8) {
      const int eb = strp[jn], ee = strp[jn + 1];
      const int c4 = sub * 4;
      const float4 acc = gather_row_chunk_lds(stcol, eb, ee, sZ2, LZ, c4);
      float* h = sH1 + jn * 32 + c4;
      h[0] = relu_bwd(h[0], acc.x);
      h[1] = relu_bwd(h[1], acc.y);
      h[2] = relu_bwd(h[2], acc.z);
      h[3] = relu_bwd(h[3], acc.w);
    }
  }
  __syncthreads();
  DRK_STAMP(10);
  // dW1cat[ch][kk] = sum_i dS1[i][ch] Z1[i][kk]: [32 x N] x [N x KP] on MFMA;
  // T = 2*KP/16 output tiles (Z1's K padding columns are zero), NW/T node
  // splits per tile (T <= 8 as F <= 64), splits combined in fixed order
  {
    const int nkt = KP >> 4, T = 2 * nkt, S = min(NW / T, 4);  // (T-tiles x (S-1) partials fit SCRATCH)
    const int tile = wave % T, sp = wave / T;
    const int ct = tile / nkt, kt = tile - ct * nkt;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    if (sp < S) {
      for (int i0 = sp * 4; i0 < N; i0 += 4 * S) {
        const int i = i0 + kq;
        float av = 0.f, bv = 0.f;
        if (i < N) {
          av = sH1[i * 32 + ct * 16 + li];
          bv = sZ1[i * LDW + kt * 16 + li];
        }
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
      }
      if (sp > 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) sScr[((tile * (S - 1) + sp - 1) * 16 + kq * 4 + r) * 16 + li] = acc[r];
      }
    }
    __syncthreads();
    const int kk = kt * 16 + li;
    if (sp == 0 && kk < F) {
      float* slab = a.p.slab + (int64_t)b * DR_SLAB_STRIDE(F);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[r];
        for (int q = 0; q < S - 1; ++q) v += sScr[((tile * (S - 1) + q) * 16 + kq * 4 + r) * 16 + li];
        slab[(ct * 16 + kq * 4 + r) * F + kk] = v;
      }
    }
  }
  __syncthreads();
  DRK_STAMP(11);
}

// ---- graphs beyond one workgroup's LDS: the pipeline of dr_ginet_nocluster_large_pass ----
constexpr int TB = 256;   // tile kernels: 4 waves, one 16-row MFMA tile each
constexpr int NCT = 64;   // rows per tile (at most)

__host__ __device__ inline int nc_part(int F) { return 64 + 64 * 16 + 32 * F; }  // H2 column sums | dW2 (raw) | dW1

struct NcLarge {
  int64_t z1, h1, z2, dz2, mask, dgn, part, total;
};
__host__ __device__ inline NcLarge nc_large_layout(int64_t R, int B, int n_tiles, int F) {
  NcLarge c;
  int64_t o = 0;
  c.z1 = o;
  o += R * r4(F);
  c.h1 = o;
  o += R * 32;
  c.z2 = o;
  o += R * 32;
  c.dz2 = o;
  o += R * 32;
  c.mask = o;
  o += R * 2;
  c.dgn = o;
  o += (int64_t)B * 64;
  c.part = o;
  o += (int64_t)n_tiles * nc_part(F);
  c.total = o;
  return c;
}

// LDS (floats) of the tile kernels: halo rows [HM][32] | tile rows A [64][LDW] |
// tile rows B [64][36] | weights [32][LDW] + 1024 | edges (uint16) | spare
__host__ __device__ inline int nc_halo_w(int F) { return imax(32, r4(F)); }  // halo row stride: X rows (r4(F)) or 32-wide node rows
__host__ __device__ inline int nc_tile_lds(int F, int HM, int EM, int TM) {
  const int LDW = r16(F) + 2;
  return HM * nc_halo_w(F) + NCT * LDW + NCT * 36 + 32 * LDW + 1024 + 256 + r4((imax(EM, TM) + 8) / 2);
}

struct NcLargeArgs {
  dr_graph_store s;
  dr_ginet_weights w;
  dr_pass p;
  const dr_graph_desc* descs;
  dr_nc_plan pl;
  NcLarge L;
  int32_t B;
};

struct NcTile {
  int t, b, nrows, i0, h0, H;
  int64_t r0, g0;
  const int* rp;
  const int* trp;
};
__device__ __forceinline__ NcTile nc_tile(const NcLargeArgs& a) {
  NcTile q;
  q.t = xcd_tile();
  q.r0 = a.pl.tile_row0[q.t];
  q.nrows = (int)(a.pl.tile_row0[q.t + 1] - q.r0);
  q.b = a.pl.row_slot[q.r0];
  q.g0 = a.pl.row0[q.b];
  q.i0 = (int)(q.r0 - q.g0);
  const dr_graph_desc& d = a.descs[q.b];
  q.rp = a.s.rowptr + d.node0 + d.gid;
  q.trp = a.s.t_rowptr + d.node0 + d.gid;
  q.h0 = a.pl.halo_off[q.t];
  q.H = a.pl.halo_off[q.t + 1] - q.h0;
  return q;
}

// rows of a [rows][W] node array (graph block at g) at the tile's halo ids -> LDS [H][W], 16-byte pieces
__device__ __forceinline__ void nc_stage_halo(float* dst, const float* g, int W, const int* ids, int H) {
  const int nch = W / 4;
  for (int p = threadIdx.x; p < H * nch; p += TB) {
    const int h = p / nch, c4 = (p - h * nch) * 4;
    *reinterpret_cast<float4*>(dst + h * W + c4) = *reinterpret_cast<const float4*>(g + (int64_t)ids[h] * W + c4);
  }
}
__device__ __forceinline__ void nc_stage_u16(uint16_t* dst, const uint16_t* src, int n) {
  for (int p = threadIdx.x; p < n; p += TB) dst[p] = src[p];
}

// 1. Z1 = A X, H1 = relu(Z1 [W1; W1e]^T)
__global__ void __launch_bounds__(TB) nc_l_conv1(NcLargeArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const NcTile q = nc_tile(a);
  const int F = a.s.n_feat, XS = r4(F), KP = r16(F), LDW = KP + 2;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, kq = lane >> 4;
  const dr_graph_desc& d = a.descs[q.b];
  float* sXh = lds;                       // [H][XS]
  float* sZ = sXh + a.pl.halo_max * nc_halo_w(F);  // [64][LDW]
  float* sW1 = sZ + NCT * LDW + NCT * 36; // [32][LDW]
  uint16_t* sLc = reinterpret_cast<uint16_t*>(sW1 + 32 * LDW + 1024 + 256);
  const int e0 = q.rp[q.i0], ne = q.rp[q.i0 + q.nrows] - e0;
  nc_stage_halo(sXh, a.s.x + d.node0 * (int64_t)XS, XS, a.pl.halo_ids + q.h0, q.H);
  nc_stage_u16(sLc, a.pl.lcol + a.pl.lcol_off[q.t], ne);
  for (int p = tid; p < 32 * LDW; p += TB) {
    const int r = p / LDW, k = p - r * LDW;
    sW1[p] = k < F ? (r < 16 ? a.w.w1[r * F + k] : a.w.w1e[(r - 16) * F + k]) : 0.f;
  }
  for (int p = tid; p < NCT * (LDW - XS); p += TB) {  // Z pad columns
    const int r = p / (LDW - XS);
    sZ[r * LDW + XS + p - r * (LDW - XS)] = 0.f;
  }
  __syncthreads();
  float* z1 = a.pl.base + a.L.z1;
  {
    const int sub = tid & 7, nch = XS >> 2;
    for (int r = tid >> 3; r < q.nrows; r += TB / 8) {
      const int eb = q.rp[q.i0 + r] - e0, ee = q.rp[q.i0 + r + 1] - e0;
      for (int ch = sub; ch < nch; ch += 8) {
        const int c4 = ch * 4;
        const float4 acc = gather_row_chunk_lds(sLc, eb, ee, sXh, XS, c4);
        float* zr = sZ + r * LDW + c4;
        zr[0] = acc.x;
        zr[1] = acc.y;
        zr[2] = acc.z;
        zr[3] = acc.w;
        *reinterpret_cast<float4*>(z1 + (q.r0 + r) * XS + c4) = acc;
      }
    }
  }
  __syncthreads();
  float* h1 = a.pl.base + a.L.h1;
  const int r0 = wave * 16;
  if (r0 < q.nrows) {
    const int ar = min(r0 + li, q.nrows - 1);
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < KP; k += 16) {
      float av[4], b0[4], b1[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int kk = k + 4 * u + kq;
        av[u] = sZ[ar * LDW + kk];
        b0[u] = sW1[li * LDW + kk];
        b1[u] = sW1[(16 + li) * LDW + kk];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], b0[u], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], b1[u], acc1, 0, 0, 0);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + kq * 4 + r;
      if (row < q.nrows) {
        h1[(q.r0 + row) * 32 + li] = relu_keepnan(acc0[r]);
        h1[(q.r0 + row) * 32 + 16 + li] = relu_keepnan(acc1[r]);
      }
    }
  }
}

// 2. Z2 = A H1, H2 = relu(Z2_b W2_b^T): relu' bits, the tile's column sums of H2
__global__ void __launch_bounds__(TB) nc_l_conv2(NcLargeArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const NcTile q = nc_tile(a);
  const int F = a.s.n_feat, KP = r16(F), LDW = KP + 2;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, kq = lane >> 4;
  float* sHh = lds;                           // [H][32]
  float* sZ2 = sHh + a.pl.halo_max * nc_halo_w(F) + NCT * LDW;  // [64][LZ]
  float* sW2 = sZ2 + NCT * 36 + 32 * LDW;     // [64][16]
  float* sRed = sW2 + 1024;                   // [4][64]
  uint16_t* sLc = reinterpret_cast<uint16_t*>(sRed + 256);
  const int e0 = q.rp[q.i0], ne = q.rp[q.i0 + q.nrows] - e0;
  const float* h1 = a.pl.base + a.L.h1;
  nc_stage_halo(sHh, h1 + q.g0 * 32, 32, a.pl.halo_ids + q.h0, q.H);
  nc_stage_u16(sLc, a.pl.lcol + a.pl.lcol_off[q.t], ne);
  for (int p = tid; p < 1024; p += TB) sW2[p] = p < 512 ? a.w.w2[p] : a.w.w2e[p - 512];
  __syncthreads();
  float* z2 = a.pl.base + a.L.z2;
  {
    const int sub = tid & 7;
    for (int r = tid >> 3; r < q.nrows; r += TB / 8) {
      const int eb = q.rp[q.i0 + r] - e0, ee = q.rp[q.i0 + r + 1] - e0;
      const int c4 = sub * 4;
      const float4 acc = gather_row_chunk_lds(sLc, eb, ee, sHh, 32, c4);
      float* zr = sZ2 + r * LZ + c4;
      zr[0] = acc.x;
      zr[1] = acc.y;
      zr[2] = acc.z;
      zr[3] = acc.w;
      *reinterpret_cast<float4*>(z2 + (q.r0 + r) * 32 + c4) = acc;
    }
  }
  __syncthreads();
  uint32_t* mask = reinterpret_cast<uint32_t*>(a.pl.base + a.L.mask);
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  const int r0 = wave * 16;
  if (r0 < q.nrows) {
    const int ar = min(r0 + li, q.nrows - 1);
#pragma unroll
    for (int br = 0; br < 2; ++br) {
      floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int kk = 4 * u + kq;
        const float av = sZ2[ar * LZ + br * 16 + kk];
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, sW2[(br * 32 + li) * 16 + kk], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, sW2[(br * 32 + 16 + li) * 16 + kk], acc1, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + kq * 4 + r;
        const bool live = row < q.nrows;
        if (live) {
          cs[br * 2] += relu_keepnan(acc0[r]);
          cs[br * 2 + 1] += relu_keepnan(acc1[r]);
        }
        const uint64_t lo = __ballot(live && !(acc0[r] <= 0.f));
        const uint64_t hi = __ballot(live && !(acc1[r] <= 0.f));
        if (li == 0 && live)
          mask[(q.r0 + row) * 2 + br] = (uint32_t)((lo >> (kq * 16)) & 0xffffu) | ((uint32_t)((hi >> (kq * 16)) & 0xffffu) << 16);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    cs[c] += __shfl_xor(cs[c], 16, 64);
    cs[c] += __shfl_xor(cs[c], 32, 64);
  }
  if (kq == 0) {
#pragma unroll
    for (int c = 0; c < 4; ++c) sRed[wave * 64 + (c >> 1) * 32 + (c & 1) * 16 + li] = cs[c];
  }
  __syncthreads();
  if (tid < 64) {
    float v = 0.f;
    for (int w = 0; w < TB / 64; ++w) v += sRed[w * 64 + tid];
    a.pl.base[a.L.part + (int64_t)q.t * nc_part(F) + tid] = v;
  }
}

// 3. per graph: mean over the tiles' column sums, the GINet head, loss and head backward
__global__ void __launch_bounds__(NT) nc_l_head(NcLargeArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x;
  const int b = blockIdx.x;
  const dr_graph_desc d = a.descs[b];
  const int F = a.s.n_feat, OUT = a.p.out_dim;
  const int N = a.pl.row0[b + 1] - a.pl.row0[b];
  float fc1_row[8], fc1_col[8], fc1_bias;
  {
    const int r = tid >> 3, part = tid & 7;
#pragma unroll
    for (int j = 0; j < 8; ++j) fc1_row[j] = a.w.fc1w[r * 64 + part * 8 + j];
    fc1_bias = a.w.fc1b[r];
    const int o = tid & 63, rc = tid >> 6;
#pragma unroll
    for (int j = 0; j < 8; ++j) fc1_col[j] = a.w.fc1w[(rc * 8 + j) * 64 + o];
  }
  GinetHeadLds hl;
  hl.fc2 = lds;
  hl.g = lds + r4(OUT * 129);
  hl.hpre = hl.g + 64;
  hl.hh = hl.hpre + 128;
  hl.hd = hl.hh + 128;
  hl.dh = hl.hd + 128;
  hl.dg = hl.dh + 128;
  hl.dout = hl.dg + 64;
  hl.dgp = hl.dout + 16;  // [NW][64]
  for (int p = tid; p < OUT * 129; p += NT) hl.fc2[p] = p < OUT * 128 ? a.w.fc2w[p] : a.w.fc2b[p - OUT * 128];
  const float y_g = a.s.y[d.gid];
  uint64_t drop_offset = a.p.drop_offset;
  if (a.p.step_counter) drop_offset = (uint64_t)a.p.step_counter[0];
  if (tid < 64) {
    // tiles in order, 8 tiles' loads in flight (as nc_l_combine)
    const float* part = a.pl.base + a.L.part + tid;
    const int te = a.pl.tile_first[b + 1], NP = nc_part(F);
    float v = 0.f;
    int t = a.pl.tile_first[b];
    for (; t + 8 <= te; t += 8) {
      float u[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) u[k] = part[(int64_t)(t + k) * NP];
#pragma unroll
      for (int k = 0; k < 8; ++k) v += u[k];
    }
    for (; t < te; ++t) v += part[(int64_t)t * NP];
    hl.g[tid] = v / (float)N;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (a.p.step_counter && b == 0 && tid == 0) a.p.step_counter[1] = (int64_t)drop_offset;  // snapshot for dr_reduce_update
  __syncthreads();
  const int row = a.p.slot ? a.p.slot[b] : b;
  if (!ginet_head<NT>(a.p, hl, fc1_row, fc1_col, fc1_bias, row, OUT, y_g, drop_offset)) return;
  if (tid < 64) a.pl.base[a.L.dgn + (int64_t)b * 64 + tid] = hl.dg[tid] / (float)N;
}

// 4. dZ2 = dS2_b W2_b (dS2 = relu'(H2) dG / N) and the tile's dW2 partial sum_i bit(i, o) Z2[i][j]
__global__ void __launch_bounds__(TB) nc_l_bwd2(NcLargeArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const NcTile q = nc_tile(a);
  const int F = a.s.n_feat;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, kq = lane >> 4;
  float* sZ2 = lds;                 // [64][LZ]
  float* sW2 = sZ2 + NCT * LZ;      // [64][16]
  float* sDgN = sW2 + 1024;         // [64]
  uint32_t* sMask = reinterpret_cast<uint32_t*>(sDgN + 64);  // [64][2]
  const float* z2 = a.pl.base + a.L.z2 + q.r0 * 32;
  const uint32_t* mask = reinterpret_cast<const uint32_t*>(a.pl.base + a.L.mask) + q.r0 * 2;
  for (int p = tid; p < NCT * 8; p += TB) {
    const int r = p >> 3, c4 = (p & 7) * 4;
    const float4 v = r < q.nrows ? *reinterpret_cast<const float4*>(z2 + r * 32 + c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(sZ2 + r * LZ + c4) = v;
  }
  for (int p = tid; p < NCT * 2; p += TB) sMask[p] = p < q.nrows * 2 ? mask[p] : 0u;
  for (int p = tid; p < 1024; p += TB) sW2[p] = p < 512 ? a.w.w2[p] : a.w.w2e[p - 512];
  if (tid < 64) sDgN[tid] = a.pl.base[a.L.dgn + (int64_t)q.b * 64 + tid];
  __syncthreads();
  // the tile's dW2 partial: output tile ot (branch br, 16 channels) per wave, K = the tile's rows
  {
    const int ot = wave, br = ot >> 1, sh = (ot & 1) * 16 + li;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int i0 = 0; i0 < q.nrows; i0 += 4) {
      const int i = i0 + kq;
      float av = 0.f, bv = 0.f;
      if (i < q.nrows) {
        av = ((sMask[i * 2 + br] >> sh) & 1u) ? 1.f : 0.f;
        bv = sZ2[i * LZ + br * 16 + li];
      }
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
    }
    float* part = a.pl.base + a.L.part + (int64_t)q.t * nc_part(F) + 64;
#pragma unroll
    for (int r = 0; r < 4; ++r) part[(ot * 16 + kq * 4 + r) * 16 + li] = acc[r];
  }
  float* dz2 = a.pl.base + a.L.dz2;
  for (int job = wave; job < ((q.nrows + 15) >> 4) * 2; job += TB / 64) {
    const int r0 = (job >> 1) * 16, br = job & 1;
    const uint32_t m = sMask[min(r0 + li, q.nrows - 1) * 2 + br];
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int ol = 4 * u + kq;
      const float av = ((m >> ol) & 1u) ? sDgN[br * 32 + ol] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, sW2[(br * 32 + ol) * 16 + li], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + kq * 4 + r;
      if (row < q.nrows) dz2[(q.r0 + row) * 32 + br * 16 + li] = acc[r];
    }
  }
}

// 5. dS1 = relu'(H1) (A^T dZ2) for the tile's rows and the tile's dW1 partial sum_i dS1_i (x) Z1_i
__global__ void __launch_bounds__(TB) nc_l_bwd1(NcLargeArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const NcTile q = nc_tile(a);
  const int F = a.s.n_feat, XS = r4(F), KP = r16(F), LDW = KP + 2;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, kq = lane >> 4;
  float* sDh = lds;                            // [H][32] halo dZ2 rows
  float* sZ1 = sDh + a.pl.halo_max * nc_halo_w(F);  // [64][LDW]
  float* sS1 = sZ1 + NCT * LDW;                // [64][LZ] H1, then dS1
  uint16_t* sLt = reinterpret_cast<uint16_t*>(sS1 + NCT * 36 + 32 * LDW + 1024 + 256);
  const int q0 = q.trp[q.i0], nq = q.trp[q.i0 + q.nrows] - q0;
  nc_stage_halo(sDh, a.pl.base + a.L.dz2 + q.g0 * 32, 32, a.pl.halo_ids + q.h0, q.H);
  nc_stage_u16(sLt, a.pl.ltcol + a.pl.ltcol_off[q.t], nq);
  const float* z1 = a.pl.base + a.L.z1 + q.r0 * XS;
  const float* h1 = a.pl.base + a.L.h1 + q.r0 * 32;
  for (int p = tid; p < NCT * LDW; p += TB) {
    const int r = p / LDW, k = p - r * LDW;
    sZ1[p] = (r < q.nrows && k < XS) ? z1[r * XS + k] : 0.f;
  }
  for (int p = tid; p < NCT * 8; p += TB) {
    const int r = p >> 3, c4 = (p & 7) * 4;
    const float4 v = r < q.nrows ? *reinterpret_cast<const float4*>(h1 + r * 32 + c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(sS1 + r * LZ + c4) = v;
  }
  __syncthreads();
  {
    const int sub = tid & 7, c4 = sub * 4;
    for (int r = tid >> 3; r < q.nrows; r += TB / 8) {
      const int eb = q.trp[q.i0 + r] - q0, ee = q.trp[q.i0 + r + 1] - q0;
      const float4 acc = gather_row_chunk_lds(sLt, eb, ee, sDh, 32, c4);
      float* h = sS1 + r * LZ + c4;
      h[0] = relu_bwd(h[0], acc.x);
      h[1] = relu_bwd(h[1], acc.y);
      h[2] = relu_bwd(h[2], acc.z);
      h[3] = relu_bwd(h[3], acc.w);
    }
  }
  __syncthreads();
  // dW1cat[ch][kk] = sum_{i in tile} dS1[i][ch] Z1[i][kk]: 2 x KP/16 output tiles over the waves, K = the tile's rows
  const int nkt = KP >> 4;
  float* part = a.pl.base + a.L.part + (int64_t)q.t * nc_part(F) + 64 + 1024;
  for (int job = wave; job < 2 * nkt; job += TB / 64) {
    const int ct = job / nkt, kt = job - ct * nkt;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int i0 = 0; i0 < q.nrows; i0 += 4) {
      const int i = i0 + kq;
      const float av = i < q.nrows ? sS1[i * LZ + ct * 16 + li] : 0.f;
      const float bv = i < q.nrows ? sZ1[i * LDW + kt * 16 + li] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
    }
    const int kk = kt * 16 + li;
    if (kk < F) {
#pragma unroll
      for (int r = 0; r < 4; ++r) part[(ct * 16 + kq * 4 + r) * F + kk] = acc[r];
    }
  }
}

// 6. per graph: the tiles' partials in tile order into the slab (dW2 scaled by
// dG / N); block (graph, chunk of TB outputs), 8 tiles' loads in flight
__global__ void __launch_bounds__(TB) nc_l_combine(NcLargeArgs a) {
  const int F = a.s.n_feat, NP = nc_part(F), NO = 32 * F + 1024;
  const int chunks = (NO + TB - 1) / TB;
  const int b = blockIdx.x / chunks, p = (blockIdx.x - b * chunks) * TB + threadIdx.x;
  if (p >= NO) return;
  const int row = a.p.slot ? a.p.slot[b] : b;
  const int tb = a.pl.tile_first[b], te = a.pl.tile_first[b + 1];
  const int off = p < 32 * F ? 64 + 1024 + p : 64 + p - 32 * F;
  const float* part = a.pl.base + a.L.part + off;
  float v = 0.f;
  int t = tb;
  for (; t + 8 <= te; t += 8) {
    float u[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) u[k] = part[(int64_t)(t + k) * NP];
#pragma unroll
    for (int k = 0; k < 8; ++k) v += u[k];
  }
  for (; t < te; ++t) v += part[(int64_t)t * NP];
  if (p >= 32 * F) v *= a.pl.base[a.L.dgn + (int64_t)b * 64 + (p - 32 * F) / 16];
  a.p.slab[(int64_t)row * DR_SLAB_STRIDE(F) + p] = v;
}

}  // namespace

extern "C" int64_t dr_ginet_nocluster_lds_bytes(int32_t n_nodes, int32_t n_edges, int32_t n_feat, int32_t out_dim) {
  return 4LL * nc_carve(n_nodes, n_edges, n_feat, out_dim).total;
}

extern "C" int dr_ginet_nocluster_graph_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                                             const dr_ginet_weights* w, const dr_pass* pass, int32_t lds_bytes,
                                             void* stream) {
  if (!store || !descs || !w || !pass || n_batch < 0) return DR_E_ARG;
  if (pass->out_dim < 1 || pass->out_dim > DR_MAX_OUT) return DR_E_UNSUPPORTED;
  if (store->n_feat < 1 || 32 * store->n_feat > 2 * NT) return DR_E_UNSUPPORTED;  // F <= 64
  if (lds_bytes > 160 * 1024) return DR_E_LDS;
  if ((pass->flags & DR_PASS_BACKWARD) && (!pass->slab || !pass->head)) return DR_E_ARG;
  if ((pass->flags & DR_PASS_BACKWARD) && pass->loss_kind == DR_LOSS_NONE && !pass->dout) return DR_E_ARG;
  if ((pass->flags & DR_PASS_FORWARD) && !pass->out) return DR_E_ARG;
  if (pass->use_dropout == DR_DROPOUT_MASK && !pass->mask) return DR_E_ARG;
  if (pass->use_dropout < DR_DROPOUT_OFF || pass->use_dropout > DR_DROPOUT_HASH) return DR_E_ARG;
  if (n_batch == 0) return DR_OK;
  DR_CHECK(dr_allow_big_lds(reinterpret_cast<const void*>(&ginet_nocluster_kernel)));
  NcArgs args;
  args.s = *store;
  args.w = *w;
  args.p = *pass;
  args.descs = descs;
  args.B = n_batch;
  hipLaunchKernelGGL(ginet_nocluster_kernel, dim3(n_batch), dim3(NT), lds_bytes, (hipStream_t)stream, args);
  return (int)hipGetLastError();
}

extern "C" int64_t dr_nc_large_scratch_floats(int64_t n_rows, int32_t n_batch, int32_t n_tiles, int32_t n_feat) {
  return nc_large_layout(n_rows, n_batch, n_tiles, n_feat).total;
}

extern "C" int64_t dr_nc_large_lds_bytes(int32_t n_feat, int32_t halo_max, int32_t tile_edges_max, int32_t tile_tedges_max,
                                         int32_t out_dim) {
  const int64_t tile = 4LL * nc_tile_lds(n_feat, halo_max, tile_edges_max, tile_tedges_max);
  const int64_t head = 4LL * (r4(out_dim * 129) + 64 + 4 * 128 + 64 + 16 + NW * 64);
  return tile > head ? tile : head;
}

extern "C" int dr_ginet_nocluster_large_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                                             const dr_nc_plan* plan, const dr_ginet_weights* w, const dr_pass* pass,
                                             void* stream) {
  if (!store || !descs || !w || !pass || !plan || n_batch < 0) return DR_E_ARG;
  if (pass->out_dim < 1 || pass->out_dim > DR_MAX_OUT) return DR_E_UNSUPPORTED;
  if (store->n_feat < 1 || store->n_feat > 64 || pass->compute_dtype != DR_DTYPE_F32) return DR_E_UNSUPPORTED;
  if (!plan->base || !plan->row0 || !plan->row_slot || !plan->tile_row0 || !plan->tile_first || !plan->halo_off ||
      !plan->halo_ids || !plan->lcol_off || !plan->lcol || !plan->ltcol_off || !plan->ltcol ||
      plan->n_tiles < 1 || plan->halo_max < 1 || plan->halo_max > 65535)
    return DR_E_ARG;
  if ((pass->flags & DR_PASS_BACKWARD) && (!pass->slab || !pass->head)) return DR_E_ARG;
  if ((pass->flags & DR_PASS_BACKWARD) && pass->loss_kind == DR_LOSS_NONE && !pass->dout) return DR_E_ARG;
  if ((pass->flags & DR_PASS_FORWARD) && !pass->out) return DR_E_ARG;
  if (pass->use_dropout == DR_DROPOUT_MASK && !pass->mask) return DR_E_ARG;
  if (pass->use_dropout < DR_DROPOUT_OFF || pass->use_dropout > DR_DROPOUT_HASH) return DR_E_ARG;
  const int64_t lds = dr_nc_large_lds_bytes(store->n_feat, plan->halo_max, plan->tile_edges_max, plan->tile_tedges_max, pass->out_dim);
  if (lds > 160 * 1024) return DR_E_LDS;
  if (n_batch == 0) return DR_OK;
  const void* fns[] = {reinterpret_cast<const void*>(&nc_l_conv1), reinterpret_cast<const void*>(&nc_l_conv2),
                       reinterpret_cast<const void*>(&nc_l_head), reinterpret_cast<const void*>(&nc_l_bwd2),
                       reinterpret_cast<const void*>(&nc_l_bwd1)};
  for (const void* f : fns) DR_CHECK(dr_allow_big_lds(f));
  NcLargeArgs a;
  a.s = *store;
  a.w = *w;
  a.p = *pass;
  a.descs = descs;
  a.pl = *plan;
  a.B = n_batch;
  a.L = nc_large_layout(plan->n_rows, n_batch, plan->n_tiles, store->n_feat);
  hipStream_t st = (hipStream_t)stream;
  const dim3 tiles((unsigned)plan->n_tiles);
  hipLaunchKernelGGL(nc_l_conv1, tiles, dim3(TB), lds, st, a);
  hipLaunchKernelGGL(nc_l_conv2, tiles, dim3(TB), lds, st, a);
  hipLaunchKernelGGL(nc_l_head, dim3(n_batch), dim3(NT), lds, st, a);
  if (pass->flags & DR_PASS_BACKWARD) {
    hipLaunchKernelGGL(nc_l_bwd2, tiles, dim3(TB), lds, st, a);
    hipLaunchKernelGGL(nc_l_bwd1, tiles, dim3(TB), lds, st, a);
    hipLaunchKernelGGL(nc_l_combine, dim3(n_batch * ((32 * store->n_feat + 1024 + TB - 1) / TB)), dim3(TB), 0, st, a);
  }
  return (int)hipGetLastError();
}

// ---- carve descriptions for the host-side carve tests (tests/test_lds_carves.py)
extern "C" int dr_debug_carve_nocluster(const int32_t* q, char* buf, int32_t len) {
  const NcCarve c = nc_carve(q[0], q[1], q[2], q[3]);
  DrCarveDesc d{buf, len, 0};
  DR_DESC_P(d, c, KP);
  DR_DESC_P(d, c, LDW);
  DR_DESC_P(d, c, XS);
  DR_DESC(d, c, w1);
  DR_DESC(d, c, dgp);
  DR_DESC(d, c, w2);
  DR_DESC(d, c, fc2);
  DR_DESC(d, c, xz2);
  DR_DESC(d, c, z1);
  DR_DESC(d, c, h1);
  DR_DESC(d, c, mask);
  DR_DESC(d, c, rp);
  DR_DESC(d, c, trp);
  DR_DESC(d, c, col);
  DR_DESC(d, c, tcol);
  DR_DESC(d, c, head);
  DR_DESC(d, c, dgn);
  DR_DESC(d, c, total);
  return d.pos;
}

