// VanillaNetwork training step, one workgroup per graph (residue-size graphs).
//
// Replaces (deeprank2 v3.1.0):
//   VanillaConvolutionalLayer.forward  deeprank2/neuralnets/gnn/vanilla_gnn.py:26-38
//   VanillaNetwork.forward             vanilla_gnn.py:59-65
//   autograd backward + loss           deeprank2/trainer.py:686-689
//
// Per layer:  m_e = relu(We [x_i | x_j | ea_e] + be)  for each edge e = (i -> j),
//             s_i = sum_{e: src i} m_e,   x'_i = relu(Wn [x_i | s_i] + bn).
// The edge GEMM is split, We = [Wa | Wb | Wc]: B = X Wb^T is a node GEMM (MFMA),
// A_i = Wa x_i + be is formed per CSR row inside the row pass, and
// pre_e = A_i + B_j + Wc ea_e is rebuilt per edge, so the E x 32 messages never
// exist.  While it sums s_i, the row pass stores each edge's ReLU pattern (one
// 32-bit word, bit c = channel c active) in CSR order, eight edges of a row per
// 32-byte store.  The backward never recomputes pre_e:
//   cnt_i[c] = #{e in row i : word_e bit c},  eap_i[c][f] = sum of ea_e[f] over those edges
//   D_i  = dS_i * cnt_i,  dWc = sum_i dS_i * eap_i,  dbe = sum_i D_i
//                                          (one CSR pass over words + edge attributes)
//   D'_j = sum_{e=(i->j) active} dS_i     (transposed pass on the words, gathered through t_eid)
//   dWa = D^T X, dWb = D'^T X, dX = [DU | D | D'] [Wn[:, :F]; Wa; Wb]   (MFMA)
// and relu'(X2) is kept as one bit word per node, so dWn2 = dmean * (mask^T [X1|S2]).
//
// Memory plan (LDS, 4-byte words; slots are N x 34, the stride that makes the
// MFMA operand reads conflict free):
//   forward : P = X0 -> B2 -> X2,  Q = B1 -> X1,  R = S1 -> S2,
//             U = one 16-byte record per edge {B row byte offset | transposed slot, ea[0..2]} (+ ea[3])
//   backward: P = dS2 -> dX1 -> DU1 -> D'1,  Q = X1 -> X0,  R = D2 -> S1 -> D1,
//             U = T (D'2 -> dS1) | ReLU words (transposed) | transposed CSR
// Written once, read back much later, and too big to keep: S1 and the ReLU
// words go to a per-graph global scratch (L2-resident) and come back by bulk
// loads (S1, own rows) and gathers (the words of the transposed slots).  GEMM weights (the MFMA B
// operand) are loaded from global into registers once per phase and wave.
//
// Split (k = 2..4 workgroups per graph, so a small batch fills the chip):
// workgroup r owns the CSR rows [r0, r1) (edge-balanced bounds every sibling
// computes alike) and runs every row-parallel phase on them; the weight
// gradients are per-workgroup partials (slab row b*k + r, summed by
// dr_reduce_update).  What crosses rows is exchanged through the scratch,
// in-launch (MI355X_MICROARCH.md hand-off row 1: sc1 stores drained by every
// wave, one agent-scope arrival per workgroup, an sc1 poll, sc1 loads):
//   1. B2 rows (B1 is recomputed by every sibling from X0),
//   2. the per-workgroup column sums of X2 (then every sibling runs the head),
//   3. dS2 rows and 4. dS1 rows (the transposed passes gather them by source);
// the edge ReLU words cross with them (stored sc1 in the forward row passes).
// Siblings sit 8 blocks apart (one XCD under round-robin dispatch; placement
// only affects speed) within a window of 8k consecutive blocks.
// Bound: HBM on the compulsory inputs (x, CSR + transpose, edge_attr) and the
// per-graph gradient partials; in practice the per-graph critical path — see
// DESIGN.md §5.

#include <hip/hip_runtime.h>

#include "../../include/deeprank2_amd.h"
#include "graph_common.h"

namespace {

using namespace drk;

constexpr int NT = 1024;  // 16 waves
constexpr int NW = NT / 64;
constexpr int MAXFE = 4;  // edge features handled by this kernel (more: the pipeline)
constexpr int LS = 34;    // slot row stride
constexpr int HEADW = 512;

struct VCarve {
  int rp, xb, head, P, Q, R, U, ext, T, bt, trp, tcol, total;
};

__host__ __device__ inline int vslot(int N, int Fe) {
  const int red = NW * 32 * (1 + Fe) + 1024;  // the D pass partials + its edge buffer (>= 1024 words) live in P or T
  return imax(r4(N * LS), imax(red, 1024));
}

__host__ __device__ inline VCarve vcarve(int N, int E, int Fe) {
  VCarve c;
  int o = 0;
#define TAKE(field, words) \
  c.field = o;             \
  o += r4(words);
  TAKE(rp, N + 1)
  TAKE(xb, N)
  TAKE(head, HEADW)
  TAKE(P, vslot(N, Fe))
  TAKE(Q, r4(N * LS))
  TAKE(R, r4(N * LS))
#undef TAKE
  c.U = o;
  // 16 zero records past the last edge: a row pass may read up to 15 records
  // beyond its row (masked), never beyond these
  c.ext = c.U + 4 * (E + 16);  // ea[3] per edge behind the records (Fe == 4)
  const int fwd = 4 * (E + 16) + (Fe > 3 ? E + 16 : 0);
  c.T = c.U;
  c.bt = c.T + vslot(N, Fe);
  c.trp = c.bt + r4(E);
  c.tcol = c.trp + r4(N + 1);
  const int bwd = c.tcol + r4((E + 1) / 2) - c.U;
  c.total = c.U + r4(imax(fwd, bwd));
  return c;
}

// per-graph global scratch (floats): S1 [32N] | bt1 [E + 1] | bt2 [E + 1] (ReLU words, CSR order) |
// split exchange: XA [32N] (B2, then dS1) | XB [32N] (dS2) | column sums [MAX_SPLIT][32]
constexpr int MAXK = DR_VANILLA_MAX_SPLIT;
__host__ __device__ inline int64_t vscratch_floats(int N, int E, int Fe) {
  (void)Fe;
  return 3LL * r4(32 * N) + 2LL * r4(E + 1) + 32 * MAXK;
}

struct VGArgs {
  dr_graph_store s;
  dr_vanilla_weights w;
  dr_pass p;
  const dr_graph_desc* descs;
  float* scr;
  const int64_t* scr_off;
  uint32_t* sync;  // [2B + 1]: per graph {arrivals, exits}; [2B]: hand-off timeout flag
  const float* wpack;  // [WPACK_FLOATS]: the weights in fragment order (vanilla_pack_kernel)
  int32_t B, k;
};

typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) uint64_t gu64;

// write-through (sc1) stores and L1-bypassing (sc1) loads of handed-off bytes
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store((gu32*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_u32(uint32_t* p, uint32_t v) {
  __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_f2(float* p, float a, float b) {
  const uint64_t v = (uint64_t)__float_as_uint(a) | ((uint64_t)__float_as_uint(b) << 32);
  __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __uint_as_float(__hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ uint32_t ld_sc1_u32(const uint32_t* p) {
  return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_sc1_u64(const float* p) {
  return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Hand-off among the k workgroups of a graph.  Every wave drains its (sc1)
// stores, then one lane arrives on the graph's counter and polls it (sc1)
// until all k siblings have arrived at this hand-off; the counter only grows
// within a launch (the h-th hand-off completes at h*k), so arrival v waits for
// (v / k + 1) * k.  Bounded (limit polls): a wait that gives up goes on with
// wrong results rather than hanging the launch, and says so: the batch's
// sticky flag sync[2B] (BatchHandle.vanilla_sync_ok), and when the caller
// passed dr_pass.fault, fault[0] = 1 for this launch (the reduce then
// withholds the update and reports a NaN loss) and fault[1] += 1 (read by the
// host once per epoch, FusedTrainStep.check_faults).
__device__ __forceinline__ void sib_handoff(uint32_t* ctr, uint32_t* flag, uint32_t* fault, int limit, int k) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t v = __hip_atomic_fetch_add((gu32*)ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t target = (v / (uint32_t)k + 1u) * (uint32_t)k;
    for (int spin = 0; ld_sc1_u32(ctr) < target; ++spin) {
      if (spin >= limit) {
        __hip_atomic_store((gu32*)flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (fault) {
          __hip_atomic_store((gu32*)fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_add((gu32*)(fault + 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
}

// After a workgroup's last hand-off wait: the last sibling out resets the
// graph's counters for the next launch (every sibling has stopped polling).
__device__ __forceinline__ void sib_exit(uint32_t* ctr, int k) {
  if (threadIdx.x == 0) {
    const uint32_t v = __hip_atomic_fetch_add((gu32*)(ctr + 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v == (uint32_t)k - 1u) {
      __hip_atomic_store((gu32*)ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((gu32*)(ctr + 1), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Rows [r0, r1) of an N x 34 LDS slot -> global rows (stride 32), 8-byte sc1 stores.
__device__ __forceinline__ void publish_rows(const float* slot, float* g, int r0, int r1) {
  for (int q = r0 * 16 + (int)threadIdx.x; q < r1 * 16; q += NT) {
    const int i = q >> 4, c = (q & 15) * 2;
    st_sc1_f2(g + i * 32 + c, slot[i * LS + c], slot[i * LS + c + 1]);
  }
}
// The other siblings' rows (all of [0, N) but [r0, r1)) of global rows -> LDS slot, 8-byte sc1 loads.
__device__ __forceinline__ void gather_rows(float* slot, const float* g, int N, int r0, int r1) {
  const int own = r1 - r0;
  for (int q = (int)threadIdx.x; q < (N - own) * 16; q += NT) {
    int i = q >> 4;
    i = i < r0 ? i : i + own;
    const int c = (q & 15) * 2;
    const uint64_t v = ld_sc1_u64(g + i * 32 + c);
    *reinterpret_cast<float2*>(slot + i * LS + c) = make_float2(__uint_as_float((uint32_t)v), __uint_as_float((uint32_t)(v >> 32)));
  }
}
// ReLU words of the transposed slots [q0, q1) -> LDS: slot q is CSR edge teid[q]
// (stored sc1, by any sibling); four slots per thread in flight.
__device__ __forceinline__ void gather_words(uint32_t* dst, const uint32_t* g, const int* teid, int q0, int q1) {
  for (int q = q0 + (int)threadIdx.x; q < q1; q += 4 * NT) {
    int te[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) te[u] = teid[min(q + u * NT, q1 - 1)];
    uint32_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld_sc1_u32(g + te[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (q + u * NT < q1) dst[q + u * NT] = v[u];
  }
}

// Edge-balanced row bound of sibling r: the first row i with rp[i] + RW i >= r (E + RW N) / k
// (a row costs about one 16-edge chunk on top of its edges: RW 2 / 8 / 16
// measured 95.2 / 94.0 / 93.5 us per step at B=64, slowest workgroup 200 / 189 / 197 K cycles).
constexpr int RW = 16;
__device__ __forceinline__ int row_bound(const int* rp, int N, int r, int k) {
  if (r <= 0) return 0;
  if (r >= k) return N;
  const int64_t t = ((int64_t)(rp[N] + RW * N) * r + k - 1) / k;
  int lo = 0, hi = N;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((int64_t)rp[mid] + RW * mid >= t) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ const float vg_zero_word = 0.f;

// Branch-free global loads: p (nullptr = the value 0) is read unconditionally,
// so a batch of them is issued back to back and waited for once.
__device__ __forceinline__ float ld0(const float* p) {
  // a global (not flat) load: a flat one would also hold every later LDS wait
  return *(const __attribute__((address_space(1))) float*)(p ? p : &vg_zero_word);
}

// Weights in MFMA-fragment order, packed once per launch by vanilla_pack_kernel
// (the parameters change every step): every fragment load of a GEMM phase is
// then one coalesced 256-byte wave read instead of 64 lanes touching 16 rows.
// GEMM operand o (NK_o 32-deep k blocks): element ((ct * 8 NK_o + s) * 64 + lane)
// = W_o(k = 4s + lane / 16, n = 16 ct + lane % 16), zero outside W_o.
enum { OP_B1, OP_X1, OP_B2, OP_X2, OP_DS2, OP_DX1, OP_DS1, N_OPS };
__host__ __device__ constexpr int op_nk(int o) { return (o == OP_X1 || o == OP_X2) ? 2 : (o == OP_DX1 ? 3 : 1); }
__host__ __device__ constexpr int op_base(int o) { return o == 0 ? 0 : op_base(o - 1) + 1024 * op_nk(o - 1); }
// row-pass weights of layer l at ROW_BASE + l * ROWPACK: float2 per lane (channels
// 2cp, 2cp+1 of the lane's pair cp = lane % 16): Wa[k = 16 (lane / 16 % 2) + m] for
// m < 16, then Wc[f] for f < 4, then be
constexpr int ROW_BASE = op_base(N_OPS), ROWPACK = 2 * 64 * (16 + 4 + 1), WPACK_FLOATS = ROW_BASE + 2 * ROWPACK;

struct PackArgs {
  dr_vanilla_weights w;
  float* out;
  uint32_t* fault;  // dr_pass.fault: [0] cleared for the graph launch that follows
  int32_t F, Fe;
};

__device__ float pack_value(const PackArgs& a, int e) {
  const int F = a.F, Fe = a.Fe, KE = 2 * F + Fe, KN = F + 32;
  if (e >= ROW_BASE) {  // row-pass block
    const int l = (e - ROW_BASE) / ROWPACK, q = (e - ROW_BASE) % ROWPACK;
    const float* we = l ? a.w.we2 : a.w.we1;
    const float* be = l ? a.w.be2 : a.w.be1;
    const int part = q >> 1, hi = q & 1;  // float2 index, which channel of the pair
    const int lane = part & 63, blk = part >> 6, c = 2 * (lane & 15) + hi;
    if (blk < 16) {
      const int k = 16 * ((lane >> 4) & 1) + blk;
      return k < F ? we[c * KE + k] : 0.f;
    }
    if (blk < 20) return blk - 16 < Fe ? we[c * KE + 2 * F + blk - 16] : 0.f;
    return be[c];
  }
  int o = 0;
  while (o + 1 < N_OPS && e >= op_base(o + 1)) ++o;
  const int q = e - op_base(o), nk = op_nk(o), lane = q & 63, s = (q >> 6) % (8 * nk), ct = (q >> 6) / (8 * nk);
  const int k = 4 * s + (lane >> 4), n = 16 * ct + (lane & 15);
  switch (o) {
    case OP_B1: return k < F ? a.w.we1[n * KE + F + k] : 0.f;
    case OP_B2: return k < F ? a.w.we2[n * KE + F + k] : 0.f;
    case OP_X1:
    case OP_X2: {
      const float* wn = o == OP_X1 ? a.w.wn1 : a.w.wn2;
      return n < F ? (k < F ? wn[n * KN + k] : (k < 32 ? 0.f : wn[n * KN + F + k - 32])) : 0.f;
    }
    case OP_DS1:
    case OP_DS2: {  // W(k, c) = Wn[k][F + c], k < F (the rows of dS = DU Wn[:, F:])
      const float* wn = o == OP_DS1 ? a.w.wn1 : a.w.wn2;
      return k < F ? wn[k * KN + F + n] : 0.f;
    }
    default:  // OP_DX1: [Wn2[:, :F]; Wa2; Wb2]
      return n < F ? (k < 32 ? (k < F ? a.w.wn2[k * KN + n] : 0.f)
                             : (k < 64 ? a.w.we2[(k - 32) * KE + n] : a.w.we2[(k - 64) * KE + F + n]))
                   : 0.f;
  }
}

__global__ void __launch_bounds__(256) vanilla_pack_kernel(PackArgs a) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e < WPACK_FLOATS) a.out[e] = pack_value(a, e);
  if (e == 0 && a.fault) a.fault[0] = 0u;  // stream order: cleared before the graph launch starts
}

// C[M, 32] = A[M, K] W[K, 32], K = 32 * NK, on v_mfma_f32_16x16x4_f32.  Wave w
// owns column tile w & 1 and row tiles w >> 1, (w >> 1) + 8, ...; its B
// fragment (packed operand frag, coalesced) and the column's bias (Bp(n),
// nullptr = 0) are loaded into registers once, before the first tile; waves
// without a row tile load nothing.  A returns the LDS operand; epi(m, n, v, bias).
template <int NK, class AF, class BF, class EF>
__device__ __forceinline__ void mm_w(int M, AF A, const float* frag, BF Bp, EF epi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, kq = lane >> 4;
  const int n = (wave & 1) * 16 + li;
  if ((wave >> 1) * 16 >= M) return;
  const __attribute__((address_space(1))) float* fr =
      (const __attribute__((address_space(1))) float*)(frag + (wave & 1) * 8 * NK * 64 + lane);
  float bw[8 * NK];
#pragma unroll
  for (int s = 0; s < 8 * NK; ++s) bw[s] = fr[s * 64];
  const float bias = ld0(Bp(n));
  const int nrt = (M + 15) >> 4;
  for (int rt = wave >> 1; rt < nrt; rt += NW / 2) {
    const int m0 = rt << 4, am = min(m0 + li, M - 1);
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 8 * NK; s += 2) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(A(am, 4 * s + kq), bw[s], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(A(am, 4 * s + 4 + kq), bw[s + 1], acc1, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + kq * 4 + r;
      if (row < M) epi(row, n, acc0[r] + acc1[r], bias);
    }
  }
}

// C[M, Nn] = sum_k A(m, k) B(k, n), both operands in LDS (weight gradients,
// K = the graph's node count), 16x16 tiles over the waves (job j on wave
// (start + j) % NW, so two GEMMs of a phase can share the waves).  A / B are
// called with k < K only.
template <class AF, class BF, class EF>
__device__ __forceinline__ void mm16(int M, int Nn, int K, int start, AF A, BF Bf, EF epi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, kq = lane >> 4;
  const int ntl = (Nn + 15) >> 4, jobs = ((M + 15) >> 4) * ntl;
  for (int job = (wave - start % NW + NW) % NW; job < jobs; job += NW) {
    const int m0 = (job / ntl) << 4, n0 = (job % ntl) << 4;
    const int am = min(m0 + li, M - 1), bn = min(n0 + li, Nn - 1);
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    // four 8-deep k-steps per iteration, their operand reads issued together;
    // past K the reads take row K-1 (so a caller's own k < K guard folds away
    // and every read is an unconditional LDS load) and the operands are zeroed
    for (int k = 0; k < K; k += 32) {
      float av[8], bv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int kk = k + 4 * u + kq, kc = min(kk, K - 1);
        av[u] = A(am, kc);
        bv[u] = Bf(kc, bn);
        av[u] = kk < K ? av[u] : 0.f;
        bv[u] = kk < K ? bv[u] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u + 1], bv[u + 1], acc1, 0, 0, 0);
      }
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

__device__ __forceinline__ float2 f2fma(float a, float2 w, float2 c) { return make_float2(fmaf(a, w.x, c.x), fmaf(a, w.y, c.y)); }
__device__ __forceinline__ float2 f2add(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 f2shfl_xor(float2 v, int m) {
  return make_float2(__shfl_xor(v.x, m, 64), __shfl_xor(v.y, m, 64));
}
// sum over the 4 edge slots of a wave (lanes l, l^16, l^32, l^48)
__device__ __forceinline__ float2 f2slot_sum(float2 v) {
  v = f2add(v, f2shfl_xor(v, 16));
  return f2add(v, f2shfl_xor(v, 32));
}

// Edge ReLU words: bit b (b < 16) = channel 2b, bit 16 + b = channel 2b + 1
// (the two ballots of the packed row pass side by side).

// Forward CSR row pass of one layer, two rows per wave.  Lane = (channel pair
// cp = lane & 15: channels 2cp, 2cp+1 as a float2; edge slot es = (lane >> 4) & 1;
// row hr = lane >> 5 of the wave's pair): each 8-edge chunk of a row is 4 steps
// of 2 edges, the pair's shorter row idling (masked) past its end.
//   S_i = sum_{e in row i} relu(A_i + B_j + Wc ea_e),   A_i = Wa x_i + be
// (A_i: each slot sums 16 of the K = 32 (padded) inputs, then the slots combine).
// Also each edge's ReLU word, CSR order (global bt): lane j < 8 of a row's
// first edge slot keeps the word of the chunk's edge j and the eight go out as
// one 32-byte store.  Edge records: {byte offset of B row col, ea0, ea1, ea2}.
__device__ __forceinline__ float2 f2half_sum(float2 v) { return f2add(v, f2shfl_xor(v, 16)); }

template <int FE>
__device__ __forceinline__ void row_fwd(const int* rp, const uint4* rec, const float* ext, const float* X,
                                        const float* Bs, float* S, float* S1g, uint32_t* btg, const float* rpack,
                                        int N, int N_E, int r0, int r1) {
  constexpr int FA = FE > 0 ? FE : 1;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, cp = lane & 15, sl = lane >> 4, c0 = 2 * cp;
  const int es = sl & 1, hr = sl >> 1;
  // this layer's Wa / Wc / be pairs, packed per lane (vanilla_pack_kernel): coalesced float2 loads
  typedef float fl2 __attribute__((ext_vector_type(2)));
  const __attribute__((address_space(1))) fl2* rp2 = (const __attribute__((address_space(1))) fl2*)(rpack) + lane;
  float2 wa[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const fl2 v = rp2[m * 64];
    wa[m] = make_float2(v.x, v.y);
  }
  float2 wc[FA];
#pragma unroll
  for (int f = 0; f < FE; ++f) {
    const fl2 v = rp2[(16 + f) * 64];
    wc[f] = make_float2(v.x, v.y);
  }
  const fl2 bev = rp2[20 * 64];
  const float2 be2 = make_float2(bev.x, bev.y);
  const int jme = cp & 7, sme = 16 * (2 * hr + (jme & 1));  // the word this lane keeps: edge jme of the chunk
  for (int i0 = r0 + 2 * wave; i0 < r1; i0 += 2 * NW) {
    const int i = i0 + hr;
    const bool rowok = i < r1;
    const int ii = rowok ? i : i0;
    const int eb = rp[ii], len = rowok ? rp[ii + 1] - eb : 0;
    const int lmax = max(len, __shfl_xor(len, 32, 64));
    float2 a = make_float2(0.f, 0.f);
    {
      const float2* xr = reinterpret_cast<const float2*>(X + ii * LS + 16 * es);
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const float2 v = xr[m];
        a = f2fma(v.x, wa[2 * m], a);
        a = f2fma(v.y, wa[2 * m + 1], a);
      }
    }
    a = f2add(f2half_sum(a), be2);
    float2 acc = make_float2(0.f, 0.f);
    for (int off = 0; off < lmax; off += 8) {
      const int nch = len - off;
      // past this row's end (the pair's other row is longer): the zero padding records
      const int base = nch > 0 ? eb + off : N_E;
      uint4 r[4];
      float e3[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        r[u] = rec[base + es + 2 * u];  // past the row end: the next rows' / padding records (masked)
        e3[u] = FE > 3 ? ext[base + es + 2 * u] : 0.f;
      }
      float2 bj[4];
      uint32_t mine = 0u;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        bj[u] = *reinterpret_cast<const float2*>(reinterpret_cast<const char*>(Bs) + (r[u].x & 0xffffu) + 8 * cp);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool ok = es + 2 * u < nch;
        const float ev[4] = {__uint_as_float(r[u].y), __uint_as_float(r[u].z), __uint_as_float(r[u].w), e3[u]};
        float2 pre = f2add(a, bj[u]);
#pragma unroll
        for (int f = 0; f < FE; ++f) pre = f2fma(ev[f], wc[f], pre);
        pre.x = ok ? pre.x : -1.f;  // slots past the row end: inactive, contribute 0
        pre.y = ok ? pre.y : -1.f;
        const bool al = !(pre.x <= 0.f), ah = !(pre.y <= 0.f);  // relu keeps NaN (active)
        acc.x += al ? pre.x : 0.f;
        acc.y += ah ? pre.y : 0.f;
        const uint64_t blo = __ballot(al), bhi = __ballot(ah);
        if ((jme >> 1) == u) mine = (uint32_t)((blo >> sme) & 0xffffu) | ((uint32_t)((bhi >> sme) & 0xffffu) << 16);
      }
      // the chunk's words (write-through: a sibling workgroup may read them)
      if (es == 0 && cp < 8 && cp < nch) st_sc1_u32(btg + eb + off + cp, mine);
    }
    acc = f2half_sum(acc);
    if (es == 0 && rowok) {
      *reinterpret_cast<float2*>(S + i * LS + c0) = acc;
      if (S1g) *reinterpret_cast<float2*>(S1g + i * 32 + c0) = acc;
    }
  }
}

// D_i = dS_i * cnt_i (0 where no edge of row i is active) into D; per-wave
// partials of dbe = sum_i D_i and dWc[c][f] = sum_i dS_i[c] eap_i[c][f] into red
// [NW][32 * (1 + FE)].  cnt_i / eap_i come from one pass over row i's ReLU
// words (global, CSR order) and edge attributes (the store).  The own rows'
// edges are contiguous, so they are copied to LDS behind red in segments of
// whole rows that fit (one bulk copy, all loads in flight: one memory round
// trip per segment, a single segment at k = 4), then each row is read from
// there (lane layout of row_fwd).  A row longer than the whole buffer reads
// global memory directly.
template <int FE>
__device__ __forceinline__ void d_pass(const int* rp, const uint32_t* btg, const float* ea, const float* dS, float* D,
                                       float* red, int N, int r0, int r1, int64_t* stp = nullptr) {
  constexpr int FA = FE > 0 ? FE : 1, RW = 32 * (1 + FE);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, cp = lane & 15, c0 = 2 * cp;
  const int es = (lane >> 4) & 1, hr = lane >> 5;
  constexpr int RS = FE <= 3 ? 4 : 8;  // one record per edge: {word, ea[0..FE)} (one 16-byte read for FE <= 3)
  float* buf = red + NW * RW;
  const int cap = (vslot(N, FE) - NW * RW) / RS;  // edges per segment
  float2 pbe = make_float2(0.f, 0.f), pwc[FA];
#pragma unroll
  for (int f = 0; f < FA; ++f) pwc[f] = make_float2(0.f, 0.f);
  for (int s0 = r0; s0 < r1;) {
    // the segment [s0, s1): whole rows whose edges fit the buffer (uniform)
    int lo = s0 + 1, hi = r1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (rp[mid] - rp[s0] <= cap) lo = mid;
      else hi = mid - 1;
    }
    const int s1 = lo, E0 = rp[s0], ne = rp[s1] - E0;
    const bool inbuf = ne <= cap;
    if (inbuf) {  // words, then attributes (AoS in HBM, as the records want them)
      const int tot = ne * (1 + FE);
      for (int q0 = tid; q0 < tot; q0 += 4 * NT) {
        float v[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int q = min(q0 + t * NT, tot - 1);
          v[t] = q < ne ? __uint_as_float(btg[E0 + q]) : (FE > 0 ? ea[(int64_t)E0 * FE + q - ne] : 0.f);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int q = q0 + t * NT;
          if (q < tot) buf[q < ne ? q * RS : ((q - ne) / FA) * RS + 1 + (q - ne) % FA] = v[t];
        }
      }
    }
    __syncthreads();
#ifdef DR_STAMPS
    if (stp && tid == 0 && s0 == r0) stp[23] = __builtin_amdgcn_s_memtime();
#endif
    // (two instantiations, so LDS and global reads stay ds_ / global_ loads)
    auto rows = [&](auto rec) {
      for (int i0 = s0 + 2 * wave; i0 < s1; i0 += 2 * NW) {
        const int i = i0 + hr;
        const bool rowok = i < s1;
        const int ii = rowok ? i : i0;
        const int eb = rp[ii], len = rowok ? rp[ii + 1] - eb : 0;
        const int lmax = max(len, __shfl_xor(len, 32, 64));
        float2 cnt = make_float2(0.f, 0.f), eap[FA];
#pragma unroll
        for (int f = 0; f < FA; ++f) eap[f] = make_float2(0.f, 0.f);
        for (int off = 0; off < lmax; off += 8) {
          const int nch = len - off;
          uint32_t wd[4];
          float ev[4][FA];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const bool ok = es + 2 * u < nch;
            const int e = ok ? eb + off + es + 2 * u : E0;  // masked: a valid edge, word forced to 0
            rec(e, wd[u], ev[u]);
            wd[u] = ok ? wd[u] : 0u;
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float bl = ((wd[u] >> cp) & 1u) ? 1.f : 0.f, bh = ((wd[u] >> (16 + cp)) & 1u) ? 1.f : 0.f;
            cnt = f2add(cnt, make_float2(bl, bh));
#pragma unroll
            for (int f = 0; f < FE; ++f) eap[f] = make_float2(fmaf(bl, ev[u][f], eap[f].x), fmaf(bh, ev[u][f], eap[f].y));
          }
        }
        cnt = f2half_sum(cnt);
    #pragma unroll
        for (int f = 0; f < FE; ++f) eap[f] = f2half_sum(eap[f]);
        if (es == 0 && rowok) {
          const float2 ds = *reinterpret_cast<const float2*>(dS + i * LS + c0);
          const float2 d = make_float2(cnt.x != 0.f ? ds.x * cnt.x : 0.f, cnt.y != 0.f ? ds.y * cnt.y : 0.f);
          *reinterpret_cast<float2*>(D + i * LS + c0) = d;
          pbe = f2add(pbe, d);
    #pragma unroll
          for (int f = 0; f < FE; ++f)
            pwc[f] = f2add(pwc[f], make_float2(cnt.x != 0.f ? ds.x * eap[f].x : 0.f, cnt.y != 0.f ? ds.y * eap[f].y : 0.f));
        }
      }
    };
    typedef __attribute__((address_space(1))) const uint32_t gcu32;
    typedef __attribute__((address_space(1))) const float gcf;
    if (inbuf)
      rows([&](int e, uint32_t& w, float* v) {
        const float4 r = *reinterpret_cast<const float4*>(buf + (e - E0) * RS);
        w = __float_as_uint(r.x);
        if (FE > 0) v[0] = r.y;
        if (FE > 1) v[1] = r.z;
        if (FE > 2) v[2] = r.w;
        if (FE > 3) v[3] = buf[(e - E0) * RS + 4];
      });
    else
      rows([&](int e, uint32_t& w, float* v) {
        w = ((gcu32*)btg)[e];
#pragma unroll
        for (int f = 0; f < FE; ++f) v[f] = ((gcf*)ea)[(int64_t)e * FE + f];
      });
    __syncthreads();  // (the next segment overwrites the buffer)
#ifdef DR_STAMPS
    if (stp && tid == 0 && s0 == r0) stp[24] = __builtin_amdgcn_s_memtime();
#endif
    s0 = s1;
  }
  // the wave's two rows (lanes cp and cp + 32, edge slot 0)
  pbe = f2add(pbe, f2shfl_xor(pbe, 32));
#pragma unroll
  for (int f = 0; f < FE; ++f) pwc[f] = f2add(pwc[f], f2shfl_xor(pwc[f], 32));
  if (lane < 16) {
    red[wave * RW + c0] = pbe.x;
    red[wave * RW + c0 + 1] = pbe.y;
#pragma unroll
    for (int f = 0; f < FE; ++f) {
      red[wave * RW + 32 + c0 * FE + f] = pwc[f].x;
      red[wave * RW + 32 + (c0 + 1) * FE + f] = pwc[f].y;
    }
  }
}

// dbe and dWc of one layer from the D pass partials (fixed wave order).
template <int FE>
__device__ __forceinline__ void d_pass_sum(const float* red, float* gw, int KE, int F) {
  constexpr int RW = 32 * (1 + FE);
  const int tid = threadIdx.x;
  if (tid < RW) {
    float t = 0.f;
    for (int wv = 0; wv < NW; ++wv) t += red[wv * RW + tid];
    if (tid < 32) gw[32 * KE + tid] = t;
    else {
      constexpr int FD = FE > 0 ? FE : 1;  // (FE == 0: this branch never runs)
      const int c = (tid - 32) / FD, f = (tid - 32) % FD;
      gw[c * KE + 2 * F + f] = t;
    }
  }
}

// Transposed pass: D'_j = sum over in-edges (i -> j) active in channel c of dS_i
// (lane layout of row_fwd: channel pair x edge slot x row of the wave's pair).
__device__ __forceinline__ void row_t(const int* trp, const uint16_t* tcol, const uint32_t* bt, const float* dS,
                                      float* Dp, int r0, int r1) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, cp = lane & 15, c0 = 2 * cp;
  const int es = (lane >> 4) & 1, hr = lane >> 5;
  for (int j0 = r0 + 2 * wave; j0 < r1; j0 += 2 * NW) {
    const int j = j0 + hr;
    const bool rowok = j < r1;
    const int jj = rowok ? j : j0;
    const int qb = trp[jj], len = rowok ? trp[jj + 1] - qb : 0;
    const int lmax = max(len, __shfl_xor(len, 32, 64));
    float2 acc = make_float2(0.f, 0.f);
    for (int off = 0; off < lmax; off += 8) {
      const int nch = len - off;
      uint32_t wd[4];
      float2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool ok = es + 2 * u < nch;
        const int q = qb + off + es + 2 * u;
        wd[u] = ok ? bt[q] : 0u;
        // masked slots (past the row end, or an empty row) read node 0's row
        v[u] = *reinterpret_cast<const float2*>(dS + (ok ? (int)tcol[q] : 0) * LS + c0);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc.x += ((wd[u] >> cp) & 1u) ? v[u].x : 0.f;
        acc.y += ((wd[u] >> (16 + cp)) & 1u) ? v[u].y : 0.f;
      }
    }
    acc = f2half_sum(acc);
    if (es == 0 && rowok) *reinterpret_cast<float2*>(Dp + j * LS + c0) = acc;
  }
}

#ifdef DR_STAMPS
#define VSTAMP(i)                                                                                           \
  do {                                                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                                      \
    if (tid == 0 && a.p.stamps) a.p.stamps[((int64_t)b * a.k + rk) * 32 + (i)] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                                      \
  } while (0)
#else
#define VSTAMP(i) \
  do {            \
  } while (0)
#endif

template <int FE>
__global__ void __launch_bounds__(NT) vanilla_graph_kernel(VGArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // block -> (graph slot b, sibling rk): siblings 8 blocks apart, 8 graphs per 8k blocks
  const int k = a.k;
  const int bx = blockIdx.x, hi = bx >> 3;
  const int rk = hi % k, b = (hi / k) * 8 + (bx & 7);
  if (b >= a.B) return;
  const dr_graph_store& s = a.s;
  const dr_vanilla_weights& w = a.w;
  const dr_pass& p = a.p;
  const dr_graph_desc d = a.descs[b];
  const int g = d.gid, N = d.n_nodes, E = d.n_edges;
  const int F = s.n_feat, Fe = FE, FeS = Fe > 0 ? Fe : 1, XS = s.x_stride;
  const int KE = 2 * F + Fe, KN = F + 32, OUT = p.out_dim;
  const VCarve cv = vcarve(N, E, Fe);
  int* srp = reinterpret_cast<int*>(lds + cv.rp);
  uint32_t* xb = reinterpret_cast<uint32_t*>(lds + cv.xb);
  float* P = lds + cv.P;
  float* Q = lds + cv.Q;
  float* R = lds + cv.R;
  uint4* rec = reinterpret_cast<uint4*>(lds + cv.U);
  float* ext = lds + cv.ext;
  float* T = lds + cv.T;
  uint32_t* bt = reinterpret_cast<uint32_t*>(lds + cv.bt);
  int* strp = reinterpret_cast<int*>(lds + cv.trp);
  uint16_t* stcol = reinterpret_cast<uint16_t*>(lds + cv.tcol);
  float* sg = lds + cv.head;
  float* sh = sg + 32;
  float* sdh = sh + 128;
  float* sdout = sdh + 128;
  float* sdm = sdout + 16;

  const float* X0 = s.x + d.node0 * (int64_t)XS;
  const float* ea = s.ea + d.col0 * (int64_t)FeS;
  float* scr = a.scr + a.scr_off[b];
  const int n32 = r4(32 * N);
  float* S1g = scr;
  uint32_t* bt1g = reinterpret_cast<uint32_t*>(S1g + n32);
  uint32_t* bt2g = bt1g + r4(E + 1);
  float* XA = reinterpret_cast<float*>(bt2g + r4(E + 1));  // B2, then dS1 rows (split)
  float* XB = XA + n32;                                    // dS2 rows (split)
  float* csum = XB + n32;                                  // [k][32] column sums of X2 (split)
  const int* teid = s.t_eid + d.col0;                      // transposed slot -> CSR edge
  uint32_t* ctr = a.sync + 2 * b;
  uint32_t* tflag = a.sync + 2 * a.B;
  const bool split = k > 1;
  const int spin_limit = a.p.spin_limit > 0 ? a.p.spin_limit : (1 << 22);
  const int LG = 32 * KE + 32 + F * KN + F;  // one layer's gradient entries in the slab
  const int row = p.slot ? p.slot[b] : b;  // the graph's rows of the batch (dr_pass.slot)
  float* slab = p.slab ? p.slab + ((int64_t)row * k + rk) * DR_VANILLA_SLAB_STRIDE(F, Fe) : nullptr;
  const bool bwd = (p.flags & DR_PASS_BACKWARD) != 0;
  const bool lead = rk == 0;  // writes the graph's outputs, loss and head vectors

  VSTAMP(0);
  // ---------------- stage: CSR rows, edge records, X0 into LDS ------------
  dma_words<NT>(srp, s.rowptr + d.node0 + g, N + 1);
  {
    const uint16_t* gcol = s.col + d.col0;
    uint32_t* r32 = reinterpret_cast<uint32_t*>(rec);
    float* rf = reinterpret_cast<float*>(rec);
    for (int e0 = tid; e0 < E; e0 += 4 * NT) {  // 4 edges per thread and step, loads first
      uint32_t cl[4];
      float ev[4][MAXFE];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + u * NT;
        const int ec = e < E ? e : 0;  // E >= 1 here (the loop runs only then)
        cl[u] = gcol[ec];
#pragma unroll
        for (int f = 0; f < MAXFE; ++f) ev[u][f] = f < Fe ? ea[(int64_t)ec * FeS + f] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + u * NT;
        if (e < E) {
          r32[4 * e] = cl[u] * (LS * 4);  // byte offset of row col in a slot
#pragma unroll
          for (int f = 0; f < 3; ++f) rf[4 * e + 1 + f] = ev[u][f];
          if (Fe > 3) ext[e] = ev[u][3];
        }
      }
    }
    for (int q = tid; q < 64; q += NT) reinterpret_cast<uint32_t*>(rec)[4 * E + q] = 0u;  // padding records
    if (Fe > 3 && tid < 16) ext[E + tid] = 0.f;
  }
  for (int q = tid; q < N * 8; q += NT) {  // X0 -> P (stride LS), zero columns >= XS
    const int i = q >> 3, c4 = (q & 7) * 4;
    const float4 v = c4 < XS ? *reinterpret_cast<const float4*>(X0 + (int64_t)i * XS + c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float2*>(P + i * LS + c4) = make_float2(v.x, v.y);
    *reinterpret_cast<float2*>(P + i * LS + c4 + 2) = make_float2(v.z, v.w);
  }
  const float y_g = s.y[g];
  if (p.step_counter && b == 0 && lead && tid == 0) p.step_counter[1] = p.step_counter[0];
  wait_vm();
  __syncthreads();
  // this workgroup's rows (the transposed passes take the same range of target rows)
  const int r0 = row_bound(srp, N, rk, k), r1 = row_bound(srp, N, rk + 1, k), nown = r1 - r0;

  VSTAMP(1);
  // ---------------- layer 1: B1 = X0 Wb1^T -> Q (every row: the row pass gathers any) --
  mm_w<1>(N, [&](int i, int k) { return P[i * LS + k]; },
          a.wpack + op_base(OP_B1), [&](int) -> const float* { return nullptr; },
          [&](int i, int n, float v, float) { Q[i * LS + n] = v; });
  __syncthreads();
  VSTAMP(2);
  row_fwd<FE>(srp, rec, ext, P, Q, R, S1g, bt1g, a.wpack + ROW_BASE, N, E, r0, r1);
  __syncthreads();
  VSTAMP(3);
  // X1 = relu([X0 | S1] Wn1^T + bn1) -> Q (pad columns 0), own rows
  mm_w<2>(nown, [&](int i, int k) { return k < 32 ? P[(r0 + i) * LS + k] : R[(r0 + i) * LS + k - 32]; },
          a.wpack + op_base(OP_X1), [&](int n) -> const float* { return n < F ? w.bn1 + n : nullptr; },
          [&](int i, int n, float v, float bias) { Q[(r0 + i) * LS + n] = n < F ? relu_keepnan(v + bias) : 0.f; });
  __syncthreads();
  VSTAMP(4);
  // ---------------- layer 2: B2 = X1 Wb2^T -> P, own rows ---------------------
  mm_w<1>(nown, [&](int i, int k) { return Q[(r0 + i) * LS + k]; },
          a.wpack + op_base(OP_B2), [&](int) -> const float* { return nullptr; },
          [&](int i, int n, float v, float) { P[(r0 + i) * LS + n] = v; });
  __syncthreads();
  if (split) {  // hand-off 1: every sibling's B2 rows (and the layer-1 ReLU words)
    publish_rows(P, XA, r0, r1);
    VSTAMP(19);
    sib_handoff(ctr, tflag, a.p.fault, spin_limit, k);
    gather_rows(P, XA, N, r0, r1);
    __syncthreads();
  }
  VSTAMP(5);
  row_fwd<FE>(srp, rec, ext, Q, P, R, nullptr, bt2g, a.wpack + ROW_BASE + ROWPACK, N, E, r0, r1);
  wait_vm();  // the ReLU words of both layers stored before anyone reads them back
  __syncthreads();
  VSTAMP(6);
  // the records are dead: the backward's transposed CSR and layer-2 ReLU words
  // land in U while the forward finishes
  if (bwd) {
    if (!split) gather_words(bt, bt2g, teid, 0, E);  // (split: after hand-off 2)
    dma_words<NT>(strp, s.t_rowptr + d.node0 + g, N + 1);
    dma_x4<NT>(stcol, s.t_col + d.col0, (E + 7) / 8);
  }
  // X2 = relu([X1 | S2] Wn2^T + bn2) -> P, own rows
  mm_w<2>(nown, [&](int i, int k) { return k < 32 ? Q[(r0 + i) * LS + k] : R[(r0 + i) * LS + k - 32]; },
          a.wpack + op_base(OP_X2), [&](int n) -> const float* { return n < F ? w.bn2 + n : nullptr; },
          [&](int i, int n, float v, float bias) { P[(r0 + i) * LS + n] = n < F ? relu_keepnan(v + bias) : 0.f; });
  __syncthreads();
  VSTAMP(7);
  // per-graph mean (scatter_mean, vanilla_gnn.py:62): 32 row slices per column
  // (partials in T), combined in order (split: then the siblings' sums, in
  // sibling order); relu'(X2) as one bit word per node
  {
    const int n = tid & 31, sl = tid >> 5;
    float acc = 0.f;
    const int i0 = r0 + ((nown * sl) >> 5), i1 = r0 + ((nown * (sl + 1)) >> 5);
    for (int i = i0; i < i1; ++i) acc += P[i * LS + n];
    T[sl * 32 + n] = acc;
    for (int i = r0 + wave * 2 + (lane >> 5); i < r1; i += 2 * NW) {
      const int c = lane & 31;
      const uint64_t m = __ballot(c < F && !(P[i * LS + c] <= 0.f));
      if (c == 0) xb[i] = (lane >> 5) ? (uint32_t)(m >> 32) : (uint32_t)m;
    }
  }
  __syncthreads();
  if (tid < 32) {
    float t = 0.f;
    for (int sl = 0; sl < 32; ++sl) t += T[sl * 32 + tid];
    if (split) st_sc1(csum + rk * 32 + tid, t);
    else sg[tid] = tid < F ? t / (float)N : 0.f;
  }
  if (split) {  // hand-off 2: the siblings' column sums (and the layer-2 ReLU words)
    VSTAMP(20);
    sib_handoff(ctr, tflag, a.p.fault, spin_limit, k);
    if (tid < 32) {
      float t = ld_sc1(csum + tid);
      for (int q = 1; q < k; ++q) t += ld_sc1(csum + q * 32 + tid);
      sg[tid] = tid < F ? t / (float)N : 0.f;
    }
    if (bwd) gather_words(bt, bt2g, teid, strp[r0], strp[r1]);  // (strp landed: waited at the hand-off)
    if (!bwd) sib_exit(ctr, k);
  }
  __syncthreads();
  VSTAMP(8);
  // ---------------- graph MLP, loss, head backward (vanilla_gnn.py:63-64, trainer.py:686-689)
  // (every sibling runs it on the same inputs; the lead writes the outputs)
  // fc1: 8 lanes per output (4 inputs each), reduced by shuffles
  {
    const int o = tid >> 3, part = tid & 7;
    float acc = 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int n = 4 * part + m;
      const float wv = w.g1w[o * F + (n < F ? n : 0)];
      if (n < F) acc = fmaf(sg[n], wv, acc);
    }
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    acc += __shfl_xor(acc, 4, 64);
    if (part == 0) sh[o] = relu_keepnan(acc + w.g1b[o]);
  }
  __syncthreads();
  for (int q = wave; q < OUT; q += NW) {
    float v = fmaf(sh[lane], w.g2w[q * 128 + lane], sh[lane + 64] * w.g2w[q * 128 + lane + 64]);
    v = dr_wave_sum(v);
    if (lane == 0) sdout[q] = v + w.g2b[q];
  }
  __syncthreads();
  if ((p.flags & DR_PASS_FORWARD) && lead && tid < OUT) p.out[(int64_t)row * OUT + tid] = sdout[tid];
  if (!bwd) return;
  if (tid == 0) {
    if (p.loss_kind == DR_LOSS_MSE) {
      const float dl = sdout[0] - y_g;
      if (p.loss_per_graph && lead) p.loss_per_graph[row] = dl * dl;
      sdout[0] = 2.f * dl * p.loss_scale;
    } else if (p.loss_kind == DR_LOSS_CE) {
      const int yi = (int)y_g;
      float mx = sdout[0];
      for (int q = 1; q < OUT; ++q) mx = fmaxf(mx, sdout[q]);
      float se = 0.f;
      for (int q = 0; q < OUT; ++q) se += expf(sdout[q] - mx);
      const float lse = mx + logf(se);
      const float wy = p.class_w ? p.class_w[yi] : 1.f;
      if (p.loss_per_graph && lead) p.loss_per_graph[row] = wy * (lse - sdout[yi]);
      for (int q = 0; q < OUT; ++q) sdout[q] = wy * (expf(sdout[q] - lse) - (q == yi ? 1.f : 0.f)) * p.loss_scale;
    } else {
      for (int q = 0; q < OUT; ++q) sdout[q] = p.dout[(int64_t)row * OUT + q];
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
    // dmean[n] = sum_o fc1.w[o][n] dh[o] / N: 32 partial sums of 4 outputs per
    // column (partials in T), combined in order
    const int n = tid & 31, part = tid >> 5;
    float acc = 0.f;
    float wv[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) wv[m] = w.g1w[(4 * part + m) * F + (n < F ? n : 0)];
#pragma unroll
    for (int m = 0; m < 4; ++m) acc = fmaf(wv[m], sdh[4 * part + m], acc);
    if (n >= F) acc = 0.f;
    T[part * 32 + n] = acc;
  }
  __syncthreads();
  {
    float* hg = p.head + (int64_t)row * DR_VANILLA_HEAD_STRIDE(F, OUT);
    const int XSH = r4(F), HD = XSH + 256 + r4(OUT);
    if (tid < 32) {
      float acc = 0.f;
      for (int part = 0; part < 32; ++part) acc += T[part * 32 + tid];
      const float dm = acc / (float)N;  // scatter_mean backward: grad / count
      sdm[tid] = tid < F ? dm : 0.f;
      if (tid < F && lead) hg[HD + tid] = dm;
    }
    if (lead) {
      if (tid < XSH) hg[tid] = tid < F ? sg[tid] : 0.f;
      if (tid < 128) {
        hg[XSH + tid] = sh[tid];
        hg[XSH + 128 + tid] = sdh[tid];
      }
      if (tid < OUT) hg[XSH + 256 + tid] = sdout[tid];
    }
  }
  __syncthreads();
  VSTAMP(9);

  // ---------------- layer 2 backward (own rows; weight gradients = this workgroup's partials)
  // DU2 = relu'(X2) * dmean (bit words).  dWn2 = DU2^T [X1 | S2], dbn2 = sum DU2
  // (a column of ones); dS2 = DU2 Wn2[:, F:] -> P.
  {
    float* gw = slab + LG;  // layer 2
    mm16(F, KN + 1, nown, 0, [&](int n, int i) { return (i < nown && ((xb[r0 + i] >> n) & 1u)) ? 1.f : 0.f; },
         [&](int i, int q) {
           return i < nown ? (q < F ? Q[(r0 + i) * LS + q] : (q < KN ? R[(r0 + i) * LS + q - F] : 1.f)) : 0.f;
         },
         [&](int n, int q, float v) {
           if (q < KN) gw[32 * KE + 32 + n * KN + q] = sdm[n] * v;
           else gw[32 * KE + 32 + F * KN + n] = sdm[n] * v;
         });
    mm_w<1>(nown, [&](int i, int n) { return ((xb[r0 + i] >> n) & 1u) ? sdm[n] : 0.f; },
            a.wpack + op_base(OP_DS2), [&](int) -> const float* { return nullptr; },
            [&](int i, int c, float v, float) { P[(r0 + i) * LS + c] = v; });
  }
  __syncthreads();
  if (split) {  // hand-off 3: every sibling's dS2 rows (the transposed pass gathers them by source)
    publish_rows(P, XB, r0, r1);
    VSTAMP(21);
    sib_handoff(ctr, tflag, a.p.fault, spin_limit, k);
    gather_rows(P, XB, N, r0, r1);
  }
  VSTAMP(10);
  // D2 = dS2 * cnt2 -> R (S2 is dead), dbe2 / dWc2 partials in T
  d_pass<FE>(srp, bt2g, ea, P, R, T, N, r0, r1,
#ifdef DR_STAMPS
             a.p.stamps ? a.p.stamps + ((int64_t)b * a.k + rk) * 32 : nullptr
#else
             nullptr
#endif
  );
  wait_vm();  // bt2 and the transposed CSR have landed in U
  __syncthreads();
  d_pass_sum<FE>(T, slab + LG, KE, F);
  __syncthreads();
  VSTAMP(11);
  row_t(strp, stcol, bt, P, T, r0, r1);  // D'2 -> T
  __syncthreads();
  VSTAMP(12);
  {
    float* gw = slab + LG;
    // dWa2 = D2^T X1,  dWb2 = D'2^T X1
    mm16(32, F, nown, 0, [&](int c, int i) { return i < nown ? R[(r0 + i) * LS + c] : 0.f; },
         [&](int i, int k) { return i < nown && k < F ? Q[(r0 + i) * LS + k] : 0.f; },
         [&](int c, int k, float v) { gw[c * KE + k] = v; });
    mm16(32, F, nown, 4, [&](int c, int i) { return i < nown ? T[(r0 + i) * LS + c] : 0.f; },
         [&](int i, int k) { return i < nown && k < F ? Q[(r0 + i) * LS + k] : 0.f; },
         [&](int c, int k, float v) { gw[c * KE + F + k] = v; });
    // dX1 = [DU2 | D2 | D'2] [Wn2[:, :F]; Wa2; Wb2], DU1 = relu'(X1) * dX1 -> P
    mm_w<3>(nown,
            [&](int i, int k) {
              const int ii = r0 + i;
              return k < 32 ? (((xb[ii] >> k) & 1u) ? sdm[k] : 0.f) : (k < 64 ? R[ii * LS + k - 32] : T[ii * LS + k - 64]);
            },
            a.wpack + op_base(OP_DX1), [&](int) -> const float* { return nullptr; },
            [&](int i, int n, float v, float) { P[(r0 + i) * LS + n] = n < F ? relu_bwd(Q[(r0 + i) * LS + n], v) : 0.f; });
  }
  __syncthreads();
  VSTAMP(13);
  // ---------------- layer 1 backward ---------------------------------------
  // X0 (HBM row stride XS) -> Q, S1 -> R (stride 32), layer-1 ReLU words -> U:
  // bulk DMA (own rows), landing while dS1 = DU1 Wn1[:, F:] -> T runs
  dma_x4<NT>(Q + r0 * XS, X0 + (int64_t)r0 * XS, nown * XS / 4);
  dma_x4<NT>(R + r0 * 32, S1g + r0 * 32, nown * 8);
  gather_words(bt, bt1g, teid, strp[r0], strp[r1]);
  mm_w<1>(nown, [&](int i, int n) { return P[(r0 + i) * LS + n]; },
          a.wpack + op_base(OP_DS1), [&](int) -> const float* { return nullptr; },
          [&](int i, int c, float v, float) { T[(r0 + i) * LS + c] = v; });
  wait_vm();
  __syncthreads();
  if (split) {  // hand-off 4: every sibling's dS1 rows
    publish_rows(T, XA, r0, r1);
    VSTAMP(22);
    sib_handoff(ctr, tflag, a.p.fault, spin_limit, k);
    sib_exit(ctr, k);
    gather_rows(T, XA, N, r0, r1);
  }
  VSTAMP(14);
  {
    float* gw = slab;  // layer 1
    // dWn1 = DU1^T [X0 | S1], dbn1 = sum DU1
    mm16(F, KN + 1, nown, 0, [&](int n, int i) { return i < nown ? P[(r0 + i) * LS + n] : 0.f; },
         [&](int i, int q) {
           const int ii = r0 + i;
           return i < nown ? (q < F ? Q[ii * XS + q] : (q < KN ? R[ii * 32 + q - F] : 1.f)) : 0.f;
         },
         [&](int n, int q, float v) {
           if (q < KN) gw[32 * KE + 32 + n * KN + q] = v;
           else gw[32 * KE + 32 + F * KN + n] = v;
         });
  }
  __syncthreads();
  VSTAMP(15);
  // D1 = dS1 * cnt1 -> R (S1 is dead), partials in P (DU1 is dead)
  d_pass<FE>(srp, bt1g, ea, T, R, P, N, r0, r1);
  __syncthreads();
  d_pass_sum<FE>(P, slab, KE, F);
  __syncthreads();
  VSTAMP(16);
  row_t(strp, stcol, bt, T, P, r0, r1);  // D'1 -> P
  __syncthreads();
  VSTAMP(17);
  {
    float* gw = slab;
    // dWa1 = D1^T X0,  dWb1 = D'1^T X0
    mm16(32, F, nown, 0, [&](int c, int i) { return i < nown ? R[(r0 + i) * LS + c] : 0.f; },
         [&](int i, int k) { return i < nown && k < F ? Q[(r0 + i) * XS + k] : 0.f; },
         [&](int c, int k, float v) { gw[c * KE + k] = v; });
    mm16(32, F, nown, 4, [&](int c, int i) { return i < nown ? P[(r0 + i) * LS + c] : 0.f; },
         [&](int i, int k) { return i < nown && k < F ? Q[(r0 + i) * XS + k] : 0.f; },
         [&](int c, int k, float v) { gw[c * KE + F + k] = v; });
  }
  VSTAMP(18);
}

}  // namespace

extern "C" int64_t dr_vanilla_fused_lds_bytes(int32_t n_nodes, int32_t n_edges, int32_t n_edge_feat) {
  return 4LL * vcarve(n_nodes, n_edges, n_edge_feat).total;
}

extern "C" int64_t dr_vanilla_fused_scratch_floats(int32_t n_nodes, int32_t n_edges, int32_t n_edge_feat) {
  return vscratch_floats(n_nodes, n_edges, n_edge_feat);
}

extern "C" int64_t dr_vanilla_wpack_floats(void) { return WPACK_FLOATS; }

extern "C" int dr_vanilla_wpack(const dr_vanilla_weights* w, int32_t n_feat, int32_t n_edge_feat, float* wpack,
                                void* stream) {
  if (!w || !wpack) return DR_E_ARG;
  if (n_feat < 1 || n_feat > 32 || n_edge_feat < 0 || n_edge_feat > MAXFE) return DR_E_UNSUPPORTED;
  PackArgs pa;
  pa.w = *w;
  pa.out = wpack;
  pa.fault = nullptr;
  pa.F = n_feat;
  pa.Fe = n_edge_feat;
  hipLaunchKernelGGL(vanilla_pack_kernel, dim3((WPACK_FLOATS + 255) / 256), dim3(256), 0, (hipStream_t)stream, pa);
  return (int)hipGetLastError();
}

extern "C" int dr_vanilla_fused_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                                     const dr_vanilla_weights* w, const dr_pass* pass, float* scratch,
                                     const int64_t* scratch_off, int32_t split, uint32_t* sync, float* wpack,
                                     int32_t lds_bytes, void* stream) {
  if (!store || !descs || !w || !pass || n_batch < 0 || !wpack) return DR_E_ARG;
  if (split < 1 || split > MAXK || (split > 1 && !sync)) return DR_E_ARG;
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
  const void* fn = nullptr;
  switch (store->n_edge_feat) {
    case 0: fn = reinterpret_cast<const void*>(&vanilla_graph_kernel<0>); break;
    case 1: fn = reinterpret_cast<const void*>(&vanilla_graph_kernel<1>); break;
    case 2: fn = reinterpret_cast<const void*>(&vanilla_graph_kernel<2>); break;
    case 3: fn = reinterpret_cast<const void*>(&vanilla_graph_kernel<3>); break;
    default: fn = reinterpret_cast<const void*>(&vanilla_graph_kernel<4>); break;
  }
  DR_CHECK(dr_allow_big_lds(fn));
  VGArgs a;
  a.s = *store;
  a.w = *w;
  a.p = *pass;
  a.descs = descs;
  a.scr = scratch;
  a.scr_off = scratch_off;
  a.sync = sync;
  a.wpack = wpack;
  a.B = n_batch;
  a.k = split;
  if (!(pass->flags & DR_PASS_WPACK_CURRENT)) {
    PackArgs pa;
    pa.w = *w;
    pa.out = wpack;
    pa.fault = pass->fault;
    pa.F = store->n_feat;
    pa.Fe = store->n_edge_feat;
    hipLaunchKernelGGL(vanilla_pack_kernel, dim3((WPACK_FLOATS + 255) / 256), dim3(256), 0, (hipStream_t)stream, pa);
  }
  // graph b's siblings are blocks 8 apart (see the kernel); grid padded to 8 graphs
  const dim3 grid((unsigned)(((n_batch + 7) / 8) * 8 * split));
  switch (store->n_edge_feat) {
    case 0: hipLaunchKernelGGL(vanilla_graph_kernel<0>, grid, dim3(NT), lds_bytes, (hipStream_t)stream, a); break;
    case 1: hipLaunchKernelGGL(vanilla_graph_kernel<1>, grid, dim3(NT), lds_bytes, (hipStream_t)stream, a); break;
    case 2: hipLaunchKernelGGL(vanilla_graph_kernel<2>, grid, dim3(NT), lds_bytes, (hipStream_t)stream, a); break;
    case 3: hipLaunchKernelGGL(vanilla_graph_kernel<3>, grid, dim3(NT), lds_bytes, (hipStream_t)stream, a); break;
    default: hipLaunchKernelGGL(vanilla_graph_kernel<4>, grid, dim3(NT), lds_bytes, (hipStream_t)stream, a); break;
  }
  return (int)hipGetLastError();
}

// ---- carve descriptions for the host-side carve tests (tests/test_lds_carves.py)
extern "C" int dr_debug_carve_vanilla_graph(const int32_t* q, char* buf, int32_t len) {
  const VCarve c = vcarve(q[0], q[1], q[2]);
  DrCarveDesc d{buf, len, 0};
  DR_DESC(d, c, rp);
  DR_DESC(d, c, xb);
  DR_DESC(d, c, head);
  DR_DESC(d, c, P);
  DR_DESC(d, c, Q);
  DR_DESC(d, c, R);
  DR_DESC(d, c, U);
  DR_DESC(d, c, ext);
  DR_DESC(d, c, T);
  DR_DESC(d, c, bt);
  DR_DESC(d, c, trp);
  DR_DESC(d, c, tcol);
  DR_DESC(d, c, total);
  return d.pos;
}

