// Host-side graph packer: per-graph arrays (what GraphDataset.load_one_graph
// returns, dataset.py:883-1052) -> the packed store layout every kernel reads
// (deeprank2_amd/store.py).  It is the collate (PyG Collater, trainer.py:541)
// plus the per-forward index work of the reference (get_preloaded_cluster,
// consecutive_cluster, pool_edge, max_pool_x relabelling —
// community_pooling.py:23-27,205-225; ginet.py:102-114) done once per graph.
//
// Two passes so the caller owns every buffer: dr_pack_sizes (per-graph K0,
// pooled-edge and K1 counts, validation), then dr_pack_fill.  Graphs are
// independent: both passes run on a pool of host threads.

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <thread>
#include <vector>

#include "../../include/deeprank2_amd.h"

namespace {

struct Local {
  std::vector<int32_t> dense0;  // node -> dense depth-0 id
  int32_t k0 = 0;
  std::vector<int64_t> pkey;    // unique pooled (row * k0 + col), sorted
  std::vector<int32_t> dense1;  // depth-0 cluster -> dense depth-1 id
  int32_t k1 = 0;
};

// dense relabel (sorted unique ids -> 0..k-1), like torch.unique(return_inverse)
bool dense_ids(const int64_t* ids, int64_t n, std::vector<int32_t>& out, int32_t& k) {
  std::vector<int64_t> u(ids, ids + n);
  std::sort(u.begin(), u.end());
  u.erase(std::unique(u.begin(), u.end()), u.end());
  if (!u.empty() && u.front() < 0) return false;
  out.resize(n);
  for (int64_t i = 0; i < n; ++i) out[i] = (int32_t)(std::lower_bound(u.begin(), u.end(), ids[i]) - u.begin());
  k = (int32_t)u.size();
  return true;
}

// stable counting sort of edges by key -> rowptr [n+1], perm [E] (slot -> edge)
void csr(const int64_t* key, int64_t E, int32_t n, int32_t* rowptr, std::vector<int32_t>& perm) {
  std::vector<int32_t> cnt(n + 1, 0);
  for (int64_t e = 0; e < E; ++e) ++cnt[key[e] + 1];
  for (int32_t i = 0; i < n; ++i) cnt[i + 1] += cnt[i];
  std::memcpy(rowptr, cnt.data(), sizeof(int32_t) * (n + 1));
  perm.resize(E);
  for (int64_t e = 0; e < E; ++e) perm[cnt[key[e]]++] = (int32_t)e;
}

struct Ctx {
  const dr_pack_input* in;
  std::vector<Local> loc;
  std::vector<int> err;   // per graph: 0 ok, else error code
  std::vector<int> sym;   // per graph: edge multiset symmetric
};

enum { E_NONE = 0, E_RANGE = 1, E_EMPTY = 2, E_C0LEN = 3, E_C1LEN = 4, E_NEG = 5, E_NOCL = 6 };

void analyse(Ctx& c, int g) {
  const dr_pack_input& in = *c.in;
  const int64_t n0 = in.node_off[g], n = in.node_off[g + 1] - n0;
  const int64_t e0 = in.edge_off[g], E = in.edge_off[g + 1] - e0;
  const int64_t Et = in.edge_off[in.n_graphs];
  Local& L = c.loc[g];
  if (n <= 0) { c.err[g] = E_EMPTY; return; }
  const int64_t* src = in.edge_index + e0;
  const int64_t* dst = in.edge_index + Et + e0;
  for (int64_t e = 0; e < E; ++e)
    if (src[e] < 0 || src[e] >= n || dst[e] < 0 || dst[e] >= n) { c.err[g] = E_RANGE; return; }
  std::vector<int64_t> c0, c1;
  if (!in.cluster0 || !in.cluster1 || in.c1_off[g + 1] - in.c1_off[g] <= 0) {
    if (in.require_clusters) { c.err[g] = E_NOCL; return; }
    c0.assign(n, 0);
    c1.assign(1, 0);
  } else {
    c0.assign(in.cluster0 + n0, in.cluster0 + n0 + n);
    c1.assign(in.cluster1 + in.c1_off[g], in.cluster1 + in.c1_off[g + 1]);
  }
  if (!dense_ids(c0.data(), n, L.dense0, L.k0)) { c.err[g] = E_NEG; return; }
  if ((int64_t)c1.size() != L.k0) { c.err[g] = E_C1LEN; return; }
  if (!dense_ids(c1.data(), L.k0, L.dense1, L.k1)) { c.err[g] = E_NEG; return; }
  // pool_edge: relabel, drop self loops, coalesce (unique, sorted by (row, col))
  L.pkey.clear();
  if ((int64_t)L.k0 * L.k0 <= (1 << 16)) {  // small pooled graphs: bitmap, read out in (row, col) order
    std::vector<uint8_t> mark((size_t)L.k0 * L.k0, 0);
    for (int64_t e = 0; e < E; ++e) {
      const int64_t pr = L.dense0[src[e]], pc = L.dense0[dst[e]];
      if (pr != pc) mark[pr * L.k0 + pc] = 1;
    }
    for (int64_t q = 0; q < (int64_t)L.k0 * L.k0; ++q)
      if (mark[q]) L.pkey.push_back(q);
  } else {
    for (int64_t e = 0; e < E; ++e) {
      const int64_t pr = L.dense0[src[e]], pc = L.dense0[dst[e]];
      if (pr != pc) L.pkey.push_back(pr * L.k0 + pc);
    }
    std::sort(L.pkey.begin(), L.pkey.end());
    L.pkey.erase(std::unique(L.pkey.begin(), L.pkey.end()), L.pkey.end());
  }
}

void fill(Ctx& c, const dr_pack_output& o, int g) {
  const dr_pack_input& in = *c.in;
  const Local& L = c.loc[g];
  const int64_t n0 = in.node_off[g], n = in.node_off[g + 1] - n0;
  const int64_t e0 = in.edge_off[g], E = in.edge_off[g + 1] - e0;
  const int64_t Et = in.edge_off[in.n_graphs];
  const int64_t* src = in.edge_index + e0;
  const int64_t* dst = in.edge_index + Et + e0;
  const int64_t k00 = o.k0_off[g], q0 = o.p1_off[g], k10 = o.k1_off[g];
  const int Fe = in.n_edge_feat;
  // CSR by edge_index[0] and its transpose, with the slot maps
  std::vector<int32_t> perm, tperm;
  csr(src, E, (int32_t)n, o.rowptr + n0 + g, perm);
  csr(dst, E, (int32_t)n, o.t_rowptr + n0 + g, tperm);
  std::vector<int32_t> inv(E);
  for (int64_t s = 0; s < E; ++s) {
    o.col[e0 + s] = (int32_t)dst[perm[s]];
    o.eperm[e0 + s] = perm[s];
    inv[perm[s]] = (int32_t)s;
  }
  for (int64_t s = 0; s < E; ++s) {
    o.t_col[e0 + s] = (int32_t)src[tperm[s]];
    o.t_eid[e0 + s] = inv[tperm[s]];
  }
  {  // symmetric edge multiset iff every CSR row and transposed row hold the same neighbours
    const int32_t* rp = o.rowptr + n0 + g;
    const int32_t* trp = o.t_rowptr + n0 + g;
    std::vector<int32_t> u, v;
    int ok = 1;
    for (int64_t i = 0; i < n && ok; ++i) {
      if (rp[i + 1] - rp[i] != trp[i + 1] - trp[i]) {
        ok = 0;
        break;
      }
      u.assign(o.col + e0 + rp[i], o.col + e0 + rp[i + 1]);
      v.assign(o.t_col + e0 + trp[i], o.t_col + e0 + trp[i + 1]);
      std::sort(u.begin(), u.end());
      std::sort(v.begin(), v.end());
      ok = (u == v);
    }
    c.sym[g] = ok;
  }
  if (Fe > 0 && in.edge_attr && o.edge_attr)
    for (int64_t s = 0; s < E; ++s)
      std::memcpy(o.edge_attr + (e0 + s) * Fe, in.edge_attr + (e0 + perm[s]) * Fe, sizeof(float) * Fe);
  // depth-0 members (ascending node order within each cluster)
  {
    int32_t* mp = o.m0_ptr + k00 + g;
    std::vector<int32_t> cnt(L.k0 + 1, 0);
    for (int64_t i = 0; i < n; ++i) ++cnt[L.dense0[i] + 1];
    for (int k = 0; k < L.k0; ++k) cnt[k + 1] += cnt[k];
    std::memcpy(mp, cnt.data(), sizeof(int32_t) * (L.k0 + 1));
    for (int64_t i = 0; i < n; ++i) {
      o.m0_idx[n0 + cnt[L.dense0[i]]++] = (int32_t)i;
      o.cl0[n0 + i] = L.dense0[i];
    }
  }
  // pooled graph CSR and its transpose (coalesced)
  {
    const int64_t P = (int64_t)L.pkey.size();
    int32_t* rp = o.p1_rowptr + k00 + g;
    std::vector<int32_t> cnt(L.k0 + 1, 0);
    for (int64_t q = 0; q < P; ++q) ++cnt[L.pkey[q] / L.k0 + 1];
    for (int k = 0; k < L.k0; ++k) cnt[k + 1] += cnt[k];
    std::memcpy(rp, cnt.data(), sizeof(int32_t) * (L.k0 + 1));
    for (int64_t q = 0; q < P; ++q) o.p1_col[q0 + q] = (int32_t)(L.pkey[q] % L.k0);
    std::vector<int64_t> tk(P);
    for (int64_t q = 0; q < P; ++q) tk[q] = (L.pkey[q] % L.k0) * L.k0 + L.pkey[q] / L.k0;
    std::sort(tk.begin(), tk.end());
    int32_t* trp = o.p1t_rowptr + k00 + g;
    std::fill(cnt.begin(), cnt.end(), 0);
    for (int64_t q = 0; q < P; ++q) ++cnt[tk[q] / L.k0 + 1];
    for (int k = 0; k < L.k0; ++k) cnt[k + 1] += cnt[k];
    std::memcpy(trp, cnt.data(), sizeof(int32_t) * (L.k0 + 1));
    for (int64_t q = 0; q < P; ++q) o.p1t_col[q0 + q] = (int32_t)(tk[q] % L.k0);
    // transposed slot (b, a) -> pooled CSR slot of the edge a -> b
    if (o.p1t_pid)
      for (int64_t q = 0; q < P; ++q) {
        const int64_t key = (tk[q] % L.k0) * L.k0 + tk[q] / L.k0;
        o.p1t_pid[q0 + q] = (int32_t)(std::lower_bound(L.pkey.begin(), L.pkey.end(), key) - L.pkey.begin());
      }
    // pooled edge_attr: PyG coalesce sums the attributes of merged edges, in
    // input edge order (community_pooling.py:212 -> pool_edge)
    if (o.p1_ea && Fe > 0 && in.edge_attr) {
      float* pe = o.p1_ea + q0 * Fe;
      std::fill(pe, pe + P * Fe, 0.f);
      for (int64_t e = 0; e < E; ++e) {
        const int64_t pr = L.dense0[src[e]], pc = L.dense0[dst[e]];
        if (pr == pc) continue;
        const int64_t q = std::lower_bound(L.pkey.begin(), L.pkey.end(), pr * L.k0 + pc) - L.pkey.begin();
        for (int f = 0; f < Fe; ++f) pe[q * Fe + f] += in.edge_attr[(e0 + e) * Fe + f];
      }
    }
  }
  // depth-1 members
  {
    int32_t* mp = o.m1_ptr + k10 + g;
    std::vector<int32_t> cnt(L.k1 + 1, 0);
    for (int k = 0; k < L.k0; ++k) ++cnt[L.dense1[k] + 1];
    for (int m = 0; m < L.k1; ++m) cnt[m + 1] += cnt[m];
    std::memcpy(mp, cnt.data(), sizeof(int32_t) * (L.k1 + 1));
    for (int k = 0; k < L.k0; ++k) {
      o.m1_idx[k00 + cnt[L.dense1[k]]++] = k;
      o.cl1[k00 + k] = L.dense1[k];
    }
  }
}

template <class Fn>
void parallel_graphs(int G, int threads, Fn fn) {
  if (threads <= 1 || G < 64) {
    for (int g = 0; g < G; ++g) fn(g);
    return;
  }
  std::atomic<int> next(0);
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&]() {
      for (int g = next.fetch_add(1); g < G; g = next.fetch_add(1)) fn(g);
    });
  for (auto& th : pool) th.join();
}

int nthreads(int requested) {
  if (requested > 0) return requested;
  const unsigned hc = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(16u, hc ? hc : 1u));
}

const char* err_text(int e) {
  switch (e) {
    case E_RANGE: return "edge_index out of range";
    case E_EMPTY: return "graph has no nodes (torch.max over an empty cluster would fail in the reference)";
    case E_C1LEN: return "cluster1 length differs from the number of depth-0 clusters";
    case E_NEG: return "negative cluster ids";
    case E_NOCL: return "no cluster0/cluster1 (set clustering_method when building the dataset)";
    default: return "invalid graph";
  }
}

}  // namespace

extern "C" int dr_pack_sizes(const dr_pack_input* in, int64_t* k0_count, int64_t* p1_count, int64_t* k1_count,
                             int32_t threads, char* err, int32_t err_len) {
  if (!in || !k0_count || !p1_count || !k1_count || in->n_graphs < 0 || in->n_feat < 0) return DR_E_ARG;
  if (!in->node_off || !in->edge_off || (in->edge_off[in->n_graphs] > 0 && !in->edge_index)) return DR_E_ARG;
  Ctx c;
  c.in = in;
  c.loc.resize(in->n_graphs);
  c.err.assign(in->n_graphs, 0);
  c.sym.assign(in->n_graphs, 1);
  parallel_graphs(in->n_graphs, nthreads(threads), [&](int g) { analyse(c, g); });
  for (int g = 0; g < in->n_graphs; ++g) {
    if (c.err[g]) {
      if (err && err_len > 0) std::snprintf(err, err_len, "graph %d: %s", g, err_text(c.err[g]));
      return DR_E_ARG;
    }
    k0_count[g] = c.loc[g].k0;
    p1_count[g] = (int64_t)c.loc[g].pkey.size();
    k1_count[g] = c.loc[g].k1;
  }
  return DR_OK;
}

extern "C" int dr_pack_fill(const dr_pack_input* in, const dr_pack_output* out, int32_t* symmetric, int32_t threads) {
  if (!in || !out || !symmetric || in->n_graphs < 0) return DR_E_ARG;
  Ctx c;
  c.in = in;
  c.loc.resize(in->n_graphs);
  c.err.assign(in->n_graphs, 0);
  c.sym.assign(in->n_graphs, 1);
  std::atomic<int> bad(0);
  parallel_graphs(in->n_graphs, nthreads(threads), [&](int g) {
    analyse(c, g);
    if (c.err[g] || c.loc[g].k0 != out->k0_off[g + 1] - out->k0_off[g] ||
        (int64_t)c.loc[g].pkey.size() != out->p1_off[g + 1] - out->p1_off[g] ||
        c.loc[g].k1 != out->k1_off[g + 1] - out->k1_off[g]) {
      bad.store(1);
      return;
    }
    fill(c, *out, g);
    Local().dense0.swap(c.loc[g].dense0);  // release per-graph scratch early
    std::vector<int64_t>().swap(c.loc[g].pkey);
  });
  if (bad.load()) return DR_E_ARG;
  int all_sym = 1;
  for (int g = 0; g < in->n_graphs; ++g) all_sym &= c.sym[g];
  *symmetric = all_sym;
  return DR_OK;
}
