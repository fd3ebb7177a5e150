/*
 * deeprank2_amd — C ABI of the MI355X (gfx950) GNN hot path for DeepRank2.
 *
 * Everything here is plain C: device pointers, sizes, a hipStream_t passed as
 * void*.  No torch types cross this boundary.  The library never allocates or
 * frees caller memory; every output is preallocated by the caller.  Every
 * entry returns 0 on success or a hipError_t / negative DR_E* code; no
 * exception crosses the ABI.  Launches go on the caller's stream and no entry
 * synchronises the host, so every call is capturable in a hipGraph.
 *
 * Reference interface each entry replaces (paths relative to the reference
 * repo deeprank2 v3.1.0):
 *
 *   dr_ginet_graph_pass     GINet.forward + autograd backward
 *                           (deeprank2/neuralnets/gnn/ginet.py:90-125, with the
 *                           GINetConvLayer of ginet.py:40-60 and
 *                           community_pooling / get_preloaded_cluster of
 *                           deeprank2/utils/community_pooling.py:23-27,165-242),
 *                           plus the loss gradient of Trainer._epoch
 *                           (deeprank2/trainer.py:686-689)
 *   dr_fout_graph_pass      FoutNet.forward + autograd backward
 *                           (deeprank2/neuralnets/gnn/foutnet.py:48-66,99-118)
 *                           plus the same loss gradient
 *   dr_reduce_update        loss_.backward() parameter-gradient reduction and
 *                           optimizer.step() of Trainer._epoch
 *                           (trainer.py:689-690; torch.optim.Adam configured at
 *                           trainer.py:419)
 *   dr_spmm_csr             torch_scatter.scatter_sum(h, row, out=zeros) over
 *                           gathered rows (ginet.py:45,55-58; vanilla_gnn.py:35)
 *   dr_spmm_csr_w           the edge-weighted scatter_mean of
 *                           SGraphAttentionLayer (sgat.py:71-80)
 *   dr_linear_xwT / dr_linear_xw / dr_linear_dw
 *                           the node-side nn.Linear(bias=False) of
 *                           GINetConvLayer.fc (ginet.py:45) and its backward
 *   dr_vanilla_graph_pass   VanillaNetwork.forward + autograd backward
 *                           (deeprank2/neuralnets/gnn/vanilla_gnn.py:26-65)
 *   dr_edge_mlp_scatter[_bwd]  VanillaConvolutionalLayer edge MLP + scatter_sum
 *                           (vanilla_gnn.py:29-35) on any edge list
 *   dr_segment_max[_bwd] / dr_segment_mean
 *                           torch_scatter scatter_max / scatter_mean and PyG
 *                           max_pool_x behind community_pooling / max_pool_x
 *                           (community_pooling.py:165-242; ginet.py:103)
 *   dr_pack_sizes / dr_pack_fill   GraphDataset collate + per-graph pooling
 *                           index work (host; dataset.py:883-1052, trainer.py:541,
 *                           community_pooling.py:23-27,205-225)
 *   dr_sgat_graph_pass      SGAT.forward + backward (sgat.py:56-133)
 *   dr_ginet_nocluster_graph_pass
 *                           ginet_nocluster.GINet.forward + backward
 *                           (ginet_nocluster.py:84-111)
 *   dr_mcl / dr_mcl_assign  community_detection(method="mcl") of
 *                           Trainer._precluster (community_pooling.py:96-162,
 *                           trainer.py:319-348)
 *   dr_csr_from_coo         the ordering torch_scatter's CPU scatter_add_
 *                           implies for edge_index[0] (ginet.py:41,58): a stable
 *                           row-sorted CSR, built on the device
 */
#ifndef DEEPRANK2_AMD_H
#define DEEPRANK2_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DR_OK 0
#define DR_E_ARG (-1)       /* bad argument (null pointer, negative size ...) */
#define DR_E_LDS (-2)       /* a graph does not fit the per-graph LDS kernel  */
#define DR_E_UNSUPPORTED (-3)

/* ------------------------------------------------------------------------
 * Packed graph store (HBM-resident).  "local" = index relative to the graph.
 * G graphs; N_all nodes; E_all directed edges (edge_index columns); K0_all
 * depth-0 (pooled) nodes; K1_all depth-1 clusters; P1_all pooled edges.
 * Per graph g the CSR is sorted by edge_index[0] (the scatter index of
 * ginet.py:58) and keeps the original edge order inside a row.
 * ---------------------------------------------------------------------- */
typedef struct dr_graph_store {
  int32_t n_graphs;          /* G                                             */
  int32_t n_feat;            /* F                                             */
  int32_t x_stride;          /* row stride of x in floats: multiple of 4, >= F, pad columns zero */
  int32_t transpose_aliased; /* 1: p1t_* arrays are the p1_* arrays (symmetric pooled graphs) */
  const float* x;            /* [N_all, x_stride] fp32 (16-byte aligned rows) */
  const int64_t* node_off;   /* [G+1]                                         */
  const int64_t* edge_off;   /* [G+1] directed edges per graph (edge_attr rows, CSR order) */
  const int64_t* col_off;    /* [G+1] 16-byte aligned start of each graph's col / t_col block */
  const int32_t* rowptr;     /* [N_all+G] local CSR row pointers (g at node_off[g]+g) */
  const uint16_t* col;       /* local gathered node (edge_index[1]), graph g at col_off[g] */
  const int32_t* t_rowptr;   /* transpose CSR (by edge_index[1], stable: original edge order) */
  const uint16_t* t_col;
  const int64_t* k0_off;     /* [G+1] depth-0 clusters per graph              */
  const int32_t* m0_ptr;     /* [K0_all+G] members of each depth-0 cluster    */
  const int32_t* m0_idx;     /* [N_all] local node ids, ascending per cluster  */
  const int64_t* p1_off;     /* [G+1] pooled (coalesced) edges per graph      */
  const int32_t* p1_rowptr;  /* [K0_all+G]                                    */
  const int32_t* p1_col;     /* [P1_all]                                      */
  const int32_t* p1t_rowptr; /* transpose of the pooled CSR                   */
  const int32_t* p1t_col;
  const int64_t* k1_off;     /* [G+1] depth-1 clusters per graph              */
  const int32_t* m1_ptr;     /* [K1_all+G]                                    */
  const int32_t* m1_idx;     /* [K0_all] local depth-0 ids, ascending          */
  const float* y;            /* [G] target (class index as float for classif) */
  const float* ea;           /* edge_attr in CSR slot order: graph g's slot e at row col_off[g]+e, [*, max(Fe,1)] */
  const int32_t* t_eid;      /* t_col slot -> CSR slot of the same edge (local), at col_off[g]+slot */
  int32_t n_edge_feat;       /* Fe                                            */
  int32_t pad0;
  const float* p1_ea;        /* [P1_all, max(Fe,1)] pooled edge_attr: sums over merged edges (PyG coalesce) */
  const int32_t* p1t_pid;    /* [P1_all] pooled transposed slot -> pooled CSR slot (local) */
  const uint16_t* x_bf16;    /* optional [N_all, x_bf16_stride] bf16 copy of x (round to nearest even),
                                16-byte rows, pad zero; read instead of x by passes with
                                compute_dtype DR_DTYPE_BF16 (BASELINE configs[3])           */
  int32_t x_bf16_stride;     /* multiple of 8, >= F                                */
  int32_t pad1;
  const int32_t* cl0;        /* [N_all] dense depth-0 cluster id of each node (local), the
                                inverse of m0_ptr/m0_idx                               */
} dr_graph_store;

/* One mini-batch slot: where graph `gid` lives in the store (64 bytes, so a
 * workgroup reads its whole descriptor with one scalar load).  Built from the
 * graph ids on the host (the store keeps host copies of the offset tables).  */
typedef struct dr_graph_desc {
  int64_t node0;  /* node_off[gid]  (also indexes rowptr as node0 + gid)   */
  int64_t col0;   /* col_off[gid]                                         */
  int64_t k0;     /* k0_off[gid]    (m0_ptr / p1_rowptr at k0 + gid)      */
  int64_t p1;     /* p1_off[gid]                                          */
  int64_t k1;     /* k1_off[gid]    (m1_ptr at k1 + gid)                  */
  int32_t n_nodes, n_edges, n_k0, n_p1, n_k1, gid;
} dr_graph_desc;

/* GINet parameters (device pointers into the nn.Parameters, fp32).  */
typedef struct dr_ginet_weights {
  const float* w1;   /* conv1.fc.weight      [16, F]  */
  const float* w1e;  /* conv1_ext.fc.weight  [16, F]  */
  const float* w2;   /* conv2.fc.weight      [32, 16] */
  const float* w2e;  /* conv2_ext.fc.weight  [32, 16] */
  const float* fc1w; /* fc1.weight           [128, 64] */
  const float* fc1b; /* fc1.bias             [128]     */
  const float* fc2w; /* fc2.weight           [out, 128] */
  const float* fc2b; /* fc2.bias             [out]      */
} dr_ginet_weights;

#define DR_PASS_FORWARD 1   /* write out[B,out]                                  */
#define DR_PASS_BACKWARD 2  /* backprop dout (given, or from the loss) to slabs   */
#define DR_PASS_WPACK_CURRENT 4 /* dr_vanilla_fused_pass: wpack already holds these weights
                                   (dr_vanilla_wpack, then kept current by dr_adam.mirror):
                                   no pack launch, and pass->fault[0] must already be zero
                                   (dr_adam.fault_clear of the previous step's update)     */
#define DR_LOSS_NONE 0      /* dout is an input (autograd)                       */
#define DR_LOSS_MSE 1       /* nn.MSELoss(mean) on pred.reshape(-1)               */
#define DR_LOSS_CE 2        /* nn.CrossEntropyLoss(mean, optional class weights)  */

#define DR_SLAB_STRIDE(F) (32 * (F) + 1024)
#define DR_HEAD_STRIDE(out) (320 + (((out) + 3) & ~3))
#define DR_MAX_OUT 16
#define DR_DROPOUT_OFF 0
#define DR_DROPOUT_MASK 1  /* keep mask given in pass->mask        */
#define DR_DROPOUT_HASH 2  /* counter-based hash, see dr_dropout_mask */

#define DR_DTYPE_F32 0
#define DR_DTYPE_BF16 1

typedef struct dr_pass {
  int32_t flags;        /* DR_PASS_* bitmask                                   */
  int32_t out_dim;      /* fc2 rows                                            */
  int32_t loss_kind;    /* DR_LOSS_*                                           */
  int32_t use_dropout;  /* DR_DROPOUT_*: training-mode dropout of fc1's output  */
  float drop_scale;     /* 1/(1-p)                                             */
  float drop_p;         /* p (DR_DROPOUT_HASH)                                 */
  uint64_t drop_seed;   /* DR_DROPOUT_HASH: keep[b,r] = u(seed, offset, 128b+r) >= p */
  uint64_t drop_offset;
  float loss_scale;     /* 1/B (MSE) or 1/sum(w_y) (CE)                        */
  int32_t compute_dtype;/* DR_DTYPE_F32, or DR_DTYPE_BF16: the conv1 node GEMM takes bf16
                           operands (x from store->x_bf16, Z = A x rounded to bf16, W1
                           rounded to bf16) on the bf16 MFMA with fp32 accumulate; all
                           other arithmetic, the outputs and the gradients stay fp32 (GINet) */
  const uint8_t* mask;  /* [B,128] keep mask (DR_DROPOUT_MASK)                 */
  const float* class_w; /* [out] CE class weights or NULL                      */
  float* out;           /* [B,out] predictions (FORWARD)                       */
  const float* dout;    /* [B,out] upstream gradient (BACKWARD, LOSS_NONE)     */
  float* loss_per_graph;/* [B] weighted per-graph loss term (fused loss), or NULL */
  float* slab;          /* [B, DR_SLAB_STRIDE(F)] per-graph conv weight-gradient partials */
  float* head;          /* [B, DR_HEAD_STRIDE(out)] per-graph head vectors g, hd, dh, dout */
  int64_t* stamps;      /* diagnostic builds only (-DDR_STAMPS): [B, 32] s_memtime per phase; NULL */
  int64_t* step_counter;/* optional device [2]: drop_offset := counter[0] (read by every
                           workgroup); workgroup 0 snapshots counter[0] into counter[1] for
                           dr_reduce_update, which advances counter[0].  Makes a
                           step's launch arguments constant (hipGraph replay).            */
  uint32_t* fault;      /* optional device [2], passes with in-launch hand-offs between
                           workgroups (dr_vanilla_fused_pass, split > 1): fault[0] is cleared
                           by the pass's pack launch and set to 1 when one of its
                           hand-off waits gave up (its partials are then wrong); fault[1]
                           counts such launches and is only ever cleared by the caller.
                           Hand the same pointer to dr_adam.fault so the step's update
                           is withheld and its loss reads NaN.  With DR_PASS_WPACK_CURRENT
                           there is no pack launch: the caller must clear fault[0] itself,
                           normally through the previous update's dr_adam.fault_clear (+
                           ticket); otherwise one give-up stays set and every later step is
                           withheld with a NaN loss.                                      */
  int32_t spin_limit;   /* polls before a hand-off wait gives up (<= 0: 1 << 22)        */
  int32_t pad0;
  const int32_t* slot;  /* optional device [B] (GINet / FoutNet / SGAT passes): launch position b
                           writes row slot[b] of out, loss_per_graph, slab, head and reads row
                           slot[b] of dout / mask, and draws dropout unit slot[b] -- a batch run
                           as several launches (graphs that fit one workgroup's LDS on the
                           per-graph kernel, the others on the large-graph path) fills the rows
                           one launch over the whole batch would                          */
} dr_pass;

/* One workgroup per graph: conv1 -> depth-0 community pooling -> conv2 ->
 * depth-1 max pooling -> per-graph mean -> fc1/relu/dropout/fc2, and (when
 * DR_PASS_BACKWARD) the full backward of that graph, all in LDS.
 * descs: [B] device descriptors of the batch's graphs.  lds_bytes: the
 * dynamic LDS the largest graph of the batch needs (dr_ginet_lds_bytes).  */
int dr_ginet_graph_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                        const dr_ginet_weights* w, const dr_pass* pass,
                        int32_t lds_bytes, void* stream);

/* Dynamic LDS bytes dr_ginet_graph_pass needs for a graph of these sizes.  */
int64_t dr_ginet_lds_bytes(int32_t n_nodes, int32_t n_edges, int32_t n_feat, int32_t k0,
                           int32_t p1_edges, int32_t k1, int32_t transpose_aliased, int32_t out_dim);

/* Accumulating training pass for batches larger than the CU count (r05):
 * the loss + backward of GINet.forward over the batch (ginet.py:90-125 under
 * trainer.py:_train_epoch's loss.backward) like dr_ginet_graph_pass, but
 * n_groups workgroups each run graphs w, w + n_groups, ... in that order and
 * keep the sums of their gradients on chip, then write ONE row per workgroup:
 * pass->slab[w * dr_ginet_acc_row_floats(F, OUT) ...] = [dW1cat 32F | dW2cat
 * 1024 | fc1.weight 128x64 | fc1.bias 128 | fc2.weight OUTx128 | fc2.bias OUT]
 * and pass->loss_per_graph[w] = the workgroup's loss sum.  pass->out gets
 * every graph's output as usual; pass->head is unused.  The reduce sums the
 * n_groups rows (dr_reduce_update with an all-slab table).  Deterministic
 * (fixed graph -> workgroup map and order); a different fp32 association
 * than the per-graph partials.  Needs BACKWARD, a fused loss, no slot; F32.
 * lds_bytes: the graph carve as for dr_ginet_graph_pass (the accumulators'
 * words are added inside; the total must fit 160 KB).  plan (optional,
 * device int32 [n_groups + 1 + n_batch]): workgroup w runs the batch
 * positions plan[n_groups + 1 + k] for k in [plan[w], plan[w + 1]) in that
 * order (every position exactly once: the caller balances the work, e.g. by
 * graph size); NULL: positions w, w + n_groups, ...
 * max_sizes (optional, host int32 [5]): the batch's largest n_nodes, n_edges,
 * n_k0, n_p1, n_k1.  When given and dr_ginet_acc_lds_bytes(max_sizes, ...)
 * fits 160 KB, the prefetch layout runs: the weights stay in LDS across a
 * workgroup's graphs and graph k+1's inputs are DMA'd while graph k's tail
 * runs; otherwise lds_bytes applies.  Same results either way.             */
int dr_ginet_acc_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                      const dr_ginet_weights* w, const dr_pass* pass, int32_t lds_bytes, int32_t n_groups,
                      const int32_t* plan, const int32_t* max_sizes, void* stream);
int32_t dr_ginet_acc_row_floats(int32_t n_feat, int32_t out_dim);
/* Dynamic LDS bytes of dr_ginet_acc_pass's prefetch layout for these batch
 * maxima (host int32 [5] as above), or -1 for NULL.                          */
int64_t dr_ginet_acc_lds_bytes(const int32_t* max_sizes, int32_t n_feat, int32_t transpose_aliased, int32_t out_dim);

/* ---- GINet on graphs larger than one workgroup's LDS (atom-level graphs) ----
 * Two launches with the same result as dr_ginet_graph_pass:
 *   1. one workgroup per tile of plan->tile_rows nodes: Z = A X for its rows
 *      (CSR gather from HBM/L2), H = relu(Z [W1;W1e]^T) on MFMA, and the
 *      tile's share of the depth-0 max pool (per cluster & channel: max and
 *      first arg) -> plan->part_val / part_arg; Z rows -> plan->z;
 *   2. one workgroup per graph: combine the tile partials in node order
 *      (first max wins, as torch_scatter), then conv2 ... head, loss and the
 *      backward exactly as the single-workgroup kernel; dW1 reads Z at the
 *      pooling args from plan->z.
 * The plan arrays are per batch (host-built, see deeprank2_amd.fused).      */
#define DR_LARGE_TILE 128
typedef struct dr_large_plan {
  const int32_t* tile_first; /* [B+1] first tile of each batch slot             */
  const int32_t* z_row0;     /* [B+1] first row of each slot's Z block          */
  const int32_t* tile_slot;  /* [n_tiles] batch slot of each tile               */
  int32_t n_tiles;
  int32_t k0_max;            /* >= every n_k0 of the batch                      */
  int32_t tile_rows;         /* nodes per tile: multiple of 16, <= DR_LARGE_TILE */
  int32_t halo_max;          /* >= every tile's halo size; 0 = no halos (gather X from HBM per edge) */
  float* z;                  /* [z_row0[B], x_stride] workspace                 */
  float* part_val;           /* [n_tiles, k0_max, 32] workspace                 */
  int32_t* part_arg;         /* [n_tiles, k0_max, 32] workspace                 */
  /* Tile halos (optional): the distinct neighbours of a tile's rows are staged
   * into LDS once, so the edge gather reads X from LDS instead of re-reading
   * each neighbour row from L2/HBM once per edge.                             */
  const int32_t* halo_off;   /* [n_tiles+1] offsets into halo_ids               */
  const int32_t* halo_ids;   /* per tile: its neighbours' local node ids, ascending */
  const int32_t* lcol_off;   /* [n_tiles+1] offsets into lcol, multiples of 8   */
  const uint16_t* lcol;      /* per tile, per CSR edge of its rows: index into the tile's halo
                                (array padded by 8 entries past the last tile)    */
  const int32_t* tile_members; /* [n_tiles, tile_rows] with halos: the tile's nodes grouped by
                                  depth-0 cluster, ascending within a cluster       */
  const int32_t* tile_mptr;    /* [n_tiles, k0_max+1] with halos: cluster k's run in tile_members */
  uint64_t* part_key;          /* optional [B, k0_max, 32], zero on entry and left zero: the depth-0
                                  max over tiles by 64-bit atomic max of (H bits << 32 | ~node), i.e.
                                  the largest value and, among equal values, the first node (H >= +0
                                  after relu, NaN never enters); replaces part_val/part_arg */
  uint32_t* arrive;            /* must be NULL (the one-launch form of r03-r05 was measured
                                  slower and removed in r06; the field keeps the layout)    */
} dr_large_plan;

int dr_ginet_large_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                        const dr_large_plan* plan, const dr_ginet_weights* w, const dr_pass* pass,
                        int32_t conv_lds_bytes, int32_t tail_lds_bytes, void* stream);

/* Dynamic LDS of the two launches of dr_ginet_large_pass (largest graph).  */
int64_t dr_ginet_large_conv_lds_bytes(int32_t n_nodes, int32_t n_feat, int32_t k0, int32_t halo_max,
                                      int32_t tile_edges_max);
/* The same for passes with compute_dtype DR_DTYPE_BF16 (bf16 halo rows and Z operand).  */
int64_t dr_ginet_large_conv_lds_bytes_bf16(int32_t n_nodes, int32_t n_feat, int32_t k0, int32_t halo_max,
                                           int32_t tile_edges_max);
int64_t dr_ginet_tail_lds_bytes(int32_t k0, int32_t p1_edges, int32_t k1, int32_t transpose_aliased,
                                int32_t out_dim);

/* ---- FoutNet (deeprank2/neuralnets/gnn/foutnet.py:72-118) ---------------- */

/* FoutNet weights, all row-major as the torch parameters are stored.       */
typedef struct dr_fout_weights {
  const float* wc1;  /* conv1.wc    [F, 16]   (foutnet.py:32) */
  const float* wn1;  /* conv1.wn    [F, 16]   (foutnet.py:33) */
  const float* b1;   /* conv1.bias  [16]                      */
  const float* wc2;  /* conv2.wc    [16, 32]                  */
  const float* wn2;  /* conv2.wn    [16, 32]                  */
  const float* b2;   /* conv2.bias  [32]                      */
  const float* fc1w; /* fc1.weight  [64, 32]                  */
  const float* fc1b; /* fc1.bias    [64]                      */
  const float* fc2w; /* fc2.weight  [out, 64]                 */
  const float* fc2b; /* fc2.bias    [out]                     */
} dr_fout_weights;

/* Per-graph partials of dr_fout_graph_pass:
 *   slab: dWc1 [F,16] | dWn1 [F,16] | db1 [16] | dWc2 [16,32] | dWn2 [16,32] | db2 [32]
 *   head: g [32] | relu(fc1) [64] | its grad [64] | dout [out]                 */
#define DR_FOUT_SLAB_STRIDE(F) (32 * (F) + 1072)
#define DR_FOUT_HEAD_STRIDE(out) (160 + (((out) + 3) & ~3))

/* One workgroup per graph: FoutLayer(F,16) (foutnet.py:48-66; NaN where a node
 * has no out-edge, as torch.mean over an empty set) -> relu -> depth-0
 * community pooling -> FoutLayer(16,32) on the pooled graph -> relu -> depth-1
 * max_pool_x -> per-graph mean -> fc1/relu/fc2, and its backward.  Same
 * dr_pass contract as dr_ginet_graph_pass (no dropout: use_dropout must be
 * DR_DROPOUT_OFF); partial layouts above.                                    */
int dr_fout_graph_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                       const dr_fout_weights* w, const dr_pass* pass, int32_t lds_bytes, void* stream);

/* Dynamic LDS bytes dr_fout_graph_pass needs for a graph of these sizes.   */
int64_t dr_fout_lds_bytes(int32_t n_nodes, int32_t n_edges, int32_t n_feat, int32_t k0, int32_t p1_edges,
                          int32_t k1, int32_t transpose_aliased, int32_t out_dim);

/* ---- ginet_nocluster.GINet (deeprank2/neuralnets/gnn/ginet_nocluster.py:66-111)
 * One workgroup per graph: both GINetConvLayer branches conv1 -> relu ->
 * conv2 -> relu on the full graph (no pooling; needs the store's transposed
 * CSR for the backward), per-graph mean, fc1/relu/dropout/fc2, loss and
 * backward.  Same weights struct, dr_pass contract and slab/head layouts as
 * dr_ginet_graph_pass (DR_SLAB_STRIDE / DR_HEAD_STRIDE), so dr_reduce_update
 * uses the GINet recipe.  Clusters in the store are ignored.               */
int dr_ginet_nocluster_graph_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                                  const dr_ginet_weights* w, const dr_pass* pass, int32_t lds_bytes, void* stream);
int64_t dr_ginet_nocluster_lds_bytes(int32_t n_nodes, int32_t n_edges, int32_t n_feat, int32_t out_dim);

/* ginet_nocluster.GINet on graphs beyond one workgroup's LDS (atom level):
 * the same arithmetic as a pipeline of tile kernels over the batch's rows
 * (tiles of <= 64 consecutive rows of one graph, their halo -- out- and
 * in-neighbours -- staged in LDS):
 *   1. Z1 = A X, H1 = relu(Z1 [W1; W1e]^T)         (MFMA)    -> Z1, H1
 *   2. Z2 = A H1, H2 = relu(Z2_b W2_b^T)           (MFMA)    -> Z2, relu' bits, tile column sums
 *   3. per graph: mean, fc1/relu/dropout/fc2, loss, head backward -> dG / N
 *   4. dZ2 = dS2 W2_b and the tile's dW2 partial  (MFMA)    -> dZ2
 *   5. dS1 = relu'(H1) (A^T dZ2) and the tile's dW1 partial (MFMA)
 *   6. per graph: the tiles' partials summed in tile order into the slab.
 * Slab / head partials as dr_ginet_nocluster_graph_pass (the GINet recipe).
 * base: dr_nc_large_scratch_floats(n_rows, B, n_tiles, F) floats.          */
typedef struct dr_nc_plan {
  float* base;
  const int32_t* row0;       /* [B+1] first batch row of each slot            */
  const int32_t* row_slot;   /* [n_rows] slot of each batch row                */
  int64_t n_rows;
  const int32_t* tile_row0;  /* [n_tiles+1] batch row ranges (one graph each, <= 64 rows) */
  const int32_t* tile_first; /* [B+1] first tile of each slot                  */
  const int32_t* halo_off;   /* [n_tiles+1] */
  const int32_t* halo_ids;   /* per tile: local ids of its rows' out- and in-neighbours, ascending */
  const int32_t* lcol_off;   /* [n_tiles+1] */
  const uint16_t* lcol;      /* halo index of each of the tile's CSR edges      */
  const int32_t* ltcol_off;  /* [n_tiles+1] */
  const uint16_t* ltcol;     /* halo index of each of the tile's transposed edges */
  int32_t n_tiles, halo_max, tile_edges_max, tile_tedges_max;
} dr_nc_plan;
int dr_ginet_nocluster_large_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                                  const dr_nc_plan* plan, const dr_ginet_weights* w, const dr_pass* pass,
                                  void* stream);
int64_t dr_nc_large_scratch_floats(int64_t n_rows, int32_t n_batch, int32_t n_tiles, int32_t n_feat);
int64_t dr_nc_large_lds_bytes(int32_t n_feat, int32_t halo_max, int32_t tile_edges_max, int32_t tile_tedges_max,
                              int32_t out_dim);

/* ---- SGAT (deeprank2/neuralnets/gnn/sgat.py:13-133) -----------------------
 * Same kernel family and partial layouts as FoutNet, with dr_fout_weights
 * pointing into SGAT's parameters: wc1 = conv1.weight rows 0..F-1, wn1 = rows
 * F..2F-1 (conv1.weight is [2F, 16]), b1 = conv1.bias, wc2/wn2 = conv2.weight
 * rows 0..15 / 16..31, b2 = conv2.bias, fc1/fc2 as FoutNet.  The slab's
 * dWc1|dWn1 and dWc2|dWn2 blocks are then d conv1.weight and d conv2.weight.
 * Requires n_edge_feat == 1 (sgat.py:71 multiplies [E, Fe] into [E, out]).
 * One workgroup per graph: SGraphAttentionLayer(F,16) (scatter_mean, edge-less
 * rows give the bias) -> relu -> depth-0 community pooling (pooled edge_attr =
 * sums, store p1_ea) -> SGraphAttentionLayer(16,32) -> relu -> depth-1
 * max_pool_x -> mean -> fc1/relu/fc2, and its backward.                     */
int dr_sgat_graph_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                       const dr_fout_weights* w, const dr_pass* pass, int32_t lds_bytes, void* stream);
int64_t dr_sgat_lds_bytes(int32_t n_nodes, int32_t n_edges, int32_t n_feat, int32_t k0, int32_t p1_edges,
                          int32_t k1, int32_t transpose_aliased, int32_t out_dim);

/* ---- FoutNet / SGAT on graphs beyond one workgroup's LDS (atom level) -----
 * Replaces FoutNet.forward / SGAT.forward + backward (foutnet.py:48-66,99-118,
 * sgat.py:56-133) where dr_fout_graph_pass / dr_sgat_graph_pass cannot hold
 * the graph; same result bit for bit on graphs both can run.  Two launches on
 * dr_large_plan (tiles, optional halos; part_key required, arrive unsupported):
 *   1. one workgroup per tile: the mean over out-neighbours (SGAT: weighted,
 *      count clamped to 1, and c1), conv1 on MFMA, relu, the tile's share of
 *      the depth-0 max per (cluster, channel) as 64-bit atomic max keys; the
 *      Zm rows (SGAT: and c1 in column r4(F)) -> plan->z with row stride
 *      z_stride = r4(F) (FoutNet) or r4(F) + 4 (SGAT);
 *   2. one workgroup per graph: the pool from the keys (keys left zero), then
 *      conv2 ... head, loss and backward as the single-workgroup kernel.    */
int dr_fout_large_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                       const dr_large_plan* plan, const dr_fout_weights* w, const dr_pass* pass, int32_t z_stride,
                       int32_t conv_lds_bytes, int32_t tail_lds_bytes, void* stream);
int dr_sgat_large_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                       const dr_large_plan* plan, const dr_fout_weights* w, const dr_pass* pass, int32_t z_stride,
                       int32_t conv_lds_bytes, int32_t tail_lds_bytes, void* stream);
int64_t dr_fout_large_conv_lds_bytes(int32_t n_nodes, int32_t n_feat, int32_t k0, int32_t halo_max,
                                     int32_t tile_edges_max, int32_t sgat);
int64_t dr_fout_tail_lds_bytes(int32_t k0, int32_t p1_edges, int32_t k1, int32_t transpose_aliased, int32_t out_dim,
                               int32_t sgat);

/* ---- VanillaNetwork (deeprank2/neuralnets/gnn/vanilla_gnn.py:10-65) ------- */

typedef struct dr_vanilla_weights {
  const float *we1, *be1; /* _external1._edge_mlp.0 weight [32, 2F+Fe], bias [32] */
  const float *wn1, *bn1; /* _external1._node_mlp.0 weight [F, F+32],  bias [F]  */
  const float *we2, *be2; /* _external2 ...                                        */
  const float *wn2, *bn2;
  const float *g1w, *g1b; /* _graph_mlp.0 weight [128, F], bias [128]             */
  const float *g2w, *g2b; /* _graph_mlp.2 weight [out, 128], bias [out]           */
} dr_vanilla_weights;

/* Per-batch HBM scratch for the node-level intermediates (no per-edge storage):
 * base: dr_vanilla_scratch_floats(n_rows, F, Fe) floats; row0[b]: first row of
 * batch slot b (row0[B] = n_rows = total nodes of the batch).                */
typedef struct dr_vanilla_scratch {
  float* base;
  const int32_t* row0;        /* [B+1]                                          */
  const int32_t* row_slot;    /* [n_rows] batch slot of each row                */
  int64_t n_rows;
  const int32_t* chunk_first; /* [B+1] first row chunk (DR_VANILLA_CHUNK rows) of each slot */
  const int32_t* chunk_slot;  /* [n_chunks]                                     */
  int32_t n_chunks;
  int32_t pad0;
  float* part;                /* [n_chunks, dr_vanilla_part_floats(F, Fe)] weight-gradient partials */
  const int32_t* edge0;       /* optional [B+1] first edge of each slot in relu_words (prefix sums of n_edges) */
  uint32_t* relu_words;       /* optional [2, edge0[B]]: per layer and edge (CSR order) bit c = channel c of
                                 the edge MLP active, written by the forward and read by the backward (which
                                 then neither re-gathers B_j nor re-reads edge_attr for the transposed sum) */
  /* Optional edge-tile plan (needs relu_words): the edge kernels then run one
   * workgroup per tile of consecutive rows of one graph, first staging in LDS
   * the tile's neighbour rows (its halo: B rows in the forward, dS rows in the
   * backward), its edge attributes, ReLU words and halo-local column ids, so
   * every per-edge gather reads LDS; same sums in the same order.           */
  const int32_t* tile_row0;   /* [n_tiles+1] batch row ranges; a tile never spans two graphs */
  const int32_t* halo_off;    /* [n_tiles+1] offsets into halo_ids                          */
  const int32_t* halo_ids;    /* per tile: local node ids of the union of its rows' out- and
                                 in-neighbours, ascending                                     */
  const int32_t* lcol_off;    /* [n_tiles+1] into lcol: the tile's CSR edges rp[i0]..rp[i1]   */
  const uint16_t* lcol;       /* halo index of each such edge's column                       */
  const int32_t* ltcol_off;   /* [n_tiles+1] into ltcol: the tile's transposed edges          */
  const uint16_t* ltcol;      /* halo index of each transposed edge's source                 */
  int32_t n_tiles;
  int32_t halo_max;           /* >= every tile's halo size (<= 65535)                        */
  int32_t tile_edges_max;     /* >= every tile's CSR edge count                               */
  int32_t tile_tedges_max;    /* >= every tile's transposed edge count                        */
  /* Optional with the tile plan when the tile rows divide DR_VANILLA_CHUNK: the
   * backward edge kernel then sums each tile's dWc share (sum over its rows of
   * dS_i * eap_i, [32][Fe]) into tile_wc [n_tiles][32 * max(Fe,1)] instead of
   * writing the per-(row, channel) eap array, and the weight-gradient chunks
   * sum their tiles (tile_first [B+1]: first tile of each slot).           */
  float* tile_wc;
  const int32_t* tile_first;
  int32_t tile_rows;
  /* 2: part holds both layers' partial rows ([2][n_chunks][part floats], layer 1
   * first).  With tile_rows == DR_VANILLA_CHUNK, tile_meta set, Fe <= 4,
   * F <= 32 and the tile carves within 160 KiB, dr_vanilla_graph_pass then runs
   * the chunk-fused kernels: one workgroup per 64-row chunk runs the edge work
   * and every row-local stage around it ([A | B] of its own and halo rows, node
   * MLP, node backward, weight-gradient partials) with the intermediates in
   * LDS -- 7 launches per step instead of 17, the same results (dWc summed in
   * another order).  0 / 1: one layer.                                       */
  int32_t part_layers;
  /* the chunk-fused kernels' per-tile records [n_tiles] (required by them):
   * every offset a chunk workgroup needs, so its prologue is one record load
   * instead of a chain of dependent index loads                             */
  const struct dr_vanilla_tile* tile_meta;
  /* optional [n_tiles][32]: the chunk-fused forward's per-tile column sums of
   * X2 (the mean's DR_VANILLA_CHUNK-row partials, rows in order); NULL: the
   * head sums the same chunks from X2 itself                                 */
  float* part_mean;
} dr_vanilla_scratch;
#define DR_VANILLA_CHUNK 64

/* One 64-row tile (chunk) of the Vanilla pipeline, 128 bytes. */
typedef struct dr_vanilla_tile {
  int64_t rt0;    /* batch row of the tile's first row                          */
  int64_t g0;     /* batch row of its graph's node 0 (row0[slot])              */
  int64_t rp0;    /* index of the graph's node 0 in rowptr / t_rowptr: node0 + gid */
  int64_t col0;   /* the graph's first CSR slot in the store: desc.col0         */
  int64_t xrow;   /* store x row of the tile's first row: node0 + i0            */
  int64_t word0;  /* relu_words index of the graph's edge 0: edge0[slot]        */
  int32_t nr;     /* rows in the tile                                          */
  int32_t slot;   /* batch slot of the graph                                   */
  int32_t i0;     /* graph-local index of the tile's first row                 */
  int32_t e0;     /* graph-local CSR slot of its first edge: rowptr[i0]         */
  int32_t ne;     /* CSR edges of its rows                                     */
  int32_t q0;     /* graph-local transposed slot of its first in-edge: t_rowptr[i0] */
  int32_t nq;     /* transposed edges of its rows                              */
  int32_t h0;     /* halo_off[tile]                                            */
  int32_t n_halo; /* halo rows                                                 */
  int32_t lcol_off, ltcol_off;
  int32_t n_graph; /* its graph's rows                                         */
  int32_t e_graph; /* its graph's CSR edges                                    */
  int32_t pad[7];
} dr_vanilla_tile;

/* slab: per layer [dWe (32 x (2F+Fe)) | dbe (32) | dWn (F x (F+32)) | dbn (F)], layer 1 then 2
 * head: g [r4(F)] | relu(fc1) [128] | its grad [128] | dout [r4(out)] | d mean [r4(F)] */
#define DR_VANILLA_SLAB_STRIDE(F, Fe) (2 * (32 * (2 * (F) + (Fe)) + 32 + (F) * ((F) + 32) + (F)))
#define DR_VANILLA_HEAD_STRIDE(F, out) (2 * (((F) + 3) & ~3) + 256 + (((out) + 3) & ~3))

/* Both VanillaConvolutionalLayers (edge MLP fused into the CSR gather,
 * scatter_sum, node MLP), scatter_mean, the graph MLP, the loss and the whole
 * backward, as a short pipeline of row-parallel kernels over every node of
 * the batch (all CUs busy) plus per-graph reductions.  Same dr_pass contract
 * as the other graph passes (no dropout).  Fe <= 8, F <= 64.                 */
int dr_vanilla_graph_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                          const dr_vanilla_weights* w, const dr_pass* pass, const dr_vanilla_scratch* scratch,
                          int32_t lds_bytes, void* stream);
int64_t dr_vanilla_scratch_floats(int64_t n_rows, int32_t n_feat, int32_t n_edge_feat);
int64_t dr_vanilla_part_floats(int32_t n_feat, int32_t n_edge_feat); /* one layer's gradient entries, rounded up to 4 (a 16-byte row) */
int64_t dr_vanilla_lds_bytes(int32_t n_feat, int32_t n_edge_feat, int32_t out_dim);

/* The same VanillaNetwork training pass (vanilla_gnn.py:26-65 + trainer.py:686-689)
 * with the graph in LDS (vanilla_graph.hip): for batches whose largest graph
 * fits (dr_vanilla_fused_lds_bytes(max N, max E) <= 160 KiB), F <= 32, Fe <= 4.
 * split (1..DR_VANILLA_MAX_SPLIT) workgroups per graph, each owning a
 * contiguous, edge-balanced range of CSR rows; they exchange B2 rows, the
 * mean's column sums and dS2 / dS1 rows through the scratch in-launch.  The
 * slab then holds `split` partial rows per graph (slab row b*split + r; set
 * dr_param_table.slab_rows = split), each graph's head vectors one row.
 * (Summing the partial rows in-launch by the last sibling out was measured
 * slower and heavier: DESIGN.md §5.)
 * Otherwise the slab/head partials of dr_vanilla_graph_pass, so
 * dr_reduce_update is shared.  scratch: device floats, slot b owns
 * dr_vanilla_fused_scratch_floats(N_b, E_b) of them from scratch_off[b]
 * (device int64 [B]).  sync: device uint32 [2B + 1], zero when allocated and
 * left zero by every launch (arrival counters; sync[2B] = nonzero after a
 * hand-off wait of any launch on this batch gave up; pass->fault reports it
 * per launch, pass->spin_limit bounds the waits).  wpack: device floats [dr_vanilla_wpack_floats()],
 * rewritten by every call (the weights in MFMA-fragment order, packed by a
 * first small launch).  Needs the store's transpose + t_eid.               */
#define DR_VANILLA_MAX_SPLIT 4
int dr_vanilla_fused_pass(const dr_graph_store* store, const dr_graph_desc* descs, int32_t n_batch,
                          const dr_vanilla_weights* w, const dr_pass* pass, float* scratch,
                          const int64_t* scratch_off, int32_t split, uint32_t* sync, float* wpack,
                          int32_t lds_bytes, void* stream);
int64_t dr_vanilla_wpack_floats(void);
/* wpack := the weights w of a VanillaNetwork(n_feat, ., n_edge_feat) in MFMA-fragment
 * order (the pack launch dr_vanilla_fused_pass makes unless DR_PASS_WPACK_CURRENT).
 * Run on weights holding 1 + their flat index it yields each wpack slot's source
 * element (0: a constant zero), from which a caller builds dr_adam.mirror_idx.   */
int dr_vanilla_wpack(const dr_vanilla_weights* w, int32_t n_feat, int32_t n_edge_feat, float* wpack, void* stream);
int64_t dr_vanilla_fused_lds_bytes(int32_t n_nodes, int32_t n_edges, int32_t n_edge_feat);
int64_t dr_vanilla_fused_scratch_floats(int32_t n_nodes, int32_t n_edges, int32_t n_edge_feat);

/* Adam (torch.optim.Adam, L2 weight decay added to the gradient) settings.  */
typedef struct dr_adam {
  float lr, beta1, beta2, eps, weight_decay;
  float bias_c1;      /* 1 - beta1^step                                        */
  float bias_c2_sqrt; /* sqrt(1 - beta2^step)                                  */
  int32_t enabled;    /* 0: only write gradients                              */
  int64_t* step_counter; /* optional device [2] (see dr_pass): step = counter[1]+1,
                            bias corrections computed on the device, and (when enabled)
                            counter[0] := step; overrides bias_c1 / bias_c2_sqrt    */
  const float* grad_div; /* optional device scalar, Adam-only calls (slab NULL): every
                            gradient is divided by it (and written back to grad) and so
                            is loss_out[0].  Weighted CrossEntropyLoss under data
                            parallelism: the weighted mean's denominator
                            (trainer.py:688, nn.CrossEntropyLoss(weight)) is only known
                            after the all-reduce, so it travels in the reduced buffer  */
  const uint32_t* fault; /* optional device flag (dr_pass.fault[0] of the graph pass whose
                            partials this call reduces): when nonzero, loss_out[0] and every
                            gradient written are NaN, and Adam leaves parameters, moments
                            and the step counter unchanged                           */
  float* mirror;         /* optional device floats: every parameter element Adam updates is
                            also stored to mirror[mirror_idx[4 f + j]] for each j < 4 whose
                            index is >= 0 (f = the element's flat index over the table's
                            parameters in order): a packed copy of the weights (e.g.
                            dr_vanilla_fused_pass's wpack) kept current with no pack launch */
  const int32_t* mirror_idx; /* device int32 [4 * sum numel], 16-byte aligned          */
  uint32_t* fault_clear; /* optional device flag zeroed once every block of the call has read
                            `fault` (the next graph pass's dr_pass.fault[0] when that pass
                            does not clear it itself, DR_PASS_WPACK_CURRENT)           */
  uint32_t* ticket;      /* device uint32, zero, left zero: required with fault_clear  */
} dr_adam;

/* How one parameter's gradient is assembled from the per-graph partials the
 * graph passes write ([B, slab_stride] slab and [B, head_stride] head rows).  */
#define DR_GRAD_ZERO 0  /* exact zeros (GINet's attention weights, ginet.py:54)      */
#define DR_GRAD_SLAB 1  /* sum_b slab[b, off1 + e]                                   */
#define DR_GRAD_OUTER 2 /* sum_b head[b, off1 + e / cols] * head[b, off2 + e % cols]  */
#define DR_GRAD_HEAD 3  /* sum_b head[b, off1 + e]                                   */
typedef struct dr_grad_recipe {
  int32_t kind, off1, off2, cols;
} dr_grad_recipe;

/* Parameter table, in the model's named_parameters() order.                 */
#define DR_MAX_PARAMS 24
typedef struct dr_param_table {
  float* param[DR_MAX_PARAMS];
  float* grad[DR_MAX_PARAMS];       /* may be NULL (gradient not materialised) */
  float* exp_avg[DR_MAX_PARAMS];
  float* exp_avg_sq[DR_MAX_PARAMS];
  int32_t numel[DR_MAX_PARAMS];
  dr_grad_recipe recipe[DR_MAX_PARAMS];
  int32_t n_params;
  int32_t slab_stride;   /* floats per slab row                                 */
  int32_t head_stride;
  int32_t slab_rows;     /* slab rows per graph (0 or 1: one): graph b's partials are
                            rows b*slab_rows .. b*slab_rows + slab_rows-1, summed with
                            the rest (dr_vanilla_fused_pass with split > 1)       */
} dr_param_table;

/* Sum the per-graph partials of a graph pass over the batch into every
 * parameter's gradient in a fixed order (deterministic, no float atomics),
 * optionally apply Adam (torch.optim.Adam semantics).  With slab == head ==
 * NULL the gradients are read from t->grad (e.g. after a data-parallel
 * all-reduce) and only Adam runs.  Also writes loss_scale * sum(loss_per_graph)
 * to loss_out[0] when both are non-NULL.                                    */
int dr_reduce_update(const dr_param_table* t, const float* slab, const float* head, int32_t n_batch,
                     const dr_adam* adam, const float* loss_per_graph, float loss_scale, float* loss_out,
                     void* stream);

/* ---- generic layer kernels (arbitrary edge lists; GINetConvLayer API) ---- */

/* Stable CSR of (row, col) pairs sorted by row: rowptr [n_rows+1], perm [E]
 * (edge ids in CSR order), col_sorted [E].  scratch: n_rows+1 int32.      */
int dr_csr_from_coo(const int64_t* row, const int64_t* col, int64_t n_edges, int32_t n_rows,
                    int32_t* rowptr, int32_t* perm, int32_t* col_sorted, int32_t* scratch,
                    void* stream);

/* out[i,:] = sum_{e in row i} y[col[e],:]  (C channels, fp32)  (ginet.py:58);
 * mode DR_SPMM_MEAN divides by the row length (foutnet.py:56-58: NaN on an
 * empty row, as torch.mean over an empty set); DR_SPMM_RELU applies relu.  */
#define DR_SPMM_RELU 1
#define DR_SPMM_MEAN 2
#define DR_SPMM_MEAN_CLAMP 4 /* divide by max(row length, 1): torch_scatter scatter_mean */
int dr_spmm_csr(const int32_t* rowptr, const int32_t* col, const float* y, int32_t n_rows,
                int32_t n_chan, int32_t mode, float* out, void* stream);
/* Weighted form: out[i,:] = sum_e w[e] y[col[e],:] (w in CSR order, NULL = 1);
 * SGraphAttentionLayer's a_ij-weighted scatter_mean (sgat.py:71-80).      */
int dr_spmm_csr_w(const int32_t* rowptr, const int32_t* col, const float* w, const float* y, int32_t n_rows,
                  int32_t n_chan, int32_t mode, float* out, void* stream);

/* y[M,N] = x[M,K] w[N,K]^T            */
int dr_linear_xwT(const float* x, const float* w, int32_t m, int32_t k, int32_t n, float* y, void* stream);
/* dx[M,K] = dy[M,N] w[N,K]            */
int dr_linear_xw(const float* dy, const float* w, int32_t m, int32_t n, int32_t k, float* dx, void* stream);
/* dw[N,K] = dy[M,N]^T x[M,K]  (deterministic split over M into scratch[n_split,N,K]) */
int dr_linear_dw(const float* dy, const float* x, int32_t m, int32_t n, int32_t k, float* dw,
                 float* scratch, int32_t n_split, void* stream);

/* VanillaConvolutionalLayer edge side (vanilla_gnn.py:29-35) on a CSR (int32,
 * by edge_index[0]), 32 message channels, A/B = X Wa^T / X Wb^T [n_rows, 32],
 * ea [E, Fe] in CSR slot order, wc = the edge-feature columns of the edge
 * MLP weight (row stride ld_we), be its bias:
 *   S[i,c] = sum_{e in row i} relu(A[i,c] + B[col e,c] + wc[c,:] ea_e + be[c]).  */
int dr_edge_mlp_scatter(const int32_t* rowptr, const int32_t* col, int32_t n_rows, const float* A, const float* B,
                        const float* ea, int32_t n_edge_feat, const float* wc, int32_t ld_we, const float* be,
                        float* S, void* stream);
/* Backward given DS = dL/dS: D (row sums of dpre), DP (dst sums of dpre, via
 * the transposed CSR trowptr/tcol and teid = transposed slot -> CSR slot) and
 * EAP [n_rows, 32, Fe] (per-row sums of dpre (x) ea).  Fe <= 8.               */
int dr_edge_mlp_scatter_bwd(const int32_t* rowptr, const int32_t* col, const int32_t* trowptr, const int32_t* tcol,
                            const int32_t* teid, int32_t n_rows, const float* A, const float* B, const float* ea,
                            int32_t n_edge_feat, const float* wc, int32_t ld_we, const float* be, const float* DS,
                            float* D, float* DP, float* EAP, void* stream);

/* Segment max / mean over member lists (segptr [n_seg+1], members [n_rows]:
 * the CSR of a cluster vector, members ascending in each segment), x/out
 * [*, n_chan] fp32.  mode 0 = torch_scatter.scatter_max (community_pooling.py
 * :209: NaN dropped, first max, empty -> 0 with arg = n_rows); mode 1 =
 * scatter_reduce amax as PyG max_pool_x (ginet.py:103, foutnet.py:111: NaN
 * propagates).  Backward: mode 0 routes dout to arg, mode 1 splits it over
 * the members equal to the max (plus one when the max is +-0: torch counts
 * its zero-initialised output as a tie).  dr_segment_mean: scatter_mean
 * (community_pooling.py:216, count clamped to 1).                          */
int dr_segment_max(const int32_t* segptr, const int32_t* members, const float* x, int32_t n_seg, int32_t n_chan,
                   int32_t n_rows, int32_t mode, float* out, int32_t* arg, void* stream);
int dr_segment_max_bwd(const int32_t* segptr, const int32_t* members, const float* x, const float* out,
                       const int32_t* arg, const float* dout, int32_t n_seg, int32_t n_chan, int32_t n_rows,
                       int32_t mode, float* dx, void* stream);
int dr_segment_mean(const int32_t* segptr, const int32_t* members, const float* x, int32_t n_seg, int32_t n_chan,
                    float* out, void* stream);

/* ---- host-side graph packer (deeprank2_amd/store.py) ----------------------
 * Per-graph arrays as GraphDataset.load_one_graph returns them
 * (dataset.py:883-1052) -> the packed store layout: stable CSR by
 * edge_index[0] and its transpose with slot maps, dense depth-0 ids + member
 * lists, the coalesced pooled graph of pool_edge (+ transpose), depth-1 member
 * lists (the collate of trainer.py:541 plus community_pooling.py:23-27,205-225
 * done once per graph).  Host memory only; threads over graphs.              */
typedef struct dr_pack_input {
  int32_t n_graphs, n_feat, n_edge_feat, require_clusters;
  const int64_t* node_off;   /* [G+1]                                          */
  const int64_t* edge_off;   /* [G+1]                                          */
  const int64_t* c1_off;     /* [G+1] offsets into cluster1                    */
  const int64_t* edge_index; /* [2, E_all] local ids: sources, then targets    */
  const float* edge_attr;    /* [E_all, Fe] or NULL                            */
  const int64_t* cluster0;   /* [N_all] or NULL                                */
  const int64_t* cluster1;   /* [c1_off[G]] or NULL                            */
} dr_pack_input;

typedef struct dr_pack_output {
  const int64_t *k0_off, *p1_off, *k1_off; /* [G+1] prefix sums of dr_pack_sizes' counts */
  int32_t *rowptr, *col, *eperm, *t_rowptr, *t_col, *t_eid; /* rowptr/t_rowptr [N_all+G], others [E_all] */
  int32_t *m0_ptr, *m0_idx, *cl0;         /* [K0_all+G], [N_all], [N_all]     */
  int32_t *p1_rowptr, *p1_col, *p1t_rowptr, *p1t_col; /* [K0_all+G], [P1_all]  */
  int32_t *m1_ptr, *m1_idx, *cl1;         /* [K1_all+G], [K0_all], [K0_all]   */
  float* edge_attr;                       /* [E_all, Fe] in CSR order, or NULL */
  float* p1_ea;                           /* [P1_all, Fe] pooled edge_attr (coalesced sums), or NULL */
  int32_t* p1t_pid;                       /* [P1_all] pooled transposed slot -> pooled CSR slot, or NULL */
} dr_pack_output;

/* Pass 1: per-graph K0, pooled-edge and K1 counts.  On invalid input returns
 * DR_E_ARG with a message in err.  threads <= 0: min(16, hardware threads). */
int dr_pack_sizes(const dr_pack_input* in, int64_t* k0_count, int64_t* p1_count, int64_t* k1_count,
                  int32_t threads, char* err, int32_t err_len);
/* Pass 2: fill the caller-allocated outputs; *symmetric = every graph's edge
 * multiset is symmetric (then the pooled transposes equal the pooled CSRs). */
int dr_pack_fill(const dr_pack_input* in, const dr_pack_output* out, int32_t* symmetric, int32_t threads);

/* ---- MCL community detection (community_pooling.py:96-162, as run by
 * Trainer._precluster, trainer.py:319-348; markov_clustering 0.0.6 defaults) --
 * One workgroup per graph, float64 like the reference.  All pointers in
 * dr_mcl_graphs are device pointers.                                          */
typedef struct dr_mcl_graphs {
  const int64_t* node_off; /* [G+1]                                             */
  const int32_t* rowptr;   /* local CSR, graph g's rows at node_off[g] + g      */
  const int64_t* edge_off; /* [G+1]                                             */
  const int32_t* col;      /* local columns, graph g's at edge_off[g]           */
  const double* weight;    /* edge weights at edge_off (symmetric, coalesced), or NULL = 1 */
  const int64_t* ws_off;   /* [G+1] workspace offsets in doubles (dr_mcl_workspace_doubles per graph) */
  double* ws;
  const int64_t* pat_off;  /* [G+1] offsets of each graph's N*N support pattern  */
  uint8_t* pattern;        /* converged support, row-major 0/1                   */
  int32_t* iters;          /* [G] iterations run, or NULL                        */
} dr_mcl_graphs;
int64_t dr_mcl_workspace_doubles(int32_t n_nodes);
int dr_mcl(const dr_mcl_graphs* graphs, int32_t n_graphs, int32_t max_iter, double pruning_threshold, void* stream);
/* Host: get_clusters + the reference's index assignment from the patterns
 * (host copies): cluster_out [N_all] at node_off, n_clusters [G] or NULL.  */
int dr_mcl_assign(const uint8_t* pattern, const int64_t* pat_off, const int64_t* node_off, int32_t n_graphs,
                  int32_t* cluster_out, int32_t* n_clusters);

/* Host-side replica of the in-kernel dropout RNG (DR_DROPOUT_HASH): writes
 * keep[i] for i in [0, n) (i = 128*b + r) into a host buffer.             */
int dr_dropout_mask(uint64_t seed, uint64_t offset, int32_t n, float p, uint8_t* keep_host);

/* Library / device info. */
const char* dr_version(void);
int dr_device_arch(char* buf, int32_t len); /* e.g. "gfx950"; 0 on success */

/* ------------------------------------------------------------------------
 * Debug: the LDS carve of a kernel family for given sizes, as text
 * "name=value;..." (region offsets in 4-byte words, "total" = words reserved,
 * "$name" = a layout parameter).  Host-only; tests/test_lds_carves.py checks
 * alignment, overlap, the host's reservation and each region's extent.
 * Returns the characters needed (buf may be shorter).  q = the carve's size
 * arguments in the order of its host-side *_lds_bytes function (fout: + sgat
 * flag + limit bytes; conv / tail variants: their own orders, see the tests).
 * ---------------------------------------------------------------------- */
int dr_debug_carve_ginet(const int32_t* q, char* buf, int32_t len);
int dr_debug_carve_ginet_conv(const int32_t* q, char* buf, int32_t len);
int dr_debug_carve_ginet_conv_bf16(const int32_t* q, char* buf, int32_t len);
int dr_debug_carve_ginet_tail(const int32_t* q, char* buf, int32_t len);
int dr_debug_carve_fout(const int32_t* q, char* buf, int32_t len);
int dr_debug_carve_fout_conv(const int32_t* q, char* buf, int32_t len);
int dr_debug_carve_fout_tail(const int32_t* q, char* buf, int32_t len);
int dr_debug_carve_nocluster(const int32_t* q, char* buf, int32_t len);
int dr_debug_carve_vanilla_graph(const int32_t* q, char* buf, int32_t len);
int dr_debug_carve_vanilla_tile(const int32_t* q, char* buf, int32_t len);
int dr_debug_carve_vanilla_chunk_fwd(const int32_t* q, char* buf, int32_t len);
int dr_debug_carve_vanilla_chunk_bwd(const int32_t* q, char* buf, int32_t len);

/* Debug: the tile each of n_blocks workgroups runs in the tile kernels
 * (large-graph GINet / FoutNet / SGAT / ginet_nocluster tiles, the Vanilla
 * chunk kernels): the XCD-contiguous order of graph_common.h xcd_tile_of.
 * Host-only; tests/test_lds_carves.py checks it is a permutation giving each
 * XCD group (block % 8) one contiguous range of tiles. */
int dr_debug_xcd_tile(int32_t n_blocks, int32_t* tiles);

#ifdef __cplusplus
}
#endif

#endif /* DEEPRANK2_AMD_H */
