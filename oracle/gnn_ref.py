"""TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Op-for-op torch-CPU restatement of the reference GNN hot path.  Parameter
names match the reference modules so ``state_dict``s are interchangeable with
the reference (``/root/reference/deeprank2/neuralnets/gnn/*.py``) and with the
MI355X product (``deeprank2_amd.neuralnets.gnn``).

Each step keeps the reference's operation order and degenerate semantics:
the singleton-dim softmax of the GINet attention (ginet.py:48-55), the in-place
per-graph cluster offsetting (community_pooling.py:23-27), the FoutNet
``mean(empty) = NaN`` rows (foutnet.py:55-58), torch_scatter's NaN-dropping
``scatter_max`` for community pooling (community_pooling.py:209) versus PyG's
NaN-propagating ``max_pool_x`` (ginet.py:103), and dropout placement
(ginet.py:122).
"""

from __future__ import annotations

import torch
from torch import nn
from torch.nn import functional as tf

from oracle import pyg_ops as P

# --------------------------------------------------------------------------
# community_pooling.py
# --------------------------------------------------------------------------


def offset_clusters_inplace(cluster: torch.Tensor, batch: torch.Tensor) -> torch.Tensor:
    """community_pooling.py:23-27: graph ib's ids are shifted by
    (max id of graph ib-1, already shifted) + 1, in place."""
    n_graphs = int(batch.max()) + 1
    for ib in range(1, n_graphs):
        prev_max = cluster[batch == ib - 1].max()
        cluster[batch == ib] += prev_max + 1
    return cluster


def pool_communities(cluster: torch.Tensor, data: P.Data) -> P.Batch:
    """community_pooling.py:165-242 for the attributes the path carries."""
    dense, perm = P.consecutive_cluster(cluster)
    x_pooled, _ = P.scatter_max(data.x, dense, dim=0)
    ei, ea = P.pool_edge(dense, data.edge_index, data.edge_attr)
    pos = P.scatter_mean(data.pos, dense, dim=0)
    out = P.Batch(batch=P.pool_batch(perm, data.batch), x=x_pooled, edge_index=ei, edge_attr=ea, pos=pos)
    out.cluster0 = data.cluster0
    out.cluster1 = data.cluster1
    return out


# --------------------------------------------------------------------------
# ginet.py
# --------------------------------------------------------------------------


class GINetConvLayer(nn.Module):
    """ginet.py:13-63.  Same parameters: fc [out,in], fc_edge_attr [Fe,Fe],
    fc_attention [1, 2*out+Fe]; U(±1/sqrt(in)) init for all three."""

    def __init__(self, in_channels, out_channels, number_edge_features=1, bias=False):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.fc = nn.Linear(in_channels, out_channels, bias=bias)
        self.fc_edge_attr = nn.Linear(number_edge_features, number_edge_features, bias=bias)
        self.fc_attention = nn.Linear(2 * out_channels + number_edge_features, 1, bias=bias)
        for lin in (self.fc, self.fc_attention, self.fc_edge_attr):
            P.uniform(in_channels, lin.weight)

    def forward(self, x, edge_index, edge_attr):
        src_side, dst_side = edge_index[0], edge_index[1]
        if edge_attr.dim() == 1:
            edge_attr = edge_attr.unsqueeze(-1)
        h_col = self.fc(x[dst_side])
        h_row = self.fc(x[src_side])
        e = self.fc_edge_attr(edge_attr)
        logit = tf.leaky_relu(self.fc_attention(torch.cat([h_row, h_col, e], dim=1)))
        att = tf.softmax(logit, dim=1)  # [E,1]: identically 1 for finite logits
        acc = torch.zeros(x.shape[0], self.out_channels).to(att.device)
        return P.scatter_sum(att * h_col, src_side, dim=0, out=acc)


class GINet(nn.Module):
    """ginet.py:66-125."""

    def __init__(self, input_shape, output_shape=1, input_shape_edge=1):
        super().__init__()
        self.conv1 = GINetConvLayer(input_shape, 16, input_shape_edge)
        self.conv2 = GINetConvLayer(16, 32, input_shape_edge)
        self.conv1_ext = GINetConvLayer(input_shape, 16, input_shape_edge)
        self.conv2_ext = GINetConvLayer(16, 32, input_shape_edge)
        self.fc1 = nn.Linear(64, 128)
        self.fc2 = nn.Linear(128, output_shape)
        self.clustering = "mcl"
        self.dropout = 0.4
        self.dropout_fn = tf.dropout  # tests swap in a fixed-mask dropout

    def _branch(self, data, conv_a, conv_b):
        data.x = tf.relu(conv_a(data.x, data.edge_index, data.edge_attr))
        data = pool_communities(offset_clusters_inplace(data.cluster0, data.batch), data)
        data.x = tf.relu(conv_b(data.x, data.edge_index, data.edge_attr))
        c1 = offset_clusters_inplace(data.cluster1, data.batch)
        return P.max_pool_x(c1, data.x, data.batch)

    def forward(self, data):
        twin = data.clone()
        x, b = self._branch(data, self.conv1, self.conv2)
        x_ext, b_ext = self._branch(twin, self.conv1_ext, self.conv2_ext)
        h = torch.cat([P.scatter_mean(x, b, dim=0), P.scatter_mean(x_ext, b_ext, dim=0)], dim=1)
        h = tf.relu(self.fc1(h))
        h = self.dropout_fn(h, self.dropout, training=self.training)
        return self.fc2(h)


# --------------------------------------------------------------------------
# foutnet.py
# --------------------------------------------------------------------------


class FoutLayer(nn.Module):
    """foutnet.py:13-69: ``x·Wc + mean_{j:(i→j)} x_j·Wn + b`` (W stored [in,out])."""

    def __init__(self, in_channels, out_channels, bias=True):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.wc = nn.Parameter(torch.empty(in_channels, out_channels))
        self.wn = nn.Parameter(torch.empty(in_channels, out_channels))
        if bias:
            self.bias = nn.Parameter(torch.empty(out_channels))
        else:
            self.register_parameter("bias", None)
        for p in (self.wc, self.wn, self.bias):
            P.uniform(in_channels, p)

    def forward(self, x, edge_index):
        centre = torch.mm(x, self.wc)
        neigh = torch.mm(x, self.wn)
        gamma = torch.zeros(x.shape[0], self.out_channels).to(centre.device)
        for n in range(x.shape[0]):  # foutnet.py:56-58, kept as the per-node loop
            nbrs = edge_index[1, edge_index[0] == n]
            gamma[n, :] = torch.mean(neigh[nbrs, :], dim=0)
        out = centre + gamma
        if self.bias is not None:
            out = out + self.bias
        return out


def fout_rowmean_vectorised(x, edge_index, wc, wn, bias):
    """Same value as FoutLayer.forward without the O(N·E) loop (used to time a
    fair CPU baseline; NaN where a node has no out-edge, as ``mean(empty)``)."""
    centre = x @ wc
    neigh = x @ wn
    n = x.shape[0]
    s = torch.zeros(n, neigh.shape[1]).index_add_(0, edge_index[0], neigh[edge_index[1]])
    cnt = torch.zeros(n).index_add_(0, edge_index[0], torch.ones(edge_index.shape[1]))
    gamma = s / cnt.unsqueeze(1)  # 0/0 = NaN for isolated rows
    out = centre + gamma
    return out if bias is None else out + bias


class FoutNet(nn.Module):
    """foutnet.py:72-118 (``input_shape_edge`` is accepted and ignored)."""

    def __init__(self, input_shape, output_shape=1, input_shape_edge=None):  # noqa: ARG002
        super().__init__()
        self.conv1 = FoutLayer(input_shape, 16)
        self.conv2 = FoutLayer(16, 32)
        self.fc1 = nn.Linear(32, 64)
        self.fc2 = nn.Linear(64, output_shape)
        self.clustering = "mcl"

    def forward(self, data):
        data.x = tf.relu(self.conv1(data.x, data.edge_index))
        data = pool_communities(offset_clusters_inplace(data.cluster0, data.batch), data)
        data.x = tf.relu(self.conv2(data.x, data.edge_index))
        x, b = P.max_pool_x(offset_clusters_inplace(data.cluster1, data.batch), data.x, data.batch)
        h = P.scatter_mean(x, b, dim=0)
        return self.fc2(tf.relu(self.fc1(h)))


# --------------------------------------------------------------------------
# vanilla_gnn.py
# --------------------------------------------------------------------------


class VanillaConvolutionalLayer(nn.Module):
    """vanilla_gnn.py:10-38."""

    def __init__(self, count_node_features, count_edge_features):
        super().__init__()
        msg = 32
        self._edge_mlp = nn.Sequential(nn.Linear(2 * count_node_features + count_edge_features, msg), nn.ReLU())
        self._node_mlp = nn.Sequential(nn.Linear(count_node_features + msg, count_node_features), nn.ReLU())

    def forward(self, node_features, edge_node_indices, edge_features):
        a, b = edge_node_indices
        m = self._edge_mlp(torch.cat([node_features[a], node_features[b], edge_features], dim=1))
        acc = torch.zeros(node_features.shape[0], m.shape[1]).to(node_features.device)
        s = P.scatter_sum(m, a, dim=0, out=acc)
        return self._node_mlp(torch.cat([node_features, s], dim=1))


class VanillaNetwork(nn.Module):
    """vanilla_gnn.py:41-65."""

    def __init__(self, input_shape, output_shape, input_shape_edge):
        super().__init__()
        self._external1 = VanillaConvolutionalLayer(input_shape, input_shape_edge)
        self._external2 = VanillaConvolutionalLayer(input_shape, input_shape_edge)
        self._graph_mlp = nn.Sequential(nn.Linear(input_shape, 128), nn.ReLU(), nn.Linear(128, output_shape))

    def forward(self, data):
        h = self._external1(data.x, data.edge_index, data.edge_attr)
        h = self._external2(h, data.edge_index, data.edge_attr)
        return self._graph_mlp(P.scatter_mean(h, data.batch, dim=0))


# --------------------------------------------------------------------------
# sgat.py
# --------------------------------------------------------------------------


class SGraphAttentionLayer(nn.Module):
    """sgat.py:13-84: ``z_i = mean_{e=(i->j)} a_e [x_i | x_j] W + b``
    (torch_scatter ``scatter_mean`` into a zero ``out``: count clamped to 1);
    ``undirected=False`` adds a second ``scatter_mean`` over ``col`` into the
    same ``out`` (which also divides the first result by the col counts)."""

    def __init__(self, in_channels, out_channels, bias=True, undirected=True):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.undirected = undirected
        self.weight = nn.Parameter(torch.empty(2 * in_channels, out_channels))
        if bias:
            self.bias = nn.Parameter(torch.empty(out_channels))
        else:
            self.register_parameter("bias", None)
        P.uniform(2 * in_channels, self.weight)
        P.uniform(2 * in_channels, self.bias)

    def forward(self, x, edge_index, edge_attr):
        row, col = edge_index
        if edge_attr.dim() == 1:
            edge_attr = edge_attr.unsqueeze(-1)
        alpha = edge_attr * torch.mm(torch.cat([x[row], x[col]], dim=-1), self.weight)
        out = torch.zeros(len(x), self.out_channels)
        out = P.scatter_mean(alpha, row, dim=0, out=out)
        if not self.undirected:
            out = P.scatter_mean(alpha, col, dim=0, out=out)
        if self.bias is not None:
            out = out + self.bias
        return out


class SGAT(nn.Module):
    """sgat.py:87-133: conv1 / community pooling (edge_attr summed by
    ``pool_edge``) / conv2 on the pooled graph / max_pool_x / mean / fc1 / fc2."""

    def __init__(self, input_shape, output_shape=1, input_shape_edge=None):  # noqa: ARG002
        super().__init__()
        self.conv1 = SGraphAttentionLayer(input_shape, 16)
        self.conv2 = SGraphAttentionLayer(16, 32)
        self.fc1 = nn.Linear(32, 64)
        self.fc2 = nn.Linear(64, output_shape)
        self.clustering = "mcl"

    def forward(self, data):
        data.x = tf.relu(self.conv1(data.x, data.edge_index, data.edge_attr))
        data = pool_communities(offset_clusters_inplace(data.cluster0, data.batch), data)
        data.x = tf.relu(self.conv2(data.x, data.edge_index, data.edge_attr))
        x, b = P.max_pool_x(offset_clusters_inplace(data.cluster1, data.batch), data.x, data.batch)
        h = P.scatter_mean(x, b, dim=0)
        return self.fc2(tf.relu(self.fc1(h)))


# --------------------------------------------------------------------------
# ginet_nocluster.py
# --------------------------------------------------------------------------


class GINetNoCluster(nn.Module):
    """ginet_nocluster.py:66-111: two GINet conv branches (same layers as
    ginet.py) on the full graph, no pooling; per-graph mean, fc1, dropout, fc2."""

    def __init__(self, input_shape, output_shape=1, input_shape_edge=1):
        super().__init__()
        self.conv1 = GINetConvLayer(input_shape, 16, input_shape_edge)
        self.conv2 = GINetConvLayer(16, 32, input_shape_edge)
        self.conv1_ext = GINetConvLayer(input_shape, 16, input_shape_edge)
        self.conv2_ext = GINetConvLayer(16, 32, input_shape_edge)
        self.fc1 = nn.Linear(64, 128)
        self.fc2 = nn.Linear(128, output_shape)
        self.dropout = 0.4
        self.dropout_fn = tf.dropout

    def forward(self, data):
        twin = data.clone()
        h = tf.relu(self.conv2(tf.relu(self.conv1(data.x, data.edge_index, data.edge_attr)), data.edge_index, data.edge_attr))
        he = tf.relu(self.conv2_ext(tf.relu(self.conv1_ext(twin.x, twin.edge_index, twin.edge_attr)), twin.edge_index, twin.edge_attr))
        g = torch.cat([P.scatter_mean(h, data.batch, dim=0), P.scatter_mean(he, twin.batch, dim=0)], dim=1)
        g = self.dropout_fn(tf.relu(self.fc1(g)), self.dropout, training=self.training)
        return self.fc2(g)


MODELS = {"GINet": GINet, "FoutNet": FoutNet, "VanillaNetwork": VanillaNetwork, "SGAT": SGAT, "GINetNoCluster": GINetNoCluster}
