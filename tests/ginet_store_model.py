"""TEST INFRASTRUCTURE: numpy model of the algorithm ``ginet_fused.hip`` runs.

It walks the packed store exactly as the kernel does (per graph: GEMM, CSR
aggregation, member-list pooling, pooled CSR, head, backward to per-graph
partials, reduction) so the algebra and the packing can be checked on the CPU
against the reference's golden vectors before any GPU time is spent.
"""

from __future__ import annotations

import numpy as np

LOWEST = np.float32(-3.402823466e38)


def relu(v):
    return np.where(v <= 0, np.float32(0), v)


def relu_bwd(out, g):
    return np.where(out <= 0, np.float32(0), g)


def run(packed, params, out_dim, *, mask=None, drop_scale=1.0, loss="mse", y=None, class_w=None, dout=None):  # noqa: PLR0915
    """Returns (out [B,out], grads dict by PARAM_NAMES index, loss)."""
    f32 = np.float32
    P = [np.asarray(p, f32) for p in params]
    w1cat = np.concatenate([P[0], P[6]], 0)  # [32,F]
    w2, w2e = P[3], P[9]
    fc1w, fc1b, fc2w, fc2b = P[12], P[13], P[14], P[15]
    B = packed.n_graphs
    F = packed.n_feat
    outs = np.zeros((B, out_dim), f32)
    slab = np.zeros((B, 32 * F + 1024), f32)
    heads = []
    lpg = np.zeros(B, f32)
    if y is None:
        y = packed.y
    for g in range(B):
        n0, n1 = packed.node_off[g], packed.node_off[g + 1]
        N = n1 - n0
        e0 = packed.edge_off[g]
        rp = packed.rowptr[n0 + g:n1 + g + 1]
        col = packed.col[e0 + rp[0]:e0 + rp[-1]]
        k0a, k0b = packed.k0_off[g], packed.k0_off[g + 1]
        K0 = k0b - k0a
        m0p = packed.m0_ptr[k0a + g:k0b + g + 1]
        m0i = packed.m0_idx[n0:n1]
        q0 = packed.p1_off[g]
        p1rp = packed.p1_rowptr[k0a + g:k0b + g + 1]
        p1c = packed.p1_col[q0:q0 + p1rp[-1]]
        p1trp = packed.p1t_rowptr[k0a + g:k0b + g + 1]
        p1tc = packed.p1t_col[q0:q0 + p1trp[-1]]
        k1a, k1b = packed.k1_off[g], packed.k1_off[g + 1]
        K1 = k1b - k1a
        m1p = packed.m1_ptr[k1a + g:k1b + g + 1]
        m1i = packed.m1_idx[k0a:k0b]
        X = packed.x[n0:n1]

        Z = np.zeros((N, F), f32)  # aggregate first: A (X W^T) == (A X) W^T
        for i in range(N):
            acc = np.zeros(F, f32)
            for e in range(rp[i], rp[i + 1]):
                acc = acc + X[col[e]]
            Z[i] = acc
        H = relu((Z @ w1cat.T).astype(f32))
        P1 = np.zeros((K0, 32), f32)
        A1 = np.full((K0, 32), N, np.int64)
        for k in range(K0):
            for c in range(32):
                best, arg = LOWEST, N
                for m in range(m0p[k], m0p[k + 1]):
                    v = H[m0i[m], c]
                    if v > best:
                        best, arg = v, m0i[m]
                P1[k, c] = 0 if best == LOWEST else best
                A1[k, c] = arg
        Y2 = np.concatenate([P1[:, :16] @ w2.T, P1[:, 16:] @ w2e.T], 1).astype(f32)
        H2 = np.zeros((K0, 64), f32)
        for k in range(K0):
            acc = np.zeros(64, f32)
            for e in range(p1rp[k], p1rp[k + 1]):
                acc = acc + Y2[p1c[e]]
            H2[k] = relu(acc)
        P2 = np.zeros((K1, 64), f32)
        NT = np.zeros((K1, 64), f32)
        for m in range(K1):
            mem = m1i[m1p[m]:m1p[m + 1]]
            vals = H2[mem]
            mx = np.where(np.isnan(vals).any(0), np.float32(np.nan), vals.max(0))
            P2[m] = mx
            NT[m] = (vals == mx).sum(0)
        G = (P2.sum(0) / f32(K1)).astype(f32)
        hpre = (fc1w @ G + fc1b).astype(f32)
        hh = relu(hpre)
        hd = hh if mask is None else (hh * mask[g] * f32(drop_scale)).astype(f32)
        o = (fc2w @ hd + fc2b).astype(f32)
        outs[g] = o
        if loss == "mse":
            d = o[0] - y[g]
            lpg[g] = d * d
            do = np.array([2 * d / B], f32)
        elif loss == "ce":
            yi = int(y[g])
            mx = o.max()
            lse = mx + np.log(np.exp(o - mx).sum())
            wy = 1.0 if class_w is None else class_w[yi]
            lpg[g] = wy * (lse - o[yi])
            denom = B if class_w is None else sum(class_w[int(v)] for v in y)
            do = (wy * (np.exp(o - lse) - np.eye(out_dim)[yi]) / denom).astype(f32)
        else:
            do = np.asarray(dout[g], f32)
        dhd = fc2w.T @ do
        if mask is not None:
            dhd = dhd * mask[g] * f32(drop_scale)
        dh = relu_bwd(hh, dhd).astype(f32)
        dG = (fc1w.T @ dh).astype(f32)
        heads.append((G, hd, dh, do))
        D2 = np.zeros((K0, 64), f32)
        for m in range(K1):
            gm = (dG / f32(K1)) / NT[m]
            for k in m1i[m1p[m]:m1p[m + 1]]:
                D2[k] = relu_bwd(H2[k], (H2[k] == P2[m]).astype(f32) * gm)
        dY2 = np.zeros((K0, 64), f32)
        for j in range(K0):
            for e in range(p1trp[j], p1trp[j + 1]):
                dY2[j] += D2[p1tc[e]]
        slab[g, 32 * F:32 * F + 512] = (dY2[:, :32].T @ P1[:, :16]).reshape(-1)
        slab[g, 32 * F + 512:] = (dY2[:, 32:].T @ P1[:, 16:]).reshape(-1)
        dP1 = np.concatenate([dY2[:, :32] @ w2, dY2[:, 32:] @ w2e], 1).astype(f32)
        dW1 = np.zeros((32, F), f32)  # dS1 is non-zero only at the depth-0 arg members
        for k in range(K0):
            for c in range(32):
                i = A1[k, c]
                if i < N:
                    dW1[c] += relu_bwd(H[i, c], dP1[k, c]) * Z[i]
        slab[g, :32 * F] = dW1.reshape(-1)

    grads = {}
    F32 = slab[:, :32 * F].sum(0).reshape(32, F)
    grads[0] = F32[:16]
    grads[6] = F32[16:]
    grads[3] = slab[:, 32 * F:32 * F + 512].sum(0).reshape(32, 16)
    grads[9] = slab[:, 32 * F + 512:].sum(0).reshape(32, 16)
    Gs = np.stack([h[0] for h in heads])
    HDs = np.stack([h[1] for h in heads])
    DHs = np.stack([h[2] for h in heads])
    DOs = np.stack([h[3] for h in heads])
    grads[12] = DHs.T @ Gs
    grads[13] = DHs.sum(0)
    grads[14] = DOs.T @ HDs
    grads[15] = DOs.sum(0)
    for i in (1, 2, 4, 5, 7, 8, 10, 11):
        grads[i] = np.zeros_like(P[i])
    if loss == "mse":
        lval = lpg.sum() / B
    elif loss == "ce":
        denom = B if class_w is None else sum(class_w[int(v)] for v in y)
        lval = lpg.sum() / denom
    else:
        lval = None
    return outs, grads, lval
