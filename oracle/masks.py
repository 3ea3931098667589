"""Oracle: per-pixel edge masks for masked precisions.  TEST INFRASTRUCTURE ONLY.

Restates /root/reference/block_3_graph_and_precisions.py:11-187 with numpy and
networkx (both importable here), pixel by pixel, for small n:

  * ``precisions``       -- make_precisions's W_i / Qij_diag (:11-43)
  * ``mask_knn``         -- _pixel_mask_knn_then_connect (:62-110)
  * ``mask_mst``         -- _pixel_mask_mst (:113-131)
  * ``mask_chain``       -- _pixel_mask_chain (:134-151)
  * ``build_all_masks``  -- _build_all_pixel_masks (:154-187), keep[i, j, p]
  * ``masked_q``         -- the Qij_diag_masked provider (:312-317)

The kNN step uses np.argpartition exactly as the reference does, so on tied
weights its choice is whatever this numpy build makes (see masks.hip).
"""
from __future__ import annotations

import networkx as nx
import numpy as np

EPS = 1e-12


def precisions(W_cols, q_mode="arithmetic"):
    """W_i = max(colsum_i, eps) given the column sums (block_3:20-23), and Qij_diag (:25-39)."""
    Wi = [np.maximum(np.asarray(w, dtype=np.float64), EPS) for w in W_cols]

    if q_mode == "harmonic":
        def q(i, j):
            return np.maximum((Wi[i] * Wi[j]) / (Wi[i] + Wi[j]), EPS)
    elif q_mode == "arithmetic":
        def q(i, j):
            return np.maximum(0.5 * (Wi[i] + Wi[j]), EPS)
    else:
        raise ValueError("q_mode must be 'harmonic' or 'arithmetic'")
    return Wi, q


def mask_knn(q_col, k, V):
    adj = np.zeros((V, V), dtype=bool)
    for i in range(V):
        cand = q_col[i, :].copy()
        cand[i] = -np.inf
        ke = min(k, V - 1)
        if ke > 0:
            adj[i, np.argpartition(cand, -ke)[-ke:]] = True
    adj = np.logical_or(adj, adj.T)
    G = nx.Graph()
    G.add_nodes_from(range(V))
    for i, j in np.argwhere(adj):
        if i < j:
            G.add_edge(int(i), int(j), weight=float(q_col[i, j]))
    if not nx.is_connected(G):
        T = nx.maximum_spanning_tree(_complete(q_col, V), weight="weight")
        for u, v, d in T.edges(data=True):
            G.add_edge(u, v, weight=d["weight"])
    return _to_mask(G, V)


def mask_mst(q_col, V):
    return _to_mask(nx.maximum_spanning_tree(_complete(q_col, V), weight="weight"), V)


def mask_chain(V, rng):
    order = rng.permutation(V)
    out = np.zeros((V, V), dtype=bool)
    for t in range(V - 1):
        out[order[t], order[t + 1]] = True
        out[order[t + 1], order[t]] = True
    return out


def build_all_masks(qfn, V, n, strategy="knn", k=2, seed=0):
    rng = np.random.default_rng(seed)
    q = np.zeros((V, V, n))
    for i in range(V):
        for j in range(V):
            if i != j:
                q[i, j, :] = qfn(i, j)
    keep = np.zeros((V, V, n), dtype=bool)
    for p in range(n):
        qs = 0.5 * (q[:, :, p] + q[:, :, p].T)
        np.fill_diagonal(qs, 0.0)
        if strategy == "knn":
            keep[:, :, p] = mask_knn(qs, k, V)
        elif strategy == "mst":
            keep[:, :, p] = mask_mst(qs, V)
        elif strategy == "chain":
            keep[:, :, p] = mask_chain(V, rng)
        else:
            raise ValueError("strategy must be one of 'knn', 'mst', or 'chain'")
    return np.logical_or(keep, np.transpose(keep, (1, 0, 2)))


def masked_q(qfn, keep, n):
    def Qm(i, j):
        if i == j:
            return np.zeros(n)
        return np.where(keep[i, j, :], qfn(i, j), 0.0)
    return Qm


def _complete(q_col, V):
    G = nx.Graph()
    G.add_nodes_from(range(V))
    for i in range(V):
        for j in range(i + 1, V):
            G.add_edge(i, j, weight=float(q_col[i, j]))
    return G


def _to_mask(G, V):
    out = np.zeros((V, V), dtype=bool)
    for u, v in G.edges():
        out[u, v] = True
        out[v, u] = True
    return out
