"""Per-pixel edge masks and the masked precision provider.

Replaces /root/reference/block_3_graph_and_precisions.py:154-187 (a networkx
loop over every pixel) with one HIP launch (admm_pixel_masks, csrc/masks.hip);
the random chains come from admm_chain_orders, a host replay of the numpy
PCG64 stream the reference draws from (``np.random.default_rng(seed)``,
:157), so chain masks match the reference bit for bit.

``keep`` is a device uint8 tensor [V, V, n] (the reference's bool keep[i, j, p]).
"""
from __future__ import annotations

import ctypes as C

import networkx as nx
import numpy as np
import torch

from . import _lib
from .geometry import current_stream_handle

STRATEGIES = {"knn": _lib.ADMM_MASK_KNN, "mst": _lib.ADMM_MASK_MST, "chain": _lib.ADMM_MASK_CHAIN}
Q_MODES = {"arithmetic": _lib.ADMM_Q_ARITHMETIC, "harmonic": _lib.ADMM_Q_HARMONIC}


def _stack_w(Wi_list, device) -> torch.Tensor:
    if device is None:
        from .geometry import default_device
        device = default_device()
    dev = torch.device("cuda", device)
    rows = [(w if isinstance(w, torch.Tensor) else torch.as_tensor(np.asarray(w))).reshape(-1)
            for w in Wi_list]
    return torch.stack([r.to(device=dev, dtype=torch.float64) for r in rows]).contiguous()


def chain_orders(V: int, n: int, seed: int = 0) -> np.ndarray:
    """[n, V] int32: the permutations rng.permutation(V) of block_3:139-140, pixel order."""
    st = np.random.default_rng(seed).bit_generator.state
    if st.get("bit_generator") != "PCG64":  # pragma: no cover - numpy default since 1.17
        raise RuntimeError("numpy default_rng is not PCG64")
    s, inc = int(st["state"]["state"]), int(st["state"]["inc"])
    m64 = (1 << 64) - 1
    pcg = (C.c_uint64 * 4)(s >> 64, s & m64, inc >> 64, inc & m64)
    out = np.empty((n, V), dtype=np.int32)
    lib = _lib.load()
    _lib.check(lib.admm_chain_orders(pcg, int(st["has_uint32"]), int(st["uinteger"]), V, n,
                                     out.ctypes.data_as(C.c_void_p), None), "admm_chain_orders")
    return out


def pixel_masks(Wi_list, strategy: str = "knn", k: int = 2, seed: int = 0,
                q_mode: str = "arithmetic", device: int | None = None) -> torch.Tensor:
    """keep[i, j, p] (uint8, device) of _build_all_pixel_masks (block_3:154-187)."""
    if strategy not in STRATEGIES:
        raise ValueError("strategy must be one of 'knn', 'mst', or 'chain'")
    if q_mode not in Q_MODES:
        raise ValueError("q_mode must be 'harmonic' or 'arithmetic'")
    V = len(Wi_list)
    if not 2 <= V <= _lib.MASK_MAX_NODES:
        raise ValueError(f"per-pixel masks support 2..{_lib.MASK_MAX_NODES} nodes, got {V}")
    W = _stack_w(Wi_list, device)
    n = W.shape[1]
    dev = W.device
    orders = None
    if strategy == "chain":
        orders = torch.from_numpy(chain_orders(V, n, seed)).to(dev)
    keep = torch.empty((V, V, n), dtype=torch.uint8, device=dev)
    lib = _lib.load()
    with torch.cuda.device(dev):
        _lib.check(lib.admm_pixel_masks(C.c_void_p(W.data_ptr()), V, n, STRATEGIES[strategy], int(k),
                                        Q_MODES[q_mode],
                                        C.c_void_p(orders.data_ptr() if orders is not None else 0),
                                        C.c_void_p(keep.data_ptr()), C.c_void_p(current_stream_handle(dev))),
                   "admm_pixel_masks")
    return keep


class MaskedQProvider:
    """Qij_diag_masked of block_3:312-317: q_ij where keep[i, j, :], else 0 (device tensors)."""

    def __init__(self, Wi_list, keep: torch.Tensor, q_mode: str = "arithmetic"):
        if q_mode not in Q_MODES:
            raise ValueError("q_mode must be 'harmonic' or 'arithmetic'")
        self.W = _stack_w(Wi_list, keep.device.index or 0)
        self.keep = keep
        self.q_mode = q_mode
        self.n = self.W.shape[1]

    def __call__(self, i, j):
        if i == j:
            return torch.zeros(self.n, dtype=torch.float64, device=self.W.device)
        wi, wj = self.W[i], self.W[j]
        q = (wi * wj) / (wi + wj) if self.q_mode == "harmonic" else 0.5 * (wi + wj)
        q = torch.clamp_min(q, 1e-12)
        return torch.where(self.keep[i, j].bool(), q, torch.zeros_like(q))

    def qslot_key(self, i, j):
        return ("masked", self.q_mode, min(i, j), max(i, j))


def union_graph(keep: torch.Tensor) -> nx.Graph:
    """Node graph with an edge wherever any pixel keeps it (block_3:196-205)."""
    V = keep.shape[0]
    any_ = keep.amax(dim=2).to("cpu").numpy()
    G = nx.Graph()
    G.add_nodes_from(range(V))
    for i in range(V):
        for j in range(i + 1, V):
            if any_[i, j]:
                G.add_edge(i, j)
    return G
