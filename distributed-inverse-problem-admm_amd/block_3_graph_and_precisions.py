"""Drop-in for /root/reference/block_3_graph_and_precisions.py.

* ``make_precisions(A_dense_list, q_mode)`` (:11-43): W_i[p] = max(||A_i[:,p]||^2,
  1e-12) from the matrix-free HIP kernel, and the arithmetic / harmonic Q_ij provider.
* ``build_pixel_connected_Q_provider(...)`` (:265-319): per-pixel kNN / MST / chain
  masks from one HIP launch (admm_hip.masks) and the masked Q_ij provider.

Deviation: the reference loads a pickled list of dense matrices from
``base_dir/A_dense_list_pickle`` (:283-287).  Pickles are not unpickled here: the operators
come from the descriptor ``load_odl_data`` writes into the same directory
(``A_dense_list.json`` next to the pickle name, admm_hip/opfile.py), from ``.npy`` /
``.npz`` matrix lists (``admm_hip.matrix.load_matrix_list``, allow_pickle=False) when
``A_dense_list_pickle`` names one, or from ``ops=`` / ``Wi_list=``.  Dense A is
infeasible past ~128^2.  ``keep`` comes back as a device uint8 tensor [V, V, n]
(the reference returns a numpy bool array).
"""
from __future__ import annotations

import os

import numpy as np

from admm_hip.data import make_precisions  # noqa: F401
from admm_hip.masks import MaskedQProvider, pixel_masks, union_graph


def build_pixel_connected_Q_provider(base_dir="saved_operators_Incmp_Span",
                                     A_dense_list_pickle="A_dense_list.pkl",
                                     strategy="knn", k=2, seed=0, q_mode="arithmetic",
                                     verbose=True, plot_union=True, show_plots=True,
                                     output_dir="pixel_graphs_out", *, ops=None, Wi_list=None,
                                     device=None):
    """Returns (G_union, Wi_list, Qij_diag_masked, keep) like block_3:265-319."""
    if Wi_list is None:
        if ops is None:
            ops = _load_ops(base_dir, A_dense_list_pickle, device)
            if verbose:
                print(f"[Block3] loaded A_dense_list from {base_dir}  nodes {len(ops)}")
        Wi_list, _ = make_precisions(ops, q_mode=q_mode)
    if device is None:
        from admm_hip.geometry import default_device
        device = ops[0].device if ops is not None else default_device()
    keep = pixel_masks(Wi_list, strategy=strategy, k=k, seed=seed, q_mode=q_mode, device=device)
    G_union = None
    if plot_union:
        tag = f"{strategy}_k{k}_{q_mode}" if strategy == "knn" else f"{strategy}_{q_mode}"
        G_union = _summarize_union(keep, output_dir, show_plots, verbose, tag)
    return G_union, Wi_list, MaskedQProvider(Wi_list, keep, q_mode), keep


def _load_ops(base_dir, name, device):
    """The operator list block_2 left in ``base_dir`` (block_3:283-287 reads the pickle):
    its descriptor (``A_dense_list.json`` / ``.npz`` next to ``A_dense_list.pkl``,
    admm_hip/opfile.py), or ``name`` itself when it is a ``.npy`` / ``.npz`` matrix list."""
    from admm_hip.opfile import load_operators
    path = os.path.join(base_dir, name)
    ops = load_operators(base_dir, name, device)
    if ops is not None:
        return ops
    if os.path.splitext(path)[1].lower() in (".npy", ".npz") and os.path.exists(path):
        from admm_hip.matrix import as_operators, load_matrix_list
        return as_operators(load_matrix_list(path), device=device)
    raise FileNotFoundError(
        f"no operators given: the reference reads {path} (pickled dense matrices, not unpickled "
        "here); run load_odl_data with this directory (it writes the operator descriptor), save "
        "the list as .npy / .npz, or pass ops= or Wi_list=")


def _summarize_union(keep, output_dir, show_plots, verbose, tag):
    """Union graph + the diagnostics block_3:190-260 prints and plots."""
    import networkx as nx
    G = union_graph(keep)
    degrees = np.array([d for _, d in G.degree()])
    active = float(keep.double().mean().item())
    if verbose:
        print(f"[Block3] strategy {tag}")
        print(f"[Block3] nodes {G.number_of_nodes()}, edges {G.number_of_edges()}")
        print(f"[Block3] connected {nx.is_connected(G)}")
        if degrees.size:
            print(f"[Block3] degree min mean max {degrees.min()}  {degrees.mean():.2f}  {degrees.max()}")
        print(f"[Block3] active pixel ratio {active:.4f}")
    try:
        import matplotlib
        if not show_plots:
            matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        os.makedirs(output_dir, exist_ok=True)
        plt.figure(figsize=(6, 6))
        nx.draw_networkx(G, pos=nx.spring_layout(G, seed=42), with_labels=True, node_size=600,
                         font_size=10)
        plt.tight_layout()
        plt.savefig(os.path.join(output_dir, f"pixel_union_graph_{tag}.png"), dpi=200)
        plt.show() if show_plots else plt.close()
        if degrees.size:
            plt.figure(figsize=(6, 4))
            plt.hist(degrees, bins=range(int(degrees.min()), int(degrees.max()) + 2))
            plt.xlabel("Degree")
            plt.ylabel("Count")
            plt.title(f"Node degree histogram, strategy {tag}")
            plt.tight_layout()
            plt.savefig(os.path.join(output_dir, f"pixel_union_degree_{tag}.png"), dpi=200)
            plt.show() if show_plots else plt.close()
    except Exception as exc:  # plotting is best-effort, as in the reference
        if verbose:
            print("[Block3] union graph plot failed:", repr(exc))
    return G
