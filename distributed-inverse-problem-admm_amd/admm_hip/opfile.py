"""Operator hand-off files: the non-executable replacement of ``A_dense_list.pkl``.

The reference's setup block pickles the dense operator list into
``save_operators_dir/A_dense_list.pkl`` (/root/reference/block_2_load_odl_data.py:197-201)
and the precision block reads it back from ``base_dir`` (/root/reference/
block_3_graph_and_precisions.py:283-287); the drivers call the two with the same
directory (block_7_main_ver3.py:343,347,63).  Dense A is 51 GB at 512^2 and a pickle
executes code when loaded, so the hand-off here is a descriptor that rebuilds the
operators:

* a list of ``RayTransform`` -> ``<stem>.json``: the parallel-beam geometry of every
  node (N, angle count, detector width factor, angle range) and the sample dtype;
* a list of ``MatrixOperator`` -> ``<stem>.npz``: the matrices as CSR arrays
  (``A_{i}_indptr`` / ``_indices`` / ``_data`` / ``_shape``), read with
  ``allow_pickle=False``.

``<stem>`` is the pickle name without its extension (``A_dense_list``), so a block_3 call
that names ``A_dense_list.pkl`` finds ``A_dense_list.json`` / ``.npz`` next to it.
"""
from __future__ import annotations

import json
import os

import numpy as np

FORMAT = "admm_hip.operators/1"


def descriptor_paths(base_dir: str, name: str = "A_dense_list.pkl") -> tuple[str, str]:
    stem = os.path.splitext(name)[0]
    return os.path.join(base_dir, stem + ".json"), os.path.join(base_dir, stem + ".npz")


def save_operators(base_dir: str, ops, name: str = "A_dense_list.pkl") -> str:
    """Write the descriptor of ``ops`` (all RayTransforms or all MatrixOperators)."""
    from .geometry import RayTransform
    from .matrix import MatrixOperator
    os.makedirs(base_dir, exist_ok=True)
    jpath, zpath = descriptor_paths(base_dir, name)
    if all(isinstance(A, RayTransform) for A in ops):
        g = [A.geom for A in ops]
        doc = {"format": FORMAT, "kind": "ray_transform", "N": int(g[0].N),
               "n_angles": [int(x.n_angles) for x in g],
               "det_width_factor": [float(x.det_width_factor) for x in g],
               "angle_min": [float(x.angle_min) for x in g], "angle_max": [float(x.angle_max) for x in g],
               "dtype": [A.dtype for A in ops]}
        if any(x.N != g[0].N for x in g):
            raise ValueError("all nodes must have the same image size N")
        tmp = jpath + ".tmp"
        with open(tmp, "w") as f:
            json.dump(doc, f, indent=1)
        os.replace(tmp, jpath)
        return jpath
    if all(isinstance(A, MatrixOperator) for A in ops):
        arrs = {"format": np.array(FORMAT), "dtype": np.array([A.dtype for A in ops]),
                "N": np.array(ops[0].geom.N)}
        for i, A in enumerate(ops):
            gm = A.geom
            arrs[f"A_{i}_indptr"] = gm.indptr
            arrs[f"A_{i}_indices"] = gm.indices
            arrs[f"A_{i}_data"] = gm.values
            arrs[f"A_{i}_shape"] = np.array([gm.m, gm.n], dtype=np.int64)
        tmp = zpath + ".tmp.npz"
        np.savez(tmp, **arrs)
        os.replace(tmp, zpath)
        return zpath
    raise TypeError("save_operators takes a list of RayTransforms or of MatrixOperators")


def load_operators(base_dir: str, name: str = "A_dense_list.pkl", device: int | None = None):
    """Operators from the descriptor next to ``base_dir/name``, or None if there is none."""
    from .geometry import ParallelBeamGeometry, RayTransform
    from .matrix import MatrixGeometry, MatrixOperator
    jpath, zpath = descriptor_paths(base_dir, name)
    if os.path.exists(jpath):
        with open(jpath) as f:
            doc = json.load(f)
        if doc.get("format") != FORMAT or doc.get("kind") != "ray_transform":
            raise ValueError(f"{jpath}: not an {FORMAT} ray-transform descriptor")
        V = len(doc["n_angles"])
        return [RayTransform(ParallelBeamGeometry(int(doc["N"]), int(doc["n_angles"][i]),
                                                  float(doc["det_width_factor"][i]), float(doc["angle_min"][i]),
                                                  float(doc["angle_max"][i])), doc["dtype"][i], device)
                for i in range(V)]
    if os.path.exists(zpath):
        with np.load(zpath, allow_pickle=False) as z:
            if "format" not in z.files or str(z["format"]) != FORMAT:
                return None  # a plain matrix archive: matrix.load_matrix_list reads those
            N = int(z["N"])
            dts = [str(d) for d in z["dtype"]]
            geoms, ops = {}, []
            for i, dt in enumerate(dts):
                m, n = (int(v) for v in z[f"A_{i}_shape"])
                gm = MatrixGeometry(N, m, np.ascontiguousarray(z[f"A_{i}_indptr"], dtype=np.int64),
                                    np.ascontiguousarray(z[f"A_{i}_indices"], dtype=np.int32),
                                    np.ascontiguousarray(z[f"A_{i}_data"], dtype=np.float64))
                gm = geoms.setdefault(gm, gm)  # equal matrices share one geometry / context
                ops.append(MatrixOperator(geom=gm, dtype=dt, device=device))
            return ops
    return None
