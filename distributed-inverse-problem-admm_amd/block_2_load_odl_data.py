"""Drop-in for /root/reference/block_2_load_odl_data.py (problem setup).

``load_odl_data`` returns the reference's dict keys (:256-271) with
``A_dense_list`` holding matrix-free ``RayTransform`` operators (the same
parallel-beam geometry as :34-83: every node spans [0, pi) with its share of
``max(180, 3N)`` angles) instead of dense ODL matrices, and sinograms
synthesised on the GPU: b_i = A_i x + noise_level * N(0,1) (:165-172).

Differences (documented): the default phantom is the modified Shepp-Logan
(the reference's ``randIm(N, seed=i)`` call at :155 is a TypeError); noise is
seeded (``seed + i``); no operator pickle is written; plots are not drawn
(visualisation is out of scope).
"""
from __future__ import annotations

import os
from datetime import datetime

import numpy as np
import torch

from admm_hip.data import make_sinograms, shepp_logan
from admm_hip.geometry import ParallelBeamGeometry, RayTransform
from admm_hip.solver import make_operators


def load_odl_data(N=128, num_nodes=5, noise_level=0.005, output_dir=None, make_plots=True,
                  show_plots=False, phantom_array=None, save_operators_dir=None, build_dense=False,
                  angles_total=None, dtype="float32", device=0, seed=1000):
    del make_plots, show_plots, save_operators_dir, build_dense
    ops = make_operators(N, num_nodes, angles_total, dtype=dtype, device=device)
    if phantom_array is None:
        phantoms = [shepp_logan(N).numpy()] * num_nodes
    elif isinstance(phantom_array, list):
        assert len(phantom_array) == num_nodes, "phantom_array list must have length num_nodes"
        phantoms = [np.asarray(p, dtype=np.float64) for p in phantom_array]
    else:
        phantoms = [np.asarray(phantom_array, dtype=np.float64)] * num_nodes
    sinos = []
    for i, A in enumerate(ops):
        s = make_sinograms([A], phantoms[i], noise_level, seed=seed + i)[0]
        sinos.append(s.to("cpu").numpy())
    W = [A.column_norms_sq(as_numpy=True) for A in ops]
    total = sum(A.geom.n_angles for A in ops)
    agg = RayTransform(ParallelBeamGeometry(N, total), dtype, device)
    if output_dir is None:
        output_dir = f"Recon_Op_ADMM_{datetime.now().strftime('%Y%m%d_%H%M%S')}"
    return {
        "A_dense_list": ops,
        "sinograms": sinos,
        "column_norms_all": [np.sqrt(w) for w in W],
        "N": N,
        "num_nodes": num_nodes,
        "agg_ray_trafo": agg,
        "A_agg": None,
        "agg_sinogram": np.vstack(sinos),
        "output_dir": output_dir,
        "phantom": phantoms[0],
        "phantoms": phantoms,
    }


load_data = load_odl_data
prepare_data = load_odl_data
