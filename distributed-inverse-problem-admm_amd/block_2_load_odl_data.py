"""Drop-in for /root/reference/block_2_load_odl_data.py (problem setup).

``load_odl_data`` returns the reference's dict keys (:239-253) with the operators
matrix-free:

* ``A_dense_list`` -- one ``RayTransform`` per node (the parallel-beam geometry of
  :16-65: every node spans [0, pi) with its share of ``max(180, 3N)`` angles, :31-38)
  instead of dense ODL matrices (:160-165);
* ``sinograms``   -- b_i = A_i x_i + noise_level * N(0,1) (:148-154), synthesised on the
  GPU in the operators' dtype (float32 like ODL's float32 space, :23-28);
* ``agg_ray_trafo`` / ``A_agg`` -- the aggregate transform over all ``angles_total``
  angles (:58-63); ``A_agg`` is that operator (the reference's dense aggregate matrix,
  :167) when ``build_dense`` else None, as in the reference;
* ``agg_sinogram`` -- with ``build_dense`` (the reference default):
  A_agg phantom_0 + noise_level * N(0,1), shape (angles_total, N) (:169-177); without:
  the stacked per-node sinograms (:159);
* ``column_norms_all`` -- ||A_i[:, p]||_2 per pixel (:181-189), from the HIP column-norm
  kernel (W_i = max(sum_r A_i[r,p]^2, 1e-12), so an uncovered pixel reads 1e-6, not 0);
* ``phantom`` / ``phantoms`` -- float32 arrays (ODL's float32 space elements, :145, :250-252).

Operators land on ``device`` (default: the current HIP device, so a rank that called
``torch.cuda.set_device(local_rank)`` builds on its own GPU).

Differences (documented): the default phantom is the modified Shepp-Logan (the
reference's ``randIm(N, seed=i)`` call at :137 is a TypeError, SURVEY.md 8 defects);
noise is seeded (node i: ``seed + i``, aggregate: ``seed + num_nodes``); no operator
pickle is written (:197-201); plots are not drawn (visualisation is out of scope).
"""
from __future__ import annotations

import os
from datetime import datetime

import numpy as np
import torch

from admm_hip.data import make_sinograms, shepp_logan
from admm_hip.geometry import ParallelBeamGeometry, RayTransform, default_device
from admm_hip.solver import make_operators


def load_odl_data(N=128, num_nodes=5, noise_level=0.005, output_dir=None, make_plots=True,
                  show_plots=False, phantom_array=None, save_operators_dir=None, build_dense=True,
                  angles_total=None, dtype="float32", device=None, seed=1000):
    del make_plots, show_plots, save_operators_dir
    if device is None:
        device = default_device()
    ops = make_operators(N, num_nodes, angles_total, dtype=dtype, device=device)
    if phantom_array is None:
        phantoms = [shepp_logan(N).numpy().astype(np.float32)] * num_nodes
    elif isinstance(phantom_array, list):
        assert len(phantom_array) == num_nodes, "phantom_array list must have length num_nodes"
        phantoms = [np.asarray(p, dtype=np.float32) for p in phantom_array]
    else:
        phantoms = [np.asarray(phantom_array, dtype=np.float32)] * num_nodes
    sinos = []
    for i, A in enumerate(ops):
        s = make_sinograms([A], phantoms[i], noise_level, seed=seed + i)[0]
        sinos.append(s.to("cpu").numpy())
    W = [A.column_norms_sq(as_numpy=True) for A in ops]
    total = sum(A.geom.n_angles for A in ops)
    agg = RayTransform(ParallelBeamGeometry(N, total), dtype, device)
    if build_dense:
        agg_sino = make_sinograms([agg], phantoms[0], noise_level, seed=seed + num_nodes)[0]
        agg_sinogram = agg_sino.to("cpu").numpy()
    else:
        agg_sinogram = np.vstack(sinos)
    if output_dir is None:
        output_dir = f"Recon_Op_ADMM_{datetime.now().strftime('%Y%m%d_%H%M%S')}"
    os.makedirs(output_dir, exist_ok=True)  # :191-195
    return {
        "A_dense_list": ops,
        "sinograms": sinos,
        "column_norms_all": [np.sqrt(w) for w in W],
        "N": N,
        "num_nodes": num_nodes,
        "agg_ray_trafo": agg,
        "A_agg": agg if build_dense else None,
        "agg_sinogram": agg_sinogram,
        "output_dir": output_dir,
        "phantom": phantoms[0],
        "phantoms": phantoms,
    }


load_data = load_odl_data
prepare_data = load_odl_data
