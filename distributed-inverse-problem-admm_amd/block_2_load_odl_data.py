"""Drop-in for /root/reference/block_2_load_odl_data.py (problem setup)
and for the legacy loader of the same name in /root/reference/block_2_test.py:15-167, which
the ``block_7_main_ver0..3`` drivers call with ``base_dir=`` (block_7_main_ver3.py:347).

``load_odl_data`` returns the reference's dict keys (:239-253, plus the legacy
``agg_fbp_recon`` / ``agg_ls_recon``, block_2_test.py:154-167) with the operators
matrix-free:

* ``A_dense_list`` -- one ``RayTransform`` per node (the parallel-beam geometry of
  :16-65: every node spans [0, pi) with its share of ``max(180, 3N)`` angles, :31-38;
  the remainder goes to the first nodes, so counts may differ by one) instead of dense ODL
  matrices (:160-165);
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
* ``phantom`` / ``phantoms`` -- float32 arrays (ODL's float32 space elements, :145, :250-252);
* ``agg_ls_recon`` -- the legacy loader's ridge least squares on the aggregate operator,
  (A_agg^T A_agg + 1e-3 I)^{-1} A_agg^T agg_sinogram as an (N, N) array
  (block_2_test.py:83-88), solved by CG on the GPU (admm_hip.data.ridge_ls); computed when
  the call uses the legacy surface (``base_dir=``) or ``agg_ls=True``, else None;
  ``agg_fbp_recon`` -- None, as the legacy loader leaves it (:77).

Operator hand-off (block_2 -> block_3).  With ``build_dense`` the reference pickles the
dense list into ``save_operators_dir/A_dense_list.pkl`` (:197-201) and block_3 reads it
from its ``base_dir`` (block_3_graph_and_precisions.py:283-287).  Here the same call writes
``save_operators_dir/A_dense_list.json``, a non-executable descriptor of the geometries
(admm_hip/opfile.py), which the block_3 drop-in rebuilds the operators from.  The legacy
surface reads its operators from ``base_dir`` (block_2_test.py:28-31): if a descriptor is
there it is used (its node count must equal ``num_nodes``, :44-45), otherwise the operators
are built and the descriptor is written to ``base_dir``, so ``block_7_main_ver3``'s call
sequence (:347, :63-72, :88-106) runs unchanged.

Operators land on ``device`` (default: the current HIP device, so a rank that called
``torch.cuda.set_device(local_rank)`` builds on its own GPU).

Differences (documented): the default phantom is the modified Shepp-Logan (the
reference's ``randIm(N, seed=i)`` call at :137 is a TypeError, SURVEY.md 8 defects);
noise is seeded (node i: ``seed + i``, aggregate: ``seed + num_nodes``); no pickle is
written or read; plots are not drawn (visualisation is out of scope).
"""
from __future__ import annotations

import os
from datetime import datetime

import numpy as np

from admm_hip.data import make_sinograms, ridge_ls, shepp_logan
from admm_hip.geometry import ParallelBeamGeometry, RayTransform, default_device
from admm_hip.opfile import load_operators, save_operators
from admm_hip.solver import make_operators

_UNSET = object()


def load_odl_data(N=128, num_nodes=5, noise_level=0.005, output_dir=None, make_plots=True,
                  show_plots=False, phantom_array=None, save_operators_dir=_UNSET, build_dense=True,
                  angles_total=None, dtype="float32", device=None, seed=1000, *, base_dir=None,
                  ray_transforms_pickle="ray_transforms.pkl", A_dense_list_pickle="A_dense_list.pkl",
                  agg_op_pickle="aggregate_op.pkl", A_agg_pickle="A_agg.pkl", agg_ls=None,
                  ls_max_iters=2000):
    """block_2_load_odl_data.py:99-253 (and block_2_test.py:15-167 when ``base_dir`` is given)."""
    del make_plots, show_plots, ray_transforms_pickle, agg_op_pickle, A_agg_pickle
    if device is None:
        device = default_device()
    legacy = base_dir is not None
    ops = None
    if legacy:
        ops = load_operators(base_dir, A_dense_list_pickle, device)
        if ops is not None:
            assert len(ops) == num_nodes, (  # block_2_test.py:44-45
                f"{base_dir}: descriptor holds {len(ops)} operators, num_nodes={num_nodes}")
            if any(A.geom.N != N for A in ops):
                raise ValueError(f"{base_dir}: descriptor operators are not {N} x {N}")
    if ops is None:
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
    agg = RayTransform(ParallelBeamGeometry(N, total), ops[0].dtype, device)
    if build_dense:
        agg_sino = make_sinograms([agg], phantoms[0], noise_level, seed=seed + num_nodes)[0]
        agg_sinogram = agg_sino.to("cpu").numpy()
    else:
        agg_sinogram = np.vstack(sinos)
    if output_dir is None:
        output_dir = f"Recon_Op_ADMM_{datetime.now().strftime('%Y%m%d_%H%M%S')}"
    os.makedirs(output_dir, exist_ok=True)  # :191-195
    # operator hand-off for block_3 (:197-201; the legacy surface keeps it in base_dir)
    if save_operators_dir is _UNSET:
        save_operators_dir = base_dir if legacy else "saved_operators_Incmp_Span"
    if build_dense and save_operators_dir is not None:
        save_operators(save_operators_dir, ops, A_dense_list_pickle)
    ls = None
    if agg_ls or (agg_ls is None and legacy):
        x_ls, _, _ = ridge_ls(agg, agg_sinogram, 1e-3, max_iters=ls_max_iters)
        ls = x_ls.to("cpu").numpy().reshape(N, N)
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
        "agg_fbp_recon": None,
        "agg_ls_recon": ls,
        "A_dense_list_path": (os.path.join(save_operators_dir, os.path.splitext(A_dense_list_pickle)[0] + ".json")
                              if build_dense and save_operators_dir is not None else None),
    }


load_data = load_odl_data
prepare_data = load_odl_data
