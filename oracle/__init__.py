"""CPU oracle for the decentralized-ADMM tomography hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package
(``distributed-inverse-problem-admm_amd/``) imports, links or executes anything
under ``oracle/``.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` use it -- as the checker, never as the
thing that is measured or shipped.

What it is: a NumPy/SciPy (float64 by default) restatement of the reference
algorithm for the hot path named in BASELINE.json ``north_star``:

* ``geometry``   -- ODL parallel-beam geometry of
  ``/root/reference/block_2_load_odl_data.py:16-65`` (space [-1,1]^2, angles
  ``uniform_partition(0, pi, a)`` midpoints, detector
  ``uniform_partition(-1, 1, N)`` midpoints), discretised as a Joseph
  (ray-driven, linear interpolation) ray transform held as a sparse matrix.
  Dense-by-basis layout convention of ``Gen_Sino_Partitioned.py:140-145``:
  column j <-> C-order pixel ``unravel_index(j, (N, N))``, row <-> C-order
  (angle, detector bin).
* ``tv``         -- forward-difference gradient ``K`` / exact adjoint ``K^T``
  following ``block_4_tv_helpers.py:17-46`` (with the adjoint's boundary sign
  defect fixed), isotropic / anisotropic shrinkage.
* ``node_solver``-- the per-node x-update of ``block_5_node_problem.py:6-32``
  (objective eq.(1) of ADMM_Algo.pdf) solved by fixed-count split-Bregman
  with a CG inner solve -- the same iteration the HIP path runs.
* ``admm``       -- the outer loop of ``block_6_admm_loop_ver2.py:15-326``:
  neighbour gather, z midpoint, scaled dual update, residuals, stop test,
  identical history keys.  Also a literal dict-based restatement of the
  ``_ver2`` edge updates used to cross-check the single-y invariant form.
* ``precisions`` -- ``make_precisions`` of
  ``block_3_graph_and_precisions.py:11-43``.

Parity status: **parity unpinned** against the reference itself.  The
reference publishes no golden vectors, its fixture ``A_dense_list.pkl`` is not
in the repo, its numerics dependencies (odl, cvxpy, scs) are absent, and
executing the reference's modules in this container was refused by the
environment.  What *is* pinned: the projector geometry
against the analytic Radon transform of the Shepp-Logan ellipses (ODL's
parallel-beam convention), adjointness, the block-3 graph invariants, and the
``_ver2`` consensus algebra against its literal restatement.
"""
