"""Drop-in subset of /root/reference/block_3_graph_and_precisions.py.

``make_precisions(A_dense_list, q_mode)`` (:11-43): W_i[p] = max(||A_i[:,p]||^2,
1e-12) from the matrix-free HIP kernel, and the arithmetic / harmonic Q_ij
provider.  The per-pixel kNN / MST / chain masks (:62-319) are not yet ported.
"""
from __future__ import annotations

from admm_hip.data import make_precisions  # noqa: F401
