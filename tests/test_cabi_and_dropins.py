"""CPU: the C-ABI library loads and exports every symbol include/admm_tomo.h
declares; the ctypes mirrors have the C layout; the drop-in modules expose the
reference's call surface (no GPU needed, no compute calls)."""
import ctypes as C
import inspect
import os
import re
import subprocess

import pytest

from admm_hip import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "admm_tomo.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(admm_\w+)\(", src, flags=re.M)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    names = declared_functions()
    assert len(names) >= 14
    for name in names:
        assert hasattr(lib, name), name
        assert name in _lib.SYMBOLS, f"{name} not bound in _lib.SYMBOLS"
    assert set(_lib.SYMBOLS) == set(names)
    assert lib.admm_abi_version() == _lib.ABI_VERSION == 9


def test_error_path_without_gpu_work():
    lib = _lib.load()
    # null arguments are rejected before any HIP call
    rc = lib.admm_ctx_create(None, None, 0, 1, 0)
    assert rc == -1 and b"null" in lib.admm_last_error()
    assert lib.admm_node_update(None, None) == -3
    with pytest.raises(_lib.AdmmError):
        _lib.check(lib.admm_consensus(None, None), "admm_consensus")


def test_struct_layout_matches_c(tmp_path):
    probe = tmp_path / "probe.c"
    fields_g = [f for f, _ in _lib.Geom._fields_]
    fields_b = [f for f, _ in _lib.Batch._fields_]
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    lines.append('printf("geom %zu\\n", sizeof(admm_geom));')
    for f in fields_g:
        lines.append(f'printf("g.{f} %zu\\n", offsetof(admm_geom, {f}));')
    lines.append('printf("batch %zu\\n", sizeof(admm_batch));')
    for f in fields_b:
        lines.append(f'printf("b.{f} %zu\\n", offsetof(admm_batch, {f}));')
    lines.append("return 0;}")
    probe.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c99", "-o", str(exe), str(probe)], check=True)
    out = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                  check=True).stdout.splitlines())
    assert int(out["geom"]) == C.sizeof(_lib.Geom)
    assert int(out["batch"]) == C.sizeof(_lib.Batch)
    for f in fields_g:
        assert int(out[f"g.{f}"]) == getattr(_lib.Geom, f).offset, f
    for f in fields_b:
        assert int(out[f"b.{f}"]) == getattr(_lib.Batch, f).offset, f


# reference call surfaces (parameter names in order), cited per module
REF_SIGNATURES = {
    # /root/reference/block_5_node_problem.py:6
    ("block_5_node_problem", "build_node_problem"): ["Ai", "bi", "rho", "neighbor_terms", "N", "lam_tv",
                                                     "Qij_terms"],
    # /root/reference/block_6_admm_loop_ver2.py:15-20
    ("block_6_admm_loop_ver2", "decentralized_admm"): [
        "A_dense_list", "sinograms", "G", "Wi_list", "Qij_diag_fn", "N", "lam_tv", "rho", "max_iters",
        "max_inner_iters", "eps_pri", "eps_dual", "verbose", "snapshot_dir", "snapshot_every",
        "snapshot_div", "phantom_true"],
    # /root/reference/block_6_admm_loop.py:72-84
    ("block_6_admm_loop", "decentralized_admm"): [
        "A_dense_list", "sinograms", "G", "Wi_list", "Qij_diag_fn", "N", "lam_tv", "rho", "max_iters",
        "eps_pri", "eps_dual", "verbose", "scs_total_iters", "scs_chunk_iters", "scs_snapshot_dir",
        "scs_use_indirect", "scs_eps", "scs_alpha", "scs_acceleration", "scs_lookback", "scs_scale",
        "scs_save_every_chunks"],
    # /root/reference/block_2_load_odl_data.py:99-109
    ("block_2_load_odl_data", "load_odl_data"): [
        "N", "num_nodes", "noise_level", "output_dir", "make_plots", "show_plots", "phantom_array",
        "save_operators_dir", "build_dense"],
    # /root/reference/block_3_graph_and_precisions.py:11
    ("block_3_graph_and_precisions", "make_precisions"): ["ops", "q_mode"],
    # /root/reference/block_3_graph_and_precisions.py:265-274
    ("block_3_graph_and_precisions", "build_pixel_connected_Q_provider"): [
        "base_dir", "A_dense_list_pickle", "strategy", "k", "seed", "q_mode", "verbose", "plot_union",
        "show_plots", "output_dir"],
}
REF_DEFAULTS = {
    ("block_6_admm_loop_ver2", "decentralized_admm"): dict(lam_tv=0.01, rho=1.0, max_iters=10,
                                                           max_inner_iters=100, eps_pri=1e-1,
                                                           eps_dual=1e-1, verbose=True, snapshot_div=10),
    ("block_6_admm_loop", "decentralized_admm"): dict(lam_tv=0.01, rho=1.0, max_iters=200, eps_pri=1e-3,
                                                      eps_dual=1e-3, scs_total_iters=100),
    # /root/reference/block_2_load_odl_data.py:99-109
    ("block_2_load_odl_data", "load_odl_data"): dict(N=128, num_nodes=5, noise_level=0.005,
                                                     build_dense=True),
}


@pytest.mark.parametrize("key", list(REF_SIGNATURES))
def test_dropin_signatures(key):
    import importlib
    mod = importlib.import_module(key[0])
    fn = getattr(mod, key[1])
    params = list(inspect.signature(fn).parameters)
    want = REF_SIGNATURES[key]
    assert params[: len(want)] == want
    for name, val in REF_DEFAULTS.get(key, {}).items():
        assert inspect.signature(fn).parameters[name].default == val, name


def test_history_keys_match_reference():
    from admm_hip.admm import HISTORY_KEYS
    # /root/reference/block_6_admm_loop_ver2.py:310-326
    assert set(HISTORY_KEYS) == {"primal", "dual", "pri_per_node", "dual_per_node", "obj_per_node",
                                 "obj_total", "mse_sino_per_node", "mse_sino_total", "img_mse_per_node",
                                 "img_mse_total", "g_norm_history", "eps_used_history",
                                 "eps_target_history"}


def test_non_operator_is_rejected_loudly():
    """Matrices are accepted (explicit-matrix operators, admm_hip/matrix.py); anything that is
    neither an operator nor a 2-D matrix fails before any GPU work."""
    import numpy as np
    import networkx as nx
    from block_6_admm_loop_ver2 import decentralized_admm
    with pytest.raises(ValueError, match="2-D"):
        decentralized_admm([np.zeros(4)], [np.zeros(4)], nx.path_graph(1), [np.ones(4)],
                           lambda i, j: np.ones(4), 2)
    with pytest.raises(ValueError, match="N\\*N"):
        decentralized_admm([np.zeros((4, 5))], [np.zeros(4)], nx.path_graph(1), [np.ones(4)],
                           lambda i, j: np.ones(4), 2)


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(_lib.AdmmLibraryError):
        _lib.load(str(tmp_path / "nope.so"))
