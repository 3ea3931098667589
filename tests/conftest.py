import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-inverse-problem-admm_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    config.addinivalue_line("markers", "long: GPU run outside the suite's time budget; runs with ADMM_TEST_LONG=1")


# GPU-suite order (the driver runs ``-m gpu`` under a fixed time limit): the dedicated parity
# files first, the whole-trajectory / full-size / bench runs last, so that an overrun can only
# cut the long tail.  Files not listed run in between, in collection order.
FIRST = ("test_gpu_projector", "test_gpu_mirror", "test_gpu_consensus", "test_gpu_dropins",
         "test_gpu_masks", "test_gpu_matrix", "test_gpu_groups", "test_gpu_multirank",
         "test_gpu_fullsize_projector", "test_gpu_fullsize", "test_gpu_admm", "test_gpu_block3_suites")
LAST = ("test_gpu_bench", "test_gpu_configs", "test_gpu_configs_full")
# the longest single tests (tens of seconds to ~2 minutes each), in this order at the very end
LONGEST = ("test_large_x_updates_match_operator_oracle", "test_c4_ranks_match_one_rank_bitwise",
           "test_bench_eight_ranks_with_strong_c4", "test_c5_full_graph_one_gpu_and_two_ranks",
           "test_c4_full_graph_matches_operator_oracle", "test_ring_trajectory_matches_oracle",
           "test_c5_share_full_inner_count_matches_operator_oracle")


def _order_key(item):
    mod = item.fspath.purebasename
    name = item.originalname or item.name
    if name in LONGEST:
        return (3, LONGEST.index(name), 0)
    if mod in FIRST:
        return (0, FIRST.index(mod), 0)
    if mod in LAST:
        return (2, LAST.index(mod), 0)
    return (1, 0, 0)


def pytest_collection_modifyitems(session, config, items):
    items[:] = [it for _, it in sorted(enumerate(items), key=lambda p: (_order_key(p[1]), p[0]))]
    if os.environ.get("ADMM_TEST_LONG") != "1":
        skip = pytest.mark.skip(reason="long run outside the GPU suite's budget (ADMM_TEST_LONG=1 runs it)")
        for it in items:
            if "long" in it.keywords:
                it.add_marker(skip)


@pytest.fixture(scope="session")
def cuda():
    import torch
    assert torch.cuda.is_available(), "gpu-marked test needs a GPU"
    return torch.device("cuda", 0)
