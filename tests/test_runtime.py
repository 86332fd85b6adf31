"""Native bucket planner / ready tracker (csrc/runtime/reducer.cpp)."""

import ctypes as C

import pytest
import torch
import torch.distributed as dist

from imagent_amd.ops import _lib
from imagent_amd.parallel.ddp import _Tracker, plan_buckets

MB = 1024 * 1024


@pytest.fixture(scope="module", autouse=True)
def _build():
    from imagent_amd import build
    build.build_runtime()


def test_plan_matches_torch_assignment():
    torch.manual_seed(0)
    sizes = [int(x) for x in torch.randint(1, 3_000_000, (60,))]
    tensors = [torch.empty(s, dtype=torch.float32) for s in sizes]
    limits = [1 * MB, 25 * MB]
    ref, _ = dist._compute_bucket_assignment_by_size(tensors, limits, [False] * len(tensors),
                                                     list(range(len(tensors))))
    ours = plan_buckets([s * 4 for s in sizes], 1 * MB, 25 * MB)
    got = {}
    for i, b in enumerate(ours):
        got.setdefault(b, []).append(i)
    assert [got[k] for k in sorted(got)] == [list(x) for x in ref]


def test_resnet18_default_buckets():
    """steady-state R18 buckets with 1 / 25 MiB caps in ready order."""
    from imagent_amd.models import resnet
    m = resnet.resnet18()
    ps = list(m.parameters())
    rev = list(reversed(ps))
    ids = plan_buckets([p.numel() * 4 for p in rev], 1 * MB, 25 * MB)
    nb = max(ids) + 1
    sizes = [sum(p.numel() * 4 for p, b in zip(rev, ids) if b == k) / MB for k in range(nb)]
    assert nb == 3
    assert abs(sizes[0] - 1.96) < 0.01          # fc.bias + fc.weight


def test_tracker_in_order_launch_and_errors():
    tr = _Tracker([0, 0, 1, 2, 2], 3)
    assert tr.mark(2) == (0, 0)      # bucket 1 complete but bucket 0 not -> nothing launchable
    assert tr.mark(0) == (0, 0)
    assert tr.mark(1) == (0, 2)      # buckets 0 and 1 now launch, in order
    with pytest.raises(RuntimeError):
        tr.mark(1)                   # double mark
    assert tr.mark(3) == (2, 0)
    missing, unready, order = tr.finalize()
    assert missing == 1 and unready == [4] and order == [2, 0, 1, 3]
    # state reset for the next iteration
    for i in range(5):
        tr.mark(i)
    missing, unready, _ = tr.finalize()
    assert missing == 0 and unready == []


def test_native_library_is_used():
    tr = _Tracker([0], 1)
    assert tr.L is not None
