"""make_communicator: when the own RCCL communicator cannot start on a
multi-rank job, every rank falls back to the c10d process group together
(no rank left waiting on the unique-id key), and collectives still average.
On this CPU container ncclCommInitRank fails at hipSetDevice, which is the
failure being exercised."""

import socket
from types import SimpleNamespace

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.slow


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port):
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    try:
        from imagent_amd.parallel.comm import make_communicator
        ctx = SimpleNamespace(rank=rank, world_size=2, device=torch.device("cpu"))
        with pytest.warns(UserWarning, match="own RCCL communicator unavailable"):
            c = make_communicator(ctx, "rccl")
        assert c.name == "torch"
        t = torch.full((4,), float(rank + 1))
        c.allreduce_(t, "avg")
        c.join()
        assert t.tolist() == [1.5] * 4
    finally:
        dist.destroy_process_group()


def test_rccl_unavailable_falls_back_on_all_ranks():
    if torch.cuda.is_available():
        pytest.skip("a GPU is present: the RCCL communicator would start")
    mp.start_processes(_worker, args=(_free_port(),), nprocs=2, start_method="spawn", join=True)
