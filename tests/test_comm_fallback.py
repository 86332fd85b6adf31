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


class _FakeRccl:
    """Stands in for libimagent_comm: rank 1's ncclCommInitRank fails at once,
    rank 0's never finishes on its own (it would wait in the RCCL bootstrap for
    the dead peer) until it is aborted."""

    def __init__(self, rank):
        self.rank, self.aborted, self.destroyed = rank, False, False

    def imc_unique_id_bytes(self):
        return 128

    def imc_get_unique_id(self, buf):
        buf.raw = b"u" * 128
        return 0

    def imc_comm_init_start(self, uid, n, rank, dev, nev, nb, out):
        if self.rank == 1:
            return -2
        out._obj.value = 0x1000  # a (fake) communicator handle
        return 0

    def imc_comm_set_stream_mode(self, h, mode):
        return 0

    def imc_comm_poll(self, h):
        return -3 if self.aborted else 1

    def imc_abort(self, h):
        self.aborted = True
        return 0

    def imc_comm_destroy(self, h):
        self.destroyed = True
        return 0

    def imc_last_error(self):
        return b"simulated init failure on rank 1"


def _partial_worker(rank, port, outdir):
    import os
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    try:
        from imagent_amd.ops import _lib
        from imagent_amd.parallel import comm as C
        fake = _FakeRccl(rank)
        _lib.comm = lambda: fake
        ctx = SimpleNamespace(rank=rank, world_size=2, device=torch.device("cpu"))
        with pytest.warns(UserWarning, match="own RCCL communicator unavailable"):
            c = C.make_communicator(ctx, "rccl")
        assert c.name == "torch"
        if rank == 0:
            assert fake.aborted, "rank 0 kept waiting on a communicator its peer abandoned"
        t = torch.full((4,), float(rank + 1))
        c.allreduce_(t, "avg")
        c.join()
        assert t.tolist() == [1.5] * 4
        open(os.path.join(outdir, f"ok{rank}"), "w").close()
    finally:
        dist.destroy_process_group()


def test_rccl_init_failing_on_one_rank_falls_back_everywhere(tmp_path):
    """ncclCommInitRank failing on ONE rank must not leave the others
    blocked in the bootstrap or on a working RCCL communicator."""
    import os
    mp.start_processes(_partial_worker, args=(_free_port(), str(tmp_path)), nprocs=2, start_method="spawn",
                       join=True)
    assert os.path.exists(tmp_path / "ok0") and os.path.exists(tmp_path / "ok1")


def test_torch_override_without_process_group(monkeypatch):
    """IMAGENT_COMM=torch in a single process with no c10d group (the training CLI at one GPU)
    gives the local communicator instead of failing in dist.get_rank."""
    from imagent_amd.parallel.comm import make_communicator
    assert not dist.is_initialized()
    monkeypatch.setenv("IMAGENT_COMM", "torch")
    ctx = SimpleNamespace(rank=0, world_size=1, device=torch.device("cpu"))
    c = make_communicator(ctx, "auto")
    assert c.name == "local"
    t = torch.ones(3)
    c.allreduce_(t, "avg")
    c.join()
    assert t.tolist() == [1.0] * 3


class _FakeRcclOk:
    """libimagent_comm stand-in where every rank's non-blocking init finishes after a few polls."""

    def __init__(self, rank):
        self.rank, self.uid, self.polls, self.aborted = rank, None, 0, False

    def imc_unique_id_bytes(self):
        return 128

    def imc_get_unique_id(self, buf):
        buf.raw = bytes(range(128))
        return 0

    def imc_comm_init_start(self, uid, n, rank, dev, nev, nb, out):
        self.uid = bytes(uid)
        out._obj.value = 0x2000 + rank
        return 0

    def imc_comm_set_stream_mode(self, h, mode):
        return 0

    def imc_comm_poll(self, h):
        self.polls += 1
        return 0 if self.polls >= 3 else 1  # "still initialising" twice, then ready

    def imc_comm_stream(self, h):
        return 0

    def imc_comm_nranks(self, h):
        return 2

    def imc_async_error(self, h):
        return 0

    def imc_abort(self, h):
        self.aborted = True
        return 0

    def imc_comm_destroy(self, h):
        return 0

    def imc_last_error(self):
        return b""


def _ok_worker(rank, port, outdir):
    import os
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    try:
        from imagent_amd.ops import _lib
        from imagent_amd.parallel import comm as C
        fake = _FakeRcclOk(rank)
        _lib.comm = lambda: fake
        torch.cuda.ExternalStream = lambda ptr, device=None: SimpleNamespace(cuda_stream=ptr)  # no GPU here
        ctx = SimpleNamespace(rank=rank, world_size=2, device=torch.device("cuda", 0))
        c = C.make_communicator(ctx, "rccl")
        assert c.name == "rccl" and isinstance(c, C.RcclCommunicator)
        assert fake.uid == bytes(range(128)), "rank 0's unique id did not reach this rank"
        assert fake.polls == 3 and not fake.aborted
        assert c.nranks == 2 and c.healthy()
        assert C.RcclCommunicator.live == 1
        c.close()
        assert C.RcclCommunicator.live == 0
        open(os.path.join(outdir, f"ok{rank}"), "w").close()
    finally:
        dist.destroy_process_group()


def test_rccl_bootstrap_success_on_all_ranks(tmp_path):
    """The success path of the own-RCCL bootstrap (unique id through the c10d store, non-blocking init
    polled to completion, the all-ranks agreement): every rank gets an RCCL communicator, none falls back
    or aborts."""
    import os
    mp.start_processes(_ok_worker, args=(_free_port(), str(tmp_path)), nprocs=2, start_method="spawn", join=True)
    assert os.path.exists(tmp_path / "ok0") and os.path.exists(tmp_path / "ok1")
