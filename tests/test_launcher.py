"""Slurm / torchrun / single discovery (reference: imagenet.py:224-262)."""

import os
import stat

from imagent_amd.parallel import launcher


def _slurm_env(**over):
    env = dict(SLURM_JOB_NUM_NODES="8", SLURM_NODEID="2", SLURM_LOCALID="1", SLURM_PROCID="5",
               SLURM_NTASKS="16", SLURM_JOB_NODELIST="ener[021-024,030]")
    env.update(over)
    return env


def test_hostlist_expansion_python():
    assert launcher._expand_hostlist_py("ener[021-023,030]") == ["ener021", "ener022", "ener023", "ener030"]
    assert launcher._expand_hostlist_py("a1,b[1-2]-ib,c") == ["a1", "b1-ib", "b2-ib", "c"]
    assert launcher._expand_hostlist_py("node07") == ["node07"]


def test_slurm_topology_matches_reference_math(monkeypatch):
    monkeypatch.setenv("PATH", "/nonexistent")  # no scontrol -> python expansion
    t = launcher.discover("auto", env=_slurm_env())
    assert t.launcher == "slurm"
    assert (t.n_nodes, t.node_id, t.local_rank, t.global_rank, t.world_size) == (8, 2, 1, 5, 16)
    assert t.n_gpu_per_node == 2          # imagenet.py:234
    assert t.master_addr == "ener021"     # first host, imagenet.py:238
    assert t.master_port == 29500         # imagenet.py:242 default
    assert not t.is_master and t.multi_node and t.multi_gpu


def test_stub_scontrol_on_path(tmp_path, monkeypatch):
    stub = tmp_path / "scontrol"
    stub.write_text("#!/bin/sh\necho hostA\necho hostB\n")
    stub.chmod(stub.stat().st_mode | stat.S_IEXEC)
    monkeypatch.setenv("PATH", str(tmp_path) + os.pathsep + os.environ.get("PATH", ""))
    t = launcher.discover("slurm", env=_slurm_env(SLURM_NODEID="0", SLURM_LOCALID="0", SLURM_PROCID="0"))
    assert t.master_addr == "hostA"
    assert t.is_master


def test_job_id_port_and_env_export():
    t = launcher.discover("slurm", env=_slurm_env(SLURM_JOB_ID="123456", MASTER_ADDR="10.0.0.1"))
    assert t.master_port == 20000 + 123456 % 20000
    env = t.export_env({})
    assert env == {"MASTER_ADDR": "10.0.0.1", "MASTER_PORT": str(t.master_port), "WORLD_SIZE": "16",
                   "RANK": "5", "LOCAL_RANK": "1"}


def test_torchrun_and_single():
    t = launcher.discover("auto", env=dict(RANK="3", WORLD_SIZE="8", LOCAL_RANK="3", LOCAL_WORLD_SIZE="8",
                                           MASTER_ADDR="127.0.0.1", MASTER_PORT="29999"))
    assert t.launcher == "torchrun" and t.world_size == 8 and t.n_nodes == 1 and t.master_port == 29999
    s = launcher.discover("auto", env={})
    assert s.launcher == "single" and s.world_size == 1 and s.is_master


def test_banner_format():
    t = launcher.discover("slurm", env=_slurm_env())
    lines = t.banner()
    assert len(lines) == 10
    assert lines[0] == "5 - Number of nodes: 8"
    assert lines[5] == "5 - GPUs per node  : 2"
    assert lines[6] == "5 - Master         : False"
    assert lines[9].startswith("5 - Hostname       : ")
