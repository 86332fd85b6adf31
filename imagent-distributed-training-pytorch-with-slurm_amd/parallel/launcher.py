"""Process-topology discovery: Slurm, torchrun, or single process.

Reference behaviour (``/root/reference/imagenet.py``):

* ``imagenet.py:224-234`` reads ``SLURM_JOB_NUM_NODES``, ``SLURM_NODEID``,
  ``SLURM_LOCALID``, ``SLURM_PROCID`` and ``SLURM_NTASKS`` and derives
  ``n_gpu_per_node = world_size // n_nodes``.
* ``imagenet.py:236-244`` expands ``SLURM_JOB_NODELIST`` with
  ``scontrol show hostnames`` and takes the first host as ``MASTER_ADDR``;
  ``MASTER_PORT`` is hard-coded to 29500 (quirk Q11 - here it is configurable
  and defaults to 29500 only when nothing else is set).
* ``imagenet.py:247-249`` computes ``is_master``, ``multi_node``,
  ``multi_gpu``; ``imagenet.py:252-262`` prints a 10-line rank banner.

On top of that this module understands the torchrun contract
(``RANK``/``LOCAL_RANK``/``WORLD_SIZE``/``LOCAL_WORLD_SIZE``/``MASTER_*``) and
a plain single-process run, selected with ``launcher='auto'`` by whichever
environment is present.
"""

from __future__ import annotations

import dataclasses
import os
import re
import socket
import subprocess
from typing import Dict, List, Optional

DEFAULT_MASTER_PORT = 29500


@dataclasses.dataclass
class Topology:
    """Where this process sits in the job."""

    launcher: str
    n_nodes: int
    node_id: int
    local_rank: int
    global_rank: int
    world_size: int
    n_gpu_per_node: int
    master_addr: str
    master_port: int

    @property
    def is_master(self) -> bool:
        # imagenet.py:247 - master = node 0, local rank 0 (== global rank 0 for
        # block-distributed Slurm tasks).
        return self.node_id == 0 and self.local_rank == 0

    @property
    def multi_node(self) -> bool:
        return self.n_nodes > 1

    @property
    def multi_gpu(self) -> bool:
        return self.world_size > 1

    def export_env(self, env: Optional[Dict[str, str]] = None) -> Dict[str, str]:
        """Export the ``env://`` rendezvous variables (imagenet.py:241-244)."""
        env = os.environ if env is None else env
        env["MASTER_ADDR"] = self.master_addr
        env["MASTER_PORT"] = str(self.master_port)
        env["WORLD_SIZE"] = str(self.world_size)
        env["RANK"] = str(self.global_rank)
        env["LOCAL_RANK"] = str(self.local_rank)
        return env

    def banner(self) -> List[str]:
        """The per-rank banner of imagenet.py:252-262 (same labels, same order)."""
        p = "%i - " % self.global_rank
        return [
            p + "Number of nodes: %i" % self.n_nodes,
            p + "Node ID        : %i" % self.node_id,
            p + "Local rank     : %i" % self.local_rank,
            p + "Global rank    : %i" % self.global_rank,
            p + "World size     : %i" % self.world_size,
            p + "GPUs per node  : %i" % self.n_gpu_per_node,
            p + "Master         : %s" % str(self.is_master),
            p + "Multi-node     : %s" % str(self.multi_node),
            p + "Multi-GPU      : %s" % str(self.multi_gpu),
            p + "Hostname       : %s" % socket.gethostname(),
        ]


# --------------------------------------------------------------------------
# Slurm hostlist expansion
# --------------------------------------------------------------------------

def _expand_hostlist_py(nodelist: str) -> List[str]:
    """Pure-Python expansion of a Slurm hostlist expression.

    Handles ``a[01-03,07],b5,c[1-2]-ib`` style lists. Used when ``scontrol``
    is not on PATH (tests, torchrun-on-slurm without the client tools).
    """
    hosts: List[str] = []
    # split on commas that are not inside brackets
    parts, depth, cur = [], 0, ""
    for ch in nodelist:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    if cur:
        parts.append(cur)
    for part in parts:
        m = re.match(r"^(.*?)\[([^\]]+)\](.*)$", part)
        if not m:
            hosts.append(part)
            continue
        prefix, ranges, suffix = m.groups()
        for rng in ranges.split(","):
            if "-" in rng:
                lo, hi = rng.split("-")
                width = len(lo)
                for i in range(int(lo), int(hi) + 1):
                    hosts.append(f"{prefix}{str(i).zfill(width)}{suffix}")
            else:
                hosts.append(f"{prefix}{rng}{suffix}")
    return hosts


def expand_hostlist(nodelist: str) -> List[str]:
    """``scontrol show hostnames <nodelist>`` (imagenet.py:237), with a
    pure-Python fallback when the Slurm client is unavailable."""
    try:
        out = subprocess.check_output(["scontrol", "show", "hostnames", nodelist],
                                      stderr=subprocess.DEVNULL)
        hosts = out.decode("utf-8").split()
        if hosts:
            return hosts
    except (OSError, subprocess.CalledProcessError):
        pass
    return _expand_hostlist_py(nodelist)


# --------------------------------------------------------------------------
# discovery
# --------------------------------------------------------------------------

def _slurm_topology(env: Dict[str, str], master_port: Optional[int]) -> Topology:
    n_nodes = int(env["SLURM_JOB_NUM_NODES"])
    node_id = int(env["SLURM_NODEID"])
    local_rank = int(env["SLURM_LOCALID"])
    global_rank = int(env["SLURM_PROCID"])
    world_size = int(env["SLURM_NTASKS"])
    nodelist = env.get("SLURM_JOB_NODELIST") or env.get("SLURM_NODELIST", "127.0.0.1")
    master_addr = env.get("MASTER_ADDR") or expand_hostlist(nodelist)[0]
    if master_port is None:
        # Q11: derive a per-job port instead of colliding on a fixed 29500
        # when two jobs share a first node; MASTER_PORT still wins.
        if "MASTER_PORT" in env:
            master_port = int(env["MASTER_PORT"])
        elif "SLURM_JOB_ID" in env:
            master_port = 20000 + int(env["SLURM_JOB_ID"]) % 20000
        else:
            master_port = DEFAULT_MASTER_PORT
    return Topology("slurm", n_nodes, node_id, local_rank, global_rank, world_size,
                    max(1, world_size // max(1, n_nodes)), master_addr, master_port)


def _torchrun_topology(env: Dict[str, str], master_port: Optional[int]) -> Topology:
    world_size = int(env["WORLD_SIZE"])
    global_rank = int(env["RANK"])
    local_rank = int(env.get("LOCAL_RANK", global_rank))
    local_ws = int(env.get("LOCAL_WORLD_SIZE", world_size))
    n_nodes = max(1, world_size // max(1, local_ws))
    node_id = int(env.get("GROUP_RANK", global_rank // max(1, local_ws)))
    port = master_port if master_port is not None else int(env.get("MASTER_PORT", DEFAULT_MASTER_PORT))
    return Topology("torchrun", n_nodes, node_id, local_rank, global_rank, world_size,
                    local_ws, env.get("MASTER_ADDR", "127.0.0.1"), port)


def _single_topology(env: Dict[str, str], master_port: Optional[int]) -> Topology:
    port = master_port if master_port is not None else int(env.get("MASTER_PORT", DEFAULT_MASTER_PORT))
    return Topology("single", 1, 0, 0, 0, 1, 1, env.get("MASTER_ADDR", "127.0.0.1"), port)


def discover(launcher: str = "auto", env: Optional[Dict[str, str]] = None,
             master_port: Optional[int] = None) -> Topology:
    """Resolve the process topology.

    ``launcher``: ``auto`` (torchrun env wins, then Slurm, then single),
    ``slurm``, ``torchrun`` or ``single``.
    """
    env = dict(os.environ) if env is None else env
    if launcher == "auto":
        if "RANK" in env and "WORLD_SIZE" in env:
            launcher = "torchrun"
        elif "SLURM_PROCID" in env and "SLURM_NTASKS" in env and "SLURM_JOB_NUM_NODES" in env:
            launcher = "slurm"
        else:
            launcher = "single"
    if launcher == "slurm":
        return _slurm_topology(env, master_port)
    if launcher == "torchrun":
        return _torchrun_topology(env, master_port)
    if launcher == "single":
        return _single_topology(env, master_port)
    raise ValueError(f"unknown launcher {launcher!r}")
