"""End-to-end CPU runs of the CLI (single process and 2-rank gloo)."""

import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, cwd, env_extra=None, timeout=300):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, "-m", "imagent_amd.cli"] + args, cwd=cwd, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-4000:]
    return r.stdout


COMMON = ["--arch", "resnet18", "--image-size", "32", "--data", "synthetic", "--synthetic-train-size", "48",
          "--synthetic-val-size", "16", "--batch-size", "8", "--num-classes", "10", "--log-interval", "3",
          "--quiet-banner"]


def test_single_process_two_epochs_and_resume(tmp_path):
    out = _run(COMMON + ["--epochs", "2", "--tb-dir", str(tmp_path / "tb"), "--save-model",
                         "--checkpoint-dir", str(tmp_path)], tmp_path)
    assert "Epoch 1 Summary: " in out and "Epoch 2 Summary: " in out
    assert "\tLearning rate: 0.1" in out
    assert "Training Summary:" in out and "Training time:" in out
    assert os.path.exists(tmp_path / "state_resnet18.pt")
    assert os.path.isdir(tmp_path / "tb" / "Loss_train")
    out2 = _run(COMMON + ["--epochs", "3", "--tb-dir", "", "--resume", str(tmp_path / "state_resnet18.pt")],
                tmp_path)
    assert "Resumed from" in out2 and "Epoch 3 Summary: " in out2 and "Epoch 1 Summary" not in out2


def test_records_data_one_epoch(tmp_path):
    """--data records: train.imrec / val.imrec through the native gather loader."""
    import numpy as np

    from imagent_amd.data.records import write_records
    rng = np.random.default_rng(0)
    for split, n in (("train", 40), ("val", 12)):
        imgs = rng.integers(0, 256, (n, 32, 32, 3), dtype=np.uint8)
        write_records(str(tmp_path / f"{split}.imrec"), zip(imgs, rng.integers(0, 10, n)), n, (32, 32), 10)
    out = _run(["--arch", "resnet18", "--image-size", "32", "--data", "records", "--data-root", str(tmp_path),
                "--workers", "2", "--batch-size", "8", "--epochs", "1", "--tb-dir", "", "--quiet-banner"], tmp_path)
    assert "Training samples: 40 images" in out and "number of classes: 10" in out
    assert "Epoch 1 Summary: " in out


@pytest.mark.slow
def test_torchrun_two_ranks_gloo(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29517", "-m", "imagent_amd.cli"] + COMMON + \
          ["--epochs", "1", "--backend", "gloo", "--tb-dir", ""]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-4000:]
    assert r.stdout.count("Epoch 1 Summary: ") == 1        # master only
    assert "Backend: gloo" in r.stdout


def test_slurm_env_single_task(tmp_path):
    env = dict(SLURM_JOB_NUM_NODES="1", SLURM_NODEID="0", SLURM_LOCALID="0", SLURM_PROCID="0",
               SLURM_NTASKS="1", SLURM_JOB_NODELIST="127.0.0.1")
    out = _run([a for a in COMMON if a != "--quiet-banner"] + ["--epochs", "1", "--tb-dir", ""], tmp_path, env)
    assert "0 - Number of nodes: 1" in out and "0 - Master         : True" in out


@pytest.mark.slow
def test_watchdog_ends_a_hung_two_rank_job(tmp_path):
    """Rank 1 stalls (fault injection) before step 3; rank 0 then blocks in the
    gradient all-reduce. With --step-timeout 4 both ranks' watchdogs dump their
    stacks, abort the communicators and exit non-zero, and the job ends within
    timeout + a few seconds instead of waiting for the 1800 s collective timeout."""
    import time
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", IMAGENT_FAULT_STALL="1:3:120")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29533", "-m", "imagent_amd.cli"] + COMMON + \
          ["--epochs", "1", "--backend", "gloo", "--tb-dir", "", "--step-timeout", "4",
           "--synthetic-train-size", "160"]
    t0 = time.monotonic()
    r = subprocess.run(cmd, cwd=tmp_path, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=200)
    dt = time.monotonic() - t0
    assert r.returncode != 0, r.stdout[-3000:]
    assert "[watchdog rank 0] no progress for 4 s" in r.stdout, r.stdout[-3000:]
    assert "exitcode  : 75" in r.stdout or "exit code 75" in r.stdout or "exitcode: 75" in r.stdout, r.stdout[-2000:]
    assert dt < 60, dt


@pytest.mark.slow
def test_slow_checkpoint_write_does_not_trip_the_watchdog(tmp_path):
    """the master writes its checkpoint for longer than --step-timeout while the other
    rank waits; both watchdogs are disarmed around the write and the ranks meet in a barrier
    afterwards, so the healthy job completes (no exit 75)."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", IMAGENT_FAULT_SLOW_SAVE="7")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29541", "-m", "imagent_amd.cli"] + COMMON + \
          ["--epochs", "2", "--backend", "gloo", "--tb-dir", "", "--step-timeout", "3", "--save-model",
           "--checkpoint-dir", str(tmp_path)]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "[fault injection] checkpoint write stalls 7 s" in r.stdout
    assert "no progress" not in r.stdout, r.stdout[-3000:]
    assert r.stdout.count("Epoch 2 Summary: ") == 1
