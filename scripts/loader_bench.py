"""Input-pipeline throughput: can the host feed the GPUs?

The reference's run was input-bound (10 PIL worker processes per
rank decode + resize + normalise every image every epoch, imagenet.py:280-283,
350-359). The HIP step consumes ~12k img/s per MI355X at R50/224 (bench.py),
~96k img/s for a node of 8. This measures, on synthetic record files held in
the page cache (the steady state of a multi-epoch run):

1. native gather (csrc/runtime/records.cpp: mmap + C++ thread pool into pinned
   buffers) for ``--ranks`` concurrent RecordFiles (one per rank, as on a node),
   images/s aggregated over ranks;
2. the same plus the pinned H2D copy on a copy stream and the GPU normalise
   kernel (RecordLoader end to end, one rank) when a GPU is present;
3. for contrast, the PIL decode + resize path per CPU core on JPEGs.

    python scripts/loader_bench.py [--sizes 224,448] [--ranks 8] [--threads 4] [--out profiles/loader.md]
"""

import argparse
import io
import os
import sys
import tempfile
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_records(path, n, size):
    from imagent_amd.data.records import write_records
    rng = np.random.default_rng(0)
    base = rng.integers(0, 256, (64, size, size, 3), dtype=np.uint8)
    write_records(path, ((base[i % 64], i % 1000) for i in range(n)), n, (size, size), 1000)


def gather_rate(path, ranks, threads, batch, iters):
    from imagent_amd.data.records import RecordFile
    files = [RecordFile(path, threads=threads) for _ in range(ranks)]
    n = len(files[0])
    bufs = [torch.empty((batch,) + files[0].shape, dtype=torch.uint8, pin_memory=torch.cuda.is_available())
            for _ in range(ranks)]
    done = [0] * ranks

    def work(r):
        g = torch.Generator().manual_seed(r)
        for _ in range(iters):
            idx = torch.randint(0, n, (batch,), generator=g)
            files[r].submit(0, idx, bufs[r], None)
            files[r].wait(0)
            done[r] += batch

    work(0)  # warm the page cache
    done[0] = 0
    ts = [threading.Thread(target=work, args=(r,)) for r in range(ranks)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt = time.perf_counter() - t0
    for f in files:
        f.close()
    return sum(done) / dt


def loader_rate(path, threads, batch, iters, out_size=None):
    from imagent_amd.data.loader import InputTransform
    from imagent_amd.data.records import RecordFile, RecordLoader
    from imagent_amd.parallel.sampler import ShardSampler
    rf = RecordFile(path, threads=threads)
    size = out_size or rf.shape[0]
    tf = InputTransform("hip", (size, size), cpad=4, resize=size != rf.shape[0])
    dl = RecordLoader(rf, ShardSampler(len(rf), 1, 0, shuffle=True, seed=0), batch, tf, "cuda:0")
    seen, t0 = 0, None
    for it in range(iters + 2):
        for k, (x, y) in enumerate(dl):
            if t0 is None and k == 2:
                torch.cuda.synchronize()
                t0, seen = time.perf_counter(), 0
            seen += y.numel()
    torch.cuda.synchronize()
    rf.close()
    return seen / (time.perf_counter() - t0)


def pil_rate(size, n=200):
    from PIL import Image
    from imagent_amd.data.imagenet import decode_resize
    d = tempfile.mkdtemp()
    rng = np.random.default_rng(0)
    for i in range(8):  # ImageNet-like JPEGs (~500x375, q90)
        Image.fromarray(rng.integers(0, 256, (375, 500, 3), dtype=np.uint8)).save(os.path.join(d, f"{i}.jpg"),
                                                                                 quality=90)
    t0 = time.perf_counter()
    for i in range(n):
        decode_resize(os.path.join(d, f"{i % 8}.jpg"), (size, size))
    return n / (time.perf_counter() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="224,448")
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = []
    d = a.dir or tempfile.mkdtemp(prefix="imrec_")
    os.makedirs(d, exist_ok=True)
    # "448@320": 448^2 model input from records stored at 320^2 (GPU resample, --record-resize)
    for spec in a.sizes.split(","):
        size, stored = (int(v) for v in spec.split("@")) if "@" in spec else (int(spec), int(spec))
        n = 4096 if size >= 448 else 8192
        path = os.path.join(d, f"bench_{stored}.imrec")
        if not os.path.exists(path):
            make_records(path, n, stored)
        g1 = gather_rate(path, 1, a.threads, a.batch, a.iters)
        gn = gather_rate(path, a.ranks, a.threads, a.batch, a.iters)
        lr = loader_rate(path, a.threads, a.batch, 2, size) if torch.cuda.is_available() else float("nan")
        pr = pil_rate(size)
        rows.append((spec.replace("@", "² from "), g1, gn, lr, pr))
        print(f"{spec}: gather 1 rank {g1:,.0f} img/s, {a.ranks} ranks {gn:,.0f} img/s; "
              f"RecordLoader+H2D+normalise (1 rank) {lr:,.0f} img/s; PIL decode+resize {pr:,.0f} img/s/core",
              flush=True)
        os.remove(path)
    if a.out:
        with open(a.out, "w") as f:
            f.write("# Input pipeline throughput (scripts/loader_bench.py)\n\n")
            f.write(f"Synthetic uint8 record files in the page cache, batch {a.batch}, {a.threads} gather threads "
                    f"per rank, random sample order; {a.ranks} concurrent ranks = one RecordFile + pool each.\n\n")
            f.write("| image | gather, 1 rank | gather, %d ranks | RecordLoader + pinned H2D + GPU normalise, "
                    "1 rank | PIL JPEG decode + resize, per core |\n|---:|---:|---:|---:|---:|\n" % a.ranks)
            for size, g1, gn, lr, pr in rows:
                f.write(f"| {size}² | {g1:,.0f} img/s | {gn:,.0f} img/s | {lr:,.0f} img/s | {pr:,.0f} img/s |\n")


if __name__ == "__main__":
    main()
