"""Training engine: set-up, train / validate loops, epoch driver.

Mirrors the reference's ``run()`` / ``train()`` / ``validate()``
(``imagenet.py:97-151, 166-210, 213-429``) and its observable outputs
(banners, per-epoch and final summaries in the same text format,
TensorBoard tags, best-model checkpoint), re-designed for MI355X:

* one training step = normalise kernel -> HIP forward -> fused softmax-xent
  (+top-1/top-5 counters on device) -> HIP backward whose weight-gradient
  kernels feed the bucketed RCCL all-reduce on a side stream -> one fused
  SGD launch. No host synchronisation inside the step (the reference does
  three ``.item()`` and a ``cuda.synchronize()`` per batch, ``:143-147``);
* metrics are reduced across ranks once per log interval and per epoch;
* epoch time is the wall time of the whole loop (the reference sums
  per-batch times, which excludes loader re-forks between epochs).
"""

from __future__ import annotations

import collections
import json
import math
import os
import sys
import time
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from ..data.loader import DeviceLoader, InputTransform, SyntheticLoader
from ..data.synthetic import SyntheticImageNet, mix_pool_cap
from ..models import resnet
from ..models.arena import ParamArena
from ..parallel import launcher
from ..parallel.comm import make_communicator
from ..parallel.ddp import DataParallel
from ..parallel.dist import init_distributed
from ..parallel.sampler import ShardSampler
from ..utils import checkpoint as ckpt
from ..utils.tb import SummaryWriter
from .lr import Schedule
from .meters import AverageMeter, DeviceMetrics
from .optim import build_optimizer
from ..utils.watchdog import maybe_stall, slow_save


class StepRunner:
    """One optimizer step over ``accum`` micro-batches."""

    def __init__(self, ddp: DataParallel, opt, metrics: DeviceMetrics, backend: str,
                 smoothing: float = 0.0, autocast_dtype: Optional[torch.dtype] = None):
        self.ddp, self.opt, self.metrics = ddp, opt, metrics
        self.backend, self.smoothing = backend, smoothing
        self.autocast_dtype = autocast_dtype
        # Run-ahead limit: with no host sync in the step the CPU can queue many steps, and
        # every queued step holds its own activations until the step's end-of-backward join
        # (they are read on the weight-gradient side stream, ops/streams.py): measured 252 GiB
        # reserved for a 40.6 GiB peak at R50 / 1024 img without a limit, which thrashes the
        # allocator once the GPU is shared. Waiting (blocking-sync event, no spinning core)
        # on the step `max_inflight` back keeps the GPU fed and the footprint bounded.
        self.max_inflight = int(os.environ.get("IMAGENT_MAX_INFLIGHT", "2"))
        self._blocking = os.environ.get("IMAGENT_THROTTLE", "block") == "block"
        # IMAGENT_STEP_SYNC=1 (diagnostics): device-synchronise after every step -- no run-ahead at all
        self._step_sync = os.environ.get("IMAGENT_STEP_SYNC", "0") == "1"
        self._inflight: collections.deque = collections.deque()

    def _throttle(self, dev: torch.device) -> None:
        if self.max_inflight <= 0 or dev.type != "cuda" or torch.cuda.is_current_stream_capturing():
            return
        ev = torch.cuda.Event(blocking=self._blocking)  # blocking: the host sleeps, it does not spin
        ev.record(torch.cuda.current_stream(dev))
        self._inflight.append(ev)
        while len(self._inflight) > self.max_inflight:
            self._inflight.popleft().synchronize()

    def loss(self, logits, y):
        if self.backend in ("hip", "hip_f32"):
            from ..ops.misc import XentFn
            if self.backend == "hip_f32":  # fp32 logits gradient
                from ..ops.f32 import XentF32Fn as XentFn
            loss = XentFn.apply(logits, y, self.metrics.buf, self.smoothing)
            self.metrics.count_batch()
            return loss
        loss = F.cross_entropy(logits.float(), y, label_smoothing=self.smoothing)
        self.metrics.update_from_logits(logits.float(), y, loss)
        return loss

    def forward(self, x):
        if self.autocast_dtype is not None and x.is_cuda:
            with torch.autocast("cuda", dtype=self.autocast_dtype):
                return self.ddp(x)
        return self.ddp(x)

    def _seed(self, loss, n: int):
        key = (loss.device, loss.dtype, n)
        cache = self.__dict__.setdefault("_seeds", {})
        t = cache.get(key)
        if t is None:
            t = cache[key] = torch.full((), 1.0 / n, device=loss.device, dtype=loss.dtype)
        return t

    def train_step(self, micro) -> None:
        from ..ops import streams
        streams.reset()
        self.opt.zero_grad()
        n = len(micro)
        try:
            for i, (x, y) in enumerate(micro):
                ctx = self.ddp.no_sync() if i + 1 < n else _null()
                with ctx:
                    loss = self.loss(self.forward(x), y)
                    # the seed gradient 1 / n from a cached device scalar: no fill / div launch per step
                    loss.backward(self._seed(loss, n))
        except BaseException:
            streams.reset()  # a failed backward may have left its join callback unrun
            self.ddp.abandon_backward()
            raise
        if streams.deferred():  # a deferred weight gradient nobody issued: a graph without a flush point
            raise RuntimeError("weight-gradient launches left queued after backward")
        self.opt.step()
        if self._step_sync and micro[0][0].is_cuda:
            torch.cuda.synchronize()
        self._throttle(micro[0][0].device)

    @torch.no_grad()
    def eval_step(self, x, y) -> None:
        self.loss(self.forward(x), y)


class GraphedStep:
    """A whole training step captured once into a HIP graph and replayed.

    ``fn(*inputs)`` (input normalisation -> forward -> loss -> backward with
    the bucketed all-reduce -> optimizer) runs eagerly for ``warmup`` calls
    (kernel-variant caches, momentum buffers, bucket rebuild, BN descriptor
    upload all settle), is then captured with ``torch.cuda.graph`` on static
    copies of its inputs, and every later call copies the new inputs in and
    replays: ~400 kernel launches become one graph launch, which is what
    bounds small per-GPU batches. The capture is keyed on the input shapes and
    on ``key_fn()`` (e.g. the learning rate, a kernel argument): a change
    re-captures. Host-side counters are not advanced by replays.
    """

    def __init__(self, fn, warmup: int = 3, key_fn=None, two_stream: bool = False):
        self.fn, self.warmup, self.key_fn = fn, warmup, key_fn
        # two_stream: capture the weight-gradient side stream too (its fork / join become event edges of the
        # graph); default off: on ROCm 7 / torch 2.10 a replayed two-branch graph measured slower than eager
        # (profiles/r50_small_batch_graph_r5.md) and the round-1 / round-5 captures segfaulted in EndCapture on
        # ResNet-18's deterministic mode (scripts/graph_capture_repro.py)
        self.two_stream = two_stream
        self.graph = None
        self.static = None
        self.key = None
        self.eager_calls = 0
        self.replays = 0

    def __call__(self, *inputs):
        key = (tuple((t.shape, t.dtype) for t in inputs), self.key_fn() if self.key_fn else None)
        if self.graph is not None and key == self.key:
            for dst, src in zip(self.static, inputs):
                dst.copy_(src, non_blocking=True)
            self.graph.replay()
            self.replays += 1
            return
        if self.eager_calls < self.warmup or self.graph is not None:
            # warm-up, or a key change: one eager step under the new key first
            self.fn(*inputs)
            self.eager_calls += 1
            if self.graph is not None:
                self.graph = None
                self.eager_calls = self.warmup
            return
        self.static = [t.clone() for t in inputs]
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        from ..ops import streams
        # captured single-stream: capturing the weight-gradient side stream's
        # fork/join (event edges between two streams) segfaults in
        # hipStreamEndCapture on this ROCm 7 / torch 2.10 stack, even with the
        # join made explicit -- measured in round 1 (capture experiment)
        overlap = streams.overlap_enabled()
        streams.set_wgrad_overlap(overlap and self.two_stream)
        try:
            with torch.cuda.graph(g):
                self.fn(*self.static)
        finally:
            streams.set_wgrad_overlap(overlap)
            streams.release_capture_events()  # the capture has ended: its fork / join events may go
        self.graph, self.key = g, key
        g.replay()  # the capture only recorded: run this step's work
        self.replays += 1


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _abort_c10d() -> None:
    import torch.distributed as dist
    if dist.is_initialized():
        dist.distributed_c10d._abort_process_group()


def _master_print(is_master, *a, **kw):
    if is_master:
        print(*a, **kw, flush=True)


class Trainer:
    def __init__(self, args):
        self.args = a = args
        torch.manual_seed(a.seed)  # imagenet.py:215
        self.topo = launcher.discover(a.launcher)
        if not a.quiet_banner:
            for line in self.topo.banner():   # imagenet.py:252-262
                print(line, flush=True)
        self.ctx = init_distributed(self.topo, a.backend, a.pg_timeout, a.device,
                                    verbose=self.topo.is_master)
        self.device = self.ctx.device
        self.is_master = self.ctx.is_master
        self.kernels = a.kernels if a.kernels != "auto" else ("hip" if self.device.type == "cuda" else "torch")
        if self.kernels == "hip" and self.device.type != "cuda":
            raise RuntimeError("--kernels hip needs a GPU")
        if self.kernels == "hip" and a.dtype == "fp32":  # the fp32 kernel path (models/native_f32.py)
            self.kernels = "hip_f32"
        self._build_data()
        self._build_model()
        self.tb = SummaryWriter(a.tb_dir, jsonl=os.path.join(a.tb_dir, "metrics.jsonl")) \
            if (self.is_master and a.tb_dir) else None

    # ------------------------------------------------------------- data
    def _build_data(self):
        a = self.args
        _master_print(self.is_master, "Initialize Dataloaders...")
        size = (a.image_size, a.image_size)
        ws, rk = self.ctx.world_size, self.ctx.rank
        if a.data == "synthetic":
            self.num_classes = a.num_classes
            task = getattr(a, "synthetic_task", "random")
            # mix: every training batch distinct (the accuracy must come from generalising, not recall)
            pool = 4 if task == "random" else 16 if task == "colour" else None
            vpool = pool
            if pool is None:
                # capped by bytes (the pool is rendered once and stays resident in HBM): at most
                # IMAGENT_MIX_POOL_GB (default 16) per pool, train and validation alike
                cap = mix_pool_cap(a.batch_size, a.image_size)
                pool = max(1, min(a.synthetic_train_size // a.batch_size, cap))
                vpool = max(1, min(a.synthetic_val_size // a.batch_size, cap))
            self.train_src = SyntheticImageNet(a.synthetic_train_size, a.image_size, a.num_classes,
                                               a.batch_size, self.device, a.seed, rank=rk, task=task,
                                               pool_batches=pool)
            self.val_src = SyntheticImageNet(a.synthetic_val_size, a.image_size, a.num_classes,
                                             a.batch_size, self.device, a.seed + 1, rank=rk, task=task,
                                             pool_batches=vpool)
            self.n_train, self.n_val = a.synthetic_train_size, a.synthetic_val_size
            self.train_sampler = ShardSampler(self.n_train, ws, rk, shuffle=True, seed=a.seed)
            self.val_sampler = ShardSampler(self.n_val, ws, rk, shuffle=True, seed=a.seed)
        elif a.data == "records":
            from ..data.records import RecordFile
            root = a.data_root or os.path.join(os.path.abspath(os.path.join(".", os.pardir)), "data/imagenet")
            self.train_set = RecordFile(os.path.join(root, "train.imrec"), threads=a.workers)
            self.val_set = RecordFile(os.path.join(root, "val.imrec"), threads=a.workers)
            H, W, _ = self.train_set.shape
            if (H < size[0] or W < size[1]) and not getattr(a, "record_resize", False):
                raise SystemExit(f"records hold {H}x{W} images, smaller than --image-size {a.image_size} "
                                 "(--record-resize: resample them on the GPU)")
            self.num_classes = self.train_set.num_classes
            self.n_train, self.n_val = len(self.train_set), len(self.val_set)
            self.train_sampler = ShardSampler(self.n_train, ws, rk, shuffle=True, seed=0)
            self.val_sampler = ShardSampler(self.n_val, ws, rk, shuffle=True, seed=0)
        else:
            from ..data.imagenet import ImageNetU8
            root = a.data_root or os.path.join(os.path.abspath(os.path.join(".", os.pardir)), "data/imagenet")
            self.train_set = ImageNetU8(root, "train", size)
            self.val_set = ImageNetU8(root, "val", size)
            self.num_classes = len(self.train_set.classes)
            self.n_train, self.n_val = len(self.train_set), len(self.val_set)
            # imagenet.py:346-347: shuffle=True for BOTH samplers (quirk Q2 kept)
            self.train_sampler = ShardSampler(self.n_train, ws, rk, shuffle=True, seed=0)
            self.val_sampler = ShardSampler(self.n_val, ws, rk, shuffle=True, seed=0)
        _master_print(self.is_master, "Training samples: {} images ".format(self.n_train))
        _master_print(self.is_master, "Test samples: {} images ".format(self.n_val))
        _master_print(self.is_master, "number of classes: {}".format(self.num_classes))
        self.dtype = {"bf16": torch.bfloat16, "fp8": torch.bfloat16, "fp32": torch.float32}[a.dtype]
        if a.dtype == "fp8" and self.kernels != "hip":
            raise SystemExit("--dtype fp8 needs the HIP kernels (--kernels hip on a MI355X)")
        rs = getattr(a, "record_resize", False)
        self.transform_train = InputTransform(self.kernels, size, cpad=resnet.ResNet.STEM_CPAD,
                                              flip=a.flip, dtype=torch.float32, resize=rs)
        self.transform_val = InputTransform(self.kernels, size, cpad=resnet.ResNet.STEM_CPAD,
                                            dtype=torch.float32, resize=rs)

    def _loaders(self, epoch: int):
        a = self.args
        self.train_sampler.set_epoch(epoch)   # imagenet.py:375 (val sampler stays at epoch 0)
        if a.data == "synthetic":
            nt = self.train_sampler.num_batches(a.batch_size)
            nv = self.val_sampler.num_batches(a.batch_size)
            return (SyntheticLoader(self.train_src, nt, self.transform_train),
                    SyntheticLoader(self.val_src, nv, self.transform_val))
        if not hasattr(self, "_train_dl") and a.data == "records":
            from ..data.records import RecordLoader
            self._train_dl = RecordLoader(self.train_set, self.train_sampler, a.batch_size, self.transform_train,
                                          self.device)
            self._val_dl = RecordLoader(self.val_set, self.val_sampler, a.batch_size, self.transform_val,
                                        self.device)
        if not hasattr(self, "_train_dl"):
            self._train_dl = DeviceLoader(self.train_set, self.train_sampler, a.batch_size,
                                          self.transform_train, self.device, a.workers)
            self._val_dl = DeviceLoader(self.val_set, self.val_sampler, a.batch_size, self.transform_val,
                                        self.device, a.workers)
        return self._train_dl, self._val_dl

    # ------------------------------------------------------------ model
    def _build_model(self):
        a = self.args
        _master_print(self.is_master, "Initialize Model...")
        model = resnet.build(a.arch, num_classes=self.num_classes)
        nparams = len(list(model.parameters()))
        order = list(reversed(range(nparams)))  # backward produces grads roughly in reverse
        self.native = None
        if self.kernels == "hip_f32":
            from ..models.native_f32 import bind_native_f32
            self.native = bind_native_f32(model, self.device, order)
            arena = self.native.arena
        elif self.kernels == "hip":
            from ..models.native import bind_native
            if getattr(a, "deterministic", False):
                from ..ops.conv import set_deterministic
                set_deterministic(True)
            # IMAGENT_WGRAD_OVERLAP=0: weight gradients on the main stream (A/B and diagnostics)
            self.native = bind_native(model, self.device, order, fp8=a.dtype == "fp8",
                                      wgrad_overlap=os.environ.get("IMAGENT_WGRAD_OVERLAP", "1") != "0")
            arena = self.native.arena
        else:
            model.to(self.device)
            arena = ParamArena(list(model.named_parameters()), self.device, order=order)
        self.model = model
        self.arena = arena
        self.comm = make_communicator(self.ctx, a.comm)
        self.ddp = DataParallel(model, arena, self.comm, bucket_cap_mb=a.bucket_mb,
                                first_bucket_mb=a.first_bucket_mb, broadcast_buffers=a.broadcast_buffers,
                                rebuild_buckets=a.rebuild_buckets,
                                grad_reduce_dtype=getattr(a, "grad_allreduce_dtype", "fp32"))
        if self.native is not None:  # the rank-0 broadcast may have rewritten the fp32 masters
            self.native.refresh_shadows(full=True)
        after = self.native.refresh_shadows if self.native else None
        full = (lambda: self.native.refresh_shadows(full=True)) if self.native else None
        self.opt = build_optimizer(a.optimizer, arena, a.lr, a.momentum, a.wd, a.nesterov,
                                   after_step=after, full_refresh=full,
                                   schedule_decay=a.schedule_decay, lars_eta=a.lars_eta)
        self.metrics = DeviceMetrics(self.device)
        from ..utils.profiling import StepTimer
        self.timer = StepTimer(enabled=self.device.type == "cuda")
        self.last_step_pct = {}
        ac = None
        if self.kernels == "torch" and self.device.type == "cuda" and a.dtype == "bf16":
            ac = torch.bfloat16
        self.step = StepRunner(self.ddp, self.opt, self.metrics, self.kernels, a.label_smoothing, ac)
        self.watchdog = None
        if a.step_timeout > 0:
            from ..utils.watchdog import Watchdog
            self.watchdog = Watchdog(a.step_timeout, aborts=[self.comm.abort, _abort_c10d],
                                     label=f"rank {self.ctx.rank}")
        self._graph_step = None
        if getattr(a, "hip_graph", False):
            if self.device.type != "cuda" or self.ctx.world_size > 1:
                raise SystemExit("--hip-graph: single-GPU runs only (the RCCL path is not captured)")
            self._graph_step = GraphedStep(lambda x, y: self.step.train_step([(x, y)]), warmup=3,
                                           key_fn=lambda: self.opt.param_groups[0]["lr"])
        self.start_epoch = 0
        self.best = dict(top1=0.0, top5=0.0, epoch_top1=0, epoch_top5=0, time=0.0)
        if a.resume and os.path.exists(a.resume):
            st = ckpt.load_state(a.resume, model, self.opt)
            if self.native:
                self.native.refresh_shadows(full=True)
            self.start_epoch = st["epoch"] + 1
            self.best.update(st.get("best", {}))
            _master_print(self.is_master, f"Resumed from {a.resume} at epoch {self.start_epoch}")
            self.ddp.sync_buffers()
            if self.comm.world_size > 1:
                self.comm.broadcast_(self.arena.P, 0)
        ipe = self.train_sampler.num_batches(a.batch_size)
        gb = a.batch_size * self.ctx.world_size
        self.sched = Schedule(a.lr, a.epochs, ipe, a.lr_schedule, a.lr_step, a.lr_gamma, a.warmup_epochs,
                              scale_batch=gb if a.scale_lr else 0)

    # ------------------------------------------------------------ loops
    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def train_epoch(self, epoch: int, train_loader) -> Tuple[float, float, float, float]:
        a = self.args
        self.model.train()
        self.metrics.reset()
        lr = self.sched.apply(self.opt, epoch)
        per_iter = self.sched.warmup > 0 or self.sched.kind == "cosine"
        self._sync()
        t0 = time.time()
        tlog, nlog = t0, 0
        accum = max(1, a.accum_steps)
        micro = []
        it = 0
        max_steps = a.max_steps if a.max_steps > 0 else math.inf
        data_wait = 0.0  # host time blocked on the input pipeline (quirk Q3: measured AND reported)
        data_time, batch_time = AverageMeter("data"), AverageMeter("batch")  # imagenet.py:99-100, per log line
        loader_it = iter(train_loader)
        tb = time.perf_counter()
        graph = self._graph_step if (accum == 1 and not per_iter) else None
        while True:
            tw = time.perf_counter()
            try:
                x, y = next(loader_it)
            except StopIteration:
                break
            data_wait += time.perf_counter() - tw
            data_time.update(time.perf_counter() - tw)
            micro.append((x, y))
            if len(micro) < accum:
                continue
            if per_iter:
                lr = self.sched.apply(self.opt, epoch, it)
            if self.watchdog:   # hang detector: no beat for --step-timeout s -> stacks, abort, exit
                self.watchdog.beat(f"epoch {epoch + 1} step {it}")
            maybe_stall(self.ctx.rank, it)
            self.timer.mark()
            if graph is not None:
                graph(*micro[0])
            else:
                self.step.train_step(micro)
            if a.check_consistency and (it + 1) % a.check_consistency == 0:
                self.ddp.check_consistency()
            # one-time bucket rebuild from the observed ready order (iteration 1)
            if getattr(self.ddp, "pending_relayout", None) is not None:
                self.opt.set_flats(self.ddp.apply_pending_relayout(self.opt.flats()))
                if self.native:
                    self.native.rebind()
            micro = []
            it += 1
            nlog += 1
            now_b = time.perf_counter()
            batch_time.update(now_b - tb)  # host-side (the GPU runs up to 2 steps behind)
            tb = now_b
            if a.log_interval and it % a.log_interval == 0:
                if not self.comm.healthy():  # asynchronous RCCL error: stop now, not at epoch end
                    raise RuntimeError("communicator reported an asynchronous error")
                loss, t1, t5, _ = self.metrics.reduced(self.comm)
                now = time.time()
                ips = nlog * a.batch_size * accum * self.ctx.world_size / (now - tlog)
                _master_print(self.is_master,
                              f"  epoch {epoch + 1} iter {it}/{len(train_loader) // accum} loss {loss:.4f} "
                              f"top1 {t1:.2f} top5 {t5:.2f} lr {lr:.4g} {ips:.1f} img/s | {batch_time} s "
                              f"| {data_time} s")
                tlog, nlog = now, 0
            if it >= max_steps:
                break
        self.timer.mark()
        self._sync()
        dt = time.time() - t0
        loss, t1, t5, n = self.metrics.reduced(self.comm)
        self.last_train_images = n
        self.last_lr = lr
        self.last_data_wait = data_wait
        self.last_step_pct = self.timer.percentiles()
        self.timer.events.clear()
        return loss, t1, t5, dt

    @torch.no_grad()
    def validate(self, val_loader) -> Tuple[float, float, float, float]:
        a = self.args
        if self.args.broadcast_buffers != "never":
            self.ddp.sync_buffers()
        self.model.eval()
        self.metrics.reset()
        self._sync()
        t0 = time.time()
        max_steps = a.max_val_steps if a.max_val_steps > 0 else math.inf
        for i, (x, y) in enumerate(val_loader):
            if self.watchdog:
                self.watchdog.beat(f"validation step {i}")
            self.step.eval_step(x, y)
            if i + 1 >= max_steps:
                break
        self._sync()
        dt = time.time() - t0
        loss, t1, t5, _ = self.metrics.reduced(self.comm)
        return loss, t1, t5, dt

    # ------------------------------------------------------------ driver
    def run(self) -> Dict:
        a = self.args
        total = self.best.get("time", 0.0)
        history = []
        for epoch in range(self.start_epoch, a.epochs):
            train_loader, val_loader = self._loaders(epoch)
            tr_loss, tr1, tr5, t_train = self.train_epoch(epoch, train_loader)
            lr = self.last_lr
            va_loss, va1, va5, t_val = self.validate(val_loader)
            total += t_train + t_val
            # checkpoint I/O is not a hang: every rank disarms its watchdog BEFORE the master starts
            # writing (the others would otherwise start the next epoch, block in its first collective
            # and time out while the master writes), and all ranks meet in a barrier after the writes,
            # still disarmed; the next step's beat re-arms
            if self.watchdog:
                self.watchdog.pause()
            if va1 > self.best["top1"]:   # imagenet.py:388-392
                self.best["top1"], self.best["epoch_top1"] = va1, epoch
                if self.is_master and a.save_model:
                    ckpt.save_best(self.model, a.arch, a.checkpoint_dir or ".")
            if va5 > self.best["top5"]:
                self.best["top5"], self.best["epoch_top5"] = va5, epoch
            self.best["time"] = total
            ips = self.last_train_images / max(t_train, 1e-9)
            if self.is_master:   # imagenet.py:397-403
                print(f"Epoch {epoch+1} Summary: ")
                print(f"\tLearning rate: {lr}")
                print(f"\tTrain loss: {tr_loss} ; Test loss: {va_loss}")
                print(f"\tTrain top1 accuracy: {tr1} ; Test top1 accuracy: {va1}")
                print(f"\tTrain top5 accuracy: {tr5} ; Test top5 accuracy: {va5}")
                print(f"\tTrain time: {t_train} seconds; Test time:{t_val} seconds")
                print(f"\tThroughput: {ips:.1f} img/s (job), {ips / self.ctx.world_size:.1f} img/s/GPU",
                      flush=True)
                print(f"\tData wait (host blocked on input): {self.last_data_wait:.2f} seconds", flush=True)
                if self.last_step_pct:
                    p = self.last_step_pct
                    print(f"\tStep time ms p50/p90/p99: {p[50]:.2f}/{p[90]:.2f}/{p[99]:.2f}", flush=True)
                if self.device.type == "cuda":
                    print(f"\tPeak HBM allocated: {torch.cuda.max_memory_allocated(self.device) / 2**30:.2f} GiB",
                          flush=True)
                if self.tb:   # imagenet.py:405-421 (lr step 0-based, quirk Q4 kept)
                    self.tb.add_scalars("Loss", {"train": tr_loss, "val": va_loss}, epoch + 1)
                    self.tb.add_scalars("Top1 accuracy", {"train": tr1, "val": va1}, epoch + 1)
                    self.tb.add_scalars("Top5 accuracy", {"train": tr5, "val": va5}, epoch + 1)
                    self.tb.add_scalar("lr", lr, epoch)
                    self.tb.add_scalar("throughput_img_s", ips, epoch + 1)
            history.append(dict(epoch=epoch + 1, lr=lr, train_loss=tr_loss, val_loss=va_loss, train_top1=tr1,
                                val_top1=va1, train_top5=tr5, val_top5=va5, train_time=t_train,
                                val_time=t_val, img_s=ips))
            if a.checkpoint_dir and self.is_master:
                slow_save()  # fault injection (IMAGENT_FAULT_SLOW_SAVE)
                ckpt.save_state(os.path.join(a.checkpoint_dir, f"state_{a.arch}.pt"), self.model, self.opt,
                                epoch, self.best)
            if self.watchdog and (a.save_model or a.checkpoint_dir):
                self.ctx.barrier()  # nobody re-arms until the master's writes are done
            if not self.comm.healthy():
                raise RuntimeError("communicator reported an asynchronous error")
        if self.is_master:   # imagenet.py:422-429
            print("\n")
            print("Training Summary:")
            print(f"\tTop1 best epoch: {self.best['epoch_top1']}")
            print(f"\t Best Test top1 accuracy: {self.best['top1']}")
            print(f"\tTop5 best epoch: {self.best['epoch_top5']}")
            print(f"\t Best Test top5 accuracy: {self.best['top5']}")
            print(f"\tTraining time: {total/60} minutes", flush=True)
        return dict(best=self.best, history=history)

    def close(self):
        if self.watchdog:
            self.watchdog.close()
        if self.tb:
            self.tb.close()
        self.comm.close()
        self.ctx.shutdown()
