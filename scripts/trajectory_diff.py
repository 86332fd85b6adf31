"""Per-step trajectory diff of the HIP training loop against PyTorch on the HIP path's own weights.

Runs the real CLI trainer (``imagent_amd.train.engine.Trainer``, every flag passes through) on the HIP
kernels and, at EVERY optimizer step, before the HIP step runs, recomputes the same step from the HIP
path's current state (fp32 masters + BN running buffers) with stock PyTorch ops, twice: fp32 and bf16
autocast. Logged per step (JSONL): lr, the three losses, each path's per-parameter gradient relative error
against fp32 (global and worst layer), the BN running mean / var error after the step, gradient norms.
At every validation the HIP-trained weights are also evaluated by the PyTorch fp32 eval forward on the same
validation batches: a HIP eval loss that differs from it points at the folded-BN eval / running statistics,
not at the training dynamics.

Reference hot loop: /root/reference/imagenet.py:113-131 (forward / loss / backward / SGD step), :446 (lr).

    python scripts/trajectory_diff.py --out gpurun_out/traj_lr005.jsonl -- \
        --arch resnet18 --image-size 64 --data synthetic --synthetic-task colour --num-classes 10 \
        --batch-size 32 --synthetic-train-size 4800 --synthetic-val-size 1024 --lr 0.05 --epochs 2
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from imagent_amd.cli import build_parser  # noqa: E402
from imagent_amd.models import resnet  # noqa: E402
from imagent_amd.train.engine import Trainer  # noqa: E402


def to_nchw(x: torch.Tensor) -> torch.Tensor:
    """HIP model input (NHWC bf16, 4 channels, channel 3 zero) -> NCHW fp32 (the same bf16 values)."""
    return x[..., :3].permute(0, 3, 1, 2).float().contiguous()


def rel(a: torch.Tensor, b: torch.Tensor) -> float:
    d = (a.float() - b.float()).norm().item()
    n = b.float().norm().item()
    return d / n if n > 0 else (0.0 if d == 0 else math.inf)


class Tracer:
    def __init__(self, tr: Trainer, out, every: int = 1, eval_check: bool = True, lockstep: bool = False):
        self.tr, self.out, self.every = tr, out, max(1, every)
        self.lockstep = lockstep
        self.model = tr.model
        dev = tr.device
        self.ref = resnet.build(tr.args.arch, num_classes=tr.num_classes).to(dev)
        self.names = [n for n, _ in self.model.named_parameters()]
        self.bn_names = [n for n, m in self.model.named_modules() if isinstance(m, resnet.BatchNorm2d)]
        self.step = 0
        self.epoch_steps = 0
        self.eval_check = eval_check
        self._G = None
        self._loss = None
        st = tr.step
        self._orig_train_step = st.train_step
        self._orig_loss = st.loss
        st.train_step = self.train_step
        st.loss = self.loss
        self._orig_validate = tr.validate
        tr.validate = self.validate

    # ---- hooks
    def loss(self, logits, y):
        t = self._orig_loss(logits, y)
        if torch.is_grad_enabled():
            self._loss = t.detach()
        return t

    def _capture_opt(self):
        opt = self.tr.opt
        orig = opt.step

        def step():
            torch.cuda.synchronize()
            ar = self.tr.arena
            self._G = ar.G.clone()
            self._P = ar.P.clone()
            self._buf = opt.buf.clone() if getattr(opt, "buf", None) is not None else None
            opt.step = orig
            orig()
        opt.step = step

    def _check_update(self, rec):
        """The SGD step the HIP kernel took vs torch.optim.SGD's math from the same (P, G, momentum) (the
        reference's optimizer, imagenet.py:325), and the bf16 compute shadows vs the new masters."""
        opt, ar = self.tr.opt, self.tr.arena
        g = opt.param_groups[0]
        lr, mu, wd = g["lr"], g["momentum"], g["weight_decay"]
        d = self._G + wd * self._P
        if mu != 0:
            buf = d if self._buf is None else self._buf * mu + d
            d = buf
        want = self._P - lr * d
        rec["sgd_step_err"] = rel(ar.P - self._P, want - self._P)
        if ar.S is not None:
            rec["shadow_err"] = rel(ar.S.float(), ar.P.to(torch.bfloat16).float())

    def _ref_grads(self, sd, x, y, autocast: bool):
        ref = self.ref
        ref.load_state_dict(sd)
        ref.train()
        ref.zero_grad(set_to_none=True)
        xt = to_nchw(x)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
            logits = ref.forward_torch(xt)
        loss = F.cross_entropy(logits.float(), y)
        loss.backward()
        grads = {n: p.grad.detach().clone() for n, p in ref.named_parameters()}
        bufs = {n: (m.running_mean.clone(), m.running_var.clone())
                for n, m in ref.named_modules() if isinstance(m, resnet.BatchNorm2d)}
        return loss.item(), grads, bufs, logits.detach().float()

    # ---- lockstep: PyTorch fp32 and bf16-autocast trainers on their OWN trajectories from the same start
    def _lockstep_init(self):
        dev = self.tr.device
        sd = {k: v.detach().clone() for k, v in self.model.state_dict().items()}
        g = self.tr.opt.param_groups[0]
        self.lock = {}
        for name in ("fp32", "bf16"):
            m = resnet.build(self.tr.args.arch, num_classes=self.tr.num_classes).to(dev)
            m.load_state_dict(sd)
            o = torch.optim.SGD(m.parameters(), lr=g["lr"], momentum=g["momentum"], weight_decay=g["weight_decay"])
            self.lock[name] = (m, o)

    def _lockstep_step(self, x, y, lr, rec):
        xt = to_nchw(x)
        flat = {}
        for name, (m, o) in self.lock.items():
            m.train()
            o.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=name == "bf16"):
                logits = m.forward_torch(xt)
            loss = F.cross_entropy(logits.float(), y)
            loss.backward()
            for pg in o.param_groups:
                pg["lr"] = lr
            o.step()
            rec[f"lock_loss_{name}"] = loss.item()
            flat[name] = torch.cat([p.detach().reshape(-1) for _, p in sorted(m.named_parameters())])
        hip = torch.cat([p.detach().reshape(-1) for _, p in sorted(self.model.named_parameters())])
        n32 = flat["fp32"].norm().item()
        rec["dist_hip_fp32"] = (hip - flat["fp32"]).norm().item() / n32
        rec["dist_bf16_fp32"] = (flat["bf16"] - flat["fp32"]).norm().item() / n32
        rec["dist_hip_bf16"] = (hip - flat["bf16"]).norm().item() / n32

    def train_step(self, micro):
        if self.lockstep and not hasattr(self, "lock"):
            self._lockstep_init()
        trace = self.step % self.every == 0 and len(micro) == 1
        if not trace:
            self._orig_train_step(micro)
            self.step += 1
            return
        x, y = micro[0]
        torch.cuda.synchronize()
        sd = {k: v.detach().clone() for k, v in self.model.state_dict().items()}
        l32, g32, b32, lg32 = self._ref_grads(sd, x, y, False)
        l16, g16, b16, lg16 = self._ref_grads(sd, x, y, True)
        self._capture_opt()
        self._orig_train_step(micro)
        torch.cuda.synchronize()
        ar = self.tr.arena
        gh = {n: ar.view(self._G, i) for i, n in enumerate(ar.names)}
        lh = self._loss.item()
        rec = dict(step=self.step, lr=self.tr.opt.param_groups[0]["lr"], loss_hip=lh, loss_fp32=l32,
                   loss_bf16=l16)
        if hasattr(self.tr.opt, "buf"):
            self._check_update(rec)
        if self.lockstep:
            self._lockstep_step(x, y, rec["lr"], rec)
        eh, eb = {}, {}
        for n in self.names:
            eh[n] = rel(gh[n], g32[n])
            eb[n] = rel(g16[n], g32[n])
        num = sum((gh[n].float() - g32[n]).pow(2).sum().item() for n in self.names)
        num16 = sum((g16[n].float() - g32[n]).pow(2).sum().item() for n in self.names)
        den = sum(g32[n].pow(2).sum().item() for n in self.names)
        rec["gnorm_fp32"] = math.sqrt(den)
        rec["gnorm_hip"] = math.sqrt(sum(gh[n].float().pow(2).sum().item() for n in self.names))
        rec["gerr_hip"] = math.sqrt(num / den) if den > 0 else 0.0
        rec["gerr_bf16"] = math.sqrt(num16 / den) if den > 0 else 0.0
        worst = max(self.names, key=lambda n: eh[n] / max(eb[n], 1e-6))
        rec["worst_layer"] = worst
        rec["worst_hip"] = eh[worst]
        rec["worst_bf16"] = eb[worst]
        rec["max_layer_hip"] = max(eh.values())
        rec["max_layer_bf16"] = max(eb.values())
        # BN running statistics after this step: HIP vs the fp32 forward from the same buffers
        mods = dict(self.model.named_modules())
        rm = rv = rm16 = rv16 = 0.0
        for n in self.bn_names:
            m = mods[n]
            rm = max(rm, rel(m.running_mean, b32[n][0]))
            rv = max(rv, rel(m.running_var, b32[n][1]))
            rm16 = max(rm16, rel(b16[n][0], b32[n][0]))
            rv16 = max(rv16, rel(b16[n][1], b32[n][1]))
        rec.update(bn_rmean_err_hip=rm, bn_rvar_err_hip=rv, bn_rmean_err_bf16=rm16, bn_rvar_err_bf16=rv16)
        rec["logit_err_bf16"] = rel(lg16, lg32)
        if self.step < 3 or self.step % 50 == 0:
            rec["per_layer_hip"] = {n: round(eh[n], 5) for n in self.names}
            rec["per_layer_bf16"] = {n: round(eb[n], 5) for n in self.names}
        self.out.write(json.dumps(rec) + "\n")
        self.out.flush()
        if self.lockstep and self.step % 10 == 0:
            print(f"[lock] step {self.step} loss hip {lh:.4f} fp32 {rec['lock_loss_fp32']:.4f} bf16 "
                  f"{rec['lock_loss_bf16']:.4f} | |P_hip - P_fp32| {rec['dist_hip_fp32']:.3e} |P_bf16 - P_fp32| "
                  f"{rec['dist_bf16_fp32']:.3e} |P_hip - P_bf16| {rec['dist_hip_bf16']:.3e}", flush=True)
        if self.step % 10 == 0:
            print(f"[traj] step {self.step} lr {rec['lr']:.4g} loss hip {lh:.4f} fp32 {l32:.4f} bf16 {l16:.4f} | "
                  f"gerr hip {rec['gerr_hip']:.4f} bf16 {rec['gerr_bf16']:.4f} | worst {worst} "
                  f"{eh[worst]:.4f}/{eb[worst]:.4f} | bn var {rv:.2e}/{rv16:.2e} | sgd {rec.get('sgd_step_err', -1):.1e} "
                  f"shadow {rec.get('shadow_err', -1):.1e}", flush=True)
        self.step += 1

    @torch.no_grad()
    def validate(self, val_loader):
        res = self._orig_validate(val_loader)
        if not self.eval_check:
            return res
        # the same validation batches through the PyTorch fp32 eval forward on the HIP-trained state
        torch.cuda.synchronize()
        self.ref.load_state_dict({k: v.detach().clone() for k, v in self.model.state_dict().items()})
        self.ref.eval()
        tot = hits = n = 0.0
        for x, y in val_loader:
            logits = self.ref.forward_torch(to_nchw(x)).float()
            tot += F.cross_entropy(logits, y, reduction="sum").item()
            hits += (logits.argmax(1) == y).sum().item()
            n += y.numel()
        rec = dict(validate=True, after_step=self.step, hip_val_loss=res[0], hip_val_top1=res[1],
                   torch_eval_val_loss=tot / n, torch_eval_val_top1=100.0 * hits / n)
        for name, (m, _) in getattr(self, "lock", {}).items():
            m.eval()
            lt = nt = 0.0
            for x, y in val_loader:
                with torch.autocast("cuda", dtype=torch.bfloat16, enabled=name == "bf16"):
                    lg = m.forward_torch(to_nchw(x)).float()
                lt += F.cross_entropy(lg, y, reduction="sum").item()
                nt += y.numel()
            rec[f"lock_{name}_val_loss"] = lt / nt
            print(f"[lock] validate after step {self.step}: {name} trajectory val loss {lt / nt:.4f}", flush=True)
        self.out.write(json.dumps(rec) + "\n")
        self.out.flush()
        print(f"[traj] validate after step {self.step}: HIP eval loss {res[0]:.4f} top1 {res[1]:.2f} | torch eval "
              f"on HIP weights loss {rec['torch_eval_val_loss']:.4f} top1 {rec['torch_eval_val_top1']:.2f}",
              flush=True)
        return res


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--out", required=True)
    ap.add_argument("--every", type=int, default=1, help="trace every N-th step")
    ap.add_argument("--lockstep", action="store_true",
                    help="also train PyTorch fp32 and bf16-autocast models on their own trajectories from the same "
                         "start (same batches, lr, SGD) and log the parameter distances between the three")
    ap.add_argument("rest", nargs=argparse.REMAINDER, help="-- then trainer CLI flags")
    a = ap.parse_args()
    rest = a.rest[1:] if a.rest[:1] == ["--"] else a.rest
    args = build_parser().parse_args(["--kernels", "hip", "--quiet-banner", "--tb-dir", ""] + rest)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    t0 = time.time()
    with open(a.out, "w") as f:
        f.write(json.dumps(dict(config=vars(args))) + "\n")
        tr = Trainer(args)
        Tracer(tr, f, every=a.every, lockstep=a.lockstep)
        try:
            tr.run()
        finally:
            tr.close()
    print(f"[traj] done in {time.time() - t0:.1f} s -> {a.out}", flush=True)


if __name__ == "__main__":
    main()
