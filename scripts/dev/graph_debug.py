"""Dev: whole-step graph capture with / without the wgrad side stream."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from imagent_amd.data.loader import InputTransform
from imagent_amd.models import resnet
from imagent_amd.models.native import bind_native
from imagent_amd.parallel.comm import LocalCommunicator
from imagent_amd.parallel.ddp import DataParallel
from imagent_amd.train.engine import GraphedStep, StepRunner
from imagent_amd.train.meters import DeviceMetrics
from imagent_amd.train.optim import FlatSGD

overlap = int(sys.argv[1])
DEV = "cuda"
torch.manual_seed(21)
model = resnet.build("resnet18", num_classes=1000)
st = bind_native(model, DEV, wgrad_overlap=bool(overlap))
ddp = DataParallel(model, st.arena, LocalCommunicator(), rebuild_buckets=False)
opt = FlatSGD(st.arena, lr=0.05, momentum=0.9, weight_decay=1e-4, after_step=st.refresh_shadows)
runner = StepRunner(ddp, opt, DeviceMetrics(DEV), "hip")
tf = InputTransform("hip", (64, 64), cpad=resnet.ResNet.STEM_CPAD)
model.train()
imgs = torch.randint(0, 256, (8, 64, 64, 3), dtype=torch.uint8, device=DEV)
labs = torch.randint(0, 1000, (8,), device=DEV)


def one(u8, y):
    runner.train_step([(tf(u8), y)])


g = GraphedStep(one, warmup=2)
for i in range(5):
    g(imgs, labs)
    print("step", i, "replays", g.replays, flush=True)
torch.cuda.synchronize()
print("ok overlap", overlap)
