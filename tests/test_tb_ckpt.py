"""TensorBoard event writer and checkpoint layout (imagenet.py:362-363, 387-421)."""

import os

import torch

from imagent_amd.models import resnet
from imagent_amd.utils import checkpoint as ck
from imagent_amd.utils import tb


def test_crc32c_known_vectors():
    assert tb.crc32c(b"123456789") == 0xE3069283
    assert tb.crc32c(b"") == 0


def test_event_roundtrip_and_layout(tmp_path):
    w = tb.SummaryWriter(str(tmp_path / "imagenet_FR"), jsonl=str(tmp_path / "m.jsonl"))
    w.add_scalars("Loss", {"train": 1.5, "val": 2.25}, 1)
    w.add_scalars("Top1 accuracy", {"train": 10.0, "val": 12.0}, 1)
    w.add_scalar("lr", 0.1, 0)
    w.close()
    d = tmp_path / "imagenet_FR"
    assert sorted(os.listdir(d)) == sorted(["Loss_train", "Loss_val", "Top1 accuracy_train",
                                            "Top1 accuracy_val"] + [f for f in os.listdir(d) if f.startswith("events")])
    ev = tb.read_events(str(next((d / "Loss_val").iterdir())))
    assert ev[1][1] == 1 and abs(ev[1][2]["Loss"] - 2.25) < 1e-6
    root = [f for f in os.listdir(d) if f.startswith("events")][0]
    ev = tb.read_events(str(d / root))
    assert abs(ev[1][2]["lr"] - 0.1) < 1e-7
    assert len(open(tmp_path / "m.jsonl").read().splitlines()) == 5


def test_reference_checkpoint_layout(tmp_path):
    m = resnet.resnet18()
    p = ck.save_best(m, "resnet18", str(tmp_path))
    assert os.path.basename(p) == "imagenet_FR_resnet18.pt"
    sd = torch.load(p, weights_only=True)
    assert len(sd) == 122
    assert all(k.startswith("module.") for k in sd)
    assert sum(k.endswith("num_batches_tracked") for k in sd) == 20
    assert sd["module.conv1.weight"].is_contiguous()
    assert sd["module.layer2.0.downsample.0.weight"].shape == (128, 64, 1, 1)
    assert sd._metadata["module.bn1"]["version"] == 2
    m50 = resnet.resnet50()
    assert len(ck.reference_state_dict(m50)) == 320
    # loads back (module. prefix stripped) bit-exactly
    m2 = resnet.resnet18()
    ck.load_reference_weights(m2, p)
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k


def test_full_state_resume_roundtrip(tmp_path):
    from imagent_amd.models.arena import ParamArena
    from imagent_amd.train.optim import FlatSGD
    m = resnet.resnet18(num_classes=10)
    ar = ParamArena(list(m.named_parameters()), "cpu", order=list(reversed(range(62))))
    opt = FlatSGD(ar, 0.1)
    ar.G.normal_()
    opt.step()
    p = ck.save_state(str(tmp_path / "s.pt"), m, opt, 4, {"top1": 1.0})
    m2 = resnet.resnet18(num_classes=10)
    ar2 = ParamArena(list(m2.named_parameters()), "cpu")   # different layout on purpose
    opt2 = FlatSGD(ar2, 0.5)
    st = ck.load_state(p, m2, opt2)
    assert st["epoch"] == 4 and st["best"]["top1"] == 1.0
    assert opt2.lr == 0.1
    for (n1, a), (n2, b) in zip(m.named_parameters(), m2.named_parameters()):
        assert torch.equal(a, b)
        i1, i2 = ar.names.index(n1), ar2.names.index(n2)
        assert torch.equal(ar.flat_slice(opt.buf, i1), ar2.flat_slice(opt2.buf, i2))
