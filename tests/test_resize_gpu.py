"""GPU bilinear resample fused into the input normalise (--record-resize): records stored smaller than the model
input (e.g. 320^2 for 448^2 training) are resized on the device. Yardstick: fp32 PyTorch
``F.interpolate(bilinear, align_corners=False)`` + ToTensor/Normalize (imagenet.py:281-283), then bf16."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
MEAN, STD = (0.5, 0.45, 0.4), (0.5, 0.25, 0.3)


def _ref(u8, size, flip=None):
    x = F.interpolate(u8.permute(0, 3, 1, 2).float(), size=size, mode="bilinear", align_corners=False) / 255.0
    x = (x - torch.tensor(MEAN, device=u8.device).view(1, 3, 1, 1)) / torch.tensor(STD, device=u8.device).view(1, 3, 1, 1)
    if flip is not None:
        x = torch.where(flip.view(-1, 1, 1, 1).bool(), x.flip(3), x)
    return x.permute(0, 2, 3, 1)


@pytest.mark.parametrize("src,dst,cpad", [((320, 320), (448, 448), 4), ((256, 200), (224, 224), 4),
                                          ((97, 131), (64, 80), 8)])
def test_resize_normalize_matches_interpolate(src, dst, cpad):
    from imagent_amd.ops.misc import resize_normalize_u8
    torch.manual_seed(0)
    u8 = torch.randint(0, 256, (5,) + src + (3,), dtype=torch.uint8, device="cuda")
    flip = torch.tensor([0, 1, 0, 1, 1], dtype=torch.uint8, device="cuda")
    for fl in (None, flip):
        y = resize_normalize_u8(u8, dst, cpad, MEAN, STD, fl)
        assert y.shape == (5,) + dst + (cpad,) and y.dtype == torch.bfloat16
        ref = _ref(u8, dst, fl)
        err = (y[..., :3].float() - ref).abs()
        assert err.max().item() <= 2 ** -7 * ref.abs().max().item() + 1e-3, err.max().item()
        assert (y[..., 3:] == 0).all()


def test_input_transform_resize_path():
    from imagent_amd.data.loader import InputTransform
    u8 = torch.randint(0, 256, (3, 160, 160, 3), dtype=torch.uint8, device="cuda")
    hip = InputTransform("hip", (224, 224), cpad=4, resize=True, mean=MEAN, std=STD)(u8)
    cpu = InputTransform("torch", (224, 224), resize=True, mean=MEAN, std=STD)(u8.cpu())
    assert hip.shape == (3, 224, 224, 4) and cpu.shape == (3, 3, 224, 224)
    assert (hip[..., :3].float().cpu() - cpu.permute(0, 2, 3, 1)).abs().max().item() < 2e-2
