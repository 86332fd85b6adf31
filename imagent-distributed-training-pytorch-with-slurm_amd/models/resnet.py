"""ResNet-18/34/50/101/152 with torchvision-identical parameter names.

The reference instantiates ``torchvision.models.resnet18(pretrained=False,
num_classes=1000)`` (``/root/reference/imagenet.py:312``); torchvision is not
available here, and the compute path is ours, so the family is re-declared
with the same module tree (``conv1, bn1, layer{1..4}.{i}.conv{1,2,3},
bn{1,2,3}, downsample.{0,1}, fc``), the same shapes and the same init
(kaiming-normal fan_out for convs, BN weight 1 / bias 0, nn.Linear default for
fc). ``state_dict()`` therefore matches torchvision key-for-key (122 keys for
ResNet-18, 320 for ResNet-50) and loads into it directly.
Bottleneck is v1.5 (stride on the 3x3 conv), as in torchvision.

Two execution backends share these parameters:

* ``backend='hip'``  - NHWC bf16 activations through the hand-written
  MI355X kernels (ops/*): MFMA implicit-GEMM convs with BN statistics fused
  into their epilogue, fused BN(+add)(+ReLU), fp32 master weights in a flat
  arena with bf16 shadows.
* ``backend='hip_f32'`` - NHWC fp32 through the fp32 kernels (models/native_f32.py),
  the reference's own precision.
* ``backend='torch'`` - NCHW through stock PyTorch ops: the numerical oracle
  for the kernel tests and the path used on CPU (gloo) runs.
"""

from __future__ import annotations

import math
from typing import Callable, List, Optional, Type, Union

import torch
import torch.nn as nn
import torch.nn.functional as F


# --------------------------------------------------------------------------
# parameter-holding modules (torchvision names, our own forward)
# --------------------------------------------------------------------------

class Conv2d(nn.Module):
    def __init__(self, cin: int, cout: int, k: int, stride: int = 1, padding: int = 0):
        super().__init__()
        self.in_channels, self.out_channels = cin, cout
        self.kh = self.kw = k
        self.stride, self.padding = stride, padding
        w = torch.empty(cout, cin, k, k)
        nn.init.kaiming_normal_(w, mode="fan_out", nonlinearity="relu")
        self.weight = nn.Parameter(w.contiguous(memory_format=torch.channels_last))
        # bf16 shadows bound by ResNet.bind_native()
        self.w_bf16: Optional[torch.Tensor] = None
        self.wt_bf16: Optional[torch.Tensor] = None

    def forward_torch(self, x):
        return F.conv2d(x, self.weight.to(x.dtype), None, self.stride, self.padding)

    def extra_repr(self):
        return (f"{self.in_channels}, {self.out_channels}, kernel_size=({self.kh}, {self.kw}), "
                f"stride=({self.stride}, {self.stride}), padding=({self.padding}, {self.padding})")


class BatchNorm2d(nn.Module):
    def __init__(self, c: int, eps: float = 1e-5, momentum: float = 0.1):
        super().__init__()
        self.num_features, self.eps, self.momentum = c, eps, momentum
        self.weight = nn.Parameter(torch.ones(c))
        self.bias = nn.Parameter(torch.zeros(c))
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))
        self.work = None  # BNWork, bound by ResNet.bind_native()

    def forward_torch(self, x):
        if self.training:
            self.num_batches_tracked.add_(1)
        return F.batch_norm(x, self.running_mean, self.running_var, self.weight.to(x.dtype),
                            self.bias.to(x.dtype), self.training, self.momentum, self.eps)

    def extra_repr(self):
        return f"{self.num_features}, eps={self.eps}, momentum={self.momentum}"


class Linear(nn.Module):
    def __init__(self, fin: int, fout: int):
        super().__init__()
        self.in_features, self.out_features = fin, fout
        w = torch.empty(fout, fin)
        b = torch.empty(fout)
        nn.init.kaiming_uniform_(w, a=math.sqrt(5))  # nn.Linear.reset_parameters
        bound = 1 / math.sqrt(fin)
        nn.init.uniform_(b, -bound, bound)
        self.weight = nn.Parameter(w)
        self.bias = nn.Parameter(b)
        self.w_bf16: Optional[torch.Tensor] = None
        self.wt_bf16: Optional[torch.Tensor] = None

    def forward_torch(self, x):
        return F.linear(x, self.weight.to(x.dtype), self.bias.to(x.dtype))


class BNWork:
    """Per-BN device workspace (views into one arena zeroed once per step)."""

    __slots__ = ("slab", "stats", "save", "scratch")

    def __init__(self, slab, stats, save, scratch):
        # slab [STAT_SLOTS, 2, C]: conv-epilogue (sum, sumsq) partials (zeroed per step)
        # stats [2, C]: folded sums; save [2, C]: (mean, invstd); scratch [3, C]: bwd sums
        self.slab, self.stats, self.save, self.scratch = slab, stats, save, scratch


# --------------------------------------------------------------------------
# blocks
# --------------------------------------------------------------------------

class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = Conv2d(inplanes, planes, 3, stride, 1)
        self.bn1 = BatchNorm2d(planes)
        self.conv2 = Conv2d(planes, planes, 3, 1, 1)
        self.bn2 = BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def convs_bns(self):
        return [(self.conv1, self.bn1, True), (self.conv2, self.bn2, False)]

    def forward_torch(self, x):
        out = F.relu(self.bn1.forward_torch(self.conv1.forward_torch(x)))
        out = self.bn2.forward_torch(self.conv2.forward_torch(out))
        idt = x if self.downsample is None else \
            self.downsample[1].forward_torch(self.downsample[0].forward_torch(x))
        return F.relu(out + idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = Conv2d(inplanes, planes, 1)
        self.bn1 = BatchNorm2d(planes)
        self.conv2 = Conv2d(planes, planes, 3, stride, 1)
        self.bn2 = BatchNorm2d(planes)
        self.conv3 = Conv2d(planes, planes * 4, 1)
        self.bn3 = BatchNorm2d(planes * 4)
        self.downsample = downsample
        self.stride = stride

    def convs_bns(self):
        return [(self.conv1, self.bn1, True), (self.conv2, self.bn2, True), (self.conv3, self.bn3, False)]

    def forward_torch(self, x):
        out = F.relu(self.bn1.forward_torch(self.conv1.forward_torch(x)))
        out = F.relu(self.bn2.forward_torch(self.conv2.forward_torch(out)))
        out = self.bn3.forward_torch(self.conv3.forward_torch(out))
        idt = x if self.downsample is None else \
            self.downsample[1].forward_torch(self.downsample[0].forward_torch(x))
        return F.relu(out + idt)


# --------------------------------------------------------------------------
# ResNet
# --------------------------------------------------------------------------

class ResNet(nn.Module):
    # NHWC input channels on the HIP path (3 real + 1 zero): the stem kernel
    # reads the 7 taps x 4 channels of a kernel row as one contiguous segment
    STEM_CPAD = 4

    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: List[int],
                 num_classes: int = 1000, zero_init_residual: bool = False):
        super().__init__()
        self.block = block
        self.inplanes = 64
        self.conv1 = Conv2d(3, 64, 7, 2, 3)
        self.bn1 = BatchNorm2d(64)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], 2)
        self.layer3 = self._make_layer(block, 256, layers[2], 2)
        self.layer4 = self._make_layer(block, 512, layers[3], 2)
        self.fc = Linear(512 * block.expansion, num_classes)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)
        self.backend = "torch"
        self.native = None  # NativeState when bound

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(Conv2d(self.inplanes, planes * block.expansion, 1, stride),
                                       BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    def blocks(self):
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            for b in layer:
                yield b

    def batchnorms(self) -> List[BatchNorm2d]:
        return [m for m in self.modules() if isinstance(m, BatchNorm2d)]

    def convs(self) -> List[Conv2d]:
        return [m for m in self.modules() if isinstance(m, Conv2d)]

    # ---------------------------------------------------------------- torch
    def forward_torch(self, x):
        x = F.relu(self.bn1.forward_torch(self.conv1.forward_torch(x)))
        x = F.max_pool2d(x, 3, 2, 1)
        for b in self.blocks():
            x = b.forward_torch(x)
        x = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
        return self.fc.forward_torch(x)

    # ------------------------------------------------------------------ hip
    def forward(self, x):
        if self.backend == "hip":
            from .native import forward_hip
            return forward_hip(self, x)
        if self.backend == "hip_f32":
            from .native_f32 import forward_hip_f32
            return forward_hip_f32(self, x)
        return self.forward_torch(x)


def _resnet(block, layers, **kw) -> ResNet:
    return ResNet(block, layers, **kw)


def resnet18(**kw) -> ResNet:
    return _resnet(BasicBlock, [2, 2, 2, 2], **kw)


def resnet34(**kw) -> ResNet:
    return _resnet(BasicBlock, [3, 4, 6, 3], **kw)


def resnet50(**kw) -> ResNet:
    return _resnet(Bottleneck, [3, 4, 6, 3], **kw)


def resnet101(**kw) -> ResNet:
    return _resnet(Bottleneck, [3, 4, 23, 3], **kw)


def resnet152(**kw) -> ResNet:
    return _resnet(Bottleneck, [3, 8, 36, 3], **kw)


ARCHS = {"resnet18": resnet18, "resnet34": resnet34, "resnet50": resnet50, "resnet101": resnet101,
         "resnet152": resnet152}


def build(arch: str, num_classes: int = 1000, **kw) -> ResNet:
    if arch not in ARCHS:
        raise ValueError(f"unknown arch {arch!r}; choose from {sorted(ARCHS)}")
    return ARCHS[arch](num_classes=num_classes, **kw)
