"""ResNet-50 (BASELINE config 3: "ResNet-50 ImageNet-shape DDP bf16, 8
replicas over xGMI").  torchvision is not a dependency; this is the
standard v1.5 architecture (stride on the 3x3 conv of each bottleneck),
25,557,032 parameters at 1000 classes.

MI355X-first choices: activations in ``channels_last`` (NHWC, what the
MIOpen/hipBLASLt implicit-GEMM convolutions want for bf16 MFMA), bf16
autocast for convs/GEMMs with fp32 master parameters and fp32 BN
statistics, zero-init of the last BN gamma in each residual branch, and
the optimizer step as one multi-tensor HIP launch (``FusedSGD``).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops.bn import BatchNormAct
from ..ops.conv1x1 import GradStash, conv1x1, conv1x1_res, gemm_supported
from ..ops.conv3x3 import ConvStats, conv3x3
from ..ops.pool import MaxPool2d
from ..ops.stem import stem_conv


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, width: int, stride: int = 1, down: bool = False):
        super().__init__()
        cout = width * self.expansion
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = BatchNormAct(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = BatchNormAct(width)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)
        self.bn3 = BatchNormAct(cout)
        self.downsample = (nn.Sequential(nn.Conv2d(cin, cout, 1, stride=stride, bias=False), BatchNormAct(cout))
                           if down else None)

    def _c2(self, y):
        """The 3x3 conv + bn2 + ReLU: the MFMA implicit-GEMM kernel, whose
        epilogue hands bn2 its batch statistics (ops/conv3x3.py)."""
        st = ConvStats()
        return self.bn2(conv3x3(y, self.conv2, st), relu=True, stats=st)

    @staticmethod
    def _c1(conv, x, st=None):
        """1x1 convs (the downsample ones strided): MFMA forward handing the
        next BN its statistics (``st``), backward on hipBLASLt
        (ops/conv1x1.py)."""
        return conv1x1(x, conv, stats=st) if gemm_supported(x, conv) else conv(x)

    def forward(self, x):
        # BN + ReLU (+ the residual add) are one fused pass each way on the
        # GPU (ops/bn.py), with the batch statistics from the producing
        # conv's epilogue; in an identity block the residual's gradient is
        # folded into conv1's input-gradient GEMM instead of an autograd add
        # (ops/conv1x1.py); state-dict keys are the stock ones
        s1, s3 = ConvStats(), ConvStats()
        if self.downsample is None and gemm_supported(x, self.conv1, stride1=True) and self.bn3.can_fuse(x):
            stash = GradStash()
            y = self.bn1(conv1x1_res(x, self.conv1, stash, stats=s1), relu=True, stats=s1)
            y = self._c2(y)
            return self.bn3(self._c1(self.conv3, y, s3), residual=x, relu=True, stash=stash, stats=s3)
        if (self.downsample is not None and gemm_supported(x, self.downsample[0])
                and gemm_supported(x, self.conv1)):
            # both 1x1 convs read x: one input gradient, the second GEMM
            # accumulating onto the first (no autograd add)
            merge, sd = GradStash(), ConvStats()
            idt = self.downsample[1](conv1x1(x, self.downsample[0], merge, stats=sd), stats=sd)
            y = self.bn1(conv1x1(x, self.conv1, merge, stats=s1), relu=True, stats=s1)
            y = self._c2(y)
            return self.bn3(self._c1(self.conv3, y, s3), residual=idt, relu=True, stats=s3)
        idt = x if self.downsample is None else self.downsample[1](self._c1(self.downsample[0], x))
        y = self.bn1(self._c1(self.conv1, x), relu=True)
        y = self._c2(y)
        return self.bn3(self._c1(self.conv3, y), residual=idt, relu=True)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes: int = 1000, zero_init_residual: bool = True):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = BatchNormAct(64)
        self.maxpool = MaxPool2d(3, stride=2, padding=1)  # HIP gather-backward pool (ops/pool.py)
        cin, stages = 64, []
        for i, (n, width) in enumerate(zip(layers, (64, 128, 256, 512))):
            stride = 1 if i == 0 else 2
            blocks = [Bottleneck(cin, width, stride, down=True)]
            cin = width * Bottleneck.expansion
            blocks += [Bottleneck(cin, width) for _ in range(n - 1)]
            stages.append(nn.Sequential(*blocks))
        self.layer1, self.layer2, self.layer3, self.layer4 = stages
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(cin, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)

    def forward(self, x):
        x = self.maxpool(self.bn1(stem_conv(x, self.conv1), relu=True))  # MFMA stem kernel (ops/stem.py)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def resnet50(num_classes: int = 1000) -> ResNet:
    return ResNet((3, 4, 6, 3), num_classes)


def synthetic_images(batch: int, device, size: int = 224, num_classes: int = 1000, seed: int = 0,
                     channels_last: bool = True, dtype=torch.float32):
    """ImageNet-shaped synthetic batch (no dataset access)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(batch, 3, size, size, generator=g).to(device=device, dtype=dtype)
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, num_classes, (batch,), generator=g).to(device)
    return x, y
