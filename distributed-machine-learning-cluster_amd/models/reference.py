"""Plain ``torch.nn`` reference networks (fp32 CPU oracle).

torchvision is not installed, so the architectures the reference serves —
``tch::vision::resnet::resnet18`` and ``tch::vision::alexnet::alexnet``
(reference: src/services.rs:515,521) — are written out here with the
torchvision/tch parameter naming (``conv1``, ``bn1``,
``layer{1..4}.{i}.{conv,bn}{1,2,3}``, ``downsample.{0,1}``, ``fc``;
``features.{0,3,6,8,10}``, ``classifier.{1,4,6}``), so a state dict maps 1:1
onto the ``.ot`` keys (with ``.`` <-> ``|``).

These modules are the numerics oracle for the HIP engine and the CPU
executor used by nodes without a GPU. ResNet-34/50 are included as the
wider model zoo (ResNet-50 is the BASELINE stretch config).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: nn.Module | None = None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return F.relu(y + idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: nn.Module | None = None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = F.relu(self.bn1(self.conv1(x)))
        y = F.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return F.relu(y + idt)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes: int = 1000):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make(block, 64, layers[0], 1)
        self.layer2 = self._make(block, 128, layers[1], 2)
        self.layer3 = self._make(block, 256, layers[2], 2)
        self.layer4 = self._make(block, 512, layers[3], 2)
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def _make(self, block, planes, blocks, stride):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(
                nn.Conv2d(self.inplanes, planes * block.expansion, 1, stride, bias=False),
                nn.BatchNorm2d(planes * block.expansion),
            )
        layers = [block(self.inplanes, planes, stride, down)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(F.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
        return self.fc(x)


class AlexNet(nn.Module):
    def __init__(self, num_classes: int = 1000):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2d(3, 64, 11, 4, 2), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2),
            nn.Conv2d(64, 192, 5, padding=2), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2),
            nn.Conv2d(192, 384, 3, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(384, 256, 3, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(256, 256, 3, padding=1), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2),
        )
        self.avgpool = nn.AdaptiveAvgPool2d((6, 6))
        self.classifier = nn.Sequential(
            nn.Dropout(), nn.Linear(256 * 6 * 6, 4096), nn.ReLU(inplace=True),
            nn.Dropout(), nn.Linear(4096, 4096), nn.ReLU(inplace=True),
            nn.Linear(4096, num_classes),
        )

    def forward(self, x):
        x = self.avgpool(self.features(x))
        return self.classifier(torch.flatten(x, 1))


ARCHS = {
    "resnet18": lambda n: ResNet(BasicBlock, [2, 2, 2, 2], n),
    "resnet34": lambda n: ResNet(BasicBlock, [3, 4, 6, 3], n),
    "resnet50": lambda n: ResNet(Bottleneck, [3, 4, 6, 3], n),
    "alexnet": lambda n: AlexNet(n),
}


def build(arch: str, num_classes: int = 1000, seed: int | None = 0, randomize_bn: bool = False) -> nn.Module:
    """Random-init reference model (the reference's pretrained weights are
    git-LFS stubs — pretrained_models/*.ot:1-3 — so every run uses random
    weights of the right architecture). ``randomize_bn`` draws non-trivial
    BN statistics so that BN folding is actually exercised by tests."""
    arch = arch[:-4] if arch.endswith("_fp8") else arch  # same weights; e4m3 is an engine precision mode
    if arch not in ARCHS:
        raise ValueError(f"unknown arch {arch!r}; choose from {sorted(ARCHS)}")
    g = torch.random.fork_rng() if seed is not None else None
    with (g if g is not None else torch.no_grad()):
        if seed is not None:
            torch.manual_seed(seed)
        m = ARCHS[arch](num_classes)
        if randomize_bn:
            with torch.no_grad():
                for mod in m.modules():
                    if isinstance(mod, nn.BatchNorm2d):
                        mod.weight.uniform_(0.5, 1.5)
                        mod.bias.uniform_(-0.2, 0.2)
                        mod.running_mean.uniform_(-0.2, 0.2)
                        mod.running_var.uniform_(0.5, 2.0)
    return m.eval()


def state_dict_f32(model: nn.Module) -> dict[str, torch.Tensor]:
    """Float32 parameters + BN running stats (drops num_batches_tracked)."""
    return {k: v.detach().float().contiguous() for k, v in model.state_dict().items()
            if not k.endswith("num_batches_tracked")}
