"""FedGKT model split (reference: `model/cv/resnet56_gkt/*`): a small on-client ResNet
(stem + a few BasicBlocks, returns (logits, features)) and a large server ResNet that
continues from the client's 16-channel 32×32 feature maps."""
import torch
import torch.nn as nn

from .resnet import BasicBlock, Bottleneck


class ResNetClient(nn.Module):
    """resnet8-style client net: conv stem + `n` BasicBlocks at 16 channels."""

    def __init__(self, num_classes=10, n_blocks=2):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 16, 3, 1, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(16)
        self.relu = nn.ReLU(inplace=True)
        self.layer1 = nn.Sequential(*[BasicBlock(16, 16) for _ in range(n_blocks)])
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(16, num_classes)

    def forward(self, x):
        feat = self.layer1(self.relu(self.bn1(self.conv1(x))))
        logits = self.fc(self.avgpool(feat).flatten(1))
        return logits, feat


class ResNetServer(nn.Module):
    """Bottleneck ResNet that consumes 16×32×32 client features (resnet56/110 trunk)."""

    def __init__(self, num_classes=10, layers=(6, 6, 6)):
        super().__init__()
        self.inplanes = 16
        self.layer1 = self._make(Bottleneck, 16, layers[0], 1)
        self.layer2 = self._make(Bottleneck, 32, layers[1], 2)
        self.layer3 = self._make(Bottleneck, 64, layers[2], 2)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(64 * Bottleneck.expansion, num_classes)

    def _make(self, block, planes, blocks, stride):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes * block.expansion, 1, stride, bias=False),
                                 nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, down)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, feat):
        x = self.layer3(self.layer2(self.layer1(feat)))
        return self.fc(self.avgpool(x).flatten(1))


def resnet8_56(c=10):
    return ResNetClient(c, 2)


def resnet56_server(c=10):
    return ResNetServer(c, (6, 6, 6))


def resnet110_server(c=10):
    return ResNetServer(c, (12, 12, 12))
