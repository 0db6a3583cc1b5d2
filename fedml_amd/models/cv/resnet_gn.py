"""ImageNet-style ResNets with GroupNorm (reference: `model/cv/resnet_gn.py:26-239`,
custom `group_normalization.py` GroupNorm2d built on F.batch_norm).

``group_norm`` = channels per group (reference convention, 32 in the FedML
papers); 0 selects BatchNorm. GroupNorm runs through ``torch.nn.GroupNorm`` on
CPU and through the native GN kernel in the batched engine. resnet18 with 1000
classes has 11,689,512 parameters like the reference (note the reference's
model hub builds it with 1000 outputs even for fed_cifar100, Appendix A #13 —
here the hub passes ``output_dim``)."""
import torch.nn as nn


def norm2d(planes, num_channels_per_group=32):
    if num_channels_per_group and num_channels_per_group > 0:
        return nn.GroupNorm(max(1, planes // num_channels_per_group), planes, affine=True)
    return nn.BatchNorm2d(planes)


class BasicBlockGN(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, group_norm=0):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = norm2d(planes, group_norm)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = norm2d(planes, group_norm)
        self.downsample = downsample

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + identity)


class BottleneckGN(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, group_norm=0):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = norm2d(planes, group_norm)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = norm2d(planes, group_norm)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = norm2d(planes * 4, group_norm)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + identity)


class ResNetGN(nn.Module):
    def __init__(self, block, layers, num_classes=1000, group_norm=0):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = norm2d(64, group_norm)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make_layer(block, 64, layers[0], 1, group_norm)
        self.layer2 = self._make_layer(block, 128, layers[1], 2, group_norm)
        self.layer3 = self._make_layer(block, 256, layers[2], 2, group_norm)
        self.layer4 = self._make_layer(block, 512, layers[3], 2, group_norm)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, block, planes, blocks, stride, group_norm):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes * block.expansion, 1, stride, bias=False),
                                 norm2d(planes * block.expansion, group_norm))
        layers = [block(self.inplanes, planes, stride, down, group_norm)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes, group_norm=group_norm) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(self.avgpool(x).flatten(1))


def resnet18(num_classes=1000, group_norm=32, **kw):
    return ResNetGN(BasicBlockGN, [2, 2, 2, 2], num_classes, group_norm)


def resnet34(num_classes=1000, group_norm=32, **kw):
    return ResNetGN(BasicBlockGN, [3, 4, 6, 3], num_classes, group_norm)


def resnet50(num_classes=1000, group_norm=32, **kw):
    return ResNetGN(BottleneckGN, [3, 4, 6, 3], num_classes, group_norm)


def resnet101(num_classes=1000, group_norm=32, **kw):
    return ResNetGN(BottleneckGN, [3, 4, 23, 3], num_classes, group_norm)


def resnet152(num_classes=1000, group_norm=32, **kw):
    return ResNetGN(BottleneckGN, [3, 8, 36, 3], num_classes, group_norm)
