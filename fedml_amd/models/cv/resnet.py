"""CIFAR ResNets (reference: `model/cv/resnet.py:38-303`).

resnet56 = ResNet(Bottleneck, [6,6,6]) with 16/32/64 planes, expansion 4:
591,322 params for 10 classes / 614,452 for 100, 350 state_dict tensors — the
north-star workload. resnet110 = [12,12,12]. ``resnet18_cifar`` (BasicBlock
[2,2,2,2], 3×3 stem, 11.17 M params) is the north-star "ResNet-18 CIFAR-10"
model, which the reference does not ship.
"""
import torch
import torch.nn as nn

from ...ops.bn_ops import batch_norm_act


def conv3x3(in_planes, out_planes, stride=1, groups=1, dilation=1):
    return nn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=dilation, groups=groups,
                     bias=False, dilation=dilation)


def conv1x1(in_planes, out_planes, stride=1):
    return nn.Conv2d(in_planes, out_planes, kernel_size=1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1,
                 norm_layer=None):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = norm_layer(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = norm_layer(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        # act(bn(conv) [+ identity]) as one fused pass on NHWC bf16 GPU activations (ops.bn_ops)
        identity = x
        out = batch_norm_act(self.bn1, self.conv1(x), relu=True)
        if self.downsample is not None:
            ds = self.downsample
            if isinstance(ds, nn.Sequential) and len(ds) == 2 and isinstance(ds[1], nn.BatchNorm2d):
                identity = batch_norm_act(ds[1], ds[0](x))
            else:
                identity = ds(x)
        return batch_norm_act(self.bn2, self.conv2(out), residual=identity, relu=True)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1,
                 norm_layer=None):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        width = int(planes * (base_width / 64.0)) * groups
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = norm_layer(width)
        self.conv2 = conv3x3(width, width, stride, groups, dilation)
        self.bn2 = norm_layer(width)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = norm_layer(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        return self.relu(out + identity)


class ResNet(nn.Module):
    """3-stage CIFAR ResNet (stem 3→16, stages 16/32/64 planes)."""

    def __init__(self, block, layers, num_classes=10, zero_init_residual=False, groups=1, width_per_group=64,
                 norm_layer=None, KD=False):
        super().__init__()
        self._norm_layer = norm_layer or nn.BatchNorm2d
        self.inplanes = 16
        self.dilation = 1
        self.groups = groups
        self.base_width = width_per_group
        self.conv1 = nn.Conv2d(3, self.inplanes, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = self._norm_layer(self.inplanes)
        self.relu = nn.ReLU(inplace=True)
        self.layer1 = self._make_layer(block, 16, layers[0])
        self.layer2 = self._make_layer(block, 32, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 64, layers[2], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(64 * block.expansion, num_classes)
        self.KD = KD
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.constant_(m.bn3.weight, 0)
                elif isinstance(m, BasicBlock):
                    nn.init.constant_(m.bn2.weight, 0)

    def _make_layer(self, block, planes, blocks, stride=1):
        norm_layer = self._norm_layer
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       norm_layer(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample, self.groups, self.base_width, 1, norm_layer)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, groups=self.groups, base_width=self.base_width,
                                norm_layer=norm_layer))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.relu(self.bn1(self.conv1(x)))
        x = self.layer3(self.layer2(self.layer1(x)))
        x_f = torch.flatten(self.avgpool(x), 1)
        out = self.fc(x_f)
        return (x_f, out) if self.KD else out


def _load_pretrained(model, path):
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    sd = ckpt.get("state_dict", ckpt)
    model.load_state_dict({k.replace("module.", ""): v for k, v in sd.items()})
    return model


def resnet56(class_num, pretrained=False, path=None, **kwargs):
    model = ResNet(Bottleneck, [6, 6, 6], class_num, **kwargs)
    return _load_pretrained(model, path) if pretrained else model


def resnet110(class_num, pretrained=False, path=None, **kwargs):
    model = ResNet(Bottleneck, [12, 12, 12], class_num, **kwargs)
    return _load_pretrained(model, path) if pretrained else model


class ResNet18Cifar(nn.Module):
    """ResNet-18 for 32×32 inputs: 3×3 stem, no max-pool, stages 64/128/256/512."""

    def __init__(self, num_classes=10, norm_layer=None):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 3, 1, 1, bias=False)
        self.bn1 = norm_layer(64)
        self.relu = nn.ReLU(inplace=True)
        self.layer1 = self._make(64, 2, 1, norm_layer)
        self.layer2 = self._make(128, 2, 2, norm_layer)
        self.layer3 = self._make(256, 2, 2, norm_layer)
        self.layer4 = self._make(512, 2, 2, norm_layer)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def _make(self, planes, blocks, stride, norm_layer):
        down = None
        if stride != 1 or self.inplanes != planes:
            down = nn.Sequential(conv1x1(self.inplanes, planes, stride), norm_layer(planes))
        layers = [BasicBlock(self.inplanes, planes, stride, down, norm_layer=norm_layer)]
        self.inplanes = planes
        for _ in range(1, blocks):
            layers.append(BasicBlock(planes, planes, norm_layer=norm_layer))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = batch_norm_act(self.bn1, self.conv1(x), relu=True)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def resnet18_cifar(class_num=10, **kwargs):
    return ResNet18Cifar(class_num, **kwargs)
