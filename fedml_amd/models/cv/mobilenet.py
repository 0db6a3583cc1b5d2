"""MobileNet-v1 for CIFAR (reference: `model/cv/mobilenet.py:58-150`): depthwise-separable blocks."""
import torch.nn as nn


class DepthwiseSeparable(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.dw = nn.Conv2d(cin, cin, 3, stride, 1, groups=cin, bias=False)
        self.bn1 = nn.BatchNorm2d(cin)
        self.pw = nn.Conv2d(cin, cout, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        return self.relu(self.bn2(self.pw(self.relu(self.bn1(self.dw(x))))))


class MobileNet(nn.Module):
    cfg = [(64, 1), (128, 2), (128, 1), (256, 2), (256, 1), (512, 2), (512, 1), (512, 1), (512, 1), (512, 1),
           (512, 1), (1024, 2), (1024, 1)]

    def __init__(self, class_num=10, width=1.0):
        super().__init__()
        c0 = int(32 * width)
        self.stem = nn.Sequential(nn.Conv2d(3, c0, 3, 1, 1, bias=False), nn.BatchNorm2d(c0), nn.ReLU(inplace=True))
        layers, cin = [], c0
        for cout, s in self.cfg:
            cout = int(cout * width)
            layers.append(DepthwiseSeparable(cin, cout, s))
            cin = cout
        self.features = nn.Sequential(*layers)
        self.pool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(cin, class_num)

    def forward(self, x):
        return self.fc(self.pool(self.features(self.stem(x))).flatten(1))


def mobilenet(class_num=10, **kw):
    return MobileNet(class_num)
