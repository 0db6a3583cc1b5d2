"""MobileNetV3 LARGE/SMALL (reference: `model/cv/mobilenet_v3.py:148-316`)."""
import torch.nn as nn
import torch.nn.functional as F


def _make_divisible(v, divisor=8):
    new_v = max(divisor, int(v + divisor / 2) // divisor * divisor)
    return new_v + divisor if new_v < 0.9 * v else new_v


class HSwish(nn.Module):
    def forward(self, x):
        return x * F.relu6(x + 3.0) / 6.0


class HSigmoid(nn.Module):
    def forward(self, x):
        return F.relu6(x + 3.0) / 6.0


class SqueezeExcite(nn.Module):
    def __init__(self, c, r=4):
        super().__init__()
        self.fc1 = nn.Conv2d(c, _make_divisible(c // r), 1)
        self.fc2 = nn.Conv2d(_make_divisible(c // r), c, 1)
        self.act = HSigmoid()

    def forward(self, x):
        s = F.adaptive_avg_pool2d(x, 1)
        return x * self.act(self.fc2(F.relu(self.fc1(s))))


class InvertedResidual(nn.Module):
    def __init__(self, cin, k, exp, cout, se, act, stride):
        super().__init__()
        self.use_res = stride == 1 and cin == cout
        A = HSwish if act == "HS" else nn.ReLU
        layers = []
        if exp != cin:
            layers += [nn.Conv2d(cin, exp, 1, bias=False), nn.BatchNorm2d(exp), A()]
        layers += [nn.Conv2d(exp, exp, k, stride, k // 2, groups=exp, bias=False), nn.BatchNorm2d(exp), A()]
        if se:
            layers.append(SqueezeExcite(exp))
        layers += [nn.Conv2d(exp, cout, 1, bias=False), nn.BatchNorm2d(cout)]
        self.block = nn.Sequential(*layers)

    def forward(self, x):
        y = self.block(x)
        return x + y if self.use_res else y


_LARGE = [(16, 3, 16, 16, False, "RE", 1), (16, 3, 64, 24, False, "RE", 2), (24, 3, 72, 24, False, "RE", 1),
          (24, 5, 72, 40, True, "RE", 2), (40, 5, 120, 40, True, "RE", 1), (40, 5, 120, 40, True, "RE", 1),
          (40, 3, 240, 80, False, "HS", 2), (80, 3, 200, 80, False, "HS", 1), (80, 3, 184, 80, False, "HS", 1),
          (80, 3, 184, 80, False, "HS", 1), (80, 3, 480, 112, True, "HS", 1), (112, 3, 672, 112, True, "HS", 1),
          (112, 5, 672, 160, True, "HS", 2), (160, 5, 960, 160, True, "HS", 1), (160, 5, 960, 160, True, "HS", 1)]
_SMALL = [(16, 3, 16, 16, True, "RE", 2), (16, 3, 72, 24, False, "RE", 2), (24, 3, 88, 24, False, "RE", 1),
          (24, 5, 96, 40, True, "HS", 2), (40, 5, 240, 40, True, "HS", 1), (40, 5, 240, 40, True, "HS", 1),
          (40, 5, 120, 48, True, "HS", 1), (48, 5, 144, 48, True, "HS", 1), (48, 5, 288, 96, True, "HS", 2),
          (96, 5, 576, 96, True, "HS", 1), (96, 5, 576, 96, True, "HS", 1)]


class MobileNetV3(nn.Module):
    def __init__(self, model_mode="LARGE", num_classes=1000, multiplier=1.0, dropout_rate=0.0):
        super().__init__()
        cfg = _LARGE if model_mode == "LARGE" else _SMALL
        self.stem = nn.Sequential(nn.Conv2d(3, 16, 3, 2, 1, bias=False), nn.BatchNorm2d(16), HSwish())
        self.blocks = nn.Sequential(*[InvertedResidual(_make_divisible(i * multiplier), k, _make_divisible(e * multiplier),
                                                       _make_divisible(o * multiplier), se, a, s)
                                      for (i, k, e, o, se, a, s) in cfg])
        last_in = _make_divisible(cfg[-1][3] * multiplier)
        last_c = _make_divisible((960 if model_mode == "LARGE" else 576) * multiplier)
        head_c = 1280 if model_mode == "LARGE" else 1024
        self.last = nn.Sequential(nn.Conv2d(last_in, last_c, 1, bias=False), nn.BatchNorm2d(last_c), HSwish())
        self.head = nn.Sequential(nn.Conv2d(last_c, head_c, 1), HSwish(), nn.Dropout(dropout_rate),
                                  nn.Conv2d(head_c, num_classes, 1))

    def forward(self, x):
        x = self.last(self.blocks(self.stem(x)))
        return self.head(F.adaptive_avg_pool2d(x, 1)).flatten(1)
