"""VGG-11/13/16/19 with BN (reference: `model/cv/vgg.py:20-203`)."""
import torch.nn as nn

_CFG = {
    "vgg11": [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "vgg13": [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "vgg16": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
    "vgg19": [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"],
}


class VGG(nn.Module):
    def __init__(self, name="vgg11", num_classes=10, batch_norm=True):
        super().__init__()
        layers, c = [], 3
        for v in _CFG[name]:
            if v == "M":
                layers.append(nn.MaxPool2d(2, 2))
            else:
                layers += [nn.Conv2d(c, v, 3, padding=1)] + ([nn.BatchNorm2d(v)] if batch_norm else []) + [nn.ReLU(inplace=True)]
                c = v
        self.features = nn.Sequential(*layers)
        self.classifier = nn.Sequential(nn.Linear(512, 512), nn.ReLU(True), nn.Linear(512, 512), nn.ReLU(True),
                                        nn.Linear(512, num_classes))

    def forward(self, x):
        x = self.features(x)
        x = nn.functional.adaptive_avg_pool2d(x, 1).flatten(1)
        return self.classifier(x)


def vgg11(num_classes=10):
    return VGG("vgg11", num_classes)


def vgg16(num_classes=10):
    return VGG("vgg16", num_classes)
