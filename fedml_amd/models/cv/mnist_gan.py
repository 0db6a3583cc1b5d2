"""MNIST GAN generator/discriminator (reference: `model/cv/mnist_gan.py:4-65`), used by FedGAN."""
import torch
import torch.nn as nn


class Generator(nn.Module):
    def __init__(self, nz=100):
        super().__init__()
        self.nz = nz
        self.main = nn.Sequential(
            nn.Linear(nz, 256), nn.LeakyReLU(0.2, True), nn.Linear(256, 512), nn.LeakyReLU(0.2, True),
            nn.Linear(512, 1024), nn.LeakyReLU(0.2, True), nn.Linear(1024, 784), nn.Tanh())

    def forward(self, z):
        return self.main(z).view(-1, 1, 28, 28)


class Discriminator(nn.Module):
    def __init__(self):
        super().__init__()
        self.main = nn.Sequential(
            nn.Linear(784, 1024), nn.LeakyReLU(0.2, True), nn.Dropout(0.3), nn.Linear(1024, 512),
            nn.LeakyReLU(0.2, True), nn.Dropout(0.3), nn.Linear(512, 256), nn.LeakyReLU(0.2, True), nn.Dropout(0.3),
            nn.Linear(256, 1), nn.Sigmoid())

    def forward(self, x):
        return self.main(x.reshape(x.shape[0], -1))


class MNISTGAN(nn.Module):
    """Container so one state_dict holds both nets (FedGAN aggregates them separately)."""

    def __init__(self, nz=100):
        super().__init__()
        self.netg = Generator(nz)
        self.netd = Discriminator()

    def forward(self, z):
        return self.netd(self.netg(z))
