"""FedAvg-paper CNNs (reference: `model/cv/cnn.py:5-142`).

CNN_OriginalFedAvg: 1,663,370 params (digits); CNN_DropOut: 1,199,882 params (digits)."""
import torch
import torch.nn as nn


class CNN_OriginalFedAvg(nn.Module):
    def __init__(self, only_digits=True):
        super().__init__()
        self.only_digits = only_digits
        self.conv2d_1 = nn.Conv2d(1, 32, kernel_size=5, padding=2)
        self.max_pooling = nn.MaxPool2d(2, stride=2)
        self.conv2d_2 = nn.Conv2d(32, 64, kernel_size=5, padding=2)
        self.flatten = nn.Flatten()
        self.linear_1 = nn.Linear(3136, 512)
        self.linear_2 = nn.Linear(512, 10 if only_digits else 62)
        self.relu = nn.ReLU()

    def forward(self, x):
        x = x.reshape(x.shape[0], 1, 28, 28)   # accepts [B,784], [B,28,28], [B,1,28,28]
        x = self.max_pooling(self.relu(self.conv2d_1(x)))
        x = self.max_pooling(self.relu(self.conv2d_2(x)))
        x = self.relu(self.linear_1(self.flatten(x)))
        return self.linear_2(x)


class CNN_DropOut(nn.Module):
    def __init__(self, only_digits=True):
        super().__init__()
        self.conv2d_1 = nn.Conv2d(1, 32, kernel_size=3)
        self.max_pooling = nn.MaxPool2d(2, stride=2)
        self.conv2d_2 = nn.Conv2d(32, 64, kernel_size=3)
        self.dropout_1 = nn.Dropout(0.25)
        self.flatten = nn.Flatten()
        self.linear_1 = nn.Linear(9216, 128)
        self.dropout_2 = nn.Dropout(0.5)
        self.linear_2 = nn.Linear(128, 10 if only_digits else 62)
        self.relu = nn.ReLU()

    def forward(self, x):
        x = x.reshape(x.shape[0], 1, 28, 28)
        x = self.relu(self.conv2d_1(x))
        x = self.relu(self.conv2d_2(x))
        x = self.dropout_1(self.max_pooling(x))
        x = self.dropout_2(self.relu(self.linear_1(self.flatten(x))))
        return self.linear_2(x)
