"""Logistic regression (reference: `model/linear/lr.py:4-11`): sigmoid(Linear(x))."""
import torch


class LogisticRegression(torch.nn.Module):
    def __init__(self, input_dim, output_dim):
        super().__init__()
        self.linear = torch.nn.Linear(input_dim, output_dim)

    def forward(self, x):
        return torch.sigmoid(self.linear(x.reshape(x.shape[0], -1)))
