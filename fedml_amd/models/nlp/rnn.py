"""LSTM language models (reference: `model/nlp/rnn.py:5-86`).

RNN_OriginalFedAvg: Embedding(90, 8) → 2×LSTM(256) → FC(90), last-step logits (822,570 params).
RNN_StackOverFlow: Embedding(10004, 96) → LSTM(670) → FC(96) → FC(10004), [B, V, L] logits."""
import torch
import torch.nn as nn


class RNN_OriginalFedAvg(nn.Module):
    def __init__(self, embedding_dim=8, vocab_size=90, hidden_size=256):
        super().__init__()
        self.embeddings = nn.Embedding(vocab_size, embedding_dim, padding_idx=0)
        self.lstm = nn.LSTM(embedding_dim, hidden_size, num_layers=2, batch_first=True)
        self.fc = nn.Linear(hidden_size, vocab_size)

    def forward(self, input_seq):
        out, _ = self.lstm(self.embeddings(input_seq))
        return self.fc(out[:, -1])


class RNN_StackOverFlow(nn.Module):
    def __init__(self, vocab_size=10000, num_oov_buckets=1, embedding_size=96, latent_size=670, num_layers=1):
        super().__init__()
        ext = vocab_size + 3 + num_oov_buckets
        self.word_embeddings = nn.Embedding(ext, embedding_size, padding_idx=0)
        self.lstm = nn.LSTM(embedding_size, latent_size, num_layers=num_layers, batch_first=True)
        self.fc1 = nn.Linear(latent_size, embedding_size)
        self.fc2 = nn.Linear(embedding_size, ext)

    def forward(self, input_seq, hidden_state=None):
        out, _ = self.lstm(self.word_embeddings(input_seq), hidden_state)
        return torch.transpose(self.fc2(self.fc1(out)), 1, 2)
