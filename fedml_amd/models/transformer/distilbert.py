"""DistilBERT-base for sequence classification (north-star "FedOpt DistilBERT" workload;
absent from the reference). 6 layers, d=768, 12 heads, FFN 3072, vocab 30522, 512 positions,
random init (no checkpoint download in this environment): 66.96 M parameters + head."""
import torch
import torch.nn as nn

from .layers import PostLNBlock, init_weights


class DistilBertEmbeddings(nn.Module):
    def __init__(self, vocab=30522, dim=768, max_pos=512, dropout=0.1):
        super().__init__()
        self.word_embeddings = nn.Embedding(vocab, dim, padding_idx=0)
        self.position_embeddings = nn.Embedding(max_pos, dim)
        self.LayerNorm = nn.LayerNorm(dim, eps=1e-12)
        self.dropout = nn.Dropout(dropout)

    def forward(self, ids):
        pos = torch.arange(ids.shape[1], device=ids.device).unsqueeze(0)
        return self.dropout(self.LayerNorm(self.word_embeddings(ids) + self.position_embeddings(pos)))


class DistilBertForSequenceClassification(nn.Module):
    def __init__(self, num_labels=2, vocab=30522, dim=768, n_layers=6, n_heads=12, hidden=3072, max_pos=512,
                 dropout=0.1, seq_classif_dropout=0.2):
        super().__init__()
        self.embeddings = DistilBertEmbeddings(vocab, dim, max_pos, dropout)
        self.layer = nn.ModuleList([PostLNBlock(dim, n_heads, hidden, dropout) for _ in range(n_layers)])
        self.pre_classifier = nn.Linear(dim, dim)
        self.classifier = nn.Linear(dim, num_labels)
        self.dropout = nn.Dropout(seq_classif_dropout)
        init_weights(self)

    def forward(self, input_ids, attention_mask=None):
        if attention_mask is None:
            attention_mask = input_ids != 0
        h = self.embeddings(input_ids)
        for blk in self.layer:
            h = blk(h, attention_mask)
        pooled = torch.relu(self.pre_classifier(h[:, 0]))
        return self.classifier(self.dropout(pooled))


def distilbert(num_labels=2, **kw):
    return DistilBertForSequenceClassification(num_labels, **kw)
