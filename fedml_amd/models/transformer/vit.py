"""ViT-B/16 (north-star cross-silo workload; absent from the reference): 224×224 input,
16×16 patches (196 + CLS = 197 tokens), 12 pre-LN blocks, d=768, 12 heads, MLP 3072:
86.57 M parameters at 1000 classes. Random init."""
import torch
import torch.nn as nn

from .layers import PreLNBlock, init_weights


class PatchEmbed(nn.Module):
    def __init__(self, img_size=224, patch=16, in_chans=3, dim=768):
        super().__init__()
        self.num_patches = (img_size // patch) ** 2
        self.proj = nn.Conv2d(in_chans, dim, patch, patch)

    def forward(self, x):
        return self.proj(x).flatten(2).transpose(1, 2)


class VisionTransformer(nn.Module):
    def __init__(self, img_size=224, patch=16, in_chans=3, num_classes=1000, dim=768, depth=12, n_heads=12,
                 mlp_ratio=4.0, dropout=0.0):
        super().__init__()
        self.patch_embed = PatchEmbed(img_size, patch, in_chans, dim)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, self.patch_embed.num_patches + 1, dim))
        self.blocks = nn.ModuleList([PreLNBlock(dim, n_heads, int(dim * mlp_ratio), dropout) for _ in range(depth)])
        self.norm = nn.LayerNorm(dim, eps=1e-6)
        self.head = nn.Linear(dim, num_classes)
        init_weights(self)
        nn.init.normal_(self.pos_embed, std=0.02)
        nn.init.normal_(self.cls_token, std=0.02)

    def forward(self, x):
        x = self.patch_embed(x)
        x = torch.cat([self.cls_token.expand(x.shape[0], -1, -1), x], 1) + self.pos_embed
        for blk in self.blocks:
            x = blk(x)
        return self.head(self.norm(x)[:, 0])


def vit_b16(num_classes=1000, img_size=224, **kw):
    return VisionTransformer(img_size=img_size, num_classes=num_classes, **kw)


def vit_tiny(num_classes=10, img_size=32, patch=4, **kw):
    cfg = dict(dim=192, depth=4, n_heads=3)
    cfg.update(kw)
    return VisionTransformer(img_size=img_size, patch=patch, num_classes=num_classes, **cfg)
