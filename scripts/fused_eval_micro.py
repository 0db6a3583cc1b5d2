"""Inference forward of C models (the valuation's chunk shape: 128 models × 64 validation images, ResNet-56 fp32):
ms per forward_eval call with the fused bottleneck kernels (FEDML_AMD_FUSED_EVAL, FEDML_AMD_BNECK_EVAL_VARIANT) —
one JSON line.  python scripts/fused_eval_micro.py [--models 128 --images 64 --iters 10]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--models", type=int, default=128)
    p.add_argument("--images", type=int, default=64)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--depth", type=int, default=56)
    a = p.parse_args()
    import torch
    from fedml_amd.core.arena import ParamLayout
    from fedml_amd.models.cv.resnet import resnet56, resnet110
    from fedml_amd.parallel.native_resnet import NativeResNetStep
    torch.manual_seed(0)
    base = resnet56(100) if a.depth == 56 else resnet110(100)
    layout = ParamLayout.from_module(base)
    flat = layout.flatten(base.state_dict(), device="cuda")
    arena = (flat.view(1, -1) + 0.01 * torch.randn(a.models, flat.numel(), device="cuda")).contiguous()
    x = torch.randn(a.models, a.images, 3, 32, 32, device="cuda")
    st = NativeResNetStep(base, layout, a.models, "cuda", eval_only=True)
    for _ in range(2):
        st.forward_eval(arena, x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        st.forward_eval(arena, x)
    torch.cuda.synchronize()
    ms = 1000 * (time.perf_counter() - t0) / a.iters
    print(json.dumps({"metric": "forward_eval ms per call", "value": round(ms, 3), "models": a.models,
                      "images": a.images, "depth": a.depth, "fused": os.environ.get("FEDML_AMD_FUSED_EVAL", "1"),
                      "variant": os.environ.get("FEDML_AMD_BNECK_EVAL_VARIANT", "5"),
                      "us_per_image": round(1000 * ms / (a.models * a.images), 3)}), flush=True)


if __name__ == "__main__":
    main()
