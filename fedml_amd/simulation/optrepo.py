"""Optimizer repository (reference: `single_process/fedopt/optrepo.py:7-63`): name → torch optimizer class."""
import torch


class OptRepo:
    name2cls = {cls.__name__.lower(): cls for cls in torch.optim.Optimizer.__subclasses__()}

    @classmethod
    def get_opt_names(cls):
        return sorted(cls.name2cls.keys())

    @classmethod
    def name2cls_fn(cls, name: str):
        try:
            return cls.name2cls[name.lower()]
        except KeyError:
            raise KeyError(f"optimizer {name} not found; known: {cls.get_opt_names()}")

    # reference spelling
    @classmethod
    def name2cls_(cls, name):
        return cls.name2cls_fn(name)


def server_optimizer(params, args):
    name = str(getattr(args, "server_optimizer", "sgd"))
    cls = OptRepo.name2cls_fn(name)
    kw = {"lr": float(getattr(args, "server_lr", 1.0))}
    if name.lower() == "sgd":
        kw["momentum"] = float(getattr(args, "server_momentum", 0.0) or 0.0)
    return cls(params, **kw)
