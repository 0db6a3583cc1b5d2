import torch


def make_optimizer(params, args):
    """Reference convention: ``sgd`` → SGD(lr[, momentum, wd]); otherwise Adam(lr, wd, amsgrad=True)."""
    params = [p for p in params if p.requires_grad]
    opt = str(getattr(args, "client_optimizer", "sgd")).lower()
    lr = float(args.learning_rate)
    wd = float(getattr(args, "weight_decay", 0.0) or 0.0)
    if opt == "sgd":
        return torch.optim.SGD(params, lr=lr, momentum=float(getattr(args, "momentum", 0.0) or 0.0),
                               weight_decay=wd if getattr(args, "sgd_weight_decay", False) else 0.0)
    if opt == "adamw":
        return torch.optim.AdamW(params, lr=lr, weight_decay=wd)
    return torch.optim.Adam(params, lr=lr, weight_decay=wd, amsgrad=True)


def create_model_trainer(model, args):
    from .classification import ModelTrainerCLS
    from .nwp import ModelTrainerNWP
    from .tag_prediction import ModelTrainerTAGPred
    ds = getattr(args, "dataset", "")
    if ds == "stackoverflow_lr":
        return ModelTrainerTAGPred(model, args)
    if ds in ("fed_shakespeare", "stackoverflow_nwp"):
        return ModelTrainerNWP(model, args)
    return ModelTrainerCLS(model, args)
