"""``fedml_amd.model.create(args, output_dim)`` (reference: `model/model_hub.py:13-53`).

Same (model, dataset) → module mapping as the reference, including its
fallback to LogisticRegression, plus the north-star models the reference lacks
(``resnet18`` for CIFAR, ``distilbert``, ``vit_b16``) and the rest of the zoo
(resnet110, vgg, gan, darts, gkt split nets).
"""
import math
import logging

from .cv.cnn import CNN_DropOut, CNN_OriginalFedAvg
from .cv.darts import Network as DartsNetwork
from .cv.darts import Network_GumbelSoftmax, NetworkCIFAR
from .cv.efficientnet import EfficientNet
from .cv.mnist_gan import MNISTGAN
from .cv.mobilenet import mobilenet
from .cv.mobilenet_v3 import MobileNetV3
from .cv.resnet import resnet18_cifar, resnet56, resnet110
from .cv.resnet_gkt import resnet8_56, resnet56_server
from .cv.resnet_gn import resnet18 as resnet18_gn
from .cv.vgg import VGG
from .linear.lr import LogisticRegression
from .nlp.rnn import RNN_OriginalFedAvg, RNN_StackOverFlow
from .transformer.distilbert import distilbert
from .transformer.vit import vit_b16, vit_tiny

_INPUT_DIMS = {"mnist": 784, "stackoverflow_lr": 10000, "synthetic_1_1": 60, "mit-bih": 187,
               "lending_club_loan": 90, "NUS_WIDE": 1634, "UCI_SUSY": 18}


def create(args, output_dim):
    name = args.model
    ds = getattr(args, "dataset", "")
    logging.info("create_model. model_name = %s, output_dim = %s", name, output_dim)
    if name == "lr":
        dim = _INPUT_DIMS.get(ds)
        if dim is None:
            from ..data.synthetic import get_spec
            try:
                dim = int(math.prod(get_spec(ds).shape))
            except (KeyError, ValueError):
                dim = 28 * 28
        return LogisticRegression(dim, output_dim)
    if name == "cnn":
        if ds in ("femnist", "fed_emnist"):
            return CNN_DropOut(False)
        return CNN_DropOut(output_dim == 10)
    if name in ("deeplabv3_plus", "deeplab"):   # FedSeg (reference mpi_p2p_mp/fedseg): DeepLabV3+ backbones
        from .cv.segmentation import DeepLabV3PlusNet
        return DeepLabV3PlusNet(output_dim, str(getattr(args, "backbone", "resnet101")),
                                int(getattr(args, "outstride", getattr(args, "output_stride", 16)) or 16),
                                bool(getattr(args, "backbone_freezed", False)))
    if name == "unet":
        from .cv.segmentation import UNet
        return UNet(output_dim)
    if name == "cnn_original":
        return CNN_OriginalFedAvg(output_dim == 10)
    if name in ("resnet18_gn",):
        return resnet18_gn(num_classes=output_dim, group_norm=int(getattr(args, "group_norm_channels", 32)))
    if name == "rnn":
        if ds == "stackoverflow_nwp":
            return RNN_StackOverFlow()
        return RNN_OriginalFedAvg()
    if name == "resnet56":
        return resnet56(class_num=output_dim)
    if name == "resnet110":
        return resnet110(class_num=output_dim)
    if name in ("resnet18", "resnet18_cifar"):
        return resnet18_cifar(class_num=output_dim)
    if name == "mobilenet":
        return mobilenet(class_num=output_dim)
    if name == "mobilenet_v3":
        return MobileNetV3(model_mode=getattr(args, "model_mode", "LARGE"), num_classes=output_dim)
    if name == "efficientnet":
        return EfficientNet(num_classes=output_dim)
    if name.startswith("efficientnet-b"):   # compound-scaled variants (efficientnet_utils.py)
        return EfficientNet.from_name(name, output_dim, stem_stride=int(getattr(args, "stem_stride", 2)))
    if name.startswith("vgg"):
        return VGG(name, output_dim)
    if name in ("distilbert", "distilbert-base-uncased"):
        return distilbert(num_labels=output_dim, max_pos=int(getattr(args, "max_seq_len", 512)))
    if name in ("vit", "vit_b16", "vit-b/16"):
        return vit_b16(num_classes=output_dim, img_size=int(getattr(args, "img_size", 224)))
    if name == "vit_tiny":
        return vit_tiny(num_classes=output_dim)
    if name == "gan":
        return MNISTGAN(int(getattr(args, "nz", 100)))
    if name in ("darts", "darts_gdas", "gdas"):
        # FedNAS (reference fednas main): `stage: search` → the supernet (DARTS, or GDAS with
        # `search_method: gdas`); `stage: train` → the genotype network named by `arch` (default FedNAS_V1)
        C, L = int(getattr(args, "init_channels", 16)), int(getattr(args, "layers", 8))
        if str(getattr(args, "stage", "search")) == "train":
            return NetworkCIFAR(C, output_dim, L, bool(getattr(args, "auxiliary", False)),
                                getattr(args, "arch", "FedNAS_V1") or "FedNAS_V1")
        if name != "darts" or str(getattr(args, "search_method", "darts")).lower() == "gdas":
            return Network_GumbelSoftmax(C, output_dim, L, tau=float(getattr(args, "tau_max", 5.0) or 5.0))
        return DartsNetwork(C, output_dim, L)
    if name == "resnet56_gkt":
        return resnet8_56(output_dim), resnet56_server(output_dim)
    logging.warning("unknown model %s → LogisticRegression fallback (reference behaviour)", name)
    return LogisticRegression(28 * 28, output_dim)
