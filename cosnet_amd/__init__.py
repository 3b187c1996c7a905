"""cosnet_amd — MI355X-native (gfx950) implementation of the RGB-D co-attention hot path of
yahoo0742/COSNet (RGBDSegmentation_RAA): DeepLab ResNet-101/50 + ASPP encoders and the
siamese co-attention block, fwd + bwd, on hand-written HIP kernels (libcosnet_hip.so).
"""
from . import _native  # noqa: F401
from .deeplab.residual_net import Bottleneck, ResNet  # noqa: F401
from .deeplab.deeplabv3_encoder import ASPP, DepthEncoder_ResNetASPP, Encoder  # noqa: F401
from .rgbd_segmentation_RAA import CoattentionModel, RGBDSegmentation_RAA  # noqa: F401


def build_model(compute_dtype=None):
    """RGBDSegmentation_RAA(Bottleneck, [3,4,23,3], [3,4,6,3], num_classes=1) (train.py:379)."""
    import torch
    m = RGBDSegmentation_RAA(Bottleneck, [3, 4, 23, 3], [3, 4, 6, 3], num_classes=1)
    if compute_dtype is not None:
        m.set_compute_dtype(compute_dtype)
    else:
        m.set_compute_dtype(torch.bfloat16)
    return m
