"""ASPP head and the RGB / depth encoders, mirroring deeplab/deeplabv3_encoder.py of the
reference (ASPP :10-86, Encoder :91-143, DepthEncoder_ResNetASPP :149-185): same classes,
signatures, parameter names and init order; forward runs the HIP ASPP block (ASPPFn).
"""
import torch.nn as nn

from .. import functions as fn
from . import residual_net as rn


class ASPP(nn.Module):
    def __init__(self, input_channels, output_channels, depth, dilation_series, padding_series):
        super(ASPP, self).__init__()
        self.mean = nn.AdaptiveAvgPool2d((1, 1))
        self.conv = nn.Conv2d(input_channels, depth, kernel_size=1, stride=1)
        self.bn_x = nn.BatchNorm2d(depth)
        self.relu = nn.ReLU(inplace=True)
        self.conv2d_0 = nn.Conv2d(input_channels, depth, kernel_size=1, stride=1)
        self.bn_0 = nn.BatchNorm2d(depth)
        self.conv2d_1 = nn.Conv2d(input_channels, depth, kernel_size=3, stride=1,
                                  padding=padding_series[0], dilation=dilation_series[0])
        self.bn_1 = nn.BatchNorm2d(depth)
        self.conv2d_2 = nn.Conv2d(input_channels, depth, kernel_size=3, stride=1,
                                  padding=padding_series[1], dilation=dilation_series[1])
        self.bn_2 = nn.BatchNorm2d(depth)
        self.conv2d_3 = nn.Conv2d(input_channels, depth, kernel_size=3, stride=1,
                                  padding=padding_series[2], dilation=dilation_series[2])
        self.bn_3 = nn.BatchNorm2d(depth)
        self.bottleneck = nn.Conv2d(depth * 5, output_channels, kernel_size=3, padding=1)
        self.bn = nn.BatchNorm2d(output_channels)
        self.prelu = nn.PReLU()
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                m.weight.data.normal_(0, 0.01)
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
        if list(dilation_series) != list(padding_series):
            raise ValueError("ASPP: padding_series must equal dilation_series (as in the reference)")
        if input_channels != 2048 or depth != 512 or output_channels != 256:
            raise ValueError("ASPP: the HIP block is built for 2048 -> 5x512 -> 256 channels")
        self.cn_dilations = tuple(dilation_series)

    def _params(self):
        p = [self.conv.weight, self.conv.bias, self.bn_x.weight, self.bn_x.bias]
        for i in range(4):
            c = getattr(self, "conv2d_%d" % i)
            b = getattr(self, "bn_%d" % i)
            p += [c.weight, c.bias, b.weight, b.bias]
        p += [self.bottleneck.weight, self.bottleneck.bias, self.bn.weight, self.bn.bias, self.prelu.weight]
        return p

    def forward_nhwc(self, x, geo):
        return fn.ASPPFn.apply(x, self, geo, *self._params()), geo


class Encoder(nn.Module):
    def __init__(self, input_channels, res_block, num_blocks_of_layers, num_classes):
        self.input_channels = input_channels
        super(Encoder, self).__init__()
        self.backbone = rn.ResNet(input_channels, res_block, num_blocks_of_layers, num_classes)
        dilations = [6, 12, 18]
        paddings = [6, 12, 18]
        self.aspp = ASPP(input_channels=2048, output_channels=256, depth=512,
                         dilation_series=dilations, padding_series=paddings)
        self.main_classifier = nn.Conv2d(256, num_classes, kernel_size=1)
        self.softmax = nn.Sigmoid()
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                m.weight.data.normal_(0, 0.01)
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()

    def get_params(self, level="none"):
        mods = []
        if level == "backbone":
            b = self.backbone
            mods += [b.conv1, b.bn1, b.layer1, b.layer2, b.layer3, b.layer4, self.aspp]
        elif level == "classifier":
            mods.append(self.main_classifier)
        return mods

    def features_nhwc(self, x):
        z, geo = self.backbone.forward_nhwc(x)
        return self.aspp.forward_nhwc(z, geo)

    def annotate_nhwc(self, feats, geo, input_size):
        """main_classifier -> bilinear upsample -> sigmoid  (:138-142); fp32 NCHW."""
        logit = fn.HeadFn.apply(feats, None, self.main_classifier.weight, self.main_classifier.bias, False)
        return fn.UpSigFn.apply(logit, geo, tuple(input_size))

    def forward(self, x):
        feats, geo = self.features_nhwc(x)
        ann = self.annotate_nhwc(feats, geo, x.shape[2:])
        n, h, w = geo
        return feats.view(n, h, w, -1).permute(0, 3, 1, 2), ann


class DepthEncoder_ResNetASPP(nn.Module):
    def __init__(self, output_channels, res_block, num_blocks_of_layers, num_classes):
        super(DepthEncoder_ResNetASPP, self).__init__()
        self.input_channels = 1
        self.backbone = rn.ResNet(self.input_channels, res_block, num_blocks_of_layers, num_classes)
        dilations = [2, 3, 7]
        paddings = [2, 3, 7]
        num_channels_from_backbone = 2048
        self.aspp = ASPP(input_channels=num_channels_from_backbone, output_channels=output_channels,
                         depth=512, dilation_series=dilations, padding_series=paddings)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                m.weight.data.normal_(0, 0.01)
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()

    def get_params(self):
        return self.backbone.get_params() + [self.aspp]

    def features_nhwc(self, x):
        z, geo = self.backbone.forward_nhwc(x)
        return self.aspp.forward_nhwc(z, geo)

    def forward(self, x):
        feats, (n, h, w) = self.features_nhwc(x)
        return feats.view(n, h, w, -1).permute(0, 3, 1, 2)
