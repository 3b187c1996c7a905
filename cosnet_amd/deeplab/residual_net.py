"""Dilated ResNet backbone — same classes, constructor signatures, parameter names and init
order as deeplab/residual_net.py of the reference, so state_dicts and seeded inits match
key-for-key.  The compute is not nn.Conv2d/BatchNorm2d: those modules only hold the fp32
parameters; forward runs the hand-written HIP block kernels (cosnet_amd.functions).

Reference: Bottleneck :47-96 (stride on conv1, original ResNet), ResNet :100-172,
_make_layer :125-142 (downsample always present on block 0; its BN affine frozen :132-133).
"""
import torch.nn as nn

from .. import functions as fn
from .. import ops
from . import config


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, in_channels, shrank_channels, stride=1, dilation=1, downsample=None):
        super(Bottleneck, self).__init__()
        self.conv1 = nn.Conv2d(in_channels, shrank_channels, kernel_size=1, stride=stride, bias=False)
        self.bn1 = nn.BatchNorm2d(shrank_channels, affine=config.k_learnable_affine_parameters)
        padding = dilation
        self.conv2 = nn.Conv2d(shrank_channels, shrank_channels, kernel_size=3, stride=1,
                               padding=padding, bias=False, dilation=dilation)
        self.bn2 = nn.BatchNorm2d(shrank_channels, affine=config.k_learnable_affine_parameters)
        self.conv3 = nn.Conv2d(shrank_channels, shrank_channels * self.expansion, kernel_size=1, bias=False)
        self.bn3 = nn.BatchNorm2d(shrank_channels * self.expansion, affine=config.k_learnable_affine_parameters)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride
        self.dilation = dilation

    def forward_nhwc(self, x, geo):
        """x: [n*h*w, Cin] NHWC -> ([n*oh*ow, 4*planes], (n, oh, ow))"""
        n, h, w = geo
        d = self.downsample
        y = fn.BottleneckFn.apply(
            x, self, geo, self.conv1.weight, self.bn1.weight, self.bn1.bias, self.conv2.weight,
            self.bn2.weight, self.bn2.bias, self.conv3.weight, self.bn3.weight, self.bn3.bias,
            d[0].weight if d is not None else None, d[1].weight if d is not None else None,
            d[1].bias if d is not None else None)
        oh, ow = ops.out_hw(h, w, 1, self.stride, 0, 1)
        return y, (n, oh, ow)


class ResNet(nn.Module):
    def __init__(self, input_channels, res_block, num_blocks_of_layers, num_classes):
        self.inner_channels = 64
        self.input_channels = input_channels
        super(ResNet, self).__init__()
        self.conv1 = nn.Conv2d(self.input_channels, self.inner_channels, kernel_size=7, stride=2,
                               padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(self.inner_channels, affine=config.k_learnable_affine_parameters)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1, ceil_mode=True)
        self.layer1 = self._make_layer(res_block, out_channels=64, num_blocks=num_blocks_of_layers[0])
        self.layer2 = self._make_layer(res_block, out_channels=128, num_blocks=num_blocks_of_layers[1], stride=2)
        self.layer3 = self._make_layer(res_block, out_channels=256, num_blocks=num_blocks_of_layers[2],
                                       stride=1, dilation=2)
        self.layer4 = self._make_layer(res_block, out_channels=512, num_blocks=num_blocks_of_layers[3],
                                       stride=1, dilation=4)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                m.weight.data.normal_(0, 0.01)
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()

    def _make_layer(self, res_block, out_channels, num_blocks, stride=1, dilation=1):
        downsample = None
        if (stride != 1 or self.inner_channels != out_channels * res_block.expansion
                or dilation == 2 or dilation == 4):
            downsample = nn.Sequential(
                nn.Conv2d(self.inner_channels, out_channels * res_block.expansion, kernel_size=1,
                          stride=stride, bias=False),
                nn.BatchNorm2d(out_channels * res_block.expansion, affine=config.k_learnable_affine_parameters))
        for i in downsample._modules['1'].parameters():
            i.requires_grad = False
        layers = [res_block(self.inner_channels, out_channels, stride, dilation=dilation, downsample=downsample)]
        self.inner_channels = out_channels * res_block.expansion
        for i in range(1, num_blocks):
            layers.append(res_block(self.inner_channels, out_channels, dilation=dilation))
        return nn.Sequential(*layers)

    def get_params(self):
        return [self.conv1, self.bn1, self.layer1, self.layer2, self.layer3, self.layer4]

    def forward_nhwc(self, img):
        """img: NCHW fp32 [n, Cin, H, W] -> ([n*h*w, 2048] NHWC, (n, h, w)) at stride 8."""
        n, _, H, W = img.shape
        z = fn.StemFn.apply(img, self, self.conv1.weight, self.bn1.weight, self.bn1.bias)
        oh, ow = ops.out_hw(H, W, 7, 2, 3, 1)
        geo = (n, ops.pool_out(oh), ops.pool_out(ow))
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            for blk in layer:
                z, geo = blk.forward_nhwc(z, geo)
        return z, geo

    def forward(self, x):
        z, (n, h, w) = self.forward_nhwc(x)
        return z.view(n, h, w, -1).permute(0, 3, 1, 2)
