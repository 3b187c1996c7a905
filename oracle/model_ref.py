"""ORACLE — test infrastructure only.  Never imported by the product path.

A functional CPU restatement (plain torch.nn.functional on CPU, fp32 or fp64) of the
reference RGBDSegmentation_RAA forward, written from the reference's behaviour:

  ResNet / Bottleneck      deeplab/residual_net.py:47-96, :100-172
  ASPP                      deeplab/deeplabv3_encoder.py:10-86
  Encoder                   deeplab/deeplabv3_encoder.py:91-143
  DepthEncoder_ResNetASPP   deeplab/deeplabv3_encoder.py:149-185
  co-attention + fusion     rgbd_segmentation_RAA.py:139-268
  loss                      train.py:176-216, :595-597 (calc_loss_BCE + 0.8 * calc_loss_L1)

It takes a plain {key: tensor} state dict with the reference's 1059 keys.  Only the
checker (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline leg) may call it.
Pinned against the reference itself through tests/golden/*.npz (make_golden.py).
"""
import torch
import torch.nn.functional as F

RGB_LAYERS = (3, 4, 23, 3)     # train.py:379 (create_model)
DEPTH_LAYERS = (3, 4, 6, 3)
BN_EPS = 1e-5
BN_MOMENTUM = 0.1


class RefModel:
    """Parameters + buffers as a dict; forward() mirrors rgbd_segmentation_RAA.py:139-268."""

    def __init__(self, state_dict, dtype=torch.float64, requires_grad=True):
        self.p = {}
        for k, v in state_dict.items():
            t = v.detach().clone()
            if t.is_floating_point():
                t = t.to(dtype)
                frozen = _is_frozen(k) or not _is_param(k)
                if requires_grad and not frozen:
                    t.requires_grad_(True)
            self.p[k] = t
        self.training = True
        self.no_grad_for_counterpart = True

    # ---- primitives --------------------------------------------------------------
    def conv(self, x, name, stride=1, padding=0, dilation=1):
        b = self.p.get(name + ".bias")
        return F.conv2d(x, self.p[name + ".weight"], b, stride, padding, dilation)

    def bn(self, x, name):
        # nn.BatchNorm2d semantics: batch stats + running update in train, running in eval.
        nbt = self.p[name + ".num_batches_tracked"]
        if self.training:
            nbt.add_(1)
        return F.batch_norm(x, self.p[name + ".running_mean"], self.p[name + ".running_var"],
                            self.p[name + ".weight"], self.p[name + ".bias"],
                            self.training, BN_MOMENTUM, BN_EPS)

    # ---- deeplab/residual_net.py ----------------------------------------------------
    def bottleneck(self, x, name, stride, dilation, has_down):
        # deeplab/residual_net.py:74-96 (stride on conv1, the original-ResNet variant)
        out = F.relu(self.bn(self.conv(x, name + ".conv1", stride=stride), name + ".bn1"))
        out = F.relu(self.bn(self.conv(out, name + ".conv2", padding=dilation, dilation=dilation),
                             name + ".bn2"))
        out = self.bn(self.conv(out, name + ".conv3"), name + ".bn3")
        if has_down:
            identity = self.bn(self.conv(x, name + ".downsample.0", stride=stride),
                               name + ".downsample.1")
        else:
            identity = x
        return F.relu(out + identity)

    def resnet(self, x, name, layers):
        # deeplab/residual_net.py:156-172
        z = F.relu(self.bn(self.conv(x, name + ".conv1", stride=2, padding=3), name + ".bn1"))
        z = F.max_pool2d(z, 3, 2, 1, ceil_mode=True)   # :109 ceil_mode=True
        cfg = [(1, 1), (2, 1), (1, 2), (1, 4)]          # :111-114 strides / dilations
        for li, (nb, (stride, dil)) in enumerate(zip(layers, cfg)):
            for bi in range(nb):
                z = self.bottleneck(z, "%s.layer%d.%d" % (name, li + 1, bi),
                                    stride if bi == 0 else 1, dil, bi == 0)
        return z

    # ---- deeplab/deeplabv3_encoder.py ------------------------------------------------
    def aspp(self, x, name, dil):
        size = x.shape[2:]
        f = F.adaptive_avg_pool2d(x, 1)
        f = F.relu(self.bn(self.conv(f, name + ".conv"), name + ".bn_x"))
        f = F.interpolate(f, size=size, mode="bilinear", align_corners=True)   # :61
        outs = [f, F.relu(self.bn(self.conv(x, name + ".conv2d_0"), name + ".bn_0"))]
        for i, d in enumerate(dil):
            outs.append(F.relu(self.bn(self.conv(x, name + ".conv2d_%d" % (i + 1), padding=d,
                                                 dilation=d), name + ".bn_%d" % (i + 1))))
        out = torch.cat(outs, 1)                                                # :79
        out = self.bn(self.conv(out, name + ".bottleneck", padding=1), name + ".bn")
        return F.prelu(out, self.p[name + ".prelu.weight"])

    def encoder(self, x):
        # deeplab/deeplabv3_encoder.py:132-143
        feats = self.aspp(self.resnet(x, "encoder.backbone", RGB_LAYERS), "encoder.aspp", (6, 12, 18))
        ann = self.conv(feats, "encoder.main_classifier")
        ann = F.interpolate(ann, size=x.shape[2:], mode="bilinear", align_corners=False)
        return feats, torch.sigmoid(ann)

    def depth_encoder(self, x):
        # deeplab/deeplabv3_encoder.py:180-185
        return self.aspp(self.resnet(x, "depth_encoder.backbone", DEPTH_LAYERS),
                         "depth_encoder.aspp", (2, 3, 7))

    # ---- rgbd_segmentation_RAA.py ----------------------------------------------------
    @staticmethod
    def coattention(_self, va, vb, w):
        """rgbd_segmentation_RAA.py:150-170: returns (Z_a, Z_b) as [N, C, H, W]."""
        n, c, h, wd = va.shape
        va_f = va.reshape(n, c, h * wd)
        vb_f = vb.reshape(n, c, h * wd)
        va_t = F.linear(va_f.transpose(1, 2), w)          # :158-159
        s = torch.bmm(va_t, vb_f)                           # :160
        s_row = F.softmax(s, dim=1)                         # :164
        s_col = F.softmax(s.transpose(1, 2), dim=1)         # :165
        z_b = torch.bmm(va_f, s_row)                        # :169
        z_a = torch.bmm(vb_f, s_col)                        # :170
        return z_a.reshape(n, c, h, wd), z_b.reshape(n, c, h, wd)

    def forward(self, rgbs_a, rgbs_b, depths_a, depths_b, stages=None):
        input_size = rgbs_a.shape[2:]
        ng = torch.no_grad if self.no_grad_for_counterpart else _null
        va, labels = self.encoder(rgbs_a)
        with ng():
            vb, labels = self.encoder(rgbs_b)               # :146 labels from frame b
        z_a, z_b = self.coattention(self, va, vb, self.p["rgb_similarity_weights.weight"])
        m_a = torch.sigmoid(self.conv(z_a, "gate"))
        with torch.no_grad():
            m_b = torch.sigmoid(self.conv(z_b, "gate"))
        z_a = torch.cat([z_a * m_a, va], 1)                 # cat order [Z, V]  :186
        z_b = torch.cat([z_b * m_b, vb], 1)
        z_a = self.bn(self.conv(z_a, "reduce_channels_A", padding=1), "bn_A")
        z_b = self.bn(self.conv(z_b, "reduce_channels_B", padding=1), "bn_B")

        da = self.depth_encoder(depths_a)
        with ng():
            db = self.depth_encoder(depths_b)
        dz_a, dz_b = self.coattention(self, da, db, self.p["depth_similarity_weights.weight"])
        dm_a = torch.sigmoid(self.conv(dz_a, "depth_gate"))
        with torch.no_grad():
            dm_b = torch.sigmoid(self.conv(dz_b, "depth_gate"))
        dz_a = torch.cat([dz_a * dm_a, da], 1)
        dz_b = torch.cat([dz_b * dm_b, db], 1)
        dz_a = self.conv(self.bn(self.conv(dz_a, "depth_reduce_channels", padding=1), "depth_bn"),
                         "depth_weights")
        with torch.no_grad():
            dz_b = self.conv(self.bn(self.conv(dz_b, "depth_reduce_channels", padding=1),
                                     "depth_bn"), "depth_weights")
        z_a = F.relu(z_a + dz_a)
        z_b = F.relu(z_b + dz_b)
        x1 = F.interpolate(self.conv(z_a, "segmentation_classifier_A"), size=input_size,
                           mode="bilinear", align_corners=False)
        x2 = F.interpolate(self.conv(z_b, "segmentation_classifier_B"), size=input_size,
                           mode="bilinear", align_corners=False)
        if stages is not None:
            stages.update(V_a=va, V_b=vb, D_a=da, D_b=db, Z_a=z_a, Z_b=z_b)
        return torch.sigmoid(x1), torch.sigmoid(x2), labels


class _null:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


def _is_param(key):
    return not (key.endswith("running_mean") or key.endswith("running_var")
                or key.endswith("num_batches_tracked"))


def _is_frozen(key):
    # downsample BN affine has requires_grad=False (deeplab/residual_net.py:132-133)
    return ".downsample.1." in key


def loss_bce_l1(pred, gt):
    """calc_loss_BCE + 0.8 * calc_loss_L1 (train.py:176-216).

    ratio = N*H*W / #(gt >= 0.5) as BCE weight (train.py:183-192); plain BCE if no positives.
    """
    npos = int((gt >= 0.5).sum())
    if npos == 0:
        bce = F.binary_cross_entropy(pred, gt)
    else:
        ratio = (gt.shape[0] * gt.shape[2] * gt.shape[3]) / npos
        bce = F.binary_cross_entropy(pred, gt, weight=torch.full_like(gt, ratio))
    return bce + 0.8 * F.l1_loss(pred, gt)


def compute_iou(prediction01, gt01):
    """Soft J of evaluation.py:3-22 (numpy, integer arithmetic)."""
    import numpy as np
    if np.all(gt01 == 0):
        return 1.0 - np.count_nonzero(prediction01) / (prediction01.shape[0] * prediction01.shape[1])
    pred = prediction01.astype(np.int16)
    gt = (gt01 * 255).astype(np.int16)
    return np.sum(pred & gt) * 1.0 / np.sum(pred | gt)
