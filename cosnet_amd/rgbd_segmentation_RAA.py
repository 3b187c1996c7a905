"""RGBDSegmentation_RAA ("ResNet + ASPP + Add") — the drop-in module of the hot path.

Same class name, constructor signature, submodule/parameter names (1059 state_dict keys),
init order, get_params / load_state and forward(rgbs_a, rgbs_b, depths_a, depths_b) ->
(x1, x2, labels) as rgbd_segmentation_RAA.py:18-268 of the reference.  Inputs and outputs
are fp32 NCHW on the GPU; internally every op is a libcosnet_hip kernel running on NHWC
activations in `compute_dtype` (bf16 for throughput, fp32 for parity).

Semantics kept from the reference: labels come from frame b (:146); cat order [Z, V]
(:186); RGB gate without bias, depth gate with bias (:28, :39); the b-side gate masks are
constants (:178-182); the whole depth b-side head is no_grad (:240-247); BN running stats
update on both a- and b-side calls in train mode.
"""
import os

import torch
import torch.nn as nn

from . import functions as fn
from .deeplab.deeplabv3_encoder import DepthEncoder_ResNetASPP, Encoder
from .encoder_fn import encode_pair


class RGBDSegmentation_RAA(nn.Module):
    def __init__(self, block, num_blocks_of_layers_4_rgb, num_blocks_of_layers_4_depth, num_classes,
                 all_channel=256, all_dim=60 * 60, no_grad_for_counterpart=True):
        super(RGBDSegmentation_RAA, self).__init__()
        # RGB
        self.encoder = Encoder(3, block, num_blocks_of_layers_4_rgb, num_classes)
        self.rgb_similarity_weights = nn.Linear(all_channel, all_channel, bias=False)
        self.gate = nn.Conv2d(all_channel, 1, kernel_size=1, bias=False)
        self.gate_s = nn.Sigmoid()
        self.reduce_channels_A = nn.Conv2d(all_channel * 2, all_channel, kernel_size=3, padding=1, bias=False)
        self.reduce_channels_B = nn.Conv2d(all_channel * 2, all_channel, kernel_size=3, padding=1, bias=False)
        self.bn_A = nn.BatchNorm2d(all_channel)
        self.bn_B = nn.BatchNorm2d(all_channel)
        self.prelu = nn.ReLU(inplace=True)
        # Depth
        self.depth_encoder = DepthEncoder_ResNetASPP(256, block, num_blocks_of_layers_4_depth, num_classes)
        self.depth_similarity_weights = nn.Linear(all_channel, all_channel, bias=False)
        self.depth_gate = nn.Conv2d(all_channel, 1, kernel_size=1, bias=True)
        self.depth_gate_s = nn.Sigmoid()
        self.depth_reduce_channels = nn.Conv2d(all_channel * 2, all_channel, kernel_size=3, padding=1, bias=False)
        self.depth_bn = nn.BatchNorm2d(all_channel)
        self.depth_weights = nn.Conv2d(all_channel, all_channel, kernel_size=1, bias=True)
        # Decoder
        self.segmentation_classifier_A = nn.Conv2d(all_channel, num_classes, kernel_size=1, bias=True)
        self.segmentation_classifier_B = nn.Conv2d(all_channel, num_classes, kernel_size=1, bias=True)
        self.softmax = nn.Sigmoid()
        self.no_grad_for_counterpart = no_grad_for_counterpart
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                m.weight.data.normal_(0, 0.01)
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
        if num_classes != 1:
            raise ValueError("the HIP decoder head is built for num_classes=1 (train.py:379)")
        self.compute_dtype = torch.bfloat16
        self.fp8 = None            # Fp8Context: e4m3 forward conv GEMMs in the encoders (configs[4])
        self.pair_encoder = True   # batch frames a and b through each encoder (encoder_fn.py)
        # depth encoder on a second stream (forward()); CN_CONCURRENT_ENCODERS=0 for A/B runs
        self.concurrent_encoders = os.environ.get("CN_CONCURRENT_ENCODERS", "1") != "0"
        self._to_channels_last()
        self.register_state_dict_pre_hook(_flush_bn_counters)

    # ---- configuration ----------------------------------------------------------------------
    def _to_channels_last(self):
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                m.weight.data = m.weight.data.contiguous(memory_format=torch.channels_last)

    def set_compute_dtype(self, dtype):
        """torch.bfloat16 (throughput) or torch.float32 (parity)."""
        assert dtype in (torch.bfloat16, torch.float32)
        self.compute_dtype = dtype
        return self

    def _apply(self, fn_, *a, **k):
        r = super(RGBDSegmentation_RAA, self)._apply(fn_, *a, **k)
        self._to_channels_last()
        return r

    def load_state_dict(self, state_dict, strict=True, assign=False):
        r = super(RGBDSegmentation_RAA, self).load_state_dict(state_dict, strict=strict, assign=assign)
        for m in self.modules():
            if isinstance(m, nn.BatchNorm2d):
                m._cn_nbt = 0
        self._to_channels_last()
        return r

    # ---- parameter groups (rgbd_segmentation_RAA.py:65-100) ----------------------------------
    def get_params(self, subset="none"):
        mods = []
        if subset == "none":
            return mods
        if subset in ("encoder", "rgb", "all"):
            mods.append(self.encoder)
        if subset in ("rgb_attention", "rgb", "all"):
            mods += [self.rgb_similarity_weights, self.gate, self.reduce_channels_A,
                     self.reduce_channels_B, self.bn_A, self.bn_B]
        if subset in ("depth", "all"):
            mods.extend(self.depth_encoder.get_params())
            mods += [self.depth_gate, self.depth_similarity_weights, self.depth_reduce_channels,
                     self.depth_bn, self.depth_weights]
        if subset in ("decoder", "all"):
            mods += [self.segmentation_classifier_A, self.segmentation_classifier_B]
        return mods

    # ---- original-COSNet key remap (rgbd_segmentation_RAA.py:103-136) ----------------------
    def load_state(self, state_dict):
        new_params = self.state_dict().copy()
        for k in state_dict:
            nk = k[7:] if k.startswith("module.") else k
            if nk.startswith("encoder.layer5."):
                nk = nk.replace("encoder.layer5.", "encoder.aspp.")
            elif nk.startswith("encoder.main_classifier"):
                pass
            elif nk.startswith("encoder."):
                nk = nk.replace("encoder.", "encoder.backbone.")
            elif nk.startswith("linear_e."):
                nk = nk.replace("linear_e.", "rgb_similarity_weights.")
            elif nk.startswith("conv1."):
                nk = nk.replace("conv1.", "reduce_channels_A.")
            elif nk.startswith("conv2."):
                nk = nk.replace("conv2.", "reduce_channels_B.")
            elif nk.startswith("bn1."):
                nk = nk.replace("bn1.", "bn_A.")
            elif nk.startswith("bn2."):
                nk = nk.replace("bn2.", "bn_B.")
            elif nk.startswith("main_classifier1."):
                nk = nk.replace("main_classifier1.", "segmentation_classifier_A.")
            elif nk.startswith("main_classifier2."):
                nk = nk.replace("main_classifier2.", "segmentation_classifier_B.")
            new_params[nk] = state_dict[k]
        self.load_state_dict(new_params)

    # ---- forward (rgbd_segmentation_RAA.py:139-268) ----------------------------------------
    def _prep(self, t):
        if not t.is_cuda:
            raise RuntimeError("RGBDSegmentation_RAA (HIP) expects inputs on the GPU")
        return t.float().contiguous()

    def set_fp8(self, on=True):
        """fp8 (OCP e4m3) operands for the encoders' forward conv GEMMs (cosnet_amd/fp8.py);
        needs the bf16 compute dtype.  The depth encoder gets a context of its own: it runs
        concurrently with the RGB encoder, and a context's scale update covers all its states."""
        if on and self.compute_dtype != torch.bfloat16:
            raise ValueError("fp8 convs run inside the bf16 path")
        from .fp8 import Fp8Context
        self.fp8 = Fp8Context() if on else None
        self._fp8_depth = Fp8Context() if on else None
        return self

    def _set_dtype(self):
        for m in self.modules():
            m._cn_dtype = self.compute_dtype
            m._cn_fp8 = self.fp8
        for m in self.depth_encoder.modules():
            m._cn_fp8 = getattr(self, "_fp8_depth", None)

    def _side_stream(self, dev):
        """Stream of the depth encoder (None: run it after the RGB encoder on one stream)."""
        if not self.concurrent_encoders or dev.type != "cuda":
            return None
        s = getattr(self, "_cn_side", None)
        if s is None or s.device != dev:
            s = self._cn_side = torch.cuda.Stream(device=dev)
        return s

    def forward(self, rgbs_a, rgbs_b, depths_a, depths_b, stages=None):
        self._set_dtype()
        rgbs_a, rgbs_b, depths_a, depths_b = map(self._prep, (rgbs_a, rgbs_b, depths_a, depths_b))
        input_size = tuple(rgbs_a.shape[2:])
        ng = torch.no_grad if self.no_grad_for_counterpart else _Null
        if self.no_grad_for_counterpart and self.pair_encoder and rgbs_a.shape == rgbs_b.shape:
            # both frames in one batched encoder pass (cosnet_amd/encoder_fn.py).  The depth
            # encoder and the depth branch of the head (:197-247) are independent of the RGB
            # side up to the fusion (:251), so they run on a second stream whose kernels fill
            # the CUs the RGB kernels leave idle (a parallel branch of the recorded graph; the
            # backward follows -- autograd runs a backward op on its forward's stream)
            side = self._side_stream(rgbs_a.device)
            if side is not None:
                cur = torch.cuda.current_stream(rgbs_a.device)
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    da, db, dgeo, dz_a, dz_b = self.depth_side(depths_a, depths_b)
                va, vb, geo, labels, z_a, z_b = self.rgb_side(rgbs_a, rgbs_b, input_size)
                cur.wait_stream(side)
                for t in (depths_a, depths_b):
                    t.record_stream(side)
                for t in (da, db, dz_a, dz_b):
                    t.record_stream(cur)
                x1, x2 = self.decode_outputs(z_a, z_b, dz_a, dz_b, geo, dgeo, input_size)
                if stages is not None:
                    stages.update(V_a=va, V_b=vb, D_a=da, D_b=db, geo=geo)
                return x1, x2, labels
            va, vb, geo = encode_pair(self.encoder, rgbs_a, rgbs_b)
            da, db, dgeo = encode_pair(self.depth_encoder, depths_a, depths_b)
        else:
            va, geo = self.encoder.features_nhwc(rgbs_a)
            with ng():
                vb, _ = self.encoder.features_nhwc(rgbs_b)
            da, dgeo = self.depth_encoder.features_nhwc(depths_a)
            with ng():
                db, _ = self.depth_encoder.features_nhwc(depths_b)
        with torch.no_grad():
            labels = self.encoder.annotate_nhwc(vb, geo, input_size)       # frame b (:146)
        if dgeo != geo:
            raise RuntimeError("RGB and depth feature maps differ: %s vs %s" % (geo, dgeo))
        x1, x2 = self.head_nhwc(va, vb, da, db, geo, input_size)
        if stages is not None:
            stages.update(V_a=va, V_b=vb, D_a=da, D_b=db, geo=geo)
        return x1, x2, labels

    # The two independent halves of the paired forward up to the fusion (:143-191 and :197-247).
    # forward() runs them on two streams; TrainStep's per-phase recordings call the same two
    # methods, one graph each, so the cut points cannot drift from forward().
    def rgb_side(self, rgbs_a, rgbs_b, input_size):
        """RGB encoder of both frames, labels (frame b, :146) and the RGB head."""
        va, vb, geo = encode_pair(self.encoder, rgbs_a, rgbs_b)
        with torch.no_grad():
            labels = self.encoder.annotate_nhwc(vb, geo, input_size)
        z_a, z_b = self._rgb_head(va, vb, geo)
        return va, vb, geo, labels, z_a, z_b

    def depth_side(self, depths_a, depths_b):
        """Depth encoder of both frames and the depth head."""
        da, db, dgeo = encode_pair(self.depth_encoder, depths_a, depths_b)
        dz_a, dz_b = self._depth_head(da, db, dgeo)
        return da, db, dgeo, dz_a, dz_b

    def decode_outputs(self, z_a, z_b, dz_a, dz_b, geo, dgeo, input_size):
        """Fusion + decoder of the two halves (:251-266)."""
        if dgeo != geo:
            raise RuntimeError("RGB and depth feature maps differ: %s vs %s" % (geo, dgeo))
        return self._decode(z_a, z_b, dz_a, dz_b, geo, input_size)

    def head_nhwc(self, va, vb, da, db, geo, input_size):
        """Co-attention (RGB and depth), gated fusion and decoder from encoder features
        (rgbd_segmentation_RAA.py:150-266).  The reference interleaves the depth encoder calls
        with the RGB head (:198-203); the encoders have no data dependence on the head, so the
        order of launches does not change any result."""
        z_a, z_b = self._rgb_head(va, vb, geo)
        dz_a, dz_b = self._depth_head(da, db, geo)
        return self._decode(z_a, z_b, dz_a, dz_b, geo, input_size)

    def _rgb_head(self, va, vb, geo):
        """RGB co-attention + gate + reduce conv + BN (rgbd_segmentation_RAA.py:150-191)."""
        n, h, w = geo
        hw = h * w
        link = {}   # V_a's two gradient contributions meet inside CoattFn's backward
        f8 = getattr(self, "fp8", None) is not None and va.dtype == torch.bfloat16   # configs[4]
        za, zb = fn.CoattFn.apply(va, vb, self.rgb_similarity_weights.weight, (n, hw), link, f8)
        cat_a = fn.GateCatFn.apply(za, va, self.gate.weight, None, False, link)
        cat_b = fn.GateCatFn.apply(zb, vb, self.gate.weight, None, True)  # mask_b no_grad (:178-182)
        z_a = fn.BNFn.apply(fn.ConvFn.apply(cat_a, self.reduce_channels_A.weight, None, geo, 3, 1, 1, 1),
                            self.bn_A.weight, self.bn_A.bias, self.bn_A)
        z_b = fn.BNFn.apply(fn.ConvFn.apply(cat_b, self.reduce_channels_B.weight, None, geo, 3, 1, 1, 1),
                            self.bn_B.weight, self.bn_B.bias, self.bn_B)
        return z_a, z_b

    def _depth_head(self, da, db, geo):
        """Depth co-attention + gate + reduce conv + BN + 1x1 (rgbd_segmentation_RAA.py:204-247)."""
        n, h, w = geo
        hw = h * w
        dlink = {}
        f8 = getattr(self, "_fp8_depth", None) is not None and da.dtype == torch.bfloat16
        dza, dzb = fn.CoattFn.apply(da, db, self.depth_similarity_weights.weight, (n, hw), dlink, f8)
        dcat_a = fn.GateCatFn.apply(dza, da, self.depth_gate.weight, self.depth_gate.bias, False, dlink)
        dz_a = fn.BNFn.apply(fn.ConvFn.apply(dcat_a, self.depth_reduce_channels.weight, None, geo, 3, 1, 1, 1),
                             self.depth_bn.weight, self.depth_bn.bias, self.depth_bn)
        dz_a = fn.ConvFn.apply(dz_a, self.depth_weights.weight, self.depth_weights.bias, geo, 1, 1, 0, 1)
        with torch.no_grad():                                               # (:229-247)
            dcat_b = fn.GateCatFn.apply(dzb, db, self.depth_gate.weight, self.depth_gate.bias, True)
            dz_b = fn.BNFn.apply(fn.ConvFn.apply(dcat_b, self.depth_reduce_channels.weight, None, geo, 3, 1, 1, 1),
                                 self.depth_bn.weight, self.depth_bn.bias, self.depth_bn)
            dz_b = fn.ConvFn.apply(dz_b, self.depth_weights.weight, self.depth_weights.bias, geo, 1, 1, 0, 1)
        return dz_a, dz_b

    def _decode(self, z_a, z_b, dz_a, dz_b, geo, input_size):
        """Fusion + decoder (rgbd_segmentation_RAA.py:251-266)."""
        la = fn.HeadFn.apply(z_a, dz_a, self.segmentation_classifier_A.weight,
                             self.segmentation_classifier_A.bias, True)
        lb = fn.HeadFn.apply(z_b, dz_b, self.segmentation_classifier_B.weight,
                             self.segmentation_classifier_B.bias, True)
        x1 = fn.UpSigFn.apply(la, geo, input_size)
        x2 = fn.UpSigFn.apply(lb, geo, input_size)
        return x1, x2


CoattentionModel = RGBDSegmentation_RAA  # name used by BASELINE.json's north_star


class _Null:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


def _flush_bn_counters(module, prefix, keep_vars):
    """num_batches_tracked is counted on the host during forward (no device op per BN call)
    and folded into the buffer whenever a state_dict is taken."""
    for m in module.modules():
        k = getattr(m, "_cn_nbt", 0)
        if k and isinstance(m, nn.BatchNorm2d):
            m.num_batches_tracked.add_(k)
            m._cn_nbt = 0
