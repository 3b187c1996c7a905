"""Block-level autograd Functions: hand-written forward AND backward for each reference
module of the hot path, every step a libcosnet_hip kernel.

  StemFn        deeplab/residual_net.py:157-160   conv7x7/s2 + BN + ReLU + maxpool(ceil)
  BottleneckFn  deeplab/residual_net.py:74-96     1x1(s) / 3x3(dil) / 1x1 + BN/ReLU + residual
  ASPPFn        deeplab/deeplabv3_encoder.py:50-86 pool/1x1/3x3x3 branches -> cat -> 3x3 -> BN -> PReLU
  CoattFn       rgbd_segmentation_RAA.py:150-170  linear, affinity bmm, row/col softmax, 2 gathers
  GateCatFn     rgbd_segmentation_RAA.py:177-187  sigmoid gate, multiply, cat [Z, V]
  ConvFn/BNFn   generic conv (+bias) and BN for the co-attention head (:188-191, :239-247)
  HeadFn        rgbd_segmentation_RAA.py:251-261  add + ReLU + 1x1 classifier
  UpSigFn       rgbd_segmentation_RAA.py:262-266  bilinear upsample (align_corners=False) + sigmoid
  BceL1Fn       train.py:176-216                  r * BCE + 0.8 * L1

Activations are [P, C] NHWC matrices in the model's compute dtype (bf16 or fp32); parameters
are the fp32 masters of the nn.Module holders, gradients are produced in fp32.
"""
import torch

from . import _native as nv
from . import ops
from .ops import WCACHE, bn_apply, bn_bwd, bn_stats, conv_dgrad, conv_fwd, conv_wgrad, as_param_grad

_GRAD = [True]  # grad mode of the caller of the innermost Function.apply in progress


class F(torch.autograd.Function):
    """autograd.Function that remembers the CALLER's grad mode: torch runs forward() under
    no_grad and still reports needs_input_grad from each input's requires_grad (a Parameter
    says True even inside torch.no_grad()), so `_need` must consult the outer mode to know
    whether a backward can ever run (and e.g. pick the fused inference kernels)."""

    @classmethod
    def apply(cls, *args, **kwargs):
        prev = _GRAD[0]
        _GRAD[0] = torch.is_grad_enabled()
        try:
            return super().apply(*args, **kwargs)
        finally:
            _GRAD[0] = prev


def _need(ctx):
    return _GRAD[0] and any(ctx.needs_input_grad)


def _check_train(ctx):
    if not ctx.training:
        raise RuntimeError("backward through BatchNorm is implemented for train mode only")


# ==============================================================================================
# The per-module encoder blocks (frames of different sizes: the model's unpaired path, e.g.
# configs[3]'s 1 target vs 5 references).  Each is an autograd wrapper over the SAME block
# functions the paired encoder pass runs (encoder_fn.stem_fwd / bottleneck_fwd / aspp_fwd and
# their backwards) with one frame segment and bf16 / fp32 operands, so the two paths cannot
# drift apart (tests/test_gpu_blocks_bf16.py::test_per_module_blocks_are_the_paired_code).
def _enc():
    from . import encoder_fn   # encoder_fn imports this module (F, _GRAD)
    return encoder_fn


class StemFn(F):
    @staticmethod
    def forward(ctx, img, mod, w, g, b):
        E = _enc()
        dt = getattr(mod, "_cn_dtype", torch.bfloat16)
        rec = [] if _need(ctx) else None
        with E.no_fp8():
            out, _ = E.stem_fwd(mod, (img,), 1, dt, rec)
        ctx.item = rec[0] if rec else None
        ctx.params = (w, g, b)
        ctx.training = mod.training
        return out

    @staticmethod
    def backward(ctx, dout):
        _check_train(ctx)
        E = _enc()
        grads = E.GradSink()
        with E.no_fp8():
            E.stem_bwd(ctx.item, dout if dout.stride(1) == 1 else dout.contiguous(), grads)
        ctx.item = None
        return (None, None) + tuple(grads.get(p) for p in ctx.params)


# ==============================================================================================
class BottleneckFn(F):
    @staticmethod
    def forward(ctx, x, blk, geo, w1, g1, b1, w2, g2, b2, w3, g3, b3, wd, gd, bd):
        E = _enc()
        rec = [] if _need(ctx) else None
        with E.no_fp8():
            y, _ = E.bottleneck_fwd(blk, x, geo, 1, rec)
        ctx.item = rec[0] if rec else None
        ctx.params = (w1, g1, b1, w2, g2, b2, w3, g3, b3, wd, gd, bd)
        ctx.training = blk.training
        return y

    @staticmethod
    def backward(ctx, dy):
        _check_train(ctx)
        E = _enc()
        grads = E.GradSink()
        need_dx = ctx.needs_input_grad[0]
        with E.no_fp8():
            dx = E.bottleneck_bwd(ctx.item, dy if dy.stride(1) == 1 else dy.contiguous(), grads,
                                  need_dx=need_dx)
        ctx.item = None
        return ((dx if need_dx else None), None, None) + tuple(
            grads.get(p) if p is not None else None for p in ctx.params)


# ==============================================================================================
class ASPPFn(F):
    @staticmethod
    def forward(ctx, x, mod, geo, *p):
        E = _enc()
        rec = [] if _need(ctx) else None
        with E.no_fp8():
            out = E.aspp_fwd(mod, x, geo, 1, rec)
        ctx.item = rec[0] if rec else None
        ctx.params = p
        ctx.training = mod.training
        return out

    @staticmethod
    def backward(ctx, dout):
        _check_train(ctx)
        E = _enc()
        grads = E.GradSink()
        with E.no_fp8():
            dx = E.aspp_bwd(ctx.item, dout if dout.stride(1) == 1 else dout.contiguous(), grads)
        ctx.item = None
        return (dx if ctx.needs_input_grad[0] else None, None, None) + tuple(grads.get(q) for q in ctx.params)


# ==============================================================================================
class CoattFn(F):
    """Z_a = softmax_j(S) V_b ; Z_b = softmax_i(S)^T V_a with S = (V_a W^T) V_b^T.

    `link` (optional dict shared with the GateCatFn that concatenates V_a): that Function's
    backward leaves its gradient for V_a in link["dv"] instead of returning it, and this
    backward starts its dV_a accumulation from it, so V_a's two gradient contributions are
    summed inside the HIP GEMM epilogues rather than by an autograd add."""

    @staticmethod
    def forward(ctx, va, vb, wsim, geo, link=None, fp8=False):
        n, hw = geo
        c = va.shape[1]
        dt = va.dtype
        dev = va.device
        ldp = (hw + 7) // 8 * 8
        wf, _ = WCACHE.get(wsim, dt, need_t=False)
        vat = ops.gemm(va, wf, n * hw, c, c, lda=ops.ld(va), ldb=c)            # :158-159
        ctx.geo = (n, hw, c, ldp)
        ctx.set_materialize_grads(False)
        if ops.coatt_fused_ok(dt, c, va, vb):
            # both directions in one flash-style launch, S never leaves the chip
            za = torch.empty((n * hw, c), dtype=dt, device=dev)
            zb = torch.empty((n * hw, c), dtype=dt, device=dev)
            if not _need(ctx):                                                   # inference
                if fp8:   # configs[4]: MX-fp8 affinity and gathers
                    ops.coatt_f8(vat, va, vb, n, hw, za, zb)                     # :160-170
                else:
                    ops.coatt_fused(vat, va, vb, n, hw, za, zb)                  # :160-170
                return za, zb
            # training: keep the per-row normalisers; the backward recomputes P from them.  fp8
            # mode (configs[4]): the MX-fp8 forward, which also hands back its operands DECODED
            # (bf16, exact); the flash backward recomputes S and P from those and this forward's
            # normalisers, so the gradient is the gradient of the fp8 forward (straight-through
            # for the quantisations)
            lse_a = torch.empty((n, ops.hw_pad(hw)), dtype=torch.float32, device=dev)
            lse_b = torch.empty_like(lse_a)
            ctx.q = None
            if fp8:
                ctx.q = ops.coatt_f8_train(vat, va, vb, n, hw, za, zb, lse_a, lse_b)  # :160-170
            else:
                ops.coatt_flash_fwd(vat, va, vb, n, hw, za, zb, lse_a, lse_b)   # :160-170
            ctx.s = (va, vb, wf, vat, za, zb, lse_a, lse_b)
            ctx.flash = True
            ctx.link = link
            return za, zb
        ctx.flash = False
        S = torch.empty((n, hw, ldp), dtype=torch.float32, device=dev)
        ops.gemm(vat, vb, hw, hw, c, lda=c, ldb=ops.ld(vb), a_bs=hw * c, b_bs=hw * ops.ld(vb),
                 out=S, ldc=ldp, c_bs=hw * ldp, batch=n, tag="affinity")          # :160
        pc = torch.empty((n, hw, ldp), dtype=dt, device=dev)
        pt = torch.empty((n, hw, ldp), dtype=dt, device=dev)
        ws = torch.empty((int(nv.query("cn_coatt_workspace_floats", n, hw, ldp)),),
                         dtype=torch.float32, device=dev)
        nv.call("cn_coatt_softmax", nv.dtype_code(dt), S.data_ptr(), n, hw, ldp, pc.data_ptr(),
                pt.data_ptr(), ws.data_ptr(), nv.stream())                        # :164-165
        del S
        za = ops.gemm(pc, vb, hw, c, ldp, layout_b=ops.GEMM_MC, lda=ldp, ldb=ops.ld(vb),
                      a_bs=hw * ldp, b_bs=hw * ops.ld(vb), batch=n, kb_lim=hw)    # :170
        zb = ops.gemm(pt, va, hw, c, ldp, layout_b=ops.GEMM_MC, lda=ldp, ldb=ops.ld(va),
                      a_bs=hw * ldp, b_bs=hw * ops.ld(va), batch=n, kb_lim=hw)    # :169
        if _need(ctx):
            ctx.s = (va, vb, wf, pc, pt, za, zb)
        ctx.link = link
        return za, zb

    @staticmethod
    def backward(ctx, dza, dzb):
        if ctx.flash:
            return CoattFn._flash_backward(ctx, dza, dzb)
        va, vb, wf, pc, pt, za, zb = ctx.s
        n, hw, c, ldp = ctx.geo
        dt = va.dtype
        dev = va.device
        P = n * hw
        dv_link = ctx.link.pop("dv", None) if ctx.link is not None else None
        if dza is None and dzb is None:
            return dv_link, None, None, None, None, None
        dza = dza.contiguous() if dza is not None else None
        dzb = dzb.contiguous() if dzb is not None else None
        if dza is not None:
            dpc = torch.empty((n * hw, ldp), dtype=torch.float32, device=dev)
            ops.gemm(dza, vb, hw, hw, c, lda=c, ldb=ops.ld(vb), a_bs=hw * c, b_bs=hw * ops.ld(vb),
                     batch=n, out=dpc, ldc=ldp, c_bs=hw * ldp)
            d1 = torch.empty((P,), dtype=torch.float32, device=dev)
            nv.call("cn_rowdot", nv.dtype_code(dt), dza.data_ptr(), c, za.data_ptr(), c, P, c,
                    d1.data_ptr(), nv.stream())
        else:
            dpc = torch.zeros((n * hw, ldp), dtype=torch.float32, device=dev)
            d1 = torch.zeros((P,), dtype=torch.float32, device=dev)
        dpr = d2 = None
        if dzb is not None:
            dpr = torch.empty((n * hw, ldp), dtype=torch.float32, device=dev)
            ops.gemm(va, dzb, hw, hw, c, lda=ops.ld(va), ldb=c, a_bs=hw * ops.ld(va), b_bs=hw * c,
                     batch=n, out=dpr, ldc=ldp, c_bs=hw * ldp)
            d2 = torch.empty((P,), dtype=torch.float32, device=dev)
            nv.call("cn_rowdot", nv.dtype_code(dt), dzb.data_ptr(), c, zb.data_ptr(), c, P, c,
                    d2.data_ptr(), nv.stream())
        ds = torch.empty((n, hw, ldp), dtype=dt, device=dev)
        nv.call("cn_coatt_dscore", nv.dtype_code(dt), pc.data_ptr(), dpc.data_ptr(), d1.data_ptr(),
                nv.ptr(pt if dzb is not None else None), nv.ptr(dpr), nv.ptr(d2), n, hw, ldp,
                ds.data_ptr(), nv.stream())
        # dVa_t = dS . Vb
        dvat = ops.gemm(ds, vb, hw, c, ldp, layout_b=ops.GEMM_MC, lda=ldp, ldb=ops.ld(vb),
                        a_bs=hw * ldp, b_bs=hw * ops.ld(vb), batch=n, kb_lim=hw)
        dva = None
        if ctx.needs_input_grad[0]:
            dva = torch.empty((P, c), dtype=dt, device=dev)
            mode = 0
            if dv_link is not None:  # the concat's gradient for V_a (GateCatFn, link)
                ops.cast_copy(dv_link, dva)
                mode = 2
            if dzb is not None:  # dVa += P_row . dZb  (A = P_row[i][j] = PT[j][i], MC layout)
                ops.gemm(pt, dzb, hw, c, hw, layout_a=ops.GEMM_MC, layout_b=ops.GEMM_MC, lda=ldp,
                         ldb=c, a_bs=hw * ldp, b_bs=hw * c, out=dva, ldc=c, c_bs=hw * c, batch=n,
                         c_mode=mode)
                mode = 2
            # dVa += dVa_t . W   (B[n=ci][k=co] = W[co][ci] -> MC)
            ops.gemm(dvat, wf, P, c, c, layout_b=ops.GEMM_MC, lda=c, ldb=c, out=dva, ldc=c,
                     c_mode=mode)
        dw = None
        if ctx.needs_input_grad[2]:
            dw = torch.empty((c, c), dtype=torch.float32, device=dev)
            ns = max(1, min(64, P // 512))
            ops.gemm(dvat, va, c, c, P, layout_a=ops.GEMM_MC, layout_b=ops.GEMM_MC, lda=c,
                     ldb=ops.ld(va), out=dw, ldc=c, c_mode=0, nsplit=ns)
        return dva, None, dw, None, None, None

    @staticmethod
    def _flash_backward(ctx, dza, dzb):
        """Flash backward (coatt_flash.hip): dS never materialised.
          dVa_t = sum_j dS[i][j] Vb[j]                (cn_coatt_flash_dvat)
          dV_a  = [link] + sum_j P1[i][j] dZb[j]       (cn_coatt_flash_pv, S_row . dZ_b)
                  + dVa_t W                           (GEMM, the linear's input gradient)
          dW    = dVa_t^T V_a                         (GEMM, the linear's weight gradient)
        fp8 mode: S, P and dS from the decoded MX operands of the fp8 forward; the linear's
        GEMMs (bf16 in both modes) use the real V_a."""
        va, vb, wf, vat, za, zb, lse_a, lse_b = ctx.s
        n, hw, c, _ = ctx.geo
        dt = va.dtype
        dev = va.device
        P = n * hw
        dv_link = ctx.link.pop("dv", None) if ctx.link is not None else None
        if dza is None and dzb is None:
            return dv_link, None, None, None, None, None
        dza = dza.contiguous() if dza is not None else None
        dzb = dzb.contiguous() if dzb is not None else None
        need_va = ctx.needs_input_grad[0]
        dva = None
        mode = 0
        if need_va:
            dva = torch.empty((P, c), dtype=dt, device=dev)
            if dv_link is not None:
                ops.cast_copy(dv_link, dva)
                mode = 2
        # the operands the forward's products read: the decoded MX-fp8 ones in fp8 mode
        qvat, qva, qvb = ctx.q if ctx.q is not None else (vat, va, vb)
        ctx.q = None
        dvat = ops.coatt_flash_bwd(qvat, qva, qvb, wf, za, zb, lse_a, lse_b, dza, dzb, n, hw,
                                   dva=dva, dva_accumulate=mode == 2)
        if need_va:
            if dzb is not None:
                mode = 2
            # dVa += dVa_t . W   (B[n=ci][k=co] = W[co][ci] -> MC)
            ops.gemm(dvat, wf, P, c, c, layout_b=ops.GEMM_MC, lda=c, ldb=c, out=dva, ldc=c,
                     c_mode=mode)
        dw = None
        if ctx.needs_input_grad[2]:
            dw = torch.empty((c, c), dtype=torch.float32, device=dev)
            ns = max(1, min(64, P // 512))
            ops.gemm(dvat, va, c, c, P, layout_a=ops.GEMM_MC, layout_b=ops.GEMM_MC, lda=c,
                     ldb=ops.ld(va), out=dw, ldc=c, c_mode=0, nsplit=ns)
        return dva, None, dw, None, None, None


# ==============================================================================================
class GateCatFn(F):
    """out = cat([z * sigmoid(z.g + gb), v], 1); mask constant (no_grad) for the b side.
    With `link` (the dict given to the CoattFn that produced z from v), v's gradient is handed
    to that CoattFn's backward through link["dv"] (see CoattFn)."""

    @staticmethod
    def forward(ctx, z, v, g, gb, mask_const, link=None):
        P, c = z.shape
        dt = z.dtype
        out = torch.empty((P, 2 * c), dtype=dt, device=z.device)
        mask = torch.empty((P,), dtype=torch.float32, device=z.device)
        gflat = g.reshape(-1)
        nv.call("cn_gate_fwd", nv.dtype_code(dt), z.data_ptr(), ops.ld(z), P, c, gflat.data_ptr(),
                nv.ptr(gb), out.data_ptr(), 2 * c, mask.data_ptr(), nv.stream())
        ops.cast_copy(v, out[:, c:])
        if _need(ctx):
            ctx.s = (z, mask, gflat)
        ctx.mask_const = mask_const
        ctx.has_gb = gb is not None
        ctx.link = link
        return out

    @staticmethod
    def backward(ctx, dout):
        z, mask, gflat = ctx.s
        P, c = z.shape
        dt = z.dtype
        dz = torch.empty_like(z)
        through = not ctx.mask_const
        dg = torch.empty((c,), dtype=torch.float32, device=z.device) if through else None
        dgb = torch.empty((1,), dtype=torch.float32, device=z.device) if (through and ctx.has_gb) else None
        ws = ops.colpart_ws(P, c, z.device) if through else None
        nv.call("cn_gate_bwd", nv.dtype_code(dt), z.data_ptr(), ops.ld(z), dout.data_ptr(),
                ops.ld(dout), mask.data_ptr(), P, c, gflat.data_ptr(), int(through), dz.data_ptr(), c,
                nv.ptr(dg), nv.ptr(dgb), nv.ptr(ws), nv.stream())
        dv = dout[:, c:] if ctx.needs_input_grad[1] else None
        if dv is not None and ctx.link is not None:
            ctx.link["dv"] = dv   # summed into dV_a by the producing CoattFn's backward
            dv = None
        if dg is not None:
            dg = dg.view(1, c, 1, 1)
        return dz, dv, dg, dgb, None, None


class ConvFn(F):
    @staticmethod
    def forward(ctx, x, w, b, geo, k, stride, pad, dil):
        n, h, wd = geo
        dt = x.dtype
        wf, wt = WCACHE.get(w, dt)
        y, oh, ow = conv_fwd(x, n, h, wd, wf, w.shape[0], k, stride, pad, dil, bias=b)
        if _need(ctx):
            ctx.s = (x, wt)
        ctx.cfg = (n, h, wd, oh, ow, k, stride, pad, dil, w.shape[0], w.shape[1], b is not None)
        ctx.w = w
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wt = ctx.s
        n, h, wd, oh, ow, k, stride, pad, dil, cout, cin, has_b = ctx.cfg
        dy = dy if dy.stride(1) == 1 else dy.contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            dx = conv_dgrad(dy, n, oh, ow, wt, cin, k, stride, pad, dil, h, wd)
        dw = as_param_grad(conv_wgrad(x, n, h, wd, cin, dy, oh, ow, cout, k, stride, pad, dil), ctx.w)
        db = ops.colsum(dy) if has_b else None
        return dx, dw, db, None, None, None, None, None


class BNFn(F):
    @staticmethod
    def forward(ctx, x, g, b, bn):
        st = bn_stats(x, bn, bn.training)
        y = bn_apply(x, st, bn, act=0)
        if _need(ctx):
            ctx.s = (x, st)
        ctx.bn = bn
        ctx.training = bn.training
        return y

    @staticmethod
    def backward(ctx, dy):
        _check_train(ctx)
        x, st = ctx.s
        dy = dy if dy.stride(1) == 1 else dy.contiguous()
        dx, dg, db, _ = bn_bwd(x, dy, None, st, ctx.bn, act=0)
        return dx, dg, db, None


class HeadFn(F):
    """logit = relu(a + b) . w + bias  (b optional, relu optional) -> fp32 [P]"""

    @staticmethod
    def forward(ctx, a, b, w, bias, relu):
        P, c = a.shape
        dt = a.dtype
        z = torch.empty((P, c), dtype=dt, device=a.device) if _need(ctx) else None
        logit = torch.empty((P,), dtype=torch.float32, device=a.device)
        wflat = w.reshape(-1)
        nv.call("cn_head_fwd", nv.dtype_code(dt), a.data_ptr(), ops.ld(a), nv.ptr(b),
                ops.ld(b) if b is not None else 0, P, c, int(relu), wflat.data_ptr(), nv.ptr(bias),
                nv.ptr(z), c, logit.data_ptr(), nv.stream())
        if z is not None:
            ctx.s = (z, wflat)
        ctx.relu = relu
        ctx.has_b = b is not None
        ctx.wshape = w.shape
        return logit

    @staticmethod
    def backward(ctx, dlogit):
        z, wflat = ctx.s
        P, c = z.shape
        dz = torch.empty_like(z)
        dw = torch.empty((c,), dtype=torch.float32, device=z.device)
        db = torch.empty((1,), dtype=torch.float32, device=z.device)
        dlogit = dlogit.contiguous()
        ws = ops.colpart_ws(P, c, z.device)
        nv.call("cn_head_bwd", nv.dtype_code(z.dtype), z.data_ptr(), c, dlogit.data_ptr(), P, c,
                int(ctx.relu), wflat.data_ptr(), dz.data_ptr(), c, dw.data_ptr(), db.data_ptr(),
                ws.data_ptr(), nv.stream())
        return dz, (dz if ctx.has_b else None), dw.view(ctx.wshape), db, None


class UpSigFn(F):
    @staticmethod
    def forward(ctx, logit, geo, out_hw):
        n, h, w = geo
        H, W = out_hw
        out = torch.empty((n, 1, H, W), dtype=torch.float32, device=logit.device)
        nv.call("cn_upsample_sigmoid", logit.data_ptr(), n, h, w, H, W, 1, out.data_ptr(), nv.stream())
        ctx.save_for_backward(out)
        ctx.geo = (n, h, w, H, W)
        return out

    @staticmethod
    def backward(ctx, dout):
        (out,) = ctx.saved_tensors
        n, h, w, H, W = ctx.geo
        dout = dout.contiguous()
        dl = torch.empty((n * h * w,), dtype=torch.float32, device=out.device)
        nv.call("cn_upsample_sigmoid_bwd", dout.data_ptr(), out.data_ptr(), n, h, w, H, W, 1,
                dl.data_ptr(), nv.stream())
        return dl, None, None


def _scaled(dpred, gout):
    """dpred * gout with gout a device scalar (cn_scale_dev; no torch op, no host sync)."""
    out = torch.empty_like(dpred)
    g = gout.reshape(1).contiguous()
    if g.dtype != torch.float32:
        g = g.float()
    nv.call("cn_scale_dev", dpred.data_ptr(), dpred.numel(), g.data_ptr(), out.data_ptr(), nv.stream())
    return out


class BceL1DevFn(F):
    """BceL1Fn with the BCE weight N*H*W / #pos taken from a device count tensor (int64 [1]):
    no host synchronisation, so the whole train step can be captured in a HIP graph."""

    @staticmethod
    def forward(ctx, pred, gt, pos_count, total, l1w):
        pred = pred.contiguous()
        gt = gt.contiguous()
        n = pred.numel()
        ws = torch.empty((int(nv.query("cn_loss_workspace_floats", n)),), dtype=torch.float32,
                         device=pred.device)
        loss = torch.empty((), dtype=torch.float32, device=pred.device)
        dpred = torch.empty_like(pred) if _need(ctx) else None
        nv.call("cn_bce_l1_devcount", pred.data_ptr(), gt.data_ptr(), n, pos_count.data_ptr(),
                float(total), float(l1w), ws.data_ptr(), loss.data_ptr(), nv.ptr(dpred), nv.stream())
        ctx.dpred = dpred
        return loss

    @staticmethod
    def backward(ctx, gout):
        return _scaled(ctx.dpred, gout), None, None, None, None


class BceL1PairDevFn(F):
    """loss = BceL1(x1, gt_a) + BceL1(x2, gt_b) (train.py:595-597) in one Function: both
    losses and their sum by HIP kernels, both weights from device counts [2] (no host sync)."""

    @staticmethod
    def forward(ctx, x1, x2, gt_a, gt_b, cnt, total, l1w):
        two = torch.empty((2,), dtype=torch.float32, device=x1.device)
        need = _need(ctx)
        ds = []
        for i, (pred, gt) in enumerate(((x1, gt_a), (x2, gt_b))):
            pred = pred.contiguous()
            gt = gt.contiguous()
            n = pred.numel()
            ws = torch.empty((int(nv.query("cn_loss_workspace_floats", n)),), dtype=torch.float32,
                             device=pred.device)
            dpred = torch.empty_like(pred) if need else None
            nv.call("cn_bce_l1_devcount", pred.data_ptr(), gt.data_ptr(), n, cnt[i:i + 1].data_ptr(),
                    float(total), float(l1w), ws.data_ptr(), two[i:i + 1].data_ptr(), nv.ptr(dpred),
                    nv.stream())
            ds.append(dpred)
        loss = torch.empty((), dtype=torch.float32, device=x1.device)
        nv.call("cn_sum_rows", two.data_ptr(), 2, 1, loss.data_ptr(), nv.stream())
        ctx.ds = ds
        return loss

    @staticmethod
    def backward(ctx, gout):
        da, db = ctx.ds
        return _scaled(da, gout), _scaled(db, gout), None, None, None, None, None


class BceL1Fn(F):
    """weight * BCE(pred, gt) + l1w * L1(pred, gt), means over all elements (train.py:176-216)."""

    @staticmethod
    def forward(ctx, pred, gt, weight, l1w):
        pred = pred.contiguous()
        gt = gt.contiguous()
        n = pred.numel()
        ws = torch.empty((int(nv.query("cn_loss_workspace_floats", n)),), dtype=torch.float32,
                         device=pred.device)
        loss = torch.empty((), dtype=torch.float32, device=pred.device)
        dpred = torch.empty_like(pred) if _need(ctx) else None
        nv.call("cn_bce_l1", pred.data_ptr(), gt.data_ptr(), n, float(weight), float(l1w),
                ws.data_ptr(), loss.data_ptr(), nv.ptr(dpred), nv.stream())
        ctx.dpred = dpred
        return loss

    @staticmethod
    def backward(ctx, gout):
        return _scaled(ctx.dpred, gout), None, None, None


def count_positive(gt, out=None):
    """#(gt >= 0.5) on device (int64 tensor, no host sync), written into `out` if given."""
    cnt = torch.empty((1,), dtype=torch.int64, device=gt.device) if out is None else out
    g = gt.contiguous()
    nv.call("cn_count_ge", g.data_ptr(), g.numel(), 0.5, cnt.data_ptr(), nv.stream())
    return cnt
