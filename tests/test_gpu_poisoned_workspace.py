"""Every caller-owned buffer the HIP path allocates uninitialised (BN / split-K / epilogue
workspaces, partial slabs, outputs) must be fully written before it is read.

This is the kernel-level test that would have caught round 2's wrong-result variant (DESIGN.md
§3.3: an in-launch BN finalize whose ticket-counter words aliased an earlier call's slab bytes, so
a counter started non-zero, the "last arriver" fired on stale partials and x1 came out 0.84 off).
Here every `torch.empty` / `empty_like` of the product modules returns memory filled with NaN
(floating point) or 0xA5 bytes (integer), and one layer-3 bottleneck forward + backward and the
stem (conv, BN statistics via the GEMM epilogue and via the separate pass, BN apply, BN backward
reduce / apply, split-K weight gradients) must be BITWISE equal to the same calls on
zero-initialised memory.  Any read of a stale or unwritten word (a counter, a partial, a padded
channel) shows up as a NaN or a changed bit."""
import pytest
import torch

import cosnet_amd as C
from cosnet_amd import encoder_fn as E
from cosnet_amd import ops
from cosnet_amd.init_recipe import recipe_state_dict

pytestmark = pytest.mark.gpu


class _Alloc:
    """Proxy of the torch module whose empty / empty_like fill the new memory."""

    def __init__(self, real, poison):
        self._real, self._poison = real, poison

    def __getattr__(self, k):
        return getattr(self._real, k)

    def _fill(self, t):
        if t.is_floating_point():
            t.fill_(float("nan") if self._poison else 0.0)
        elif t.dtype != torch.bool:
            t.fill_(0xA5 if self._poison and t.dtype == torch.uint8 else (-0x5A5A if self._poison else 0))
        return t

    def empty(self, *a, **k):
        return self._fill(self._real.empty(*a, **k))

    def empty_like(self, *a, **k):
        return self._fill(self._real.empty_like(*a, **k))


def _run(cuda, monkeypatch, poison):
    from cosnet_amd import functions
    for mod in (ops, E, functions):
        monkeypatch.setattr(mod, "torch", _Alloc(torch, poison))
    torch.manual_seed(0)
    m = C.build_model(torch.bfloat16)
    m.load_state_dict(recipe_state_dict(m.state_dict()))
    m = m.to(cuda).train()
    g = torch.Generator().manual_seed(5)
    n1, h, w = 2, 60, 60
    out = {}
    # layer-3 block (fused BN-statistics / BN-backward epilogues on its 1024-deep convs)
    blk = m.encoder.backbone.layer3[3]
    x = torch.relu(torch.randn((2 * n1 * h * w, 1024), generator=g)).to(torch.bfloat16).to(cuda)
    dy = (torch.randn((n1 * h * w, 1024), generator=g) * 0.1).to(torch.bfloat16).to(cuda)
    rec = []
    out["y"], _ = E.bottleneck_fwd(blk, x, (2 * n1, h, w), 2, rec)
    grads = E.GradSink()
    out["dx"] = E.bottleneck_bwd(rec[0], dy, grads)
    for i, p in enumerate((blk.conv1.weight, blk.conv2.weight, blk.conv3.weight, blk.bn1.weight,
                           blk.bn2.bias, blk.bn3.weight)):
        out["g%d" % i] = grads[p]
    # stem (input conversion with padded channels, 7x7 conv, separate BN statistics pass, maxpool)
    img = (torch.rand((n1, 3, 97, 97), generator=g) * 255).to(cuda)
    rec = []
    out["stem"], _ = E.stem_fwd(m.encoder.backbone, (img, img.flip(3)), 2, torch.bfloat16, rec)
    sg = E.GradSink()
    E.stem_bwd(rec[0], (torch.randn(out["stem"][:out["stem"].shape[0] // 2].shape, generator=g) * 0.1)
               .to(torch.bfloat16).to(cuda), sg)
    out["stem_dw"] = sg[m.encoder.backbone.conv1.weight]
    out["rm"] = blk.bn2.running_mean.clone()
    torch.cuda.synchronize()
    return {k: v.detach().float().cpu() for k, v in out.items()}


def test_uninitialised_buffers_are_never_read(cuda, monkeypatch):
    clean = _run(cuda, monkeypatch, poison=False)
    dirty = _run(cuda, monkeypatch, poison=True)
    for k in clean:
        assert torch.isfinite(clean[k]).all(), k
        assert torch.equal(clean[k], dirty[k]), (k, (clean[k] - dirty[k]).abs().max().item())


def test_coatt_f8_workspace_tail_is_never_read(cuda, monkeypatch):
    """The MX-fp8 co-attention's workspace (row images, V^T tiles, E8M0 scales) at HW = 3600,
    where the 64-key padding (3648) leaves half a 128-row query block: the last block's Q rows and
    scales must come from the zero-padded image of its own batch entry, never from whatever the
    workspace holds next (0xA5 bytes = finite e4m3 values with 2^38 scales when poisoned)."""
    n, hw, c = 2, 3600, 256
    g = torch.Generator().manual_seed(9)
    vat, va, vb = [(torch.randn((n * hw, c), generator=g) * 0.7).to(torch.bfloat16).to(cuda)
                   for _ in range(3)]
    res = []
    for poison in (False, True):
        monkeypatch.setattr(ops, "torch", _Alloc(torch, poison))
        za = torch.zeros((n * hw, c), dtype=torch.bfloat16, device=cuda)
        zb = torch.zeros_like(za)
        la = torch.zeros((n, ops.hw_pad(hw)), dtype=torch.float32, device=cuda)
        lb = torch.zeros_like(la)
        ops.coatt_f8(vat, va, vb, n, hw, za, zb, la, lb)
        torch.cuda.synchronize()
        res.append([t.float().cpu() for t in (za, zb, la[:, :hw], lb[:, :hw])])
    for a, b in zip(*res):
        assert torch.isfinite(a).all() and torch.equal(a, b)
