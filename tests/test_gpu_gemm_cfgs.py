"""Every bf16 tile configuration of the implicit GEMM (gemm.hip kCfg, forced with
cn_gemm_force_config) on the operand kinds the heuristic can route to it: conv forward (1x1
dense and 3x3 gathered loaders), stride-1 dgrad, the BN-statistics and BN-backward epilogues,
and the weight gradient (transposed loaders; the ping-pong ids fall back there) -- against torch
fp64, at shapes whose M, N and K all end in partial tiles.  The ping-pong tiles (ids 18-20)
change the K loop's synchronisation (and 24-25, the K-split wave groups, sum two partial
accumulators), so each is also run several times on the same inputs and
must give bitwise-identical results (a fragment read racing an LDS-DMA fill shows up as
run-to-run differences)."""
import pytest
import torch

from cosnet_amd import _native as nv

import test_gpu_kernels as K

pytestmark = pytest.mark.gpu

CFGS = [11, 13, 10, 15, 4, 18, 19, 20, 21, 22, 23, 24, 25]
EPI_CFGS = {10, 11, 12, 13, 18, 19, 20, 21, 22, 24, 25}   # the tiles launch_epi instantiates


EXPERIMENTAL_CFGS = {21, 22, 23, 24, 25}   # development builds only (make EXPERIMENTAL=1)


@pytest.fixture
def force_cfg(request):
    lib = nv.load()
    cfg = request.node.callspec.params.get("cfg") if hasattr(request.node, "callspec") else None
    if cfg in EXPERIMENTAL_CFGS and not lib.cn_build_experimental():
        assert lib.cn_gemm_force_config(cfg) == -1   # the product library refuses it
        pytest.skip("tile configuration %d is built only with EXPERIMENTAL=1 (COSNET_HIP_LIB)" % cfg)
    yield lib.cn_gemm_force_config
    lib.cn_gemm_force_config(-1)


@pytest.mark.parametrize("cfg", CFGS)
def test_conv_paths_per_config(cuda, force_cfg, cfg):
    assert force_cfg(cfg) > cfg
    bf = torch.bfloat16
    for case in [(2, 96, 21, 23, 320, 1, 1, 0, 1), (2, 128, 19, 21, 192, 3, 1, 2, 2),
                 (1, 64, 9, 9, 512, 3, 1, 6, 6)]:
        K.test_conv_fwd_dgrad_wgrad(cuda, bf, case)
    if cfg not in EPI_CFGS:
        return
    for case in [(2, 64, 13, 11, 128, 1, 1, 0, 1, 2), (1, 256, 30, 20, 256, 1, 1, 0, 1, 2),
                 (2, 128, 15, 9, 384, 3, 1, 1, 1, 1)]:
        K.test_conv_fwd_bn_epilogue_stats(cuda, bf, case)
    for case in [(4, 256, 30, 30, 64, 3, 1, 1), (1, 128, 9, 9, 256, 1, 0, 1)]:
        K.test_conv_dgrad_bn_epilogue_reduce(cuda, bf, case)


@pytest.mark.parametrize("cfg", [18, 19, 20, 24, 25])
def test_ping_pong_tiles_are_deterministic(cuda, force_cfg, cfg):
    from cosnet_amd import ops
    force_cfg(cfg)
    g = torch.Generator(device="cpu").manual_seed(cfg)
    n, cin, h, w, cout, k, pad, dil = 4, 256, 45, 47, 256, 3, 2, 2
    x = torch.randn((n * h * w, cin), generator=g).to(torch.bfloat16).to(cuda)
    wp = (torch.randn((cout, cin, k, k), generator=g) * 0.03).to(cuda).contiguous(memory_format=torch.channels_last)
    wf, _ = ops.WCACHE.get(wp, torch.bfloat16)
    outs = []
    for _ in range(6):
        y, _, _ = ops.conv_fwd(x, n, h, w, wf, cout, k, 1, pad, dil)
        outs.append(y)
    torch.cuda.synchronize()
    for y in outs[1:]:
        assert torch.equal(y, outs[0])
