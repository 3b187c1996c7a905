"""Per-shape throughput of the implicit-GEMM kernel for the convs of one 473x473 B=4 step."""
import sys, torch, time
sys.path.insert(0, '.')
from cosnet_amd import ops
dev = torch.device('cuda:0')
dt = torch.bfloat16 if (len(sys.argv) < 2 or sys.argv[1] == 'bf16') else torch.float32
# n, cin, h, w, cout, k, stride, pad, dil, count-per-step-ish
SHAPES = [
    ("stem7x7", 4, 8, 473, 473, 64, 7, 2, 3, 1),
    ("l1_1x1_256to64", 4, 256, 119, 119, 64, 1, 1, 0, 1),
    ("l1_3x3_64", 4, 64, 119, 119, 64, 3, 1, 1, 1),
    ("l1_1x1_64to256", 4, 64, 119, 119, 256, 1, 1, 0, 1),
    ("l2_3x3_128", 4, 128, 60, 60, 128, 3, 1, 1, 1),
    ("l3_1x1_1024to256", 4, 1024, 60, 60, 256, 1, 1, 0, 1),
    ("l3_3x3_256_d2", 4, 256, 60, 60, 256, 3, 1, 2, 2),
    ("l3_1x1_256to1024", 4, 256, 60, 60, 1024, 1, 1, 0, 1),
    ("l4_3x3_512_d4", 4, 512, 60, 60, 512, 3, 1, 4, 4),
    ("aspp_3x3_2048to512_d12", 4, 2048, 60, 60, 512, 3, 1, 12, 12),
    ("aspp_bott_2560to256", 4, 2560, 60, 60, 256, 3, 1, 1, 1),
]
def bench(fn, reps=20):
    fn(); torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3
for (name, n, cin, h, w, cout, k, s, p, d) in SHAPES:
    x = torch.randn(n * h * w, cin, device=dev).to(dt)
    wp = (torch.randn(cout, cin, k, k, device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
    wf, wt = ops.WCACHE.get(wp, dt)
    y, oh, ow = ops.conv_fwd(x, n, h, w, wf, cout, k, s, p, d)
    fl = 2.0 * n * oh * ow * cout * k * k * cin
    tf = bench(lambda: ops.conv_fwd(x, n, h, w, wf, cout, k, s, p, d, out=y))
    dy = torch.randn_like(y)
    dw = torch.zeros(cout, k * k * cin, device=dev)
    tw = bench(lambda: ops.conv_wgrad(x, n, h, w, cin, dy, oh, ow, cout, k, s, p, d, dw=dw))
    res = "%-24s M=%7d N=%5d K=%6d  fwd %7.1f TF (%6.1f us)  wgrad %7.1f TF (%6.1f us)" % (
        name, n * oh * ow, cout, k * k * cin, fl / tf / 1e12, tf * 1e6, fl / tw / 1e12, tw * 1e6)
    if s == 1 and name != "stem7x7":
        dx = torch.empty_like(x)
        td = bench(lambda: ops.conv_dgrad(dy, n, oh, ow, wt, cin, k, s, p, d, h, w, out=dx))
        res += "  dgrad %7.1f TF (%6.1f us)" % (fl / td / 1e12, td * 1e6)
    print(res, flush=True)
