"""Shader clock and socket power around bench.py's phases (read-only amdsmi queries, ~5 ms apart
from a sampler thread): idle, the recorded bf16 train step (configs[1]: 473x473, 4 pairs), then
the configs[3] co-attention graph replays right after it, each replay's time printed beside the
clock it ran at.  The question it answers: is the configs[3] kernel's speed-up over the first
tens of ms after the training lines (162 -> 144 us per launch in a trace) the clocks recovering?

    python tools/clock_probe.py [train_seconds] [coatt_seconds]
"""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    t_train = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
    t_co = float(sys.argv[2]) if len(sys.argv) > 2 else 0.6
    import amdsmi
    import torch
    import cosnet_amd as C
    from cosnet_amd import ops
    from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs
    from cosnet_amd.optim import SGD, reference_param_groups
    from cosnet_amd.train_step import TrainStep

    amdsmi.amdsmi_init()
    h = amdsmi.amdsmi_get_processor_handles()[0]
    samples = []            # (t, gfx MHz, socket W, {MEM, DF, SOC} MHz)
    stop = threading.Event()
    t0 = time.perf_counter()

    def sampler():
        while not stop.is_set():
            try:
                clk = amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.GFX).get("clk")
            except Exception as e:   # report, keep sampling
                clk = repr(e)
            other = {}
            for k in ("MEM", "DF", "SOC"):
                try:
                    other[k] = amdsmi.amdsmi_get_clock_info(h, getattr(amdsmi.AmdSmiClkType, k)).get("clk")
                except Exception as e:
                    other[k] = type(e).__name__
            try:
                p = amdsmi.amdsmi_get_power_info(h)
                pw = p.get("current_socket_power", p.get("average_socket_power"))
            except Exception as e:
                pw = repr(e)
            samples.append((time.perf_counter() - t0, clk, pw, other))
            time.sleep(0.005)

    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    marks = {}

    def mark(name):
        torch.cuda.synchronize()
        marks[name] = time.perf_counter() - t0

    dev = torch.device("cuda:0")
    time.sleep(1.0)
    mark("idle_end")
    m = C.build_model(torch.bfloat16)
    m.load_state_dict(recipe_state_dict(m.state_dict()))
    m.encoder.main_classifier.requires_grad_(False)
    m = m.to(dev).train()
    g0, g1 = reference_param_groups(m)
    opt = SGD([g0, g1], [2.5e-6, 2.5e-3], momentum=0.9, weight_decay=5e-4)
    st = TrainStep(m, opt, 4, 473, graphed=True)
    st.load(*[t.to(dev) for t in synthetic_inputs(4, 473, 473, seed=1234)])
    st.capture(warmup=3)
    mark("train_start")
    n = 0
    while time.perf_counter() - t0 - marks["train_start"] < t_train:
        st([2.5e-6, 2.5e-3])
        n += 1
        if n % 10 == 0:
            torch.cuda.synchronize()
    mark("train_end")
    train_ms = (marks["train_end"] - marks["train_start"]) / n * 1e3

    g = torch.Generator(device="cpu").manual_seed(3)
    nn, hw, c, iters = 5, 3600, 256, 20
    vat, va, vb = [(torch.randn((nn * hw, c), generator=g) * 0.7).to(torch.bfloat16).to(dev)
                   for _ in range(3)]
    za, zb = torch.empty_like(va), torch.empty_like(va)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            ops.coatt_fused(vat, va, vb, nn, hw, za, zb)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        for _ in range(iters):
            ops.coatt_fused(vat, va, vb, nn, hw, za, zb)
    mark("coatt_start")
    reps = []
    while time.perf_counter() - t0 - marks["coatt_start"] < t_co:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        graph.replay()
        e1.record()
        torch.cuda.synchronize()
        reps.append((time.perf_counter() - t0, e0.elapsed_time(e1) * 1e3 / iters))
    mark("coatt_end")
    stop.set()
    th.join()
    amdsmi.amdsmi_shut_down()

    def phase(a, b):
        xs = [x for x in samples if a <= x[0] < b and isinstance(x[1], (int, float))]
        if not xs:
            return "no samples"
        clks = sorted(x[1] for x in xs)
        pws = sorted(x[2] for x in xs if isinstance(x[2], (int, float)))
        med = lambda v: v[len(v) // 2] if v else None
        oth = {k: sorted(x[3][k] for x in xs if isinstance(x[3].get(k), (int, float)))
               for k in ("MEM", "DF", "SOC")}
        return ("%d samples, gfx clock median %s MHz (min %s, max %s), socket power median %s W, "
                "MEM / DF / SOC median %s / %s / %s MHz (min %s / %s / %s)" % (
                    len(xs), med(clks), clks[0], clks[-1], med(pws),
                    med(oth["MEM"]), med(oth["DF"]), med(oth["SOC"]),
                    oth["MEM"][0] if oth["MEM"] else None, oth["DF"][0] if oth["DF"] else None,
                    oth["SOC"][0] if oth["SOC"] else None))

    print("idle:        ", phase(0.2, marks["idle_end"]))
    print("train step:  ", phase(marks["train_start"] + 0.5, marks["train_end"]),
          "| %.2f ms/step over %d steps" % (train_ms, n))
    print("co-attention:", phase(marks["coatt_start"], marks["coatt_end"]))
    print("co-attention replays (time since the training lines ended, us per launch, nearest clock):")
    for t, us in reps[:40]:
        near = min(samples, key=lambda x: abs(x[0] - t))
        print("  +%6.1f ms  %6.1f us  gfx %s MHz  %s W  %s" % ((t - marks["train_end"]) * 1e3, us,
                                                             near[1], near[2], near[3]))
    if len(reps) > 40:
        t, us = reps[-1]
        print("  ... last: +%.1f ms  %.1f us (%d replays)" % ((t - marks["train_end"]) * 1e3, us, len(reps)))


if __name__ == "__main__":
    main()
