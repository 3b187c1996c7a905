"""Run bench.py with BN launch-shape knobs set first (cn_bn_set_tuning keys: 0 stats blocks,
1 stats rows, 2 apply blocks, 3 apply rows, 4 bwd-reduce blocks, 5 rows, 6 bwd-apply blocks,
7 rows).  usage: python tools/bn_tune_ab.py KEY=VALUE[,KEY=VALUE...] -- bench args"""
import runpy
import sys

sys.path.insert(0, ".")
from cosnet_amd import _native as nv  # noqa: E402

spec, rest = sys.argv[1], sys.argv[3:]
if spec != "default":
    for kv in spec.split(","):
        k, v = kv.split("=")
        nv.call("cn_bn_set_tuning", int(k), int(v))
sys.argv = ["bench.py"] + rest
runpy.run_path("bench.py", run_name="__main__")
