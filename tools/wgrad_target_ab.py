"""Run bench.py with the weight-gradient K-split block target set first
(cn_gemm_set_wgrad_target; default 512).  usage: python tools/wgrad_target_ab.py N|default -- bench args"""
import runpy
import sys

sys.path.insert(0, ".")
from cosnet_amd import _native as nv  # noqa: E402

spec, rest = sys.argv[1], sys.argv[3:]
if spec != "default":
    nv.call("cn_gemm_set_wgrad_target", int(spec))
sys.argv = ["bench.py"] + rest
runpy.run_path("bench.py", run_name="__main__")
