"""train.py / test.py drop-in CLIs (reference train.py:73-111, :399-634; test.py:61-83,
:168-344), checkpoint format (train.py:624-626, test.py:140-161) and the synthetic dataset."""
import os
import re

import numpy as np
import pytest
import torch

from conftest import REPO

import train as train_cli
import test as test_cli
from cosnet_amd.checkpoint import convert_state_dict, load_checkpoint, save_snapshot, snapshot_path
from cosnet_amd.data import SyntheticRGBDPairs


def test_train_flags_match_reference_defaults():
    a = train_cli.get_arguments([])
    assert (a.learning_rate, a.weight_decay, a.momentum, a.power) == (0.00025, 0.0005, 0.9, 0.9)
    assert (a.random_seed, a.model) == (1234, "raa")
    a = train_cli.get_arguments(["--dataset", "sbmrgbd", "--model", "raa", "--gpus", "0,1",
                                 "--learning-rate", "1e-3", "--random-mirror"])
    assert a.learning_rate == 1e-3 and a.random_mirror and a.gpus == "0,1"


def test_train_configure_from_yaml(tmp_path):
    a = train_cli.get_arguments(["--dataset", "sbmrgbd", "--snapshot-root", str(tmp_path)])
    cfg = train_cli.load_config(a.config)
    train_cli.configure_dataset_init_model(a, cfg, "20260101_000000")
    assert a.batch_size == 4 and a.maxEpoches == 200 and a.output_HW == (240, 320)
    assert a.full_model_name == "resnet_aspp_add"
    assert a.snapshot_dir.endswith(os.path.join("snapshots", "sbmrgbd", "resnet_aspp_add", "H240W320",
                                                "20260101_000000"))
    with pytest.raises(Exception, match="Invalid model name"):
        train_cli.get_fullname_of_model("bogus")


def test_test_config_yaml_overrides_sample_range():
    a = test_cli.get_arguments(["--dataset", "synthetic", "--sample_range", "9"])
    import yaml
    with open(a.config) as f:
        cfg = yaml.safe_load(f)
    test_cli.config(a, cfg)
    assert a.sample_range == 5 and a.batch_size == 1
    assert a.image_HW_4_model == (240, 320) and a.output_WH == (320, 240)


def test_checkpoint_roundtrip_with_dataparallel_keys(tmp_path):
    import cosnet_amd as C
    torch.manual_seed(3)
    m = C.build_model()
    p = snapshot_path(str(tmp_path), "synthetic", "resnet_aspp_add", (240, 320), "t", 0)
    save_snapshot(p, 1, m, dataparallel_keys=True)
    ck = load_checkpoint(p)
    assert ck["epoch"] == 1 and all(k.startswith("module.") for k in ck["model"])
    assert len(ck["model"]) == 1059
    torch.manual_seed(4)
    m2 = C.build_model()
    m2.load_state_dict(convert_state_dict(ck["model"]))
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k


def test_synthetic_pairs_are_seeded_and_shaped():
    d = SyntheticRGBDPairs(3, (33, 45), 2, sample_range=2, seed=5)
    b = d[1]
    assert b["target"].shape == (2, 3, 33, 45) and b["target_depth"].shape == (2, 1, 33, 45)
    assert b["target_gt"].shape == (2, 33, 45) and b["search_1_depth"].shape == (2, 1, 33, 45)
    assert set(np.unique(b["target_gt"].numpy())) <= {0.0, 1.0}
    assert float(b["target_depth"].min()) >= 0 and float(b["target_depth"].max()) <= 255
    assert torch.equal(b["search_0"], SyntheticRGBDPairs(3, (33, 45), 2, sample_range=2, seed=5)[1]["search_0"])
    assert not torch.equal(b["target"], d[2]["target"])
    with pytest.raises(IndexError):
        d[3]


def _readlog_losses(path):
    """plot_from_log.py:10-22's parser."""
    out = []
    for line in open(path):
        if not line.startswith("Epoch["):
            continue
        parts = line.split("     ")
        if len(parts) > 2 and parts[1].startswith("Loss: "):
            out.append(float(parts[1].replace("Loss: ", "")))
    return out


@pytest.mark.gpu
def test_train_then_test_cli_end_to_end(cuda, tmp_path):
    rc = train_cli.main(["--dataset", "synthetic", "--model", "raa", "--gpus", "0",
                         "--max-epoches", "1", "--iters-per-epoch", "3",
                         "--snapshot-root", str(tmp_path)])
    assert rc == 0
    snaps = []
    logs = []
    for root, _, files in os.walk(str(tmp_path)):
        snaps += [os.path.join(root, f) for f in files if f.endswith(".pth")]
        logs += [os.path.join(root, f) for f in files if f.endswith("_train_log.txt")]
    assert len(snaps) == 1 and os.path.basename(snaps[0]) == "snapshot_synthetic_0.pth"
    losses = _readlog_losses(logs[0])
    assert len(losses) == 3 and all(np.isfinite(losses))
    ck = load_checkpoint(snaps[0])
    assert ck["epoch"] == 1 and len(ck["model"]) == 1059
    rc = test_cli.main(["--dataset", "synthetic", "--model", "raa", "--gpus", "0",
                        "--checkpoint", snaps[0], "--frames", "2", "--result-root", str(tmp_path)])
    assert rc == 0
    tl = []
    pngs = []
    for root, _, files in os.walk(os.path.join(str(tmp_path), "vos_test_results")):
        tl += [os.path.join(root, f) for f in files if f.endswith("_test_log.txt")]
        pngs += [f for f in files if f.endswith(".png")]
    text = open(tl[0]).read()
    ious = [float(x) for x in re.findall(r"IOU: ([0-9.eE+-]+)==##", text)]
    assert len(ious) == 3 and len(pngs) == 2  # 2 frames + the final mean
    assert 0.0 <= ious[-1] <= 1.0 and abs(ious[-1] - np.mean(ious[:2])) < 1e-12


def _bench_json(out):
    import json
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_gpus_n_spawns_n_ranks():
    """`bench.py --gpus 2` (no WORLD_SIZE: the driver's BENCH command shape) starts a child
    torch.distributed.run with 2 ranks and relays rank 0's single JSON line
    (reference train.py:491-496: one replica per GPU of --gpus)."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--dist-backend", "gloo", "--steps", "1", "--cpu-baseline", "0",
                        "--no-roofline", "--dry-run"],
                       env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    j = _bench_json(r.stdout)
    assert j["n_gpus"] == 2 and j["config"]["parallelism"] == "dp2"
    assert j["max_rank_seconds"] >= 0.02          # max over ranks: rank 1 sleeps 20 ms


@pytest.mark.gpu
def test_bench_gpus_2_gloo_rehearsal_on_one_device(cuda):
    """The same spawn path with the real model: 2 ranks on the box's one device over gloo
    (the RCCL/xGMI figure is the driver's 8-GPU run), small shape to stay short."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--dist-backend", "gloo", "--steps", "2", "--warmup", "2",
                        "--cpu-baseline", "0", "--no-roofline", "--batch", "2", "--size", "97"],
                       env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    j = _bench_json(r.stdout)
    assert j["n_gpus"] == 2 and j["config"]["parallelism"] == "dp2"
    assert j["config"]["global_batch"] == 4 and j["value"] > 0 and np.isfinite(j["config"]["loss"])
