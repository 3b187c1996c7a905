"""SBM-RGBD input pipeline: cosnet_amd.sbm_rgbd against the numpy
restatement oracle/sbm_ref.py (dataloaders/sbm_rgbd_loader.py, dataloaders/utils.py).
The cv2.resize arithmetic itself is restated from OpenCV's rules (cv2 is not installed):
parity of that part is unpinned; the file logic and ROI quirks follow the reference code."""
import os

import numpy as np
import pytest
import torch

from oracle import sbm_ref
from cosnet_amd import sbm_rgbd as S


def _roi_masks():
    g = np.random.default_rng(3)
    out = []
    for h, w in [(48, 64), (33, 41), (20, 20)]:
        m = np.zeros((h, w), np.uint8)
        y0, y1 = sorted(g.integers(0, h, 2))
        x0, x1 = sorted(g.integers(0, w, 2))
        m[y0:y1 + 1, x0:x1 + 1] = 255
        out.append(m)
        out.append(np.full((h, w), 255, np.uint8))             # no zero at all: the quirk path
        r = (g.random((h, w)) > 0.2).astype(np.uint8) * 255     # ragged mask
        out.append(r)
    return out


def test_find_roi_matches_reference_loops():
    for m in _roi_masks():
        assert [list(v) for v in S.find_roi(m)] == [list(v) for v in sbm_ref.find_roi(m)]


def test_roi_window_python_slice_semantics():
    m = np.full((12, 16), 255, np.uint8)   # reference: boundaries (-1, len) -> img[-1:len+1]
    roi = S.find_roi(m)
    y0, y1, x0, x1 = S.roi_window(roi, 12, 16)
    ref = sbm_ref.roi_crop(np.arange(12 * 16).reshape(12, 16), roi)
    assert ref.shape == (y1 - y0, x1 - x0)
    assert np.array_equal(np.arange(12 * 16).reshape(12, 16)[y0:y1, x0:x1], ref)


def _write_tree(root, seqs=(("Shadows", "s1", 4), ("OutOfRange", "s2", 3)), hw=(40, 52)):
    from PIL import Image
    g = np.random.default_rng(11)
    h, w = hw
    for cat, seq, nf in seqs:
        base = os.path.join(root, cat, seq)
        for d in ("input", "depth", "groundtruth"):
            os.makedirs(os.path.join(base, d), exist_ok=True)
        roi = np.zeros((h, w), np.uint8)
        roi[3:h - 4, 5:w - 2] = 255
        Image.fromarray(roi).save(os.path.join(base, "ROI.bmp"))
        for i in range(nf):
            fid = "%06d" % (10 * i + 7)
            Image.fromarray(g.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(
                os.path.join(base, "input", "in%s.png" % fid))
            Image.fromarray(g.integers(0, 256, (h, w), dtype=np.uint8)).save(
                os.path.join(base, "depth", "d%s.png" % fid))
            gt = (g.random((h, w)) > 0.7).astype(np.uint8) * 255
            Image.fromarray(gt).save(os.path.join(base, "groundtruth", "gt%s.png" % fid))
        # an unlabelled input frame and a stray file are ignored (only gt ids count)
        Image.fromarray(g.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(
            os.path.join(base, "input", "in999999.png"))


def test_file_scan_and_splits(tmp_path):
    _write_tree(str(tmp_path))
    ds = S.SBMRGBD(str(tmp_path), 1, (24, 32), for_training=False, batch_size=2, subset_percentage=1.0,
                   device="cpu")
    names = [str(f) for f in ds.sets["test"]["names_of_frames"]]
    assert len(names) == 7 and len(ds) == 6          # floored to a batch multiple (:583-588)
    assert sorted(ds.ROI) == [os.path.join("OutOfRange", "s2"), os.path.join("Shadows", "s1")]
    sub = {os.path.join("Shadows", "s1"): ["000017", "000007"]}
    ds2 = S.SBMRGBD(str(tmp_path), 1, (24, 32), for_training=False, subset=sub, device="cpu")
    assert [f.id for f in ds2.sets["test"]["names_of_frames"]] == ["000017", "000007"]
    tr = S.SBMRGBD(str(tmp_path), 1, (24, 32), for_training=True, batch_size=2, subset_percentage=0.5,
                   device="cpu")
    rng = tr.sets["train"]["frame_range_of_sequences"]
    assert all(r["end"] - r["start"] == 2 for r in rng.values())  # floor(n * 0.5) -> >= 2 in train


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("flip", [False, True])
def test_frame_resize_kernel(cuda, mode, flip):
    g = np.random.default_rng(5)
    for (h, w), (H, W), win in [((40, 52), (24, 32), (3, 36, 5, 50)), ((17, 23), (45, 61), (0, 17, 0, 23)),
                                ((60, 60), (60, 60), (2, 59, 1, 58)), ((31, 41), (13, 7), (4, 30, 2, 39))]:
        img = g.integers(0, 256, (h, w, 3), dtype=np.uint8)
        mean = (104.0, 116.7, 122.7)
        out = S.frame_resize(torch.from_numpy(img).to(cuda), win, (H, W), mode, flip=flip,
                             mean=mean, channels_last=True).cpu().numpy()
        y0, y1, x0, x1 = win
        ref = []
        for c in range(3):
            p = img[:, :, c].astype(np.float32) - np.float32(mean[c])
            r = sbm_ref.resize(p[y0:y1, x0:x1], (H, W), mode)
            ref.append(np.fliplr(r) if flip else r)
        ref = np.stack(ref)
        assert out.shape == ref.shape
        np.testing.assert_allclose(out, ref, rtol=0, atol=2e-4 if mode == 0 else 0)


@pytest.mark.gpu
@pytest.mark.parametrize("train", [False, True])
def test_load_frame_matches_restatement(cuda, tmp_path, train):
    _write_tree(str(tmp_path))
    ds = S.SBMRGBD(str(tmp_path), 1, (24, 32), for_training=train, batch_size=1, subset_percentage=1.0,
                   seed=9, device=cuda)
    ds.next_batch()
    fi = ds.sets[ds.stage]["names_of_frames"][2]
    state = ds.rng.getstate()
    rgb, dep, gt = ds.load_frame(fi)
    # replay the same random draws for the restatement
    ds.rng.setstate(state)
    roi = ds.ROI[fi.seq_name]
    tr = None
    if train:
        hh, ww = 24, 32
        ch, cw = int(ds._crop_ratio * hh), int(ds._crop_ratio * ww)
        oy = ds.rng.choice(range(hh - ch))
        off = {"x": ds.rng.choice(range(ww - cw)), "y": oy}
        tr = (ds._crop_ratio, off, ds._scale_ratio, ds.flip_prob[fi.seq_name] > 0.5)
    bgr = S.read_png(ds._path(fi, "input", fi.name_of_rgb_frame), "color")
    d = S.read_png(ds._path(fi, "depth", fi.name_of_depth_frame), "gray")
    gt0 = (S.read_png(ds._path(fi, "groundtruth", fi.name_of_groundtruth_frame), "gray") != 0).astype(np.uint8)
    r_rgb = sbm_ref.prepare([bgr[:, :, c] for c in range(3)], roi, (24, 32), 0, mean=ds.meanval, train=tr)
    r_dep = sbm_ref.prepare([d], roi, (24, 32), 0, train=tr)
    r_gt = sbm_ref.prepare([gt0], roi, (24, 32), 1, train=tr)[0]
    np.testing.assert_allclose(rgb.cpu().numpy(), r_rgb, rtol=0, atol=3e-4)
    np.testing.assert_allclose(dep.cpu().numpy(), r_dep, rtol=0, atol=3e-4)
    assert np.array_equal(gt.cpu().numpy(), r_gt.astype(np.uint8))
    if train:
        assert rgb.shape[1:] == (int(int(ds._crop_ratio * 24) * ds._scale_ratio),
                                 int(int(ds._crop_ratio * 32) * ds._scale_ratio))


@pytest.mark.gpu
def test_train_and_test_cli_on_sbm_tree(cuda, tmp_path):
    """train.py / test.py --dataset sbmrgbd over a small SBM-RGBD-shaped tree (eager, augmented
    batches of changing size), then the N-reference evaluation with soft-J logging."""
    import re
    import yaml
    import train as train_cli
    import test as test_cli
    root = os.path.join(str(tmp_path), "sbm")
    _write_tree(root, seqs=(("Shadows", "s1", 4), ("OutOfRange", "s2", 4)), hw=(72, 96))
    cfg = yaml.safe_load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                           "config.yaml")))
    cfg["train"]["dataset"]["sbmrgbd"].update({"data_path": root, "batch_size": 2, "output_HW": "64,80",
                                               "subset": {}})
    cfg["test"]["dataset"]["sbmrgbd"].update({"data_path": root, "output_WH": "80,64",
                                              "image_HW_4_model": "64,80", "sample_range": 2, "subset": {}})
    cpath = os.path.join(str(tmp_path), "config.yaml")
    with open(cpath, "w") as f:
        yaml.safe_dump(cfg, f)
    rc = train_cli.main(["--dataset", "sbmrgbd", "--model", "raa", "--gpus", "0", "--config", cpath,
                         "--max-epoches", "1", "--snapshot-root", str(tmp_path)])
    assert rc == 0
    snaps = [os.path.join(r, f) for r, _, fs in os.walk(os.path.join(str(tmp_path), "snapshots"))
             for f in fs if f.endswith(".pth")]
    assert len(snaps) == 1
    rc = test_cli.main(["--dataset", "sbmrgbd", "--model", "raa", "--gpus", "0", "--config", cpath,
                        "--checkpoint", snaps[0], "--result-root", str(tmp_path)])
    assert rc == 0
    logs = [os.path.join(r, f) for r, _, fs in os.walk(os.path.join(str(tmp_path), "vos_test_results"))
            for f in fs if f.endswith("_test_log.txt")]
    ious = [float(x) for x in re.findall(r"IOU: ([0-9.eE+-]+)==##", open(logs[0]).read())]
    assert len(ious) == 8 + 1 and all(0.0 <= v <= 1.0 for v in ious)


def test_graph_cache_policy_on_loader_sizes():
    """ShapeGraphCache's admission policy (no GPU: TrainStep is never built here) on the frame
    sizes the loader produces (per-batch uniform scale 0.7-1.3 x crop 0.8-1, sbm_rgbd_loader.py:
    700-702, output 473x473): ~340 distinct sizes, so 24 LRU slots hit on under 20 % of batches.
    Sizes are recorded at most once (an evicted size stays eager), so the records are bounded by
    the number of distinct sizes instead of growing with every batch; train.py leaves the cache
    off by default."""
    import random
    from cosnet_amd.train_step import ShapeGraphCache
    import train
    assert train.get_arguments(["--dataset", "sbmrgbd"]).graph_cache == 0
    rng = random.Random(0)
    c = ShapeGraphCache(None, None, 4, capacity=24, min_hits=2)
    seen = set()
    n = 3000
    for _ in range(n):
        scale, crop = rng.uniform(0.7, 1.3), rng.uniform(0.8, 1)
        _, hw = S.augmented_hw(473, 473, crop, scale)
        seen.add(hw)
        c.admit(hw, 4)
    assert c.hits + c.records + c.eager_steps == n
    assert c.hits / n < 0.2 and c.records <= len(seen), (c.hits, c.records, len(seen))
    assert len(c.evicted) == c.records - len(c.graphs)
    # a recurring size is recorded once and then replayed
    c2 = ShapeGraphCache(None, None, 2, capacity=2, min_hits=2)
    acts = [c2.admit(hw, 2) for hw in [(65, 81), (65, 81), (65, 81), (49, 65), (49, 65), (73, 57),
                                       (73, 57), (65, 81), (65, 81)]]
    assert acts == ["eager", "record", "hit", "eager", "record", "eager", "record", "eager", "eager"]
