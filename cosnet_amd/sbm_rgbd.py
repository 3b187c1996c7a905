"""SBM-RGBD frame-pair source: the reference's `sbm_rgbd` Dataset
(dataloaders/sbm_rgbd_loader.py:201-722) with the per-frame arithmetic on the GPU.

Host side (file system, integers): the directory scan of `_collect_file_list` (:392-467:
<root>/<category>/<sequence>/{input/inXXXXXX.png, depth/dXXXXXX.png, groundtruth/gtXXXXXX.png,
ROI.bmp}, a frame is every ground-truth id with all three files), the ROI box of `find_roi`
(:141-198, including its quirks: the box edges are the first ZERO pixels left/right of the
centre, kept inclusive), the subset split of `_split_dataset` (:469-514), counterpart sampling
(:538-579), the per-batch crop / scale ratios of `next_batch` (:700-702) and the per-sequence
flip probability of `_augmente_image` (:704-722).  Random draws use a seeded random.Random
(the reference's module-level `random` is unseeded).

Device side: the decoded uint8 frames are uploaded once and every resize / crop / scale / flip
/ BGR-mean subtraction of `_load_images` (:590-697) and dataloaders/utils.py:5-55 runs as the
HIP kernel cn_frame_resize (cv2.resize INTER_LINEAR / INTER_NEAREST coordinate rules).

Decoding uses PIL (cv2 is not available): IMREAD_COLOR order = BGR, IMREAD_GRAYSCALE of a
16-bit PNG = value >> 8.
"""
import math
import os
import random

import numpy as np
import torch

from . import _native as nv

ROI_FILE_NAME = "ROI.bmp"
BGR_MEAN = (104.00699, 116.66877, 122.67892)  # sbm_rgbd.__init__ default (:218)


class VideoFrameInfo:
    """dataloaders/sbm_rgbd_loader.py:130-139"""

    def __init__(self, seq_name, fid, rgb, depth, gt):
        self.seq_name, self.id = seq_name, fid
        self.name_of_rgb_frame, self.name_of_depth_frame, self.name_of_groundtruth_frame = rgb, depth, gt

    def __str__(self):
        return self.seq_name + "/[" + self.id + "]:" + self.name_of_rgb_frame + "," + self.name_of_groundtruth_frame


def _boundary_from_center(line):
    """find_boundary_from_center (:141-159): index of the first zero left of (and including)
    the centre, -1 if none; first zero right of it, len if none."""
    n = len(line)
    half = n // 2
    zl = np.flatnonzero(line[:half + 1] == 0)
    zr = np.flatnonzero(line[half:] == 0)
    left = int(zl[-1]) if len(zl) else -1
    right = int(zr[0]) + half if len(zr) else n
    return left, right


def find_roi(img2d):
    """find_roi (:174-198): ([x_min, x_max], [y_min, y_max]) from every 2nd row / column."""
    xb = [-1, 0xFFFFFFFF]
    yb = [-1, 0xFFFFFFFF]
    for r in range(0, img2d.shape[0], 2):
        lo, hi = _boundary_from_center(img2d[r])
        if lo < hi:
            xb[0] = max(xb[0], lo)
            xb[1] = min(xb[1], hi)
    for c in range(0, img2d.shape[1], 2):
        lo, hi = _boundary_from_center(img2d[:, c])
        if lo < hi:
            yb[0] = max(yb[0], lo)
            yb[1] = min(yb[1], hi)
    return xb, yb


def roi_window(roi, h, w):
    """The (y0, y1, x0, x1) rows / cols img2d[y0:y1+1, x0:x1+1] selects (:379-383), with
    Python slice semantics (a -1 start counts from the end, like the reference)."""
    (xa, xb), (ya, yb) = roi
    ys = slice(ya, yb + 1).indices(h)
    xs = slice(xa, xb + 1).indices(w)
    return ys[0], max(ys[1], ys[0]), xs[0], max(xs[1], xs[0])


def read_png(path, mode):
    """cv2.imread(path, IMREAD_COLOR -> BGR uint8 HWC | IMREAD_GRAYSCALE -> uint8 HW)."""
    from PIL import Image
    with Image.open(path) as im:
        if mode == "color":
            return np.ascontiguousarray(np.asarray(im.convert("RGB"))[:, :, ::-1])
        a = np.asarray(im)
        if a.dtype == np.uint16 or im.mode.startswith("I;16"):
            return (a.astype(np.uint32) >> 8).astype(np.uint8)
        if a.ndim == 3:
            a = np.asarray(im.convert("L"))
        return np.ascontiguousarray(a.astype(np.uint8))


def frame_resize(src, window, out_hw, mode, flip=False, mean=None, channels_last=False):
    """GPU resize of a window of `src` (uint8 HWC / HW or fp32 CHW, on the GPU) to fp32 CHW."""
    if not src.is_cuda:
        raise RuntimeError("frame_resize: source must be on the GPU (no CPU fallback)")
    y0, y1, x0, x1 = window
    H, W = out_hw
    if channels_last:  # uint8 HWC: plane stride 1, row stride W*C, column stride C
        hh, ww, c = src.shape
        sp, sr, sc = src.stride(2), src.stride(0), src.stride(1)
    elif src.dim() == 2:
        hh, ww = src.shape
        c, sp, sr, sc = 1, 0, src.stride(0), src.stride(1)
    else:
        c, hh, ww = src.shape
        sp, sr, sc = src.stride(0), src.stride(1), src.stride(2)
    out = torch.empty((c, H, W), dtype=torch.float32, device=src.device)
    meant = None
    if mean is not None:
        meant = torch.tensor(mean, dtype=torch.float32).to(src.device, non_blocking=True)
    nv.call("cn_frame_resize", int(src.dtype == torch.uint8), src.data_ptr(), c, sp, sr, sc, y0, x0,
            y1 - y0, x1 - x0, nv.ptr(meant), out.data_ptr(), H, W, mode, int(bool(flip)), nv.stream())
    return out


def augmented_hw(hh, ww, crop_ratio, scale_ratio):
    """Crop then scale sizes of one training frame (utils.crop2d :32-46, int(ratio * size);
    utils.scale2d :18-23): ((ch, cw), (sh, sw))."""
    ch, cw = int(crop_ratio * hh), int(crop_ratio * ww)
    return (ch, cw), (int(ch * scale_ratio), int(cw * scale_ratio))


class SBMRGBD:
    """sbm_rgbd (dataloaders/sbm_rgbd_loader.py:201-722) returning GPU tensors.

    __getitem__ -> dict with the reference's keys: target [3,H,W], target_depth [1,H,W],
    target_gt [H,W] (uint8 {0,1}), search_<i>, search_<i>_depth, search_<i>_gt, seq_name,
    frame_index.  `collate(samples)` stacks a batch like torch's default collate.
    """

    def __init__(self, dataset_root, sample_range, output_HW=None, for_training=True, batch_size=1,
                 subset_percentage=0.8, subset=None, meanval=BGR_MEAN, seed=1234, device="cuda",
                 log=None):
        self.dataset_root = dataset_root
        self.sample_range = int(sample_range)
        self.output_HW = tuple(output_HW) if output_HW is not None else None
        self.subset_percentage = subset_percentage
        self.meanval = tuple(float(m) for m in meanval)
        self.device = torch.device(device)
        self.rng = random.Random(seed)
        self.log = log
        self.flip_prob = {}
        self._scale_ratio, self._crop_ratio = 0.9, 0.9   # :236-237
        self.ROI = {}
        self.sets = {k: {"names_of_sequences": [], "frame_range_of_sequences": {}, "names_of_frames": []}
                     for k in ("entire", "train", "validate", "test")}
        self.batch_size = 1
        self.stage = "initing"
        self._collect_file_list()
        self.batch_size = batch_size
        self.stage = "train" if for_training else "test"
        self._split_dataset(subset)

    # ---- file list (:392-467) -------------------------------------------------------------------
    def _collect_file_list(self):
        seqs = []
        for cat in sorted(os.listdir(self.dataset_root)):
            p = os.path.join(self.dataset_root, cat)
            if os.path.isdir(p):
                seqs += [os.path.join(cat, s) for s in sorted(os.listdir(p))]
        ent = self.sets["entire"]
        for seq in seqs:
            root = os.path.join(self.dataset_root, seq)
            dirs = [os.path.join(root, d) for d in ("input", "depth", "groundtruth")]
            if not all(os.path.isdir(d) for d in dirs):
                continue
            rgb, dep, gt = (set(os.listdir(d)) for d in dirs)
            roi_path = os.path.join(root, ROI_FILE_NAME)
            if os.path.exists(roi_path):
                self.ROI[seq] = find_roi(read_png(roi_path, "gray"))
            frames = []
            for g in sorted(gt):
                if not g.endswith(".png"):
                    continue
                fid = g[2:-4]
                if ("in" + fid + ".png") in rgb and ("d" + fid + ".png") in dep:
                    frames.append(VideoFrameInfo(seq, fid, "in" + fid + ".png", "d" + fid + ".png", g))
            if frames:
                s = len(ent["names_of_frames"])
                ent["frame_range_of_sequences"][seq] = {"start": s, "end": s + len(frames)}
                ent["names_of_frames"].extend(frames)
                ent["names_of_sequences"].append(seq)

    def _split_dataset(self, subset):
        """:469-514"""
        st = self.sets[self.stage]
        if subset and isinstance(subset, dict):
            for seq, ids in subset.items():
                start = len(st["names_of_frames"])
                frames = [f for i in ids for f in [self._frame_by_id(seq, i)] if f is not None]
                st["names_of_sequences"].append(seq)
                st["frame_range_of_sequences"][seq] = {"start": start, "end": start + len(frames)}
                st["names_of_frames"].extend(frames)
            return
        for seq in self.sets["entire"]["names_of_sequences"]:
            frames = self._frames_of_seq("entire", seq)
            if len(frames) < 2 and self.stage == "train":
                continue
            n = int(math.floor(len(frames) * self.subset_percentage))
            if n < 2 and self.stage == "train":
                n = 2
            sel = frames if n == len(frames) else self.rng.sample(frames, n)
            start = len(st["names_of_frames"])
            st["names_of_sequences"].append(seq)
            st["frame_range_of_sequences"][seq] = {"start": start, "end": start + n}
            st["names_of_frames"].extend(sel)

    def _frames_of_seq(self, set_name, seq):
        r = self.sets[set_name]["frame_range_of_sequences"][seq]
        return self.sets[set_name]["names_of_frames"][r["start"]:r["end"]]

    def _frame_by_id(self, seq, fid):
        for f in self.sets["entire"]["names_of_frames"]:
            if f.id == fid and f.seq_name == seq:
                return f
        return None

    def __len__(self):
        n = len(self.sets[self.stage]["names_of_frames"])
        return n - n % self.batch_size

    # ---- augmentation state (:700-722) ------------------------------------------------------------
    def next_batch(self):
        self._scale_ratio = self.rng.uniform(0.7, 1.3)
        self._crop_ratio = self.rng.uniform(0.8, 1)

    def _flip_p(self, seq):
        if seq not in self.flip_prob:
            self.flip_prob[seq] = self.rng.uniform(0, 1)
        return self.flip_prob[seq]

    # ---- one frame (:590-697) ------------------------------------------------------------------------
    def _path(self, fi, folder, name):
        return os.path.join(self.dataset_root, fi.seq_name, folder, name)

    def _prep(self, img, roi, mode, mean, channels_last, offset, seq):
        """ROI -> resize to output_HW -> (train) crop / scale / flip, as one or three kernels."""
        h, w = img.shape[:2] if channels_last or img.dim() == 2 else img.shape[1:]
        win = roi_window(roi, h, w) if roi is not None else (0, h, 0, w)
        out_hw = self.output_HW or (win[1] - win[0], win[3] - win[2])
        x = frame_resize(img, win, out_hw, mode, mean=mean, channels_last=channels_last)
        if self.stage != "train":
            return x, offset
        # utils.crop2d (:32-46): int(ratio * size), offset drawn once per frame (shared by rgb,
        # depth, gt of that frame)
        hh, ww = x.shape[1], x.shape[2]
        (ch, cw), (sh, sw) = augmented_hw(hh, ww, self._crop_ratio, self._scale_ratio)
        if offset is None:  # rows first, then columns (utils.py:36-37)
            oy = self.rng.choice(range(hh - ch))
            offset = {"x": self.rng.choice(range(ww - cw)), "y": oy}
        # utils.scale2d (:18-23) then flip2d (:5-9)
        y = frame_resize(x, (offset["y"], offset["y"] + ch, offset["x"], offset["x"] + cw), (sh, sw),
                         mode, flip=self._flip_p(seq) > 0.5)
        return y, offset

    def load_frame(self, fi):
        roi = self.ROI.get(fi.seq_name)
        dev = self.device
        bgr = torch.from_numpy(read_png(self._path(fi, "input", fi.name_of_rgb_frame), "color")).to(dev)
        dep = torch.from_numpy(read_png(self._path(fi, "depth", fi.name_of_depth_frame), "gray")).to(dev)
        gtn = read_png(self._path(fi, "groundtruth", fi.name_of_groundtruth_frame), "gray")
        gt = torch.from_numpy((gtn != 0).astype(np.uint8)).to(dev)
        # the reference draws the crop offset while cropping the rgb image first, then reuses it
        # for depth and ground truth (:615-616, :630-631, :647-648)
        rgb, off = self._prep(bgr, roi, 0, self.meanval, True, None, fi.seq_name)
        d, off = self._prep(dep, roi, 0, None, False, off, fi.seq_name)
        g, _ = self._prep(gt, roi, 1, None, False, off, fi.seq_name)
        return rgb, d, g[0].round().to(torch.uint8)

    def __getitem__(self, idx):
        st = self.sets[self.stage]
        if idx >= len(st["names_of_frames"]):
            raise IndexError(idx)
        fi = st["names_of_frames"][idx]
        s = {"seq_name": fi.seq_name, "frame_index": fi.id}
        s["target"], s["target_depth"], s["target_gt"] = self.load_frame(fi)
        r = st["frame_range_of_sequences"][fi.seq_name]
        if self.sample_range >= 1:
            cps = self.rng.sample(list(range(r["start"], r["end"])), self.sample_range)
        else:
            cps = [idx]
        for i, j in enumerate(cps):
            k = "search_%d" % i
            s[k], s[k + "_depth"], s[k + "_gt"] = self.load_frame(st["names_of_frames"][j])
        return s

    @staticmethod
    def collate(samples):
        out = {}
        for k in samples[0]:
            v = [s[k] for s in samples]
            out[k] = torch.stack(v) if torch.is_tensor(v[0]) else v
        return out
