"""Frame-pair sources for the train.py / test.py drop-ins.

The reference's datasets (dataloaders/sbm_rgbd_loader.py:201-722, hzfu_rgbd_loader.py) read
SBM-RGBD / HzFu files with cv2 and h5py; they are outside the hot path
and their data is not available offline.  `SyntheticRGBDPairs` yields batches with the SAME
dict keys and tensor conventions as `sbm_rgbd.__getitem__` (:538-579), collated:

    target        [B,3,H,W] float32  BGR minus img_mean (config.yaml:83), unscaled
    target_depth  [B,1,H,W] float32  in [0, 255], not mean-subtracted
    target_gt     [B,H,W]   float32  {0, 1}
    search_<i>, search_<i>_depth, search_<i>_gt   the counterpart frame(s), i < sample_range
    seq_name, frame_index  lists of str (test mode)

Frames are seeded per index (the same index always gives the same pair), and the counterpart
is the target moved by a few pixels plus noise, so the affinity is peaked like a video's.
"""
import torch

from .init_recipe import BGR_MEAN


class SyntheticRGBDPairs:
    def __init__(self, length, output_HW, batch_size, sample_range=1, seed=1234,
                 img_mean=BGR_MEAN, n_seqs=4):
        self.length = int(length)           # batches per epoch
        self.h, self.w = output_HW
        self.batch_size = int(batch_size)
        self.sample_range = int(sample_range)
        self.seed = int(seed)
        self.mean = torch.tensor(img_mean, dtype=torch.float32).view(1, 3, 1, 1)
        self.n_seqs = n_seqs

    def __len__(self):
        return self.length

    def next_batch(self):
        """sbm_rgbd.next_batch (:700-702) draws new crop/scale ratios; frames here are fixed-size."""

    def _frame(self, g, shift):
        h, w = self.h, self.w
        base = torch.rand((1, 3, h, w), generator=g) * 255.0
        depth = torch.rand((1, 1, h, w), generator=g) * 255.0
        yy = torch.arange(h, dtype=torch.float32).view(h, 1)
        xx = torch.arange(w, dtype=torch.float32).view(1, w)
        gt = torch.zeros((h, w))
        for _ in range(2):
            cy = float(torch.rand((), generator=g)) * h
            cx = float(torch.rand((), generator=g)) * w
            r = (0.12 + 0.2 * float(torch.rand((), generator=g))) * min(h, w)
            gt = torch.maximum(gt, (((yy - cy) ** 2 + (xx - cx) ** 2) <= r * r).float())
        # the object is brighter / closer than the background
        base = base * (1 - 0.5 * gt) + 200.0 * gt * 0.5
        depth = depth * (1 - 0.6 * gt) + 60.0 * gt * 0.6
        out = []
        for s in shift:
            out.append((torch.roll(base, s, -1) - self.mean, torch.roll(depth, s, -1),
                        torch.roll(gt, s, -1)))
        return out

    def __getitem__(self, idx):
        if idx >= self.length:
            raise IndexError(idx)
        b = self.batch_size
        g = torch.Generator().manual_seed(self.seed * 1000003 + idx)
        shifts = [0] + [3 * (i + 1) for i in range(self.sample_range)]
        frames = [self._frame(g, shifts) for _ in range(b)]
        d = {"target": torch.cat([f[0][0] for f in frames]),
             "target_depth": torch.cat([f[0][1] for f in frames]),
             "target_gt": torch.stack([f[0][2] for f in frames])}
        for i in range(self.sample_range):
            d["search_%d" % i] = torch.cat([f[i + 1][0] for f in frames])
            d["search_%d_depth" % i] = torch.cat([f[i + 1][1] for f in frames])
            d["search_%d_gt" % i] = torch.stack([f[i + 1][2] for f in frames])
        d["seq_name"] = ["synthetic_%02d" % ((idx * b + j) % self.n_seqs) for j in range(b)]
        d["frame_index"] = ["%06d" % (idx * b + j) for j in range(b)]
        return d

    def __iter__(self):
        for i in range(self.length):
            yield self[i]
