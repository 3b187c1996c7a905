"""Checkpoint format of the reference.

* train.py:624-626 saves {"epoch": e + 1, "model": model.state_dict()} after every epoch to
  snapshots/<dataset>/<full_model_name>/H<h>W<w>/<ymd_hms>/snapshot_<dataset>_<epoch>.pth.
  Under DataParallel (more than one GPU) every key carries the "module." prefix.
* test.py:140-161 (convert_state_dict) strips "module."; train.py:501-508 resumes model and
  epoch (optimizer momentum and RNG state are not saved).
* RGBDSegmentation_RAA.load_state (rgbd_segmentation_RAA.py:103-136) additionally remaps the
  original COSNet keys (cosnet_amd/rgbd_segmentation_RAA.py:load_state).

Loading never unpickles code: torch.load(..., weights_only=True).
"""
import os
from collections import OrderedDict

import torch


def convert_state_dict(state_dict):
    """Strip the DataParallel "module." prefix (test.py:140-161)."""
    out = OrderedDict()
    for k, v in state_dict.items():
        out[k[len("module."):] if k.startswith("module.") else k] = v
    return out


def model_state(model, dataparallel_keys=False):
    """state_dict on the CPU; `dataparallel_keys` adds "module." like a DataParallel wrapper."""
    sd = model.state_dict()
    pre = "module." if dataparallel_keys else ""
    return OrderedDict((pre + k, v.detach().cpu()) for k, v in sd.items())


def save_snapshot(path, epoch, model, dataparallel_keys=False):
    """{"epoch": epoch, "model": state_dict} (train.py:625); returns the path."""
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    torch.save({"epoch": int(epoch), "model": model_state(model, dataparallel_keys)}, path)
    return path


def load_checkpoint(path):
    """Safe load of a reference / own checkpoint: returns the dict ({"epoch", "model"} or a
    bare state_dict wrapped as {"model": sd})."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    if not isinstance(ck, dict):
        raise ValueError("%s: not a state dict checkpoint" % path)
    if "model" not in ck:
        ck = {"model": ck}
    return ck


def snapshot_path(root, dataset, full_model_name, hw, stamp, epoch):
    """train.py:157 + :626 naming."""
    h, w = hw
    return os.path.join(root, "snapshots", dataset, full_model_name, "H%dW%d" % (h, w), stamp,
                        "snapshot_%s_%d.pth" % (dataset, epoch))
