"""Soft-J metric of the reference (evaluation.py:3-22) on uint8 masks.

J = sum(pred & 255*gt) / sum(pred | 255*gt) over int16 bit patterns; with an all-zero gt
J = 1 - fraction of non-zero predicted pixels.  Host-side integer work on one [H, W] mask.
"""
import numpy as np


def compute_iou(prediction01, gt01):
    if np.all(gt01 == 0):
        return 1.0 - np.count_nonzero(prediction01) / (prediction01.shape[0] * prediction01.shape[1])
    pred = prediction01.astype(np.int16)
    gt = (gt01 * 255).astype(np.int16)
    return np.sum(pred & gt) * 1.0 / np.sum(pred | gt)
