"""CPU restatement (numpy) of the SBM-RGBD frame preparation -- TEST INFRASTRUCTURE ONLY.

Restates dataloaders/sbm_rgbd_loader.py:141-198 (find_boundary_from_center / find_roi, literal
loops), :590-697 (_load_images) and dataloaders/utils.py:5-55 (crop2d / scale2d / flip2d) with
OpenCV's documented cv2.resize rules (imgproc/src/resize.cpp, generic path):
  INTER_LINEAR : fx = (float)((dx + 0.5) * scale - 0.5), sx = floor(fx), fx -= sx;
                 sx < 0 -> (sx, fx) = (0, 0); sx >= n - 1 -> (sx, fx) = (n - 1, 0);
                 value = rows (1 - fy, fy) of columns (1 - fx, fx), fp32
  INTER_NEAREST: sx = min(floor(dx * scale), n - 1)
with scale = 1 / (dsize / ssize) in double.  OpenCV (cv2) is not installed here, so this
restatement is checked against hand-computed cases only: parity of the cv2 arithmetic is
UNPINNED (no reference outputs exist offline); the file-level logic is pinned to the
reference code it restates line by line.
"""
import numpy as np


def find_boundary_from_center(ary1d):
    """dataloaders/sbm_rgbd_loader.py:141-159 (literal)."""
    half = int(np.floor(len(ary1d) / 2))
    l = half
    while l >= 0:
        if ary1d[l] == 0:
            break
        l -= 1
    r = half
    while r < len(ary1d):
        if ary1d[r] == 0:
            break
        r += 1
    return [l, r]


def find_roi(img2d):
    """dataloaders/sbm_rgbd_loader.py:174-198 (literal)."""
    x_boundary = [-1, 0xFFFFFFFF]
    y_boundary = [-1, 0xFFFFFFFF]
    for r in range(0, img2d.shape[0], 2):
        b = find_boundary_from_center(img2d[r])
        if b[0] < b[1]:
            x_boundary[0] = max(x_boundary[0], b[0])
            x_boundary[1] = min(x_boundary[1], b[1])
    for c in range(0, img2d.shape[1], 2):
        b = find_boundary_from_center(img2d[:, c])
        if b[0] < b[1]:
            y_boundary[0] = max(y_boundary[0], b[0])
            y_boundary[1] = min(y_boundary[1], b[1])
    return (x_boundary, y_boundary)


def _taps_linear(dst, src):
    scale = 1.0 / (dst / src)
    idx0, idx1, wt = [], [], []
    for d in range(dst):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = int(np.floor(f))
        f = np.float32(f - np.float32(s))
        if s < 0:
            s, f = 0, np.float32(0)
        if s >= src - 1:
            s, f = src - 1, np.float32(0)
        idx0.append(s)
        idx1.append(min(s + 1, src - 1))
        wt.append(f)
    return np.array(idx0), np.array(idx1), np.array(wt, dtype=np.float32)


def resize(img2d, out_hw, mode):
    """cv2.resize(img2d (2-D), (W, H), INTER_LINEAR if mode == 0 else INTER_NEAREST)."""
    H, W = out_hw
    h, w = img2d.shape
    if mode == 1:
        ys = np.minimum(np.floor(np.arange(H) * (1.0 / (H / h))).astype(np.int64), h - 1)
        xs = np.minimum(np.floor(np.arange(W) * (1.0 / (W / w))).astype(np.int64), w - 1)
        return img2d[ys][:, xs]
    a = img2d.astype(np.float32)
    y0, y1, fy = _taps_linear(H, h)
    x0, x1, fx = _taps_linear(W, w)
    one = np.float32(1)
    r0 = a[y0][:, x0] * (one - fx)[None, :] + a[y0][:, x1] * fx[None, :]
    r1 = a[y1][:, x0] * (one - fx)[None, :] + a[y1][:, x1] * fx[None, :]
    return (r0 * (one - fy)[:, None] + r1 * fy[:, None]).astype(np.float32)


def roi_crop(img2d, roi):
    """_get_content_in_roi (:379-383)."""
    (xa, xb), (ya, yb) = roi
    return img2d[ya:yb + 1, xa:xb + 1]


def prepare(planes, roi, output_hw, mode, mean=None, train=None):
    """One frame's planes (list of 2-D arrays) through _load_images: mean subtraction, ROI,
    resize to output_hw, then in train mode crop (ratio, offset) / scale / flip.
    train = (crop_ratio, offset {'x','y'}, scale_ratio, flip) or None."""
    out = []
    for c, p in enumerate(planes):
        x = p.astype(np.float32) - np.float32(mean[c]) if mean is not None else p
        if roi is not None:
            x = roi_crop(x, roi)
        if output_hw is not None:
            x = resize(x, output_hw, mode)
        if train is not None:
            cr, off, sr, flip = train
            hh, ww = x.shape
            ch, cw = int(cr * hh), int(cr * ww)
            x = x[off["y"]:off["y"] + ch, off["x"]:off["x"] + cw]
            x = resize(x, (int(ch * sr), int(cw * sr)), mode)
            if flip:
                x = np.fliplr(x)
        out.append(np.asarray(x, dtype=np.float32))
    return np.stack(out)
