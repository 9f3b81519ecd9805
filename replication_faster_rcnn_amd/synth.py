"""Synthetic VOC-shaped inputs (SURVEY.md §8(d) "Synthetic inputs").

Every array is generated from ``numpy.random.default_rng(seed + image_index)``
so a batch sharded over ranks is bit-identical to the unsharded batch
(P-invariance), and the same inputs can be rebuilt on the GPU box without any
fixture file.  There is no dataset access here (no network): the shapes follow
the reference loader (``utils/data_loader.py:21,88-89,105,115``) and the
BASELINE.json configs.
"""
from __future__ import annotations

import numpy as np

# BASELINE.json configs -> shapes (SURVEY.md §8 header)
CONFIGS = {
    # name: (img_h, img_w, feat_h, feat_w, ratios, scales, pre_nms, post_nms, C, batch)
    "cfg1": dict(img_h=600, img_w=1000, feat_h=38, feat_w=63, scales=(8, 16, 32),
                 pre_nms=12000, post_nms=2000, C=256, batch=1),
    "cfg2": dict(img_h=600, img_w=1000, feat_h=38, feat_w=63, scales=(8, 16, 32),
                 pre_nms=6000, post_nms=300, C=256, batch=8),
    "cfg3": dict(img_h=600, img_w=1000, feat_h=38, feat_w=63, scales=(8, 16, 32),
                 pre_nms=6000, post_nms=300, C=256, batch=64),
    "cfg4": dict(img_h=800, img_w=1333, feat_h=50, feat_w=84, scales=(2, 4, 8, 16, 32),
                 pre_nms=30000, post_nms=2000, C=512, batch=1),
    "cfg5": dict(img_h=600, img_w=600, feat_h=38, feat_w=38, scales=(8, 16, 32),
                 pre_nms=12000, post_nms=600, C=256, batch=16),
}
RATIOS = (0.5, 1.0, 2.0)


def rng_for(seed: int, image_index: int, stream: int = 0) -> np.random.Generator:
    return np.random.default_rng([int(seed), int(image_index), int(stream)])


def rpn_scores(A: int, seed: int, image_index: int) -> np.ndarray:
    """Tie-free fg scores in (0,1): ``(perm(A) + 0.5) / A``."""
    r = rng_for(seed, image_index, 0)
    return ((r.permutation(A).astype(np.float64) + 0.5) / A).astype(np.float32)


def rpn_deltas(A: int, seed: int, image_index: int, sigma: float = 0.2) -> np.ndarray:
    r = rng_for(seed, image_index, 1)
    return (r.standard_normal((A, 4)) * sigma).astype(np.float32)


def features(C: int, H: int, W: int, seed: int, image_index: int) -> np.ndarray:
    r = rng_for(seed, image_index, 2)
    return r.standard_normal((C, H, W), dtype=np.float32)


def gt_boxes(img_h: int, img_w: int, G: int, seed: int, image_index: int, n_valid=None):
    """32-slot padded gt like ``utils/data_loader.py:88-115``: layout
    ``[ymin, xmin, ymax, xmax]`` fp64, ``np.around``-ed; padded rows are -1
    with label -1.  Returns (boxes [G,4] f64, labels [G] f64)."""
    r = rng_for(seed, image_index, 3)
    if n_valid is None:
        n_valid = G
    boxes = -1 * np.ones([G, 4])
    labels = -1 * np.ones(G)
    for g in range(n_valid):
        while True:
            y = np.sort(r.uniform(0, img_h, 2))
            x = np.sort(r.uniform(0, img_w, 2))
            b = np.around(np.array([y[0], x[0], y[1], x[1]]))
            if b[2] - b[0] >= 4 and b[3] - b[1] >= 4:
                break
        boxes[g] = b
        labels[g] = float(r.integers(1, 21))
    return np.around(boxes), labels
