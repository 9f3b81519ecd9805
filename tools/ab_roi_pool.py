"""A/B timing of the RoIPool forward paths on one device, interleaved rounds.

    python tools/ab_roi_pool.py [--config cfg2] [--variants blocks,blocks:4,dense@3,dense/u,generic]

A variant is `path[:cg][@split][/u]`: path = blocks | dense | generic
(frcnn_set_path("roi_pool_fwd", path)), cg = channels per workgroup
("roi_pool_cg"), split = RoI / unit shares per image ("roi_pool_split"), /u =
RoIs passed as unsorted (per-image lists first).

Inputs are the bench's: the config's features + the proposals of the batch.
Every variant's output is checked bit-equal to the first variant's.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_inputs  # noqa: E402
from replication_faster_rcnn_amd import _lib, ops, synth  # noqa: E402
from replication_faster_rcnn_amd import anchors as A  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--variants", default="blocks,dense")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--exclude-cus", type=int, default=0,
                    help="run on a stream masked to all CUs but this many (spread over XCDs)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    c = synth.CONFIGS[a.config]
    c, sc, de, x = make_inputs(a.config, range(c["batch"]), dev)
    N = sc.size(0)
    base = A.generate_anchor_base_device(anchor_scales=c["scales"])
    rois, idx, cnt = ops.propose(sc, de, img_w=c["img_w"], img_h=c["img_h"], pre_nms=c["pre_nms"],
                                 post_nms=c["post_nms"], anchor_base=base, feat_h=c["feat_h"],
                                 feat_w=c["feat_w"])
    inds = torch.arange(N, device=dev, dtype=torch.float32).repeat_interleave(c["post_nms"])
    boxes = ops.roi_transform(rois.view(-1, 4), inds, c["img_h"], c["img_w"], c["feat_h"], c["feat_w"])
    R = boxes.size(0)
    C, H, W = x.shape[1:]
    alg = N * C * H * W * 4 + R * 20 + 2 * R * C * 49 * 4
    if a.exclude_cus > 0:
        from bench import reserved_cus
        n = _lib.cu_count()
        res = set(reserved_cus(n, a.exclude_cus, "rr"))
        torch.cuda.synchronize()
        torch.cuda.set_stream(_lib.cu_stream([i for i in range(n) if i not in res]))
    variants = a.variants.split(",")
    ref = None
    times = {v: [] for v in variants}
    for rnd in range(a.rounds):
        for vs in variants:
            v, uns = (vs[:-2], True) if vs.endswith("/u") else (vs, False)
            v, _, sp = v.partition("@")
            v, _, cg = v.partition(":")
            _lib.set_path("roi_pool_split", sp or "auto")
            _lib.set_path("roi_pool_cg", cg or "auto")
            _lib.set_path("roi_pool_fwd", v)
            srt = not uns
            out, am = ops._roi_pool_fwd(x, boxes, 7, 7, 1.0, srt)
            if ref is None:
                ref = (out.clone(), am.clone())
            elif rnd == 0:
                assert torch.equal(out, ref[0]) and torch.equal(am, ref[1]), f"variant {vs} differs"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                ops._roi_pool_fwd(x, boxes, 7, 7, 1.0, srt)
            e1.record()
            torch.cuda.synchronize()
            times[vs].append(e0.elapsed_time(e1) / a.iters * 1e3)
    for op in ("roi_pool_split", "roi_pool_cg", "roi_pool_fwd"):
        _lib.set_path(op, "auto")
    res = {v: {"us_median": float(np.median(t)), "us_min": float(np.min(t)),
               "GBps": alg / (np.median(t) * 1e-6) / 1e9} for v, t in times.items()}
    print(json.dumps({"config": a.config, "R": R, "alg_bytes": alg, "variants": res}, indent=1))


if __name__ == "__main__":
    main()
