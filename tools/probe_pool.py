"""Timeline of the wave-per-RoI RoIPool forward from a -DFRCNN_POOL_PROF build:
per workgroup the realtime clock (100 MHz) at entry, after the RoI range, after
the tile + first geometry chunk, and at the last wave's exit.  Prints the
kernel span and the distribution of each phase over the workgroups.

    make -C replication_faster_rcnn_amd/csrc BUILD=build_pp EXTRA=-DFRCNN_POOL_PROF \
        OUT=../../tools/prev/libfrcnn_PP.so
    FRCNN_LIB_PATH=$PWD/tools/prev/libfrcnn_PP.so python tools/probe_pool.py --config cfg2
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_inputs  # noqa: E402
from replication_faster_rcnn_amd import _lib, ops, synth  # noqa: E402
from replication_faster_rcnn_amd import anchors as A  # noqa: E402

SLOTS = 8192


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--path", default="auto", help="frcnn_set_path roi_pool_fwd")
    a = ap.parse_args()
    lib = _lib.load()
    _lib.set_path("roi_pool_fwd", a.path)
    fn = lib.frcnn_debug_pool_prof
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    c = synth.CONFIGS[a.config]
    c, sc, de, x = make_inputs(a.config, range(c["batch"]), dev)
    N = sc.size(0)
    base = A.generate_anchor_base_device(anchor_scales=c["scales"])
    rois, idx, cnt = ops.propose(sc, de, img_w=c["img_w"], img_h=c["img_h"], pre_nms=c["pre_nms"],
                                 post_nms=c["post_nms"], anchor_base=base, feat_h=c["feat_h"],
                                 feat_w=c["feat_w"])
    inds = torch.arange(N, device=dev, dtype=torch.float32).repeat_interleave(c["post_nms"])
    r4 = rois.view(-1, 4).contiguous()
    times = np.zeros((SLOTS, 4), np.uint64)
    nro = np.zeros(SLOTS, np.uint32)
    res = []
    for rep in range(a.reps + 1):
        torch.cuda.synchronize()
        fn(times.ctypes.data, nro.ctypes.data, 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.roi_pool_head(x, r4, inds, 7, c["img_h"], c["img_w"], 1.0, rois_sorted=True)
        e1.record()
        torch.cuda.synchronize()
        fn(times.ctypes.data, nro.ctypes.data, 0)
        if rep == 0:
            continue  # warm-up
        used = np.nonzero(times[:, 0])[0]
        t = times[used].astype(np.int64)
        live = t[:, 2] > 0  # workgroups that pooled RoIs
        t0 = t[:, 0].min()
        us = lambda v: v / 100.0  # noqa: E731  (100 MHz ticks -> us)
        tl = t[live]
        ph = {
            "start": us(tl[:, 0] - t0), "range": us(tl[:, 1] - tl[:, 0]),
            "stage": us(tl[:, 2] - tl[:, 1]), "compute": us(tl[:, 3] - tl[:, 2]),
            "end": us(tl[:, 3] - t0),
        }
        # per workgroup: pooling time by XCD (dispatch order round-robins the
        # workgroup id over the 8 XCDs) and by image (slowest grid dimension)
        comp = (t[:, 3] - t[:, 2]) / 100.0
        G = x.size(1) // (16 if x.size(2) * x.size(3) <= 2400 else 8)
        split = max(1, len(used) // max(1, (N + 1) * G))
        by_xcd = [round(float(np.mean(comp[live & (used % 8 == k)])), 2) for k in range(8)]
        by_img = [round(float(np.mean(comp[live & (used // (G * split) == b)])), 2) for b in range(N)]
        res.append({
            "compute_by_xcd": by_xcd, "compute_by_image": by_img,
            "events_us": e0.elapsed_time(e1) * 1e3, "span_us": us(t[:, 3].max() - t0),
            "wgs": int(len(used)), "live_wgs": int(live.sum()),
            "rois_per_wg": [int(nro[used][live].min()), float(nro[used][live].mean()), int(nro[used][live].max())],
            "phases": {k: [round(float(np.percentile(v, q)), 2) for q in (0, 10, 50, 90, 100)]
                       for k, v in ph.items()},
        })
    print(json.dumps({"config": a.config, "runs": res}, indent=1))


if __name__ == "__main__":
    main()
