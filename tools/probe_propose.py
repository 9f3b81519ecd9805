"""Phases of the fused proposal kernel from a -DFRCNN_PROP_PROF build (realtime
clock per image and mode): keys loaded, first select, compaction, chunk sort,
exit -- at a BASELINE config, hybrid path.

    make -C replication_faster_rcnn_amd/csrc BUILD=build_pr EXTRA=-DFRCNN_PROP_PROF \
        OUT=../../tools/prev/libfrcnn_PR.so
    FRCNN_LIB_PATH=$PWD/tools/prev/libfrcnn_PR.so python tools/probe_propose.py --config cfg2
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    a = ap.parse_args()
    lib = _lib.load()
    fn = lib.frcnn_debug_prop_prof
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    c = synth.CONFIGS[a.config]
    c, sc, de, x = make_inputs(a.config, range(c["batch"]), dev)
    N = sc.size(0)
    base = A.generate_anchor_base_device(anchor_scales=c["scales"])
    buf = np.zeros((3, 256, 8), np.uint64)
    out = []
    for rep in range(4):
        torch.cuda.synchronize()
        fn(buf.ctypes.data, 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.propose(sc, de, img_w=c["img_w"], img_h=c["img_h"], pre_nms=c["pre_nms"], post_nms=c["post_nms"],
                    anchor_base=base, feat_h=c["feat_h"], feat_w=c["feat_w"])
        e1.record()
        torch.cuda.synchronize()
        fn(buf.ctypes.data, 0)
        if rep == 0:
            continue
        t = buf[:, :N, :].astype(np.int64)
        res = {"events_us": round(e0.elapsed_time(e1) * 1e3, 1)}
        for m in (1, 2):
            tm = t[m]
            if not tm[:, 0].any():
                continue
            d = lambda i, j: [round(float(v) / 100, 2) for v in np.percentile(  # noqa: E731
                np.where(tm[:, j] > 0, tm[:, j] - tm[:, i], 0), [0, 50, 100])]
            res[f"mode{m}"] = {"load": d(0, 1), "select1": d(1, 2), "compact": d(2, 3), "sort": d(3, 4),
                               "to_exit": d(4, 5) if m == 1 else d(1, 5)}
        out.append(res)
    print(json.dumps({"config": a.config, "runs": out}, indent=1))


if __name__ == "__main__":
    main()
