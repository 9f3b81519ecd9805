"""Per-wave spans of the leader RoIPool backward from a -DFRCNN_BWD_PROF
build, on the training-step inputs of tools/ab_roi_pool_bwd.py (ProposalTarget's
128 sampled RoIs per image): wave start / end on the 100 MHz constant clock,
RoIs walked and flagged RoIs per wave, and what the slowest waves hold.

    make -C replication_faster_rcnn_amd/csrc BUILD=build_bp EXTRA=-DFRCNN_BWD_PROF \\
        OUT=../../tools/prev/libfrcnn_BP.so
    FRCNN_LIB_PATH=$PWD/tools/prev/libfrcnn_BP.so python tools/probe_bwd_spans.py --variants auto
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ab_roi_pool_bwd import build, set_variant  # noqa: E402
from replication_faster_rcnn_amd import _lib, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="auto")
    a = ap.parse_args()
    lib = _lib.load()
    fn = lib.frcnn_debug_bwd_prof
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]

    g, boxes, am, xs = build()
    N, C, H, W = xs
    out = {}
    for v in a.variants.split(","):
        set_variant(v)
        K = 1
        buf = np.zeros((8192, 8), np.uint64)
        runs = []
        for rep in range(3):
            torch.cuda.synchronize()
            fn(buf.ctypes.data, 1)

            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops._roi_pool_bwd(g, boxes, am, xs, 1.0)
            e1.record()
            torch.cuda.synchronize()
            fn(buf.ctypes.data, 0)

            gw = np.nonzero(buf[:, 5] > 0)[0]
            w = buf[gw].astype(np.float64)
            t0 = w[:, 4].min()
            st, en = (w[:, 4] - t0) / 100.0, (w[:, 5] - t0) / 100.0  # us
            # gw = (y * gridDim.x + x) * CPW + w, CPW = 16 at cfg5; wave w of workgroup row y
            # owns image (y + w) mod N (images mixed within a workgroup)
            img = (gw // (C * K) + gw % 16) % N
            span = en - st
            slow = np.argsort(span)[-32:]
            nfl = np.maximum(w[:, 6], 1)
            flagged = {"gather_cycles_per_flagged": round(float((w[:, 7] / nfl).mean()), 0)}
            runs.append({"op_us": round(e0.elapsed_time(e1) * 1e3, 1), "waves": int(len(gw)), "flagged_detail": flagged,
                         "span_us_p10_p50_p90_max": [round(float(x), 1) for x in np.percentile(span, [10, 50, 90, 100])],
                         "last_end_us": round(float(en.max()), 1),
                         "rois_per_wave_mean_max": [round(float(w[:, 3].mean()), 1), int(w[:, 3].max())],
                         "flagged_per_wave_mean_max": [round(float(w[:, 6].mean()), 1), int(w[:, 6].max())],
                         "slowest32_rois_flagged_mean": [round(float(w[slow, 3].mean()), 1),
                                                         round(float(w[slow, 6].mean()), 1)],
                         "per_image_last_end_us": [round(float(en[img == i].max()), 1) for i in range(N)],
                         "us_per_roi_by_flagged_share": np.polyfit(w[:, 6] / np.maximum(w[:, 3], 1),
                                                                   span / np.maximum(w[:, 3], 1), 1).round(4).tolist()})
        out[v] = runs[1:]
    set_variant("auto")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
