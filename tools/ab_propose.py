"""A/B timing of the proposal paths (frcnn_set_path("propose", hybrid | lazy | wide))
on the bench inputs, interleaved rounds; every path's output is checked
bit-equal to the first path's.

    python tools/ab_propose.py [--config cfg2] [--paths hybrid,lazy,wide]
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
    ap.add_argument("--paths", default="hybrid,lazy,wide")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cus", type=int, default=0, help="run on a stream masked to this many CUs (spread over XCDs)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    c = synth.CONFIGS[a.config]
    c, sc, de, x = make_inputs(a.config, range(c["batch"]), dev)
    base = A.generate_anchor_base_device(anchor_scales=c["scales"])

    def run():
        return ops.propose(sc, de, img_w=c["img_w"], img_h=c["img_h"], pre_nms=c["pre_nms"],
                           post_nms=c["post_nms"], anchor_base=base, feat_h=c["feat_h"],
                           feat_w=c["feat_w"])

    if a.cus > 0:
        from bench import reserved_cus
        torch.cuda.synchronize()
        torch.cuda.set_stream(_lib.cu_stream(reserved_cus(_lib.cu_count(), a.cus, "rr")))
    paths = a.paths.split(",")
    times = {p: [] for p in paths}
    ref = None
    for rnd in range(a.rounds):
        for p in paths:
            _lib.set_path("propose", p)
            out = run()
            if ref is None:
                ref = [t.clone() for t in out]
            elif rnd == 0:
                assert all(torch.equal(u, v) for u, v in zip(out, ref)), f"path {p} differs"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            times[p].append(e0.elapsed_time(e1) / a.iters * 1e3)
    print(json.dumps({"config": a.config, "counts": ref[2].tolist(),
                      "paths": {p: {"us_median": float(np.median(t)), "us_min": float(np.min(t))}
                                for p, t in times.items()}}, indent=1))


if __name__ == "__main__":
    main()
