"""Host-issue cost of the cfg2 bench step, piece by piece (enqueue time only,
no synchronisation inside the timed loops), plus a cProfile of bench steps.

    python tools/issue_profile.py
"""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from replication_faster_rcnn_amd import _lib, ops, synth  # noqa: E402
from replication_faster_rcnn_amd import anchors as A  # noqa: E402


def per_call(fn, n=400):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t = (time.perf_counter() - t0) / n * 1e6
    torch.cuda.synchronize()
    return t


def main():
    dev = torch.device("cuda", 0)
    c, sc, de, x = bench.make_inputs("cfg2", range(8), dev)
    base = A.generate_anchor_base_device(anchor_scales=c["scales"])
    N, post = 8, c["post_nms"]
    out = (torch.empty((N, post, 4), device=dev), torch.empty((N, post), dtype=torch.int32, device=dev),
           torch.empty((N,), dtype=torch.int32, device=dev))
    rois = out[0]
    inds = torch.arange(N, device=dev, dtype=torch.float32).repeat_interleave(post)
    pool_out = (torch.empty((N * post, 256, 7, 7), device=dev),
                torch.empty((N * post, 256, 7, 7), dtype=torch.int32, device=dev),
                torch.empty((N * post, 5), device=dev))
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    ev = torch.cuda.Event()
    res = {}
    res["propose(out=)"] = per_call(lambda: ops.propose(
        sc, de, img_w=c["img_w"], img_h=c["img_h"], pre_nms=c["pre_nms"], post_nms=post, anchor_base=base,
        feat_h=c["feat_h"], feat_w=c["feat_w"], out=out))
    ops.propose(sc, de, img_w=c["img_w"], img_h=c["img_h"], pre_nms=c["pre_nms"], post_nms=post,
                anchor_base=base, feat_h=c["feat_h"], feat_w=c["feat_w"], out=out)
    res["roi_pool_head(out=)"] = per_call(lambda: ops.roi_pool_head(
        x, rois.view(-1, 4), inds, 7, c["img_h"], c["img_w"], rois_sorted=True, out=pool_out), n=100)

    def ctx():
        with torch.cuda.stream(s1):
            pass
    res["with torch.cuda.stream"] = per_call(ctx)
    res["event.record"] = per_call(lambda: ev.record(s1))
    res["stream.wait_event"] = per_call(lambda: s2.wait_event(ev))
    res["current_stream()"] = per_call(lambda: torch.cuda.current_stream().cuda_stream)
    lib = _lib.load()
    res["ctypes frcnn_version"] = per_call(lambda: lib.frcnn_version())
    for k, v in res.items():
        print(f"{k:28s} {v:7.1f} us")
    # cProfile of bench steps
    sys.argv = ["bench.py", "--cpu-seconds", "0", "--steps", "300", "--warmup", "20"]
    pr = cProfile.Profile()
    pr.enable()
    bench.main()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
