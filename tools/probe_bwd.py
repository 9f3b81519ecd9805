"""Phase timer of the leader RoIPool backward from a -DFRCNN_BWD_PROF build:
per wave, shader-clock cycles taking / refilling the ring (incl. load waits),
in the neighbour exchanges, and applying to the plane, per RoI.

    make -C replication_faster_rcnn_amd/csrc BUILD=build_bp EXTRA=-DFRCNN_BWD_PROF \
        OUT=../../tools/prev/libfrcnn_BP.so
    FRCNN_LIB_PATH=$PWD/tools/prev/libfrcnn_BP.so python tools/probe_bwd.py
"""
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
    lib = _lib.load()
    fn = lib.frcnn_debug_bwd_prof
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    c = synth.CONFIGS["cfg5"]
    c, sc, de, x = make_inputs("cfg5", range(c["batch"]), dev)
    N, S = sc.size(0), 128
    base = A.generate_anchor_base_device(anchor_scales=c["scales"])
    rois, _, _ = ops.propose(sc, de, img_w=c["img_w"], img_h=c["img_h"], pre_nms=c["pre_nms"],
                             post_nms=c["post_nms"], anchor_base=base, feat_h=c["feat_h"], feat_w=c["feat_w"])
    sr = rois[:, :S].reshape(-1, 4).contiguous()
    inds = torch.arange(N, device=dev, dtype=torch.float32).repeat_interleave(S)
    _, am, boxes = ops.roi_pool_head(x, sr, inds, 7, c["img_h"], c["img_w"], rois_sorted=True)
    g = torch.randn(am.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    buf = np.zeros((8192, 8), np.uint64)
    res = []
    for rep in range(4):
        torch.cuda.synchronize()
        fn(buf.ctypes.data, 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops._roi_pool_bwd(g, boxes, am, tuple(x.shape), 1.0)
        e1.record()
        torch.cuda.synchronize()
        fn(buf.ctypes.data, 0)
        if rep == 0:
            continue
        w = buf[buf[:, 3] > 0].astype(np.float64)
        per = w[:, :3] / w[:, 3:4]
        # wave spans on the 100 MHz constant clock (10 ns ticks), relative to the first start
        t0 = w[:, 4].min()
        st, en = (w[:, 4] - t0) / 100.0, (w[:, 5] - t0) / 100.0  # us
        gw = np.arange(len(buf))[buf[:, 3] > 0]  # (by * 16 + bx) * 16 + wid at cfg5 (CPW 16, 16 x 16 grid)
        img = gw // 256
        per_img_end = [round(float(en[img == i].max()), 1) for i in range(int(img.max()) + 1)]
        spans = {"first_start_to_last_end_us": round(float(en.max()), 1),
                 "start_us_p50_max": [round(float(np.median(st)), 1), round(float(st.max()), 1)],
                 "span_us_p10_p50_p90_max": [round(float(v), 1) for v in np.percentile(en - st, [10, 50, 90, 100])],
                 "end_us_p10_p50_p90": [round(float(v), 1) for v in np.percentile(en, [10, 50, 90])],
                 "per_image_last_end_us": per_img_end,
                 "per_image_mean_cycles_per_roi": [round(float(w[img == i, :3].sum(1).mean() / w[img == i, 3].mean()), 0)
                                                   for i in range(int(img.max()) + 1)],
                 "per_image_flagged_rois": [int(np.median(w[img == i, 6])) for i in range(int(img.max()) + 1)]}
        # ring steps (D RoIs each) holding a flagged RoI vs the others, cycles per step
        raw7 = buf[buf[:, 3] > 0][:, 7]
        fl_cyc, fl_n = (raw7 >> np.uint64(16)).astype(np.float64), (raw7 & np.uint64(0xFFFF)).astype(np.float64)
        steps = np.ceil(w[:, 3] / 4.0)  # D = 4
        tot = w[:, :3].sum(1)
        has = fl_n > 0
        spans["cycles_per_step_flagged_vs_plain"] = [
            round(float(fl_cyc[has].sum() / fl_n[has].sum()), 0),
            round(float((tot - fl_cyc).sum() / (steps - fl_n).sum()), 0)]
        res.append({"us": e0.elapsed_time(e1) * 1e3, "waves": int(len(w)), "spans": spans,
                    "cycles_per_roi_mean": [round(float(v), 1) for v in per.mean(0)],
                    "cycles_per_roi_p90": [round(float(v), 1) for v in np.percentile(per, 90, axis=0)],
                    "wave_total_kcycles_mean": round(float(w[:, :3].sum(1).mean() / 1e3), 1)})
    print(json.dumps({"phases": ["ring take+refill", "exchange", "apply"], "runs": res}, indent=1))


if __name__ == "__main__":
    main()
