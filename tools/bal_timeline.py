"""Timeline probe of the cost-balanced RoIPool forward (variant "baldbg"):
per workgroup start / partition done / first tile staged / end, from
s_memrealtime (100 MHz).  Prints phase statistics (us)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_inputs  # noqa: E402
from replication_faster_rcnn_amd import _lib, anchors as A, ops, synth  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
    dev = torch.device("cuda", 0)
    c = synth.CONFIGS[cfg]
    c, sc, de, x = make_inputs(cfg, c["batch"], 0, dev)
    N = sc.size(0)
    base = A.generate_anchor_base_device(anchor_scales=c["scales"])
    rois, idx, cnt = ops.propose(sc, de, img_w=c["img_w"], img_h=c["img_h"], pre_nms=c["pre_nms"],
                                 post_nms=c["post_nms"], anchor_base=base, feat_h=c["feat_h"],
                                 feat_w=c["feat_w"])
    inds = torch.arange(N, device=dev, dtype=torch.float32).repeat_interleave(c["post_nms"])
    boxes = ops.roi_transform(rois.view(-1, 4), inds, c["img_h"], c["img_w"], c["feat_h"], c["feat_w"])
    os.environ["FRCNN_ROIPOOL_VARIANT"] = "baldbg"
    for _ in range(3):
        ops._roi_pool_fwd(x, boxes, 7, 7, 1.0, True)
    torch.cuda.synchronize()
    lib = _lib.load()
    buf = (ctypes.c_ulonglong * (8 * 8192))()
    lib.frcnn_dbg_bal_stamps.restype = ctypes.c_int
    assert lib.frcnn_dbg_bal_stamps(buf, 8 * 8192) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 8).astype(np.int64)
    a = a[a[:, 0] > 0]
    t0 = a[:, 0].min()
    st, p1, stg, end = [(a[:, k] - t0) / 100.0 for k in range(4)]  # us
    nr = (a[:, 6] >> 32)
    hw = a[:, 5]
    cu = (hw >> 8) & 0xF  # CU_ID
    se = (hw >> 13) & 0x7
    res = {"wgs": int(len(a)), "start_us": [float(st.min()), float(np.median(st)), float(st.max())],
           "partition_us": [float(np.median(p1 - st)), float((p1 - st).max())],
           "stage_us": [float(np.median(stg - p1)), float((stg - p1).max())],
           "compute_us": [float(np.median(end - stg)), float((end - stg).min()), float((end - stg).max())],
           "end_us": [float(end.min()), float(np.median(end)), float(end.max())],
           "rois_per_wg": [int(nr.min()), int(np.median(nr)), int(nr.max())],
           "runs": np.bincount((a[:, 6] & 0xFFFFFFFF).astype(int)).tolist()}
    print(json.dumps(res, indent=1))
    order = np.argsort(end)
    print("latest-ending WGs (wg, start, part, stage, end, rois):")
    for i in order[-8:]:
        print(int(i), round(st[i], 1), round(p1[i] - st[i], 1), round(stg[i] - p1[i], 1), round(end[i], 1), int(nr[i]))


if __name__ == "__main__":
    main()
