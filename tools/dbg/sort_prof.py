"""Timeline probe of the row-sorted RoIPool forward (-DFRCNN_SORT_PROF build):
per workgroup, 100-MHz stamps at entry, tile staged, tables built, last wave
out of the ring, exit."""
import ctypes, os, sys
import numpy as np
import torch
sys.path.insert(0, os.getcwd())
from bench import make_inputs
from replication_faster_rcnn_amd import _lib, ops, synth
from replication_faster_rcnn_amd import anchors as A
cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
dev = torch.device("cuda", 0)
c = synth.CONFIGS[cfg]
c, sc, de, x = make_inputs(cfg, range(c["batch"]), dev)
N = sc.size(0)
base = A.generate_anchor_base_device(anchor_scales=c["scales"])
rois, idx, cnt = ops.propose(sc, de, img_w=c["img_w"], img_h=c["img_h"], pre_nms=c["pre_nms"], post_nms=c["post_nms"],
                             anchor_base=base, feat_h=c["feat_h"], feat_w=c["feat_w"])
inds = torch.arange(N, device=dev, dtype=torch.float32).repeat_interleave(c["post_nms"])
boxes = ops.roi_transform(rois.view(-1, 4), inds, c["img_h"], c["img_w"], c["feat_h"], c["feat_w"])
lib = _lib.load()
_lib.set_path("roi_pool_fwd", "sort")
buf = np.zeros((4096, 6), np.uint64)
for it in range(3):
    ops._roi_pool_fwd(x, boxes, 7, 7, 1.0, True)
    torch.cuda.synchronize()
    lib.frcnn_debug_sort_prof(ctypes.c_void_p(buf.ctypes.data), 1)
t = buf.astype(np.int64)
live = t[:, 0] > 0
t = t[live]
t0 = t[:, 0].min()
rel = (t - t0) / 100.0  # us
print("workgroups", live.sum())
for k, name in enumerate(["entry", "tile", "tables", "ring_end", "exit"]):
    print(f"{name:9s} median {np.median(rel[:, k]):7.2f}  max {rel[:, k].max():7.2f} us")
print("ring span median", np.median(rel[:, 3] - rel[:, 2]), "max", (rel[:, 3] - rel[:, 2]).max())
