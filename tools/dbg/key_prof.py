"""Fallback counters of the ordered-key RoIPool forward on the bench's cfg
inputs (a -DFRCNN_KEY_PROF build, FRCNN_LIB_PATH=tools/prev/libfrcnn_keyprof.so)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench import make_inputs  # noqa: E402
from replication_faster_rcnn_amd import _lib, ops, synth  # noqa: E402
from replication_faster_rcnn_amd import anchors as A  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
dev = torch.device("cuda", 0)
c = synth.CONFIGS[cfg]
c, sc, de, x = make_inputs(cfg, range(c["batch"]), dev)
N = sc.size(0)
base = A.generate_anchor_base_device(anchor_scales=c["scales"])
rois, idx, cnt = ops.propose(sc, de, img_w=c["img_w"], img_h=c["img_h"], pre_nms=c["pre_nms"],
                             post_nms=c["post_nms"], anchor_base=base, feat_h=c["feat_h"], feat_w=c["feat_w"])
inds = torch.arange(N, device=dev, dtype=torch.float32).repeat_interleave(c["post_nms"])
lib = _lib.load()
_lib.set_path("roi_pool_fwd", "key")
buf = (ctypes.c_ulonglong * 4)()
lib.frcnn_debug_key_prof(buf, 1)
ops.roi_pool_head(x, rois.view(-1, 4), inds, 7, c["img_h"], c["img_w"], rois_sorted=True)
torch.cuda.synchronize()
lib.frcnn_debug_key_prof(buf, 1)
fast, fb_waves, fb_lanes, exact = list(buf)
print(f"{cfg}: fast RoI-waves {fast}, re-scanning waves {fb_waves} ({fb_waves / max(fast, 1):.4f}), "
      f"re-scanned lanes {fb_lanes}, exact RoI-waves {exact}")
