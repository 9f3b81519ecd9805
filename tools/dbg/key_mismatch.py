"""Debug: print the RoIPool forward mismatches of the key kernel on the
signed_zeros case of tests/test_gpu_parity.py::test_roi_pool_key_class_collisions."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import ref_numpy as orc  # noqa: E402
from replication_faster_rcnn_amd import _lib, ops  # noqa: E402
from tests.test_gpu_parity import _rand_rois  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "signed_zeros"
r = np.random.default_rng(sum(map(ord, case)))
N, C, H, W, R = 2, 16, 24, 40, 400
v = np.array([0.0, -0.0, -1.0, 1e-45], np.float32)
x = v[r.choice(4, (N, C, H, W), p=[0.4, 0.4, 0.15, 0.05])]
b = np.sort(r.integers(0, N, R))
rois = _rand_rois(r, b, H, W, span=30)
for path in ("key", "wave"):
    with _lib.kernel_path("roi_pool_fwd", path):
        out, am = ops.roi_pool_with_argmax(torch.from_numpy(x).cuda(), torch.from_numpy(rois).cuda(), 7,
                                           rois_sorted=True)
    oo, oa = orc.roi_pool_forward(x, rois, 7)
    o = out.cpu().numpy().view(np.uint32)
    bad = np.argwhere(o != oo.view(np.uint32))
    print(path, "argmax equal", np.array_equal(am.cpu().numpy(), oa), "value mismatches", len(bad))
    for k in bad[:12]:
        rr, c, ph, pw = k
        print("  roi", rr, rois[rr], "c", c, "bin", ph, pw, "got %08x" % o[tuple(k)], "want %08x" % oo.view(np.uint32)[tuple(k)],
              "am", am.cpu().numpy()[tuple(k)], oa[tuple(k)])
