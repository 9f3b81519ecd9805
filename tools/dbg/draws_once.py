"""The cfg5 draws alone (AnchorTarget then ProposalTarget on a device-resident
stream), --reps times: a short program for rocprofv3 / PMC passes over the
draw_* kernels."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from replication_faster_rcnn_amd import _lib, targets  # noqa: E402
from replication_faster_rcnn_amd import utils as U  # noqa: E402
from tests.test_gpu_sampler_paths import _cfg5_inputs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--path", default="auto")
a = ap.parse_args()
anchors, boxes, labels, rois, cnt = _cfg5_inputs(5)
aplan = targets.anchor_targets_prepare(boxes, labels, anchors)
pplan = targets.proposal_targets_prepare(rois, cnt, boxes, labels)
_lib.set_path("sampler", a.path)
np.random.seed(3)
rng, _ = U.rng_state_to_device(torch.device("cuda"))
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.reps):
    targets.anchor_targets_draw(aplan, rng=rng)
    targets.proposal_targets_draw(pplan, rng=rng)
e1.record()
torch.cuda.synchronize()
print({"path": a.path, "us_per_draw_pair": e0.elapsed_time(e1) * 1e3 / a.reps,
       "at": targets.anchor_targets_draw_status(aplan), "pt": targets.proposal_targets_draw_status(pplan)})
