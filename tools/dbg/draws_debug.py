"""Which draw of a chained cfg5 run first differs between sampler paths, and
whether it was a domain miss (chip_only leaves the RNG state untouched then)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from replication_faster_rcnn_amd import _lib, targets  # noqa: E402
from replication_faster_rcnn_amd import utils as U  # noqa: E402
from tests.test_gpu_sampler_paths import _cfg5_inputs  # noqa: E402


def run(path, inputs, seed, n):
    anchors, boxes, labels, rois, cnt = inputs
    _lib.set_path("sampler", path)
    np.random.seed(seed)
    rng, _ = U.rng_state_to_device(torch.device("cuda"))
    log = []
    for _ in range(n):
        s0 = rng.clone()
        plan = targets.anchor_targets_prepare(boxes, labels, anchors)
        targets.anchor_targets_draw(plan, rng=rng)
        r, l = targets.anchor_targets_finish(plan)
        log.append(("AT", s0, rng.clone(), l.clone(), targets.anchor_targets_draw_status(plan)))
        s0 = rng.clone()
        pplan = targets.proposal_targets_prepare(rois, cnt, boxes, labels)
        out = targets.proposal_targets_sample(pplan, rng=rng)
        log.append(("PT", s0, rng.clone(), out[0].clone(), targets.proposal_targets_draw_status(pplan)))
    torch.cuda.synchronize()
    _lib.set_path("sampler", "auto")
    return log


def main():
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    inputs = _cfg5_inputs(seed)
    a = run("walk", inputs, 100 + seed, 4)
    b = run("chip_only", inputs, 100 + seed, 4)
    for k, (x, y) in enumerate(zip(a, b)):
        same_in = torch.equal(x[1], y[1])
        same_out = torch.equal(x[2], y[2])
        untouched = torch.equal(y[1], y[2])
        same_res = torch.equal(x[3], y[3])
        pos_in = int(x[1][624].item()) & 0xffffffff
        pos_out = int(x[2][624].item()) & 0xffffffff
        print(f"{k} {x[0]} state_in_equal={same_in} state_out_equal={same_out} chip_untouched={untouched} "
              f"result_equal={same_res} pos_in={pos_in} pos_out(walk)={pos_out} "
              f"pos_out(chip)={int(y[2][624].item()) & 0xffffffff} status={y[4]}")


if __name__ == "__main__":
    main()
