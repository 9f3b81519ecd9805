"""Where the MT19937 sampler kernels spend their time, from s_memtime counters
of a -DFRCNN_SAMPLER_PROF build (FRCNN_LIB_PATH=tools/prev/libfrcnn_SP.so):
windows, twists, fixed-point rounds and the cycles of each phase, per launch,
at the cfg5 training shape (16 images, 38x38x9 anchors, 32 gt, 600 RoIs).

    FRCNN_LIB_PATH=$PWD/tools/prev/libfrcnn_SP.so python tools/probe_sampler.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ref_numpy as orc  # noqa: E402  (inputs only)
from replication_faster_rcnn_amd import _lib, synth, targets  # noqa: E402
from replication_faster_rcnn_amd import utils as U  # noqa: E402

NAMES = ["windows", "twists", "twist_cyc", "rounds", "round_cyc", "final_cyc", "kernel_cyc", "steps", "pt_calls", "seq_chunks", "seq_cyc"]


def read(lib, reset=True):
    buf = (ctypes.c_ulonglong * 16)()
    lib.frcnn_debug_sampler_prof(buf, 1 if reset else 0)
    return list(buf)[:len(NAMES)]


def main():
    lib = _lib.load()
    dev = torch.device("cuda")
    N, G, img = 16, 32, 600
    anchors = orc.generate_anchors(orc.generate_anchor_base(), 16, 38, 38)
    at = torch.from_numpy(anchors).to(dev)
    bl = [synth.gt_boxes(img, img, G, 0, i) for i in range(N)]
    boxes = torch.from_numpy(np.stack([b for b, _ in bl])).to(dev)
    labels = torch.from_numpy(np.stack([l for _, l in bl])).to(dev)
    rois = []
    for i in range(N):
        r, _ = orc.propose_one(anchors, synth.rpn_scores(len(anchors), 0, i), synth.rpn_deltas(len(anchors), 0, i),
                               img, img, 12000, 600)
        rois.append(r)
    rp = np.zeros((N, 600, 4), np.float32)
    for i, r in enumerate(rois):
        rp[i, :len(r)] = r
    rp = torch.from_numpy(rp).to(dev)
    cnt = torch.tensor([len(r) for r in rois], dtype=torch.int32, device=dev)
    np.random.seed(0)
    rng, _ = U.rng_state_to_device(dev)
    for what in ("anchor_targets", "proposal_targets"):
        for it in range(4):
            read(lib)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if what == "anchor_targets":
                targets.anchor_targets(boxes, labels, at, rng=rng)
            else:
                targets.proposal_targets(rp, cnt, boxes, labels, rng=rng)
            e1.record()
            torch.cuda.synchronize()
            v = read(lib)
            if it:
                d = dict(zip(NAMES, v))
                k = max(d["kernel_cyc"], 1)
                print(what, f"{e0.elapsed_time(e1) * 1e3:.0f} us (whole op)", d,
                      f"twist {d['twist_cyc'] / k:.2f} rounds {d['round_cyc'] / k:.2f} final {d['final_cyc'] / k:.2f}",
                      f"cyc/window {d['kernel_cyc'] / max(d['windows'], 1):.0f}",
                      f"rounds/window {d['rounds'] / max(d['windows'], 1):.2f}")


if __name__ == "__main__":
    main()
