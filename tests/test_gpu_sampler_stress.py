"""Stress cases of the device MT19937 samplers (numpy legacy choice(replace=False)
chained over images, targets.hip fy_walk / fy_final) against the oracle's
per-image loops on numpy's global RNG: large permutations (AnchorTarget over
the 50x84x15 anchors of BASELINE cfg4: ~60k negatives per image, so many
1024-word windows and every mask width), ProposalTarget with 2,000 RoIs per
image, and stream positions at block edges (pos 0, 623, 624 and mid-block).
Needs an MI355X.  Bar: labels / samples and the RNG state bit-exact."""
import numpy as np
import pytest
import torch

from oracle import ref_numpy as orc
from replication_faster_rcnn_amd import synth, targets

pytestmark = pytest.mark.gpu


def _set_pos(seed, pos):
    """numpy's global state = the key after seed(seed), read position `pos` (0..624)."""
    np.random.seed(seed)
    st = np.random.get_state()
    np.random.set_state((st[0], st[1], pos, 0, 0.0))
    return np.random.get_state()


@pytest.mark.parametrize("skip", [0, 1, 623, 624])
def test_anchor_target_large(rng_guard, skip):
    N, G, H, W = 2, 12, 50, 84
    anchors = orc.generate_anchors(orc.generate_anchor_base(anchor_scales=(2, 4, 8, 16, 32)), 16, W, H)
    bl = [synth.gt_boxes(800, 1333, G, 41, i, n_valid=[12, 3][i]) for i in range(N)]
    boxes = np.stack([b for b, _ in bl])
    labels = np.stack([l for _, l in bl])
    st0 = _set_pos(11, skip)
    reg, lab = targets.anchor_targets(boxes, labels, anchors)
    st_dev = np.random.get_state()
    np.random.set_state(st0)
    for i in range(N):
        v = labels[i] != -1
        _, olab = orc.anchor_target(boxes[i, v], anchors)
        assert np.array_equal(lab[i].cpu().numpy(), olab), f"image {i}"
    st_ref = np.random.get_state()
    assert st_dev[2] == st_ref[2]
    assert np.array_equal(st_dev[1], st_ref[1])


@pytest.mark.parametrize("skip", [0, 300, 624])
def test_proposal_target_large(rng_guard, skip):
    N, G, img = 2, 32, 600
    r = np.random.default_rng(9)
    rois = []
    for i in range(N):
        lo = r.uniform(0, 500, (2000, 2))
        rois.append(np.concatenate([lo, lo + r.uniform(8, 300, (2000, 2))], 1).clip(0, img).astype(np.float32))
    bl = [synth.gt_boxes(img, img, G, 42, i, n_valid=[32, 9][i]) for i in range(N)]
    boxes = np.stack([b for b, _ in bl])
    labels = np.stack([l for _, l in bl])
    rp = torch.from_numpy(np.stack(rois))
    cnt = torch.tensor([2000, 1500], dtype=torch.int32)
    st0 = _set_pos(12, skip)
    s_roi, s_reg, s_lab, s_cnt = targets.proposal_targets(rp, cnt, boxes, labels, n_sample=512)
    st_dev = np.random.get_state()
    np.random.set_state(st0)
    for i in range(N):
        v = labels[i] != -1
        o_roi, _, o_lab = orc.proposal_target(rois[i][:int(cnt[i])], boxes[i, v], labels[i][v],
                                              n_sample=512)
        k = int(s_cnt[i])
        assert k == len(o_roi)
        assert np.array_equal(s_roi[i, :k].cpu().numpy(), o_roi)
        assert np.array_equal(s_lab[i, :k].cpu().numpy(), o_lab)
    st_ref = np.random.get_state()
    assert st_dev[2] == st_ref[2]
    assert np.array_equal(st_dev[1], st_ref[1])
