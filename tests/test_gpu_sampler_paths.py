"""The two sampler paths (frcnn_set_path("sampler", ...)): the serial walk (one
workgroup walks numpy's MT19937 stream) and the chip-wide segment tables
(targets.hip draw_*_kernel).  "chip_only" launches the chip-wide draws with no
walk behind them, so a table, chain or record error shows as a wrong label /
sample / RNG state; "chip_tight" plans zero-margin domains, so the walk behind
them (gated on the plan's fail flag) does the draws.  Bars: labels, samples,
counts and the RNG state bit-exact against the oracle's per-image loops on
numpy's global RNG, and the paths bit-equal to each other.  Needs an MI355X."""
import numpy as np
import pytest
import torch

from oracle import ref_numpy as orc
from replication_faster_rcnn_amd import _lib, synth, targets
from replication_faster_rcnn_amd import utils as U

pytestmark = pytest.mark.gpu

PATHS = ["walk", "chip_only", "chip_tight"]


@pytest.fixture
def sampler_path(request):
    _lib.set_path("sampler", request.param)
    yield request.param
    _lib.set_path("sampler", "auto")


def _set_pos(seed, pos):
    np.random.seed(seed)
    st = np.random.get_state()
    np.random.set_state((st[0], st[1], pos, 0, 0.0))
    return np.random.get_state()


@pytest.mark.parametrize("sampler_path", PATHS, indirect=True)
@pytest.mark.parametrize("skip", [0, 623, 624])
def test_anchor_targets_paths_vs_oracle(rng_guard, sampler_path, skip):
    """AnchorTarget over BASELINE cfg4's 50x84x15 anchors (~60k negatives per
    image: every mask width, many segments), stream positions at block edges."""
    N, G, H, W = 2, 12, 50, 84
    anchors = orc.generate_anchors(orc.generate_anchor_base(anchor_scales=(2, 4, 8, 16, 32)), 16, W, H)
    bl = [synth.gt_boxes(800, 1333, G, 43, i, n_valid=[12, 2][i]) for i in range(N)]
    boxes = np.stack([b for b, _ in bl])
    labels = np.stack([l for _, l in bl])
    st0 = _set_pos(13, skip)
    _, lab = targets.anchor_targets(boxes, labels, anchors)
    st_dev = np.random.get_state()
    np.random.set_state(st0)
    for i in range(N):
        v = labels[i] != -1
        _, olab = orc.anchor_target(boxes[i, v], anchors)
        assert np.array_equal(lab[i].cpu().numpy(), olab), f"image {i}"
    st_ref = np.random.get_state()
    assert st_dev[2] == st_ref[2]
    assert np.array_equal(st_dev[1], st_ref[1])


@pytest.mark.parametrize("sampler_path", PATHS, indirect=True)
def test_proposal_targets_paths_vs_oracle(rng_guard, sampler_path):
    """ProposalTarget with ragged RoI counts: 2,000 / 1,500 / 3 / 1 / 0 RoIs per
    image (calls of 0, 1 and 2 elements: no words, one step)."""
    N, G, img = 5, 32, 600
    r = np.random.default_rng(19)
    rois = []
    for i in range(N):
        lo = r.uniform(0, 500, (2000, 2))
        rois.append(np.concatenate([lo, lo + r.uniform(8, 300, (2000, 2))], 1).clip(0, img).astype(np.float32))
    bl = [synth.gt_boxes(img, img, G, 44, i, n_valid=[32, 9, 3, 1, 0][i]) for i in range(N)]
    boxes = np.stack([b for b, _ in bl])
    labels = np.stack([l for _, l in bl])
    cnt = torch.tensor([2000, 1500, 3, 1, 0], dtype=torch.int32)
    st0 = _set_pos(14, 300)
    s_roi, _, s_lab, s_cnt = targets.proposal_targets(torch.from_numpy(np.stack(rois)), cnt, boxes, labels,
                                                      n_sample=512)
    st_dev = np.random.get_state()
    np.random.set_state(st0)
    for i in range(N):
        v = labels[i] != -1
        o_roi, _, o_lab = orc.proposal_target(rois[i][:int(cnt[i])], boxes[i, v], labels[i][v], n_sample=512)
        k = int(s_cnt[i])
        assert k == len(o_roi), f"image {i}"
        assert np.array_equal(s_roi[i, :k].cpu().numpy(), o_roi), f"image {i}"
        assert np.array_equal(s_lab[i, :k].cpu().numpy(), o_lab), f"image {i}"
    st_ref = np.random.get_state()
    assert st_dev[2] == st_ref[2]
    assert np.array_equal(st_dev[1], st_ref[1])


def _cfg5_inputs(seed):
    from replication_faster_rcnn_amd import anchors as A, ops
    c = synth.CONFIGS["cfg5"]
    N, G, img = c["batch"], 32, c["img_h"]
    anchors = orc.generate_anchors(orc.generate_anchor_base(), 16, c["feat_w"], c["feat_h"])
    nA = len(anchors)
    bl = [synth.gt_boxes(img, img, G, seed, i, n_valid=1 + (5 * i + seed) % 32) for i in range(N)]
    dev = torch.device("cuda", 0)
    boxes = torch.from_numpy(np.stack([b for b, _ in bl])).to(dev)
    labels = torch.from_numpy(np.stack([l for _, l in bl])).to(dev)
    sc = torch.from_numpy(np.stack([synth.rpn_scores(nA, seed, i) for i in range(N)])).to(dev)
    de = torch.from_numpy(np.stack([synth.rpn_deltas(nA, seed, i) for i in range(N)])).to(dev)
    rois, _, cnt = ops.propose(sc, de, img_w=img, img_h=img, pre_nms=c["pre_nms"], post_nms=c["post_nms"],
                               anchor_base=A.generate_anchor_base_device(), feat_h=c["feat_h"], feat_w=c["feat_w"])
    return torch.from_numpy(anchors).to(dev), boxes, labels, rois, cnt


def _steps(path, inputs, seed, n_steps):
    """n_steps training steps' draws (all AnchorTarget, then all ProposalTarget)
    on a device-resident stream under one sampler path."""
    anchors, boxes, labels, rois, cnt = inputs
    _lib.set_path("sampler", path)
    try:
        np.random.seed(seed)
        rng, _ = U.rng_state_to_device(torch.device("cuda"))
        outs = []
        for _ in range(n_steps):
            outs.append(targets.anchor_targets(boxes, labels, anchors, rng=rng))
            outs.append(targets.proposal_targets(rois, cnt, boxes, labels, rng=rng))
        torch.cuda.synchronize()
        return outs, rng.clone()
    finally:
        _lib.set_path("sampler", "auto")


@pytest.mark.parametrize("seed", [5, 6])
def test_cfg5_paths_agree_over_steps(rng_guard, seed):
    """BASELINE configs[4] (16 images, 38x38x9 anchors, 2,000 proposals each),
    three chained training steps on a device-resident stream: the chip-wide
    draws alone equal the walk step by step (labels, targets, samples, counts,
    the state after every step), and auto equals both."""
    inputs = _cfg5_inputs(seed)
    ref, st_ref = _steps("walk", inputs, 100 + seed, 3)
    for path in ("chip_only", "auto"):
        got, st = _steps(path, inputs, 100 + seed, 3)
        for k, (a, b) in enumerate(zip(ref, got)):
            for x, y in zip(a, b):
                assert torch.equal(x, y), f"{path}: call {k}"
        assert torch.equal(st, st_ref), path


def test_cfg5_chip_only_vs_oracle(rng_guard):
    """The chip-wide draws alone at cfg5 against the reference's per-image loops."""
    anchors, boxes, labels, rois, cnt = _cfg5_inputs(7)
    _lib.set_path("sampler", "chip_only")
    try:
        np.random.seed(77)
        aplan = targets.anchor_targets_prepare(boxes, labels, anchors)
        _, lab = targets.anchor_targets_sample(aplan)
        ast = targets.anchor_targets_draw_status(aplan)
        pplan = targets.proposal_targets_prepare(rois, cnt, boxes, labels)
        s_roi, _, s_lab, s_cnt = targets.proposal_targets_sample(pplan)
        pst = targets.proposal_targets_draw_status(pplan)
        st_dev = np.random.get_state()
    finally:
        _lib.set_path("sampler", "auto")
    # the segment tables held (no walk ran): 16 images' 32 calls, ~150k steps
    assert ast["fail"] == 0 and ast["segments"] > 100 and ast["walks"] >= 16, ast
    assert pst["fail"] == 0 and pst["segments"] > 0, pst
    np.random.seed(77)
    an, bx, lb = anchors.cpu().numpy(), boxes.cpu().numpy(), labels.cpu().numpy()
    for i in range(bx.shape[0]):
        v = lb[i] != -1
        _, olab = orc.anchor_target(bx[i, v], an)
        assert np.array_equal(lab[i].cpu().numpy(), olab), f"anchor labels, image {i}"
    rc = rois.cpu().numpy()
    for i in range(bx.shape[0]):
        v = lb[i] != -1
        o_roi, _, o_lab = orc.proposal_target(rc[i, :int(cnt[i])], bx[i, v], lb[i][v])
        k = int(s_cnt[i])
        assert k == len(o_roi) and np.array_equal(s_roi[i, :k].cpu().numpy(), o_roi), f"image {i}"
        assert np.array_equal(s_lab[i, :k].cpu().numpy(), o_lab), f"image {i}"
    st_ref = np.random.get_state()
    assert st_dev[2] == st_ref[2]
    assert np.array_equal(st_dev[1], st_ref[1])


@pytest.mark.parametrize("path", ["auto", "walk", "chip_only", "chip_tight"])
def test_target_draws_one_pass_equals_two(rng_guard, path):
    """frcnn_target_draws (both creators' draws as one pass, as the cfg5 bench
    runs them) == anchor_targets_draw then proposal_targets_draw under the walk:
    two chained steps at cfg5, every output and the RNG state after each."""
    anchors, boxes, labels, rois, cnt = _cfg5_inputs(8)

    def run(one_pass, p):
        _lib.set_path("sampler", p)
        try:
            np.random.seed(55)
            rng, _ = U.rng_state_to_device(torch.device("cuda"))
            outs, status = [], None
            for _ in range(2):
                ap = targets.anchor_targets_prepare(boxes, labels, anchors)
                pp = targets.proposal_targets_prepare(rois, cnt, boxes, labels)
                if one_pass:
                    c = targets.target_draws(ap, pp, rng)
                    status = targets.anchor_targets_draw_status(ap)
                else:
                    targets.anchor_targets_draw(ap, rng=rng)
                    c = targets.proposal_targets_draw(pp, rng=rng)
                outs.append(tuple(targets.anchor_targets_finish(ap)) + tuple(targets.proposal_targets_finish(pp, c))
                            + (c, rng.clone()))
            torch.cuda.synchronize()
            return outs, status
        finally:
            _lib.set_path("sampler", "auto")

    ref, _ = run(False, "walk")
    got, status = run(True, path)
    for k, (a, b) in enumerate(zip(ref, got)):
        for i, (x, y) in enumerate(zip(a, b)):
            assert torch.equal(x, y), f"{path}: step {k}, output {i}"
    if path in ("auto", "chip_only"):  # one plan over all 64 calls, and it held
        assert status["fail"] == 0 and status["walks"] > 32, status
    if path == "chip_tight":
        assert status["fail"] != 0, status
