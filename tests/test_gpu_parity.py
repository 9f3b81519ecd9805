"""HIP path vs oracle / golden fixtures.  Needs an MI355X.

Bars (BASELINE.json north_star): kept-proposal indices, RoIPool outputs and
argmax bit-exact; decoded boxes within 1e-5 relative (fp32 exp is
host-dependent in the reference); RoIPool gradients bit-exact here (the
kernel reproduces the CPU summation order), 1e-5 relative is the contract.
"""
import hashlib

import numpy as np
import pytest
import torch

from oracle import ref_numpy as orc
from replication_faster_rcnn_amd import anchors as A
from replication_faster_rcnn_amd import _lib, ops, synth

pytestmark = pytest.mark.gpu
DEV = "cuda"
RTOL = 1e-5


@pytest.fixture(params=["hybrid", "lazy", "wide"])
def path(request):
    """The proposal paths: fused per-image with the chip-wide first-chunk mask
    (default), fused lazy per-block, chip-wide bitmask NMS."""
    with _lib.kernel_path("propose", request.param):
        yield request.param


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_anchor_base_and_grid(golden):
    g = golden("anchors.npz")
    for tag, scales in [("k9", (8, 16, 32)), ("k15", (2, 4, 8, 16, 32))]:
        base = A.generate_anchor_base(anchor_scales=list(scales))
        assert np.array_equal(base, g[f"base_{tag}"]), tag
        for (w, h) in [(10, 10), (63, 38), (38, 38), (84, 50), (7, 3)]:
            a = A.generate_anchors(base, 16, w, h)
            assert a.dtype == np.float32
            assert sha(a) == str(g[f"sha_{tag}_{w}x{h}"]), (tag, w, h)
    a10 = A.generate_anchors(A.generate_anchor_base(), 10, 10, 10)
    assert np.array_equal(a10, g["anchors_main_10"])


def test_reg2bbox(golden):
    from replication_faster_rcnn_amd import utils as U
    g = golden("reg2bbox.npz")
    out = U.reg2bbox(torch.from_numpy(g["anchors"]), torch.from_numpy(g["reg"])).numpy()
    ora = orc.reg2bbox(g["anchors"], g["reg"])
    fin = np.isfinite(ora)
    assert np.array_equal(np.isfinite(out), fin)
    assert np.array_equal(out[fin], ora[fin])           # both correctly rounded
    np.testing.assert_allclose(out[fin], g["out"][fin], rtol=RTOL, atol=1e-3)  # vs MKL exp


def _propose_one_gpu(anchors, scores, deltas, img_w, img_h, pre, post):
    rois, idx, cnt = ops.propose(torch.from_numpy(scores)[None].to(DEV),
                                 torch.from_numpy(deltas)[None].to(DEV), img_w=img_w, img_h=img_h,
                                 pre_nms=pre, post_nms=post,
                                 anchors=torch.from_numpy(anchors).to(DEV))
    k = int(cnt[0])
    return rois[0, :k].cpu().numpy(), idx[0, :k].cpu().numpy().astype(np.int64)


@pytest.mark.parametrize("case", [0, 1, 2])
def test_propose_small_vs_reference(golden, case, path):
    g = golden(f"proposal_small{case}.npz")
    anchors = orc.generate_anchors(orc.generate_anchor_base(), 16, int(g["feat_w"]), int(g["feat_h"]))
    rois, idx = _propose_one_gpu(anchors, g["scores"], g["deltas"], int(g["img_w"]), int(g["img_h"]),
                                 int(g["pre"]), int(g["post"]))
    assert np.array_equal(idx, g["idx"])
    np.testing.assert_allclose(rois, g["rois"], rtol=RTOL, atol=1e-4)
    # and bit-exact against the oracle (same correctly-rounded exp)
    orois, oidx = orc.propose_one(anchors, g["scores"], g["deltas"], int(g["img_w"]),
                                  int(g["img_h"]), int(g["pre"]), int(g["post"]))
    assert np.array_equal(rois, orois)


@pytest.mark.parametrize("cfg,imgs", [("cfg1", (0, 1)), ("cfg2", (0, 1, 2, 3)), ("cfg4", (0,)),
                                      ("cfg5", (0, 1))])
def test_propose_batched_full_size(golden, cfg, imgs, path):
    """Batched path with in-kernel anchors at the BASELINE shapes."""
    g = golden("proposal_full.npz")
    c = synth.CONFIGS[cfg]
    base = A.generate_anchor_base_device(anchor_scales=c["scales"])
    K = base.size(0)
    Anc = c["feat_h"] * c["feat_w"] * K
    sc = torch.from_numpy(np.stack([synth.rpn_scores(Anc, 0, i) for i in imgs])).to(DEV)
    de = torch.from_numpy(np.stack([synth.rpn_deltas(Anc, 0, i) for i in imgs])).to(DEV)
    rois, idx, cnt = ops.propose(sc, de, img_w=c["img_w"], img_h=c["img_h"], pre_nms=c["pre_nms"],
                                 post_nms=c["post_nms"], anchor_base=base, feat_h=c["feat_h"],
                                 feat_w=c["feat_w"])
    for j, i in enumerate(imgs):
        k = int(cnt[j])
        gi = g[f"{cfg}_img{i}_idx"]
        assert k == len(gi)
        assert np.array_equal(idx[j, :k].cpu().numpy().astype(np.int64), gi), (cfg, i)
        np.testing.assert_allclose(rois[j, :k].cpu().numpy(), g[f"{cfg}_img{i}_rois"], rtol=RTOL,
                                   atol=1e-4)
        assert (idx[j, k:] == -1).all()


def test_propose_continuation_vs_oracle(path):
    """Scores peaked at the image centre: NMS suppresses most of the top candidates,
    so the 300th kept box is candidate ~1,250 of 6,000 (asserted on the oracle) and
    the hybrid path's sweep (first chunk 512 rows, from global scratch) must run
    the lazy continuation over two more chunks.  Bit-exact vs the oracle."""
    c = synth.CONFIGS["cfg2"]
    anchors = orc.generate_anchors(orc.generate_anchor_base(), 16, c["feat_w"], c["feat_h"])
    n = len(anchors)
    r = np.random.default_rng(3)
    cy = (anchors[:, 0] + anchors[:, 2]) / 2
    cx = (anchors[:, 1] + anchors[:, 3]) / 2
    scores = (np.exp(-((cy - 300) ** 2 + (cx - 500) ** 2) / 200.0 ** 2) + 0.01 * r.random(n)).astype(np.float32)
    deltas = np.zeros((n, 4), np.float32)
    bbox = orc.reg2bbox(anchors, deltas)
    bbox[:, [0, 2]] = np.clip(bbox[:, [0, 2]], 0, c["img_h"])
    bbox[:, [1, 3]] = np.clip(bbox[:, [1, 3]], 0, c["img_w"])
    m = (bbox[:, 2] - bbox[:, 0] >= 16) & (bbox[:, 3] - bbox[:, 1] >= 16)
    s = scores[np.nonzero(m)[0]]
    rank = np.argsort(-s, kind="stable")[:c["pre_nms"]]
    keep_all = orc.nms(bbox[np.nonzero(m)[0]][rank], s[rank], 0.7)
    assert keep_all[c["post_nms"] - 1] >= 1024  # the continuation is exercised
    rois, idx = _propose_one_gpu(anchors, scores, deltas, c["img_w"], c["img_h"], c["pre_nms"], c["post_nms"])
    orois, oidx = orc.propose_one(anchors, scores, deltas, c["img_w"], c["img_h"], c["pre_nms"], c["post_nms"])
    assert np.array_equal(idx, oidx)
    assert np.array_equal(rois, orois)


def test_propose_batch_invariance(path):
    """P-invariance: an image's proposals do not depend on its batch mates."""
    c = synth.CONFIGS["cfg2"]
    base = A.generate_anchor_base_device()
    Anc = c["feat_h"] * c["feat_w"] * 9
    sc = torch.from_numpy(np.stack([synth.rpn_scores(Anc, 5, i) for i in range(6)])).to(DEV)
    de = torch.from_numpy(np.stack([synth.rpn_deltas(Anc, 5, i) for i in range(6)])).to(DEV)
    kw = dict(img_w=c["img_w"], img_h=c["img_h"], pre_nms=c["pre_nms"], post_nms=c["post_nms"],
              anchor_base=base, feat_h=c["feat_h"], feat_w=c["feat_w"])
    full = ops.propose(sc, de, **kw)
    part = ops.propose(sc[3:5], de[3:5], **kw)
    for a, b in zip(full, part):
        assert torch.equal(a[3:5], b)


def test_nms_fixtures(golden):
    g = golden("nms.npz")
    names = sorted({k.rsplit("_", 1)[0] for k in g if k.endswith("_keep")})
    for n in names:
        keep = ops.nms(torch.from_numpy(g[f"{n}_boxes"]), torch.from_numpy(g[f"{n}_scores"]),
                       float(g[f"{n}_thr"]))
        assert keep.dtype == torch.int64
        assert np.array_equal(keep.numpy(), g[f"{n}_keep"]), n


def test_nms_random_thresholds():
    r = np.random.default_rng(3)
    for n, thr in [(1, 0.5), (63, 0.7), (64, 0.7), (65, 0.3), (1000, 0.9), (4097, 0.7)]:
        xy = r.uniform(0, 100, (n, 2)).astype(np.float32)
        wh = r.uniform(1, 40, (n, 2)).astype(np.float32)
        b = np.concatenate([xy, xy + wh], 1)
        s = r.random(n).astype(np.float32)
        keep = ops.nms(torch.from_numpy(b), torch.from_numpy(s), thr).numpy()
        assert np.array_equal(keep, orc.nms(b, s, thr)), (n, thr)
    empty = ops.nms(torch.zeros((0, 4)), torch.zeros(0), 0.7)
    assert empty.numel() == 0


def test_roi_pool_golden(golden):
    g = golden("roi_pool.npz")
    x = torch.from_numpy(g["x"]).to(DEV)
    rois = torch.from_numpy(g["rois_img"]).to(DEV)
    inds = torch.from_numpy(g["roi_inds"]).to(DEV)
    boxes = ops.roi_transform(rois, inds, int(g["img_h"]), int(g["img_w"]), x.shape[2], x.shape[3])
    assert np.array_equal(boxes.cpu().numpy(), g["boxes"])
    xg = x.clone().requires_grad_(True)
    out, am = ops.roi_pool_with_argmax(xg, boxes, (7, 7), 1.0)
    assert np.array_equal(out.detach().cpu().numpy(), g["out"])
    assert np.array_equal(am.cpu().numpy(), g["argmax"])
    out.backward(torch.from_numpy(g["grad"]).to(DEV))
    gi = xg.grad.cpu().numpy()
    np.testing.assert_allclose(gi, g["grad_in"], rtol=RTOL, atol=1e-6)
    assert np.array_equal(gi, g["grad_in"])  # CPU summation order reproduced


@pytest.mark.parametrize("N,C,H,W,R,ph", [(8, 256, 38, 63, 2400, 7), (2, 3, 9, 11, 77, 3),
                                          (1, 5, 4, 4, 40, 7), (2, 64, 50, 84, 300, 7),
                                          (16, 24, 38, 38, 2048, 7), (5, 4, 12, 12, 3, 7),
                                          (3, 8, 16, 16, 21, 8),
                                          # rectangular outputs: 7 wide with 9 / 5 / 1 rows
                                          # (the leader backward), 5 wide (the ring backward)
                                          (4, 12, 20, 24, 300, (9, 7)), (2, 6, 14, 10, 120, (5, 7)),
                                          (2, 6, 14, 10, 90, (1, 7)), (3, 6, 16, 12, 150, (7, 5))])
def test_roi_pool_vs_oracle(N, C, H, W, R, ph):
    r = np.random.default_rng(R)
    x = r.standard_normal((N, C, H, W), dtype=np.float32)
    x[:, :, ::3, ::2] = x[:, :, ::3, 1::2].max()  # ties: first max must win
    b = r.integers(0, N, R).astype(np.float32)
    xy = r.uniform(-3, max(H, W) + 2, (R, 2)).astype(np.float32)
    wh = r.uniform(-2, max(H, W), (R, 2)).astype(np.float32)
    rois = np.concatenate([b[:, None], xy, xy + wh], 1).astype(np.float32)
    out, am = ops.roi_pool_with_argmax(torch.from_numpy(x).to(DEV), torch.from_numpy(rois).to(DEV),
                                       ph, 1.0)
    oo, oa = orc.roi_pool_forward(x, rois, ph, 1.0)
    assert np.array_equal(out.cpu().numpy(), oo)
    assert np.array_equal(am.cpu().numpy(), oa)
    gr = r.standard_normal(oo.shape).astype(np.float32)
    from replication_faster_rcnn_amd.ops import _roi_pool_bwd
    gi = _roi_pool_bwd(torch.from_numpy(gr).to(DEV), torch.from_numpy(rois).to(DEV), am, x.shape, 1.0)
    ref = orc.roi_pool_backward(gr, rois, oa, x.shape)
    np.testing.assert_allclose(gi.cpu().numpy(), ref, rtol=RTOL, atol=1e-6)
    assert np.array_equal(gi.cpu().numpy(), ref)


def test_roi_pool_bwd_deterministic():
    r = np.random.default_rng(1)
    x = torch.from_numpy(r.standard_normal((2, 16, 20, 20), dtype=np.float32)).to(DEV)
    rois = torch.tensor([[0, 0, 0, 19, 19], [1, 2, 2, 3, 3], [0, 5, 5, 5.4, 5.4]] * 30,
                        dtype=torch.float32, device=DEV)
    out, am = ops.roi_pool_with_argmax(x, rois, 7)
    g = torch.randn(out.shape, device=DEV)
    from replication_faster_rcnn_amd.ops import _roi_pool_bwd
    a = _roi_pool_bwd(g, rois, am, x.shape, 1.0)
    b = _roi_pool_bwd(g, rois, am, x.shape, 1.0)
    assert torch.equal(a, b)


@pytest.mark.parametrize("sorted_", [False, True])
def test_roi_pool_out_of_range_batch_index(sorted_):
    """Extension: RoIs whose batch index is outside [0, N) pool to 0 / -1
    (torchvision reads out of bounds there)."""
    x = torch.randn(2, 8, 10, 12, device=DEV)
    rois = torch.tensor([[-1, 0, 0, 5, 5], [1, 0, 0, 9, 9], [2, 1, 1, 4, 4], [7, 0, 0, 3, 3]],
                        dtype=torch.float32, device=DEV)
    out, am = ops.roi_pool_with_argmax(x, rois, 7, rois_sorted=sorted_)
    assert (out[[0, 2, 3]] == 0).all() and (am[[0, 2, 3]] == -1).all()
    oo, oa = orc.roi_pool_forward(x.cpu().numpy(), rois[1:2].cpu().numpy(), 7, 1.0)
    assert np.array_equal(out[1:2].cpu().numpy(), oo) and np.array_equal(am[1:2].cpu().numpy(), oa)


@pytest.mark.parametrize("case", ["ties", "pre1", "post_gt_kept", "all_filtered", "thr0", "thr1",
                                  "chunk_edges"])
def test_propose_edge_cases(case, path):
    """Edge cases vs the oracle (ties ordered by ascending anchor index)."""
    fh, fw, img_h, img_w = 20, 30, 320, 480
    anchors = orc.generate_anchors(orc.generate_anchor_base(), 16, fw, fh)
    n = len(anchors)
    r = np.random.default_rng(sum(map(ord, case)))
    sc = synth.rpn_scores(n, 9, 0)
    de = synth.rpn_deltas(n, 9, 0)
    pre, post, thr = 3000, 300, 0.7
    if case == "ties":
        sc = (r.integers(0, 40, n) / 40).astype(np.float32)
    elif case == "pre1":
        pre, post = 1, 1
    elif case == "post_gt_kept":
        pre, post = 1025, 5000
    elif case == "all_filtered":
        de[:, 2:] = -6.0
    elif case == "thr0":
        thr = 0.0
    elif case == "thr1":
        thr, post = 1.0, 4000
    elif case == "chunk_edges":
        pre, post = 2049, 4000
    rois, idx, cnt = ops.propose(torch.from_numpy(sc)[None].to(DEV), torch.from_numpy(de)[None].to(DEV),
                                 img_w=img_w, img_h=img_h, pre_nms=pre, post_nms=post, nms_thresh=thr,
                                 anchors=torch.from_numpy(anchors).to(DEV))
    orois, oidx = orc.propose_one(anchors, sc, de, img_w, img_h, pre, post, nms_thresh=thr)
    k = int(cnt[0])
    assert k == len(oidx), (k, len(oidx))
    assert np.array_equal(idx[0, :k].cpu().numpy(), oidx)
    assert np.array_equal(rois[0, :k].cpu().numpy(), orois)


# forward paths: (kernel path, RoIs promised grouped by image)
FWD_PATHS = [("wave", True), ("dense", True), ("dense", False), ("generic", False)]


def _special_x(r, N=2, C=16, H=12, W=14):
    x = r.standard_normal((N, C, H, W)).astype(np.float32)
    x[0, 0] = 0.0
    x[0, 0, ::2, ::3] = -0.0                       # +-0 ties: first zero's sign wins
    x[0, 1] = -np.float32(3.4028235e38)            # all -FLT_MAX: nothing selected
    x[0, 2] = -np.inf
    x[0, 3, ::2] = np.nan
    x[0, 4, 3:6, 3:6] = np.inf
    x[1, 5] = np.nan
    x[1, 6, :, 5] = 7.0                            # column plateau of equal maxima
    x[1, 7] = -0.0
    x[1, 8:16] = np.round(x[1, 8:16])
    x[1, 9] = np.maximum(x[1, 9], 0.0)             # ReLU: zero maxima, some -0
    x[1, 9, 1::4, ::3] = -0.0
    return x


@pytest.mark.parametrize("hw", [(12, 14), (38, 38)])
@pytest.mark.parametrize("fpath,sorted_", FWD_PATHS)
def test_roi_pool_special_values(fpath, sorted_, hw):
    """Signed zeros, -FLT_MAX, +-inf and NaN inside pooling windows, RoIs partly /
    fully outside the map: every path reproduces the reference's strict-'>'
    first-max scan bit for bit (values compared as bits).  38 x 38 takes the
    wave kernel's compile-time plane stride (one workgroup per CU), 12 x 14 the
    run-time stride."""
    r = np.random.default_rng(7)
    x = _special_x(r, H=hw[0], W=hw[1])
    N = x.shape[0]
    rois = np.array([[b, x1, y1, x1 + w, y1 + h] for b in range(N) for (x1, y1, w, h) in
                     [(0, 0, 13, 11), (1, 2, 5, 3), (3, 3, 0, 0), (2, 1, 9, 9), (-3, -2, 20, 20),
                      (10, 8, 30, 30), (-20, -20, 5, 5), (4, 1, 1.4, 7)]], np.float32)
    if not sorted_:
        rois = rois[r.permutation(len(rois))]
    with _lib.kernel_path("roi_pool_fwd", fpath):
        out, am = ops.roi_pool_with_argmax(torch.from_numpy(x).to(DEV), torch.from_numpy(rois).to(DEV), 7,
                                           rois_sorted=sorted_)
    oo, oa = orc.roi_pool_forward(x, rois, 7)
    assert np.array_equal(am.cpu().numpy(), oa)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), oo.view(np.uint32))


def test_roi_pool_nontemporal_stores():
    """The wave forward with non-temporal output stores (roi_pool_fwd_store nt):
    the same bits as the oracle, special values included."""
    r = np.random.default_rng(7)
    x = _special_x(r, H=38, W=38)
    N = x.shape[0]
    rois = np.array([[b, x1, y1, x1 + w, y1 + h] for b in range(N) for (x1, y1, w, h) in
                     [(0, 0, 13, 11), (1, 2, 5, 3), (3, 3, 0, 0), (2, 1, 9, 9), (-3, -2, 20, 20)]], np.float32)
    with _lib.kernel_path("roi_pool_fwd", "wave"), _lib.kernel_path("roi_pool_fwd_store", "nt"):
        out, am = ops.roi_pool_with_argmax(torch.from_numpy(x).to(DEV), torch.from_numpy(rois).to(DEV), 7,
                                           rois_sorted=True)
        assert _lib.roi_pool_fwd_kernel(len(rois), N, x.shape[1], x.shape[2], x.shape[3]).endswith(", true, 38400>")
    oo, oa = orc.roi_pool_forward(x, rois, 7)
    assert np.array_equal(am.cpu().numpy(), oa)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), oo.view(np.uint32))


@pytest.mark.parametrize("fpath,sorted_", FWD_PATHS)
def test_roi_pool_paths_random(fpath, sorted_):
    """Every forward path, cfg2-like random RoIs with plenty of ties, bit-exact vs the oracle."""
    r = np.random.default_rng(11)
    N, C, H, W, R = 3, 32, 38, 63, 600
    x = r.standard_normal((N, C, H, W), dtype=np.float32)
    x[:, :, 10:20, 10:30] = np.round(x[:, :, 10:20, 10:30])  # plenty of ties
    b = np.sort(r.integers(0, N, R)).astype(np.float32)
    if not sorted_:
        r.shuffle(b)
    xy = r.uniform(-3, 60, (R, 2)).astype(np.float32)
    wh = r.uniform(0, 40, (R, 2)).astype(np.float32)
    rois = np.concatenate([b[:, None], xy, xy + wh], 1).astype(np.float32)
    with _lib.kernel_path("roi_pool_fwd", fpath):
        out, am = ops.roi_pool_with_argmax(torch.from_numpy(x).to(DEV), torch.from_numpy(rois).to(DEV), 7,
                                           rois_sorted=sorted_)
    oo, oa = orc.roi_pool_forward(x, rois, 7)
    assert np.array_equal(am.cpu().numpy(), oa)
    assert np.array_equal(out.cpu().numpy(), oo)


def _rand_rois(r, b, H, W, lo=-3, span=40):
    xy = r.uniform(lo, max(H, W) + 2, (len(b), 2)).astype(np.float32)
    wh = r.uniform(0, span, (len(b), 2)).astype(np.float32)
    return np.concatenate([np.asarray(b, np.float32)[:, None], xy, xy + wh], 1).astype(np.float32)


@pytest.mark.parametrize("fpath", ["wave", "dense"])
@pytest.mark.parametrize("split", ["auto", "1", "3", "64"])
@pytest.mark.parametrize("case", ["many_images", "invalid_ends", "unsorted", "single_roi", "gaps",
                                  "one_image_tiny_rois", "uniform_sizes", "ph5", "ph8x8", "ph3x9",
                                  "cfg4_shape", "c8", "c4", "ph1_huge", "ph2_wide",
                                  "kps_7x7", "kps_1x49", "kps_49x1"])
def test_roi_pool_tile_cases(case, split, fpath):
    """The image-tile forwards (shape-sorted bins, and RoI-packed "dense"):
    cost-balanced shares (`split` per image), geometry chunks, every window
    shape class (dw 1-4 unrolled, 5-62 uniform loop, > 62 per-lane), any
    PH x PW <= 64, out-of-range batch indices, 16 / 8 / 4-channel tiles, and
    any RoI order (per-image lists) -- bit-exact vs the oracle."""
    r = np.random.default_rng(sum(map(ord, case)))
    ph, pw = {"ph5": (5, 5), "ph8x8": (8, 8), "ph3x9": (3, 9), "ph1_huge": (1, 1),
              "ph2_wide": (2, 3), "kps_1x49": (1, 49), "kps_49x1": (49, 1)}.get(case, (7, 7))
    N, C, H, W = 4, 16, 20, 27
    span = 40
    sorted_ = case != "unsorted"
    if case == "ph1_huge":  # one bin = the whole RoI: windows up to 80 x 100 (> 62)
        N, C, H, W, span = 2, 8, 80, 100, 110
        b = np.sort(r.integers(0, N, 300))
    elif case == "ph2_wide":
        N, C, H, W, span = 2, 16, 30, 90, 80
        b = np.sort(r.integers(0, N, 300))
    elif case == "many_images":  # more images than one geometry chunk
        N, C, H, W, span = 20000, 8, 4, 5, 6
        b = np.sort(r.integers(0, N, 40000))
    elif case == "invalid_ends":
        b = np.concatenate([[-1, -1], np.sort(r.integers(0, N, 200)), [N, N, N + 3]])
    elif case == "unsorted":
        b = np.concatenate([r.integers(0, N, 500), [-1, N + 2]])
        r.shuffle(b)
    elif case == "single_roi":
        b = np.array([2])
    elif case == "gaps":  # images 1 and 2 have no RoIs
        b = np.sort(np.concatenate([np.zeros(60, int), np.full(90, 3)]))
    elif case == "cfg4_shape":  # 50x84 tile: 8-channel planes, one workgroup per CU
        N, C, H, W = 1, 16, 50, 84
        b = np.zeros(500, int)
    elif case == "one_image_tiny_rois":  # > one geometry chunk per workgroup
        N, b, span = 1, np.zeros(6000, int), 2
    elif case.startswith("kps_"):  # a map whose 16-plane tile holds the CU alone: the fixed
        # plane stride for 7x7 only, never for the other 49-bin shapes
        N, C, H, W = 2, 16, 38, 38
        b = np.sort(r.integers(0, N, 400))
    elif case in ("c8", "c4"):
        C = 8 if case == "c8" else 12
        b = np.sort(r.integers(0, N, 300))
    else:
        b = np.sort(r.integers(0, N, 700))
    x = r.standard_normal((N, C, H, W), dtype=np.float32)
    x[:, :, 2:9, 3:12] = np.round(x[:, :, 2:9, 3:12])  # ties
    rois = _rand_rois(r, b, H, W, span=span)
    if case == "uniform_sizes":
        rois[:, 3:] = rois[:, 1:3] + 6.0
    with _lib.kernel_path("roi_pool_split", split), _lib.kernel_path("roi_pool_fwd", fpath):
        out, am = ops.roi_pool_with_argmax(torch.from_numpy(x).to(DEV), torch.from_numpy(rois).to(DEV),
                                           (ph, pw), rois_sorted=sorted_)
        if case.startswith("kps_"):
            kn = _lib.roi_pool_fwd_kernel(len(b), N, C, H, W, ph, pw, head=False)
            assert kn.endswith(", 38400>") == (case == "kps_7x7" and fpath == "wave"), kn
    oo, oa = orc.roi_pool_forward(x, rois, (ph, pw))
    valid = (b >= 0) & (b < N)
    assert np.array_equal(am.cpu().numpy()[valid], oa[valid])
    assert np.array_equal(out.cpu().numpy()[valid].view(np.uint32), oo[valid].view(np.uint32))
    assert (out.cpu().numpy()[~valid] == 0).all() and (am.cpu().numpy()[~valid] == -1).all()


@pytest.mark.parametrize("sorted_", [True, False])
def test_roi_pool_cfg2_shape(sorted_):
    """The bench shape (8 x 256 x 38 x 63, 300 RoIs per image): dense forward
    bit for bit vs the oracle on a sample of RoIs from every image."""
    r = np.random.default_rng(5)
    N, C, H, W, per = 8, 256, 38, 63, 300
    x = r.standard_normal((N, C, H, W), dtype=np.float32)
    b = np.repeat(np.arange(N), per)
    rois = _rand_rois(r, b, H, W, span=45)
    perm = np.arange(len(b)) if sorted_ else r.permutation(len(b))
    rois = rois[perm]
    out, am = ops.roi_pool_with_argmax(torch.from_numpy(x).to(DEV), torch.from_numpy(rois).to(DEV), 7,
                                       rois_sorted=sorted_)
    pick = np.concatenate([np.arange(i * per, i * per + 25) for i in range(N)] + [np.arange(2390, 2400)])
    oo, oa = orc.roi_pool_forward(x, rois[pick], 7)
    assert np.array_equal(am.cpu().numpy()[pick], oa)
    assert np.array_equal(out.cpu().numpy()[pick], oo)


def test_roi_pool_cfg4_full_shape():
    """BASELINE configs[3] in full: 1 x 512 x 50 x 84 features, 2000 proposals of
    an 800x1333 image through the head's transform + RoIPool (one launch), every
    output and argmax bit-exact vs the oracle; gradient bit-exact too."""
    c = synth.CONFIGS["cfg4"]
    r = np.random.default_rng(44)
    H, W, C, R = c["feat_h"], c["feat_w"], c["C"], c["post_nms"]
    x = synth.features(C, H, W, 0, 0)[None]
    y1 = r.uniform(-20, c["img_h"], R).astype(np.float32)
    x1 = r.uniform(-20, c["img_w"], R).astype(np.float32)
    rois = np.stack([y1, x1, y1 + r.uniform(8, 520, R).astype(np.float32),
                     x1 + r.uniform(8, 700, R).astype(np.float32)], 1).astype(np.float32)
    inds = np.zeros(R, np.float32)
    xt = torch.from_numpy(x).to(DEV).requires_grad_(True)
    out, am, boxes = ops.roi_pool_head(xt, torch.from_numpy(rois).to(DEV), torch.from_numpy(inds).to(DEV),
                                       7, c["img_h"], c["img_w"], rois_sorted=True)
    oboxes = orc.roi_transform(rois, inds, c["img_h"], c["img_w"], H, W)
    assert np.array_equal(boxes.cpu().numpy(), oboxes)
    oo, oa = orc.roi_pool_forward(x, oboxes, 7)
    assert np.array_equal(am.cpu().numpy(), oa)
    assert np.array_equal(out.detach().cpu().numpy(), oo)
    g = torch.from_numpy(r.standard_normal(out.shape, dtype=np.float32)).to(DEV)
    (out * g).sum().backward()
    og = orc.roi_pool_backward(g.cpu().numpy(), oboxes, oa, x.shape)
    assert np.array_equal(xt.grad.cpu().numpy(), og)


@pytest.mark.parametrize("case", ["grouped", "grouped_split3", "grouped_cg8", "ungrouped", "out_of_range",
                                  "c_not8", "many_per_image"])
def test_roi_pool_head_fused(case):
    """ops.roi_pool_head = nets/heads.py:42-48 (transform + pack + roi_pool) in
    one call: boxes, out and argmax bit-exact vs the oracle's roi_transform +
    roi_pool, and its gradient identical to roi_pool's on the same boxes."""
    split = {"grouped_split3": "3", "many_per_image": "1"}.get(case, "auto")
    r = np.random.default_rng(sum(map(ord, case)))
    N, C, H, W, img_h, img_w = 3, 16, 38, 63, 600.0, 1000.0
    if case == "c_not8":
        C = 12
    if case == "grouped_cg8":
        C = 24
    R = 257
    if case == "many_per_image":  # > geo_cap RoIs per workgroup: several geometry chunks
        N, C, R = 1, 16, 9000
    inds = np.sort(r.integers(0, N, R)).astype(np.float32)
    if case == "ungrouped":
        r.shuffle(inds)
    if case == "out_of_range":
        inds[:3] = -1.0
        inds[-4:] = N + 1
        inds = np.sort(inds)
    y1 = r.uniform(-20, img_h, R).astype(np.float32)
    x1 = r.uniform(-20, img_w, R).astype(np.float32)
    rois = np.stack([y1, x1, y1 + r.uniform(0, 400, R).astype(np.float32),
                     x1 + r.uniform(0, 600, R).astype(np.float32)], 1).astype(np.float32)
    x = r.standard_normal((N, C, H, W), dtype=np.float32)
    x[:, :, 5:15, 5:25] = np.round(x[:, :, 5:15, 5:25])  # ties
    xt = torch.from_numpy(x).to(DEV).requires_grad_(True)
    with _lib.kernel_path("roi_pool_split", split):
        out, am, boxes = ops.roi_pool_head(xt, torch.from_numpy(rois).to(DEV), torch.from_numpy(inds).to(DEV),
                                           7, img_h, img_w, rois_sorted=case != "ungrouped")
    oboxes = orc.roi_transform(rois, inds, img_h, img_w, H, W)
    assert np.array_equal(boxes.cpu().numpy().view(np.uint32), oboxes.view(np.uint32))
    oo, oa = orc.roi_pool_forward(x, oboxes, 7)
    valid = (inds.astype(np.int64) >= 0) & (inds.astype(np.int64) < N)
    assert np.array_equal(am.cpu().numpy()[valid], oa[valid])
    assert np.array_equal(out.detach().cpu().numpy()[valid].view(np.uint32), oo[valid].view(np.uint32))
    assert (out.detach().cpu().numpy()[~valid] == 0).all() and (am.cpu().numpy()[~valid] == -1).all()
    g = torch.from_numpy(r.standard_normal(out.shape, dtype=np.float32)).to(DEV)
    (out * g).sum().backward()
    og = orc.roi_pool_backward(g.cpu().numpy(), oboxes, am.cpu().numpy(), x.shape)  # -1 rows skipped
    assert np.array_equal(xt.grad.cpu().numpy(), og)


BWD_VARIANTS = ["auto", "ring"]


@pytest.mark.parametrize("path", BWD_VARIANTS)
def test_roi_pool_bwd_ring_equals_plain(path):
    """The latency-hidden backwards (the leader-gather kernel -- the default
    for 7-wide outputs -- and the RoI-at-a-time ring) and the plain
    plane-owner kernel give identical bits, incl. duplicated RoIs (same argmax
    pixels across RoIs and bins), images with 0 / fewer than 6 / 6k+r RoIs."""
    from replication_faster_rcnn_amd.ops import _roi_pool_bwd
    r = np.random.default_rng(7)
    N, C, H, W = 4, 20, 38, 38
    x = torch.from_numpy(r.standard_normal((N, C, H, W), dtype=np.float32)).to(DEV)
    per = [0, 5, 8, 77]
    rows = []
    for b, k in enumerate(per):
        for _ in range(k):
            x0, y0 = r.uniform(-2, 30, 2)
            w, h = r.uniform(0, 20, 2)
            rows.append([b, x0, y0, x0 + w, y0 + h])
    rows += rows[-10:]  # duplicates in the last image
    rois = torch.tensor(rows, dtype=torch.float32, device=DEV)
    out, am = ops.roi_pool_with_argmax(x, rois, 7)
    g = torch.randn(out.shape, device=DEV)
    with _lib.kernel_path("roi_pool_bwd", path):
        a = _roi_pool_bwd(g, rois, am, x.shape, 1.0)
    with _lib.kernel_path("roi_pool_bwd", "plain"):
        b = _roi_pool_bwd(g, rois, am, x.shape, 1.0)
    assert torch.equal(a, b)
    ref = orc.roi_pool_backward(g.cpu().numpy(), rois.cpu().numpy(), am.cpu().numpy(), x.shape)
    assert np.array_equal(a.cpu().numpy(), ref)


@pytest.mark.parametrize("path", BWD_VARIANTS + ["plain"])
def test_roi_pool_bwd_denormal_and_colliding_grads(path):
    """The backward's LDS adds keep IEEE semantics: denormal gradients and sums
    (no flush to zero), many same-pixel contributions (tiny RoIs whose 49 bins
    share a few pixels), signed zeros -- bit-identical to the CPU order."""
    from replication_faster_rcnn_amd.ops import _roi_pool_bwd
    r = np.random.default_rng(11)
    N, C, H, W = 2, 6, 16, 10
    x = torch.from_numpy(r.standard_normal((N, C, H, W), dtype=np.float32)).to(DEV)
    rows = [[0, 2, 2, 2.4, 2.4], [0, 1, 1, 2, 2], [1, 0, 0, 9, 15], [1, 3, 3, 5, 4], [0, 4, 7, 5, 8.4]] * 5
    rows += [[b, *r.uniform(0, 9, 2), *r.uniform(0, 15, 2)] for b in (0, 1) for _ in range(9)]
    rois = torch.tensor(rows, dtype=torch.float32, device=DEV)
    out, am = ops.roi_pool_with_argmax(x, rois, 7)
    g = r.standard_normal(tuple(out.shape)).astype(np.float32)
    scale = np.where(r.random(g.shape) < 0.5, np.float32(1e-39), np.float32(1.0)).astype(np.float32)
    g = (g * scale).astype(np.float32)
    g[r.random(g.shape) < 0.05] = -0.0
    assert (np.abs(g[g != 0]) < np.finfo(np.float32).tiny).any()
    with _lib.kernel_path("roi_pool_bwd", path):
        gi = _roi_pool_bwd(torch.from_numpy(g).to(DEV), rois, am, x.shape, 1.0)
    ref = orc.roi_pool_backward(g, rois.cpu().numpy(), am.cpu().numpy(), x.shape)
    assert np.array_equal(gi.cpu().numpy().view(np.uint32), ref.view(np.uint32))


def test_propose_caller_buffers():
    """ops.propose(out=..., workspace=...) writes the same result into caller-owned
    buffers (the static-buffer path of bench.py --issue capi and of graph capture)."""
    na = 38 * 63 * 9
    sc = torch.from_numpy(np.stack([synth.rpn_scores(na, 3, i) for i in range(3)])).cuda()
    de = torch.from_numpy(np.stack([synth.rpn_deltas(na, 3, i) for i in range(3)])).cuda()
    base = A.generate_anchor_base_device()
    kw = dict(img_w=1000, img_h=600, pre_nms=6000, post_nms=300, anchor_base=base, feat_h=38,
              feat_w=63)
    r0, i0, c0 = ops.propose(sc, de, **kw)
    out = (torch.full_like(r0, 7.0), torch.full_like(i0, 5), torch.full_like(c0, 9))
    ws = torch.empty(1 << 26, dtype=torch.uint8, device="cuda")
    r1, i1, c1 = ops.propose(sc, de, out=out, workspace=ws, **kw)
    assert r1.data_ptr() == out[0].data_ptr()
    assert torch.equal(r0, r1) and torch.equal(i0, i1) and torch.equal(c0, c1)
    with pytest.raises(RuntimeError):
        ops.propose(sc, de, out=(out[0][:, :10], out[1], out[2]), **kw)



def test_benched_step_cfg2_vs_oracle():
    """The exact composition bench.py times at cfg2 (BASELINE configs[1]): the
    batched proposal layer over 8 x 38 x 63 x 9 anchors (6000 -> 300) feeding
    the head's transform + pack + RoIPool (roi_pool_fwd_wave_kernel<.., HEAD>,
    rois_sorted) over all 2400 padded proposal rows, against the oracle's
    nets/rpn.py:58-77 per image -> nets/heads.py:42-47 -> torchvision roi_pool.
    Runs on a plain side stream: the pool sizes its shares to the launch
    stream's CUs, as in the bench's step streams."""
    from bench import make_inputs
    c = synth.CONFIGS["cfg2"]
    N, post, H, W = c["batch"], c["post_nms"], c["feat_h"], c["feat_w"]
    _, sc, de, x = make_inputs("cfg2", range(N), torch.device(DEV))
    base = A.generate_anchor_base_device(anchor_scales=c["scales"])
    inds = torch.arange(N, device=DEV, dtype=torch.float32).repeat_interleave(post)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        rois, idx, cnt = ops.propose(sc, de, img_w=c["img_w"], img_h=c["img_h"], pre_nms=c["pre_nms"],
                                     post_nms=post, anchor_base=base, feat_h=H, feat_w=W)
        out, am, boxes = ops.roi_pool_head(x, rois.view(-1, 4), inds, 7, c["img_h"], c["img_w"],
                                           rois_sorted=True)
    s.synchronize()
    anchors = orc.generate_anchors(orc.generate_anchor_base(anchor_scales=c["scales"]), 16, W, H)
    Anc = len(anchors)
    o_rois = np.zeros((N, post, 4), np.float32)
    for i in range(N):
        r_i, i_i = orc.propose_one(anchors, synth.rpn_scores(Anc, 0, i), synth.rpn_deltas(Anc, 0, i),
                                   c["img_w"], c["img_h"], c["pre_nms"], post)
        k = int(cnt[i])
        assert k == len(i_i), i
        assert np.array_equal(idx[i, :k].cpu().numpy().astype(np.int64), i_i), i
        o_rois[i, :k] = r_i
    assert np.array_equal(rois.cpu().numpy().view(np.uint32), o_rois.view(np.uint32))
    oboxes = orc.roi_transform(o_rois.reshape(-1, 4), inds.cpu().numpy(), c["img_h"], c["img_w"], H, W)
    assert np.array_equal(boxes.cpu().numpy().view(np.uint32), oboxes.view(np.uint32))
    oo, oa = orc.roi_pool_forward(x.cpu().numpy(), oboxes, 7)
    assert np.array_equal(am.cpu().numpy(), oa)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), oo.view(np.uint32))


@pytest.mark.parametrize("ss", [0.5, 0.0625, 2.0])
@pytest.mark.parametrize("sorted_", [True, False])
def test_roi_pool_spatial_scale(ss, sorted_):
    """spatial_scale != 1 (torchvision's roundf(roi * spatial_scale) RoI ends):
    forward (wave / dense paths) and backward bit-exact vs the oracle.  The
    reference itself passes 1 (nets/heads.py:8,48)."""
    r = np.random.default_rng(int(ss * 1000) + sorted_)
    N, C, H, W, R = 3, 16, 24, 30, 240
    x = r.standard_normal((N, C, H, W), dtype=np.float32)
    b = np.sort(r.integers(0, N, R)) if sorted_ else r.integers(0, N, R)
    lim = max(H, W) / ss
    xy = r.uniform(-3 / ss, lim, (R, 2)).astype(np.float32)
    wh = r.uniform(0, lim, (R, 2)).astype(np.float32)
    rois = np.concatenate([b[:, None].astype(np.float32), xy, xy + wh], 1).astype(np.float32)
    out, am = ops.roi_pool_with_argmax(torch.from_numpy(x).to(DEV), torch.from_numpy(rois).to(DEV), 7,
                                       ss, rois_sorted=bool(sorted_))
    oo, oa = orc.roi_pool_forward(x, rois, 7, ss)
    assert np.array_equal(am.cpu().numpy(), oa)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), oo.view(np.uint32))
    gr = r.standard_normal(oo.shape).astype(np.float32)
    from replication_faster_rcnn_amd.ops import _roi_pool_bwd
    gi = _roi_pool_bwd(torch.from_numpy(gr).to(DEV), torch.from_numpy(rois).to(DEV), am, x.shape, ss)
    assert np.array_equal(gi.cpu().numpy(), orc.roi_pool_backward(gr, rois, oa, x.shape))


@pytest.mark.parametrize("path", BWD_VARIANTS)
def test_roi_pool_bwd_poisoned_workspace(path):
    """The backward's per-image RoI lists are written only up to each image's
    count; the kernels must not read past it.  The cached workspace is filled
    with 0x7f bytes (RoI index 0x7f7f7f7f) before the call."""
    from replication_faster_rcnn_amd.ops import _roi_pool_bwd
    r = np.random.default_rng(77)
    N, C, H, W, R = 4, 8, 20, 22, 37  # image RoI counts not multiples of the ring depth
    x = r.standard_normal((N, C, H, W), dtype=np.float32)
    b = r.integers(0, N, R).astype(np.float32)
    xy = r.uniform(-2, 20, (R, 2)).astype(np.float32)
    rois = np.concatenate([b[:, None], xy, xy + r.uniform(0, 15, (R, 2)).astype(np.float32)], 1)
    rois = rois.astype(np.float32)
    oo, oa = orc.roi_pool_forward(x, rois, 7)
    gr = r.standard_normal(oo.shape).astype(np.float32)
    ref = orc.roi_pool_backward(gr, rois, oa, x.shape)
    lib = _lib.load()
    need = lib.frcnn_roi_pool_bwd_workspace_size(R, N, 7, 7)
    with _lib.kernel_path("roi_pool_bwd", path):
        ws = _lib.cached_workspace("roi_pool_bwd", need, torch.device(DEV))
        ws.fill_(0x7f)
        gi = _roi_pool_bwd(torch.from_numpy(gr).to(DEV), torch.from_numpy(rois).to(DEV),
                           torch.from_numpy(oa).to(DEV), x.shape, 1.0)
        torch.cuda.synchronize()
    assert np.array_equal(gi.cpu().numpy(), ref)


def test_roi_pool_fwd_kernel_label():
    """frcnn_roi_pool_fwd_kernel names what frcnn_roi_pool_fwd(_head) launches:
    the wave kernel by default for RoIs grouped by image, the dense kernel for
    unsorted RoIs (bench.py's roofline label)."""
    R, N, C, H, W = 2400, 8, 256, 38, 63
    assert _lib.roi_pool_fwd_kernel(R, N, C, H, W) == "roi_pool_fwd_wave_kernel<1024, 16, 7, true, false, 38400>"
    assert _lib.roi_pool_fwd_kernel(R, N, C, H, W, head=False) == "roi_pool_fwd_wave_kernel<1024, 16, 7, false, false, 38400>"
    assert _lib.roi_pool_fwd_kernel(2000, 1, 512, 50, 84) == "roi_pool_fwd_wave_kernel<1024, 8, 7, true>"
    assert _lib.roi_pool_fwd_kernel(R, N, C, H, W, rois_sorted=False, head=False).startswith(
        "roi_pool_fwd_dense_kernel<1024, 16, 7, false, true>")
    # the backward's label follows its plan (band kernel for 7-wide bins, leader / ring / plain on request)
    assert _lib.roi_pool_bwd_kernel(2048, 16, 256, 38, 38) == "roi_pool_bwd_lead_kernel<4, 7, 7>"
    assert _lib.roi_pool_bwd_kernel(2048, 16, 256, 38, 38, 9, 7) == "roi_pool_bwd_lead_kernel<4, 7, 0>"
    assert _lib.roi_pool_bwd_kernel(2048, 16, 256, 38, 38, 5, 5) == "roi_pool_bwd_pf_kernel<8>"
    with _lib.kernel_path("roi_pool_bwd", "ring"):
        assert _lib.roi_pool_bwd_kernel(2048, 16, 256, 38, 38) == "roi_pool_bwd_pf_kernel<8>"
    with _lib.kernel_path("roi_pool_bwd", "plain"):
        assert _lib.roi_pool_bwd_kernel(2048, 16, 256, 38, 38) == "roi_pool_bwd_kernel<true>"
