"""Throughput bench of the region-proposal + RoI hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2]

One "step" = one pass of the hot path over one batch of synthetic VOC-shaped
input already resident in HBM (BASELINE.json configs[1] = cfg2: 8 images of
600x1000, stride-16 38x63x9 anchors, 6000->300 NMS@0.7, RoIPool 7x7x256):

    propose (decode+clamp+filter+top-k+NMS+post, anchors generated in-kernel)
    -> RoI transform + pack + RoIPool forward (nets/heads.py:42-48, one launch)

By default the proposal layer and the RoIPool run on two HIP streams, so step
k+1's proposals (8 one-image workgroups + two small chip-wide kernels) run
beside step k's RoIPool (every step still does all of its work; --streams 1
serialises them).  The proposal layers of consecutive steps alternate over two
HIP streams (--prop-streams, default 2), so two latency-bound proposal chains
overlap each other as well as the pool (measured cfg2: 81k -> 86-87k images/s).

For N>1 (torch.distributed.run, one process per GPU) every rank runs its own
batch of 8 images (weak scaling, images seeded by global index) and the
padded detections are all-gathered over RCCL at the end of each step -- the
only collective on this path.

Prints ONE JSON line (rank 0) with the metric of BASELINE.json plus
"roofline" (the RoIPool forward launch, achieved algorithmic HBM GB/s from
HIP events on the launch stream vs the 8 TB/s peak) and "cpu_baseline" (the oracle CPU path on this host).
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--streams", type=int, default=2, choices=(1, 2),
                    help="2: the proposal layer of step k+1 runs on its own HIP stream beside "
                         "step k's RoIPool (each step still does all of its work)")
    ap.add_argument("--prop-cus", type=int, default=0,
                    help="with --streams 2: run the proposal stream on this many CUs and the "
                         "RoIPool stream on the rest (hipExtStreamCreateWithCUMask); 0 = shared")
    ap.add_argument("--prop-streams", type=int, default=2,
                    help="with --streams 2 (inference configs): proposal layers of consecutive "
                         "steps round-robin over this many HIP streams, so step k+1's and "
                         "k+2's proposals (latency bound, few CUs busy) overlap each other too")
    ap.add_argument("--prop-buffers", type=int, default=4,
                    help="--issue capi: proposal output sets in flight (multiple of --prop-streams)")
    ap.add_argument("--host-io", type=int, default=0, choices=(0, 1),
                    help="1: PCIe-inclusive variant -- each step copies its inputs (scores, "
                         "deltas, features) from pinned host memory and the rois + pooled "
                         "features back, like the reference's host-resident tensors (never the "
                         "default value)")
    ap.add_argument("--issue", default="ops", choices=("capi", "ops"),
                    help="inference configs: ops = the Python drop-in ops (default); capi = "
                         "each step is two direct C-ABI calls on preallocated buffers (a native "
                         "host's issue path: 40 vs 88 us of host time per step, but the proposal "
                         "chains then run ahead into the RoIPool and the step is slower, "
                         "110 vs 99 us -- kept as an A/B)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="bounded CPU-baseline sample (rank 0, N=1 only); 0 disables")
    return ap.parse_args()


def setup_dist(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def make_inputs(cfg, batch, first_image, device):
    from replication_faster_rcnn_amd import synth
    c = synth.CONFIGS[cfg]
    K = 3 * len(c["scales"])
    A = c["feat_h"] * c["feat_w"] * K
    imgs = range(first_image, first_image + batch)
    sc = torch.from_numpy(np.stack([synth.rpn_scores(A, 0, i) for i in imgs])).to(device)
    de = torch.from_numpy(np.stack([synth.rpn_deltas(A, 0, i) for i in imgs])).to(device)
    x = torch.from_numpy(np.stack([synth.features(c["C"], c["feat_h"], c["feat_w"], 0, i)
                                   for i in imgs])).to(device)
    return c, sc, de, x


def cpu_baseline(cfg, seconds):
    """Oracle CPU path (numpy restatement + single-threaded C nms/roi_pool,
    the reference's own per-image loop nets/rpn.py:131) on a bounded sample."""
    from oracle import ref_numpy as orc
    from replication_faster_rcnn_amd import synth
    c = synth.CONFIGS[cfg]
    base = orc.generate_anchor_base(anchor_scales=c["scales"])
    done, t0, i = 0, time.perf_counter(), 0
    warm = True
    while True:
        anchors = orc.generate_anchors(base, 16, c["feat_w"], c["feat_h"])
        A = len(anchors)
        sc, de = synth.rpn_scores(A, 0, i), synth.rpn_deltas(A, 0, i)
        x = synth.features(c["C"], c["feat_h"], c["feat_w"], 0, i)[None]
        if warm:
            t0 = time.perf_counter()
        ts = time.perf_counter()
        rois, _ = orc.propose_one(anchors, sc, de, c["img_w"], c["img_h"], c["pre_nms"], c["post_nms"])
        boxes = orc.roi_transform(rois, np.zeros(len(rois), np.float32), c["img_h"], c["img_w"],
                                  c["feat_h"], c["feat_w"])
        orc.roi_pool_forward(x, boxes, 7, 1.0)
        te = time.perf_counter()
        if warm:
            warm = False
            t0 = te
            continue
        done += 1
        i += 1
        if te - t0 >= seconds:
            break
    el = time.perf_counter() - t0
    return {"value": done / el, "unit": "images/sec", "cores": 1, "kind": "port",
            "sample": f"{done} {cfg}-shaped images, one at a time (oracle: numpy + 1-thread C "
                      f"nms/roi_pool), after 1 warm-up image; {el:.1f} s on {os.cpu_count()}-cpu host"}


def cpu_baseline_train(cfg, seconds):
    """Oracle CPU training-step path per image (train.py:67-108 loops + the
    RoIPool forward/backward of nets/heads.py:48), bounded sample."""
    from oracle import ref_numpy as orc
    from replication_faster_rcnn_amd import synth
    c = synth.CONFIGS[cfg]
    base = orc.generate_anchor_base(anchor_scales=c["scales"])
    anchors = orc.generate_anchors(base, 16, c["feat_w"], c["feat_h"])
    A = len(anchors)
    g = np.random.default_rng(1).standard_normal((128, c["C"], 7, 7), dtype=np.float32)
    np.random.seed(0)
    done, t0, i, warm = 0, time.perf_counter(), 0, True
    while True:
        sc, de = synth.rpn_scores(A, 0, i), synth.rpn_deltas(A, 0, i)
        x = synth.features(c["C"], c["feat_h"], c["feat_w"], 0, i)[None]
        bx, lb = synth.gt_boxes(c["img_h"], c["img_w"], 32, 0, i)
        v = lb != -1
        ts = time.perf_counter()
        rois, _ = orc.propose_one(anchors, sc, de, c["img_w"], c["img_h"], c["pre_nms"], c["post_nms"])
        orc.anchor_target(bx[v], anchors)
        s_roi = orc.proposal_target(rois, bx[v], lb[v])[0]
        boxes = orc.roi_transform(s_roi.astype(np.float32), np.zeros(len(s_roi), np.float32),
                                  c["img_h"], c["img_w"], c["feat_h"], c["feat_w"])
        _, am = orc.roi_pool_forward(x, boxes, 7, 1.0)
        orc.roi_pool_backward(g[:len(boxes)], boxes, am, x.shape)
        te = time.perf_counter()
        if warm:
            warm, t0 = False, te
            continue
        done += 1
        i += 1
        if te - t0 >= seconds:
            break
    el = time.perf_counter() - t0
    return {"value": done / el, "unit": "images/sec", "cores": 1, "kind": "port",
            "sample": f"{done} {cfg}-shaped training images, one at a time (oracle: numpy targets with "
                      f"the global MT19937 + 1-thread C nms/roi_pool fwd+bwd), after 1 warm-up image; "
                      f"{el:.1f} s on {os.cpu_count()}-cpu host"}


def make_streams(args, device):
    """(proposal stream, RoIPool stream).  --streams 1: both the current
    stream.  --prop-cus K: a CU partition -- K CUs for the latency-bound
    proposal layer (spread so that every XCD and every 8-CU block gets its
    share whichever way the mask bits map to XCDs), the rest for the pool."""
    if args.streams == 1:
        s = torch.cuda.current_stream()
        return s, s
    if args.prop_cus <= 0:
        n_prop = max(1, args.prop_streams)
        props = [torch.cuda.Stream() for _ in range(n_prop)]
        return (props if n_prop > 1 else props[0]), torch.cuda.Stream()
    from replication_faster_rcnn_amd import _lib
    n = _lib.cu_count()
    k = min(args.prop_cus, n // 2)
    prop = sorted({(j * 8 + (j % 8)) % n for j in range(k)})
    pool = [i for i in range(n) if i not in set(prop)]
    return _lib.cu_masked_stream(prop, device), _lib.cu_masked_stream(pool, device)


def inference_step_fn(args, c, sc, de, x, base, world, ev):
    """cfg1-4: propose -> (RCCL all-gather of detections) -> RoI transform +
    pack + RoIPool forward (nets/rpn.py:102-138, nets/heads.py:42-48)."""
    from replication_faster_rcnn_amd import ops
    from replication_faster_rcnn_amd import dist as fdist
    N, dev = sc.size(0), sc.device
    post = c["post_nms"]
    inds = torch.arange(N, device=dev, dtype=torch.float32).repeat_interleave(post)
    # streams=2: two HIP streams, step k+1's proposals beside step k's RoIPool
    # (measured: stream priorities change nothing; holding step k+1's proposals
    # until step k's pool is issued gives the pool the whole chip, 68 vs 75 us,
    # but costs 17 % of the throughput)
    s_props, s_pool = make_streams(args, dev)
    if not isinstance(s_props, list):
        s_props = [s_props]
    k_step = [0]
    if args.host_io:  # reference-style host tensors: inputs H2D, rois + pooled D2H per step
        h_in = [t.cpu().pin_memory() for t in (sc, de, x)]
        d_in = [[torch.empty_like(t) for t in (sc, de, x)] for _ in s_props]
        h_rois = torch.empty((N, post, 4), dtype=torch.float32).pin_memory()
        h_pool = torch.empty((N * post, x.size(1), 7, 7), dtype=torch.float32).pin_memory()
        done = [None] * len(s_props)

    def step(timed):
        j = k_step[0] % len(s_props)
        s_prop = s_props[j]
        k_step[0] += 1
        with torch.cuda.stream(s_prop):
            sc_, de_, x_ = sc, de, x
            if args.host_io:
                if done[j] is not None:
                    s_prop.wait_event(done[j])  # the pool that read d_in[j] last time
                for d, h in zip(d_in[j], h_in):
                    d.copy_(h, non_blocking=True)
                sc_, de_, x_ = d_in[j]
            rois, idx, cnt = ops.propose(sc_, de_, img_w=c["img_w"], img_h=c["img_h"],
                                         pre_nms=c["pre_nms"], post_nms=post, anchor_base=base,
                                         feat_h=c["feat_h"], feat_w=c["feat_w"])
            if world > 1:  # the only collective: detections of all ranks (RCCL over xGMI)
                fdist.all_gather_detections(rois, idx, cnt)
            if args.host_io:
                h_rois.copy_(rois, non_blocking=True)
            ready = torch.cuda.Event()
            ready.record(s_prop)
        with torch.cuda.stream(s_pool):
            s_pool.wait_event(ready)
            rois.record_stream(s_pool)  # allocated on s_prop, read on s_pool
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s_pool)
            # ResnetHead's transform + pack + roi_pool (nets/heads.py:42-48): one launch
            pooled, am, boxes = ops.roi_pool_head(x_, rois.view(-1, 4), inds, 7, c["img_h"], c["img_w"],
                                                  rois_sorted=True)
            if timed:
                e1.record(s_pool)
                ev["fwd"].append((e0, e1))
            if args.host_io:
                h_pool.copy_(pooled, non_blocking=True)
                done[j] = torch.cuda.Event()
                done[j].record(s_pool)
        return cnt
    return step


def inference_capi_fn(args, c, sc, de, x, base, world, ev):
    """cfg1-4, issued straight through the C-ABI (include/frcnn_capi.h) the way
    a native host would: parameters, device buffers and workspaces set up once,
    so a step is two library calls plus stream events (~40 us of host time vs
    ~88 us for the torch-op step, host_issue_us_per_step).  Measured (cfg2):
    the faster issue lets proposal chains run ahead beside the RoIPool, which
    then slows (90 vs 78 us) and the step is slower (110 vs 99 us) for 2, 4 or
    8 buffer sets and 2-4 proposal streams, so --issue ops stays the default.
    Same streams and overlap: step k's proposals on proposal stream k % P, its
    RoIPool on the pool stream after them; a proposal buffer is rewritten only
    after the pool that read it (event), so buffers are per proposal stream.
    HIP graphs were measured as the alternative: a replay serialises the
    captured branches and costs ~40 us of host time (126 us per step)."""
    import ctypes
    from replication_faster_rcnn_amd import _lib
    from replication_faster_rcnn_amd import dist as fdist
    lib = _lib.load()
    N, dev = sc.size(0), sc.device
    post = c["post_nms"]
    Cc, H, W = x.shape[1:]
    R = N * post
    s_props, s_pool = make_streams(args, dev)
    if not isinstance(s_props, list):
        s_props = [s_props]
    P = len(s_props)
    B = max(P, args.prop_buffers)  # proposal output sets: run-ahead of B-1 steps
    p = _lib.ProposeParams()
    p.N, p.A, p.K = N, sc.size(1), base.size(0)
    p.feat_h, p.feat_w, p.feat_stride = c["feat_h"], c["feat_w"], 16
    p.img_h, p.img_w, p.min_size = float(c["img_h"]), float(c["img_w"]), 16.0
    p.pre_nms, p.post_nms, p.iou_threshold = int(c["pre_nms"]), int(post), 0.7
    pref = ctypes.byref(p)
    ws_p = [_lib.workspace(lib.frcnn_propose_workspace_size(pref), dev) for _ in range(P)]
    bufs = [(torch.zeros((N, post, 4), dtype=torch.float32, device=dev),
             torch.full((N, post), -1, dtype=torch.int32, device=dev),
             torch.zeros((N,), dtype=torch.int32, device=dev)) for _ in range(B)]
    inds = torch.arange(N, device=dev, dtype=torch.float32).repeat_interleave(post)
    out = torch.empty((R, Cc, 7, 7), dtype=torch.float32, device=dev)
    am = torch.empty((R, Cc, 7, 7), dtype=torch.int32, device=dev)
    boxes = torch.empty((R, 5), dtype=torch.float32, device=dev)
    ws_r = _lib.workspace(lib.frcnn_roi_pool_fwd_workspace_size(R, N, Cc), dev)
    V = ctypes.c_void_p
    sp = [V(s.cuda_stream) for s in s_props]
    spool = V(s_pool.cuda_stream)
    prop_args = [(pref, V(sc.data_ptr()), V(de.data_ptr()), V(0), V(base.data_ptr()),
                  V(b[0].data_ptr()), V(b[1].data_ptr()), V(b[2].data_ptr()),
                  V(ws_p[i % P].data_ptr()), ws_p[i % P].numel(), sp[i % P])
                 for i, b in enumerate(bufs)]
    pool_args = [(V(x.data_ptr()), V(b[0].data_ptr()), V(inds.data_ptr()), R, N, Cc, H, W, 7, 7,
                  float(c["img_h"]), float(c["img_w"]), 1.0, 1, V(boxes.data_ptr()),
                  V(out.data_ptr()), V(am.data_ptr()), V(ws_r.data_ptr()), ws_r.numel(), spool)
                 for b in bufs]
    ready = [torch.cuda.Event() for _ in range(B)]
    done = [None] * B
    n_ev = args.steps + 1
    tev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(n_ev)]
    k = [0, 0]

    def step(timed):
        j = k[0] % B  # buffer set; stream k % P (B is a multiple of P)
        s = s_props[k[0] % P]
        k[0] += 1
        if done[j] is not None:
            s.wait_event(done[j])  # the pool that read bufs[j] last time
        _lib.check(lib.frcnn_propose(*prop_args[j]), "propose")
        if world > 1:  # the only collective: detections of all ranks (RCCL over xGMI)
            with torch.cuda.stream(s):
                fdist.all_gather_detections(*bufs[j])
        ready[j].record(s)
        s_pool.wait_event(ready[j])
        if timed:
            e0, e1 = tev[k[1] % n_ev]
            k[1] += 1
            e0.record(s_pool)
        _lib.check(lib.frcnn_roi_pool_fwd_head(*pool_args[j]), "roi_pool_head")
        if timed:
            e1.record(s_pool)
            ev["fwd"].append((e0, e1))
        if done[j] is None:
            done[j] = torch.cuda.Event()
        done[j].record(s_pool)
        return bufs[j][2]
    return step


def train_step_fn(args, c, sc, de, x, base, world, ev, first_image):
    """cfg5 (training step, train.py:59-127 minus the dense layers): propose
    (12000->600) -> anchor targets of every image -> proposal targets of every
    image (numpy's MT19937 stream kept on the device, sync-free, in the
    reference's order: all AT, then all PT) -> sampled RoIs fp64->fp32 ->
    RoI transform + pack + RoIPool forward -> RoIPool backward of a resident
    upstream gradient (the head's dL/dpool)."""
    from replication_faster_rcnn_amd import anchors as A, ops, synth, targets
    from replication_faster_rcnn_amd.utils import rng_state_to_device
    N, dev = sc.size(0), sc.device
    S = 128
    anchors = A.generate_anchors(base, 16, c["feat_w"], c["feat_h"]).to(dev)
    gl = [synth.gt_boxes(c["img_h"], c["img_w"], 32, 0, first_image + i) for i in range(N)]
    boxes = torch.from_numpy(np.stack([b for b, _ in gl])).to(dev)
    labels = torch.from_numpy(np.stack([l for _, l in gl])).to(dev)
    np.random.seed(0)
    rng, _ = rng_state_to_device(dev)
    inds = torch.arange(N, device=dev, dtype=torch.float32).repeat_interleave(S)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)
    grad = torch.randn((N * S, x.size(1), 7, 7), device=dev, generator=gen)
    s_prop, s_pool = make_streams(args, dev)
    if isinstance(s_prop, list):  # the device RNG stream orders steps: one proposal stream
        s_prop = s_prop[0]
    state = {}

    def step(timed):
        with torch.cuda.stream(s_prop):
            rois, _, cnt = ops.propose(sc, de, img_w=c["img_w"], img_h=c["img_h"],
                                       pre_nms=c["pre_nms"], post_nms=c["post_nms"],
                                       anchor_base=base, feat_h=c["feat_h"], feat_w=c["feat_w"])
            reg_t, lab = targets.anchor_targets(boxes, labels, anchors, rng=rng)
            s_roi, s_reg, s_lab, s_cnt = targets.proposal_targets(rois, cnt, boxes, labels,
                                                                  n_sample=S, rng=rng)
            sample_rois = s_roi.float().view(-1, 4)          # train.py:86,102,107
            ready = torch.cuda.Event()
            ready.record(s_prop)
        with torch.cuda.stream(s_pool):
            s_pool.wait_event(ready)
            sample_rois.record_stream(s_pool)
            if timed:
                e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                e[0].record(s_pool)
            pooled, am, bx = ops.roi_pool_head(x, sample_rois, inds, 7, c["img_h"], c["img_w"],
                                               rois_sorted=True)
            if timed:
                e[1].record(s_pool)
            gi = ops._roi_pool_bwd(grad, bx, am, tuple(x.shape), 1.0)
            if timed:
                e[2].record(s_pool)
                ev["fwd"].append((e[0], e[1]))
                ev["bwd"].append((e[1], e[2]))
        state.update(s_cnt=s_cnt, lab=lab, gi=gi)
        return s_cnt
    step.state = state
    return step


def main():
    args = parse()
    world, rank, local = setup_dist(args.gpus)
    dev = torch.device("cuda", local)
    from replication_faster_rcnn_amd import anchors as A
    from replication_faster_rcnn_amd import dist as fdist
    train = args.config == "cfg5"
    capi = args.issue == "capi" and not train
    if args.host_io and (capi or train):
        raise SystemExit("--host-io is measured on the inference ops path only")
    per_rank = c_batch(args.config)
    mine = fdist.shard(per_rank * world, rank, world)  # weak scaling: per_rank images per GPU
    c, sc, de, x = make_inputs(args.config, len(mine), mine.start, dev)
    N = sc.size(0)
    base = A.generate_anchor_base_device(anchor_scales=c["scales"])
    ev = {"fwd": [], "bwd": []}
    if train:
        step = train_step_fn(args, c, sc, de, x, base, world, ev, mine.start)
    else:
        step = (inference_capi_fn if capi else inference_step_fn)(args, c, sc, de, x, base, world, ev)

    for _ in range(args.warmup):
        cnt = step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        cnt = step(True)
    t_issue = time.perf_counter() - t0  # host time to enqueue the K steps
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    R = int(cnt.sum().item())
    if train and R != N * 128:  # train.py:102 assumes exactly 128 samples per image
        raise RuntimeError(f"proposal targets: {cnt.tolist()} samples per image, expected 128")
    C, H, W = x.shape[1:]
    alg_bytes = N * C * H * W * 4 + R * 20 + 2 * R * C * 49 * 4
    fwd_ms = float(np.mean([a.elapsed_time(b) for a, b in ev["fwd"]]))
    # the dominant kernel: RoIPool fwd (inference), RoIPool bwd (training step;
    # same algorithmic bytes: grad + argmax read, rois, grad_in written)
    dom_ms = float(np.mean([a.elapsed_time(b) for a, b in ev["bwd"]])) if train else fwd_ms
    achieved = alg_bytes / (dom_ms * 1e-3) / 1e9
    traffic = None
    tpath = os.path.join(ROOT, "profiles", "roi_pool_bwd_traffic.json" if train
                         else "roi_pool_fwd_traffic.json")
    if os.path.exists(tpath):
        traffic = json.load(open(tpath)).get(args.config, {}).get("hbm_bytes_per_launch")
    images = world * N * args.steps
    if train:
        workload = (f"{args.config}: training step, {N} images/GPU {c['img_h']}x{c['img_w']}, "
                    f"{c['feat_h']}x{c['feat_w']}x9 anchors, {c['pre_nms']}->{c['post_nms']} NMS@0.7, "
                    f"anchor targets vs 32 gt + proposal targets (128/img), RoIPool 7x7x{C} fwd+bwd")
    else:
        workload = (f"{args.config}: {N} VOC-shape images/GPU {c['img_h']}x{c['img_w']}, "
                    f"{c['feat_h']}x{c['feat_w']}x{3 * len(c['scales'])} anchors, "
                    f"{c['pre_nms']}->{c['post_nms']} NMS@0.7, RoIPool 7x7x{C}")
    rec = {
        "metric": "images/sec through RPN proposal+NMS+RoIPool; RoIPool HBM GB/s vs peak",
        "value": images / el, "unit": "images/sec", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
        "config": {"workload": workload, "global_batch": world * N,
                   "parallelism": f"dp{world} (per-image sharding)", "streams": args.streams,
                   "prop_streams": args.prop_streams if (args.streams == 2 and not train) else 1,
                   "issue": "capi" if capi else "ops",
                   "host_io": bool(args.host_io),
                   "prop_cus": args.prop_cus if args.streams == 2 else 0},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "roi_pool_bwd_kernel" if train else "roi_pool_fwd_px8q_kernel<head>",
                     "kernel_us": dom_ms * 1e3, "alg_bytes_per_launch": alg_bytes},
        "cpu_baseline": None,
        "host_issue_us_per_step": t_issue / args.steps * 1e6,
    }
    if train:
        rec["roofline"]["fwd_us"] = fwd_ms * 1e3
        rec["roofline"]["fwd_frac"] = alg_bytes / (fwd_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cb = cpu_baseline_train if train else cpu_baseline
        rec["cpu_baseline"] = cb(args.config, args.cpu_seconds)
        rec["cpu_baseline"]["gpu_over_cpu"] = rec["value"] / rec["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


def c_batch(cfg):
    from replication_faster_rcnn_amd import synth
    return synth.CONFIGS[cfg]["batch"]


if __name__ == "__main__":
    main()
