"""Time the RPN head epilogue (nets/rpn.py:117-124): the one-launch HIP kernel
(ops.rpn_head_epilogue) vs the reference's torch chain on the same device
(permute/contiguous, softmax, slice/contiguous, permute/contiguous).

Prints one JSON line per config: us per call, algorithmic bytes
(6K*H*W*4 read + 7K*H*W*4 written per image) and achieved GB/s.
"""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from replication_faster_rcnn_amd import ops  # noqa: E402

CONFIGS = {"cfg2": (8, 9, 38, 63), "cfg4": (1, 15, 50, 84), "cfg5": (16, 9, 38, 38),
           "cfg3_dp1": (64, 9, 38, 63)}


def torch_chain(cls, reg, n):
    c = cls.permute(0, 2, 3, 1).contiguous().view(n, -1, 2)
    fg = F.softmax(c, dim=-1)[:, :, 1].contiguous().view(n, -1)
    r = reg.permute(0, 2, 3, 1).contiguous().view(n, -1, 4)
    return c, fg, r


def timeit(fn, iters=200):
    for _ in range(20):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    for name, (N, K, H, W) in CONFIGS.items():
        cls = torch.randn(N, 2 * K, H, W, device="cuda")
        reg = torch.randn(N, 4 * K, H, W, device="cuda")
        with torch.no_grad():
            us_k = timeit(lambda: ops.rpn_head_epilogue(cls, reg, K))
            us_t = timeit(lambda: torch_chain(cls, reg, N))
        alg = N * 13 * K * H * W * 4
        print(json.dumps({"config": name, "N": N, "K": K, "H": H, "W": W,
                          "kernel_us": round(us_k, 2), "torch_chain_us": round(us_t, 2),
                          "alg_bytes": alg, "kernel_GBps": round(alg / us_k / 1e3, 1),
                          "speedup": round(us_t / us_k, 2)}), flush=True)


if __name__ == "__main__":
    main()
