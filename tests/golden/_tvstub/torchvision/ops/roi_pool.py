import numpy as np
import torch

from oracle import ref_numpy as _o

CALLS = []


def roi_pool(input, boxes, output_size, spatial_scale=1.0):
    x = input.detach().cpu().numpy().astype(np.float32)
    b = boxes.detach().cpu().numpy().astype(np.float32)
    out, am = _o.roi_pool_forward(x, b, output_size, spatial_scale)
    CALLS.append(("roi_pool", x, b, out, am))
    return torch.from_numpy(out)
