"""Ray-image gradient (mirror of mast3r_slam/image.py:5-38).

Same arithmetic as the reference: a depthwise ``F.conv2d`` with the 3x3 kernels
``(1/32) * [[-3,0,3],[-10,0,10],[-3,0,3]]`` and its transpose (built in the input dtype, the
1/32 scaling applied to the kernel tensor, not the output) on a 1-pixel reflect pad, so the
result is bitwise the reference's on the same device (tests/test_glue_golden.py).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

_GX = ((-3.0, 0.0, 3.0), (-10.0, 0.0, 10.0), (-3.0, 0.0, 3.0))
_GY = ((-3.0, -10.0, -3.0), (0.0, 0.0, 0.0), (3.0, 10.0, 3.0))


def _stencil(rows, c, img):
    k = (1.0 / 32.0) * torch.tensor(rows, device=img.device, dtype=img.dtype)
    return k.repeat(c, 1, 1, 1)  # [c,1,3,3], one filter per channel (groups=c)


def img_gradient(img: torch.Tensor):
    """img [b,c,h,w] -> (gx, gy), each [b,c,h,w]."""
    c = img.shape[1]
    padded = F.pad(img, (1, 1, 1, 1), mode="reflect")
    gx = F.conv2d(padded, _stencil(_GX, c, img), groups=c)
    gy = F.conv2d(padded, _stencil(_GY, c, img), groups=c)
    return gx, gy
