"""Ray-image gradient (mirror of mast3r_slam/image.py:5-38).

The reference convolves each channel with the 3x3 kernels
``gx = [[-3,0,3],[-10,0,10],[-3,0,3]] / 32`` and ``gy = gx^T`` after a 1-pixel
reflect pad.  Here the same stencil is written as shifted-slice arithmetic so it runs
identically on any device (values agree with the reference conv2d to float rounding;
see tests/test_glue_golden.py).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def img_gradient(img: torch.Tensor):
    """img [b,c,h,w] -> (gx, gy), each [b,c,h,w]."""
    p = F.pad(img, (1, 1, 1, 1), mode="reflect")
    h, w = img.shape[-2:]

    def win(dy, dx):  # p[..., 1+dy : 1+dy+h, 1+dx : 1+dx+w]
        return p[..., 1 + dy : 1 + dy + h, 1 + dx : 1 + dx + w]

    a = 3.0 / 32.0
    b = 10.0 / 32.0
    gx = a * (win(-1, 1) - win(-1, -1)) + b * (win(0, 1) - win(0, -1)) + a * (win(1, 1) - win(1, -1))
    gy = a * (win(1, -1) - win(-1, -1)) + b * (win(1, 0) - win(-1, 0)) + a * (win(1, 1) - win(-1, 1))
    return gx, gy
