"""Probe (GPU box): torch's F.normalize / reflect-pad conv2d gradient / linalg.norm outputs on
cuda for random inputs, saved for host-side comparison with candidate float orders
(the fused matching prep must reproduce them bitwise)."""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mast3r-slam_amd"))
from m3s.image import img_gradient  # noqa: E402

g = torch.Generator().manual_seed(0)
X = (torch.randn((2, 48, 64, 3), generator=g) * torch.rand((2, 48, 64, 1), generator=g) * 3).cuda()
Y = torch.randn((2, 48 * 64, 3), generator=g).cuda()
rays = F.normalize(X, dim=-1)
gx, gy = img_gradient(rays.permute(0, 3, 1, 2))
nrm = torch.linalg.norm(X - Y.view(2, 48, 64, 3), dim=-1)
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/probe_glue.npz", X=X.cpu().numpy(), Y=Y.cpu().numpy(), rays=rays.cpu().numpy(),
         gx=gx.cpu().numpy(), gy=gy.cpu().numpy(), nrm=nrm.cpu().numpy())
print("ok", torch.__version__, torch.backends.cudnn.enabled)
