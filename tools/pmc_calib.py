"""PMC calibration (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE): torch kernels with KNOWN byte
counts in the access shapes of the GN accumulate kernel.  Run under rocprofv3; compare the
counters with the printed byte counts (MI355X_MICROARCH.md §HBM asks for exactly this)."""
import torch

n = 1 << 28  # 1 GiB of f32
x = torch.ones(n, device="cuda")
torch.cuda.synchronize()
s = x.sum()                       # coalesced wide stream, 1 GiB read
y = x.view(-1, 4)[:, :3].contiguous()  # 0.75 GiB read (strided), 0.75 GiB written
idx = torch.arange(y.shape[0], device="cuda")
idx = (idx & ~63) | ((idx * 37 + 11) & 63)  # local permutation (flow-like gather)
g = y.index_select(0, idx)        # 12-B record gather: 0.75 GiB read (+ idx 0.5 GiB), 0.75 GiB written
torch.cuda.synchronize()
print("sum bytes", n * 4, "contig_copy read", y.numel() * 4 * 4 // 3, "write", y.numel() * 4,
      "gather read", y.numel() * 4, "+ idx", idx.numel() * 8, "write", g.numel() * 4, float(s))
