"""Print a bench config's directed edge list for tools/plan_bench.cpp: "N E" then "ii jj" lines
(the op's ii/jj: m3s.synth.make_graph's forward half then backward half)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mast3r-slam_amd"))
from m3s import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg4"
spec = synth.CONFIGS[cfg]
seed = {"cfg1": 1, "cfg2": 2, "cfg3": 3, "cfg4": 4}[cfg]
und = synth.make_edges(spec["N"], spec["E"], seed)
ii = [a for a, b in und] + [b for a, b in und]
jj = [b for a, b in und] + [a for a, b in und]
print(spec["N"], len(ii))
for a, b in zip(ii, jj):
    print(a, b)
