"""m3s -- host-side mirror of the reference's callers of the backend hot path.

* ``m3s.matching`` / ``m3s.image``  -- ``mast3r_slam/matching.py`` + ``image.py`` (row a3)
* ``m3s.geometry``                  -- ``constrain_points_to_ray`` / ``backproject``
* ``m3s.global_opt``                -- ``FactorGraph.solve_GN_rays/calib`` flow (row a13)
* ``m3s.dist``                      -- edge-sharded multi-GPU GN (RCCL all-gather of per-edge records)
* ``m3s.synth``                     -- deterministic synthetic 512x384 workloads
* ``m3s.config``                    -- the hot-path parameters of config/base.yaml
"""
import os
import sys

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG_ROOT not in sys.path:
    sys.path.insert(0, _PKG_ROOT)
