"""One GN call per bench config with M3S_PCG_DEBUG=1 (PCG phase clocks on stderr) and the
call's PCG counters.  python tools/r06/pcg_debug.py [cfg3|cfg4 ...]"""
import os, sys
os.environ.setdefault("M3S_PCG_DEBUG", "1")
os.environ["M3S_GN_DEBUG_FLAGS"] = "2"
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]
import torch
import mast3r_slam_backends as mb
from m3s import synth
from m3s.geometry import constrain_points_to_ray
L = dict(sigma_ray=0.003, sigma_dist=10.0, sigma_pixel=1.0, sigma_depth=10.0, C_conf=0.0, Q_conf=1.5,
         pixel_border=-10, depth_eps=1e-6)
for cfg in (sys.argv[1:] or ["cfg3", "cfg4"]):
    g = synth.make_graph(cfg, device="cuda")
    mode = synth.CONFIGS[cfg]["mode"]
    if mode == "calib":
        g.Xs = constrain_points_to_ray((g.H, g.W), g.Xs, g.K).contiguous()
    for rep in range(2):
        T = g.Twc.clone()
        print(f"== {cfg} call {rep}", file=sys.stderr, flush=True)
        if mode == "calib":
            mb.gauss_newton_calib(T, g.Xs, g.Cs, g.K, g.ii, g.jj, g.idx, g.valid, g.Q, g.H, g.W, L["pixel_border"],
                                  L["depth_eps"], L["sigma_pixel"], L["sigma_depth"], L["C_conf"], L["Q_conf"], 10, 0.0)
        else:
            mb.gauss_newton_rays(T, g.Xs, g.Cs, g.ii, g.jj, g.idx, g.valid, g.Q, L["sigma_ray"], L["sigma_dist"],
                                 L["C_conf"], L["Q_conf"], 10, 0.0)
        torch.cuda.synchronize()
        mb.gn_check()
        print(cfg, mb.gn_debug_flags(), file=sys.stderr, flush=True)
    del g
    torch.cuda.empty_cache()
