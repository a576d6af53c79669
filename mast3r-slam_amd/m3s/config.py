"""Hot-path parameters of the reference configuration (values only).

Source: /root/reference/config/base.yaml:8-14 (matching), :16-33 (tracking), :35-50 (local_opt);
calib.yaml:1-6 switches ``use_calib`` on.  ``load_config`` reads the reference's YAML
format (``inherit:`` chaining, floats like ``1e-8``) with a SafeLoader, like
mast3r_slam/config.py:7-48.
"""
from __future__ import annotations

import copy
import re

import yaml

DEFAULT_CONFIG = {
    "use_calib": False,
    "matching": {
        "max_iter": 10,
        "lambda_init": 1e-8,
        "convergence_thresh": 1e-6,
        "dist_thresh": 1e-1,
        "radius": 3,
        "dilation_max": 5,
    },
    "tracking": {  # base.yaml:16-33
        "min_match_frac": 0.05,
        "max_iters": 50,
        "C_conf": 0.0,
        "Q_conf": 1.5,
        "rel_error": 1e-3,
        "delta_norm": 1e-3,
        "huber": 1.345,
        "match_frac_thresh": 0.333,
        "sigma_ray": 0.003,
        "sigma_dist": 1e1,
        "sigma_pixel": 1.0,
        "sigma_depth": 1e1,
        "sigma_point": 0.05,
        "pixel_border": -10,
        "depth_eps": 1e-6,
        "filtering_mode": "weighted_pointmap",
        "filtering_score": "median",
    },
    "local_opt": {
        "pin": 1,
        "window_size": 1e6,
        "C_conf": 0.0,
        "Q_conf": 1.5,
        "min_match_frac": 0.1,
        "pixel_border": -10,
        "depth_eps": 1e-6,
        "max_iters": 10,
        "sigma_ray": 0.003,
        "sigma_dist": 1e1,
        "sigma_pixel": 1.0,
        "sigma_depth": 1e1,
        "sigma_point": 0.05,
        "delta_norm": 1e-8,
        "use_cuda": True,
    },
}

config = copy.deepcopy(DEFAULT_CONFIG)

_FLOAT_RE = re.compile(
    r"""^(?:[-+]?(?:[0-9][0-9_]*)\.[0-9_]*(?:[eE][-+]?[0-9]+)?
        |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
        |\.[0-9_]+(?:[eE][-+][0-9]+)?
        |[-+]?\.(?:inf|Inf|INF)
        |\.(?:nan|NaN|NAN))$""",
    re.X,
)


class _Loader(yaml.SafeLoader):
    pass


_Loader.add_implicit_resolver("tag:yaml.org,2002:float", _FLOAT_RE, list("-+0123456789."))


def _merge(dst, src):
    for k, v in src.items():
        if isinstance(v, dict):
            dst.setdefault(k, {})
            _merge(dst[k], v)
        else:
            dst[k] = v
    return dst


def load_config(path, base_dir=None):
    """Load a reference-style YAML (with ``inherit:``) into the module-level ``config``."""
    import os

    def _load(p):
        full = p if os.path.isabs(p) or base_dir is None else os.path.join(base_dir, p)
        with open(full) as f:
            cfg = yaml.load(f, Loader=_Loader) or {}
        parent = cfg.pop("inherit", None)
        out = _load(parent) if parent else {}
        return _merge(out, cfg)

    cfg = _load(path)
    _merge(config, cfg)
    return config
