"""Golden-vector helpers shared by the CPU and GPU parity tests."""
import ast
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ("mixture_L1", "mixture_L3_T", "mixture_L3_proj", "super_L3", "ctf_L1")
STATE_KEYS = ("muu", "muv", "sigu", "sigv", "pn", "rou", "w", "alpha")


def load(name):
    d = dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))
    d["opts"] = ast.literal_eval(str(d["opts"]))
    return d


def state(d, prefix="init_"):
    return {k: np.array(d[prefix + k], order="F", copy=True) for k in STATE_KEYS}
