"""Save/load helpers for the golden fixtures in tests/golden/ (data only:
inputs and the oracle's outputs, written by tests/golden/make_golden.py)."""
import os
from dataclasses import fields

import numpy as np

from uasl_motion_estimation_amd import synthetic as S

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def path(name):
    return os.path.join(GOLDEN, name + ".npz")


def save(name, **arrays):
    np.savez_compressed(path(name), **{k: np.asarray(v) for k, v in arrays.items()})


def load(name):
    with np.load(path(name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def dataclass_arrays(prefix, obj):
    out = {}
    for f in fields(obj):
        v = getattr(obj, f.name)
        if v is not None:
            out[prefix + f.name] = np.asarray(v)
    return out


def _restore(cls, prefix, d):
    kw = {}
    for f in fields(cls):
        k = prefix + f.name
        if k in d:
            v = d[k]
            kw[f.name] = v.item() if v.ndim == 0 else v.copy()
    return cls(**kw)


def scale_problem(d, prefix="sp_"):
    return _restore(S.ScaleProblem, prefix, d)


def ba_problem(d, prefix="bp_"):
    return _restore(S.BAProblem, prefix, d)
