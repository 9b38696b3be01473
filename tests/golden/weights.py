"""Deterministic parameter values for the golden fixtures (test infrastructure).

Every parameter / buffer of a Generator state dict (reference key names, see
SURVEY.md §8b) gets U[lo,hi) values from ``oracle.det_uniform`` (an integer
hash of the flat index, so identical on any host) with ranges that follow the
reference's own init scales (sdf_model.py:23-69, 437-466, 541-701, grid.py:136-140),
except the hash table, which uses U(-1,1) so index errors cannot hide behind
the reference's tiny U(-1e-4,1e-4) init.  ``table_amp`` selects another table
amplitude: the reference's own init scale (1e-4) and a trained-like one (0.05)
pin the split-fp16 field kernel at the operand scales it meets in practice.
"""
from __future__ import annotations

import math
import zlib

import numpy as np
import torch

from oracle.oracle import det_uniform

KAIMING_LRELU_STD = math.sqrt(2.0 / (1 + 0.2 ** 2))   # kaiming_normal_(a=0.2) gain


def name_seed(name: str) -> int:
    return zlib.crc32(name.encode()) & 0x7FFFFFFF


def det_table(rows, cols, seed=7, amp=1.0):
    return det_uniform((rows, cols), -amp, amp, seed)


def _u(std):
    a = std * math.sqrt(3.0)
    return (-a, a)


def init_range(name: str, shape):
    """(lo, hi) for a state-dict entry, or None to keep its constructed value."""
    if name.endswith("offsets") or name.endswith(".kernel"):
        return None
    if name.endswith("sigmoid_beta"):
        return None
    if name.endswith("encoder.embeddings"):
        return (-1.0, 1.0)
    fan_in = shape[-1] if len(shape) >= 2 else None
    if name.startswith("renderer."):
        if name.endswith("gamma.weight") or name.endswith("beta.weight"):
            return _u(0.25 * KAIMING_LRELU_STD / math.sqrt(fan_in))
        if name.endswith("gamma.bias") or name.endswith("beta.bias"):
            return (-1 / 16, 1 / 16)
        if name.endswith("pts_linears.0.weight") and shape[-1] in (256, 3):
            return (-1 / 3, 1 / 3)          # FiLMSiren(is_first=True), ngp and siren
        if name.endswith(".weight"):
            a = math.sqrt(6 / fan_in) / 25
            return (-a, a)
        if name.endswith(".bias"):
            n = {"input_linear": 32, "views_linears": 272}
            for k, v in n.items():
                if k in name:
                    return (-1 / math.sqrt(v), 1 / math.sqrt(v))
            return (-1 / 16, 1 / 16)
    if name.startswith("style."):
        if name.endswith(".weight"):
            return _u(KAIMING_LRELU_STD / math.sqrt(fan_in))
        return (-1 / 16, 1 / 16)
    if name.startswith("decoder."):
        if name.startswith("decoder.style.") and name.endswith(".weight"):
            return _u(100.0)             # randn / lr_mul(0.01), sdf_model.py:584
        if name.startswith("decoder.style.") and name.endswith(".bias"):
            return (-1.0, 1.0)
        if name.endswith("modulation.bias"):
            return (0.9, 1.1)
        if "noises.noise_" in name or name.endswith(".weight") and len(shape) >= 2:
            return _u(1.0)
        if name.endswith("noise.weight"):
            return (-0.1, 0.1)
        if name.endswith("bias"):
            return (-0.1, 0.1)
    return None


@torch.no_grad()
def det_init_(module: torch.nn.Module, table_amp=1.0):
    sd = module.state_dict()
    for name in sorted(sd.keys()):
        t = sd[name]
        if not torch.is_floating_point(t):
            continue
        rng = init_range(name, tuple(t.shape))
        if rng is None:
            continue
        if name.endswith("encoder.embeddings"):
            v = det_table(t.shape[0], t.shape[1], seed=7, amp=table_amp)
        else:
            v = det_uniform(tuple(t.shape), rng[0], rng[1], name_seed(name))
        t.copy_(torch.from_numpy(v).reshape(t.shape))
    return module


def det_state_dict(entries, prefix="", table_amp=1.0):
    """Build {name: tensor} for (name, shape) entries without any module.

    Keys whose value is fixed at construction get it here: the grid offsets
    (grid.py:117-128) and sigmoid_beta = 0.1 (sdf_model.py:164).  Entries that
    keep their constructed value otherwise (blur kernels) are skipped.
    """
    from oracle.oracle import grid_offsets
    sd = {}
    for name, shape in entries:
        if not name.startswith(prefix):
            continue
        if name.endswith("encoder.offsets"):
            sd[name] = torch.from_numpy(grid_offsets()[0])
        elif name.endswith("sigmoid_beta"):
            sd[name] = torch.full(tuple(shape), 0.1)
        elif name.endswith("encoder.embeddings"):
            sd[name] = torch.from_numpy(det_table(shape[0], shape[1], seed=7, amp=table_amp))
        else:
            rng = init_range(name, tuple(shape))
            if rng is None:
                continue
            sd[name] = torch.from_numpy(det_uniform(tuple(shape), rng[0], rng[1],
                                                    name_seed(name))).reshape(tuple(shape))
    return sd


def golden_entries(golden_dir, siren=False, kind=None):
    """(name, shape) of the reference Generator's state dict: the ngp one, or with
    siren=True / kind="siren" the SirenGenerator renderer's, kind="fc" the
    FCGenerator renderer's (both full_pipeline=False)."""
    import ast
    kind = kind or ("siren" if siren else "ngp")
    fname = {"ngp": "state_dict_keys.npz", "siren": "state_dict_keys_siren.npz",
             "fc": "state_dict_keys_fc.npz"}[kind]
    z = np.load(golden_dir / fname)
    return [ast.literal_eval(str(e)) for e in z["entries"]]
