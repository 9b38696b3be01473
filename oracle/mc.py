"""CPU ORACLE for the marching-cubes extractor -- TEST INFRASTRUCTURE.

Only ``tests/`` may import this module, as the checker of ``csrc/mesh.hip``
(``sdfr_mc_count`` / ``sdfr_mc_emit``); the product path never falls back to it.

A numpy restatement of the same algorithm: inside = value < level; one vertex
per sign-changing grid edge by linear interpolation in fp32
(t = (level - v_a) / (v_b - v_a), x = i + t); the cell's triangles from the case
table that ``sdface-gan_amd/csrc/mc_table_gen.py`` derives; vertex ids
edge-major (axis, then point index), triangles in cell order then table order.

Parity: UNPINNED against the reference.  The reference's extractor is
scikit-image's ``marching_cubes(sdf_vol, 0)`` (sdf_utils.py:195, Lewiner
tables), which this image does not ship and no reference fixture holds; this
oracle pins the HIP kernel bit for bit to the documented algorithm, and
``tests/test_mesh.py`` checks the algorithm's properties (closed, consistently
oriented surfaces; vertices on the zero crossing) instead.
"""
from __future__ import annotations

import importlib.util
from pathlib import Path

import numpy as np

_GEN = Path(__file__).resolve().parents[1] / "sdface-gan_amd" / "csrc" / "mc_table_gen.py"
_table = None


def table_module():
    spec = importlib.util.spec_from_file_location("mc_table_gen", _GEN)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def table():
    global _table
    if _table is None:
        _table = table_module().build_table()
    return _table


# local edge -> (axis, dx, dy, dz) of its low end (mc_table_gen.py numbering)
EDGE_LOW = np.array([(0, 0, e & 1, e >> 1) for e in range(4)]
                    + [(1, e & 1, 0, e >> 1) for e in range(4)]
                    + [(2, e & 1, e >> 1, 0) for e in range(4)], np.int64)


def marching_cubes(vol, level=0.0):
    """(verts [V, 3] float32 in index coordinates, faces [F, 3] int64)."""
    vol = np.asarray(vol, np.float32)
    n0, n1, n2 = vol.shape
    N = vol.size
    lvl = np.float32(level)
    inside = vol < lvl
    S = np.zeros(4 * N, np.int64)
    flags = []
    for d in range(3):
        f = np.zeros(vol.shape, bool)
        a = [slice(None)] * 3
        b = [slice(None)] * 3
        a[d], b[d] = slice(0, -1), slice(1, None)
        f[tuple(a)] = inside[tuple(a)] != inside[tuple(b)]
        flags.append(f)
        S[d * N:(d + 1) * N] = f.ravel()
    tri, ntri = table()
    cs = np.zeros((n0 - 1, n1 - 1, n2 - 1), np.int64)
    for c in range(8):
        x, y, z = c & 1, (c >> 1) & 1, c >> 2
        cs |= inside[x:n0 - 1 + x, y:n1 - 1 + y, z:n2 - 1 + z].astype(np.int64) << c
    cell_case = np.zeros(vol.shape, np.int64)
    cell_case[:-1, :-1, :-1] = cs
    cell_nt = ntri[cell_case].astype(np.int64)
    cell_nt[-1, :, :] = 0
    cell_nt[:, -1, :] = 0
    cell_nt[:, :, -1] = 0
    S[3 * N:] = cell_nt.ravel()
    ex = np.concatenate([[0], np.cumsum(S)])[:-1]

    nv = int(ex[3 * N])
    verts = np.zeros((nv, 3), np.float32)
    grid = np.indices(vol.shape).reshape(3, -1)
    for d in range(3):
        p = np.flatnonzero(flags[d].ravel())
        i, j, k = grid[:, p]
        va = vol.ravel()[p]
        q = [i, j, k]
        q[d] = q[d] + 1
        vb = vol[q[0], q[1], q[2]]
        t = (lvl - va) / (vb - va)
        pos = np.stack([i, j, k], 1).astype(np.float32)
        pos[:, d] = pos[:, d] + t
        verts[ex[d * N + p]] = pos

    cells = np.flatnonzero(cell_nt.ravel())
    nt = cell_nt.ravel()[cells]
    cell_rep = np.repeat(cells, nt)
    t_in_cell = np.arange(len(cell_rep)) - np.repeat(np.cumsum(nt) - nt, nt)
    case_rep = cell_case.ravel()[cell_rep]
    faces = np.zeros((len(cell_rep), 3), np.int64)
    for r in range(3):
        e = tri[case_rep, 3 * t_in_cell + r].astype(np.int64)
        d, dx, dy, dz = EDGE_LOW[e].T
        q = cell_rep + dx * n1 * n2 + dy * n2 + dz
        faces[:, r] = ex[d * N + q]
    return verts, faces
