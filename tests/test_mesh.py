"""Marching cubes on the CPU: the generated case table, the numpy oracle's
surfaces (closed, consistently oriented, vertices on the zero crossing) and the
.obj writer.  Parity against the reference's extractor (scikit-image's
marching_cubes, sdf_utils.py:195) is UNPINNED: scikit-image is not in this image
and no reference fixture holds a mesh; these are the algorithm's own properties.
The HIP kernels are compared with this oracle bit for bit in test_gpu_mesh.py."""
from collections import Counter

import numpy as np
import pytest

from oracle import mc


def _closed_and_oriented(faces):
    """Every undirected edge in exactly two triangles, traversed once each way."""
    directed = Counter()
    for a, b, c in faces.tolist():
        for u, v in ((a, b), (b, c), (c, a)):
            directed[(u, v)] += 1
    assert all(n == 1 for n in directed.values()), "a directed edge is used twice"
    missing = [e for e in directed if (e[1], e[0]) not in directed]
    assert not missing, f"{len(missing)} boundary edges (cracks)"


def _euler(verts, faces):
    edges = {tuple(sorted(e)) for f in faces.tolist() for e in ((f[0], f[1]), (f[1], f[2]), (f[2], f[0]))}
    return len(verts) - len(edges) + len(faces)


def _signed_volume(verts, faces):
    a, b, c = (verts[faces[:, r]].astype(np.float64) for r in range(3))
    return float(np.einsum("ij,ij->i", a, np.cross(b, c)).sum() / 6.0)


def test_table_header_is_generated():
    gen = mc.table_module()
    with open(mc._GEN.parent / "mc_table.h") as f:
        assert f.read() == gen.header_text(), "mc_table.h is stale: rerun csrc/mc_table_gen.py"
    tri, ntri = mc.table()
    assert ntri[0] == ntri[255] == 0 and ntri.max() == gen.MAX_TRI
    # complementary cases cross the same edges
    for case in range(256):
        edges = {e for e in tri[case] if e >= 0}
        comp = {e for e in tri[255 - case] if e >= 0}
        assert edges == comp, case


@pytest.mark.parametrize("case", range(1, 255))
def test_every_case_closes(case):
    """One cell's corners set by the case inside a volume whose border is outside:
    the surface around the inside corners is closed and oriented outward."""
    vol = np.ones((4, 4, 4), np.float32)
    for c in range(8):
        if (case >> c) & 1:
            vol[1 + (c & 1), 1 + ((c >> 1) & 1), 1 + (c >> 2)] = -1.0
    verts, faces = mc.marching_cubes(vol, 0.0)
    _closed_and_oriented(faces)
    assert _signed_volume(verts, faces) > 0


def test_random_volumes_are_crack_free():
    rng = np.random.default_rng(0)
    for shape in ((9, 7, 11), (12, 12, 12), (5, 16, 6)):
        vol = rng.standard_normal(shape).astype(np.float32)
        vol[[0, -1], :, :] = vol[:, [0, -1], :] = 1.0
        vol[:, :, [0, -1]] = 1.0
        verts, faces = mc.marching_cubes(vol, 0.0)
        _closed_and_oriented(faces)
        assert _signed_volume(verts, faces) > 0        # encloses the inside points


def test_sphere_properties():
    n, r = 48, 17.3
    g = np.indices((n, n, n)).astype(np.float32) - (n - 1) / 2
    vol = (np.sqrt((g ** 2).sum(0)) - r).astype(np.float32)
    verts, faces = mc.marching_cubes(vol, 0.0)
    _closed_and_oriented(faces)
    assert _euler(verts, faces) == 2
    rad = np.linalg.norm(verts - (n - 1) / 2, axis=1)
    assert np.abs(rad - r).max() < 0.05                # linear interpolation of a distance field
    assert abs(_signed_volume(verts, faces) / (4 / 3 * np.pi * r ** 3) - 1) < 0.01
    assert len(np.unique(verts, axis=0)) == len(verts)


def test_vertices_on_the_level_crossing():
    rng = np.random.default_rng(1)
    vol = rng.standard_normal((10, 9, 8)).astype(np.float32)
    level = 0.25
    verts, _ = mc.marching_cubes(vol, level)
    idx = np.floor(verts).astype(int)
    frac = verts - idx
    for v, i, f in zip(verts, idx, frac):
        d = int(np.argmax(f))
        lo = tuple(i)
        hi = list(i)
        hi[d] += 1
        va, vb = vol[lo], vol[tuple(hi)]
        assert (va < level) != (vb < level)
        assert abs(va + f[d] * (vb - va) - level) <= 1e-5 * max(1.0, abs(va), abs(vb))


def test_obj_export_roundtrip(sdfr, tmp_path):
    verts = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1]], np.float32) * 0.12
    faces = np.array([[0, 2, 1], [0, 1, 3], [0, 3, 2], [1, 2, 3]])
    m = sdfr.Mesh(verts, faces)
    path = tmp_path / "m.obj"
    with open(path, "w") as f:
        m.export(f, file_type="obj")
    v, fs = [], []
    for line in path.read_text().splitlines():
        tag, *rest = line.split()
        (v if tag == "v" else fs).append([float(x) if tag == "v" else int(x) for x in rest])
    np.testing.assert_allclose(np.array(v), verts, atol=5e-9)
    np.testing.assert_array_equal(np.array(fs) - 1, faces)
    with pytest.raises(ValueError):
        m.export(file_type="ply")
