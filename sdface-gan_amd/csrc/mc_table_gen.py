"""Generates mc_table.h: the marching-cubes case table of csrc/mesh.hip.

The reference extracts the zero level set with scikit-image's marching_cubes
(sdf_utils.py:195; Lewiner's tables).  scikit-image is not in this image and its
tables are not restated here; instead the 256 cases are DERIVED from one rule,
so the table is checkable and the mesh is crack-free by construction:

  * corner c = x + 2y + 4z of a cell is "inside" when its value < level;
  * on each of the 6 cell faces the iso-contour is 0, 1 or 2 segments between
    the crossed face edges; a face whose inside corners sit on a diagonal
    (4 crossings) takes two segments that cut off the INSIDE corners.  The
    choice depends only on the face's four corners, which the neighbouring cell
    shares, so both cells cut that face the same way (no cracks);
  * each segment is oriented t = g x n (g: in-face direction from the inside to
    the outside corners, n: the face's outward normal); the segments then chain
    into closed loops through the crossed edges, each loop is one polygon of the
    surface, wound counter-clockwise about the normal that points to increasing
    values (outward for an SDF), and it is fanned into triangles from its first
    edge.

Edge numbering (local edge -> (axis, corner offset of its lower end)):
  0-3   axis 0, (y, z) = (e & 1, e >> 1)
  4-7   axis 1, (x, z) = (e & 1, e >> 1)   (e - 4)
  8-11  axis 2, (x, y) = (e & 1, e >> 1)   (e - 8)

    python mc_table_gen.py            # rewrites mc_table.h next to this file
"""
from __future__ import annotations

import os

import numpy as np

MAX_TRI = 5          # checked by build_table()


def corner_pos(c):
    return np.array([c & 1, (c >> 1) & 1, (c >> 2) & 1], np.float64)


def edges():
    """[(axis, corner_a, corner_b)] for the 12 local edges; corner_a is the lower end."""
    out = []
    for axis in range(3):
        u, v = (axis + 1) % 3, (axis + 2) % 3
        lo, hi = (u, v) if u < v else (v, u)     # the two other axes, ascending
        for e in range(4):
            p = [0, 0, 0]
            p[lo], p[hi] = e & 1, e >> 1
            a = p[0] + 2 * p[1] + 4 * p[2]
            out.append((axis, a, a + (1 << axis)))
    return out


EDGES = edges()
EDGE_OF = {frozenset((a, b)): i for i, (_, a, b) in enumerate(EDGES)}


def faces():
    """[(outward normal, [4 corners in cyclic order])] for the 6 cell faces."""
    out = []
    for axis in range(3):
        u, v = (axis + 1) % 3, (axis + 2) % 3
        for side in (0, 1):
            cs = []
            for (a, b) in ((0, 0), (1, 0), (1, 1), (0, 1)):
                p = [0, 0, 0]
                p[axis], p[u], p[v] = side, a, b
                cs.append(p[0] + 2 * p[1] + 4 * p[2])
            n = np.zeros(3)
            n[axis] = 1.0 if side else -1.0
            out.append((n, cs))
    return out


FACES = faces()


def _mid(e):
    _, a, b = EDGES[e]
    return 0.5 * (corner_pos(a) + corner_pos(b))


def case_segments(case):
    """Oriented face segments (edge_from, edge_to) of one case."""
    inside = [(case >> c) & 1 == 1 for c in range(8)]
    segs = []
    for n, cs in FACES:
        ins = [c for c in cs if inside[c]]
        if len(ins) in (0, 4):
            continue
        ring = [EDGE_OF[frozenset((cs[i], cs[(i + 1) % 4]))] for i in range(4)]
        crossed = [ring[i] for i in range(4) if inside[cs[i]] != inside[cs[(i + 1) % 4]]]
        centre = np.mean([corner_pos(c) for c in cs], 0)
        if len(crossed) == 2:
            outs = [c for c in cs if not inside[c]]
            g = np.mean([corner_pos(c) for c in outs], 0) - np.mean([corner_pos(c) for c in ins], 0)
            pairs = [(crossed, g)]
        else:                                    # diagonal: cut off each inside corner
            pairs = []
            for c in ins:
                es = [e for e in crossed if c in EDGES[e][1:]]
                pairs.append((es, centre - corner_pos(c)))
        for (e0, e1), g in pairs:
            t = np.cross(g, n)
            if np.dot(_mid(e1) - _mid(e0), t) > 0:
                segs.append((e0, e1))
            else:
                segs.append((e1, e0))
    return segs


def case_loops(case):
    segs = case_segments(case)
    nxt = {}
    for a, b in segs:
        assert a not in nxt, (case, segs)
        nxt[a] = b
    assert sorted(nxt) == sorted(nxt.values()), (case, segs)
    loops, seen = [], set()
    for a, _ in segs:
        if a in seen:
            continue
        loop, e = [], a
        while e not in seen:
            seen.add(e)
            loop.append(e)
            e = nxt[e]
        assert e == a
        loops.append(loop)
    return loops


def case_triangles(case):
    tris = []
    for loop in case_loops(case):
        for i in range(1, len(loop) - 1):
            tris.append((loop[0], loop[i], loop[i + 1]))
    return tris


def build_table():
    """(tri [256, 16] int8 local-edge triples, -1 padded; ntri [256] uint8)."""
    tri = np.full((256, 16), -1, np.int8)
    ntri = np.zeros(256, np.uint8)
    for case in range(256):
        t = case_triangles(case)
        assert len(t) <= MAX_TRI, (case, t)
        ntri[case] = len(t)
        for i, (a, b, c) in enumerate(t):
            tri[case, 3 * i:3 * i + 3] = (a, b, c)
    return tri, ntri


def header_text():
    tri, ntri = build_table()
    rows = ",\n".join("    {" + ", ".join(str(int(v)) for v in r) + "}" for r in tri)
    return (
        "// GENERATED by csrc/mc_table_gen.py -- do not edit (the derivation rule is\n"
        "// documented there).  kMcTri[case]: local-edge triples of the case's triangles,\n"
        "// -1 padded; kMcNTri[case]: their count.\n"
        "#pragma once\n#include <cstdint>\n\nnamespace sdfr {\n"
        f"constexpr int kMcMaxTri = {MAX_TRI};\n"
        "__constant__ const int8_t kMcTri[256][16] = {\n" + rows + "\n};\n"
        "__constant__ const uint8_t kMcNTri[256] = {" + ", ".join(str(int(v)) for v in ntri) + "};\n"
        "}  // namespace sdfr\n")


if __name__ == "__main__":
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mc_table.h")
    with open(path, "w") as f:
        f.write(header_text())
    print("wrote", path)
