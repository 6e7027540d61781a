#!/usr/bin/env python3
"""Write scenes/diningroom/diningroom.obj: a synthetic stand-in for the
reference's diningroom scene (BASELINE.json configs[3], C4).

The reference's diningroom geometry is not recoverable here: diningroom.obj is
git-ignored upstream and diningroom.mb is a missing large blob (SURVEY.md §0.3,
§5.9).  SURVEY.md §8(d) therefore asks for a proxy that keeps what IS known:

  * the camera of MonteCarloPathTracing/config.json:75-81 (position
    (-0.5, 3, 5.5), look-at (-0.5, 2, 0), up y, vertical fov 60);
  * the materials of Scene/diningroom/diningroom.mtl, used by name (white
    walls; gold / silver (Ns 4000) / lamp / bottle Phong surfaces, all GLOSSY
    under the reference's classification; emitters light1 and light3);
  * ~100 K triangles of room + furniture + glossy objects in view.

The layout is a deterministic function of this file (no RNG): a closed room,
a table on four legs, four chairs, tessellated spheres (silver, gold), lathed
bottles, a pendant lamp shade with an emissive bulb (light1) and a ceiling
panel (light3).  Triangles are written directly ('f a b c'), grouped by
'usemtl', so the OBJ loader's triangulation cannot reorder them.

    python tools/make_diningroom_proxy.py   -> scenes/diningroom/diningroom.obj
"""
import math
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "scenes", "diningroom", "diningroom.obj")


class Mesh:
    def __init__(self):
        self.groups = []  # (material, vertices (n,3), faces (m,3) 0-based)

    def add(self, mat, v, f):
        v = np.asarray(v, np.float64)
        f = np.asarray(f, np.int64)
        # drop degenerate triangles (repeated corner index)
        keep = (f[:, 0] != f[:, 1]) & (f[:, 1] != f[:, 2]) & (f[:, 0] != f[:, 2])
        self.groups.append((mat, v, f[keep]))

    def tris(self):
        return sum(len(f) for _, _, f in self.groups)

    def write(self, path):
        lines = ["# diningroom proxy (tools/make_diningroom_proxy.py) - synthetic stand-in, see SURVEY.md 8(d)",
                 "mtllib diningroom.mtl"]
        base = 1
        for k, (mat, v, f) in enumerate(self.groups):
            lines.append("o part%d" % k)
            lines.extend("v %.6f %.6f %.6f" % tuple(p) for p in v)
            lines.append("usemtl " + mat)
            lines.extend("f %d %d %d" % tuple(t + base) for t in f)
            base += len(v)
        with open(path, "w") as fh:
            fh.write("\n".join(lines) + "\n")


def grid(origin, du, dv, nu, nv):
    """A planar quad grid origin + i/nu du + j/nv dv, as triangles."""
    o, du, dv = (np.asarray(x, np.float64) for x in (origin, du, dv))
    i, j = np.meshgrid(np.arange(nu + 1), np.arange(nv + 1), indexing="ij")
    v = o + (i[..., None] / nu) * du + (j[..., None] / nv) * dv
    idx = lambda a, b: a * (nv + 1) + b  # noqa: E731
    f = []
    for a in range(nu):
        for b in range(nv):
            f.append((idx(a, b), idx(a + 1, b), idx(a + 1, b + 1)))
            f.append((idx(a, b), idx(a + 1, b + 1), idx(a, b + 1)))
    return v.reshape(-1, 3), np.array(f)


def box(m, mat, lo, hi, n=1):
    """Axis-aligned box as six n x n grids, normals outward."""
    lo, hi = np.asarray(lo, float), np.asarray(hi, float)
    d = hi - lo
    ex, ey, ez = np.array([d[0], 0, 0]), np.array([0, d[1], 0]), np.array([0, 0, d[2]])
    for o, u, v in ((lo, ey, ex), (lo + ez, ex, ey), (lo, ez, ey), (lo + ex, ey, ez), (lo, ex, ez),
                    (lo + ey, ez, ex)):
        m.add(mat, *grid(o, u, v, n, n))


def room(m, lo, hi, n):
    """The room's six walls facing inward (white), finely tessellated."""
    lo, hi = np.asarray(lo, float), np.asarray(hi, float)
    d = hi - lo
    ex, ey, ez = np.array([d[0], 0, 0]), np.array([0, d[1], 0]), np.array([0, 0, d[2]])
    for o, u, v in ((lo, ex, ey), (lo + ez, ey, ex), (lo, ey, ez), (lo + ex, ez, ey), (lo, ez, ex),
                    (lo + ey, ex, ez)):
        m.add("scene1:white", *grid(o, u, v, n, n))


def lathe(m, mat, center, profile, nseg):
    """Surface of revolution about the y axis through `center` of the
    (radius, height) polyline `profile`; open ends closed by fans."""
    c = np.asarray(center, float)
    prof = np.asarray(profile, float)
    k = len(prof)
    ang = 2 * math.pi * np.arange(nseg) / nseg
    v = []
    for r, y in prof:
        for a in ang:
            v.append(c + (r * math.cos(a), y, r * math.sin(a)))
    f = []
    for i in range(k - 1):
        for s in range(nseg):
            a, b = i * nseg + s, i * nseg + (s + 1) % nseg
            f.append((a, b + nseg, b))
            f.append((a, a + nseg, b + nseg))
    v = np.array(v)
    # caps
    for i, flip in ((0, False), (k - 1, True)):
        if prof[i][0] > 0:
            ci = len(v)
            v = np.vstack([v, c + (0.0, prof[i][1], 0.0)])
            for s in range(nseg):
                a, b = i * nseg + s, i * nseg + (s + 1) % nseg
                f.append((ci, b, a) if flip else (ci, a, b))
    m.add(mat, v, np.array(f))


def sphere(m, mat, center, r, nu, nv):
    prof = [(r * math.sin(math.pi * j / nv), -r * math.cos(math.pi * j / nv)) for j in range(nv + 1)]
    prof[0] = (0.0, -r)
    prof[-1] = (0.0, r)
    c = np.asarray(center, float)
    # lathe with collapsed poles: keep the poles as single vertices
    ang = 2 * math.pi * np.arange(nu) / nu
    v = [c + (0.0, -r, 0.0)]
    for j in range(1, nv):
        rr, y = prof[j]
        for a in ang:
            v.append(c + (rr * math.cos(a), y, rr * math.sin(a)))
    v.append(c + (0.0, r, 0.0))
    top = len(v) - 1
    ring = lambda j, s: 1 + (j - 1) * nu + (s % nu)  # noqa: E731
    f = []
    for s in range(nu):
        f.append((0, ring(1, s + 1), ring(1, s)))
        f.append((top, ring(nv - 1, s), ring(nv - 1, s + 1)))
    for j in range(1, nv - 1):
        for s in range(nu):
            a, b = ring(j, s), ring(j, s + 1)
            c2, d2 = ring(j + 1, s), ring(j + 1, s + 1)
            f.append((a, b, d2))
            f.append((a, d2, c2))
    m.add(mat, np.array(v), np.array(f))


def build():
    m = Mesh()
    # table: top + four gold legs
    box(m, "scene1:white", (-3.2, 1.40, -1.4), (2.2, 1.52, 1.4), 8)
    for x in (-3.0, 1.9):
        for z in (-1.2, 1.1):
            lathe(m, "scene1:gold", (x + 0.05, 0.0, z + 0.05), [(0.07, 0.0), (0.05, 0.7), (0.07, 1.4)], 24)
    # four chairs (seat + back), white
    for x, z, back in ((-2.2, -2.2, -1), (0.8, -2.2, -1), (-2.2, 2.2, 1), (0.8, 2.2, 1)):
        box(m, "scene1:white", (x - 0.45, 0.85, z - 0.45), (x + 0.45, 0.95, z + 0.45), 4)
        bz = z + back * 0.45
        box(m, "scene1:white", (x - 0.45, 0.95, min(bz, bz - back * 0.08)), (x + 0.45, 1.9, max(bz, bz - back * 0.08)),
            4)
        for dx in (-0.4, 0.35):
            for dz in (-0.4, 0.35):
                box(m, "scene1:gold", (x + dx, 0.0, z + dz), (x + dx + 0.05, 0.85, z + dz + 0.05))
    # glossy objects on the table
    sphere(m, "scene1:silver", (-2.3, 1.82, 0.3), 0.30, 96, 48)
    sphere(m, "scene1:silver", (1.3, 1.77, -0.4), 0.25, 96, 48)
    sphere(m, "scene1:gold", (-0.6, 1.72, 0.7), 0.20, 96, 48)
    sphere(m, "scene1:gold", (0.4, 1.67, 0.9), 0.15, 64, 32)
    sphere(m, "scene1:silver", (4.2, 0.6, -2.8), 0.60, 128, 64)  # a large mirror ball in the corner
    bottle = [(0.0, 0.0), (0.16, 0.0), (0.18, 0.05), (0.18, 0.55), (0.15, 0.65), (0.07, 0.75), (0.06, 0.95),
              (0.07, 1.0), (0.0, 1.0)]
    for k, (x, z) in enumerate(((-1.6, -0.5), (-1.1, -0.7), (-0.2, -0.3), (0.6, -0.8))):
        prof = [(r, y) for r, y in bottle]
        # refine the profile to 40 rings
        ys = np.linspace(0, 1, 40)
        rs = np.interp(ys, [p[1] for p in prof[1:-1]], [p[0] for p in prof[1:-1]])
        lathe(m, "scene1:bottle", (x, 1.52, z), list(zip(rs, ys)), 64)
    # pendant lamp: shade (lamp) + bulb (light1), ceiling panel (light3)
    lathe(m, "scene1:lamp", (-0.5, 0.0, 0.0), [(0.08, 5.98), (0.08, 5.0), (0.25, 4.7), (0.55, 4.35)], 64)
    sphere(m, "scene1:light1", (-0.5, 4.5, 0.0), 0.2, 32, 16)
    v, f = grid((2.0, 5.995, -2.5), (2.2, 0, 0), (0, 0, 5.0), 2, 4)
    m.add("scene1:light1", v, f[:, ::-1])
    v, f = grid((-3.5, 5.995, -2.5), (2.2, 0, 0), (0, 0, 5.0), 2, 4)
    m.add("scene1:light3", v, f[:, ::-1])  # facing down
    # the room last: its corner triangle has the smallest Morton code, and as
    # triangle 0 it would land in leaf n-1 and make the reference's treelet
    # SAH recursion cycle (treeletBVH.cpp:327, see mcpt_treelet_device)
    room(m, (-7.0, 0.0, -4.0), (6.0, 6.0, 8.0), 48)
    return m


def main():
    m = build()
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    m.write(OUT)
    print("wrote %s: %d triangles" % (OUT, m.tris()))


if __name__ == "__main__":
    main()
