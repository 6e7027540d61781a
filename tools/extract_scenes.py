#!/usr/bin/env python3
"""Recover the reference's test scenes as OBJ files from the Maya binaries.

The reference renders ``Scene/cbox/cbox.obj`` and ``Scene/veach_mis/mis.obj``
(``MonteCarloPathTracing/config.json:12-13,40-41``), but ``*.obj`` is git-ignored
upstream, so only the Maya ``.mb`` sources and the ``.mtl`` files ship
(SURVEY.md §5.9).  This tool decodes the ``.mb`` IFF-64 container directly:

* chunk header = tag[4] | flags[4] | size u64 BE; ``FOR8``/``LIS8``/``CAT8``
  groups carry a 4-byte type and unpadded children, leaf chunks are padded to 8;
* ``DMSH`` groups hold a ``MESH`` chunk: ``'o\\0' 0x20``, u32 float count +
  BE f32 xyz (world space — every mesh ``XFRM`` is identity in both files),
  u32 count + edge pairs ``(v0 | hard-flag<<31, v1)``, u32 count + face-edge
  list (bit 31 = edge reversed, ``0x60000000`` = last edge of a loop);
* the ``CONS``/``CONN`` list connects ``<shape>.iog.og[0]`` to a shading group
  whose name is the ``newmtl`` name in the scene's ``.mtl``.

Faces are written as OBJ polygons (quads stay quads, exactly what a Maya OBJ
export holds); the loader triangulates them.  The one face with a hole (the
cbox ceiling: an outer loop plus the reversed luminaire outline) cannot be an
OBJ polygon, so its ring is written as the four convex trapezoids between the
two loops — the luminaire quad stays a separate light mesh, with no coplanar
ceiling underneath it.

Run here (the reference is mounted only in the build container); the outputs
are committed under ``scenes/`` and travel to the GPU box.
"""
import os
import shutil
import struct
import sys

REF = "/root/reference/Scene"
GROUPS = (b"FOR8", b"LIS8", b"CAT8")


def _chunks(data, off, end):
    while off + 16 <= end:
        tag = data[off:off + 4]
        size = struct.unpack(">Q", data[off + 8:off + 16])[0]
        body = off + 16
        grp = tag in GROUPS
        yield tag, body, size, grp
        off = body + (size if grp else ((size + 7) & ~7))


def _walk(data, off, end):
    for tag, body, size, grp in _chunks(data, off, end):
        if grp:
            yield tag, data[body:body + 4], body, size
            yield from _walk(data, body + 4, body + size)


def _decode_mesh(b):
    p = 3  # 'o\0' + type byte 0x20
    nf = struct.unpack(">I", b[p:p + 4])[0]; p += 4
    v = struct.unpack(">%df" % nf, b[p:p + 4 * nf]); p += 4 * nf
    ne = struct.unpack(">I", b[p:p + 4])[0]; p += 4
    e = struct.unpack(">%dI" % ne, b[p:p + 4 * ne]); p += 4 * ne
    nfe = struct.unpack(">I", b[p:p + 4])[0]; p += 4
    fe = struct.unpack(">%dI" % nfe, b[p:p + 4 * nfe])
    verts = [v[i:i + 3] for i in range(0, nf, 3)]
    edges = [(e[i] & 0x7FFFFFFF, e[i + 1]) for i in range(0, ne, 2)]
    faces, loops = [], []
    for x in fe:
        a, c = edges[x & 0x1FFFFFFF]
        loops.append(c if x & 0x80000000 else a)
        if (x & 0x60000000) == 0x60000000:
            faces.append(loops)
            loops = []
    return verts, faces


def read_mb(path):
    """Return [(shape_name, material, verts, faces_with_loops)] in file order."""
    data = open(path, "rb").read()
    meshes = []
    conn = {}
    for tag, typ, body, size in _walk(data, 20, len(data)):
        if typ == b"DMSH":
            name = None
            for t2, b2, s2, _ in _chunks(data, body + 4, body + size):
                if t2 == b"CREA":
                    name = data[b2 + 1:b2 + s2].split(b"\0")[0].decode()
                elif t2 == b"MESH":
                    verts, faces = _decode_mesh(data[b2:b2 + s2])
                    meshes.append([name, None, verts, faces])
        elif typ == b"CONN":
            for t2, b2, s2, _ in _chunks(data, body + 4, body + size):
                if t2 != b"CWFL":
                    continue
                src, dst = data[b2 + 1:b2 + s2].split(b"\0")[:2]
                src, dst = src.decode(), dst.decode()
                # "<shape>.iog.og[0]" -> "<SG>.dsm"  (shape belongs to shading group SG)
                if src.endswith(".iog.og[0]") and dst.endswith(".dsm"):
                    conn[src[:-len(".iog.og[0]")]] = dst[:-len(".dsm")]
    for m in meshes:
        m[1] = conn.get(m[0])
    return meshes


def _mtl_names(path):
    return [l.split(None, 1)[1].strip() for l in open(path) if l.startswith("newmtl")]


def _resolve(sg, names):
    """Shading-group name -> .mtl name.  The Maya namespace differs between the
    .mb and the .mtl of veach_mis ("mis:plate_1" vs "mi:plate_1"), so match on
    the part after the namespace separator."""
    if sg in names:
        return sg
    hits = [n for n in names if n.split(":")[-1] == sg.split(":")[-1]]
    if len(hits) != 1:
        raise ValueError("cannot map shading group %r onto %s" % (sg, names))
    return hits[0]


def write_obj(meshes, mtlname, out_path, mtl_names):
    lines = ["# recovered from the reference's Maya scene by tools/extract_scenes.py",
             "mtllib %s" % mtlname]
    base = 1
    for name, mat, verts, faces in meshes:
        lines.append("o %s" % name.replace("Shape", ""))
        for x, y, z in verts:
            lines.append("v %.9g %.9g %.9g" % (x, y, z))
        lines.append("usemtl %s" % _resolve(mat, mtl_names))
        if len(faces) == 2 and all(len(f) == 4 for f in faces) and "ceiling" in name:
            outer, inner = faces
            inner = inner[::-1]  # stored reversed (a hole); align with the outer winding
            # pair each outer corner with the nearest inner corner, then emit the ring
            shift = min(range(4), key=lambda s: sum(
                (verts[outer[k]][0] - verts[inner[(k + s) % 4]][0]) ** 2 +
                (verts[outer[k]][2] - verts[inner[(k + s) % 4]][2]) ** 2 for k in range(4)))
            inner = [inner[(k + shift) % 4] for k in range(4)]
            faces = [[outer[k], outer[(k + 1) % 4], inner[(k + 1) % 4], inner[k]] for k in range(4)]
        for f in faces:
            lines.append("f " + " ".join(str(base + i) for i in f))
        base += len(verts)
    with open(out_path, "w") as fh:
        fh.write("\n".join(lines) + "\n")


def main(repo):
    jobs = [("cbox", "cbox.mb", "cbox.obj", "cbox.mtl"),
            ("veach_mis", "mis.mb", "mis.obj", "mis.mtl")]
    for d, mb, obj, mtl in jobs:
        meshes = read_mb(os.path.join(REF, d, mb))
        os.makedirs(os.path.join(repo, "scenes", d), exist_ok=True)
        write_obj(meshes, mtl, os.path.join(repo, "scenes", d, obj), _mtl_names(os.path.join(REF, d, mtl)))
        shutil.copyfile(os.path.join(REF, d, mtl), os.path.join(repo, "scenes", d, mtl))
        nf = sum(len(m[3]) for m in meshes)
        print("%s: %d meshes, %d faces -> scenes/%s/%s" % (d, len(meshes), nf, d, obj))
    # the diningroom geometry is not recoverable (.MISSING_LARGE_BLOBS); keep its materials
    os.makedirs(os.path.join(repo, "scenes", "diningroom"), exist_ok=True)
    shutil.copyfile(os.path.join(REF, "diningroom", "diningroom.mtl"),
                    os.path.join(repo, "scenes", "diningroom", "diningroom.mtl"))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
