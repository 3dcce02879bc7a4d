"""Render meshes of the compiled scenes: vertex-clustering level of detail, triangles per body.

The reference renders every `class="visual"` mesh geom through MuJoCo's OpenGL renderer
(envs/mujoco/MujocoEnvBase.py:103-126; e.g. the UR5e link meshes of
envs/assets/mujoco/robots/ur5e/ur5e_integrated_body.xml:4-18).  The batched renderer
(csrc/rmbx_render.hip) draws the same triangles, shared read-only by every env and camera, with a
visibility pass: every triangle of every env is tested against the camera rays of the pixel
centres its projection covers and the nearest wins per pixel (a 64-bit atomic min of
(depth, triangle)), then the ray-cast pass over the analytic primitives starts each pixel from that
hit.  Here the triangle tables are built:

* level of detail: each mesh's vertices are clustered on a grid of `cell` metres in its file frame
  (each cluster replaced by the mean of its vertices; triangles that collapse to a line or point
  and duplicates dropped), so no vertex moves by more than the cell's diagonal (sqrt(3) cell) -- at
  the default 1 mm, 1.7 mm, below the ~2.6 mm one pixel spans at the front camera's distance from
  the arm (640 x 480, fovy 45 deg, ~1.5 m);
* grouped by BODY, in the body frame (v_body = R(geom quat) v_file + geom pos: a body's meshes move
  rigidly together), so one transform per env and body places them;
* layout: triangle f32 [ntri][16] = (v0.xyz, e1.xyz, e2.xyz, n.xyz, tag, rgb) with e1 = v1 - v0,
  e2 = v2 - v0, n the unit face normal and tag = (mesh body slot << 16) | geom id as int32 bits;
  per mesh body slot k: rmesh_body[k], its triangle range rmesh_tri_adr / rmesh_tri_num, and the
  bounding radius of its triangles about the body origin rmesh_rad.
"""

import numpy as np


def cluster_vertices(verts, faces, cell):
    """Vertex clustering on a `cell`-metre grid: (verts', faces') with every cluster's vertices
    replaced by their mean, degenerate and duplicate triangles removed (orientation kept)."""
    if cell <= 0 or len(faces) == 0:
        return verts, faces
    key = np.floor(verts / cell).astype(np.int64)
    _, cid, counts = np.unique(key, axis=0, return_inverse=True, return_counts=True)
    cid = cid.reshape(-1)
    nv = len(counts)
    sums = np.zeros((nv, 3))
    np.add.at(sums, cid, verts)
    nverts = sums / counts[:, None]
    f = cid[faces]
    ok = (f[:, 0] != f[:, 1]) & (f[:, 1] != f[:, 2]) & (f[:, 0] != f[:, 2])
    f = f[ok]
    srt = np.sort(f, axis=1)
    _, first = np.unique(srt, axis=0, return_index=True)
    f = f[np.sort(first)]
    v0, v1, v2 = nverts[f[:, 0]], nverts[f[:, 1]], nverts[f[:, 2]]
    area2 = np.linalg.norm(np.cross(v1 - v0, v2 - v0), axis=1)
    f = f[area2 > 1e-14]
    used = np.unique(f)
    remap = np.full(nv, -1, np.int64)
    remap[used] = np.arange(len(used))
    return nverts[used], remap[f]


def render_meshes(geoms, cell=1e-3, max_group=2):
    """Render-mesh arrays for the compiled geoms (mjcf/compiler.py output): every mesh geom of a
    rendered group (MuJoCo draws groups 0-2 by default) whose mesh file is present, grouped by
    body (see the module docstring).  Returns a dict of arrays (empty without meshes)."""
    from .compiler import quat2mat

    per_body = {}
    for gi, g in enumerate(geoms):
        if g["type"] != 7 or g["group"] > max_group or g.get("mesh") is None:
            continue
        verts, faces = g["mesh"]
        v, f = cluster_vertices(np.asarray(verts, np.float64), np.asarray(faces), cell)
        if len(f) == 0:
            continue
        vb = v @ quat2mat(g["quat"]).T + np.asarray(g["pos"], np.float64)
        per_body.setdefault(g["body"], []).append((gi, vb[f], np.asarray(g["rgba"][:3], np.float64), len(faces)))
    if not per_body:
        return {}
    assert len(per_body) < 32768 and len(geoms) < 65536, "triangle tags hold 15 + 16 bits"
    bodies, tri_adr, tri_num, rad, src, tris_all = [], [], [], [], [], []
    n_tris = 0
    for k, b in enumerate(sorted(per_body)):
        parts = per_body[b]
        tris = np.concatenate([p[1] for p in parts])
        tag = np.concatenate([np.full(len(p[1]), (k << 16) | p[0], np.int32) for p in parts])
        rgb = np.concatenate([np.tile(p[2], (len(p[1]), 1)) for p in parts])
        v0, e1, e2 = tris[:, 0], tris[:, 1] - tris[:, 0], tris[:, 2] - tris[:, 0]
        nrm = np.cross(e1, e2)
        nrm /= np.maximum(np.linalg.norm(nrm, axis=1, keepdims=True), 1e-300)
        packed = np.zeros((len(tris), 16), np.float32)
        packed[:, 0:3], packed[:, 3:6], packed[:, 6:9], packed[:, 9:12] = v0, e1, e2, nrm
        packed[:, 12] = tag.view(np.float32)
        packed[:, 13:16] = rgb
        bodies.append(b)
        tri_adr.append(n_tris)
        tri_num.append(len(tris))
        rad.append(float(np.linalg.norm(tris.reshape(-1, 3), axis=1).max()))
        src.append(sum(p[3] for p in parts))
        tris_all.append(packed)
        n_tris += len(tris)
    assert n_tris < (1 << 26), "the visibility key holds 26-bit triangle indices"
    return {"rmesh_body": np.asarray(bodies, np.int32), "rmesh_tri_adr": np.asarray(tri_adr, np.int32),
            "rmesh_tri_num": np.asarray(tri_num, np.int32), "rmesh_rad": np.asarray(rad, np.float32),
            "rmesh_src_tris": np.asarray(src, np.int32), "rmesh_cell": np.float64(cell),
            "rmesh_geoms": np.asarray(sorted(gi for b in per_body for gi, *_ in per_body[b]), np.int32),
            "rmesh_tri": np.ascontiguousarray(np.concatenate(tris_all))}
