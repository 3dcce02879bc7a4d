"""MJCF-subset compiler -> flat model arrays for the batched engine (numpy, host side).

Covers the subset of MuJoCo's model compiler (mujoco==3.1.6, external dependency of the
reference, pyproject.toml:34) that the reference's MujocoUR5eCable scene uses
(envs/assets/mujoco/envs/ur5e/env_ur5e_cable.xml and its includes):

  * <include>, <compiler angle autolimits meshdir>, <option timestep gravity>, <statistic extent>
  * <default> classes with inheritance and body childclass
  * bodies with pos/quat/euler/zaxis, <inertial> or geom-derived mass properties
    (box/capsule/cylinder/sphere/mesh at density 1000, parallel-axis composition)
  * joints (hinge, free) with range/autolimits, armature, damping, stiffness/springref,
    solreflimit/solimplimit
  * geoms (plane, sphere, capsule, cylinder, box, mesh) with contype/conaffinity, priority,
    friction, solref/solimp; static contact-pair filtering (weld groups, parent filter,
    <exclude>) and per-pair parameter mixing as MuJoCo's mj_contactParam
  * <general> actuators with joint/fixed-tendon transmission, fixed gain, affine bias
  * <fixed> tendons, <equality> weld/connect/joint, force/torque site sensors, cameras
  * mj_setConst-style constants at qpos0: body/dof inverse weights, mean inertia, connect
    anchors in body2 frames.
  * <composite type="loop"> (env_ur5e_ring.xml): expanded into its body chain before compiling
    (_expand_composites).

Substitutions (MuJoCo parity is unpinned: no MuJoCo in this image):
  * by default collision meshes are replaced by their oriented bounding box in the geom frame
    (box-box narrowphase) and cylinders collide as capsules of the same radius and half-length;
    with convex_meshes=True mesh geoms collide through their convex hull and cylinders exactly
    (MPR narrow phase, as MuJoCo 3.1.6's mjc_Convex does through libccd);
  * a mesh that is missing from the checkout (the reference's .MISSING_LARGE_BLOBS) falls back
    to a box of the D435i housing size 90x25x25 mm.
"""

import math
import os
import struct
import xml.etree.ElementTree as ET

import numpy as np

# geom types (MuJoCo mjtGeom order)
GEOM_PLANE, GEOM_HFIELD, GEOM_SPHERE, GEOM_CAPSULE, GEOM_ELLIPSOID, GEOM_CYLINDER, GEOM_BOX, GEOM_MESH = range(8)
GEOM_TYPES = {"plane": 0, "hfield": 1, "sphere": 2, "capsule": 3, "ellipsoid": 4, "cylinder": 5, "box": 6, "mesh": 7}
# joint types (mjtJoint)
JNT_FREE, JNT_BALL, JNT_SLIDE, JNT_HINGE = range(4)
# equality types (mjtEq)
EQ_CONNECT, EQ_WELD, EQ_JOINT = 0, 1, 2
# actuator transmission
TRN_JOINT, TRN_TENDON = 0, 3
# sensors
SENS_FORCE, SENS_TORQUE = 0, 1

DEFAULT_SOLREF = (0.02, 1.0)
DEFAULT_SOLIMP = (0.9, 0.95, 0.001, 0.5, 2.0)
DEFAULT_FRICTION = (1.0, 0.005, 0.0001)


# ------------------------------------------------------------------------------------------
# math helpers
# ------------------------------------------------------------------------------------------
def quat_normalize(q):
    q = np.asarray(q, dtype=np.float64)
    n = np.linalg.norm(q)
    return q / n if n > 0 else np.array([1.0, 0, 0, 0])


def quat_mul(a, b):
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return np.array(
        [
            w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
            w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
            w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
            w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2,
        ]
    )


def quat2mat(q):
    w, x, y, z = q
    return np.array(
        [
            [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
            [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
            [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
        ]
    )


def mat2quat(R):
    t = np.trace(R)
    if t > 0:
        s = math.sqrt(t + 1.0) * 2
        q = [0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s]
    else:
        i = int(np.argmax(np.diag(R)))
        if i == 0:
            s = math.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
            q = [(R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s]
        elif i == 1:
            s = math.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
            q = [(R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s]
        else:
            s = math.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
            q = [(R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s]
    q = np.array(q)
    return q if q[0] >= 0 else -q


def axisangle2quat(axis, angle):
    axis = np.asarray(axis, np.float64)
    axis = axis / np.linalg.norm(axis)
    return np.concatenate([[math.cos(angle / 2)], math.sin(angle / 2) * axis])


def euler2quat(e, seq="xyz"):
    q = np.array([1.0, 0, 0, 0])
    for ang, ax in zip(e, seq):
        v = {"x": [1, 0, 0], "y": [0, 1, 0], "z": [0, 0, 1]}[ax.lower()]
        r = axisangle2quat(v, ang)
        q = quat_mul(q, r) if ax.islower() else quat_mul(r, q)
    return quat_normalize(q)


def zaxis2quat(z):
    """Minimal rotation taking (0,0,1) to z (mju_quatZ2Vec)."""
    z = np.asarray(z, np.float64)
    z = z / np.linalg.norm(z)
    a = np.array([0.0, 0.0, 1.0])
    c = np.cross(a, z)
    s = np.linalg.norm(c)
    if s < 1e-10:
        return np.array([1.0, 0, 0, 0]) if z[2] > 0 else np.array([0.0, 1.0, 0, 0])
    ang = math.atan2(s, float(np.dot(a, z)))
    return axisangle2quat(c / s, ang)


def _floats(s):
    return [float(x) for x in s.split()]


# ------------------------------------------------------------------------------------------
# mesh loading and mass properties
# ------------------------------------------------------------------------------------------
def load_mesh(path, scale):
    """Return (vertices [n,3], faces [m,3]) of an STL (binary) or OBJ file, scaled."""
    if path.lower().endswith(".stl"):
        with open(path, "rb") as f:
            data = f.read()
        n = struct.unpack("<I", data[80:84])[0]
        rec = np.frombuffer(data[84 : 84 + 50 * n], dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]))
        tri = rec["v"].astype(np.float64).reshape(-1, 3)
        verts, inv = np.unique(tri, axis=0, return_inverse=True)
        faces = inv.reshape(-1, 3)
    else:
        vs, fs = [], []
        with open(path) as f:
            for line in f:
                if line.startswith("v "):
                    vs.append([float(x) for x in line.split()[1:4]])
                elif line.startswith("f "):
                    idx = [int(t.split("/")[0]) for t in line.split()[1:]]
                    idx = [i - 1 if i > 0 else len(vs) + i for i in idx]
                    for k in range(1, len(idx) - 1):
                        fs.append([idx[0], idx[k], idx[k + 1]])
        verts, faces = np.array(vs, np.float64), np.array(fs, np.int64)
    return verts * np.asarray(scale, np.float64), faces


def mesh_mass_props(verts, faces):
    """Volume, COM and inertia-per-unit-density about the COM of a closed triangle mesh
    (signed tetrahedra, canonical covariance)."""
    v0, v1, v2 = verts[faces[:, 0]], verts[faces[:, 1]], verts[faces[:, 2]]
    det = np.einsum("ij,ij->i", v0, np.cross(v1, v2))
    vol = det.sum() / 6.0
    sign = 1.0 if vol >= 0 else -1.0
    vol *= sign
    det *= sign
    com = (det[:, None] * (v0 + v1 + v2)).sum(0) / (24.0 * vol)
    C_can = np.array([[2, 1, 1], [1, 2, 1], [1, 1, 2]]) / 120.0
    A = np.stack([v0, v1, v2], axis=2)  # [m,3,3] columns are vertices
    C = np.einsum("m,mij,jk,mlk->il", det, A, C_can, A)
    C = C - vol * np.outer(com, com)
    inertia = np.trace(C) * np.eye(3) - C
    return vol, com, inertia


def box_inertia(m, s):
    x, y, z = (2 * np.asarray(s[:3])) ** 2
    return m / 12.0 * np.diag([y + z, x + z, x + y])


def geom_mass_props(gtype, size, density, mesh=None):
    """(mass, com (geom frame), inertia about com (geom frame)) — MuJoCo mjCGeom::SetInertia."""
    if gtype == GEOM_SPHERE:
        r = size[0]
        m = density * 4.0 / 3.0 * math.pi * r**3
        return m, np.zeros(3), np.eye(3) * 0.4 * m * r * r
    if gtype == GEOM_CAPSULE:
        r, h = size[0], size[1]
        height = 2 * h
        vol = math.pi * r * r * height + 4.0 / 3.0 * math.pi * r**3
        m = density * vol
        sm = m * 4 * r / (4 * r + 3 * height)
        cm = m - sm
        ixx = cm * (3 * r * r + height * height) / 12.0
        izz = cm * r * r / 2.0
        si = 2 * sm * r * r / 5.0
        ixx += si + sm * height * (3 * r + 2 * height) / 8.0
        izz += si
        return m, np.zeros(3), np.diag([ixx, ixx, izz])
    if gtype == GEOM_CYLINDER:
        r, h = size[0], size[1]
        m = density * math.pi * r * r * 2 * h
        ixx = m * (3 * r * r + 4 * h * h) / 12.0
        return m, np.zeros(3), np.diag([ixx, ixx, m * r * r / 2.0])
    if gtype == GEOM_BOX:
        m = density * 8 * size[0] * size[1] * size[2]
        return m, np.zeros(3), box_inertia(m, size)
    if gtype == GEOM_MESH:
        vol, com, I = mesh_mass_props(*mesh)
        return density * vol, com, density * I
    return 0.0, np.zeros(3), np.zeros((3, 3))


# ------------------------------------------------------------------------------------------
# XML front end
# ------------------------------------------------------------------------------------------
class _Defaults:
    def __init__(self):
        self.classes = {}  # name -> (parent, {elem: {attr: val}})

    def add(self, name, parent, node):
        attrs = {}
        for child in node:
            if child.tag == "default":
                continue
            attrs.setdefault(child.tag, {}).update(child.attrib)
        self.classes[name] = (parent, attrs)

    def resolve(self, cls, tag):
        chain = []
        c = cls
        while c is not None:
            parent, attrs = self.classes[c]
            chain.append(attrs.get(tag, {}))
            c = parent
        out = {}
        for a in reversed(chain):
            out.update(a)
        return out


class Model:
    """Plain container of compiled arrays (see compile_mjcf)."""


_ASSET_FILE_TAGS = ("mesh", "texture", "hfield", "skin")


def _expand_includes(node, main_dir, missing):
    out = []
    for child in list(node):
        if child.tag == "include":
            path = os.path.join(main_dir, child.attrib["file"])
            if not os.path.exists(path) and missing is not None:
                missing.append(child.attrib["file"])  # absent from the checkout (e.g. YCB_sim)
                continue
            root = ET.parse(path).getroot()
            _expand_includes_inplace(root, main_dir, missing)
            # asset files of an included file that sit next to it (MuJoCo resolves them from the
            # including file's directory, e.g. mujoco_scanned_objects/<obj>/model.obj)
            inc_dir = os.path.dirname(path)
            for el in root.iter():
                f = el.attrib.get("file")
                if el.tag in _ASSET_FILE_TAGS and f and not os.path.isabs(f) and os.path.exists(os.path.join(inc_dir, f)):
                    el.attrib["file"] = os.path.abspath(os.path.join(inc_dir, f))
            out.extend(list(root))
        else:
            _expand_includes_inplace(child, main_dir, missing)
            out.append(child)
    return out


def _expand_includes_inplace(node, main_dir, missing=None):
    new = _expand_includes(node, main_dir, missing)
    for c in list(node):
        node.remove(c)
    for c in new:
        node.append(c)


def _drop_empty_free_bodies(node):
    """Remove bodies left with a free joint and nothing else (their geoms came from an include
    that is absent from the checkout): MuJoCo rejects massless moving bodies."""
    dropped = []
    for child in list(node):
        if child.tag == "body":
            _drop_empty_free_bodies(child)
            kinds = {c.tag for c in child}
            if kinds and kinds <= {"freejoint", "joint"} and any(
                    c.tag == "freejoint" or c.attrib.get("type") == "free" for c in child):
                node.remove(child)
                dropped.append(child.attrib.get("name", child.attrib.get("pos", "")))
        else:
            dropped += _drop_empty_free_bodies(child)
    return dropped


def _expand_composites(node):
    """Expand <composite type="loop"> (MuJoCo 3.1.6 user_composite: MakeRope + the loop closure;
    used by env_ur5e_ring.xml) into explicit MJCF before compiling.  The host body must be named
    `{prefix}B{ox}`; `count` elements of length `spacing` follow it as a chain of child bodies
    `{prefix}B{i}` (right of ox, then left of it), each with geom `{prefix}G{i}` (the composite's
    geom, its axis along the chain: quat rotating z to x) and, except the host, two hinge joints
    `{prefix}J0_{i}` / `{prefix}J1_{i}` (axes y and z, at the element's start vertex, attributes
    of <joint kind="main">).  A loop is laid out as the regular polygon it closes into (each
    element turned 2 pi / count about its z axis from the previous one, so every joint vertex
    and the closure coincide at qpos0) and closed by a connect equality between the first
    element's start vertex and the last element's end vertex.  The two closing elements are
    excluded from colliding with each other like the chain's parent/child neighbours (MuJoCo
    parity unpinned: MuJoCo is absent from the image).  Returns the number expanded."""
    count_expanded = 0
    for body in list(node.iter("body")):
        for comp in [c for c in body if c.tag == "composite"]:
            a = comp.attrib
            if a.get("type") != "loop":
                raise ValueError(f"composite type {a.get('type')!r} is not supported")
            prefix = a.get("prefix", "")
            n = int(_floats(a["count"])[0])
            s = float(a["spacing"])
            name = body.attrib.get("name", "")
            if not name.startswith(prefix + "B"):
                raise ValueError(f"composite host body {name!r} must be named {prefix}B<index>")
            ox = int(name[len(prefix) + 1:])
            if not 0 <= ox < n:
                raise ValueError("composite host body index out of range")
            geom_a = next((dict(c.attrib) for c in comp if c.tag == "geom"), {})
            joint_a = next((dict(c.attrib) for c in comp if c.tag == "joint" and c.attrib.get("kind") == "main"), {})
            joint_a.pop("kind", None)
            alpha = 2.0 * math.pi / n
            r2 = math.sqrt(0.5)

            def element(parent, i):
                g = ET.SubElement(parent, "geom", dict(geom_a))
                g.set("name", f"{prefix}G{i}")
                g.set("pos", "0 0 0")
                g.set("quat", f"{r2!r} 0 {r2!r} 0")

            body.remove(comp)
            element(body, ox)
            for direction in (1, -1):
                parent = body
                for i in range(ox + direction, n if direction > 0 else -1, direction):
                    # next element: to the shared vertex, turn by +-alpha about z, half a spacing on
                    turn = direction * alpha
                    child = ET.SubElement(parent, "body", {
                        "name": f"{prefix}B{i}",
                        "pos": f"{direction * 0.5 * s * (1 + math.cos(alpha))!r} {0.5 * s * math.sin(alpha)!r} 0",
                        "quat": f"{math.cos(0.5 * turn)!r} 0 0 {math.sin(0.5 * turn)!r}"})
                    for k, ax in enumerate(("0 1 0", "0 0 1")):
                        j = ET.SubElement(child, "joint", dict(joint_a))
                        j.set("name", f"{prefix}J{k}_{i}")
                        j.set("type", "hinge")
                        j.set("pos", f"{-direction * 0.5 * s!r} 0 0")
                        j.set("axis", ax)
                    element(child, i)
                    parent = child
            eq = ET.SubElement(node, "equality")
            ET.SubElement(eq, "connect", {"body1": f"{prefix}B0", "body2": f"{prefix}B{n - 1}",
                                          "anchor": f"{-0.5 * s!r} 0 0"})
            ct = ET.SubElement(node, "contact")
            ET.SubElement(ct, "exclude", {"body1": f"{prefix}B0", "body2": f"{prefix}B{n - 1}"})
            count_expanded += 1
    return count_expanded


def compile_mjcf(path, missing_mesh_box=(0.045, 0.0125, 0.0125), convex_meshes=False, skip_missing_includes=False):
    """Compile the MJCF at `path`.  convex_meshes: mesh geoms collide through the convex hull of
    their vertices (MuJoCo's own mesh collision model) and cylinders as true cylinders, both
    through the MPR narrow phase, instead of the mesh-OBB / capsule substitutes.
    skip_missing_includes: includes absent from the checkout are dropped together with the free
    bodies they would have filled (the Pick scene minus its YCB_sim objects)."""
    main_dir = os.path.dirname(os.path.abspath(path))
    root = ET.parse(path).getroot()
    missing = [] if skip_missing_includes else None
    _expand_includes_inplace(root, main_dir, missing)
    dropped_bodies = _drop_empty_free_bodies(root) if skip_missing_includes else []
    _expand_composites(root)

    # ---- compiler / option / statistic / visual
    meshdir = main_dir
    texturedir = main_dir
    autolimits = True
    angle_deg = True
    timestep, gravity = 0.002, np.array([0, 0, -9.81])
    extent = None
    znear, zfar = 0.01, 50.0
    for c in root.iter("compiler"):
        if "meshdir" in c.attrib:
            meshdir = os.path.join(main_dir, c.attrib["meshdir"])
        if "texturedir" in c.attrib:
            texturedir = os.path.join(main_dir, c.attrib["texturedir"])
        if "autolimits" in c.attrib:
            autolimits = c.attrib["autolimits"] == "true"
        if "angle" in c.attrib:
            angle_deg = c.attrib["angle"] == "degree"
    for c in root.iter("option"):
        timestep = float(c.attrib.get("timestep", timestep))
        if "gravity" in c.attrib:
            gravity = np.array(_floats(c.attrib["gravity"]))
        integrator = c.attrib.get("integrator", "Euler")
    for c in root.iter("statistic"):
        if "extent" in c.attrib:
            extent = float(c.attrib["extent"])
    for c in root.iter("map"):
        znear = float(c.attrib.get("znear", znear))
        zfar = float(c.attrib.get("zfar", zfar))
    ang = (math.pi / 180.0) if angle_deg else 1.0

    # ---- defaults
    defs = _Defaults()

    def walk_defaults(node, parent):
        name = node.attrib.get("class", "main")
        defs.add(name, parent, node)
        for ch in node:
            if ch.tag == "default":
                walk_defaults(ch, name)

    if "main" not in defs.classes:
        defs.classes["main"] = (None, {})
    for d in root.findall("default"):
        walk_defaults(d, "main" if d.attrib.get("class", "main") != "main" else None)

    def attrs_of(elem, cls):
        a = dict(defs.resolve(elem.attrib.get("class", cls), elem.tag))
        a.update(elem.attrib)
        return a

    # ---- assets: meshes and materials
    meshes = {}
    mesh_scales = {}
    materials = {}
    material_props = {}  # name -> texture, texrepeat, texuniform, specular, shininess, emission
    textures = {}  # name -> type, file (or builtin), rgb1, rgb2
    skybox = None
    for asset in root.findall("asset"):
        for m in asset:
            a = attrs_of(m, m.attrib.get("class", "main"))
            if m.tag == "mesh":
                name = a.get("name", os.path.splitext(os.path.basename(a["file"]))[0])
                meshes[name] = os.path.join(meshdir, a["file"])
                mesh_scales[name] = _floats(a.get("scale", "1 1 1"))
            elif m.tag == "material":
                materials[m.attrib["name"]] = _floats(a.get("rgba", "1 1 1 1"))
                material_props[m.attrib["name"]] = dict(
                    texture=a.get("texture"), texrepeat=(_floats(a.get("texrepeat", "1 1")) + [1.0])[:2],
                    texuniform=a.get("texuniform", "false") == "true", specular=float(a.get("specular", 0.5)),
                    shininess=float(a.get("shininess", 0.5)), emission=float(a.get("emission", 0.0)))
            elif m.tag == "texture":
                t = dict(type=a.get("type", "cube"), builtin=a.get("builtin", "none"),
                         rgb1=_floats(a.get("rgb1", "0.8 0.8 0.8")), rgb2=_floats(a.get("rgb2", "0.5 0.5 0.5")),
                         file=None)
                if "file" in a:
                    t["file"] = a["file"] if os.path.isabs(a["file"]) else os.path.join(texturedir, a["file"])
                if t["type"] == "skybox":
                    skybox = t
                else:
                    # MuJoCo names an unnamed file texture after its file
                    name = a.get("name", os.path.splitext(os.path.basename(a.get("file", "")))[0])
                    textures[name] = t

    def frame_quat(a):
        if "quat" in a:
            return quat_normalize(_floats(a["quat"]))
        if "euler" in a:
            return euler2quat(np.array(_floats(a["euler"])) * ang)
        if "axisangle" in a:
            v = _floats(a["axisangle"])
            return axisangle2quat(v[:3], v[3] * ang)
        if "zaxis" in a:
            return zaxis2quat(_floats(a["zaxis"]))
        return np.array([1.0, 0, 0, 0])

    # ---- body tree
    bodies = []  # dicts
    joints, geoms, sites, cams = [], [], [], []
    mesh_cache = {}

    def get_mesh(name):
        if name not in mesh_cache:
            p = meshes.get(name)
            if p is None or not os.path.exists(p):
                mesh_cache[name] = None
            else:
                mesh_cache[name] = load_mesh(p, mesh_scales[name])
        return mesh_cache[name]

    def add_body(node, parent, childclass):
        bid = len(bodies)
        if parent < 0:
            b = dict(name="world", parent=-1, pos=np.zeros(3), quat=np.array([1.0, 0, 0, 0]), inertial=None)
        else:
            b = dict(name=node.attrib.get("name", f"body{bid}"), parent=parent,
                     pos=np.array(_floats(node.attrib.get("pos", "0 0 0"))), quat=frame_quat(node.attrib), inertial=None)
        bodies.append(b)
        cc = node.attrib.get("childclass", childclass) if parent >= 0 else childclass
        for ch in node:
            if ch.tag == "inertial":
                a = ch.attrib
                q = frame_quat(a)
                I = np.diag(_floats(a["diaginertia"])) if "diaginertia" in a else None
                if I is None:
                    f = _floats(a["fullinertia"])
                    I = np.array([[f[0], f[3], f[4]], [f[3], f[1], f[5]], [f[4], f[5], f[2]]])
                R = quat2mat(q)
                b["inertial"] = (float(a["mass"]), np.array(_floats(a.get("pos", "0 0 0"))), R @ I @ R.T)
            elif ch.tag in ("joint", "freejoint"):
                a = attrs_of(ch, cc) if ch.tag == "joint" else dict(ch.attrib)
                jt = JNT_FREE if ch.tag == "freejoint" or a.get("type") == "free" else {
                    "hinge": JNT_HINGE, "slide": JNT_SLIDE, "ball": JNT_BALL}[a.get("type", "hinge")]
                rng = _floats(a["range"]) if "range" in a else [0.0, 0.0]
                limited = a.get("limited", "auto")
                limited = (("range" in a) if autolimits else False) if limited == "auto" else limited == "true"
                joints.append(dict(
                    name=a.get("name", ""), type=jt, body=bid,
                    pos=np.array(_floats(a.get("pos", "0 0 0"))),
                    axis=np.array(_floats(a.get("axis", "0 0 1"))) / np.linalg.norm(_floats(a.get("axis", "0 0 1"))),
                    range=np.array(rng) * (ang if jt == JNT_HINGE else 1.0), limited=bool(limited) and jt in (JNT_HINGE, JNT_SLIDE),
                    armature=float(a.get("armature", 0)), damping=float(a.get("damping", 0)),
                    stiffness=float(a.get("stiffness", 0)), springref=float(a.get("springref", 0)) * (ang if jt == JNT_HINGE else 1.0),
                    solref=_floats(a.get("solreflimit", "0.02 1")), solimp=(_floats(a.get("solimplimit", "0.9 0.95 0.001 0.5 2")) + [0.5, 2.0])[:5],
                    ref=float(a.get("ref", 0)) * (ang if jt == JNT_HINGE else 1.0)))
            elif ch.tag == "geom":
                a = attrs_of(ch, cc)
                gt = GEOM_TYPES[a.get("type", "sphere")]
                size = np.array((_floats(a.get("size", "0 0 0")) + [0, 0, 0])[:3])
                mesh = None
                mname = a.get("mesh")
                if mname is not None:
                    mesh = get_mesh(mname)
                q = frame_quat(a)
                rgba = materials.get(a.get("material"), None)
                if "rgba" in a:
                    rgba = _floats(a["rgba"])
                if rgba is None:
                    rgba = [0.5, 0.5, 0.5, 1.0]
                geoms.append(dict(
                    name=a.get("name", ""), type=gt, body=bid, size=size, mesh_name=mname, mesh=mesh,
                    pos=np.array(_floats(a.get("pos", "0 0 0"))), quat=q,
                    contype=int(a.get("contype", 1)), conaffinity=int(a.get("conaffinity", 1)),
                    condim=int(a.get("condim", 3)), priority=int(a.get("priority", 0)),
                    friction=(_floats(a.get("friction", "1 0.005 0.0001")) + [0.005, 0.0001])[:3],
                    solref=_floats(a.get("solref", "0.02 1")), solimp=(_floats(a.get("solimp", "0.9 0.95 0.001 0.5 2")) + [0.5, 2.0])[:5],
                    solmix=float(a.get("solmix", 1.0)), margin=float(a.get("margin", 0)), gap=float(a.get("gap", 0)),
                    mass=float(a["mass"]) if "mass" in a else None, density=float(a.get("density", 1000.0)),
                    group=int(a.get("group", 0)), rgba=np.array(rgba), material=a.get("material")))
            elif ch.tag == "site":
                a = attrs_of(ch, cc)
                sites.append(dict(name=a.get("name", ""), body=bid, pos=np.array(_floats(a.get("pos", "0 0 0"))), quat=frame_quat(a)))
            elif ch.tag == "camera":
                a = attrs_of(ch, cc)
                cams.append(dict(name=a.get("name", ""), body=bid, pos=np.array(_floats(a.get("pos", "0 0 0"))), quat=frame_quat(a),
                                 fovy=float(a.get("fovy", 45.0))))
        for ch in node:
            if ch.tag == "body":
                add_body(ch, bid, cc)

    for wb in root.findall("worldbody"):
        add_body(wb, -1, "main")
        break

    nbody = len(bodies)
    bname = [b["name"] for b in bodies]

    # ---- geom post-processing: mesh OBBs (collision) and missing meshes
    for g in geoms:
        g["exact_cylinder"] = convex_meshes
        if g["type"] == GEOM_MESH or (g["mesh_name"] is not None and g["type"] in (GEOM_CAPSULE, GEOM_BOX)):
            if g["mesh"] is None:
                # missing blob: box of the D435i housing (documented substitution)
                g["obb_center"] = np.zeros(3)
                g["obb_rot"] = np.eye(3)
                g["obb_half"] = np.array(missing_mesh_box)
                g["mesh_missing"] = True
            else:
                v = g["mesh"][0]
                lo, hi = v.min(0), v.max(0)
                g["obb_center"] = (lo + hi) / 2
                g["obb_rot"] = np.eye(3)
                g["obb_half"] = (hi - lo) / 2
                g["mesh_missing"] = False
            if (convex_meshes and g["type"] == GEOM_MESH and not g["mesh_missing"]
                    and (g["contype"] or g["conaffinity"])):
                hull = _convex_hull(g["mesh"])
                if hull is not None:
                    g["hull"], g["hull_com"] = hull
            if g["type"] == GEOM_CAPSULE:
                # capsule fitted to the mesh AABB along its longest axis (MuJoCo fitaabb-like)
                h = g["obb_half"]
                ax = int(np.argmax(h))
                r = float(np.max(np.delete(h, ax)))
                g["size"] = np.array([r, max(h[ax] - r, 0.0), 0.0])
                Rfit = np.eye(3)[:, [(ax + 1) % 3, (ax + 2) % 3, ax]]
                g["pos"] = g["pos"] + quat2mat(g["quat"]) @ g["obb_center"]
                g["quat"] = quat_normalize(quat_mul(g["quat"], mat2quat(Rfit)))
                g["fitted"] = True

    # ---- mass properties
    body_mass = np.zeros(nbody)
    body_ipos = np.zeros((nbody, 3))
    body_inertia = np.zeros((nbody, 9))
    for bid, b in enumerate(bodies):
        if bid == 0:
            continue
        if b["inertial"] is not None:
            m, c, I = b["inertial"]
        else:
            parts = []
            for g in geoms:
                if g["body"] != bid or g["type"] == GEOM_PLANE:
                    continue
                if g["mass"] == 0.0:
                    continue
                R = quat2mat(g["quat"])
                if g["type"] == GEOM_MESH or g.get("fitted"):
                    if g["type"] == GEOM_MESH and g["mesh"] is not None:
                        gm, gc, gI = geom_mass_props(GEOM_MESH, g["size"], g["density"], g["mesh"])
                    elif g["type"] == GEOM_MESH:
                        gm = g["density"] * 8 * np.prod(g["obb_half"])
                        gc, gI = g["obb_center"], box_inertia(gm, g["obb_half"])
                    else:
                        gm, gc, gI = geom_mass_props(g["type"], g["size"], g["density"])
                else:
                    gm, gc, gI = geom_mass_props(g["type"], g["size"], g["density"])
                if g["mass"] is not None and gm > 0:
                    gI = gI * (g["mass"] / gm)
                    gm = g["mass"]
                parts.append((gm, g["pos"] + R @ gc, R @ gI @ R.T))
            m = sum(p[0] for p in parts)
            if m > 0:
                c = sum(p[0] * p[1] for p in parts) / m
                I = np.zeros((3, 3))
                for pm, pc, pI in parts:
                    d = pc - c
                    I += pI + pm * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
            else:
                c, I = np.zeros(3), np.zeros((3, 3))
        body_mass[bid] = m
        body_ipos[bid] = c
        body_inertia[bid] = I.reshape(-1)

    # ---- joints / dofs / qpos layout
    body_jntadr = np.full(nbody, -1, np.int32)
    body_jntnum = np.zeros(nbody, np.int32)
    body_dofadr = np.full(nbody, -1, np.int32)
    body_dofnum = np.zeros(nbody, np.int32)
    jnt_qposadr, jnt_dofadr = [], []
    nq = nv = 0
    dof_body, dof_jnt, dof_parent = [], [], []
    last_dof_of_body = np.full(nbody, -1, np.int64)
    order = sorted(range(len(joints)), key=lambda j: joints[j]["body"])  # already in body order
    assert order == list(range(len(joints)))
    for j, jt in enumerate(joints):
        b = jt["body"]
        if body_jntadr[b] < 0:
            body_jntadr[b] = j
            body_dofadr[b] = nv
        body_jntnum[b] += 1
        jnt_qposadr.append(nq)
        jnt_dofadr.append(nv)
        nd = {JNT_FREE: 6, JNT_BALL: 3}.get(jt["type"], 1)
        nq += {JNT_FREE: 7, JNT_BALL: 4}.get(jt["type"], 1)
        for k in range(nd):
            # parent dof: previous dof in this body, else last dof of nearest ancestor with dofs
            if last_dof_of_body[b] >= 0:
                par = last_dof_of_body[b]
            else:
                p = bodies[b]["parent"]
                while p > 0 and last_dof_of_body[p] < 0:
                    p = bodies[p]["parent"]
                par = last_dof_of_body[p] if p > 0 else -1
            dof_body.append(b)
            dof_jnt.append(j)
            dof_parent.append(par)
            last_dof_of_body[b] = nv
            nv += 1
        body_dofnum[b] += nd

    # weld ids and root ids
    body_parent = np.array([b["parent"] for b in bodies], np.int32)
    body_weldid = np.zeros(nbody, np.int32)
    body_rootid = np.zeros(nbody, np.int32)
    for b in range(1, nbody):
        body_weldid[b] = b if body_jntnum[b] > 0 else body_weldid[body_parent[b]]
        body_rootid[b] = b if body_parent[b] == 0 else body_rootid[body_parent[b]]

    qpos0 = np.zeros(nq)
    for j, jt in enumerate(joints):
        a = jnt_qposadr[j]
        if jt["type"] == JNT_FREE:
            # free joint qpos0 = body pose in world (parent is world here)
            assert bodies[jt["body"]]["parent"] == 0
            qpos0[a : a + 3] = bodies[jt["body"]]["pos"]
            qpos0[a + 3 : a + 7] = bodies[jt["body"]]["quat"]
        elif jt["type"] == JNT_BALL:
            qpos0[a : a + 4] = [1, 0, 0, 0]
        else:
            qpos0[a] = jt["ref"]

    M = Model()
    M.missing_includes = missing or []
    M.dropped_bodies = dropped_bodies
    M.name = root.attrib.get("model", "")
    M.timestep = timestep
    M.gravity = gravity
    M.integrator = integrator
    M.extent = extent if extent is not None else 2.0
    M.znear, M.zfar = znear, zfar
    M.nq, M.nv, M.nbody, M.njnt = nq, nv, nbody, len(joints)
    M.body_name = bname
    M.body_parent = body_parent
    M.body_pos = np.array([b["pos"] for b in bodies])
    M.body_quat = np.array([b["quat"] for b in bodies])
    M.body_mass = body_mass
    M.body_ipos = body_ipos
    M.body_inertia = body_inertia
    M.body_jntadr, M.body_jntnum = body_jntadr, body_jntnum
    M.body_dofadr, M.body_dofnum = body_dofadr, body_dofnum
    M.body_weldid, M.body_rootid = body_weldid, body_rootid
    M.jnt_name = [j["name"] for j in joints]
    M.jnt_type = np.array([j["type"] for j in joints], np.int32)
    M.jnt_body = np.array([j["body"] for j in joints], np.int32)
    M.jnt_qposadr = np.array(jnt_qposadr, np.int32)
    M.jnt_dofadr = np.array(jnt_dofadr, np.int32)
    M.jnt_pos = np.array([j["pos"] for j in joints])
    M.jnt_axis = np.array([j["axis"] for j in joints])
    M.jnt_range = np.array([j["range"] for j in joints])
    M.jnt_limited = np.array([j["limited"] for j in joints], np.int32)
    M.jnt_stiffness = np.array([j["stiffness"] for j in joints])
    M.jnt_springref = np.array([j["springref"] for j in joints])
    M.jnt_solref = np.array([j["solref"] for j in joints])
    M.jnt_solimp = np.array([j["solimp"] for j in joints])
    M.dof_body = np.array(dof_body, np.int32)
    M.dof_jnt = np.array(dof_jnt, np.int32)
    M.dof_parent = np.array(dof_parent, np.int32)
    M.dof_armature = np.array([joints[j]["armature"] for j in dof_jnt])
    M.dof_damping = np.array([joints[j]["damping"] for j in dof_jnt])
    M.qpos0 = qpos0
    M.geoms = geoms
    M.textures, M.material_props, M.skybox = textures, material_props, skybox
    M.sites = sites
    M.cams = cams

    # ---- actuators, tendons, equality, sensors, excludes
    tendons = []
    for t in root.iter("tendon"):
        for fx in t:
            if fx.tag != "fixed":
                continue
            wr = [(M.jnt_name.index(j.attrib["joint"]), float(j.attrib.get("coef", 1))) for j in fx if j.tag == "joint"]
            tendons.append(dict(name=fx.attrib.get("name", ""), wraps=wr))
    M.tendons = tendons

    acts = []
    for act in root.findall("actuator"):
        for g in act:
            a = attrs_of(g, g.attrib.get("class", "main"))
            if g.tag not in ("general", "position", "motor"):
                continue
            if "joint" in a:
                trn, tid = TRN_JOINT, M.jnt_name.index(a["joint"])
            else:
                trn, tid = TRN_TENDON, [t["name"] for t in tendons].index(a["tendon"])
            gain = (_floats(a.get("gainprm", "1")) + [0, 0])[:3]
            bias = (_floats(a.get("biasprm", "0 0 0")) + [0, 0, 0])[:3]
            if a.get("biastype", "none") == "none":
                bias = [0.0, 0.0, 0.0]
            if g.tag == "position":  # MuJoCo shortcut: gain kp, affine bias (0, -kp, -kv)
                kp, kv = float(a.get("kp", 1)), float(a.get("kv", 0))
                gain, bias = [kp, 0.0, 0.0], [0.0, -kp, -kv]
            elif g.tag == "motor":  # gain 1 (gear 1), no bias
                gain, bias = [1.0, 0.0, 0.0], [0.0, 0.0, 0.0]
            cr = _floats(a["ctrlrange"]) if "ctrlrange" in a else [0, 0]
            fr = _floats(a["forcerange"]) if "forcerange" in a else [0, 0]
            acts.append(dict(name=a.get("name", ""), trn=trn, trnid=tid, gain=gain[0], bias=bias,
                             ctrlrange=cr, ctrllimited="ctrlrange" in a, forcerange=fr, forcelimited="forcerange" in a))
    M.actuators = acts
    M.nu = len(acts)

    eqs = []
    for eq in root.findall("equality"):
        for e in eq:
            a = dict(e.attrib)
            sr = _floats(a.get("solref", "0.02 1"))
            si = (_floats(a.get("solimp", "0.9 0.95 0.001 0.5 2")) + [0.5, 2.0])[:5]
            if e.tag == "weld":
                rp = _floats(a.get("relpose", "0 0 0 0 0 0 0"))
                eqs.append(dict(type=EQ_WELD, obj1=bname.index(a["body1"]), obj2=bname.index(a["body2"]),
                                anchor=_floats(a.get("anchor", "0 0 0")), relpose=rp, torquescale=float(a.get("torquescale", 1)),
                                solref=sr, solimp=si))
            elif e.tag == "connect":
                eqs.append(dict(type=EQ_CONNECT, obj1=bname.index(a["body1"]), obj2=bname.index(a["body2"]),
                                anchor=_floats(a["anchor"]), solref=sr, solimp=si))
            elif e.tag == "joint":
                eqs.append(dict(type=EQ_JOINT, obj1=M.jnt_name.index(a["joint1"]), obj2=M.jnt_name.index(a["joint2"]),
                                polycoef=(_floats(a.get("polycoef", "0 1 0 0 0")) + [0] * 5)[:5], solref=sr, solimp=si))
    M.equalities = eqs

    sens = []
    for s in root.findall("sensor"):
        for e in s:
            if e.tag in ("force", "torque"):
                sid = [x["name"] for x in sites].index(e.attrib["site"])
                sens.append(dict(name=e.attrib.get("name", ""), type=SENS_FORCE if e.tag == "force" else SENS_TORQUE, site=sid))
    M.sensors = sens

    excl = set()
    for c in root.findall("contact"):
        for e in c:
            if e.tag == "exclude":
                b1, b2 = bname.index(e.attrib["body1"]), bname.index(e.attrib["body2"])
                excl.add((min(b1, b2), max(b1, b2)))
    M.excludes = excl
    _contact_pairs(M)
    _set_const(M)
    return M


# ------------------------------------------------------------------------------------------
# static contact-pair filtering + parameter mixing (mj_collision filters, mj_contactParam)
# ------------------------------------------------------------------------------------------
def _convex_hull(mesh):
    """(hull vertices relative to the mesh's centre of mass, that centre) -- MuJoCo collides mesh
    geoms through the convex hull of their vertices (qhull; scipy wraps the same library), in
    the mesh frame it recentres at the mesh's centre of mass."""
    from scipy.spatial import ConvexHull

    verts, faces = mesh
    try:
        idx = np.sort(ConvexHull(verts).vertices)
    except Exception:  # degenerate (flat) mesh: keep the OBB substitute
        return None
    _, com, _ = mesh_mass_props(verts, faces)
    if not np.all(np.isfinite(com)):
        com = verts[idx].mean(0)
    return verts[idx] - com, com


def _collision_type(g):
    t = g["type"]
    if t == GEOM_MESH:
        return GEOM_MESH if "hull" in g else GEOM_BOX
    if t == GEOM_CYLINDER:
        return GEOM_CYLINDER if g.get("exact_cylinder") else GEOM_CAPSULE
    return t


def _contact_pairs(M):
    col = [i for i, g in enumerate(M.geoms) if g["contype"] or g["conaffinity"]]
    pairs = []
    for ii, g1 in enumerate(col):
        for g2 in col[ii + 1 :]:
            a, b = M.geoms[g1], M.geoms[g2]
            b1, b2 = a["body"], b["body"]
            w1, w2 = M.body_weldid[b1], M.body_weldid[b2]
            if w1 == w2:
                continue
            if not ((a["contype"] & b["conaffinity"]) or (b["contype"] & a["conaffinity"])):
                continue
            if w1 and w2 and (w1 == M.body_weldid[M.body_parent[w2]] or w2 == M.body_weldid[M.body_parent[w1]]):
                continue
            if (min(b1, b2), max(b1, b2)) in M.excludes:
                continue
            # OBB-substituted meshes inflate thin links: drop such pairs inside one kinematic
            # tree (e.g. gripper driver vs spring link), keep them against other objects.
            if (a["type"] == GEOM_MESH or b["type"] == GEOM_MESH) and M.body_rootid[b1] == M.body_rootid[b2]:
                continue
            pairs.append((g1, g2))
    M.pairs = pairs


def mix_contact_params(a, b):
    """mj_contactParam: priority wins, else max condim/friction and solmix-weighted solref/solimp."""
    if a["priority"] != b["priority"]:
        w = a if a["priority"] > b["priority"] else b
        return w["condim"], list(w["friction"]), list(w["solref"]), list(w["solimp"]), max(a["margin"], b["margin"]), max(a["gap"], b["gap"])
    condim = max(a["condim"], b["condim"])
    fr = [max(x, y) for x, y in zip(a["friction"], b["friction"])]
    s1, s2 = a["solmix"], b["solmix"]
    mix = 0.5 if (s1 + s2) <= 0 else s1 / (s1 + s2)
    sr = [mix * x + (1 - mix) * y for x, y in zip(a["solref"], b["solref"])]
    si = [mix * x + (1 - mix) * y for x, y in zip(a["solimp"], b["solimp"])]
    return condim, fr, sr, si, max(a["margin"], b["margin"]), max(a["gap"], b["gap"])


# ------------------------------------------------------------------------------------------
# numpy kinematics at qpos0 for mj_setConst-style constants
# ------------------------------------------------------------------------------------------
def kinematics(M, qpos):
    """Body world poses (xpos [nbody,3], xmat [nbody,3,3]) and joint anchors/axes."""
    xpos = np.zeros((M.nbody, 3))
    xmat = np.zeros((M.nbody, 3, 3))
    xmat[0] = np.eye(3)
    xanchor = np.zeros((M.njnt, 3))
    xaxis = np.zeros((M.njnt, 3))
    for b in range(1, M.nbody):
        p = M.body_parent[b]
        ja, jn = M.body_jntadr[b], M.body_jntnum[b]
        if jn and M.jnt_type[ja] == JNT_FREE:
            a = M.jnt_qposadr[ja]
            xpos[b] = qpos[a : a + 3]
            q = quat_normalize(qpos[a + 3 : a + 7])
            xmat[b] = quat2mat(q)
            xanchor[ja] = xpos[b]
            xaxis[ja] = [0, 0, 1]
            continue
        xpos[b] = xpos[p] + xmat[p] @ M.body_pos[b]
        R = xmat[p] @ quat2mat(M.body_quat[b])
        for j in range(ja, ja + jn):
            anc = xpos[b] + R @ M.jnt_pos[j]
            ax = R @ M.jnt_axis[j]
            xanchor[j], xaxis[j] = anc, ax
            if M.jnt_type[j] == JNT_HINGE:
                R = R @ quat2mat(axisangle2quat(M.jnt_axis[j], qpos[M.jnt_qposadr[j]] - M.qpos0[M.jnt_qposadr[j]]))
                xpos[b] = anc - R @ M.jnt_pos[j]
            elif M.jnt_type[j] == JNT_SLIDE:
                xpos[b] = xpos[b] + ax * (qpos[M.jnt_qposadr[j]] - M.qpos0[M.jnt_qposadr[j]])
        xmat[b] = R
    return xpos, xmat, xanchor, xaxis


def point_jacobian(M, xpos, xmat, xanchor, xaxis, body, point):
    """Translational and rotational Jacobians (3 x nv each) of a point fixed to `body`."""
    Jp = np.zeros((3, M.nv))
    Jr = np.zeros((3, M.nv))
    b = body
    while b > 0:
        for j in range(M.body_jntadr[b], M.body_jntadr[b] + M.body_jntnum[b]):
            d = M.jnt_dofadr[j]
            t = M.jnt_type[j]
            if t == JNT_HINGE:
                Jr[:, d] = xaxis[j]
                Jp[:, d] = np.cross(xaxis[j], point - xanchor[j])
            elif t == JNT_SLIDE:
                Jp[:, d] = xaxis[j]
            elif t == JNT_FREE:
                Jp[:, d : d + 3] = np.eye(3)
                R = xmat[b]
                for k in range(3):
                    ax = R[:, k]
                    Jr[:, d + 3 + k] = ax
                    Jp[:, d + 3 + k] = np.cross(ax, point - xpos[b])
        b = M.body_parent[b]
    return Jp, Jr


def mass_matrix(M, qpos):
    xpos, xmat, xanchor, xaxis = kinematics(M, qpos)
    H = np.zeros((M.nv, M.nv))
    for b in range(1, M.nbody):
        if M.body_mass[b] <= 0:
            continue
        c = xpos[b] + xmat[b] @ M.body_ipos[b]
        Jp, Jr = point_jacobian(M, xpos, xmat, xanchor, xaxis, b, c)
        Iw = xmat[b] @ M.body_inertia[b].reshape(3, 3) @ xmat[b].T
        H += M.body_mass[b] * Jp.T @ Jp + Jr.T @ Iw @ Jr
    H += np.diag(M.dof_armature)
    return H, (xpos, xmat, xanchor, xaxis)


def _set_const(M):
    H, (xpos, xmat, xanchor, xaxis) = mass_matrix(M, M.qpos0)
    Hinv = np.linalg.inv(H)
    M.meaninertia = float(np.mean(np.diag(H)))
    iw = np.zeros((M.nbody, 2))
    for b in range(1, M.nbody):
        if M.body_weldid[b] == 0:
            continue
        c = xpos[b] + xmat[b] @ M.body_ipos[b]
        Jp, Jr = point_jacobian(M, xpos, xmat, xanchor, xaxis, b, c)
        iw[b, 0] = max(np.trace(Jp @ Hinv @ Jp.T) / 3.0, 1e-15)
        iw[b, 1] = max(np.trace(Jr @ Hinv @ Jr.T) / 3.0, 1e-15)
    M.body_invweight0 = iw
    dinv = np.diag(Hinv).copy()
    for j in range(M.njnt):
        if M.jnt_type[j] == JNT_FREE:
            d = M.jnt_dofadr[j]
            dinv[d : d + 3] = dinv[d : d + 3].mean()
            dinv[d + 3 : d + 6] = dinv[d + 3 : d + 6].mean()
    M.dof_invweight0 = dinv
    # connect: anchor in body2 frame at qpos0
    for e in M.equalities:
        if e["type"] == EQ_CONNECT:
            p = xpos[e["obj1"]] + xmat[e["obj1"]] @ np.asarray(e["anchor"])
            e["anchor2"] = xmat[e["obj2"]].T @ (p - xpos[e["obj2"]])
        if e["type"] == EQ_WELD:
            rp = np.asarray(e["relpose"], np.float64)
            if np.all(rp[3:7] == 0):
                # relative pose at qpos0
                b1, b2 = e["obj1"], e["obj2"]
                rp[:3] = xmat[b1].T @ (xpos[b2] - xpos[b1])
                rp[3:7] = mat2quat(xmat[b1].T @ xmat[b2])
            e["relpose"] = list(rp[:3]) + list(quat_normalize(rp[3:7]))


# default material of a geom without one (mjsMaterial defaults, [ext] mujoco 3.1.6)
DEFAULT_SPECULAR, DEFAULT_SHININESS = 0.5, 0.5
TEX_2D, TEX_CUBE = 0, 1


def visual_arrays(M):
    """The renderer's material tables of a compiled model (csrc/rmbx_render.hip):

    * geom_texid i32 [ngeom]: texture of the geom's material (-1: none)
    * geom_matinfo f32 [ngeom, 6]: specular, shininess, texrepeat (2), texuniform, emission
    * tex_type i32 [ntex] (0: 2d, 1: cube; a single image on all six faces), tex_size i32 [ntex, 2]
      (height, width), tex_adr i32 [ntex] (first texel), tex_rgb u8 [texels, 3]: the texture files,
      decoded (common/image_io.decode_png), rows in file order
    * sky_rgb f64 [2, 3]: the builtin gradient skybox's rgb1 (up) / rgb2 (down); the default
      background of MuJoCo when there is none is black

    Only file textures and the gradient skybox are supported (the reference's scenes use nothing
    else); a material whose texture file is missing from the checkout keeps its colour only."""
    from ..common.image_io import decode_png

    tex_ids, tex_type, tex_size, tex_adr, texels = {}, [], [], [], []
    by_file = {}  # (file, type) -> texture index: one copy of an image several textures name
    adr = 0
    # textures the renderer samples: those of primitive geoms (a mesh's texture needs its UV
    # coordinates, which the render meshes do not carry: textured meshes keep their colour)
    used = {M.material_props[g["material"]]["texture"] for g in M.geoms
            if g["type"] != GEOM_MESH and g.get("material") in M.material_props}
    for name, t in M.textures.items():
        if (name not in used or t["file"] is None or not os.path.exists(t["file"])
                or t["type"] not in ("2d", "cube")):
            continue
        key = (os.path.realpath(t["file"]), t["type"])
        if key in by_file:
            tex_ids[name] = by_file[key]
            continue
        by_file[key] = len(tex_type)
        with open(t["file"], "rb") as f:
            img = decode_png(f.read())
        if img.shape[2] in (1, 2):
            img = np.repeat(img[..., :1], 3, axis=2)
        img = np.ascontiguousarray(img[..., :3])
        tex_ids[name] = len(tex_type)
        tex_type.append(TEX_2D if t["type"] == "2d" else TEX_CUBE)
        tex_size.append(img.shape[:2])
        tex_adr.append(adr)
        texels.append(img.reshape(-1, 3))
        adr += img.shape[0] * img.shape[1]
    ng = len(M.geoms)
    texid = np.full(ng, -1, np.int32)
    info = np.zeros((ng, 6), np.float32)
    for g, geom in enumerate(M.geoms):
        mp = M.material_props.get(geom.get("material"))
        if mp is None:
            info[g] = [DEFAULT_SPECULAR, DEFAULT_SHININESS, 1.0, 1.0, 0.0, 0.0]
            continue
        info[g] = [mp["specular"], mp["shininess"], mp["texrepeat"][0], mp["texrepeat"][1],
                   1.0 if mp["texuniform"] else 0.0, mp["emission"]]
        if mp["texture"] is not None and geom["type"] != GEOM_MESH:
            texid[g] = tex_ids.get(mp["texture"], -1)
    sky = np.zeros((2, 3))
    if M.skybox is not None and M.skybox["builtin"] == "gradient":
        sky[0], sky[1] = M.skybox["rgb1"], M.skybox["rgb2"]
    return {"geom_texid": texid, "geom_matinfo": info,
            "tex_type": np.array(tex_type, np.int32), "tex_size": np.array(tex_size, np.int32).reshape(-1, 2),
            "tex_adr": np.array(tex_adr, np.int32),
            "tex_rgb": np.concatenate(texels) if texels else np.zeros((0, 3), np.uint8), "sky_rgb": sky}
