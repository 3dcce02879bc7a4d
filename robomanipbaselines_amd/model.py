"""Packed model arrays (rmbx_model, include/rmbx_model.h) and their ctypes view.

`pack(M)` flattens a compiled MJCF model (mjcf/compiler.py) into named numpy arrays;
`save`/`load` keep them as a .npz asset (the GPU box has no reference checkout, so the
compiled scene ships in-tree under robomanipbaselines_amd/assets/); `as_ctypes(arrays)` builds
the C struct whose pointers reference those arrays.
"""

import ctypes
import os

import numpy as np

from .mjcf import compiler as C

ASSET_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")

I32 = np.int32
F64 = np.float64

_INT_FIELDS = ["nq", "nv", "nbody", "njnt", "ngeom", "nsite", "nu", "neq", "ntendon", "nwrap",
               "npair", "nsensor", "ncam", "solver_iterations", "ls_iterations", "max_contacts", "nhullvert"]
_DBL_FIELDS = ["timestep", ("gravity", 3), "meaninertia", "solver_tolerance", "extent", "znear", "zfar"]
# (name, dtype) in struct order
_PTR_FIELDS = [
    ("body_parent", I32), ("body_jntadr", I32), ("body_jntnum", I32), ("body_dofadr", I32),
    ("body_dofnum", I32), ("body_weldid", I32), ("body_rootid", I32),
    ("body_pos", F64), ("body_quat", F64), ("body_mass", F64), ("body_ipos", F64),
    ("body_inertia", F64), ("body_invweight0", F64),
    ("jnt_type", I32), ("jnt_body", I32), ("jnt_qposadr", I32), ("jnt_dofadr", I32), ("jnt_limited", I32),
    ("jnt_pos", F64), ("jnt_axis", F64), ("jnt_range", F64), ("jnt_stiffness", F64),
    ("jnt_springref", F64), ("jnt_solref", F64), ("jnt_solimp", F64),
    ("dof_body", I32), ("dof_jnt", I32), ("dof_parent", I32),
    ("dof_armature", F64), ("dof_damping", F64), ("dof_invweight0", F64),
    ("qpos0", F64),
    ("geom_type", I32), ("geom_body", I32), ("geom_ctype", I32),
    ("geom_size", F64), ("geom_pos", F64), ("geom_quat", F64), ("geom_rgba", F64),
    ("geom_csize", F64), ("geom_cpos", F64), ("geom_cquat", F64), ("geom_rbound", F64),
    ("pair_geom1", I32), ("pair_geom2", I32), ("pair_condim", I32),
    ("pair_friction", F64), ("pair_solref", F64), ("pair_solimp", F64), ("pair_margin", F64),
    ("site_body", I32), ("site_pos", F64), ("site_quat", F64),
    ("act_trntype", I32), ("act_trnid", I32), ("act_ctrllimited", I32), ("act_forcelimited", I32),
    ("act_gain", F64), ("act_bias", F64), ("act_ctrlrange", F64), ("act_forcerange", F64),
    ("ten_adr", I32), ("ten_num", I32), ("wrap_jnt", I32), ("wrap_coef", F64),
    ("eq_type", I32), ("eq_obj1", I32), ("eq_obj2", I32), ("eq_data", F64), ("eq_solref", F64),
    ("eq_solimp", F64),
    ("sensor_type", I32), ("sensor_site", I32),
    ("cam_body", I32), ("cam_pos", F64), ("cam_quat", F64), ("cam_fovy", F64),
    ("geom_hulladr", I32), ("geom_hullnum", I32), ("hull_vert", F64),
]


class RmbxModel(ctypes.Structure):
    _fields_ = (
        [(n, ctypes.c_int32) for n in _INT_FIELDS]
        + [(f, ctypes.c_double) if isinstance(f, str) else (f[0], ctypes.c_double * f[1]) for f in _DBL_FIELDS]
        + [(n, ctypes.c_void_p) for n, _ in _PTR_FIELDS]
    )


def pack(M, max_contacts=128, solver_iterations=100, ls_iterations=30, solver_tolerance=1e-8):
    a = {}
    a["body_parent"] = M.body_parent
    for k in ("jntadr", "jntnum", "dofadr", "dofnum", "weldid", "rootid"):
        a["body_" + k] = getattr(M, "body_" + k)
    a["body_pos"], a["body_quat"] = M.body_pos, M.body_quat
    a["body_mass"], a["body_ipos"], a["body_inertia"] = M.body_mass, M.body_ipos, M.body_inertia
    a["body_invweight0"] = M.body_invweight0
    for k in ("type", "body", "qposadr", "dofadr", "limited", "pos", "axis", "range", "stiffness",
              "springref", "solref", "solimp"):
        a["jnt_" + k] = getattr(M, "jnt_" + k)
    for k in ("body", "jnt", "parent", "armature", "damping", "invweight0"):
        a["dof_" + k] = getattr(M, "dof_" + k)
    a["qpos0"] = M.qpos0
    g = M.geoms
    a["geom_type"] = [x["type"] for x in g]
    a["geom_body"] = [x["body"] for x in g]
    a["geom_size"] = [x["size"] for x in g]
    a["geom_pos"] = [x["pos"] for x in g]
    a["geom_quat"] = [x["quat"] for x in g]
    a["geom_rgba"] = [x["rgba"] for x in g]
    ct, cs, cp, cq, rb = [], [], [], [], []
    for x in g:
        if not (x["contype"] or x["conaffinity"]):
            ct.append(-1)
            if x["type"] == C.GEOM_MESH and "obb_half" in x:  # visual mesh: its box (renderer)
                cs.append(np.asarray(x["obb_half"]))
                cp.append(x["pos"] + C.quat2mat(x["quat"]) @ x["obb_center"])
            else:
                cs.append(x["size"])
                cp.append(x["pos"])
            cq.append(x["quat"])
            rb.append(0.0)
            continue
        t = C._collision_type(x)
        if t == C.GEOM_MESH:  # convex hull, in its frame at the mesh's centre of mass
            size = np.abs(x["hull"]).max(0)
            pos = x["pos"] + C.quat2mat(x["quat"]) @ x["hull_com"]
            quat = x["quat"]
        elif x["type"] == C.GEOM_MESH:
            size = np.asarray(x["obb_half"])
            pos = x["pos"] + C.quat2mat(x["quat"]) @ x["obb_center"]
            quat = x["quat"]
        else:
            size, pos, quat = x["size"], x["pos"], x["quat"]
        ct.append(t)
        cs.append(size)
        cp.append(pos)
        cq.append(quat)
        if t == C.GEOM_SPHERE:
            rb.append(size[0])
        elif t == C.GEOM_CAPSULE:
            rb.append(size[0] + size[1])
        elif t == C.GEOM_BOX:
            rb.append(float(np.linalg.norm(size)))
        elif t == C.GEOM_CYLINDER:
            rb.append(float(np.hypot(size[0], size[1])))
        elif t == C.GEOM_MESH:
            rb.append(float(np.linalg.norm(x["hull"], axis=1).max()))
        else:
            rb.append(0.0)  # plane: unbounded
    a["geom_ctype"], a["geom_csize"], a["geom_cpos"], a["geom_cquat"], a["geom_rbound"] = ct, cs, cp, cq, rb
    hadr, hnum, hv = [], [], []
    for x, t in zip(g, ct):
        if t == C.GEOM_MESH:
            hadr.append(len(hv))
            hnum.append(len(x["hull"]))
            hv.extend(x["hull"])
        else:
            hadr.append(-1)
            hnum.append(0)
    a["geom_hulladr"], a["geom_hullnum"] = hadr, hnum
    a["hull_vert"] = np.asarray(hv, F64).reshape(-1, 3)
    p1, p2, cd, fr, sr, si, mg = [], [], [], [], [], [], []
    for i, j in M.pairs:
        condim, f, r, s, margin, gap = C.mix_contact_params(g[i], g[j])
        p1.append(i)
        p2.append(j)
        cd.append(condim)
        fr.append(f[:3])
        sr.append(r)
        si.append(s)
        mg.append(margin)
    a["pair_geom1"], a["pair_geom2"], a["pair_condim"] = p1, p2, cd
    a["pair_friction"], a["pair_solref"], a["pair_solimp"], a["pair_margin"] = fr, sr, si, mg
    a["site_body"] = [s["body"] for s in M.sites]
    a["site_pos"] = [s["pos"] for s in M.sites]
    a["site_quat"] = [s["quat"] for s in M.sites]
    acts = M.actuators
    a["act_trntype"] = [x["trn"] for x in acts]
    a["act_trnid"] = [x["trnid"] for x in acts]
    a["act_ctrllimited"] = [int(x["ctrllimited"]) for x in acts]
    a["act_forcelimited"] = [int(x["forcelimited"]) for x in acts]
    a["act_gain"] = [x["gain"] for x in acts]
    a["act_bias"] = [x["bias"] for x in acts]
    a["act_ctrlrange"] = [x["ctrlrange"] for x in acts]
    a["act_forcerange"] = [x["forcerange"] for x in acts]
    adr, num, wj, wc = [], [], [], []
    for t in M.tendons:
        adr.append(len(wj))
        num.append(len(t["wraps"]))
        for j, c in t["wraps"]:
            wj.append(j)
            wc.append(c)
    a["ten_adr"], a["ten_num"], a["wrap_jnt"], a["wrap_coef"] = adr, num, wj, wc
    et, o1, o2, ed, esr, esi = [], [], [], [], [], []
    for e in M.equalities:
        d = np.zeros(11)
        if e["type"] == C.EQ_CONNECT:
            d[0:3], d[3:6] = e["anchor"], e["anchor2"]
        elif e["type"] == C.EQ_WELD:
            d[0:3] = e["anchor"]
            d[3:10] = e["relpose"]
            d[10] = e["torquescale"]
        else:
            d[0:5] = e["polycoef"]
        et.append(e["type"])
        o1.append(e["obj1"])
        o2.append(e["obj2"])
        ed.append(d)
        esr.append(e["solref"])
        esi.append(e["solimp"])
    a["eq_type"], a["eq_obj1"], a["eq_obj2"], a["eq_data"], a["eq_solref"], a["eq_solimp"] = et, o1, o2, ed, esr, esi
    a["sensor_type"] = [s["type"] for s in M.sensors]
    a["sensor_site"] = [s["site"] for s in M.sensors]
    a["cam_body"] = [c["body"] for c in M.cams]
    a["cam_pos"] = [c["pos"] for c in M.cams]
    a["cam_quat"] = [c["quat"] for c in M.cams]
    a["cam_fovy"] = [c["fovy"] for c in M.cams]

    out = {}
    for name, dt in _PTR_FIELDS:
        arr = np.asarray(a[name], dtype=dt)
        if arr.size == 0:
            out[name] = np.ascontiguousarray(arr.reshape(0) if arr.ndim <= 1 else arr.reshape(0, int(np.prod(arr.shape[1:]))))
            continue
        out[name] = np.ascontiguousarray(arr.reshape(-1) if arr.ndim <= 1 else arr.reshape(arr.shape[0], -1))
    sizes = dict(nq=M.nq, nv=M.nv, nbody=M.nbody, njnt=M.njnt, ngeom=len(g), nsite=len(M.sites), nu=M.nu,
                 neq=len(M.equalities), ntendon=len(M.tendons), nwrap=len(a["wrap_jnt"]), npair=len(M.pairs),
                 nsensor=len(M.sensors), ncam=len(M.cams), solver_iterations=solver_iterations,
                 ls_iterations=ls_iterations, max_contacts=max_contacts, nhullvert=len(a["hull_vert"]))
    for k, v in sizes.items():
        out["_" + k] = np.int32(v)
    out["_timestep"] = np.float64(M.timestep)
    out["_gravity"] = np.asarray(M.gravity, F64)
    out["_meaninertia"] = np.float64(M.meaninertia)
    out["_solver_tolerance"] = np.float64(solver_tolerance)
    out["_extent"], out["_znear"], out["_zfar"] = np.float64(M.extent), np.float64(M.znear), np.float64(M.zfar)
    # names for lookups (host only)
    out["names_body"] = np.array(M.body_name)
    out["names_jnt"] = np.array(M.jnt_name)
    out["names_geom"] = np.array([x["name"] for x in g])
    out["names_site"] = np.array([s["name"] for s in M.sites])
    out["names_cam"] = np.array([c["name"] for c in M.cams])
    out["names_act"] = np.array([x["name"] for x in acts])
    # render-only attributes (not part of rmbx_model)
    out["geom_group"] = np.array([x["group"] for x in g], dtype=np.int32)
    out["cam_fovy_deg"] = np.array([c["fovy"] for c in M.cams], dtype=np.float64)
    return out


def save(arrays, path):
    np.savez_compressed(path, **arrays)


def load(name_or_path):
    path = name_or_path if os.path.exists(name_or_path) else os.path.join(ASSET_DIR, name_or_path + ".npz")
    with np.load(path, allow_pickle=False) as f:
        return _with_defaults({k: f[k] for k in f.files})


def _with_defaults(arrays):
    """Assets packed before the convex-hull fields existed: no hulls."""
    if "geom_hulladr" not in arrays:
        ng = int(arrays["_ngeom"])
        arrays["geom_hulladr"] = np.full(ng, -1, I32)
        arrays["geom_hullnum"] = np.zeros(ng, I32)
        arrays["hull_vert"] = np.zeros((0, 3), F64)
        arrays["_nhullvert"] = np.int32(0)
    return arrays


def as_ctypes(arrays):
    """rmbx_model struct referencing the arrays (keep `arrays` alive while it is used)."""
    arrays = _with_defaults(arrays)
    m = RmbxModel()
    for n in _INT_FIELDS:
        setattr(m, n, int(arrays["_" + n]))
    m.timestep = float(arrays["_timestep"])
    for i in range(3):
        m.gravity[i] = float(arrays["_gravity"][i])
    m.meaninertia = float(arrays["_meaninertia"])
    m.solver_tolerance = float(arrays["_solver_tolerance"])
    m.extent, m.znear, m.zfar = float(arrays["_extent"]), float(arrays["_znear"]), float(arrays["_zfar"])
    for name, dt in _PTR_FIELDS:
        arr = arrays[name]
        assert arr.dtype == dt and arr.flags.c_contiguous, name
        setattr(m, name, arr.ctypes.data if arr.size else None)
    return m


class ModelInfo:
    """Name lookups over packed arrays."""

    def __init__(self, arrays):
        self.a = arrays
        self.body = {n: i for i, n in enumerate(arrays["names_body"])}
        self.jnt = {n: i for i, n in enumerate(arrays["names_jnt"])}
        self.geom = {n: i for i, n in enumerate(arrays["names_geom"]) if n}
        self.site = {n: i for i, n in enumerate(arrays["names_site"]) if n}
        self.cam = {n: i for i, n in enumerate(arrays["names_cam"]) if n}
        self.nq, self.nv, self.nu = int(arrays["_nq"]), int(arrays["_nv"]), int(arrays["_nu"])

    def qposadr(self, jname):
        return int(self.a["jnt_qposadr"][self.jnt[jname]])

    def dofadr(self, jname):
        return int(self.a["jnt_dofadr"][self.jnt[jname]])
