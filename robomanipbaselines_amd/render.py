"""Batched camera rendering front end (C ABI rmbx_render_scene).

Builds the drawing tables of a compiled scene and renders one camera for all envs of a
PhysicsEngine.  The geoms MuJoCo draws by default (groups 0-2) are drawn: primitive geoms as they
are (ray cast), visual mesh geoms as their triangles (scenes compiled with render meshes,
mjcf/rmesh.py: vertex-clustered at 1 mm, grouped per body; rasterised into a per-pixel visibility
buffer first), a mesh whose file is missing from the reference checkout as its bounding box;
material colours times the primitives' 2d / cube textures, the directional light's specular term,
flat-shaded triangles, the gradient skybox (include/rmbx.h rmbx_scene_tables; documented
substitution: images are not pixel-identical to MuJoCo's OpenGL renderer).  Assets packed without
render meshes fall back to the round-3 form (visual meshes drawn through their body's collision
primitives).
"""

import ctypes

import numpy as np
import torch

from . import _native as N
from .mjcf import compiler as C

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def build_prims(arrays):
    """(prim_i32 [nprim, 4], prim_f32 [nprim, 8]) of the scene (include/rmbx.h rmbx_scene_tables)."""
    if "rmesh_body" in arrays:
        return _build_prims_meshes(arrays)
    return _build_prims_substitutes(arrays)


def _build_prims_meshes(arrays):
    """Every geom of groups 0-2 except the visual meshes with render triangles (drawn by the
    visibility pass): primitives as they are, a mesh whose file is missing from the checkout as its
    bounding box."""
    gt, gg = arrays["geom_type"], arrays["geom_group"]
    ct, cs, size, rgba = arrays["geom_ctype"], arrays["geom_csize"], arrays["geom_size"], arrays["geom_rgba"]
    meshed = set(int(g) for g in arrays["rmesh_geoms"])
    pi, pf = [], []
    for g in range(len(gt)):
        t = int(gt[g])
        if gg[g] > 2 or g in meshed:
            continue
        if t in (C.GEOM_PLANE, C.GEOM_SPHERE, C.GEOM_CAPSULE, C.GEOM_CYLINDER, C.GEOM_BOX):
            pi.append([g, t, 0, 0])
            pf.append(list(size[g][:3]) + list(rgba[g][:3]) + [0, 0])
        elif t == C.GEOM_MESH and ct[g] < 0 and np.any(cs[g][:3] > 0):
            pi.append([g, C.GEOM_BOX, 0, 0])  # missing mesh file: its bounding box
            pf.append(list(cs[g][:3]) + list(rgba[g][:3]) + [0, 0])
    return np.array(pi, np.int32), np.array(pf, np.float32)


def _build_prims_substitutes(arrays):
    gt, gb, gg = arrays["geom_type"], arrays["geom_body"], arrays["geom_group"]
    ct, cs, size, rgba = arrays["geom_ctype"], arrays["geom_csize"], arrays["geom_size"], arrays["geom_rgba"]
    mesh_color = {}
    for g in range(len(gt)):
        if gt[g] == C.GEOM_MESH and gg[g] <= 2 and gb[g] not in mesh_color:
            mesh_color[int(gb[g])] = rgba[g][:3]
    pi, pf = [], []
    # visual meshes that carry their own bounding box (scenes packed with it) are drawn as that
    # box; the other mesh bodies through their collision primitives (boxes / capsules)
    boxed = {int(gb[g]) for g in range(len(gt))
             if gt[g] == C.GEOM_MESH and gg[g] <= 2 and ct[g] < 0 and np.any(cs[g][:3] > 0)}
    for g in range(len(gt)):
        t = int(gt[g])
        if t != C.GEOM_MESH and gg[g] <= 2 and t in (C.GEOM_PLANE, C.GEOM_SPHERE, C.GEOM_CAPSULE, C.GEOM_CYLINDER, C.GEOM_BOX):
            pi.append([g, t, 0, 0])
            pf.append(list(size[g][:3]) + list(rgba[g][:3]) + [0, 0])
        elif t == C.GEOM_MESH and gg[g] <= 2 and int(gb[g]) in boxed and ct[g] < 0:
            pi.append([g, C.GEOM_BOX, 0, 0])
            pf.append(list(cs[g][:3]) + list(rgba[g][:3]) + [0, 0])
        elif (ct[g] >= 0 and gg[g] >= 3 and int(gb[g]) in mesh_color and int(gb[g]) not in boxed
              and int(ct[g]) in (C.GEOM_SPHERE, C.GEOM_CAPSULE, C.GEOM_CYLINDER, C.GEOM_BOX)):
            typ = int(ct[g])
            pi.append([g, typ, 0, 0])
            pf.append(list(cs[g][:3]) + list(mesh_color[int(gb[g])]) + [0, 0])
    return np.array(pi, np.int32), np.array(pf, np.float32)


def mip_pyramid(img):
    """Level 0 = img [H, W, 3] (integers), then box-filtered halvings down to 1 x 1: level l is
    max(H >> l, 1) x max(W >> l, 1), texel (y, x) = (sum of the level above's rows 2y, 2y + 1 and
    columns 2x, 2x + 1, each clamped to its last row / column, + 2) // 4 -- the levels OpenGL's
    glGenerateMipmap box filter makes, in integers (include/rmbx.h rmbx_scene_tables)."""
    img = np.asarray(img, np.uint32)
    H, W = img.shape[:2]
    out = [img]
    l = 1
    while (H >> l) > 0 or (W >> l) > 0:
        prev = out[-1]
        h, w = max(H >> l, 1), max(W >> l, 1)
        ph, pw = prev.shape[:2]
        r0, r1 = np.minimum(2 * np.arange(h), ph - 1), np.minimum(2 * np.arange(h) + 1, ph - 1)
        c0, c1 = np.minimum(2 * np.arange(w), pw - 1), np.minimum(2 * np.arange(w) + 1, pw - 1)
        acc = (prev[r0][:, c0] + prev[r0][:, c1] + prev[r1][:, c0] + prev[r1][:, c1] + 2) // 4
        out.append(acc.astype(np.uint32))
        l += 1
    return out


class Renderer:
    def __init__(self, arrays, device, width=640, height=480):
        self.arrays = arrays
        pi, pf = build_prims(arrays)
        self.nprim = len(pi)
        self.prim_i32 = torch.tensor(pi, device=device)
        self.prim_f32 = torch.tensor(pf, device=device)
        self.device = torch.device(device)
        if "rmesh_body" in arrays:
            self.mesh_tri = torch.tensor(arrays["rmesh_tri"], dtype=torch.float32, device=device).contiguous()
            self.mesh_body = torch.tensor(arrays["rmesh_body"], dtype=torch.int32, device=device)
            self.mesh_rad = torch.tensor(arrays["rmesh_rad"], dtype=torch.float32, device=device)
        else:
            self.mesh_tri = self.mesh_body = self.mesh_rad = None
        self._vis = None  # visibility workspace u64 [n, H, W], allocated at the first render
        self._tflag = None  # tiles the visibility pass wrote, u8 [n, tiles]
        sc = N.SceneTables()
        sc.prim_i32, sc.prim_f32, sc.nprim = self.prim_i32.data_ptr(), self.prim_f32.data_ptr(), self.nprim
        if self.mesh_tri is not None:
            sc.ntri, sc.nmesh = self.mesh_tri.shape[0], self.mesh_body.shape[0]
            sc.mesh_tri, sc.mesh_body, sc.mesh_rad = (self.mesh_tri.data_ptr(), self.mesh_body.data_ptr(),
                                                      self.mesh_rad.data_ptr())
        # materials: texture, specular / shininess per geom, the texture images, the skybox
        # (compiler.visual_arrays; assets compiled before round 6 keep the flat shading)
        self.materials = "geom_matinfo" in arrays
        if self.materials:
            self.geom_texid = torch.tensor(arrays["geom_texid"], dtype=torch.int32, device=device)
            self.geom_matinfo = torch.tensor(arrays["geom_matinfo"], dtype=torch.float32, device=device).contiguous()
            # every texture with its box-filtered mip pyramid (the kernel samples trilinearly)
            desc = np.zeros((len(arrays["tex_type"]), 4), np.int32)
            ladr = np.zeros((max(1, len(desc)), N.TEX_LEVELS), np.int32)
            chunks, adr = [], 0
            for i in range(len(desc)):
                h, w = (int(x) for x in arrays["tex_size"][i])
                a0 = int(arrays["tex_adr"][i])
                base = np.asarray(arrays["tex_rgb"][a0:a0 + h * w], np.uint32).reshape(h, w, 3)
                levels = mip_pyramid(base)
                if len(levels) > N.TEX_LEVELS:
                    raise ValueError(f"texture {i}: {h} x {w} needs more than {N.TEX_LEVELS} mip levels")
                desc[i] = (int(arrays["tex_type"][i]), h, w, adr)
                rel = 0
                for l, lv in enumerate(levels):
                    ladr[i, l] = rel
                    chunks.append(lv.reshape(-1, 3))
                    rel += lv.shape[0] * lv.shape[1]
                adr += rel
            self.tex_level_adr = torch.tensor(ladr, device=device).contiguous()
            rgb = np.concatenate(chunks) if chunks else np.zeros((0, 3), np.uint32)
            words = rgb[:, 0] | (rgb[:, 1] << 8) | (rgb[:, 2] << 16) | np.uint32(255 << 24)
            self.tex_rgba = torch.tensor(words.view(np.int32), device=device) if len(words) else None
            self.tex_desc = torch.tensor(desc, device=device).contiguous() if len(desc) else None
            sc.geom_texid, sc.geom_matinfo = self.geom_texid.data_ptr(), self.geom_matinfo.data_ptr()
            sc.tex_rgba = self.tex_rgba.data_ptr() if self.tex_rgba is not None else None
            sc.tex_desc = self.tex_desc.data_ptr() if self.tex_desc is not None else None
            sc.tex_level_adr = self.tex_level_adr.data_ptr()
            sc.ntex = len(desc)
            for i, v in enumerate(np.asarray(arrays["sky_rgb"], np.float64).reshape(-1)):
                sc.sky_rgb[i] = float(v)
        self._scene = sc
        # static-background caches (rmbx_render_scene_cached): the primitives of bodies welded to the
        # world, one cache per world-fixed camera (allocated at its first render)
        if "body_weldid" in arrays and self.nprim:
            weld, gbody = np.asarray(arrays["body_weldid"]), np.asarray(arrays["geom_body"])
            mocap = set(int(b) for b in np.asarray(arrays["body_mocapid"]).nonzero()[0]) if "body_mocapid" in arrays else set()
            stat = np.array([1 if weld[gbody[g]] == 0 and int(gbody[g]) not in mocap else 0 for g in pi[:, 0]], np.uint8)
        else:
            stat = np.zeros(self.nprim, np.uint8)
        self.prim_static = torch.tensor(stat, device=device) if self.nprim else None
        self.static_prims = torch.tensor(np.nonzero(stat)[0].astype(np.int32), device=device)
        self._caches = {}
        self.width, self.height = width, height
        self.cam_names = [str(x) for x in arrays["names_cam"]]
        self.znear = float(arrays["_znear"]) * float(arrays["_extent"])
        self.zfar = float(arrays["_zfar"]) * float(arrays["_extent"])

    def camera(self, name):
        a = self.arrays
        i = self.cam_names.index(name)
        c = N.Camera()
        c.body = int(a["cam_body"][i])
        c.width, c.height = self.width, self.height
        c.fovy_deg = float(a["cam_fovy"][i])
        for k in range(3):
            c.pos[k] = float(a["cam_pos"][i][k])
        for k in range(4):
            c.quat[k] = float(a["cam_quat"][i][k])
        c.znear, c.zfar = self.znear, self.zfar
        for k in range(3):
            c.mean[k] = IMAGENET_MEAN[k]
            c.std[k] = IMAGENET_STD[k]
        return c

    def _cache(self, camera_name, cam, n):
        """The static-background cache of a world-fixed camera (include/rmbx.h rmbx_render_cache), or
        None (a camera on a moving body, a scene without static primitives)."""
        nst = int(self.static_prims.numel())
        weld = self.arrays["body_weldid"] if "body_weldid" in self.arrays else None
        if nst == 0 or weld is None or int(np.asarray(weld)[cam.body]) != 0:
            return None
        H, W = self.height, self.width
        ent = self._caches.get(camera_name)
        if ent is None or ent[0] != (n, H, W):
            buf = torch.empty(n * H * W * 2, dtype=torch.int32, device=self.device)
            snap = torch.full((n * (7 + 12 * nst),), float("nan"), dtype=torch.float64, device=self.device)
            dirty = torch.zeros(n, dtype=torch.uint8, device=self.device)
            c = N.RenderCache()
            c.prim_static, c.static_prims, c.nstatic = self.prim_static.data_ptr(), self.static_prims.data_ptr(), nst
            c.cache, c.snap, c.dirty = buf.data_ptr(), snap.data_ptr(), dirty.data_ptr()
            ent = ((n, H, W), c, buf, snap, dirty)
            self._caches[camera_name] = ent
        return ent[1]

    def render(self, engine, camera_name, rgb=None, depth=None, policy=None, active=None, mean=None, std=None,
               hit_geom=None):
        """Render `camera_name` for every env of `engine` into the given (optional) tensors:
        rgb u8 [n,H,W,3], depth f32 [n,H,W], policy bf16/f32 [n,3,H,W], hit_geom i32 [n,H,W] (the
        geom id of each pixel's surface, -1 for the background)."""
        cam = self.camera(camera_name)
        if mean is not None:
            for k in range(3):
                cam.mean[k] = float(mean[k])
                cam.std[k] = float(std[k])
        n, H, W = engine.n_env, self.height, self.width
        if rgb is not None:
            assert rgb.dtype == torch.uint8 and tuple(rgb.shape) == (n, H, W, 3) and rgb.is_contiguous()
        if depth is not None:
            assert depth.dtype == torch.float32 and tuple(depth.shape) == (n, H, W) and depth.is_contiguous()
        pdt = 0
        if policy is not None:
            assert policy.is_contiguous() and policy.dtype in (torch.float32, torch.bfloat16, torch.uint8)
            if tuple(policy.shape) == (n, H // 2, W // 2, 16):  # space-to-depth stem input
                pdt = {torch.bfloat16: 2, torch.float32: 3, torch.uint8: 4}[policy.dtype]
            elif policy.dtype == torch.uint8:
                raise ValueError("a uint8 policy tensor must be the space-to-depth form [n, H/2, W/2, 16]")
            else:
                assert tuple(policy.shape) == (n, 3, H, W)
                pdt = 1 if policy.dtype == torch.bfloat16 else 0
        if hit_geom is not None:
            assert hit_geom.dtype == torch.int32 and tuple(hit_geom.shape) == (n, H, W) and hit_geom.is_contiguous()
        if self.mesh_tri is not None:
            ntiles = -(-H // 16) * -(-W // 16)
            if self._vis is None or self._vis.shape[0] < n * H * W or self._tflag.shape[0] < n * ntiles:
                # empty on entry to every call (the call leaves them so): all-ones keys, zero flags
                self._vis = torch.full((n * H * W,), -1, dtype=torch.int64, device=self.device)
                self._tflag = torch.zeros(n * ntiles, dtype=torch.uint8, device=self.device)
            self._scene.vis, self._scene.tflag = self._vis.data_ptr(), self._tflag.data_ptr()
        cache = self._cache(camera_name, cam, n)
        try:
            N.call("rmbx_render_scene_cached", ctypes.byref(cam), ctypes.byref(self._scene),
                   N.ptr(engine.gxpos), N.ptr(engine.gxmat), N.ptr(engine.xpos), N.ptr(engine.xquat),
                   engine.ngeom, engine.nbody, N.ptr(rgb), N.ptr(depth), N.ptr(hit_geom), N.ptr(policy), pdt,
                   N.ptr(active), n, ctypes.byref(cache) if cache is not None else None, N.stream_ptr())
        except BaseException:
            # the ray-cast pass is what empties the workspaces again: if the call failed after the
            # visibility pass wrote them (or was interrupted between the launches), empty them here
            # so no later frame of this Renderer sees stale mesh hits
            if self._vis is not None:
                self._vis.fill_(-1)
                self._tflag.zero_()
            raise
