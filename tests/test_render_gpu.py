"""The batched renderer (rmbx_render_scene, csrc/rmbx_render.hip) against the brute-force f64 ray
caster of oracle/render_oracle.c, on the reference's visual meshes (row a15: the per-camera renders
of envs/mujoco/MujocoEnvBase.py:103-126).

For every camera of the Cable scene (front, side, hand) and three envs in different arm poses, the
GPU frame is sampled on a 64 x 48 grid (every 10th pixel centre) and compared pixel by pixel with
the oracle's ray through the same pixel centre: the surface hit (geom id, -1 for the background),
its camera depth, and the 8-bit colour.  The oracle tests every ray against every drawn primitive
and every triangle (no tiles, culling, ordering or BVH), so a culling, ordering, traversal or
indexing error of the kernel shows as a differing pixel.  A difference is accepted only where the
oracle itself is ambiguous: another geom's surface coincides with the hit within the depth
tolerance (coplanar parts, e.g. a gripper pad and its silicone layer), or rays jittered by +-0.02
pixel around the sample see another surface, a depth or a colour beyond the tolerances (a
silhouette or crease passing through the sample); such pixels must stay rare."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
STEP = 10
JIT = 0.02
DEPTH_RTOL, DEPTH_ATOL = 1e-4, 1e-5
RGB_TOL = 2


def _env_states():
    """A Cable rollout's env advanced through its reach phases; env 2's arm joints moved too."""
    from robomanipbaselines_amd.envs.operation.OperationMujocoUR5eCable import OperationMujocoUR5eCable
    from robomanipbaselines_amd.policy.mlp.rollout_mlp import RolloutMlp

    class Rollout(OperationMujocoUR5eCable, RolloutMlp):
        pass

    ro = Rollout(argv=["--num_envs", "3", "--device", DEV, "--world_idx_list", "0", "3", "5",
                       "--world_random_scale", "0.01", "0.01", "0.0"])
    ro.reset()
    for _ in range(40):  # Initial 1.0 s + part of Reach1: the arm moves towards the cable
        ro.step_once()
    eng = ro.env.engine
    q = eng.qpos.clone()
    q[2, :6] += torch.tensor([0.4, -0.3, 0.5, -0.6, 0.3, 0.8], dtype=torch.float64, device=DEV)
    eng.qpos.copy_(q)
    eng.forward()
    torch.cuda.synchronize()
    return ro.env


def _samples(W, H):
    xs = np.arange(STEP // 2, W, STEP)
    ys = np.arange(STEP // 2, H, STEP)
    X, Y = np.meshgrid(xs, ys)
    return X.reshape(-1), Y.reshape(-1)


@torch.no_grad()
def test_renderer_matches_the_brute_force_oracle_on_every_camera():
    from oracle import render as OR

    env = _env_states()
    arrays, eng, rnd = env.arrays, env.engine, env.renderer
    assert "rmesh_tri" in arrays and rnd.mesh_tri is not None  # the scene carries its visual meshes
    prims = OR.scene_prims(arrays)
    n, H, W = eng.n_env, rnd.height, rnd.width
    xs, ys = _samples(W, H)
    gx, gm = eng.gxpos.cpu().numpy(), eng.gxmat.cpu().numpy()
    bx, bq = eng.xpos.cpu().numpy(), eng.xquat.cpu().numpy()
    mesh_geoms = set(int(g) for g in arrays["rmesh_geoms"])
    # the scene's materials: every pixel of a textured geom samples its texture in both renderers
    assert "geom_matinfo" in arrays and rnd.materials
    textured = set(int(g) for g in np.nonzero(arrays["geom_texid"] >= 0)[0])
    report = []
    for cam in env.camera_names:
        rgb = torch.empty((n, H, W, 3), dtype=torch.uint8, device=DEV)
        depth = torch.empty((n, H, W), dtype=torch.float32, device=DEV)
        hit = torch.empty((n, H, W), dtype=torch.int32, device=DEV)
        rnd.render(eng, cam, rgb=rgb, depth=depth, hit_geom=hit)
        rgb, depth, hit = rgb.cpu().numpy(), depth.cpu().numpy(), hit.cpu().numpy()
        for e in range(n):
            pix = np.stack([xs + 0.5, ys + 0.5], 1)
            og, od, oc, od2 = OR.cast(arrays, prims, gx[e], gm[e], bx[e], bq[e], cam, W, H, pix, second=True)
            o8 = OR.to_u8(oc)
            gg, gd, g8 = hit[e, ys, xs], depth[e, ys, xs], rgb[e, ys, xs]
            bad = gg != og
            same = ~bad & (og >= 0)
            bad |= same & (np.abs(gd - od) > DEPTH_RTOL * np.abs(od) + DEPTH_ATOL)
            bad |= np.abs(g8.astype(int) - o8.astype(int)).max(1) > RGB_TOL
            amb = np.zeros(len(xs), bool)
            for k in np.nonzero(bad)[0]:
                if og[k] >= 0 and od2[k] - od[k] <= DEPTH_RTOL * od[k] + DEPTH_ATOL:
                    amb[k] = True  # a coincident surface of another geom: the pixel's geom is a tie
                    continue
                jit = np.array([[dx, dy] for dx in (-JIT, JIT) for dy in (-JIT, JIT)]) + pix[k]
                jg, jd, jc = OR.cast(arrays, prims, gx[e], gm[e], bx[e], bq[e], cam, W, H, jit)
                j8 = OR.to_u8(jc).astype(int)
                spread = (len(set(jg.tolist()) | {int(og[k])}) > 1
                          or np.abs(jd - od[k]).max() > DEPTH_RTOL * abs(od[k]) + DEPTH_ATOL
                          or np.abs(j8 - o8[k].astype(int)).max() > RGB_TOL)
                amb[k] = spread
            unexplained = np.nonzero(bad & ~amb)[0]
            mesh_frac = float(np.isin(og, list(mesh_geoms)).mean())
            tex_frac = float(np.isin(og, list(textured)).mean())
            report.append(f"{cam} env{e}: mesh pixels {mesh_frac:.3f}, textured pixels {tex_frac:.3f}, differing "
                          f"{int(bad.sum())}, all ambiguous in the oracle: {int(amb.sum())}")
            assert len(unexplained) == 0, (cam, e, [(int(xs[k]), int(ys[k]), int(gg[k]), int(og[k]), float(gd[k]),
                                                     float(od[k]), g8[k].tolist(), o8[k].tolist())
                                                    for k in unexplained[:8]])
            assert amb.sum() <= 0.02 * len(xs), (cam, e, int(amb.sum()))
            if cam == "front":
                assert mesh_frac > 0.01, (cam, e, mesh_frac)  # the arm's meshes are in the policy view
                assert tex_frac > 0.3, (cam, e, tex_frac)  # table, floor, poles, cable: textured
    print("\n" + "\n".join(report))


@torch.no_grad()
def test_rerender_after_motion_equals_a_fresh_renderer():
    """The visibility workspaces come back empty after every call (the ray-cast pass consumes every
    key and tile flag it reads): a Renderer that drew a camera, then draws it again after the arm has
    moved, produces bitwise the frame a fresh Renderer draws of the new state -- no stale mesh hits
    of the first frame survive -- on every camera."""
    from robomanipbaselines_amd.render import Renderer

    env = _env_states()
    eng, rnd = env.engine, env.renderer
    n, H, W = eng.n_env, rnd.height, rnd.width

    def frame(r, cam):
        rgb = torch.empty((n, H, W, 3), dtype=torch.uint8, device=DEV)
        depth = torch.empty((n, H, W), dtype=torch.float32, device=DEV)
        hit = torch.empty((n, H, W), dtype=torch.int32, device=DEV)
        r.render(eng, cam, rgb=rgb, depth=depth, hit_geom=hit)
        return rgb, depth, hit

    for cam in env.camera_names:
        before = frame(rnd, cam)
        q = eng.qpos.clone()
        q[:, :6] += torch.tensor([0.3, 0.2, -0.25, 0.4, -0.3, 0.5], dtype=torch.float64, device=DEV)
        eng.qpos.copy_(q)
        eng.forward()
        again = frame(rnd, cam)
        fresh = frame(Renderer(env.arrays, DEV, width=W, height=H), cam)
        for a, b in zip(again, fresh):
            assert torch.equal(a, b), cam
        assert not torch.equal(before[2], again[2]), cam  # the arm moved in the frame


@torch.no_grad()
def test_static_background_cache_equals_the_full_render(monkeypatch):
    """The static-background cache (rmbx_render_scene_cached: the primitives of bodies welded to the
    world drawn once per world-fixed camera and reused while their poses and the camera's hold)
    gives bitwise the frames of the full render (RMBX_RENDER_CACHE=0) -- rgb, depth, hit geom and the
    policy tensors -- when the cache is built, when it is reused after the arm moved, and when one
    env's static primitive moved (that env alone rebuilds it); the hand camera (on a moving body)
    keeps no cache."""
    env = _env_states()
    eng, rnd = env.engine, env.renderer
    n, H, W = eng.n_env, rnd.height, rnd.width
    assert int(rnd.static_prims.numel()) > 0

    def frame(cam, cached):
        monkeypatch.setenv("RMBX_RENDER_CACHE", "1" if cached else "0")
        rgb = torch.empty((n, H, W, 3), dtype=torch.uint8, device=DEV)
        depth = torch.empty((n, H, W), dtype=torch.float32, device=DEV)
        hit = torch.empty((n, H, W), dtype=torch.int32, device=DEV)
        s2d = torch.empty((n, H // 2, W // 2, 16), dtype=torch.uint8, device=DEV)
        chw = torch.empty((n, 3, H, W), dtype=torch.float32, device=DEV)
        rnd.render(eng, cam, rgb=rgb, depth=depth, hit_geom=hit)
        ent = rnd._caches.get(cam)
        dirty = ent[4].tolist() if (cached and ent is not None) else None  # the first call's rebuilds
        rnd.render(eng, cam, policy=s2d)
        rnd.render(eng, cam, policy=chw)
        torch.cuda.synchronize()
        return (rgb, depth, hit, s2d, chw), dirty

    def check(cam, what):
        (got, dirty), (want, _) = frame(cam, True), frame(cam, False)
        for name, a, b in zip(("rgb", "depth", "hit_geom", "s2d", "chw"), got, want):
            assert torch.equal(a, b), (cam, what, name, int((a != b).sum()))
        return dirty

    stat_geom = int(rnd.prim_i32[rnd.static_prims[-1], 0])
    for cam in env.camera_names:
        world_cam = int(env.arrays["body_weldid"][int(env.arrays["cam_body"][env.camera_names.index(cam)])]) == 0
        eng.forward()  # (undoes the previous camera's moved primitive before this camera's cache is built)
        dirty = check(cam, "cache built")
        assert (dirty is not None) == world_cam, cam
        if world_cam:
            assert dirty == [1, 1, 1], cam  # every cache built on first use
        q = eng.qpos.clone()
        q[:, :6] += torch.tensor([0.2, -0.15, 0.2, 0.3, -0.2, 0.4], dtype=torch.float64, device=DEV)
        eng.qpos.copy_(q)
        eng.forward()
        dirty = check(cam, "arm moved")
        if world_cam:
            assert dirty == [0, 0, 0], cam  # no env rebuilt its cache: only the arm moved
        eng.gxpos[1, stat_geom, 0] += 0.05  # one env's static primitive moves (a modify_world)
        dirty = check(cam, "static primitive moved")
        if world_cam:
            assert dirty == [0, 1, 0], cam
        dirty = check(cam, "after the rebuild")
        if world_cam:
            assert dirty == [0, 0, 0], cam
