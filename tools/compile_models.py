"""Compile the reference's MJCF scenes into packed model assets (run in the build container;
the GPU box has no reference checkout).  Output: robomanipbaselines_amd/assets/<name>.npz."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from robomanipbaselines_amd import model as MD  # noqa: E402
from robomanipbaselines_amd.mjcf import compiler as C  # noqa: E402
from robomanipbaselines_amd.mjcf import rmesh as MB  # noqa: E402

RENDER_MESH_CELL = 1e-3  # m: vertex-clustering grid of the render meshes (mjcf/rmesh.py)

REF_ENVS = "/root/reference/robo_manip_baselines/envs/assets/mujoco/envs"
SCENES = {"ur5e_cable": os.path.join(REF_ENVS, "ur5e", "env_ur5e_cable.xml"),
          "ur5e_insert": os.path.join(REF_ENVS, "ur5e", "env_ur5e_insert.xml"),
          "ur5e_door": os.path.join(REF_ENVS, "ur5e", "env_ur5e_door.xml"),
          "ur5e_cabinet": os.path.join(REF_ENVS, "ur5e", "env_ur5e_cabinet.xml"),
          "ur5e_toolbox": os.path.join(REF_ENVS, "ur5e", "env_ur5e_toolbox.xml"),
          "ur5e_pick": os.path.join(REF_ENVS, "ur5e", "env_ur5e_pick.xml"),
          "ur5e_ring": os.path.join(REF_ENVS, "ur5e", "env_ur5e_ring.xml")}
# per-scene compile options: every scene collides its mesh geoms (the gripper_collision class of
# ur5e_integrated_shared_config.xml:51-52, the scanned objects) through their convex hulls (MPR)
# and its cylinders exactly, as MuJoCo does; the Pick scene (BASELINE configs 4/5) drops the
# YCB_sim objects, absent from the checkout
OPTIONS = {name: dict(convex_meshes=True) for name in SCENES}
OPTIONS["ur5e_pick"] = dict(convex_meshes=True, skip_missing_includes=True)
PACK_OPTIONS = {"ur5e_pick": dict(max_contacts=200)}
UR5E_URDF = "/root/reference/robo_manip_baselines/envs/assets/common/robots/ur5e/ur5e.urdf"


def add_arm_ik(M, arrays, root_body="ur5e_root_frame"):
    """Pinocchio-equivalent joint placements of the UR5e URDF chain with the arm root pose read
    from the compiled MJCF at qpos0 (MujocoUR5eEnvBase.py:40-45, ArmManager.py:48-71)."""
    import numpy as np
    from robomanipbaselines_amd.mjcf import urdf

    xpos, xmat, _, _ = C.kinematics(M, M.qpos0)
    b = M.body_name.index(root_body)
    root = np.eye(4)
    root[:3, :3] = xmat[b]
    root[:3, 3] = xpos[b]
    P, axes, names = urdf.arm_chain(UR5E_URDF, 6, root)
    arrays["arm_placement"] = np.ascontiguousarray(np.concatenate([P[:, :3, :3].reshape(6, 9), P[:, :3, 3]], 1))
    arrays["arm_axis"] = np.ascontiguousarray(axes)
    arrays["arm_joint_names"] = np.array(names)

def add_visual(name, path):
    """Merge the renderer's material / texture tables (compiler.visual_arrays) into an existing
    asset, leaving every physics array as it is (checked: the geom order must be the compiled one)."""
    import numpy as np

    M = C.compile_mjcf(path, **OPTIONS.get(name, {}))
    out = os.path.join(MD.ASSET_DIR, name + ".npz")
    arrays = MD.load(out)
    names = [str(x) for x in arrays["names_geom"]]
    if names != [g["name"] for g in M.geoms] or not np.array_equal(arrays["geom_type"], [g["type"] for g in M.geoms]):
        raise RuntimeError(f"{name}: the asset's geoms are not the compiled model's: recompile the asset")
    arrays.update(C.visual_arrays(M))
    MD.save(arrays, out)
    print(name, "textures", len(arrays["tex_type"]), "textured geoms", int((arrays["geom_texid"] >= 0).sum()), "->", out,
          os.path.getsize(out), "bytes")


if __name__ == "__main__":
    os.makedirs(MD.ASSET_DIR, exist_ok=True)
    only = [a for a in sys.argv[1:] if not a.startswith("--")]
    if "--visual" in sys.argv:
        for name, path in SCENES.items():
            if not only or name in only:
                add_visual(name, path)
        sys.exit(0)
    for name, path in SCENES.items():
        if only and name not in only:
            continue
        M = C.compile_mjcf(path, **OPTIONS.get(name, {}))
        arrays = MD.pack(M, **PACK_OPTIONS.get(name, {}))
        add_arm_ik(M, arrays)
        # render meshes: the visual mesh geoms' triangles per body (1 mm vertex clustering)
        arrays.update(MB.render_meshes(M.geoms, cell=RENDER_MESH_CELL))
        # materials and textures of the renderer
        arrays.update(C.visual_arrays(M))
        out = os.path.join(MD.ASSET_DIR, name + ".npz")
        MD.save(arrays, out)
        print(name, "nq", M.nq, "nv", M.nv, "pairs", len(M.pairs), "->", out, os.path.getsize(out), "bytes")
