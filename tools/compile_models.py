"""Compile the reference's MJCF scenes into packed model assets (run in the build container;
the GPU box has no reference checkout).  Output: robomanipbaselines_amd/assets/<name>.npz."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from robomanipbaselines_amd import model as MD  # noqa: E402
from robomanipbaselines_amd.mjcf import compiler as C  # noqa: E402

REF_ENVS = "/root/reference/robo_manip_baselines/envs/assets/mujoco/envs"
SCENES = {"ur5e_cable": os.path.join(REF_ENVS, "ur5e", "env_ur5e_cable.xml")}

if __name__ == "__main__":
    os.makedirs(MD.ASSET_DIR, exist_ok=True)
    for name, path in SCENES.items():
        M = C.compile_mjcf(path)
        arrays = MD.pack(M)
        out = os.path.join(MD.ASSET_DIR, name + ".npz")
        MD.save(arrays, out)
        print(name, "nq", M.nq, "nv", M.nv, "pairs", len(M.pairs), "->", out, os.path.getsize(out), "bytes")
