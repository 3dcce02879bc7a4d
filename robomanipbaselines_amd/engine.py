"""Host-side handle of the batched physics engine (C ABI rmbx_engine_*, include/rmbx.h).

Owns the torch device buffers bound to the engine (state, outputs, workspace) and exposes them
as zero-copy tensors.  All work is enqueued on the current torch stream.
"""

import ctypes

import numpy as np
import torch

from . import _native as N
from . import model as MD


class PhysicsEngine:
    def __init__(self, arrays, n_env, device="cuda:0"):
        self.arrays = arrays
        self.info = MD.ModelInfo(arrays)
        self.n_env = int(n_env)
        self.device = torch.device(device)
        a = arrays
        self.nq, self.nv, self.nu = int(a["_nq"]), int(a["_nv"]), int(a["_nu"])
        self.nbody, self.ngeom = int(a["_nbody"]), int(a["_ngeom"])
        self.timestep = float(a["_timestep"])
        self._cmodel = MD.as_ctypes(arrays)
        h = ctypes.c_void_p()
        N.call("rmbx_engine_create", ctypes.byref(self._cmodel), self.n_env, ctypes.byref(h))
        self._h = h
        nbytes = ctypes.c_size_t()
        N.call("rmbx_engine_workspace_bytes", self._h, ctypes.byref(nbytes))
        n, dev, f64 = self.n_env, self.device, torch.float64
        self.time = torch.zeros(n, dtype=f64, device=dev)
        self.qpos = torch.tensor(np.tile(a["qpos0"], (n, 1)), dtype=f64, device=dev)
        self.qvel = torch.zeros((n, self.nv), dtype=f64, device=dev)
        self.qacc_ws = torch.zeros((n, self.nv), dtype=f64, device=dev)
        # (a model without actuators still binds a non-NULL ctrl: a 1-column store viewed as 0)
        self._ctrl_store = torch.zeros((n, max(self.nu, 1)), dtype=f64, device=dev)
        self.ctrl = self._ctrl_store[:, : self.nu]
        self.body_pos = torch.tensor(np.tile(a["body_pos"].reshape(1, -1), (n, 1)), dtype=f64, device=dev).view(n, self.nbody, 3).contiguous()
        self.xpos = torch.zeros((n, self.nbody, 3), dtype=f64, device=dev)
        self.xquat = torch.zeros((n, self.nbody, 4), dtype=f64, device=dev)
        self.gxpos = torch.zeros((n, self.ngeom, 3), dtype=f64, device=dev)
        self.gxmat = torch.zeros((n, self.ngeom, 9), dtype=f64, device=dev)
        self.sensordata = torch.zeros((n, 6), dtype=f64, device=dev)
        self.stats = torch.zeros((n, 4), dtype=torch.int32, device=dev)
        self.workspace = torch.zeros(nbytes.value, dtype=torch.uint8, device=dev)
        assert self.workspace.data_ptr() % 256 == 0
        b = N.EnvBuffers()
        for name in ("time", "qpos", "qvel", "qacc_ws", "ctrl", "body_pos", "xpos", "xquat", "gxpos", "gxmat",
                     "sensordata", "stats", "workspace"):
            setattr(b, name, (self._ctrl_store if name == "ctrl" else getattr(self, name)).data_ptr())
        self._bufs = b
        N.call("rmbx_engine_bind", self._h, ctypes.byref(b))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                N.load().rmbx_engine_destroy(h)
            except Exception:
                pass
            self._h = None

    def step(self, nsub=8, active=None):
        if active is not None and (active.dtype != torch.uint8 or active.numel() != self.n_env):
            raise ValueError("active must be a uint8 tensor of n_env elements")
        N.call("rmbx_engine_step", self._h, int(nsub), N.ptr(active), N.stream_ptr())

    STAGES = ("kinematics", "com_crb", "velocity_rne_act", "collision", "constraints", "solver",
              "sensors", "integrate")
    # sub-stages of "solver" (slots 8..14)
    SOLVER_STAGES = ("smooth_factor_solve", "initial_costs", "gradient", "newton_factor_solve",
                     "line_search", "step_cost", "forces", "hessian")
    # sub-stages of "collision" (slots 16..18) and "constraints" (slots 20..23)
    COLLISION_STAGES = ("geom_records", "classify_compact", "narrow")
    CONSTRAINT_STAGES = ("count_zero", "equality", "limit_contact_rows", "aref")
    # J^T w (slots 24..27) and J x / M x (28..30) pass internals
    ROWPASS_STAGES = ("jtw_contact_wrench", "jtw_body_collect", "jtw_subtree", "jtw_dof",
                      "bodyvel_local", "bodyvel_prefix", "mass_tail")

    def step_profiled(self, nsub=8, raw=False):
        """Diagnostic step: returns mean shader cycles per stage (summed over substeps); with
        raw=True the [n_env, 32] per-env cycle array instead."""
        prof = torch.zeros((self.n_env, 32), dtype=torch.int64, device=self.device)
        N.call("rmbx_engine_step_profiled", self._h, int(nsub), N.ptr(prof), N.stream_ptr())
        if raw:
            return prof.cpu().numpy()
        p = prof.double().mean(0).cpu().numpy()
        out = dict(zip(self.STAGES, p[: len(self.STAGES)]))
        out.update({"solver." + k: v for k, v in zip(self.SOLVER_STAGES, p[8: 8 + len(self.SOLVER_STAGES)])})
        out.update({"collision." + k: v for k, v in zip(self.COLLISION_STAGES, p[16:19])})
        out.update({"constraints." + k: v for k, v in zip(self.CONSTRAINT_STAGES, p[20:24])})
        out.update({"rowpass." + k: v for k, v in zip(self.ROWPASS_STAGES, p[24:31])})
        out.update({"hessian.describe": p[19], "hessian.entries": p[31]})
        return out

    def forward(self, active=None):
        N.call("rmbx_engine_forward", self._h, N.ptr(active), N.stream_ptr())

    def _off(self, name):
        off, cnt = ctypes.c_size_t(), ctypes.c_size_t()
        N.call("rmbx_engine_ws_offset", self._h, name.encode(), ctypes.byref(off), ctypes.byref(cnt))
        return off.value, cnt.value

    def mass_matrix(self, name="Mblk"):
        """Dense [n_env, nv*nv] copy of the mass matrix (the engine keeps only the packed lower
        4x4 blocks the solver loads: block t = bi(bi+1)/2 + bj, entry 4p+q = M[4bi+p][4bj+q]);
        name="hsave": the Newton Hessian of the last build, in the same packing."""
        nv = self.nv
        nb = (nv + 3) // 4
        blk = self.ws(name).view(self.n_env, -1, 4, 4)
        full = torch.zeros((self.n_env, 4 * nb, 4 * nb), dtype=torch.float64, device=self.device)
        t = 0
        for bi in range(nb):
            for bj in range(bi + 1):
                full[:, 4 * bi: 4 * bi + 4, 4 * bj: 4 * bj + 4] = blk[:, t]
                t += 1
        low = torch.tril(full)
        full = low + low.transpose(1, 2) - torch.diag_embed(torch.diagonal(low, dim1=1, dim2=2))
        return full[:, :nv, :nv].reshape(self.n_env, nv * nv)

    def ws(self, name):
        """Zero-copy [n_env, count] f64 view of a named workspace array (after step/forward);
        "M" is the exception: a dense copy unpacked from the solver's blocks."""
        if name == "M":
            return self.mass_matrix()
        stride, _ = self._off("stride")
        off, cnt = self._off(name)
        return self.workspace.view(torch.float64).view(self.n_env, stride)[:, off : off + cnt]

    def wsi(self, name):
        """Zero-copy [n_env, count] int32 view of a named integer workspace array (con_b1, con_b2)."""
        stride, _ = self._off("stride")
        off, cnt = self._off(name)
        return self.workspace.view(torch.int32).view(self.n_env, 2 * stride)[:, off : off + cnt]
