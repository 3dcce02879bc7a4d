"""Build a profiling variant of the library into robomanipbaselines_amd/_lib/librmbx_<name>.so
(loaded with RMBX_LIB_VARIANT=<name>; the product loads librmbx.so).  Variants:
  slp -- rmbx_gemm.hip without -fno-slp-vectorize (the SLP vectorizer's packed f32 split ops);
  render4 .. render7 -- rmbx_render.hip with its registers for 4 (unconstrained) .. 7 waves per
  SIMD (the default build targets 8);
  rsmall<N> -- rmbx_render.hip with RASTER_SMALL = N (pixel centres a lane covers itself);
  hoist -- rmbx_engine.hip with the solver's per-iteration addresses hoisted out of the Newton loop
  (RMBX_SOLVER_HOIST: the round-3 code generation, spilled at 128 registers);
  at-<rev> -- every csrc/*.hip source as of git revision <rev> (headers from the working tree): the
  A/B of a kernel change against the commit before it, on one box."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import build as B  # noqa: E402

name = sys.argv[1]
if name == "slp":
    B.FILE_FLAGS = {}
elif name in ("render4", "render5", "render6", "render7"):
    w = 1 if name == "render4" else int(name[-1])
    B.FILE_FLAGS = dict(B.FILE_FLAGS, **{"rmbx_render.hip": [f"-DRMBX_RENDER_MINW={w}"]})
elif name.startswith("rsmall"):
    B.FILE_FLAGS = dict(B.FILE_FLAGS, **{"rmbx_render.hip": [f"-DRASTER_SMALL={int(name[6:])}"]})
elif name == "hoist":
    B.FILE_FLAGS = dict(B.FILE_FLAGS, **{"rmbx_engine.hip": ["-DRMBX_SOLVER_HOIST"]})
elif name.startswith("at-"):
    rev = name[3:]
    tmp = os.path.join("/tmp", f"rmbx_src_{rev}")
    os.makedirs(tmp, exist_ok=True)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    srcs = []
    for f in sorted(os.listdir(B.CSRC)):
        if not (f.endswith(".hip") or f.endswith(".cpp")):
            continue
        r = subprocess.run(["git", "show", f"{rev}:robomanipbaselines_amd/csrc/{f}"], cwd=repo, capture_output=True)
        if r.returncode != 0:
            continue  # a source added after <rev>
        with open(os.path.join(tmp, f), "wb") as fh:
            fh.write(r.stdout)
        srcs.append(os.path.join(tmp, f))
    B._sources = lambda: srcs
else:
    raise SystemExit(f"unknown variant {name}")
B.LIB_PATH = os.path.join(B.LIB_DIR, f"librmbx_{name}.so")
print(B.build())
