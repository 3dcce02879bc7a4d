"""Build a profiling variant of the library into robomanipbaselines_amd/_lib/librmbx_<name>.so
(loaded with RMBX_LIB_VARIANT=<name>; the product loads librmbx.so).  Variants:
  slp -- rmbx_gemm.hip without -fno-slp-vectorize (the SLP vectorizer's packed f32 split ops);
  render4 .. render7 -- rmbx_render.hip with its registers for 4 (unconstrained) .. 7 waves per
  SIMD (the default build targets 8);
  hoist -- rmbx_engine.hip with the solver's per-iteration addresses hoisted out of the Newton loop
  (RMBX_SOLVER_HOIST: the round-3 code generation, spilled at 128 registers)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd import build as B  # noqa: E402

name = sys.argv[1]
if name == "slp":
    B.FILE_FLAGS = {}
elif name in ("render4", "render5", "render6", "render7"):
    w = 1 if name == "render4" else int(name[-1])
    B.FILE_FLAGS = dict(B.FILE_FLAGS, **{"rmbx_render.hip": [f"-DRMBX_RENDER_MINW={w}"]})
elif name == "hoist":
    B.FILE_FLAGS = dict(B.FILE_FLAGS, **{"rmbx_engine.hip": ["-DRMBX_SOLVER_HOIST"]})
else:
    raise SystemExit(f"unknown variant {name}")
B.LIB_PATH = os.path.join(B.LIB_DIR, f"librmbx_{name}.so")
print(B.build())
