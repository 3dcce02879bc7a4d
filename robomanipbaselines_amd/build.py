"""Build the in-tree HIP library `librmbx.so` (gfx950) with hipcc.

Every `csrc/*.hip` translation unit is compiled to an object (in parallel, cached by source
hash) and linked into `robomanipbaselines_amd/_lib/librmbx.so`.  The library is in-tree so it
travels to the GPU box with the repository snapshot.
"""

import concurrent.futures
import hashlib
import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_DIR = os.path.join(PKG_DIR, "_lib")
OBJ_DIR = os.path.join(REPO_DIR, "build", "obj")
INCLUDE = os.path.join(REPO_DIR, "include")
LIB_PATH = os.path.join(LIB_DIR, "librmbx.so")

ARCH = os.environ.get("RMBX_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
COMMON_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-I",
    INCLUDE,
    "-I",
    CSRC,
    "-Wall",
    "-Wno-unused-function",
    "-Wno-unused-variable",
]


def _sources():
    return sorted(
        os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip") or f.endswith(".cpp")
    )


def _headers_digest():
    h = hashlib.sha1()
    for d in (CSRC, INCLUDE):
        for f in sorted(os.listdir(d)):
            if f.endswith(".h") or f.endswith(".hpp") or f.endswith(".inc"):
                with open(os.path.join(d, f), "rb") as fh:
                    h.update(fh.read())
    return h.hexdigest()


# per-source extra flags: the GEMM's split runs beside the MFMAs, where the packed f32 ops the SLP
# vectorizer forms (v_pk_add_f32 / v_pk_mul_f32) cost more than the scalar pairs they replace
# (MI355X_MICROARCH.md, "price of one filler beside MFMAs")
FILE_FLAGS = {"rmbx_gemm.hip": ["-fno-slp-vectorize"],
              # the renderer's ray-cast kernel at 6 waves per SIMD (80 registers): with the textured
              # shading, 13.7 vs 14.3 ms per 1024-env front-camera call at 8 (64 registers, spills)
              # and 14.1 at 5 (profiles/r6_render_waves_ab.log)
              "rmbx_render.hip": ["-DRMBX_RENDER_MINW=6"],
              # the attention kernels rescale their MFMA accumulators in the online softmax: in the
              # VGPR form they are multiplied in place (the AGPR form moved 112 registers per key tile
              # through v_accvgpr_read / write)
              "rmbx_attn.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}


def _compile(src, hdr_digest, verbose):
    flags = COMMON_FLAGS + FILE_FLAGS.get(os.path.basename(src), [])
    with open(src, "rb") as fh:
        digest = hashlib.sha1(fh.read() + hdr_digest.encode() + " ".join(flags).encode())
    obj = os.path.join(OBJ_DIR, os.path.basename(src) + "." + digest.hexdigest()[:12] + ".o")
    if os.path.exists(obj):
        return obj
    cmd = [HIPCC, *flags, "-c", src, "-o", obj]
    if src.endswith(".hip"):
        cmd[1:1] = ["-x", "hip"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(verbose=False, jobs=None):
    """Compile every HIP source and link librmbx.so; return the library path."""
    os.makedirs(LIB_DIR, exist_ok=True)
    os.makedirs(OBJ_DIR, exist_ok=True)
    hdr = _headers_digest()
    srcs = _sources()
    jobs = jobs or min(8, len(srcs)) or 1
    with concurrent.futures.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr, verbose), srcs))
    tmp = LIB_PATH + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
