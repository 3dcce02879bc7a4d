"""HBM traffic per launch from two rocprofv3 counter passes (FETCH_SIZE, WRITE_SIZE), calibrated.

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d <dir>/pmc_fetch -o run -- python3 scripts/prof_physics.py --calib
    rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d <dir>/pmc_write -o run -- python3 scripts/prof_physics.py --calib
    python tools/pmc_traffic.py <dir> --out profiles/rN_pmc_physics_traffic.json

Calibration (MI355X_MICROARCH.md §HBM: widths other than 16 B/lane are uncalibrated): the
`--calib` launches of scripts/pmc_calib.hip read and write exactly 512 MiB each with 8-B (f64)
and 16-B lanes; the read/write correction factors are known bytes / counted bytes of those
launches, and the physics kernels' medians are scaled by the 8-B factors (their access width).
"""

import argparse
import collections
import csv
import json
import os
import re
import statistics

CAL_BYTES = 512 << 20


def medians(path):
    vals = collections.defaultdict(list)
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].removeprefix("void ")
        vals[name].append(float(r["Counter_Value"]) * 1024.0)  # counters report KiB
        dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return ({k: statistics.median(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()},
            {k: statistics.median(v) for k, v in dur.items()})


def winograd(a):
    """--winograd: the Winograd launches of scripts/prof_winograd_pmc.py in dispatch order, 3 per
    layer shape (shapes and algorithmic bytes parsed from its log), scaled by the 16-B-lane factors
    (the kernel's global accesses are float4)."""
    def per_launch(path):
        rows = sorted((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0,
                       (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in csv.DictReader(open(path)))
        cal = [v for _, n, v, _ in rows if n.startswith("calib_f32x4")]
        return [(v, us) for _, n, v, us in rows if "wino" in n], statistics.median(cal)
    fetch, cf = per_launch(os.path.join(a.dir, "pmc_fetch", "run_counter_collection.csv"))
    write, cw = per_launch(os.path.join(a.dir, "pmc_write", "run_counter_collection.csv"))
    rf, wf = CAL_BYTES / cf, CAL_BYTES / cw
    shapes = re.findall(r"(f\d) C=(\d+) (\d+)x(\d+): algorithmic bytes per launch (\d+)",
                        open(os.path.join(a.dir, "fetch.log")).read())
    # a call over more elements than *_MAX_ELEMS runs as several launches (slices of whole frames):
    # traffic per call = sum over its launches
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from robomanipbaselines_amd import kernels as K
    frames = a.frames
    calls = []
    for tile, c, h, w, alg in shapes:
        lim = K.WINOGRAD4_MAX_ELEMS if tile == "f4" else K.WINOGRAD_MAX_ELEMS
        calls.append(-(-frames // max(1, lim // (int(h) * int(w) * int(c)))))
    assert len(fetch) == len(write) == 3 * sum(calls), (len(fetch), len(write), calls)
    out = {"calibration": {"x16_read_factor": rf, "x16_write_factor": wf}, "frames": frames, "layers": {}}
    i = 0
    for (tile, c, h, w, alg), L in zip(shapes, calls):
        rd = statistics.median(sum(v for v, _ in fetch[i + j * L:i + (j + 1) * L]) for j in range(3)) * rf
        wr = statistics.median(sum(v for v, _ in write[i + j * L:i + (j + 1) * L]) for j in range(3)) * wf
        us = statistics.median(sum(t for _, t in fetch[i + j * L:i + (j + 1) * L]) for j in range(3))
        i += 3 * L
        out["layers"][f"C{c}_{h}x{w}"] = {
            "tile": tile, "launches_per_call": L, "read_bytes_per_call": rd, "write_bytes_per_call": wr,
            "traffic_bytes_per_launch": (rd + wr) / L, "traffic_bytes_per_call": rd + wr,
            "algorithmic_bytes_per_call": int(alg), "traffic_over_algorithmic": (rd + wr) / int(alg),
            "median_us_per_call_under_pmc": us}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


def gemm(a, pattern=("gemm_f32x6", "gemm_f16x3_presplit"), kernel="rmbx::gemm_f32x6_kernel + rmbx::gemm_f16x3_presplit3_kernel"):
    """--gemm: the gemm_f32x6_kernel launches of the SECOND fp32 ACT inference of
    scripts/prof_act_gemm_pmc.py (dispatch order), scaled by the 16-B-lane factors (its global loads
    are dwordx4 and LDS-DMA of 16 B per lane): HBM bytes per launch, mean over the inference."""
    def per_launch(path):
        rows = sorted((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0,
                       (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in csv.DictReader(open(path)))
        cal = [v for _, n, v, _ in rows if n.startswith("calib_f32x4")]
        pats = (pattern,) if isinstance(pattern, str) else pattern
        g = [(v, us) for _, n, v, us in rows if any(q in n for q in pats)]
        assert len(g) % 2 == 0, len(g)
        return g[len(g) // 2:], statistics.median(cal)
    fetch, cf = per_launch(os.path.join(a.dir, "pmc_fetch", "run_counter_collection.csv"))
    write, cw = per_launch(os.path.join(a.dir, "pmc_write", "run_counter_collection.csv"))
    assert len(fetch) == len(write)
    rf, wf = CAL_BYTES / cf, CAL_BYTES / cw
    rd = sum(v for v, _ in fetch) * rf
    wr = sum(v for v, _ in write) * wf
    n = len(fetch)
    out = {"calibration": {"x16_read_factor": rf, "x16_write_factor": wf}, "kernel": kernel,
           "launches_per_inference": n, "read_bytes_per_inference": rd, "write_bytes_per_inference": wr,
           "traffic_bytes_per_launch": (rd + wr) / n,
           "us_per_inference_under_pmc": sum(t for _, t in fetch),
           "per_launch": [{"read_bytes": f[0] * rf, "write_bytes": w[0] * wf, "us_under_pmc": f[1]}
                          for f, w in zip(fetch, write)]}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "per_launch"}, indent=1))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--winograd", action="store_true", help="reduce scripts/gpurun/wino_pmc.sh output")
    p.add_argument("--gemm", action="store_true", help="reduce scripts/gpurun/gemm_pmc.sh output")
    p.add_argument("--convp", action="store_true",
                   help="the patch-staged conv dispatches of the same scripts/gpurun/gemm_pmc.sh output")
    p.add_argument("--frames", type=int, default=1024, help="--winograd: frames per call")
    p.add_argument("dir")
    p.add_argument("--out", required=True)
    p.add_argument("--kernels", nargs="+", default=["rmbx::front_kernel<false>", "rmbx::solver_kernel<4>"])
    p.add_argument("--launches_per_unit", type=int, default=8, help="launches of each kernel per env-step")
    p.add_argument("--units", type=int, default=1024, help="envs per launch")
    a = p.parse_args()
    if a.winograd:
        return winograd(a)
    if a.gemm:
        return gemm(a)
    if a.convp:
        return gemm(a, "conv3x3p_f16x3", "rmbx::conv3x3p_f16x3_kernel")
    fetch, nf, dur = medians(os.path.join(a.dir, "pmc_fetch", "run_counter_collection.csv"))
    write, nw, _ = medians(os.path.join(a.dir, "pmc_write", "run_counter_collection.csv"))
    cal = {
        "f64_read_factor": CAL_BYTES / fetch["calib_f64"], "f64_write_factor": CAL_BYTES / write["calib_f64"],
        "x16_read_factor": CAL_BYTES / fetch["calib_f32x4"], "x16_write_factor": CAL_BYTES / write["calib_f32x4"],
    }
    per = {}
    total = 0.0
    for k in a.kernels:
        rd = fetch[k] * cal["f64_read_factor"]
        wr = write[k] * cal["f64_write_factor"]
        per[k] = {"dispatches": nf[k], "fetch_size_raw_bytes": fetch[k], "write_size_raw_bytes": write[k],
                  "read_bytes": rd, "write_bytes": wr, "bytes_per_launch": rd + wr,
                  "bytes_per_env_per_launch": (rd + wr) / a.units, "median_us_under_pmc": dur[k],
                  "achieved_GBs_under_pmc": (rd + wr) / dur[k] / 1e3}
        total += (rd + wr) * a.launches_per_unit
    out = {"calibration": cal, "kernels": per, "bytes_per_env_step_all_envs": total,
           "bytes_per_env_step_per_env": total / a.units, "units_per_launch": a.units,
           "launches_per_env_step": {k: a.launches_per_unit for k in a.kernels}}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
