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
import statistics

CAL_BYTES = 512 << 20


def medians(path):
    vals = collections.defaultdict(list)
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0]
        vals[name].append(float(r["Counter_Value"]) * 1024.0)  # counters report KiB
        dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return ({k: statistics.median(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()},
            {k: statistics.median(v) for k, v in dur.items()})


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--out", required=True)
    p.add_argument("--kernels", nargs="+", default=["rmbx::front_kernel", "rmbx::solver_kernel"])
    p.add_argument("--launches_per_unit", type=int, default=8, help="launches of each kernel per env-step")
    p.add_argument("--units", type=int, default=1024, help="envs per launch")
    a = p.parse_args()
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
