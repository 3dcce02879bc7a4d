"""MFMA utilisation per kernel from a rocprofv3 pass of SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE
(+ --kernel-trace): busy = sum over the chip's SIMDs of their matrix-core busy cycles
(MI355X_MICROARCH.md: cycles = 16 per v_mfma_f32_16x16x32_*, 32 per 32x32x16); the dispatch's
cycles = GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs); utilisation = busy / (1024 SIMDs x
cycles), i.e. at the clock the chip held (DVFS), and that clock = cycles / wall time.
usage: python3 scripts/mfma_util.py <counter_collection.csv> [<kernel-name substring> ...]"""
import csv
import sys
from collections import defaultdict

SIMDS = 1024


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    rows = defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if pats and not any(p in name for p in pats):
            continue
        d = int(r["Dispatch_Id"])
        rows[d][r["Counter_Name"]] = float(r["Counter_Value"])
        short = name.replace("(anonymous namespace)::", "").removeprefix("void ")
        short = short[: short.index("(")] if "(" in short else short  # drop the argument list
        meta[d] = (short, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    agg = defaultdict(lambda: [0, 0.0, 0.0, 0.0])  # launches, busy, cycles, us
    for d in sorted(rows):
        c = rows[d]
        if "SQ_VALU_MFMA_BUSY_CYCLES" not in c or "GRBM_GUI_ACTIVE" not in c:
            continue
        name, us = meta[d]
        a = agg[name]
        a[0] += 1
        a[1] += c["SQ_VALU_MFMA_BUSY_CYCLES"]
        a[2] += c["GRBM_GUI_ACTIVE"] / 8.0
        a[3] += us
    print("kernel | launches | MFMA busy / (1024 SIMDs x cycles) | held clock GHz | us per launch")
    for name, (n, busy, cyc, us) in sorted(agg.items(), key=lambda kv: -kv[1][3]):
        print(f"{name} | {n} | {busy / (SIMDS * cyc):.3f} | {cyc / us / 1e3:.2f} | {us / n:.1f}")


if __name__ == "__main__":
    main()
