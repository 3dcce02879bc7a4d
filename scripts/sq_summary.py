"""Summarise rocprofv3 --pmc counter CSVs: per matching dispatch (in order), counter = value.
usage: python3 scripts/sq_summary.py <dir with p*/ runs> <kernel-name substring>"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root, pat = sys.argv[1], sys.argv[2]
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        rows = defaultdict(dict)
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if pat not in r.get("Kernel_Name", ""):
                    continue
                rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        print(f"# {os.path.relpath(f, root)}")
        for i, d in enumerate(sorted(rows)):
            print(f"launch {i}: " + ", ".join(f"{k}={v:.0f}" for k, v in sorted(rows[d].items())))
    print()


if __name__ == "__main__":
    main()
