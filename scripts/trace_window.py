"""Per-kernel totals over the last `--ms` milliseconds of a rocprofv3 kernel-trace CSV (the
bench's timed region: K steps x ms_per_step), grouped by kernel name.

    python scripts/trace_window.py gpurun_out/prof_bench/run_kernel_trace.csv --ms 1091 [--steps 30]

With `--marker NAME` the window is instead the span between the last two launches of kernel NAME
(bench.py launches torch's spin kernel around its timed loop when RMBX_TRACE_MARKERS=1).
"""
import argparse
import collections
import csv


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--ms", type=float, default=None)
    p.add_argument("--marker", default=None)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--top", type=int, default=40)
    a = p.parse_args()
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(a.trace))]
    if a.marker:
        marks = sorted(r for r in rows if a.marker in r[2])
        assert len(marks) >= 2, f"fewer than two {a.marker} launches in the trace"
        t0, end = marks[-2][1], marks[-1][0]
        a.ms = (end - t0) / 1e6
    else:
        end = max(r[1] for r in rows)
        t0 = end - a.ms * 1e6
    tot = collections.Counter()
    cnt = collections.Counter()
    for s, e, n in rows:
        if t0 <= s and e <= end and not (a.marker and a.marker in n):
            tot[n] += e - s
            cnt[n] += 1
    busy = sum(tot.values())
    print(f"window {a.ms:.1f} ms, kernel-busy {busy/1e6:.1f} ms ({100*busy/(a.ms*1e6):.1f}%), per step {busy/1e6/a.steps:.2f} ms")
    for n, v in tot.most_common(a.top):
        print(f"{v/1e6:9.2f} ms {100*v/busy:5.1f}% per-step {v/1e6/a.steps:7.3f} ms n={cnt[n]:>5} avg={v/cnt[n]/1e3:9.1f}us  {n[:100]}")


if __name__ == "__main__":
    main()
