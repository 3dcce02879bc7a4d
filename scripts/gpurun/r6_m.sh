#!/bin/bash
# round-6: counters of the two f16x3 attention kernels (register-staged vs LDS-DMA-staged)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6m
O=gpurun_out/r6m
for dma in 0 1; do
  export RMBX_ATTN_DMA=$dma
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/a$dma -o run -- python3 scripts/prof_attn_pmc.py > $O/a$dma.log 2>&1 || { tail -5 $O/a$dma.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/b$dma -o run -- python3 scripts/prof_attn_pmc.py > $O/b$dma.log 2>&1 || { tail -5 $O/b$dma.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for d in ("a0", "b0", "a1", "b1"):
    f = glob.glob(f"gpurun_out/r6m/{d}/**/*counter_collection.csv", recursive=True)
    if not f:
        print(d, "no csv"); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f[0])):
        n = r["Kernel_Name"]
        if "attn_fwd_f16x3" not in n: continue
        acc[n[:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for n, cs in acc.items():
        print(d, n, {c: round(sum(v) / max(1, len(set(r for r in range(len(v))))) / 1e6, 2) for c, v in cs.items()})
PY
