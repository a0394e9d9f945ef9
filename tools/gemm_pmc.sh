#!/bin/bash
# PMC passes over tools/gemm_pmc.py (cram_gemm vs hipBLASLt at the gate/up sweep shape): one counter set per
# rocprofv3 run, kernel-trace only (MI355X_MICROARCH.md, rocprofv3 PMC slots).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/gemm_pmc
mkdir -p $OUT
run() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$name -o $name \
    -- python3 tools/gemm_pmc.py 29184 3 > $OUT/$name.log 2>&1
}
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
run p2 SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD TCC_HIT_sum TCC_MISS_sum
run p3 FETCH_SIZE
run p4 WRITE_SIZE
for f in $OUT/p*/p*_counter_collection.csv; do echo "== $f"; python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:60s} {c:26s} n={len(v):2d} mean={sum(v)/len(v):.4g}")
PY
done
