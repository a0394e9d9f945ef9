#!/bin/bash
# PMC passes of prefill_x64_kernel and prefill_kernel at one ab_x64 case (separate --pmc runs, kernel-trace only).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-$R/gpurun_out/pmc_x64}
CASE=${1:-sweep}
mkdir -p $OUT
run() {
  name=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-include-regex "prefill" --pmc "$@" --kernel-trace --output-format csv \
    -d $OUT/$name -o $name -- $R/tools/ab_x64 3 "$CASE" > $OUT/$name.log 2>&1
}
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES
run p2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
run p3 SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH
for f in $OUT/p*/p*_counter_collection.csv; do echo "== $f"; python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:42s} {c:28s} n={len(v):3d} mean={sum(v)/len(v):.4g}")
PY
done
