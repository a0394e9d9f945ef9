#!/bin/bash
# PMC passes for the sweep's dominant GEMM launch (gemm_w4_kernel, gate/up + SiLU-mul at M = 29,184): separate --pmc
# runs, kernel-trace only, the same counter sets as tools/pmc_attn.sh (MI355X_MICROARCH.md HBM / rocprofv3).
# MODE=lt KREGEX=Cijk: hipBLASLt's kernel for the same product (comparison); MODE=store: the plain-store epilogue.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-$R/gpurun_out/gemm_pmc}
mkdir -p $OUT
run() {
  name=$1; shift
  timeout -k 10 180 rocprofv3 --kernel-include-regex "${KREGEX:-gemm_w4_kernel}" --pmc "$@" --kernel-trace \
    --output-format csv -d $OUT/$name -o $name -- python3 tools/gemm_pmc.py 29184 4 ${MODE:-silu} > $OUT/$name.log 2>&1
}
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES
run p2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
run p3 FETCH_SIZE
run p4 WRITE_SIZE
run p5 TCC_HIT_sum TCC_MISS_sum SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32
if [ "${EXTRA:-0}" = 1 ]; then
  # the L2's fabric read requests by size (what FETCH_SIZE is derived from) and by destination, written requests:
  # a direct byte count of the beyond-L2 traffic, independent of FETCH_SIZE's gfx950 correction
  run p6 TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
  run p7 TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_GMI_32B_sum TCC_BUBBLE_sum TCC_EA0_WRREQ_64B_sum
fi
for f in $OUT/p*/p*_counter_collection.csv; do echo "== $f"; python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(f"{k:28s} dispatches={len(v):3d} mean={sum(v)/len(v):.4g}")
PY
done
