#!/bin/bash
# rocprofv3 kernel-trace summaries: the IE sweep alone (its prefill_kernel average is the one bench.py's
# roofline reports) and the default bench (sweep + decode); then the attention PMC passes.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o sweep \
  -- python3 bench.py --no-cpu-baseline --no-decode > $R/gpurun_out/prof/sweep.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench \
  -- python3 bench.py --no-cpu-baseline > $R/gpurun_out/prof/bench.log 2>&1
find $R/gpurun_out/prof -name "*kernel_trace.csv" -delete
bash tools/pmc_attn.sh > $R/gpurun_out/pmc_summary.txt 2>&1
