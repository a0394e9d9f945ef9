#!/bin/bash
# Round-3 measurement call: the default bench line, a rocprofv3 kernel-trace summary of the sweep-only bench, and the
# attention PMC passes that profiles/attn_pmc.json is regenerated from (tagged with the kernel source hash).  Each GPU
# step has its own time limit; a failing step ends the script.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03/${1:-final}
mkdir -p $O
cd $R
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err
head -c 300 $O/bench.json; echo
mkdir -p $O/prof
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o sweep \
  -- python3 bench.py --no-cpu-baseline --no-decode > $O/prof/sweep.json 2> $O/prof/sweep.err
python3 tools/trace_gaps.py $O/prof > $O/prof/gaps.txt 2>&1 || true
find $O/prof -name "*kernel_trace.csv" -delete
OUT=$O/pmc bash tools/pmc_attn.sh > $O/pmc_summary.txt 2>&1
python3 tools/pmc_to_json.py $O/pmc > $O/attn_pmc.json
cp profiles/attn_pmc.json $O/attn_pmc_written.json
tail -5 $O/pmc_summary.txt
