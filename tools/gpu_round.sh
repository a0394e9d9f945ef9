#!/bin/bash
# One GPU call that re-verifies the tree: GPU test suite, smoke, default bench, a rocprofv3 kernel-trace summary of
# the sweep-only bench and the attention PMC passes.  Every step has its own time limit; the first failure ends it.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/round
mkdir -p $O
cd $R
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gputest.txt 2>&1
tail -3 $O/gputest.txt
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json | head -c 600; echo
if [ "${1:-}" = "prof" ]; then
  mkdir -p $O/prof
  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o sweep \
    -- python3 bench.py --no-cpu-baseline --no-decode > $O/prof/sweep.json 2> $O/prof/sweep.err
  find $O/prof -name "*kernel_trace.csv" -delete
  OUT=$O/pmc bash tools/pmc_attn.sh > $O/pmc_summary.txt 2>&1
fi
