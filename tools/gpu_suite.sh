#!/bin/bash
# GPU suite (no -x: every failure is listed) + the default bench line; outputs under gpurun_out/<name>.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-suite}
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/gputest.txt 2>&1 || echo "pytest rc=$?"
tail -5 $O/gputest.txt
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err
head -c 600 $O/bench.json; echo
