#!/bin/bash
# The GPU suite alone (no -x: every failure listed) + smoke(); outputs under gpurun_out/<name>.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-suite}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputest.txt 2>&1 || echo "pytest rc=$?"
tail -4 $O/gputest.txt
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; tail -2 $O/smoke.txt
