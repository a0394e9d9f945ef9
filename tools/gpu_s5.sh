#!/bin/bash
# Round-3 session-5 start: the GPU suite (no -x: every failure is listed), then tools/gpu_measure_r03.sh (bench line,
# rocprofv3 sweep summary, attention PMC passes -> attn_pmc.json for the current kernel build).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03/${1:-s5}
mkdir -p $O
cd $R
if [ "${2:-suite}" = "suite" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputest.txt 2>&1 || echo "pytest rc=$?"
  tail -3 $O/gputest.txt
fi
bash tools/gpu_measure_r03.sh ${1:-s5}
