#!/bin/bash
# x32 A/B (tools/ab_x64.hip: library kernel vs x64 vs x32, same inputs), x32 stamps at the sweep shape, the prefill
# parity tests on every variant; then (argument "suite") the whole GPU suite and the default bench line.
set -o pipefail
O=gpurun_out/${2:-x32a}; mkdir -p $O
timeout -k 10 120 tools/ab_x64 10 > $O/ab.txt 2>&1; rc=$?; echo "ab rc=$rc" >> $O/ab.txt
[ $rc -eq 0 -o $rc -eq 2 ] || exit $rc
timeout -k 10 60 tools/ab_x32_stamps 3 sweep > $O/stamps.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp16_gpu.py -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
if [ "$1" = "suite" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/gputest.txt 2>&1 || echo "pytest rc=$?"
  tail -3 $O/gputest.txt
  timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
  head -c 600 $O/bench.json; echo
fi
