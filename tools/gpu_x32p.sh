#!/bin/bash
# Persistent x32 (knob 5) vs one-shot x32 (knob 4): same-process A/B + bit identity, then the prefill parity tests on
# every variant (incl. x32p) and the x32p identity test.  Each GPU step has its own limit.
set -e
export TMPDIR=/tmp
O=gpurun_out/x32p/${1:-a}; mkdir -p $O
timeout -k 10 200 python -u tools/ab_knob.py 4 5 7 > $O/ab.txt 2>&1; grep -v "amdgpu.ids" $O/ab.txt
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp16_gpu.py -q -x --timeout 150 \
  --timeout-method thread > $O/tests.txt 2>&1; tail -3 $O/tests.txt
