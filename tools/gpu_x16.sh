#!/bin/bash
# prefill_x16_kernel (knob 5) against prefill_x32_kernel (knob 4): same-process A/B and agreement, then the prefill
# parity tests of the x16 variant (and x32 for reference).  Each GPU step has its own limit.
set -e
export TMPDIR=/tmp
O=gpurun_out/x16/${1:-a}; mkdir -p $O
timeout -k 10 120 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp16_gpu.py -q -x -k "x16" --timeout 100 \
  --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 200 python -u tools/ab_knob.py 4 5 7 > $O/ab.txt 2>&1; grep -v "amdgpu.ids" $O/ab.txt
