#!/bin/bash
# Final evidence of a session: the decode / drop-in GPU tests touched by the engine, then tools/gpu_measure_r03.sh
# (default bench line, rocprofv3 sweep summary, attention PMC passes).  Each GPU step has its own limit.
set -e
export TMPDIR=/tmp
O=gpurun_out/r03/${1:-final}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_dropin_gpu.py tests/test_config4_gpu.py tests/test_fp16_gpu.py -q -x \
  --timeout 200 --timeout-method thread > $O/tests_engine.txt 2>&1; tail -2 $O/tests_engine.txt
bash tools/gpu_measure_r03.sh ${1:-final}
