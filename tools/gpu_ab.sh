#!/bin/bash
# Prefill A/B call: same-process A/B of the working tree's library against tools/ablib/libcram_base.so (built by
# tools/ab_attn_builds.sh <rev>), the x32 stamps + in-kernel clock at the sweep shape, then the prefill parity tests.
# Argument 1: output name; argument 2 "tests" runs the kernel / fp16 GPU tests too.  Each GPU step has its own limit.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab/${1:-ab}
mkdir -p $O
cd $R
timeout -k 10 240 python -u tools/ab_attn_builds.py tools/ablib/libcram_base.so cram_amd/libcram_attn.so 7 > $O/ab_builds.txt 2>&1
cat $O/ab_builds.txt
timeout -k 10 120 tools/ab_x32_stamps 3 sweep > $O/stamps.txt 2>&1
cat $O/stamps.txt
if [ "$2" = "tests" ]; then
  timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp16_gpu.py -q -x --timeout 120 \
    --timeout-method thread > $O/tests.txt 2>&1
  tail -3 $O/tests.txt
fi
