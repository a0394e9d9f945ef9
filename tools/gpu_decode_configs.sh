#!/bin/bash
# Decode-leg bench lines of configs 2, 4 and 5 at the reference's 100 new tokens (re_weighting.py:127).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/dec
timeout -k 10 280 python3 -u bench.py --config 2 --no-cpu-baseline > $R/gpurun_out/dec/c2.json 2> $R/gpurun_out/dec/c2.err || exit 1
timeout -k 10 280 python3 -u bench.py --config 4 --no-cpu-baseline > $R/gpurun_out/dec/c4.json 2> $R/gpurun_out/dec/c4.err || exit 1
timeout -k 10 280 python3 -u bench.py --config 5 --decode-batch 16 --no-cpu-baseline > $R/gpurun_out/dec/c5.json 2> $R/gpurun_out/dec/c5.err || exit 1
