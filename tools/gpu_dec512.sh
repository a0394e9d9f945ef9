#!/bin/bash
# Kernel trace of one batched generate at 512 prompts x 100 tokens (config 2) and the per-step breakdown of its steps.
set -e
export TMPDIR=/tmp
O=gpurun_out/dec512; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o gen \
  -- python3 tools/prof_generate.py --B 512 --new 100 --reps 1 > $O/gen.log 2>&1
python3 tools/decode_step_breakdown.py $O/prof > $O/steps.txt
cat $O/steps.txt
find $O/prof -name "*kernel_trace.csv" -delete
