#!/bin/bash
# Same box: the Llama-3-8B-shape top-k noise-floor test and the IE-sweep bench line with the 4-wave kernel
# (CRAM_PREFILL_VARIANT=0) and with the automatic choice (x32).
set -o pipefail
O=gpurun_out/${1:-x32live}; mkdir -p $O
for v in 0 auto; do
  if [ $v = auto ]; then unset CRAM_PREFILL_VARIANT; else export CRAM_PREFILL_VARIANT=$v; fi
  timeout -k 10 400 python -u -m pytest tests/test_fullsize_ie_gpu.py -k "topk_sets_at_the_path_k or matches_fp32_truth" -s -q --timeout 300 --timeout-method thread > $O/fullsize_$v.txt 2>&1; echo "fullsize $v rc=$?"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-decode > $O/bench_$v.json 2> $O/bench_$v.err || exit $?
done
for v in 0 auto; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-decode > $O/bench2_$v.json 2> $O/bench2_$v.err || exit $?
done
