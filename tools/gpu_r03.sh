#!/bin/bash
# Round-3 GPU call: the GPU suite (no -x: every failure is listed), then config-2 decode A/B of the split-K decode
# projection (CRAM_DECODE_GEMM on / off) with the leg roofline, then the Qwen2 decode GEMM probe.  Every GPU step has
# its own time limit; a step that times out or crashes ends the script (set -e).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03/${1:-run}
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/gputest.txt 2>&1 || echo "pytest rc=$?"
tail -5 $O/gputest.txt
timeout -k 10 300 python -u bench.py --config 2 --steps 2 --warmup 1 > $O/bench_c2.json 2> $O/bench_c2.err
head -c 400 $O/bench_c2.json; echo
CRAM_DECODE_GEMM=0 timeout -k 10 300 python -u bench.py --config 2 --steps 2 --warmup 1 > $O/bench_c2_nosplitk.json 2> $O/bench_c2_nosplitk.err
head -c 400 $O/bench_c2_nosplitk.json; echo
timeout -k 10 300 python -u tools/decode_gemm_probe.py --model qwen2 > $O/decode_gemm_probe_qwen2.jsonl 2> $O/probe.err
grep -c shape $O/decode_gemm_probe_qwen2.jsonl
