#!/bin/bash
# Decode projections at M = 512 rows (the bench's decode batch since session 5): TunableOp picks vs the default with
# cold caches, and the split-K kernel vs hipBLASLt per shape.  Each GPU step has its own limit.
set -e
export TMPDIR=/tmp
O=gpurun_out/m512; mkdir -p $O
timeout -k 10 400 python -u tools/tune_decode_gemms.py --m 512 --out $O/decode_gemms_m512.json > $O/tune.txt 2>&1
cat $O/tune.txt | grep -v Warning
timeout -k 10 200 python -u tools/decode_gemm_probe.py --model llama3 --M 512 > $O/probe_llama3.jsonl 2> $O/probe.err
timeout -k 10 200 python -u tools/decode_gemm_probe.py --model qwen2 --M 512 > $O/probe_qwen2.jsonl 2>> $O/probe.err
cat $O/probe_llama3.jsonl $O/probe_qwen2.jsonl
