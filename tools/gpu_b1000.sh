#!/bin/bash
# Decode leg batch size on one GPU: config 2 at 512 and 1000 prompts (NQ-1000 in one batch), config 4 at 1000, and
# config 5 (8.3k prompts, 16 per GPU) with the current kernels.  Each GPU step has its own limit.
set -e
export TMPDIR=/tmp
O=gpurun_out/b1000; mkdir -p $O
timeout -k 10 300 python -u bench.py --config 2 --no-cpu-baseline --decode-batch 512 > $O/c2_b512.json 2> $O/c2_b512.err
timeout -k 10 400 python -u bench.py --config 2 --no-cpu-baseline --decode-batch 1000 > $O/c2_b1000.json 2> $O/c2_b1000.err
timeout -k 10 400 python -u bench.py --config 4 --no-cpu-baseline --decode-batch 1000 > $O/c4_b1000.json 2> $O/c4_b1000.err
timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline --decode-batch 16 > $O/c5.json 2> $O/c5.err
python3 - <<'PY'
import json
for f in ("c2_b512", "c2_b1000", "c4_b1000", "c5"):
    d = json.load(open(f"gpurun_out/b1000/{f}.json"))
    dd = d.get("decode", d)
    lr = dd.get("leg_roofline") or {}
    print(f, d["value"], dd.get("batch_per_gpu"), "prefill ms", lr.get("prefill", {}).get("ms"),
          "step ms", lr.get("steps", {}).get("ms_per_step"))
PY
