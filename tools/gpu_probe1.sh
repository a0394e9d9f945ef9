#!/bin/bash
# MFMA-shape probe (attention-shaped step, both bf16 shapes, clock) and the config-2 decode leg at 256 / 512 prompts
# per GPU on one box.  Each GPU step has its own limit; a failing step ends the script.
set -e
export TMPDIR=/tmp
O=gpurun_out/probe1; mkdir -p $O
timeout -k 10 120 tools/mfma_shape_probe 400 > $O/shape.txt 2>&1; cat $O/shape.txt
timeout -k 10 300 python -u bench.py --config 2 --no-cpu-baseline --decode-batch 256 > $O/c2_b256.json 2> $O/c2_b256.err
timeout -k 10 400 python -u bench.py --config 2 --no-cpu-baseline --decode-batch 512 > $O/c2_b512.json 2> $O/c2_b512.err
python3 - <<'PY'
import json
for b in (256, 512):
    d = json.load(open(f"gpurun_out/probe1/c2_b{b}.json"))
    dd = d.get("decode", d)
    print(b, dd.get("value"), json.dumps(dd.get("leg_roofline")))
PY
