#!/bin/bash
# M = 512 decode follow-up: numerics of every decode pin (incl. the new lm_head M = 512 picks), the decode / GEMM /
# drop-in GPU tests, and the config-2 / config-4 decode legs at 512 prompts per GPU.  Each GPU step has its own limit.
set -e
export TMPDIR=/tmp
O=gpurun_out/m512b; mkdir -p $O
timeout -k 10 200 python -u tools/check_decode_pins.py > $O/check_pins.txt 2>&1; grep -v Warn $O/check_pins.txt | tail -12
timeout -k 10 500 python -u -m pytest tests/test_gemm_gpu.py tests/test_dropin_gpu.py tests/test_config4_gpu.py -q -x \
  --timeout 200 --timeout-method thread > $O/tests.txt 2>&1; tail -2 $O/tests.txt
timeout -k 10 300 python -u bench.py --config 2 --no-cpu-baseline > $O/c2.json 2> $O/c2.err
timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline > $O/c4.json 2> $O/c4.err
python3 - <<'PY'
import json
for c in (2, 4):
    d = json.load(open(f"gpurun_out/m512b/c{c}.json"))
    print(c, d["value"], d.get("decode", {}).get("batch_per_gpu"), json.dumps(d.get("decode", {}).get("leg_roofline")))
PY
