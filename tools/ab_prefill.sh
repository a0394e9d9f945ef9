#!/bin/bash
# Same-box A/B of prefill-kernel variants (box-to-box spread is ~4 %, so compare only within one call):
# a build that switches kernels on CRAM_PREFILL_VARIANT, values in $@, sweep and 8k shapes, 3 rounds.
V=${@:-0 1 2}
for round in 1 2 3; do
  for v in $V; do
    echo "variant $v: $(CRAM_PREFILL_VARIANT=$v timeout -k 10 100 python tools/prof_attn.py) | $(CRAM_PREFILL_VARIANT=$v timeout -k 10 100 python tools/prof_attn.py --B 1 --T 8300)" || exit 1
  done
done
