#!/bin/bash
# Build the library with each CRAM_SILU_FORM (cram_silu.inc) into tools/absilu/libcram_f<form>.so for
# tools/ab_silu_forms.py (accuracy against torch's silu and the fused gate/up GEMM's time, one process).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/tools/absilu
for f in 0 1 2 3; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DCRAM_SILU_FORM=$f -I $R/include \
    $R/cram_amd/csrc/cram_attn.hip $R/cram_amd/csrc/cram_fused.hip $R/cram_amd/csrc/cram_gemm.hip \
    $R/cram_amd/csrc/cram_spans.cpp -o $R/tools/absilu/libcram_f$f.so &
done
wait
ls $R/tools/absilu
