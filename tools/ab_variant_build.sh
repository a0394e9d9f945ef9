#!/bin/bash
# Build the WORKING TREE's library with extra compiler flags (A/B variants behind macros) into
# tools/abvar/libcram_$NAME.so (git-ignored, travels to the GPU box), for tools/ab_attn_builds.py / tools/ab_gemm_builds.py.
#   bash tools/ab_variant_build.sh NAME [-DFLAG=1 ...]
set -e
NAME=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/tools/abvar
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I $R/include "$@" \
  $R/cram_amd/csrc/cram_attn.hip $R/cram_amd/csrc/cram_fused.hip $R/cram_amd/csrc/cram_spans.cpp \
  $R/cram_amd/csrc/cram_gemm.hip -o $R/tools/abvar/libcram_$NAME.so
echo $R/tools/abvar/libcram_$NAME.so
