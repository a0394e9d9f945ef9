#!/bin/bash
# Build the library of git revision $1 (default HEAD) into tools/ablib/libcram_base.so for tools/ab_attn_builds.py.
set -e
REV=${1:-HEAD}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p $T/cram_amd/csrc $T/include
for f in cram_amd/csrc/cram_attn.hip cram_amd/csrc/cram_fused.hip cram_amd/csrc/cram_spans.cpp include/cram_attn.h \
         $(git -C $R ls-tree --name-only $REV cram_amd/csrc/ | grep "\.inc$"); do
  git -C $R show $REV:$f > $T/$f
done
SRCS="$T/cram_amd/csrc/cram_attn.hip $T/cram_amd/csrc/cram_fused.hip $T/cram_amd/csrc/cram_spans.cpp"
if git -C $R cat-file -e $REV:cram_amd/csrc/cram_gemm.hip 2>/dev/null; then
  git -C $R show $REV:cram_amd/csrc/cram_gemm.hip > $T/cram_amd/csrc/cram_gemm.hip
  SRCS="$SRCS $T/cram_amd/csrc/cram_gemm.hip"
fi
OUTDIR=${OUTDIR:-$R/tools/ablib}
mkdir -p $OUTDIR
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I $T/include $SRCS -o $OUTDIR/libcram_base.so
rm -rf $T
echo $OUTDIR/libcram_base.so
