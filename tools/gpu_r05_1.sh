set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r05/g1
timeout -k 10 300 python -u tools/ab_gemm_builds.py tools/abbase/libcram_base.so cram_amd/libcram_attn.so 29184 7 > gpurun_out/r05/g1/ab_gemm.txt 2>&1
cat gpurun_out/r05/g1/ab_gemm.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "gemm or fused or silu or decode_routing or dist_gpu" > gpurun_out/r05/g1/tests.txt 2>&1
tail -5 gpurun_out/r05/g1/tests.txt
