set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread -k "decode" > gpurun_out/dec_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/ab_decode_u.py 256 1024 > gpurun_out/dec_ab_llama.log 2>&1 || exit 1
AB_HEADS=28,4,128 timeout -k 10 120 python -u tools/ab_decode_u.py 256 1024 > gpurun_out/dec_ab_qwen.log 2>&1 || exit 1
AB_HEADS=32,8,128 AB_SPLITS=4 timeout -k 10 120 python -u tools/ab_decode_u.py 16 8400 > gpurun_out/dec_ab_c5.log 2>&1 || exit 1
