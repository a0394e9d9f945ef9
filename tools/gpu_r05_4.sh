set -e
export TMPDIR=/tmp
O=gpurun_out/r05/g4
mkdir -p $O
timeout -k 10 300 python -u tools/ab_silu_forms.py > $O/silu_forms.txt 2>&1
grep -v "Warning\|amdgpu.ids" $O/silu_forms.txt
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q -k small --timeout 120 --timeout-method thread > $O/small_tests.txt 2>&1
tail -2 $O/small_tests.txt
for m in 512 128; do
  timeout -k 10 300 python -u tools/decode_gemm_probe.py --M $m > $O/probe_llama3_M$m.txt 2>&1
  grep -v amdgpu.ids $O/probe_llama3_M$m.txt | python3 -c "
import sys,json
for l in sys.stdin:
    try: r=json.loads(l)
    except Exception: continue
    if r['method'].startswith(('sm','hipblaslt_decode','splitk8','w4')): print(r['shape'], r['M'], r['method'], r['us'])"
done
