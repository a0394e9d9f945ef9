set -e
export TMPDIR=/tmp
O=gpurun_out/r05/g5
mkdir -p $O
filt() { grep -v amdgpu.ids | python3 -c "
import sys,json
for l in sys.stdin:
    try: r=json.loads(l)
    except Exception: continue
    if r['method'].startswith(('sm1','sm2','sm4','hipblaslt_decode')): print(r['shape'], r['M'], r['method'], r['us'])"; }
for m in 512 128; do
  echo "== hot M=$m reg"; timeout -k 10 300 python -u tools/decode_gemm_probe.py --M $m --hot --only qkv,o_proj > $O/hot_reg_M$m.txt 2>&1; filt < $O/hot_reg_M$m.txt
  echo "== hot M=$m dma"; CRAM_SM_STAGING=dma timeout -k 10 300 python -u tools/decode_gemm_probe.py --M $m --hot --only qkv,o_proj > $O/hot_dma_M$m.txt 2>&1; filt < $O/hot_dma_M$m.txt
  echo "== cold M=$m dma"; CRAM_SM_STAGING=dma timeout -k 10 300 python -u tools/decode_gemm_probe.py --M $m --only qkv,o_proj > $O/cold_dma_M$m.txt 2>&1; filt < $O/cold_dma_M$m.txt
done
