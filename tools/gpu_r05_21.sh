set -e
export TMPDIR=/tmp
O=gpurun_out/r05/g21
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -k "splitk" -v --timeout 300 --timeout-method thread > $O/splitk_tests.txt 2>&1 || { tail -30 $O/splitk_tests.txt; exit 1; }
grep -cE "PASSED" $O/splitk_tests.txt
for m in llama3 qwen2; do
  for M in 512 128; do
    for w in 1 0; do
      CRAM_W4_SPLITK=$w timeout -k 10 300 python -u tools/decode_gemm_probe.py --model $m --M $M --only qkv,o_proj,down > $O/probe_${m}_M${M}_w4$w.txt 2>&1
      python - $O/probe_${m}_M${M}_w4$w.txt $w <<'PY'
import json, sys
best = {}
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    d = json.loads(l)
    k = d["shape"]
    if d["method"].startswith("splitk") or d["method"].startswith("hipblaslt_decode"):
        best.setdefault(k, []).append((d["us"], d["method"]))
print("w4", sys.argv[2], {k: sorted(v)[:3] for k, v in best.items()})
PY
    done
  done
done
