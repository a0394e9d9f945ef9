set -e
export TMPDIR=/tmp
O=gpurun_out/r05/g24
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_fullsize_ie_gpu.py tests/test_gemm_gpu.py -k "answer_rows_only or rope or row_exact" -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
grep -cE "PASSED" $O/tests.txt
i=0
for arm in 1 0 1; do
  i=$((i+1))
  CRAM_LAST_Q_ROWS=$arm timeout -k 10 400 python -u bench.py --no-decode --no-cpu-baseline > $O/sweep_${i}_q$arm.json 2> $O/sweep_$i.err
  python -c "import json; d=json.loads(open('$O/sweep_${i}_q$arm.json').read().strip().splitlines()[-1]); print('arm', $arm, d['value'], d['roofline']['frac'])"
done
