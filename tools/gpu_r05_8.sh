set -e
export TMPDIR=/tmp
O=gpurun_out/r05/g8
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fullsize_ie_gpu.py -k "row_exact or matches_fp32" -v -s --timeout 300 --timeout-method thread > $O/rowexact.txt 2>&1
grep -E "PASSED|FAILED|ours-truth" $O/rowexact.txt
i=0
for arm in 1 0 1; do
  i=$((i+1))
  CRAM_SWEEP_ROW_EXACT=$arm timeout -k 10 400 python -u bench.py --no-decode --no-cpu-baseline > $O/sweep_${i}_re$arm.json 2> $O/sweep_$i.err
  python -c "import json,sys; d=json.loads(open('$O/sweep_${i}_re$arm.json').read().strip().splitlines()[-1]); print('arm', $arm, d['value'], d.get('roofline',{}).get('frac'))"
done
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err
head -c 1500 $O/bench.json
