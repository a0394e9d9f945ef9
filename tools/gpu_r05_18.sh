set -e
export TMPDIR=/tmp
O=gpurun_out/r05/g18
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_config4_gpu.py -v --timeout 300 --timeout-method thread > $O/c4tests.txt 2>&1 || { tail -30 $O/c4tests.txt; exit 1; }
grep -E "PASSED|FAILED" $O/c4tests.txt
for arm in 1 0; do
  CRAM_DECODE_MLP_TAIL=$arm timeout -k 10 700 python -u bench.py --config 4 --no-cpu-baseline > $O/c4_tail$arm.json 2> $O/c4_tail$arm.err
  python -c "import json; d=json.loads(open('$O/c4_tail$arm.json').read().strip().splitlines()[-1]); dd=d.get('decode',d); print('tail', $arm, d['metric'][:40], d['value'], d['unit'], 'decode', dd.get('value'), dd.get('leg_roofline',{}).get('steps'))"
done
