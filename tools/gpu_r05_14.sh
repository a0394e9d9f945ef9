set -e
export TMPDIR=/tmp
O=gpurun_out/r05/g14
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_decode_routing_gpu.py -k "varlen_cached or shared_prefix" -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
grep -E "PASSED|FAILED|shared-prefix" $O/tests.txt
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('heads/s', d['value'], 'decode', d['decode']['value'], d['decode']['leg_roofline']['prefill'])"
CRAM_PREFIX_SHARE=0 timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench_noshare.json 2> $O/bench_noshare.err
python -c "import json; d=json.loads(open('$O/bench_noshare.json').read().strip().splitlines()[-1]); print('noshare heads/s', d['value'], 'decode', d['decode']['value'], d['decode']['leg_roofline']['prefill'])"
for m in llama3-8b qwen2-7b; do
  for n in 4 20; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${m}_n$n -o run -- python -u tools/prof_generate.py --model $m --B 512 --new $n --reps 2 > $O/${m}_n$n.log 2>&1
    grep "^rep" $O/${m}_n$n.log
  done
  python tools/decode_step_diff.py $O/${m}_n4 4 $O/${m}_n20 20 2 > $O/${m}_step.txt
  head -25 $O/${m}_step.txt
done
find $O -name "*kernel_trace.csv" -delete
