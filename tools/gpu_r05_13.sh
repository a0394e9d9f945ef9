set -e
export TMPDIR=/tmp
O=gpurun_out/r05/g13
mkdir -p $O
timeout -k 10 600 python -u tools/rowexact_noise_probe.py 0 10 > $O/rowexact_probe.txt 2>&1
grep -v amdgpu.ids $O/rowexact_probe.txt | tail -14
for m in llama3-8b qwen2-7b; do
  for n in 4 20; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${m}_n$n -o run -- python -u tools/prof_generate.py --model $m --B 512 --new $n --reps 2 > $O/${m}_n$n.log 2>&1
    tail -2 $O/${m}_n$n.log
  done
  python tools/decode_step_diff.py $O/${m}_n4 4 $O/${m}_n20 20 2 > $O/${m}_step.txt
  head -25 $O/${m}_step.txt
done
find $O -name "*kernel_trace.csv" -delete
