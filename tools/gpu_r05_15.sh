set -e
export TMPDIR=/tmp
O=gpurun_out/r05/g15
mkdir -p $O
for q in 3 5 7 8 0; do
  timeout -k 10 300 python -u tools/rowexact_noise_probe.py $q 1 grid > $O/grid_q$q.txt 2>&1
  grep "^q" $O/grid_q$q.txt
done
