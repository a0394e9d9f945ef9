set -e
export TMPDIR=/tmp
O=gpurun_out/r05/g27
mkdir -p $O
for q in 1 2 4 6 9 10 11 12; do
  timeout -k 10 300 python -u tools/rowexact_noise_probe.py $q 1 grid > $O/grid_q$q.txt 2>&1
  grep "^q" $O/grid_q$q.txt
done
