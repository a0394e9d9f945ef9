set -e
export TMPDIR=/tmp
O=gpurun_out/r05/g6
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
head -c 1500 $O/bench.json; echo
CRAM_PARITY_LOG=$PWD/$O/parity.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputest.txt 2>&1 || echo "pytest rc=$?"
tail -6 $O/gputest.txt
