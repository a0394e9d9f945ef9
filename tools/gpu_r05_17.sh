set -e
export TMPDIR=/tmp
O=gpurun_out/r05/g17
mkdir -p $O
CRAM_PARITY_LOG=$PWD/$O/parity.jsonl timeout -k 10 1050 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputest.txt 2>&1 || echo "pytest rc=$?"
tail -4 $O/gputest.txt
grep -E "FAILED" $O/gputest.txt | head -20 || true
