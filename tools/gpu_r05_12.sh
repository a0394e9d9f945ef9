set -e
export TMPDIR=/tmp
O=gpurun_out/r05/g12
mkdir -p $O
for q in 3 7; do
  for mode in re1 re1_notail re0; do
    case $mode in
      re1) E="CRAM_SWEEP_ROW_EXACT=1";;
      re1_notail) E="CRAM_SWEEP_ROW_EXACT=1 CRAM_TAIL_SPLIT=0";;
      re0) E="CRAM_SWEEP_ROW_EXACT=0";;
    esac
    env $E CRAM_FULLSIZE_Q=$q timeout -k 10 400 python -u -m pytest tests/test_fullsize_ie_gpu.py -k "full_grid or matches_fp32" -v -s --timeout 300 --timeout-method thread > $O/q${q}_$mode.txt 2>&1 || true
    echo "== q$q $mode"; grep -E "k=894|k=100|rms ratio|spearman vs|\|ours-truth\||PASSED|FAILED" $O/q${q}_$mode.txt | cut -c1-200 || true
  done
done
