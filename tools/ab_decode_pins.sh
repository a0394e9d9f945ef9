set -e
mkdir -p gpurun_out/abdec
for m in llama3-8b qwen2-7b; do
  for pin in 1 0 1; do
    CRAM_GEMM_PIN=$pin timeout -k 10 200 python -u tools/prof_generate.py --model $m --B 256 --new 100 --reps 2 > gpurun_out/abdec/${m}_pin${pin}_$RANDOM.txt 2>&1
  done
done
grep -H "rep 1" gpurun_out/abdec/*.txt
