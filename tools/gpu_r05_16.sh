set -e
export TMPDIR=/tmp
O=gpurun_out/r05/g16
mkdir -p $O
timeout -k 10 300 python -u tools/baseline_cache_probe.py 3 > $O/cache_q3.txt 2>&1
grep -v "amdgpu.ids\|Warning" $O/cache_q3.txt
timeout -k 10 300 python -u tools/baseline_cache_probe.py 5 > $O/cache_q5.txt 2>&1
grep -v "amdgpu.ids\|Warning" $O/cache_q5.txt
OUT=$O/gemm_pmc bash tools/pmc_gemm.sh > $O/gemm_pmc_summary.txt 2>&1
python3 tools/pmc_to_json.py --gemm $O/gemm_pmc $O/gemm_pmc.json | grep -E "mfma_busy|clock|valu_per|traffic_over|tflops"
MODE=lt KREGEX=Cijk OUT=$O/lt_pmc bash tools/pmc_gemm.sh > $O/lt_pmc_summary.txt 2>&1
python3 tools/pmc_to_json.py --lt $O/lt_pmc $O/lt_pmc.json | grep -E "mfma_busy|clock|valu_per|traffic_over|tflops"
OUT=$O/pmc bash tools/pmc_attn.sh > $O/pmc_summary.txt 2>&1
python3 tools/pmc_to_json.py $O/pmc $O/attn_pmc.json | grep -E "mfma_busy|clock|valu_per|traffic_over|tflops"
