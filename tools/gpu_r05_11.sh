set -e
export TMPDIR=/tmp
O=gpurun_out/r05/g11
mkdir -p $O
for v in C D E; do
  timeout -k 10 300 python -u tools/ab_gemm_builds.py tools/abloop/libcram_A.so tools/abloop/libcram_$v.so 29184 7 > $O/ab_loop$v.txt 2>&1
  echo "== A vs $v"; grep -v amdgpu.ids $O/ab_loop$v.txt
done
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 1 --warmup 1 --no-cpu-baseline --decode-questions 128 --decode-batch 64 > $O/n2.json 2> $O/n2.err
tail -c 1200 $O/n2.json
