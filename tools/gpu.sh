#!/bin/bash
# The one GPU-call wrapper (replaces the round-1..3 one-off gpu_*.sh scripts).  Runs the named steps in order, each
# under its own time limit, into gpurun_out/$TAG/; the first failing GPU step ends the call (no retries).
#
#   TAG=r04/x bash tools/gpu.sh STEP [STEP ...]
#
# steps:
#   suite            pytest -m gpu (every GPU test, -x)
#   suite-all        pytest -m gpu without -x (every failure listed)
#   smoke            __graft_entry__.smoke()
#   bench            the default bench line (config 3 + decode, CPU baselines)
#   bench:ARGS       bench.py with ARGS (commas become spaces), e.g. bench:--config,2,--no-cpu-baseline
#   benv:ENV:ARGS    bench.py ARGS under ENV (NAME=V pairs joined by +), e.g. benv:CRAM_FUSED_QKV=0:--no-decode (A/B arms)
#   prof             rocprofv3 --kernel-trace --stats of the sweep-only bench (summary kept, traces deleted)
#   pmc              the attention kernel's PMC passes (tools/pmc_attn.sh) -> pmc_summary.txt + attn_pmc.json
#   pmcgemm          the dominant GEMM launch's PMC passes (tools/pmc_gemm.sh) -> gemm_pmc_summary.txt + gemm_pmc.json
#   pmclt            the same passes on hipBLASLt's kernel for the same product -> lt_pmc.json (EXTRA=1: + request sizes)
#   test:PATTERN     pytest -m gpu -k PATTERN
#   py:SCRIPT,ARGS   python SCRIPT ARGS (a probe under tools/)
#   pyt:SEC:SCRIPT,ARGS  the same under a time limit of SEC seconds
#   dist2:ARGS       bench.py ARGS at N = 2 (torch.distributed.run, gloo, both ranks on the one GPU)
set -e
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-run}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
PYT="python -u -m pytest tests -m gpu --timeout 300 --timeout-method thread"
for step in "$@"; do
  echo "== $step ($(date +%T))"
  case "$step" in
    suite)     timeout -k 10 1000 $PYT -x -v --durations=60 > $O/gputest.txt 2>&1; tail -3 $O/gputest.txt ;;
    suite-all) timeout -k 10 1000 $PYT -v > $O/gputest.txt 2>&1 || echo "pytest rc=$?"; tail -5 $O/gputest.txt ;;
    smoke)     timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
               tail -2 $O/smoke.txt ;;
    bench)     timeout -k 10 560 python -u bench.py > $O/bench.json 2> $O/bench.err; head -c 700 $O/bench.json; echo ;;
    bench:*)   a=${step#bench:}; n=$(echo "$a" | tr -c 'a-zA-Z0-9' '_' | cut -c1-60)
               timeout -k 10 900 python -u bench.py ${a//,/ } > $O/bench_$n.json 2> $O/bench_$n.err
               head -c 700 $O/bench_$n.json; echo ;;
    benv:*)    a=${step#benv:}; e=${a%%:*}; a=${a#*:}; n=$(echo "$e$a" | tr -c 'a-zA-Z0-9' '_' | cut -c1-70)
               timeout -k 10 900 env ${e//+/ } python -u bench.py ${a//,/ } > $O/benv_$n.json 2> $O/benv_$n.err
               head -c 400 $O/benv_$n.json; echo ;;
    prof)      mkdir -p $O/prof
               timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o sweep \
                 -- python3 bench.py --no-cpu-baseline --no-decode > $O/prof/sweep.json 2> $O/prof/sweep.err
               python3 tools/trace_gaps.py $O/prof > $O/prof/gaps.txt 2>&1 || true
               find $O/prof -name "*kernel_trace.csv" -delete
               head -8 $O/prof/sweep_kernel_stats.csv | cut -c1-160 ;;
    pmc)       OUT=$O/pmc bash tools/pmc_attn.sh > $O/pmc_summary.txt 2>&1
               python3 tools/pmc_to_json.py $O/pmc $O/attn_pmc.json > /dev/null; cat $O/pmc_summary.txt ;;
    pmcgemm)   OUT=$O/gemm_pmc bash tools/pmc_gemm.sh > $O/gemm_pmc_summary.txt 2>&1
               python3 tools/pmc_to_json.py --gemm $O/gemm_pmc $O/gemm_pmc.json > /dev/null; cat $O/gemm_pmc_summary.txt ;;
    pmclt)     MODE=lt KREGEX=Cijk OUT=$O/lt_pmc bash tools/pmc_gemm.sh > $O/lt_pmc_summary.txt 2>&1
               python3 tools/pmc_to_json.py --lt $O/lt_pmc $O/lt_pmc.json > /dev/null; cat $O/lt_pmc_summary.txt ;;
    test:*)    k=${step#test:}; n=$(echo "$k" | tr -c 'a-zA-Z0-9' '_' | cut -c1-60)
               timeout -k 10 900 $PYT -x -v -s -k "$k" > $O/test_$n.txt 2>&1; tail -3 $O/test_$n.txt ;;
    py:*)      a=${step#py:}; n=$(basename "${a%%,*}" .py)$(echo "${a#*,}" | tr -c 'a-zA-Z0-9' '_' | cut -c1-40)
               timeout -k 10 600 python -u ${a//,/ } > $O/$n.txt 2>&1; tail -30 $O/$n.txt ;;
    dist2:*)   a=${step#dist2:}; n=$(echo "$a" | tr -c 'a-zA-Z0-9' '_' | cut -c1-60)
               # the bench's N = 2 path rehearsed on the one GPU: two gloo ranks share the device (RCCL refuses two
               # ranks on one GPU), torch.distributed.run as the driver launches it
               timeout -k 10 900 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
                 --master-port 29533 bench.py --gpus 2 --dist-backend gloo ${a//,/ } > $O/dist2_$n.json 2> $O/dist2_$n.err
               head -c 700 $O/dist2_$n.json; echo ;;
    pyt:*)     a=${step#pyt:}; lim=${a%%:*}; a=${a#*:}; n=$(basename "${a%%,*}" .py)$(echo "${a#*,}" | tr -c 'a-zA-Z0-9' '_' | cut -c1-40)
               timeout -k 10 $lim python -u ${a//,/ } > $O/$n.txt 2>&1; tail -30 $O/$n.txt ;;
    *)         echo "unknown step $step"; exit 2 ;;
  esac
done
