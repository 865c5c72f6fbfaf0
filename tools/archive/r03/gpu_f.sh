#!/bin/bash
# Round 3, call F: suite with sem_apply_dot, PCG fused p.q vs separate pass,
# enqueue time of the 2-rank step eager vs captured.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 170 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest.log
fatal $rc pytest
for rep in 1 2; do
  for mode in fused separate; do
    if [ $mode = separate ]; then export SEM_PCG_SEPARATE_PQ=1; else unset SEM_PCG_SEPARATE_PQ; fi
    timeout -k 10 300 python bench.py --op pcg --steps 100 --warmup 5 > $O/pcg_${mode}_$rep.json 2> $O/pcg_${mode}_$rep.log; rc=$?
    echo "pcg $mode $rep rc=$rc $(python -c "import json;d=json.load(open('$O/pcg_${mode}_$rep.json'));print(round(d['ms_per_step'],4))" 2>/dev/null)"
    fatal $rc pcg
  done
done
unset SEM_PCG_SEPARATE_PQ
timeout -k 10 300 python bench.py --op pcg --pcg-rtol 1e-10 --nex 128 --ney 128 > $O/pcg_solve_128.json 2> $O/pcg_solve_128.log; rc=$?
echo "pcg solve rc=$rc $(python -c "import json;d=json.load(open('$O/pcg_solve_128.json'));print(d['pcg'])" 2>/dev/null)"
fatal $rc pcgsolve
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/pcg_trace -o run -- python bench.py --op pcg --steps 30 --warmup 3 > $O/pcg_trace.log 2>&1; rc=$?; echo "pcg trace rc=$rc"
fatal $rc pcgtrace
head -8 $O/pcg_trace/run_kernel_stats.csv | cut -c1-120
for g in 1 0; do
  SEM_DD_GRAPH=$g timeout -k 10 300 python bench.py --rehearse-one-gpu --gpus 2 --steps 100 --warmup 5 --no-cpu-baseline --deadline 250 > $O/rehearse2_graph$g.json 2> $O/rehearse2_graph$g.log; rc=$?
  echo "rehearse2 graph=$g rc=$rc $(python -c "import json;d=json.load(open('$O/rehearse2_graph$g.json'));print(round(d['ms_per_step'],4), d['config']['decomposition'])" 2>/dev/null)"
  fatal $rc rehearse
done
