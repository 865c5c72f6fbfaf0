#!/bin/bash
# Round 3, call A: GPU suite on the block layout + compensated geometry,
# then the driver's bench command across block rounds / seam choices.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r03a
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 170 --timeout-method thread \
  -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 $O/pytest.log
fatal $rc pytest
for cfg in "0 0" "0 2" "2 2" "4 0" "4 1" "8 0" "8 1"; do
  set -- $cfg
  if [ "$2" = 2 ]; then unset SEM_SEAM; else export SEM_SEAM=$2; fi
  export SEM_BLOCK_ROUNDS=$1
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_R$1_S$2.json 2> $O/bench_R$1_S$2.log
  rc=$?
  echo "bench R=$1 seam=$2 rc=$rc $(python -c "import json;d=json.load(open('$O/bench_R$1_S$2.json'));print(round(d['ms_per_step'],4), round(d['config']['kernel_ms_avg'],4), d['config']['scatter_plan']['plan'], d['config']['scatter_plan']['chains_per_colour'], d['parity']['rel_l2'])" 2>/dev/null)"
  fatal $rc bench
done
