#!/bin/bash
# Round 3, call E: suite after the LDS-D revert and the PCG inverse diagonal,
# PCG bench + trace, headline nodal vs stored alternating on one box.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 170 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
fatal $rc pytest
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"
fatal $rc smoke
timeout -k 10 300 python bench.py --op pcg --steps 100 --warmup 5 > $O/pcg.json 2> $O/pcg.log; rc=$?
echo "pcg rc=$rc $(python -c "import json;d=json.load(open('$O/pcg.json'));print(d['ms_per_step'])" 2>/dev/null)"
fatal $rc pcg
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/pcg_trace -o run -- python bench.py --op pcg --steps 30 --warmup 3 > $O/pcg_trace.log 2>&1; rc=$?; echo "pcg trace rc=$rc"
fatal $rc pcgtrace
head -8 $O/pcg_trace/run_kernel_stats.csv | cut -c1-120
for rep in 1 2 3; do
for g in nodal stored; do
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --geometry $g > $O/bench_${g}_$rep.json 2> $O/bench_${g}_$rep.log; rc=$?
  echo "bench $g $rep rc=$rc $(python -c "import json;d=json.load(open('$O/bench_${g}_$rep.json'));c=d['config'];print(round(d['ms_per_step'],4), [round(x,4) for x in c['kernel_ms_quartiles']], c['scatter_plan']['plan'])" 2>/dev/null)"
  fatal $rc bench
done
done
