#!/bin/bash
# Round 3, final build: the whole GPU suite, smoke(), the driver's bench
# command and its kernel trace, PMC traffic of the default action, and the
# sweep of the BASELINE configurations.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03final
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
line() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(round(d['ms_per_step'],4), [round(x,4) for x in c['kernel_ms_quartiles']], round(d['roofline']['frac'],3), d.get('parity',{}).get('rel_l2'), c['scatter_plan']['plan'])" $1 2>/dev/null; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 170 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
fatal $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"
fatal $rc smoke
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.log; rc=$?
echo "bench default rc=$rc $(python -c "import json;d=json.load(open('$O/bench_default.json'));c=d['config'];print(d['value'], round(d['ms_per_step'],4), [round(x,4) for x in c['kernel_ms_quartiles']], d['roofline']['frac'], d['cpu_baseline']['value'])" 2>/dev/null)"
fatal $rc bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/bench_trace -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_trace.json 2> $O/bench_trace.log; rc=$?; echo "trace rc=$rc"
fatal $rc trace
head -4 $O/bench_trace/run_kernel_stats.csv | cut -c1-150
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "k_poisson_apply|k_seam_sum" --output-format csv -d $O/pmc_$c -o run -- python bench.py --no-cpu-baseline --no-check --steps 8 --warmup 2 > $O/pmc_$c.log 2>&1; rc=$?; echo "pmc $c rc=$rc"
  fatal $rc pmc
done
python tools/pmc_traffic.py $O/pmc_FETCH_SIZE/run_counter_collection.csv $O/pmc_WRITE_SIZE/run_counter_collection.csv $O/traffic.json --kernel k_poisson_apply --launches-per-action 1 > /dev/null 2>&1; head -c 400 $O/traffic.json; echo
for cfg in "8 256" "2 1581" "4 790" "6 527" "8 395" "10 316" "12 263" "14 227" "16 198"; do
  set -- $cfg
  timeout -k 10 180 python bench.py --no-cpu-baseline --p $1 --nex $2 --ney $2 > $O/sweep_p$1_$2.json 2> $O/sweep_p$1_$2.log; rc=$?
  echo "sweep p=$1 $2^2 rc=$rc $(line $O/sweep_p$1_$2.json)"
  fatal $rc sweep
done
timeout -k 10 180 python bench.py --no-cpu-baseline --op axisym_stokes --p 6 --nex 512 --ney 512 > $O/sweep_cfg5.json 2> $O/sweep_cfg5.log; rc=$?
echo "sweep cfg5 rc=$rc $(line $O/sweep_cfg5.json)"
fatal $rc cfg5
timeout -k 10 300 python bench.py --op pcg --steps 100 --warmup 5 --no-cpu-baseline > $O/pcg.json 2> $O/pcg.log; rc=$?
echo "pcg rc=$rc $(python -c "import json;d=json.load(open('$O/pcg.json'));print(round(d['ms_per_step'],4))" 2>/dev/null)"
