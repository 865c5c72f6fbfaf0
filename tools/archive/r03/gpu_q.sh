#!/bin/bash
# Round 3, call Q: the whole GPU suite on the build with k_poisson_mfma17 and
# the device banded-LU solve, smoke(), the driver's bench command and its
# kernel trace.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03q
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 170 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
fatal $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"
fatal $rc smoke
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.log; rc=$?
echo "bench default rc=$rc $(python -c "import json;d=json.load(open('$O/bench_default.json'));c=d['config'];print(d['value'], round(d['ms_per_step'],4), [round(x,4) for x in c['kernel_ms_quartiles']], d['roofline']['frac'], d['cpu_baseline']['value'])" 2>/dev/null)"
fatal $rc bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/bench_trace -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_trace.json 2> $O/bench_trace.log; rc=$?; echo "trace rc=$rc"
fatal $rc trace
head -4 $O/bench_trace/run_kernel_stats.csv | cut -c1-150
