#!/bin/bash
# Round 3, call I: suite on the new defaults (split LDS reads, nontemporal
# 16-byte PCG passes, graphs opt-in), the driver's bench line, the PCG, and
# split column reads in the stored-factor kernel (A/B at cfg4 orders).
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 170 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
fatal $rc pytest
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.log; rc=$?
echo "bench default rc=$rc $(python -c "import json;d=json.load(open('$O/bench_default.json'));c=d['config'];print(d['value'], round(d['ms_per_step'],4), [round(x,4) for x in c['kernel_ms_quartiles']], d['roofline']['frac'], d['cpu_baseline']['value'])" 2>/dev/null)"
fatal $rc bench
timeout -k 10 300 python bench.py --op pcg --steps 100 --warmup 5 > $O/pcg.json 2> $O/pcg.log; rc=$?
echo "pcg rc=$rc $(python -c "import json;d=json.load(open('$O/pcg.json'));print(round(d['ms_per_step'],4))" 2>/dev/null)"
fatal $rc pcg
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/pcg_trace -o run -- python bench.py --op pcg --steps 30 --warmup 3 > $O/pcg_trace.log 2>&1; rc=$?; echo "pcg trace rc=$rc"
fatal $rc pcgtrace
head -6 $O/pcg_trace/run_kernel_stats.csv | cut -c1-120
for cfg in "6 527" "12 263" "16 198"; do
  set -- $cfg
  for rep in 1 2; do
    for v in main split_stored; do
      if [ $v = main ]; then unset SEM_LIB_PATH; else export SEM_LIB_PATH=$PWD/build_variants/libsem_$v.so; fi
      timeout -k 10 180 python bench.py --no-cpu-baseline --p $1 --nex $2 --ney $2 --geometry stored > $O/p$1_${v}_$rep.json 2> $O/p$1_${v}_$rep.log; rc=$?
      echo "p$1 $v $rep rc=$rc $(python -c "import json;d=json.load(open('$O/p$1_${v}_$rep.json'));c=d['config'];print(round(d['ms_per_step'],4), [round(x,4) for x in c['kernel_ms_quartiles']])" 2>/dev/null)"
      fatal $rc bench
    done
  done
done
