#!/bin/bash
# Round 3, call J: split column reads in the axisymmetric nodal kernel (cfg5
# A/B), then the round-3 sweep of the BASELINE configurations on the final
# defaults (driver's 20 / 5 steps) and the rocprofv3 stats of the default line.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03j
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
line() { python -c "import json;d=json.load(open('$1'));c=d['config'];r=d['roofline'];print(d['value'], round(d['ms_per_step'],4), round(c['kernel_ms_avg'],4), [round(x,4) for x in c['kernel_ms_quartiles']], round(r['frac'],3), c['scatter_plan']['plan'], c['geometry'], d.get('parity',{}).get('rel_l2'))" 2>/dev/null; }
for rep in 1 2; do
  for v in main split_axi; do
    if [ $v = main ]; then unset SEM_LIB_PATH; else export SEM_LIB_PATH=$PWD/build_variants/libsem_$v.so; fi
    timeout -k 10 180 python bench.py --no-cpu-baseline --op axisym_stokes --p 6 --nex 512 --ney 512 > $O/cfg5_${v}_$rep.json 2> $O/cfg5_${v}_$rep.log; rc=$?
    echo "cfg5 $v $rep rc=$rc $(line $O/cfg5_${v}_$rep.json)"
    fatal $rc cfg5
  done
done
unset SEM_LIB_PATH
for cfg in "8 256" "2 1581" "4 790" "6 527" "8 395" "10 316" "12 263" "14 227" "16 198"; do
  set -- $cfg
  timeout -k 10 180 python bench.py --no-cpu-baseline --p $1 --nex $2 --ney $2 > $O/sweep_p$1_$2.json 2> $O/sweep_p$1_$2.log; rc=$?
  echo "sweep p=$1 $2^2 rc=$rc $(line $O/sweep_p$1_$2.json)"
  fatal $rc sweep
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/default_trace -o run -- python bench.py > $O/bench_default_under_rocprof.json 2> $O/default_trace.log; rc=$?
echo "default under rocprof rc=$rc $(line $O/bench_default_under_rocprof.json)"
fatal $rc trace
head -5 $O/default_trace/run_kernel_stats.csv | cut -c1-120
