#!/bin/bash
# Round 3, call V: the seam plan's y / slot stores plain instead of
# nontemporal (write amplification at wave-segment edges?): cfg3 timing
# alternating on one box, then WRITE_SIZE / FETCH_SIZE of both builds.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03v
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
line() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(round(d['ms_per_step'],4), [round(x,4) for x in c['kernel_ms_quartiles']], round(d['roofline']['frac'],3))" $1 2>/dev/null; }
for rep in 1 2 3; do
  for v in main ntseam0; do
    unset SEM_LIB_PATH
    [ $v != main ] && export SEM_LIB_PATH=$PWD/build_variants/libsem_$v.so
    timeout -k 10 180 python bench.py --no-cpu-baseline > $O/cfg3_${v}_$rep.json 2> $O/cfg3_${v}_$rep.log; rc=$?
    echo "cfg3 $v $rep rc=$rc $(line $O/cfg3_${v}_$rep.json)"
    fatal $rc bench
    timeout -k 10 180 python bench.py --no-cpu-baseline --op axisym_stokes --p 6 --nex 512 --ney 512 > $O/cfg5_${v}_$rep.json 2> $O/cfg5_${v}_$rep.log; rc=$?
    echo "cfg5 $v $rep rc=$rc $(line $O/cfg5_${v}_$rep.json)"
    fatal $rc bench
  done
done
for v in main ntseam0; do
  unset SEM_LIB_PATH
  [ $v != main ] && export SEM_LIB_PATH=$PWD/build_variants/libsem_$v.so
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "k_poisson_apply|k_seam_sum" --output-format csv -d $O/pmc_${v}_$c -o run -- python bench.py --no-cpu-baseline --no-check --steps 8 --warmup 2 > $O/pmc_${v}_$c.log 2>&1; rc=$?; echo "pmc $v $c rc=$rc"
    fatal $rc pmc
  done
  python tools/pmc_traffic.py $O/pmc_${v}_FETCH_SIZE/run_counter_collection.csv $O/pmc_${v}_WRITE_SIZE/run_counter_collection.csv $O/traffic_$v.json --kernel k_poisson_apply --launches-per-action 1 > /dev/null 2>&1; python -c "import json;d=json.load(open('$O/traffic_$v.json'));print('$v', {k:v for k,v in d.items() if 'bytes' in k})"
done
