#!/bin/bash
# Round 3, call T: what moved p = 16 (198^2) since call J: the DPP in-group
# merge and the 3-wave bound, alternating on one box; cfg3 and cfg5 beside.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03t
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
line() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(round(d['ms_per_step'],4), [round(x,4) for x in c['kernel_ms_quartiles']], round(d['roofline']['frac'],3))" $1 2>/dev/null; }
for rep in 1 2 3; do
  for v in main dpp0w1 dpp0w3; do
    unset SEM_LIB_PATH
    [ $v != main ] && export SEM_LIB_PATH=$PWD/build_variants/libsem_$v.so
    timeout -k 10 180 python bench.py --no-cpu-baseline --p 16 --nex 198 --ney 198 > $O/p16_${v}_$rep.json 2> $O/p16_${v}_$rep.log; rc=$?
    echo "p16 $v $rep rc=$rc $(line $O/p16_${v}_$rep.json)"
    fatal $rc bench
  done
done
for rep in 1 2; do
  for v in main dpp0w3; do
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
