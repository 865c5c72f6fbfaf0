#!/bin/bash
# Round 3, call AA: launch-bound (min waves per SIMD) variants of the
# stored-factor column kernel at p = 10 / 12 / 14 (natural 5 / 4 / 4 waves),
# alternating on one box.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03aa
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
line() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(round(d['ms_per_step'],4), [round(x,4) for x in c['kernel_ms_quartiles']], round(d['roofline']['frac'],3))" $1 2>/dev/null; }
for rep in 1 2; do
  for cfg in "10 316" "12 263" "14 227"; do
    set -- $cfg
    for v in main mw3 mw5; do
      unset SEM_LIB_PATH
      [ $v != main ] && export SEM_LIB_PATH=$PWD/build_variants/libsem_$v.so
      timeout -k 10 180 python bench.py --no-cpu-baseline --no-check --p $1 --nex $2 --ney $2 > $O/p$1_${v}_$rep.json 2> $O/p$1_${v}_$rep.log; rc=$?
      echo "p$1 $v $rep rc=$rc $(line $O/p$1_${v}_$rep.json)"
      fatal $rc bench
    done
  done
done
