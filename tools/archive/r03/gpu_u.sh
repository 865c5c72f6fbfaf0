#!/bin/bash
# Round 3, call U: the headline kernel at its natural 3 waves/SIMD (133
# VGPRs, no scratch) against the 4-wave bound (128 VGPRs, 20 B scratch),
# alternating on one box, the driver's command; p = 16 on the shfl merge.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03u
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
line() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(round(d['ms_per_step'],4), [round(x,4) for x in c['kernel_ms_quartiles']], round(d['roofline']['frac'],3))" $1 2>/dev/null; }
for rep in 1 2 3 4; do
  for v in main w3; do
    unset SEM_LIB_PATH
    [ $v != main ] && export SEM_LIB_PATH=$PWD/build_variants/libsem_$v.so
    timeout -k 10 180 python bench.py --no-cpu-baseline > $O/cfg3_${v}_$rep.json 2> $O/cfg3_${v}_$rep.log; rc=$?
    echo "cfg3 $v $rep rc=$rc $(line $O/cfg3_${v}_$rep.json)"
    fatal $rc bench
  done
done
unset SEM_LIB_PATH
timeout -k 10 180 python bench.py --no-cpu-baseline --p 16 --nex 198 --ney 198 > $O/p16_main.json 2> $O/p16_main.log; rc=$?
echo "p16 main rc=$rc $(line $O/p16_main.json)"
