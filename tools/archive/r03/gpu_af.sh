#!/bin/bash
# Round 3, call AF: row-direction coordinates gathered through a 4-byte LDS
# map transpose (SEM_GEOM_ROW_GATHER) against the two 8-byte coordinate
# transposes: parity of the variant, then cfg3 alternating on one box.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03af
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
line() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(round(d['ms_per_step'],4), [round(x,4) for x in c['kernel_ms_quartiles']], round(d['roofline']['frac'],3), d.get('parity',{}).get('rel_l2'))" $1 2>/dev/null; }
SEM_LIB_PATH=$PWD/build_variants/libsem_rowg.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_blocks.py tests/test_gpu_seams.py -m gpu -q -k "nodal or seams or blocks" --timeout 170 --timeout-method thread -p no:cacheprovider > $O/pytest_rowg.log 2>&1; rc=$?; echo "pytest rowg rc=$rc"; tail -1 $O/pytest_rowg.log
fatal $rc pytest
for rep in 1 2 3 4; do
  for v in main rowg; do
    unset SEM_LIB_PATH
    [ $v != main ] && export SEM_LIB_PATH=$PWD/build_variants/libsem_$v.so
    timeout -k 10 180 python bench.py --no-cpu-baseline > $O/cfg3_${v}_$rep.json 2> $O/cfg3_${v}_$rep.log; rc=$?
    echo "cfg3 $v $rep rc=$rc $(line $O/cfg3_${v}_$rep.json)"
    fatal $rc bench
  done
done
