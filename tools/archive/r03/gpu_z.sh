#!/bin/bash
# Round 3, call Z: only half of the symmetric quadrature weights as kernel
# arguments (headline kernel: SGPR spills 67 -> 39, v_readlane 103 -> 81):
# parity, then A/B against the previous build alternating on one box.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03z
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
line() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(round(d['ms_per_step'],4), [round(x,4) for x in c['kernel_ms_quartiles']], round(d['roofline']['frac'],3), d.get('parity',{}).get('rel_l2'))" $1 2>/dev/null; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_seams.py tests/test_gpu_blocks.py tests/test_host_lib.py -m gpu -q --timeout 170 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
fatal $rc pytest
grep -q " passed" $O/pytest.log || exit 1
for rep in 1 2 3 4; do
  for v in main base; do
    unset SEM_LIB_PATH
    [ $v != main ] && export SEM_LIB_PATH=$PWD/build_variants/libsem_$v.so
    timeout -k 10 180 python bench.py --no-cpu-baseline > $O/cfg3_${v}_$rep.json 2> $O/cfg3_${v}_$rep.log; rc=$?
    echo "cfg3 $v $rep rc=$rc $(line $O/cfg3_${v}_$rep.json)"
    fatal $rc bench
  done
done
for rep in 1 2; do
  for v in main base; do
    unset SEM_LIB_PATH
    [ $v != main ] && export SEM_LIB_PATH=$PWD/build_variants/libsem_$v.so
    timeout -k 10 180 python bench.py --no-cpu-baseline --op axisym_stokes --p 6 --nex 512 --ney 512 > $O/cfg5_${v}_$rep.json 2> $O/cfg5_${v}_$rep.log; rc=$?
    echo "cfg5 $v $rep rc=$rc $(line $O/cfg5_${v}_$rep.json)"
    fatal $rc bench
    timeout -k 10 180 python bench.py --no-cpu-baseline --p 4 --nex 790 --ney 790 > $O/p4_${v}_$rep.json 2> $O/p4_${v}_$rep.log; rc=$?
    echo "p4 $v $rep rc=$rc $(line $O/p4_${v}_$rep.json)"
    fatal $rc bench
  done
done
