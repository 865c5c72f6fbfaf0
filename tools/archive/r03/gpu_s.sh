#!/bin/bash
# Round 3, call S: p = 16 column kernel held at 3 waves/SIMD (the seam
# instantiation had drifted to 169 VGPRs, 2 waves) against the previous
# build, the n = 17 MFMA kernel beside it, p = 16 parity, then the sweep of
# the BASELINE configurations on this build.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03s
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
line() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(round(d['ms_per_step'],4), [round(x,4) for x in c['kernel_ms_quartiles']], round(d['roofline']['frac'],3), d.get('parity',{}).get('rel_l2'), c['scatter_plan']['plan'])" $1 2>/dev/null; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_seams.py tests/test_gpu_parity.py -m gpu -q -s --timeout 170 --timeout-method thread -p no:cacheprovider -k "16" > $O/pytest_p16.log 2>&1; rc=$?; echo "pytest p16 rc=$rc"; grep -E "extended|passed|failed" $O/pytest_p16.log | tail -5
fatal $rc pytest
grep -q " passed" $O/pytest_p16.log || exit 1
for rep in 1 2 3; do
  for v in w3 w1 mfma; do
    k=column; unset SEM_LIB_PATH
    [ $v = w1 ] && export SEM_LIB_PATH=$PWD/build_variants/libsem_p16w1.so
    [ $v = mfma ] && k=mfma
    timeout -k 10 180 python bench.py --no-cpu-baseline --p 16 --nex 198 --ney 198 --kernel $k > $O/p16_${v}_$rep.json 2> $O/p16_${v}_$rep.log; rc=$?
    echo "p16 $v $rep rc=$rc $(line $O/p16_${v}_$rep.json)"
    fatal $rc bench
  done
done
unset SEM_LIB_PATH
for cfg in "8 256" "2 1581" "4 790" "6 527" "8 395" "10 316" "12 263" "14 227" "16 198"; do
  set -- $cfg
  timeout -k 10 180 python bench.py --no-cpu-baseline --p $1 --nex $2 --ney $2 > $O/sweep_p$1_$2.json 2> $O/sweep_p$1_$2.log; rc=$?
  echo "sweep p=$1 $2^2 rc=$rc $(line $O/sweep_p$1_$2.json)"
  fatal $rc sweep
done
timeout -k 10 180 python bench.py --no-cpu-baseline --op axisym_stokes --p 6 --nex 512 --ney 512 > $O/sweep_cfg5.json 2> $O/sweep_cfg5.log; rc=$?
echo "sweep cfg5 rc=$rc $(line $O/sweep_cfg5.json)"
fatal $rc cfg5
timeout -k 10 180 python bench.py --no-cpu-baseline --p 8 --nex 1024 --ney 1024 > $O/sweep_cfg3.json 2> $O/sweep_cfg3.log; rc=$?
echo "sweep cfg3 rc=$rc $(line $O/sweep_cfg3.json)"
