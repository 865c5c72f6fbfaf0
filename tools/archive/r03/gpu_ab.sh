#!/bin/bash
# Round 3, call AB: PCG with the float / flag-folded Jacobi preconditioner
# (72 instead of 81 B/DOF of vector traffic per iteration): solver tests,
# then per-iteration time against the previous build alternating on one box;
# then call AA (launch-bound variants at p = 10 / 12 / 14).
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03ab
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -k "pcg or solve or PCG or dd" --timeout 170 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
fatal $rc pytest
grep -q " passed" $O/pytest.log || exit 1
for rep in 1 2 3; do
  for v in main pc64; do
    unset SEM_LIB_PATH
    [ $v != main ] && export SEM_LIB_PATH=$PWD/build_variants/libsem_$v.so
    timeout -k 10 300 python bench.py --op pcg --steps 100 --warmup 5 --no-cpu-baseline > $O/pcg_${v}_$rep.json 2> $O/pcg_${v}_$rep.log; rc=$?
    echo "pcg $v $rep rc=$rc $(python -c "import json;d=json.load(open('$O/pcg_${v}_$rep.json'));print(round(d['ms_per_step'],4))" 2>/dev/null)"
    fatal $rc pcg
  done
done
unset SEM_LIB_PATH
bash tools/r03/gpu_aa.sh
