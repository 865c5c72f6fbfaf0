#!/bin/bash
# Round 3, call X: seam sums with 1 / 2 (default) / 4 nodes per thread in
# flight: seam tests, then kernel traces of cfg3 and p = 16 per build.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03x
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_seams.py tests/test_gpu_blocks.py tests/test_gpu_multirank.py -m gpu -q --timeout 170 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
fatal $rc pytest
grep -q " passed" $O/pytest.log || exit 1
for rep in 1 2; do
  for v in main ilp1 ilp4; do
    unset SEM_LIB_PATH
    [ $v != main ] && export SEM_LIB_PATH=$PWD/build_variants/libsem_$v.so
    for cfg in "8 1024" "16 198"; do
      set -- $cfg
      timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/tr_${v}_p$1_$rep -o run -- python bench.py --no-cpu-baseline --no-check --p $1 --nex $2 --ney $2 > $O/tr_${v}_p$1_$rep.json 2> $O/tr_${v}_p$1_$rep.log; rc=$?
      fatal $rc trace
      echo "$v p$1 $rep rc=$rc $(grep -E 'k_seam_sum|k_poisson_apply' $O/tr_${v}_p$1_$rep/run_kernel_stats.csv | cut -d, -f1,2,4 | tr '\n' ' ')"
    done
  done
done
