#!/bin/bash
# Round 3, call AD: p = 10 with 6 / 7-wave requests (natural 5), and the
# p = 4 6-wave bound of the new default confirmed, alternating on one box.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03ad
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
line() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(round(d['ms_per_step'],4), [round(x,4) for x in c['kernel_ms_quartiles']], round(d['roofline']['frac'],3), d.get('parity',{}).get('rel_l2'))" $1 2>/dev/null; }
for rep in 1 2; do
  for v in main mw6 mw7; do
    unset SEM_LIB_PATH
    [ $v != main ] && export SEM_LIB_PATH=$PWD/build_variants/libsem_$v.so
    timeout -k 10 180 python bench.py --no-cpu-baseline --no-check --p 10 --nex 316 --ney 316 > $O/p10_${v}_$rep.json 2> $O/p10_${v}_$rep.log; rc=$?
    echo "p10 $v $rep rc=$rc $(line $O/p10_${v}_$rep.json)"
    fatal $rc bench
  done
  unset SEM_LIB_PATH
  timeout -k 10 180 python bench.py --no-cpu-baseline --p 4 --nex 790 --ney 790 > $O/p4_main_$rep.json 2> $O/p4_main_$rep.log; rc=$?
  echo "p4 main $rep rc=$rc $(line $O/p4_main_$rep.json)"
  fatal $rc bench
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -q -k "all_orders or config4_action" --timeout 170 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log
