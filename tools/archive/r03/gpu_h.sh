#!/bin/bash
# Round 3, call H: PCG vector-pass forms and graph-replay host cost
# (tools/r03/stream_bench.cpp), then the headline with split LDS reads
# (SEM_LDS_SPLIT) on both tile layouts against the default, alternating.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03h
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 120 ./tools/r03/stream_bench.bin > $O/stream_bench.txt 2>&1; rc=$?; echo "stream rc=$rc"; cat $O/stream_bench.txt
fatal $rc stream
for rep in 1 2 3; do
  for v in main split_wl0 split_wl1; do
    if [ $v = main ]; then unset SEM_LIB_PATH; else export SEM_LIB_PATH=$PWD/build_variants/libsem_$v.so; fi
    timeout -k 10 180 python bench.py --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.log; rc=$?
    echo "bench $v $rep rc=$rc $(python -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));c=d['config'];print(round(d['ms_per_step'],4), [round(x,4) for x in c['kernel_ms_quartiles']], d['parity']['rel_l2'])" 2>/dev/null)"
    fatal $rc bench
  done
done
