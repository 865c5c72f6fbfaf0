#!/bin/bash
# Round 3, call W: cfg5 (axisymmetric Stokes, p = 6, 512^2) plan knobs
# alternating on one box: 16-bit vs 32-bit map (the 16-bit instantiation
# spills 12 B/lane), block rounds 2 / 4 (AUTO) / 8.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03w
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
line() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(round(d['ms_per_step'],4), [round(x,4) for x in c['kernel_ms_quartiles']], round(d['roofline']['frac'],3), c['scatter_plan']['rounds'], c.get('map_entry_bytes'))" $1 2>/dev/null; }
for rep in 1 2 3; do
  for v in main m32 r2 r8; do
    unset SEM_MAP16 SEM_BLOCK_ROUNDS
    [ $v = m32 ] && export SEM_MAP16=0
    [ $v = r2 ] && export SEM_BLOCK_ROUNDS=2
    [ $v = r8 ] && export SEM_BLOCK_ROUNDS=8
    timeout -k 10 180 python bench.py --no-cpu-baseline --op axisym_stokes --p 6 --nex 512 --ney 512 > $O/cfg5_${v}_$rep.json 2> $O/cfg5_${v}_$rep.log; rc=$?
    echo "cfg5 $v $rep rc=$rc $(line $O/cfg5_${v}_$rep.json)"
    fatal $rc bench
  done
done
