#!/bin/bash
# PCG per iteration at 1024^2 p = 8 for library variants, alternating:
#   tools/gpu_pcg_ab.sh OUT variant...   (base = the in-tree library)
set -o pipefail
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
for k in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then L=""; else L="SEM_LIB_PATH=build_variants/$v/libsem_hip.so"; fi
    env $L timeout -k 10 300 python3 bench.py --op pcg --no-cpu-baseline --steps 100 --warmup 10 > $O/${v}_r$k.json 2> $O/${v}_r$k.err || { echo "$v failed"; tail -5 $O/${v}_r$k.err; exit 1; }
    python3 -c "
import json; r = json.load(open('$O/${v}_r$k.json')); print('%-8s r$k ms/iter %.4f' % ('$v', r['ms_per_step']))"
  done
done
