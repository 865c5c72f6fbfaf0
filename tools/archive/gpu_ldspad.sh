#!/bin/bash
# Occupancy probe of the constant-D column kernels: SEM_LDS_PAD bytes of
# dynamic LDS per workgroup (fewer workgroups per CU), p = 12 / 14 / 16.
#   tools/gpu_ldspad.sh OUT pad...
# (SEM_LDS_PAD existed only in the probe build of that call -- the launch padding
#  was removed afterwards; results in profiles/r05/high_order_lds_pad/.)
set -o pipefail
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
for k in 1 2; do
  for pad in 0 $PADS; do
    for cfg in "16 198" "14 227" "12 263"; do
      set -- $cfg
      SEM_LDS_PAD=$pad timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-check --p $1 --nex $2 --ney $2 > $O/p$1_pad${pad}_r$k.json 2> $O/p$1_pad${pad}_r$k.err || { echo "p$1 pad $pad failed"; tail -5 $O/p$1_pad${pad}_r$k.err; exit 1; }
      python3 -c "
import json; r = json.load(open('$O/p$1_pad${pad}_r$k.json')); c = r['config']
print('p=$1 pad=%-6s r$k kernel %.4f frac %.3f' % ('$pad', c['kernel_ms_avg'], r['roofline']['frac']))"
    done
  done
done
