#!/bin/bash
# Hexahedral p-sweep at ~1e7 DOF:  tools/gpu_hex_sweep.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=$1; mkdir -p $O
for cfg in "2 108" "4 54" "6 36" "8 27" "10 22"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --dim 3 --no-cpu-baseline --p $1 --hex-ne $2 > $O/hex_p$1.json 2> $O/hex_p$1.err || { echo "p$1 failed"; tail -5 $O/hex_p$1.err; exit 1; }
  python3 -c "
import json; r = json.load(open('$O/hex_p$1.json')); c = r['config']
print('p=$1 ne=$2 ndof %d ms/step %.4f kernel %.4f %.2fe10 DOF/s frac %.3f parity %.1e wg %d seams %d' % (c['ndof'], r['ms_per_step'], c['kernel_ms_avg'], r['value']/1e10, r['roofline']['frac'], r['parity']['rel_l2'], c['plan']['workgroups'], c['plan']['seam_nodes']))"
done
