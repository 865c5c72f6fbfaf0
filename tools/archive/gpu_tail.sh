#!/bin/bash
# Launch-tail probe: p = 16 / 14 on meshes whose chain count is just under /
# over a whole number of resident generations (1,024 workgroups of 4 waves):
#   tools/gpu_tail.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=$1; mkdir -p $O
for cfg in "16 192" "16 198" "16 204" "16 222" "14 221" "14 227" "14 240" "14 256"; do
  set -- $cfg
  nm=p$1_$2
  timeout -k 10 200 python3 bench.py --p $1 --nex $2 --ney $2 --no-cpu-baseline --no-check > $O/$nm.json 2> $O/$nm.err || { echo "$nm failed"; tail -5 $O/$nm.err; exit 1; }
  python3 -c "
import json; r = json.load(open('$O/$nm.json')); c = r['config']; s = c['scatter_plan']
ch = sum(s['chains_per_colour'])
print('%-8s chains %5d gens %.2f ms/step %.4f kernel %.4f q50 %.4f frac %.3f DOF/s %.3g' % ('$nm', ch, ch / 1024.0, r['ms_per_step'], c['kernel_ms_avg'], c['kernel_ms_quartiles'][1], r['roofline']['frac'], r['value']))"
done
