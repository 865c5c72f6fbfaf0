#!/bin/bash
# Hex sub-chain length cap (SEM_HEX_CHAIN, plan time) sweep, alternating.
#   tools/gpu_hex_chain.sh OUT lc...
set -o pipefail
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
for k in 1 2; do
  for lc in default "$@"; do
    if [ $lc = default ]; then E=""; else E="SEM_HEX_CHAIN=$lc"; fi
    env $E timeout -k 10 200 python3 bench.py --dim 3 --no-cpu-baseline --no-check > $O/lc${lc}_r$k.json 2> $O/lc${lc}_r$k.err || { echo "lc=$lc failed"; tail -5 $O/lc${lc}_r$k.err; exit 1; }
    python3 -c "
import json; r = json.load(open('$O/lc${lc}_r$k.json')); c = r['config']; p = c['plan']
print('lc=%-7s r$k ms/step %.4f kernel %.4f wg %d seam_nodes %d' % ('$lc', r['ms_per_step'], c['kernel_ms_avg'], p['workgroups'], p['seam_nodes']))"
  done
done
