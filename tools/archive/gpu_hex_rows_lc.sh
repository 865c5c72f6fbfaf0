#!/bin/bash
# Row form at forced sub-chain lengths (SEM_HEX_CHAIN) against AUTO, p = 8 / 10:
#   tools/gpu_hex_rows_lc.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=$1; mkdir -p $O
run() {  # name, p, ne, env...
  local nm=$1 p=$2 ne=$3; shift 3
  env "$@" timeout -k 10 200 python3 bench.py --dim 3 --p $p --hex-ne $ne --no-cpu-baseline > $O/$nm.json 2> $O/$nm.err || { echo "$nm failed"; tail -5 $O/$nm.err; return 1; }
  python3 -c "
import json; r = json.load(open('$O/$nm.json')); c = r['config']; p = c['plan']
print('%-18s ms/step %.4f kernel %.4f frac %.3f wg %d lc %d seams %d parity %.1e' % ('$nm', r['ms_per_step'], c['kernel_ms_avg'], r['roofline']['frac'], p['workgroups'], p['chain_length_cap'], p['seam_nodes'], r['parity']['rel_l2']))"
}
for k in 1 2; do
  run p8_old_r$k 8 27 SEM_HEX_ROWS=0 || exit 1
  run p8_rows_auto_r$k 8 27 SEM_HEX_ROWS=1 || exit 1
  for lc in 9 14 27; do run p8_rows_lc${lc}_r$k 8 27 SEM_HEX_ROWS=1 SEM_HEX_CHAIN=$lc || exit 1; done
  run p10_old_r$k 10 22 SEM_HEX_ROWS=0 || exit 1
  for lc in 8 11 22; do run p10_rows_lc${lc}_r$k 10 22 SEM_HEX_ROWS=1 SEM_HEX_CHAIN=$lc || exit 1; done
done
