#!/bin/bash
# (SEM_HEX_RV existed only in the variant build of that measurement,
#  profiles/r05/hex/rows/rows_per_barrier/; the script documents how it was run)
# Row-form variants (SEM_HEX_RV = 10 * rows per barrier + map reload at the
# store) against the three-block kernel, alternating:
#   tools/gpu_hex_rv.sh OUT p...
set -o pipefail
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
for p in "$@"; do
  case $p in 2) ne=108;; 4) ne=54;; 6) ne=36;; 8) ne=27;; 10) ne=22;; *) ne=20;; esac
  for k in 1 2; do
    for v in 10 11 20 21 old; do
      if [ $v = old ]; then E="SEM_HEX_ROWS=0"; else E="SEM_HEX_ROWS=1 SEM_HEX_RV=$v"; fi
      nm=p${p}_rv${v}_r$k
      env $E timeout -k 10 200 python3 bench.py --dim 3 --p $p --hex-ne $ne --no-cpu-baseline > $O/$nm.json 2> $O/$nm.err || { echo "$nm failed"; tail -5 $O/$nm.err; exit 1; }
      python3 -c "
import json; r = json.load(open('$O/$nm.json')); c = r['config']; p = c['plan']
print('%-16s ms/step %.4f kernel %.4f frac %.3f wg %d parity %.2e' % ('$nm', r['ms_per_step'], c['kernel_ms_avg'], r['roofline']['frac'], p['workgroups'], r['parity']['rel_l2']))"
    done
  done
done
