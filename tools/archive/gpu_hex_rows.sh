#!/bin/bash
# Hex action: row form (k_hex_rows, default) against the three-block kernel
# (SEM_HEX_ROWS=0), with and without the z-merge, alternating; the hex GPU
# tests first (default: row form with z-merge).
#   tools/gpu_hex_rows.sh OUT [p ...]
set -o pipefail
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
PS=${*:-8}
[ -n "$NOTEST" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_hex.py -x -v --timeout 120 --timeout-method thread > $O/tests_rows.log 2>&1 || { echo "tests failed"; tail -30 $O/tests_rows.log; exit 1; }
[ -n "$NOTEST" ] || tail -1 $O/tests_rows.log
for p in $PS; do
  case $p in 2) ne=108;; 4) ne=54;; 6) ne=36;; 8) ne=27;; 10) ne=22;; *) ne=20;; esac
  for k in 1 2; do
    for v in ${VARIANTS:-rows_zm rows old}; do
      case $v in rows_zm) E="SEM_HEX_ROWS=1";; rows) E="SEM_HEX_ROWS=1 SEM_HEX_ZMERGE=0";; old) E="SEM_HEX_ROWS=0";; esac
      nm=p${p}_${v}_r$k
      env $E timeout -k 10 200 python3 bench.py --dim 3 --p $p --hex-ne $ne --no-cpu-baseline > $O/$nm.json 2> $O/$nm.err || { echo "$nm failed"; tail -5 $O/$nm.err; exit 1; }
      python3 -c "
import json; r = json.load(open('$O/$nm.json')); c = r['config']; p = c['plan']
print('%-16s ms/step %.4f kernel %.4f frac %.3f wg %d lc %s parity %s' % ('$nm', r['ms_per_step'], c['kernel_ms_avg'], r['roofline']['frac'], p['workgroups'], p.get('chain_len'), r.get('parity', {}).get('rel_l2')))"
    done
  done
done
