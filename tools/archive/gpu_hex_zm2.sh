#!/bin/bash
# z-merge in the three-block kernel through its w1 block (no LDS of its own):
# the hex GPU tests, then p = 8 / 10 with it on (default) / off, alternating.
#   tools/gpu_hex_zm2.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_hex.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
  for cfg in "8 27" "10 22"; do
    set -- $cfg
    for zm in 1 0; do
      nm=p$1_zm${zm}_r$k
      SEM_HEX_ZMERGE=$zm timeout -k 10 200 python3 bench.py --dim 3 --p $1 --hex-ne $2 --no-cpu-baseline > $O/$nm.json 2> $O/$nm.err || { echo "$nm failed"; tail -5 $O/$nm.err; exit 1; }
      python3 -c "
import json; r = json.load(open('$O/$nm.json')); c = r['config']; p = c['plan']
print('%-14s ms/step %.4f kernel %.4f frac %.3f wg %d seams %d zmerge %s %s parity %.1e' % ('$nm', r['ms_per_step'], c['kernel_ms_avg'], r['roofline']['frac'], p['workgroups'], p['seam_nodes'], p['zmerge'], p['hex_kernel'], r['parity']['rel_l2']))"
    done
  done
done
