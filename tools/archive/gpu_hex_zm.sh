#!/bin/bash
# Hex: parity tests, then z-merge on / off alternating (plan-time switch
# SEM_HEX_ZMERGE=0), kernel trace of the default.   tools/gpu_hex_zm.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_hex.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
  for zm in 1 0; do
    SEM_HEX_ZMERGE=$zm timeout -k 10 300 python3 bench.py --dim 3 --no-cpu-baseline > $O/zm${zm}_r$k.json 2> $O/zm${zm}_r$k.err || { echo "bench zm=$zm failed"; tail -5 $O/zm${zm}_r$k.err; exit 1; }
    python3 -c "
import json; r = json.load(open('$O/zm${zm}_r$k.json')); c = r['config']
print('zm=$zm r$k ms/step %.4f kernel %.4f frac %.3f seam_nodes %d parity %.1e' % (r['ms_per_step'], c['kernel_ms_avg'], r['roofline']['frac'], c['plan']['seam_nodes'], r['parity']['rel_l2']))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --dim 3 --no-cpu-baseline --no-check > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
grep -h "k_hex" $O/trace/run_kernel_stats.csv | cut -c1-60,200-260
