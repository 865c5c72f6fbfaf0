#!/bin/bash
# (SEM_DD_IFACE_FIRST was removed after this measurement, profiles/r05/dd/iface_first/;
#  the script documents how it was run)
# Interface elements before the interior (SEM_DD_IFACE_FIRST): tests, then one rank of the 8-strip split
# timed alone (RCCL to itself) with it on / off, alternating.
#   tools/gpu_dd_ifirst.sh OUT (tests with it on)
set -o pipefail
export TMPDIR=/tmp
O=$1; mkdir -p $O
SEM_DD_IFACE_FIRST=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_seams.py tests/test_gpu_multirank.py tests/test_gpu_cfg3.py -x -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
  for fp in 1 0; do  # SEM_DD_IFACE_FIRST
    SEM_DD_IFACE_FIRST=$fp timeout -k 10 300 python -u bench.py --gpus 8 --time-rank 3 --steps 200 --warmup 20 > $O/tr3_fp${fp}_r$k.json 2> $O/tr3_fp${fp}_r$k.err || { echo "fp=$fp failed"; tail -5 $O/tr3_fp${fp}_r$k.err; exit 1; }
    python3 -c "
import json; r = json.load(open('$O/tr3_fp${fp}_r$k.json'))
s = r['single_gpu_whole_mesh']['wall_ms_per_step']
print('iface_first=$fp r$k step wall %.4f ev %.4f' % (r['step']['wall_ms_per_step'], r['step']['event_ms_avg']), 'exposed %.4f' % r['exposed_beyond_interior_ms'], 'host/apply %.1f us' % r['host']['host_us_per_apply'], 'single %.4f -> %.2fx' % (s, s / r['step']['wall_ms_per_step']))"
  done
done
