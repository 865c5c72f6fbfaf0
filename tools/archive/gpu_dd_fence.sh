#!/bin/bash
# Decomposition-step events without the system-scope fence
# (SEM_DD_EVENT_FENCE=device): the decomposition GPU tests with it, then one
# rank of the 8-strip split timed alone, device / system alternating.
#   tools/gpu_dd_fence.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=$1; mkdir -p $O
SEM_DD_EVENT_FENCE=device timeout -k 10 600 python -u -m pytest tests/test_gpu_seams.py tests/test_gpu_multirank.py tests/test_gpu_cfg3.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
  for f in device system; do
    SEM_DD_EVENT_FENCE=$f timeout -k 10 300 python -u bench.py --gpus 8 --time-rank 3 --steps 200 --warmup 20 > $O/tr3_${f}_r$k.json 2> $O/tr3_${f}_r$k.err || { echo "$f failed"; tail -5 $O/tr3_${f}_r$k.err; exit 1; }
    python3 -c "
import json; r = json.load(open('$O/tr3_${f}_r$k.json'))
s = r['single_gpu_whole_mesh']['wall_ms_per_step']
print('fence=$f r$k step wall %.4f ev %.4f' % (r['step']['wall_ms_per_step'], r['step']['event_ms_avg']), 'exposed %.4f' % r['exposed_beyond_interior_ms'], 'host/apply %.1f us' % r['host']['host_us_per_apply'], 'single %.4f -> %.2fx' % (s, s / r['step']['wall_ms_per_step']))"
  done
done
