#!/bin/bash
# (SEM_DD_CU_SIDE was removed after this measurement, profiles/r05/dd/cu_split/;
#  the script documents how it was run)
# CU split of the decomposition step (SEM_DD_CU_SIDE = K CUs for the side
# stream), one rank of the 8-strip split timed alone with RCCL to itself,
# alternating with K = 0.   tools/gpu_dd_cu.sh OUT K...
set -o pipefail
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
SEM_DD_CU_SIDE=16 timeout -k 10 600 python -u -m pytest tests/test_gpu_seams.py -k "dd_" -x -q --timeout 300 --timeout-method thread > $O/tests_cu16.log 2>&1 || { echo "tests failed"; tail -20 $O/tests_cu16.log; exit 1; }
tail -1 $O/tests_cu16.log
for k in 1 2; do
  for K in 0 $KS; do
    SEM_DD_CU_SIDE=$K timeout -k 10 300 python -u bench.py --gpus 8 --time-rank 3 --steps 200 --warmup 20 > $O/tr3_cu${K}_r$k.json 2> $O/tr3_cu${K}_r$k.err || { echo "K=$K failed"; tail -5 $O/tr3_cu${K}_r$k.err; exit 1; }
    python3 -c "
import json; r = json.load(open('$O/tr3_cu${K}_r$k.json'))
s = r['single_gpu_whole_mesh']['wall_ms_per_step']
print('cu_side=%-3s r$k step wall %.4f ev %.4f' % ('$K', r['step']['wall_ms_per_step'], r['step']['event_ms_avg']), 'exposed %.4f' % r['exposed_beyond_interior_ms'], 'host/apply %.1f us' % r['host']['host_us_per_apply'], 'single %.4f -> %.2fx' % (s, s / r['step']['wall_ms_per_step']))"
  done
done
