#!/bin/bash
# One rank of the 8-strip split timed alone: RCCL send/recv to itself vs the
# loopback copy, side stream at high / normal priority, RCCL protocol LL.
#   tools/gpu_dd_rccl.sh OUT [tests]
# (SEM_DD_SIDE_PRIORITY / NCCL_PROTO were measured with the build of that call; the
#  priority switch was removed afterwards: no effect, profiles/r05/dd/.)
set -o pipefail
export TMPDIR=/tmp
O=$1; mkdir -p $O
if [ "$2" = tests ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_seams.py tests/test_gpu_cfg3.py tests/test_gpu_multirank.py -x -v --timeout 500 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
tr() {  # name, "ENV=v ...", bench args...
  local nm=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python -u bench.py --gpus 8 --steps 200 --warmup 20 "$@" > $O/$nm.json 2> $O/$nm.err || { echo "$nm failed"; tail -5 $O/$nm.err; return 1; }
  python3 -c "
import json; r = json.load(open('$O/$nm.json'))
s = r['single_gpu_whole_mesh']['wall_ms_per_step']
print('%-34s step wall %.4f ev %.4f' % ('$nm', r['step']['wall_ms_per_step'], r['step']['event_ms_avg']), 'exposed %.4f' % (r['exposed_beyond_interior_ms'] or 0), 'host/apply %.1f us (transport %.1f)' % (r['host']['host_us_per_apply'], r['host']['host_us_transport']), 'enqueue/step %.4f' % r['step']['host_enqueue_ms_per_step'], 'single %.4f -> %.2fx' % (s, s / r['step']['wall_ms_per_step']))
"
}
for k in 1 2; do
tr time_rank3_rccl_self_r$k "SEM_DD_SIDE_PRIORITY=1" --time-rank 3 || exit 1
tr time_rank3_rccl_self_normalprio_r$k "SEM_DD_SIDE_PRIORITY=0" --time-rank 3 || exit 1
tr time_rank3_loopback_r$k "SEM_DD_SIDE_PRIORITY=1" --time-rank 3 --time-rank-transport loopback || exit 1
tr time_rank3_rccl_self_LL_r$k "SEM_DD_SIDE_PRIORITY=1 NCCL_PROTO=LL" --time-rank 3 || exit 1
done
tr time_rank0_rccl_self "SEM_DD_SIDE_PRIORITY=1" --time-rank 0 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 8 --time-rank 3 --steps 50 --warmup 10 --no-check > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
