#!/bin/bash
# HIP events around every timed step (--step-events each, the default) against
# one pair around the timed region: one rank of the 8-strip split timed alone
# and the driver command, alternating.   tools/gpu_step_events.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=$1; mkdir -p $O
for k in 1 2; do
  for se in each region; do
    timeout -k 10 300 python -u bench.py --gpus 8 --time-rank 3 --steps 200 --warmup 20 --step-events $se > $O/tr3_${se}_r$k.json 2> $O/tr3_${se}_r$k.err || { echo "tr $se failed"; tail -5 $O/tr3_${se}_r$k.err; exit 1; }
    python3 -c "
import json; r = json.load(open('$O/tr3_${se}_r$k.json'))
s = r['single_gpu_whole_mesh']['wall_ms_per_step']
print('time-rank $se r$k step wall %.4f ev %.4f' % (r['step']['wall_ms_per_step'], r['step']['event_ms_avg']), 'single %.4f -> %.2fx' % (s, s / r['step']['wall_ms_per_step']))"
  done
  for se in each region; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --step-events $se > $O/bench_${se}_r$k.json 2> $O/bench_${se}_r$k.err || { echo "bench $se failed"; tail -5 $O/bench_${se}_r$k.err; exit 1; }
    python3 -c "
import json; r = json.load(open('$O/bench_${se}_r$k.json'))
print('driver cmd $se r$k ms/step %.4f kernel %.4f frac %.3f' % (r['ms_per_step'], r['config']['kernel_ms_avg'], r['roofline']['frac']))"
  done
done
