#!/bin/bash
# HIP_FORCE_DEV_KERNARG=1 / 0 (kernel arguments in device memory or not) on
# the driver command and one decomposition rank, alternating.
#   tools/gpu_kernarg.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=$1; mkdir -p $O
for k in 1 2; do
  for v in 1 0; do
    HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_k${v}_r$k.json 2> $O/bench_k${v}_r$k.err || { echo "bench $v failed"; exit 1; }
    python3 -c "import json; r=json.load(open('$O/bench_k${v}_r$k.json')); print('kernarg=$v r$k driver ms/step %.4f frac %.3f host %.4f' % (r['ms_per_step'], r['roofline']['frac'], r['config']['host_enqueue_ms_per_step']))"
    HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python -u bench.py --gpus 8 --time-rank 3 --steps 200 --warmup 20 > $O/tr3_k${v}_r$k.json 2> $O/tr3_k${v}_r$k.err || { echo "tr $v failed"; exit 1; }
    python3 -c "
import json; r = json.load(open('$O/tr3_k${v}_r$k.json'))
s = r['single_gpu_whole_mesh']['wall_ms_per_step']
print('kernarg=$v r$k rank step %.4f host/apply %.1f us single %.4f -> %.2fx' % (r['step']['wall_ms_per_step'], r['host']['host_us_per_apply'], s, s / r['step']['wall_ms_per_step']))"
  done
done
