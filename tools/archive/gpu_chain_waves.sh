#!/bin/bash
# 8-wave chains (a variant library built first with
#   python -c "from spectralelementmethod_amd import _build; _build.build(force=True,
#     out='build_variants/libsem_cw8.so', defines=['SEM_CHAIN_WAVES=8'])")
# against the default 4, the driver
# command, alternating.   tools/gpu_chain_waves.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=$1; mkdir -p $O
for k in 1 2; do
  for v in cw8 cw4; do
    if [ $v = cw8 ]; then E="SEM_LIB_PATH=build_variants/libsem_cw8.so"; else E=""; fi
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline > $O/${v}_r$k.json 2> $O/${v}_r$k.err || { echo "$v failed"; tail -5 $O/${v}_r$k.err; exit 1; }
    python3 -c "
import json; r = json.load(open('$O/${v}_r$k.json')); c = r['config']
print('$v r$k ms/step %.4f kernel %.4f q %s frac %.3f parity %.1e plan %s' % (r['ms_per_step'], c['kernel_ms_avg'], [round(x, 4) for x in c['kernel_ms_quartiles']], r['roofline']['frac'], r['parity']['rel_l2'], c['scatter_plan']))"
  done
done
