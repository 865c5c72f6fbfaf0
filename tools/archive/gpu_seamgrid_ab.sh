#!/bin/bash
# Seam-sum grid cap A/B: kernel traces of the default bench and the hex bench
# per library variant.   tools/gpu_seamgrid_ab.sh OUT variant...
set -o pipefail
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
for k in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then L=""; else L="SEM_LIB_PATH=build_variants/$v/libsem_hip.so"; fi
    for dim in 2 3; do
      env $L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_d${dim}_r$k -o run -- python3 bench.py --dim $dim --no-cpu-baseline --no-check > $O/${v}_d${dim}_r$k.log 2>&1 || { echo "$v d$dim failed"; tail -5 $O/${v}_d${dim}_r$k.log; exit 1; }
      python3 -c "
import csv
for r in csv.DictReader(open('$O/${v}_d${dim}_r$k/run_kernel_stats.csv')):
    n = r['Name']
    if 'seam_sum' in n or 'k_poisson_apply' in n or 'k_hex_poisson' in n: print('%-6s d$dim r$k %-28s %8.1f us' % ('$v', n.split('(')[0][-28:], float(r['AverageNs']) / 1e3))
"
    done
  done
done
