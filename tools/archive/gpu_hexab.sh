#!/bin/bash
# hex tests + one kernel trace per library variant:  tools/gpu_hexab.sh OUT variant...
export TMPDIR=/tmp
O=$1; shift
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_hex.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in base "$@"; do
  if [ $v = base ]; then L=""; else L="SEM_LIB_PATH=build_variants/$v/libsem_hip.so"; fi
  env $L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 bench.py --dim 3 --no-cpu-baseline --no-check > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$O/$v/run_kernel_stats.csv')):
    if 'hex_poisson' in r['Name'] or 'seam' in r['Name']: print('$v', r['Name'][:34], r['AverageNs'])
"
done
