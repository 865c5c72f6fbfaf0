#!/bin/bash
# After the three-block z-merge: row form vs three-block (both z-merged) at
# p = 2 / 4 / 6, then the p = 8 bench line's PMC traffic and kernel trace.
#   tools/gpu_hex_zm3.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=$1; mkdir -p $O
for k in 1 2; do
  for cfg in "2 108" "4 54" "6 36"; do
    set -- $cfg
    for rows in 1 0; do
      nm=p$1_rows${rows}_r$k
      SEM_HEX_ROWS=$rows timeout -k 10 200 python3 bench.py --dim 3 --p $1 --hex-ne $2 --no-cpu-baseline > $O/$nm.json 2> $O/$nm.err || { echo "$nm failed"; tail -5 $O/$nm.err; exit 1; }
      python3 -c "
import json; r = json.load(open('$O/$nm.json')); c = r['config']; p = c['plan']
print('%-14s ms/step %.4f kernel %.4f frac %.3f wg %d seams %d %s parity %.1e' % ('$nm', r['ms_per_step'], c['kernel_ms_avg'], r['roofline']['frac'], p['workgroups'], p['seam_nodes'], p['hex_kernel'], r['parity']['rel_l2']))"
    done
  done
done
B="python3 bench.py --dim 3 --no-cpu-baseline --no-check --steps 4 --warmup 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_hex_poisson|k_hex_seam_sum" --output-format csv -d $O/pmc_fetch -o run -- $B > $O/pmc_fetch.log 2>&1 || { echo "fetch pass failed"; tail -5 $O/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_hex_poisson|k_hex_seam_sum" --output-format csv -d $O/pmc_write -o run -- $B > $O/pmc_write.log 2>&1 || { echo "write pass failed"; tail -5 $O/pmc_write.log; exit 1; }
python3 tools/hex_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv $O/hex_traffic.json || exit 1
timeout -k 10 600 python3 bench.py --dim 3 --traffic-json $O/hex_traffic.json > $O/bench_hex.json 2> $O/bench_hex.err || { echo "hex bench failed"; tail -5 $O/bench_hex.err; exit 1; }
python3 -c "import json; r=json.load(open('$O/bench_hex.json')); print('hex p8', r['ms_per_step'], r['config']['kernel_ms_avg'], r['roofline'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_hex -o run -- python3 bench.py --dim 3 --no-cpu-baseline --no-check > $O/trace_hex.log 2>&1 || { echo "hex trace failed"; exit 1; }
find $O/trace_hex -name "*kernel_stats.csv" -exec head -5 {} \; | cut -c1-200
