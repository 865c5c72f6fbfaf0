#!/bin/bash
# Hexahedral bench line with PMC traffic + kernel trace; PCG kernel trace at 1024^2.
#   tools/gpu_hex_pmc.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=$1; mkdir -p $O
B="python3 bench.py --dim 3 --no-cpu-baseline --no-check --steps 4 --warmup 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_hex_poisson|k_hex_seam_sum" --output-format csv -d $O/pmc_fetch -o run -- $B > $O/pmc_fetch.log 2>&1 || { echo "fetch pass failed"; tail -5 $O/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_hex_poisson|k_hex_seam_sum" --output-format csv -d $O/pmc_write -o run -- $B > $O/pmc_write.log 2>&1 || { echo "write pass failed"; tail -5 $O/pmc_write.log; exit 1; }
python3 tools/hex_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv $O/hex_traffic.json || exit 1
timeout -k 10 600 python3 bench.py --dim 3 --traffic-json $O/hex_traffic.json > $O/bench_hex.json 2> $O/bench_hex.err || { echo "hex bench failed"; tail -5 $O/bench_hex.err; exit 1; }
cat $O/bench_hex.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_hex -o run -- python3 bench.py --dim 3 --no-cpu-baseline --no-check > $O/trace_hex.log 2>&1 || { echo "hex trace failed"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_pcg -o run -- python3 bench.py --op pcg --no-cpu-baseline --steps 100 --warmup 10 > $O/trace_pcg.log 2>&1 || { echo "pcg trace failed"; exit 1; }
find $O/trace_pcg -name "*kernel_stats.csv" -exec head -12 {} \;
