#!/bin/bash
# Settled-clock lines (200 timed actions) of the hex bench and the driver
# command, and a kernel trace of one decomposition rank's step (final build).
#   tools/gpu_settled_r05.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=$1; mkdir -p $O
timeout -k 10 300 python bench.py --dim 3 --no-cpu-baseline --steps 200 --warmup 20 > $O/hex_200.json 2> $O/hex_200.err || { echo "hex failed"; exit 1; }
python3 -c "import json; r=json.load(open('$O/hex_200.json')); print('hex 200', r['ms_per_step'], r['config']['kernel_ms_avg'], r['config']['kernel_ms_quartiles'], r['roofline']['frac'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20 > $O/default_200.json 2> $O/default_200.err || { echo "default failed"; exit 1; }
python3 -c "import json; r=json.load(open('$O/default_200.json')); print('default 200', r['ms_per_step'], r['config']['kernel_ms_avg'], r['config']['kernel_ms_quartiles'], r['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_tr3 -o run -- python3 bench.py --gpus 8 --time-rank 3 --steps 50 --warmup 10 --no-check > $O/trace_tr3.log 2>&1 || { echo "trace failed"; tail -5 $O/trace_tr3.log; exit 1; }
find $O/trace_tr3 -name "*kernel_trace.csv" | head -1
