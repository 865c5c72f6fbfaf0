#!/bin/bash
# Hexahedral path on the GPU box: parity tests, bench line, kernel trace.
#   tools/gpu_hex.sh OUTDIR [extra bench args]
set -o pipefail
O=${1:-gpurun_out/hex}; shift
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_hex.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py --dim 3 "$@" > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --dim 3 --no-cpu-baseline --no-check "$@" > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" -exec head -6 {} \;
