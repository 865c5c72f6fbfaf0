# Round profile: full GPU tests, smoke, default bench, kernel-trace stats and
# PMC traffic (separate FETCH_SIZE / WRITE_SIZE passes) of the headline workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r02}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests failed"; grep -v "^    \|^  File" $OUT/gpu_tests.log | tail -30; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
fi
timeout -k 10 300 python bench.py --steps 20 > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_default.json')); print('bench', '%.4g' % d['value'], d['config']['kernel_ms_avg'], d['roofline']['frac'], d.get('parity'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python bench.py --no-cpu-baseline --no-check --steps 20 > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_poisson_apply --output-format csv -d $OUT/pmc_fetch -o run -- python bench.py --no-cpu-baseline --no-check --steps 4 --warmup 1 > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -5 $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_poisson_apply --output-format csv -d $OUT/pmc_write -o run -- python bench.py --no-cpu-baseline --no-check --steps 4 --warmup 1 > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -5 $OUT/pmc_write.log; exit 1; }
F=$(find $OUT/pmc_fetch -name "*counter_collection.csv" | head -1)
W=$(find $OUT/pmc_write -name "*counter_collection.csv" | head -1)
python tools/pmc_traffic.py $F $W $OUT/traffic.json --bench-json $OUT/bench_default.json
find $OUT/trace -name "*kernel_stats.csv" -exec head -6 {} \;
echo done
