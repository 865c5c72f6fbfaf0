# full GPU tests, then the cfg5 bench (AUTO -> NODAL) with kernel trace and
# PMC traffic of k_axisym_nodal
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/axi2
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests failed"; grep -v "^    \|^  File" $OUT/gpu_tests.log | tail -30; exit 1; }
tail -1 $OUT/gpu_tests.log
A="--op axisym_stokes --p 6 --nex 512 --ney 512"
timeout -k 10 300 python bench.py --no-cpu-baseline $A --steps 30 > $OUT/cfg5.json 2> $OUT/cfg5.err || { echo "bench failed"; tail -20 $OUT/cfg5.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python bench.py --no-cpu-baseline --no-check $A --steps 20 > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_axisym --output-format csv -d $OUT/pmc_fetch -o run -- python bench.py --no-cpu-baseline --no-check $A --steps 4 --warmup 1 > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -5 $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_axisym --output-format csv -d $OUT/pmc_write -o run -- python bench.py --no-cpu-baseline --no-check $A --steps 4 --warmup 1 > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -5 $OUT/pmc_write.log; exit 1; }
F=$(find $OUT/pmc_fetch -name "*counter_collection.csv" | head -1)
W=$(find $OUT/pmc_write -name "*counter_collection.csv" | head -1)
python tools/pmc_traffic.py $F $W $OUT/traffic.json --bench-json $OUT/cfg5.json
find $OUT/trace -name "*kernel_stats.csv" -exec head -6 {} \;
echo done
