# Round profile: p-sweep + axisym + cfg2 bench lines, kernel-trace stats and
# PMC traffic (separate passes) for the default workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-r01}
mkdir -p $OUT/sweep
for cfg in "2 1581 1581" "4 790 790" "6 527 527" "8 395 395" "12 263 263" "16 198 198"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-cpu-baseline --p $1 --nex $2 --ney $3 --steps 20 > $OUT/sweep/p$1.json 2> $OUT/sweep/p$1.err || { echo "sweep p$1 failed"; exit 1; }
done
timeout -k 10 300 python bench.py --no-cpu-baseline --op axisym_stokes --p 6 --nex 512 --ney 512 --steps 20 > $OUT/sweep/axisym_p6_512.json 2> $OUT/sweep/axisym.err || { echo "axisym failed"; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --nex 256 --ney 256 --steps 50 > $OUT/sweep/cfg2_256.json 2> $OUT/sweep/cfg2.err || { echo "cfg2 failed"; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python bench.py --no-cpu-baseline --steps 20 > $OUT/trace.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_poisson_apply --output-format csv -d $OUT/pmc_fetch -o run -- python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_poisson_apply --output-format csv -d $OUT/pmc_write -o run -- python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
python tools/pmc_traffic.py $OUT/pmc_fetch/run_counter_collection.csv $OUT/pmc_write/run_counter_collection.csv $OUT/traffic.json --bench-json $OUT/bench_default.json
echo done
