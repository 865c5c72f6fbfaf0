set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
for cfg in "2 1581 1581" "4 790 790" "6 527 527" "8 395 395" "12 263 263" "16 198 198"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-cpu-baseline --p $1 --nex $2 --ney $3 --steps 20 > gpurun_out/sweep/p$1.json 2> gpurun_out/sweep/p$1.err || { echo "sweep p$1 failed"; exit 1; }
done
timeout -k 10 300 python bench.py --no-cpu-baseline --op axisym_stokes --p 6 --nex 512 --ney 512 --steps 20 > gpurun_out/sweep/axisym.json 2> gpurun_out/sweep/axisym.err || { echo "axisym failed"; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --nex 256 --ney 256 --steps 50 > gpurun_out/sweep/cfg2.json 2> gpurun_out/sweep/cfg2.err || { echo "cfg2 failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_poisson_apply --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_poisson_apply --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
echo done
