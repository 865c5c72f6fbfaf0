set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for m in 1 0 1 0; do
  SEM_MAP16=$m timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 ${BENCH_ARGS} > gpurun_out/m16_$m.json 2> gpurun_out/m16_$m.err || { echo "bench failed"; tail -5 gpurun_out/m16_$m.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/m16_$m.json')); print('map16=$m', round(d['config']['kernel_ms_avg'],4), round(d['roofline']['frac'],4), d['config']['map_entry_bytes'])"
done
