set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1; tail -3 gpurun_out/gpu_tests.log
for r in 1 2 4 8; do
  SEM_CHAIN_ROUNDS=$r timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/rounds_$r.json 2> gpurun_out/rounds_$r.err || { echo "rounds $r failed"; tail -3 gpurun_out/rounds_$r.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/rounds_$r.json')); print('rounds $r', round(d['config']['kernel_ms_avg'],4), round(d['roofline']['frac'],4), d['config']['scatter_plan'])"
done
