# GPU tests, then the headline bench in both geometry modes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
for g in nodal stored; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --geometry $g ${BENCH_ARGS} > gpurun_out/bench_$g.json 2> gpurun_out/bench_$g.err || { echo "bench $g failed"; tail -20 gpurun_out/bench_$g.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_$g.json')); print('$g', '%.4g' % d['value'], d['config']['kernel_ms_avg'], d['roofline']['frac'], d['roofline']['fp64_tflops'])"
done
