set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2i
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2i/tests.log 2>&1 || { echo "tests failed"; grep -v "^    \|^  File" gpurun_out/r2i/tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r2i/tests.log
timeout -k 10 200 python bench.py --no-cpu-baseline --p 16 --nex 198 --ney 198 --steps 30 > gpurun_out/r2i/p16.json 2> gpurun_out/r2i/p16.err || { echo "p16 failed"; tail -3 gpurun_out/r2i/p16.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r2i/p16.json')); print('p16', round(d['config']['kernel_ms_avg'],4), 'frac', round(d['roofline']['frac'],3), d['config']['scatter_plan']['colours'])"
/usr/bin/time -v timeout -k 10 600 python bench.py > gpurun_out/r2i/bench_default.json 2> gpurun_out/r2i/bench_default.err || { echo "bench failed"; tail -5 gpurun_out/r2i/bench_default.err; exit 1; }
grep -E "Elapsed|Maximum resident" gpurun_out/r2i/bench_default.err
python -c "import json; d=json.load(open('gpurun_out/r2i/bench_default.json')); print('default', '%.4g' % d['value'], round(d['config']['kernel_ms_avg'],4), 'frac', round(d['roofline']['frac'],3), d['cpu_baseline']['value'])"
