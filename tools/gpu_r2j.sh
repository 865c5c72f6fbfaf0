set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2j
t0=$(date +%s.%N)
timeout -k 10 600 python bench.py > gpurun_out/r2j/bench_default.json 2> gpurun_out/r2j/bench_default.err || { echo "bench failed"; tail -5 gpurun_out/r2j/bench_default.err; exit 1; }
t1=$(date +%s.%N)
echo "bench wall seconds: $(python -c "print($t1 - $t0)")"
python -c "import json; d=json.load(open('gpurun_out/r2j/bench_default.json')); print('default', '%.4g' % d['value'], round(d['config']['kernel_ms_avg'],4), 'frac', round(d['roofline']['frac'],3), d['cpu_baseline']['value'], d['parity'])"
