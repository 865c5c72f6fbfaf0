#!/bin/bash
# Round-5 validation: GPU suite, smoke, driver command x2, hex line, BASELINE
# sweep, kernel trace of the driver command.   tools/gpu_final5.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=$1; mkdir -p $O/sweep
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || { echo "suite failed"; tail -30 $O/gpu_suite.log; exit 1; }
tail -1 $O/gpu_suite.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -10 $O/smoke.log; exit 1; }
cat $O/smoke.log | grep smoke
for k in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_default_$k.json 2> $O/bench_default_$k.err || { echo "bench failed"; tail -5 $O/bench_default_$k.err; exit 1; }
  python3 -c "import json; r=json.load(open('$O/bench_default_$k.json')); print('default', r['value'], r['ms_per_step'], r['roofline']['frac'], r['parity']['rel_l2'], r['cpu_baseline']['value'])"
done
timeout -k 10 300 python bench.py --dim 3 > $O/bench_hex.json 2> $O/bench_hex.err || { echo "hex bench failed"; exit 1; }
python3 -c "import json; r=json.load(open('$O/bench_hex.json')); print('hex', r['value'], r['ms_per_step'], r['roofline']['frac'], r['parity']['rel_l2'])"
for cfg in "cfg2 8 256" "p2 2 1581" "p4 4 790" "p6 6 527" "p8 8 395" "p10 10 316" "p12 12 263" "p14 14 227" "p16 16 198"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --no-cpu-baseline --p $2 --nex $3 --ney $3 > $O/sweep/$1.json 2> $O/sweep/$1.err || { echo "sweep $1 failed"; exit 1; }
done
timeout -k 10 200 python bench.py --no-cpu-baseline --op axisym_stokes --p 6 --nex 512 --ney 512 > $O/sweep/cfg5.json 2> $O/sweep/cfg5.err || { echo "cfg5 failed"; exit 1; }
timeout -k 10 300 python bench.py --op pcg --no-cpu-baseline --steps 100 --warmup 10 > $O/sweep/pcg_1024.json 2> $O/sweep/pcg.err || { echo "pcg failed"; exit 1; }
for f in $O/sweep/*.json; do python3 -c "
import json; r=json.load(open('$f')); c=r['config']
print('%-10s ms/step %.4f kernel %s frac %s parity %s' % ('$f'.split('/')[-1], r['ms_per_step'], c.get('kernel_ms_avg'), (r.get('roofline') or {}).get('frac'), (r.get('parity') or {}).get('rel_l2')))"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
head -3 $O/trace/run_kernel_stats.csv | cut -c1-80,190-260
