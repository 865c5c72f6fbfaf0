# GPU tests, then column vs MFMA kernel at the headline mesh and the p-sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/mfma
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
  tail -3 $OUT/gpu_tests.log
fi
for cfg in ${CFGS:-"8 1024 1024" "12 263 263" "10 316 316" "14 226 226" "15 211 211" "9 351 351"}; do
  set -- $cfg
  for k in column mfma; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --p $1 --nex $2 --ney $3 --steps 20 --kernel $k --geometry ${GEOM:-auto} > $OUT/p$1_$k.json 2> $OUT/p$1_$k.err || { echo "bench p$1 $k failed"; tail -5 $OUT/p$1_$k.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/p$1_$k.json')); print('p$1 $k', d['config']['geometry'], '%.4g' % d['value'], round(d['config']['kernel_ms_avg'],4), round(d['roofline']['frac'],3))"
  done
done
echo done
