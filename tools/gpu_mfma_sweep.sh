# kernel x geometry sweep at ~1e7 DOF per order (+ the MFMA parity tests)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/sweep_kg
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "${TESTK:-mfma}" --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
IFS=';' read -ra CFGLIST <<< "${CFGS:-2 1581 1581;3 1054 1054;4 790 790;5 632 632;6 527 527;7 452 452;8 395 395;12 263 263;15 211 211}"
for cfg in "${CFGLIST[@]}"; do
  IFS=' ' set -- $cfg
  for v in ${VARIANTS:-column:nodal column:stored mfma:nodal mfma:stored}; do
    K=${v%%:*}; G=${v##*:}
    timeout -k 10 300 python bench.py --no-cpu-baseline --p $1 --nex $2 --ney $3 --steps 20 --kernel $K --geometry $G > $OUT/p$1_${K}_$G.json 2> $OUT/p$1_${K}_$G.err || { echo "bench p$1 $v failed"; tail -5 $OUT/p$1_${K}_$G.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/p$1_${K}_$G.json')); print('p$1 $K $G', '%.4g' % d['value'], round(d['config']['kernel_ms_avg'],4), round(d['roofline']['frac'],3))"
  done
done
echo done
