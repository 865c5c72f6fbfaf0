# Column kernel vs MFMA kernel builds (build_variants/lib_<v>.so): parity
# tests of the MFMA path, then timings per order.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/mfma_ab
mkdir -p $OUT
[ "$TESTK" = nothing_at_all_zz ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "${TESTK:-mfma}" --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
IFS=';' read -ra CFGLIST <<< "${CFGS:-12 263 263;10 316 316;15 211 211}"
for cfg in "${CFGLIST[@]}"; do
  IFS=' ' set -- $cfg
  for v in ${VARIANTS:-column base}; do
    case $v in column) K=column; L=$PWD/spectralelementmethod_amd/libsem_hip.so;; *) K=mfma; L=$PWD/build_variants/lib_$v.so;; esac
    SEM_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu-baseline --p $1 --nex $2 --ney $3 --steps 20 --kernel $K --geometry ${GEOM:-stored} > $OUT/p$1_$v.json 2> $OUT/p$1_$v.err || { echo "bench p$1 $v failed"; tail -5 $OUT/p$1_$v.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/p$1_$v.json')); print('p$1 $v', '%.4g' % d['value'], round(d['config']['kernel_ms_avg'],4), round(d['roofline']['frac'],3))"
  done
done
echo done
