# axisymmetric Stokes block: parity with NODAL geometry, then A/B of the
# geometry modes and the 3-wave variant on the cfg5 workload
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/axi
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -k "axisym or config5" > gpurun_out/axi/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/axi/tests.log; exit 1; }
tail -3 gpurun_out/axi/tests.log
for pass in 1 2; do
  for spec in "default|stored" "default|nodal" "axl3|nodal"; do
    v="${spec%%|*}"; g="${spec#*|}"
    if [ "$v" != default ]; then export SEM_LIB_PATH=$PWD/build_variants/lib_$v.so; else unset SEM_LIB_PATH; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --op axisym_stokes --p 6 --nex 512 --ney 512 --steps 30 --geometry $g > gpurun_out/axi/$v-$g-$pass.json 2> gpurun_out/axi/$v-$g-$pass.err || { echo "$v $g failed"; tail -5 gpurun_out/axi/$v-$g-$pass.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/axi/$v-$g-$pass.json')); print('%-8s %-7s' % ('$v', '$g'), round(d['config']['kernel_ms_avg'],4), 'min', round(d['config']['kernel_ms_min'],4), 'frac', round(d['roofline']['frac'],3))"
  done
done
