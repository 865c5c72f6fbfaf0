#!/bin/bash
# Round 3, call D: D coefficients in LDS vs scalar loads at n >= 10 (A/B in
# one call), GPU suite, PCG kernel trace, cfg5 on the AUTO block layout.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 170 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
fatal $rc pytest
run() {  # tag, env, args
  tag=$1; shift; envs=$1; shift
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --warmup 5 "$@" > $O/$tag.json 2> $O/$tag.log; rc=$?
  echo "$tag rc=$rc $(python -c "import json;d=json.load(open('$O/$tag.json'));c=d['config'];print(round(d['ms_per_step'],4), round(c['kernel_ms_avg'],4), [round(x,4) for x in c['kernel_ms_quartiles']], c['scatter_plan']['plan'], c['geometry'], round(d['roofline']['frac'],3), d.get('parity',{}).get('rel_l2'))" 2>/dev/null)"
  fatal $rc $tag
}
for rep in 1 2; do
for cfg in "10 316" "12 263" "14 227" "16 198"; do
  set -- $cfg
  run p$1_lds_$rep SEM_X=1 --p $1 --nex $2 --ney $2 --steps 50
  run p$1_sgpr_$rep SEM_LIB_PATH=$PWD/build_variants/lib_dsgpr.so --p $1 --nex $2 --ney $2 --steps 50
done
done
for rep in 1 2; do
run cfg5_fields_first_$rep SEM_X=1 --op axisym_stokes --p 6 --nex 512 --ney 512 --steps 50
run cfg5_two_planes_$rep SEM_LIB_PATH=$PWD/build_variants/lib_axi2plane.so --op axisym_stokes --p 6 --nex 512 --ney 512 --steps 50
done
timeout -k 10 200 python -u -m pytest tests/test_gpu_multirank.py::test_captured_step_equals_eager -s -q --timeout 170 --timeout-method thread -p no:cacheprovider > $O/captured.log 2>&1; rc=$?; echo "captured rc=$rc"; grep -E "enqueue|passed|failed" $O/captured.log
fatal $rc captured
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/pcg_trace -o run -- python bench.py --op pcg --steps 30 --warmup 3 > $O/pcg_trace.log 2>&1; rc=$?; echo "pcg trace rc=$rc"
fatal $rc pcgtrace
head -12 $O/pcg_trace/run_kernel_stats.csv | cut -c1-200
