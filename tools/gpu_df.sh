# One-launch (dataflow) plan vs one launch per colour: tests, then an A/B
# over the BASELINE configurations in one call (bench.py, 30 steps; the
# parity spot check stays on).  Usage: bash tools/gpu_df.sh [tests|ab|all]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/df
what=${1:-all}
if [ "$what" != ab ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_one_launch.py > gpurun_out/df/tests.log 2>&1 || { tail -30 gpurun_out/df/tests.log; exit 1; }
  tail -3 gpurun_out/df/tests.log
fi
[ "$what" = tests ] && exit 0
run() {  # tag, env, bench args
  local tag=$1; shift
  local envs=$1; shift
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 "$@" > gpurun_out/df/$tag.json 2> gpurun_out/df/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/df/$tag.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/df/$tag.json')); c=d['config']; s=c['scatter_plan']; print('%-22s' % '$tag', round(c['kernel_ms_avg'],4), 'min', round(c['kernel_ms_min'],4), 'frac', round(d['roofline']['frac'],3), s['plan'], 'deps', s['dependencies'], 'lag', s['lag'], 'timeouts', s['wait_timeouts'], 'parity', d['parity']['rel_l2'])"
}
for pass in 1 2; do
  for spec in "8 1024" "16 198" "4 790" "8 256" "12 263"; do
    set -- $spec
    run p$1_$2_colours_$pass "SEM_DF=0" --p $1 --nex $2 --ney $2 || exit 1
    run p$1_$2_df_$pass "SEM_DF=1" --p $1 --nex $2 --ney $2 || exit 1
  done
done
for lag in 512 1024 4096; do
  run p8_1024_lag$lag "SEM_DF_LAG=$lag" || exit 1
done
run p8_1024_noticket "SEM_DF_TICKET=0" || exit 1
run axi6_512_colours "SEM_DF=0" --op axisym_stokes --p 6 --nex 512 --ney 512 || exit 1
run axi6_512_df "SEM_DF=1" --op axisym_stokes --p 6 --nex 512 --ney 512 || exit 1
run p16_198_lag1024 "SEM_DF_LAG=1024" --p 16 --nex 198 --ney 198 || exit 1
run p16_198_lag4096 "SEM_DF_LAG=4096" --p 16 --nex 198 --ney 198 || exit 1
