# Round 2 (late): full GPU suite on the AUTO seam plan, the seam threshold
# probe, the default bench line and its kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2k
what=${1:-all}
if [ "$what" = all ] || [ "$what" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/r2k/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r2k/gpu_tests.log; exit 1; }
  tail -3 gpurun_out/r2k/gpu_tests.log
fi
run() {  # tag, env, bench args
  local tag=$1; shift
  local envs=$1; shift
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 "$@" > gpurun_out/r2k/$tag.json 2> gpurun_out/r2k/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/r2k/$tag.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/r2k/$tag.json')); c=d['config']; s=c['scatter_plan']; print('%-24s' % '$tag', round(c['kernel_ms_avg'],4), 'min', round(c['kernel_ms_min'],4), 'frac', round(d['roofline']['frac'],3), s['plan'], 'cpc', s['chains_per_colour'][:1], 'parity', (d.get('parity') or {}).get('rel_l2'))"
}
if [ "$what" = all ] || [ "$what" = probe ]; then
  for spec in "8 128 1024" "8 384 384" "8 512 512" "10 316 316" "6 256 256" "4 395 395" "9 351 351"; do
    set -- $spec
    run p$1_$2x$3_colours "SEM_SEAM=0" --p $1 --nex $2 --ney $3 || exit 1
    run p$1_$2x$3_seams "SEM_SEAM=1" --p $1 --nex $2 --ney $3 || exit 1
  done
fi
if [ "$what" = all ] || [ "$what" = bench ]; then
  timeout -k 10 300 python bench.py > gpurun_out/r2k/bench_default.json 2> gpurun_out/r2k/bench_default.err || { tail -5 gpurun_out/r2k/bench_default.err; exit 1; }
  cat gpurun_out/r2k/bench_default.json
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2k/prof -o kt -- python3 bench.py --no-cpu-baseline --steps 20 > gpurun_out/r2k/prof_bench.json 2> gpurun_out/r2k/prof.err || { tail -5 gpurun_out/r2k/prof.err; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2k/prof16 -o kt -- python3 bench.py --no-cpu-baseline --steps 20 --p 16 --nex 198 --ney 198 > gpurun_out/r2k/prof16_bench.json 2> gpurun_out/r2k/prof16.err || { tail -5 gpurun_out/r2k/prof16.err; exit 1; }
  find gpurun_out/r2k/prof gpurun_out/r2k/prof16 -name '*stats*' | head
fi
