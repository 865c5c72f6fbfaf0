# Seam plan (SEM_SEAM=1: one launch in element order + k_seam_sum) vs the
# colour launches: tests, then an A/B over the BASELINE configurations.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/seam2
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_gpu_seams.py > gpurun_out/seam2/tests.log 2>&1 || { tail -30 gpurun_out/seam2/tests.log; exit 1; }
tail -2 gpurun_out/seam2/tests.log
run() {  # tag, env, bench args
  local tag=$1; shift
  local envs=$1; shift
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 "$@" > gpurun_out/seam2/$tag.json 2> gpurun_out/seam2/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/seam2/$tag.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/seam2/$tag.json')); c=d['config']; s=c['scatter_plan']; print('%-22s' % '$tag', round(c['kernel_ms_avg'],4), 'min', round(c['kernel_ms_min'],4), 'frac', round(d['roofline']['frac'],3), s['plan'], 'parity', (d.get('parity') or {}).get('rel_l2'))"
}
for pass in 1 2; do
  for spec in "8 1024" "16 198" "4 790" "8 256" "12 263" "2 1581" "6 527"; do
    set -- $spec
    run p$1_$2_colours_$pass "SEM_SEAM=0" --p $1 --nex $2 --ney $2 || exit 1
    run p$1_$2_seams_$pass "SEM_SEAM=1" --p $1 --nex $2 --ney $2 || exit 1
  done
done
