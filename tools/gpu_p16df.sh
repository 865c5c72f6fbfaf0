# p = 16 (198^2) on the one-launch plan: chain width (2 / 4 waves, variant
# builds from tools/build_variants.py ... --only-n 17) x rounds per chain.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/p16df
run() {  # tag, lib, env
  SEM_LIB_PATH=$PWD/build_variants/lib_$2.so env $3 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --p 16 --nex 198 --ney 198 > gpurun_out/p16df/$1.json 2> gpurun_out/p16df/$1.err || { echo "$1 failed"; tail -5 gpurun_out/p16df/$1.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/p16df/$1.json')); c=d['config']; s=c['scatter_plan']; print('%-18s' % '$1', round(c['kernel_ms_avg'],4), 'min', round(c['kernel_ms_min'],4), 'frac', round(d['roofline']['frac'],3), s['plan'], 'timeouts', s['wait_timeouts'], 'parity', d['parity']['rel_l2'])"
}
for pass in 1 2; do
  for lib in p17base p17cw4; do
    for r in 1 2; do
      run ${lib}_r${r}_$pass $lib "SEM_CHAIN_ROUNDS=$r" || exit 1
    done
  done
  run p17base_colours_$pass p17base "SEM_DF=0" || exit 1
done
