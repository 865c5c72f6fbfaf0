# p = 16 (198^2, stored, column kernel) timing ablations (diagnostic variant
# builds; their results are wrong by design): where the time goes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/p16diag
run() {  # tag, lib, env
  SEM_LIB_PATH=$PWD/build_variants/lib_$2.so env $3 timeout -k 10 200 python bench.py --no-cpu-baseline --no-check --steps 30 --p 16 --nex 198 --ney 198 > gpurun_out/p16diag/$1.json 2> gpurun_out/p16diag/$1.err || { echo "$1 failed"; tail -5 gpurun_out/p16diag/$1.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/p16diag/$1.json')); c=d['config']; print('%-18s' % '$1', round(c['kernel_ms_avg'],4), 'min', round(c['kernel_ms_min'],4), 'frac', round(d['roofline']['frac'],3))"
}
for pass in 1 2; do
  for lib in p17base p17nostore p17nocomp p17nog p17nou p17nosync p17rmwst; do
    run ${lib}_$pass $lib "" || exit 1
  done
  run p17base_r2_$pass p17base "SEM_CHAIN_ROUNDS=2" || exit 1
  run p17base_df_$pass p17base "SEM_DF=1" || exit 1
done
