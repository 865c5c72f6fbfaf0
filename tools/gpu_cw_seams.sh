# chain width (waves per workgroup) and rounds on the seam plan
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cws
run() {  # tag, lib, env, bench args
  local tag=$1 lib=$2 envs=$3; shift 3
  SEM_LIB_PATH=$PWD/build_variants/lib_$lib.so env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 "$@" > gpurun_out/cws/$tag.json 2> gpurun_out/cws/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/cws/$tag.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/cws/$tag.json')); c=d['config']; s=c['scatter_plan']; print('%-20s' % '$tag', round(c['kernel_ms_avg'],4), 'min', round(c['kernel_ms_min'],4), 'frac', round(d['roofline']['frac'],3), s['plan'], 'parity', (d.get('parity') or {}).get('rel_l2'))"
}
for pass in 1 2; do
  run p16_cw2_$pass p17base "" --p 16 --nex 198 --ney 198 || exit 1
  run p16_cw4_$pass p17cw4 "" --p 16 --nex 198 --ney 198 || exit 1
  run p16_cw2r2_$pass p17base "SEM_CHAIN_ROUNDS=2" --p 16 --nex 198 --ney 198 || exit 1
  run p12_cw4_$pass p13base "" --p 12 --nex 263 --ney 263 || exit 1
  run p12_cw2_$pass p13cw2 "" --p 12 --nex 263 --ney 263 || exit 1
  run p8s_cw4_$pass p9base "" --p 8 --nex 256 --ney 256 || exit 1
  run p8s_cw2_$pass p9cw2 "" --p 8 --nex 256 --ney 256 || exit 1
  run p8s_cw4r2_$pass p9base "SEM_CHAIN_ROUNDS=2" --p 8 --nex 256 --ney 256 || exit 1
done
