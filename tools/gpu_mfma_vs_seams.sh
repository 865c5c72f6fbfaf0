# p = 13..15 at ~1e7 DOF: the MFMA element kernel (AUTO's pick) vs the column
# kernel on the seam plan
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/mvs
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 "$@" > gpurun_out/mvs/$tag.json 2> gpurun_out/mvs/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/mvs/$tag.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/mvs/$tag.json')); c=d['config']; s=c['scatter_plan']; print('%-20s' % '$tag', round(c['kernel_ms_avg'],4), 'min', round(c['kernel_ms_min'],4), 'frac', round(d['roofline']['frac'],3), c['kernel_family'], s['plan'], 'parity', (d.get('parity') or {}).get('rel_l2'))"
}
for pass in 1 2; do
  for spec in "13 243" "14 227" "15 212" "10 316"; do
    set -- $spec
    run p$1_mfma_$pass --p $1 --nex $2 --ney $2 --kernel mfma || exit 1
    run p$1_column_$pass --p $1 --nex $2 --ney $2 --kernel column || exit 1
  done
done
