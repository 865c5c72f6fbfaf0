# BASELINE cfg2 / cfg4 / cfg5 on the final build with the sustained bench defaults
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2t
mkdir -p $O
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); c=d['config']; r=d['roofline']; print('%-10s' % '$tag', round(c['kernel_ms_avg'],4), round(d['value']/1e10,2), round(r['frac'],3), round(r['frac_streamed_min'],3), c['geometry'], c['scatter_plan']['plan'], (d.get('parity') or {}).get('rel_l2'))"
}
for spec in "8 256" "2 1581" "4 790" "6 527" "8 395" "12 263" "16 198"; do
  set -- $spec
  run p$1_$2 --p $1 --nex $2 --ney $2 || exit 1
done
run axi6_512 --op axisym_stokes --p 6 --nex 512 --ney 512 || exit 1
