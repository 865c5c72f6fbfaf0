# after the seam-sum change and AUTO without MFMA: seam / one-launch /
# parity tests, the p-sweep on AUTO, chain width on the seam plan
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2m
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_seams.py tests/test_gpu_scale.py tests/test_gpu_parity.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); c=d['config']; s=c['scatter_plan']; print('%-14s' % '$tag', round(c['kernel_ms_avg'],4), 'min', round(c['kernel_ms_min'],4), 'frac', round(d['roofline']['frac'],3), c['kernel_family'], s['plan'], 'parity', (d.get('parity') or {}).get('rel_l2'))"
}
for spec in "2 1581" "4 790" "6 527" "8 395" "10 316" "12 263" "14 227" "16 198" "8 256"; do
  set -- $spec
  run p$1_$2 --p $1 --nex $2 --ney $2 || exit 1
done
run axi6_512 --op axisym_stokes --p 6 --nex 512 --ney 512 || exit 1
bash tools/gpu_cw_seams.sh || exit 1
