# A/B of diagnostic variants (build_variants/), two passes each, in one call
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/var
run() {  # name, bench args
  SEM_LIB_PATH=$PWD/build_variants/lib_$1.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-check --steps 30 $2 > gpurun_out/var/$1.json 2> gpurun_out/var/$1.err || { echo "variant $1 failed"; tail -3 gpurun_out/var/$1.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/var/$1.json')); print('$1', round(d['config']['kernel_ms_avg'],4), 'min', round(d['config']['kernel_ms_min'],4), 'frac', round(d['roofline']['frac'],3))"
}
for pass in 1 2; do
  for v in $V9; do run $v "" || exit 1; done
  for v in $V17; do run $v "--p 16 --nex 198 --ney 198" || exit 1; done
done
