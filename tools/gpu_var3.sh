# A/B of diagnostic variants (build_variants/): SPECS="variant|bench args;..." , two passes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/var
i=0
for pass in 1 2; do
  IFS=';' read -ra items <<< "$SPECS"
  for it in "${items[@]}"; do
    v="${it%%|*}"; a="${it#*|}"; i=$((i+1))
    SEM_LIB_PATH=$PWD/build_variants/lib_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-check --steps 30 $a > gpurun_out/var/$i.json 2> gpurun_out/var/$i.err || { echo "variant $v failed"; tail -3 gpurun_out/var/$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/var/$i.json')); print('%-8s %-40s' % ('$v', '$a'), round(d['config']['kernel_ms_avg'],4), 'min', round(d['config']['kernel_ms_min'],4), 'frac', round(d['roofline']['frac'],3))"
  done
done
