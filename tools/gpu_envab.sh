# A/B of runtime environment knobs: SPECS="ENV=VAL|bench args;..." (ENV part may be '-'), two passes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/envab
i=0
for pass in 1 2; do
  IFS=';' read -ra items <<< "$SPECS"
  for it in "${items[@]}"; do
    e="${it%%|*}"; a="${it#*|}"; i=$((i+1))
    if [ "$e" = "-" ]; then e="SEM_NOTHING=1"; fi
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --no-check --steps 30 $a > gpurun_out/envab/$i.json 2> gpurun_out/envab/$i.err || { echo "run $e failed"; tail -3 gpurun_out/envab/$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/envab/$i.json')); print('%-20s %-36s' % ('$e', '$a'), round(d['config']['kernel_ms_avg'],4), 'min', round(d['config']['kernel_ms_min'],4), 'frac', round(d['roofline']['frac'],3))"
  done
done
