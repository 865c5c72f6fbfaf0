set -o pipefail
cd $GRAFT_REPO_ROOT
for v in ${VARIANTS:-base}; do
  SEM_LIB_PATH=$PWD/build_variants/lib_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 ${BENCH_ARGS} > gpurun_out/var_$v.json 2>gpurun_out/var_$v.err || { echo "variant $v failed"; tail -3 gpurun_out/var_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/var_$v.json')); print('$v', round(d['config']['kernel_ms_avg'],4), round(d['roofline']['frac'],4), d['config']['scatter_plan'])"
done
