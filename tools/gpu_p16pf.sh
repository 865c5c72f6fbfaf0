# p = 16 (198^2, stored, column kernel): read-modify-write operand prefetch
# variants at n = 17 (SEM_RMW_PREFETCH_17, occupancy bound) and no-return
# atomics for the read-modify-writes (SEM_RMW_ATOMIC)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/p16pf
run() {  # tag, lib, env
  SEM_LIB_PATH=$PWD/build_variants/lib_$2.so env $3 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --p 16 --nex 198 --ney 198 > gpurun_out/p16pf/$1.json 2> gpurun_out/p16pf/$1.err || { echo "$1 failed"; tail -5 gpurun_out/p16pf/$1.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/p16pf/$1.json')); c=d['config']; print('%-18s' % '$1', round(c['kernel_ms_avg'],4), 'min', round(c['kernel_ms_min'],4), 'frac', round(d['roofline']['frac'],3), 'parity', d['parity']['rel_l2'])"
}
for pass in 1 2; do
  for lib in p17base p17pf1w3 p17pf2w3 p17pf1 p17pf2 p17rmwat; do
    run ${lib}_$pass $lib "" || exit 1
  done
done
