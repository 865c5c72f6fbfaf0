# p = 16 (cfg4, 198^2): occupancy variants of the column kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/p16
i=0
for pass in 1 2; do
  for spec in "default|1" "w4_17|1" "w4_17|0" "default|0"; do
    v="${spec%%|*}"; m="${spec#*|}"; i=$((i+1))
    if [ "$v" != default ]; then export SEM_LIB_PATH=$PWD/build_variants/lib_$v.so; else unset SEM_LIB_PATH; fi
    SEM_MAP16=$m timeout -k 10 200 python bench.py --no-cpu-baseline --p 16 --nex 198 --ney 198 --steps 30 > gpurun_out/p16/$i.json 2> gpurun_out/p16/$i.err || { echo "$v failed"; tail -5 gpurun_out/p16/$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/p16/$i.json')); print('%-8s map16=%s' % ('$v', '$m'), round(d['config']['kernel_ms_avg'],4), 'min', round(d['config']['kernel_ms_min'],4), 'frac', round(d['roofline']['frac'],3), d['parity']['rel_l2'])"
  done
done
