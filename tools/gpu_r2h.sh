set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2h




mkdir -p gpurun_out/r2h/sweep
for cfg in "14 227" "16 198"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --no-cpu-baseline --p $1 --nex $2 --ney $2 --steps 20 > gpurun_out/r2h/sweep/p$1.json 2> gpurun_out/r2h/sweep/p$1.err || { echo "sweep p$1 failed"; tail -3 gpurun_out/r2h/sweep/p$1.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r2h/sweep/p$1.json')); print('p=$1', '%.4g' % d['value'], round(d['config']['kernel_ms_avg'],4), d['config']['kernel_family'], d['config']['geometry'], 'frac', round(d['roofline']['frac'],3), 'parity', d['parity']['rel_l2'])"
done
timeout -k 10 200 python bench.py --no-cpu-baseline --nex 256 --ney 256 --steps 50 > gpurun_out/r2h/sweep/cfg2.json 2> gpurun_out/r2h/sweep/cfg2.err || { echo "cfg2 failed"; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r2h/sweep/cfg2.json')); print('cfg2', '%.4g' % d['value'], round(d['config']['kernel_ms_avg'],4), 'frac', round(d['roofline']['frac'],3))"
timeout -k 10 200 python bench.py --no-cpu-baseline --op axisym_stokes --p 6 --nex 512 --ney 512 --steps 20 > gpurun_out/r2h/sweep/cfg5.json 2> gpurun_out/r2h/sweep/cfg5.err || { echo "cfg5 failed"; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r2h/sweep/cfg5.json')); print('cfg5', '%.4g' % d['value'], round(d['config']['kernel_ms_avg'],4), 'frac', round(d['roofline']['frac'],3))"
