# axisymmetric Stokes block: NODAL vs STORED geometry per order (~9.4e6 nodes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/axisweep
for spec in "2 1536" "4 768" "8 384" "10 307" "12 256" "16 192"; do
  set -- $spec
  for g in stored nodal; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --op axisym_stokes --p $1 --nex $2 --ney $2 --steps 30 --geometry $g > gpurun_out/axisweep/p$1-$g.json 2> gpurun_out/axisweep/p$1-$g.err || { echo "p$1 $g failed"; tail -5 gpurun_out/axisweep/p$1-$g.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/axisweep/p$1-$g.json')); print('p=%-3s %-7s' % ('$1', '$g'), round(d['config']['kernel_ms_avg'],4), 'min', round(d['config']['kernel_ms_min'],4), 'frac', round(d['roofline']['frac'],3))"
  done
done
