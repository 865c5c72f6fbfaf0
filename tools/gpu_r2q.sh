# headline under sustained load: geometry x plan, 50 and 200 steps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2q
mkdir -p $O
for steps in 50 200; do
  for geo in nodal stored; do
    for pm in 0 1; do
      tag=${geo}_seam${pm}_s$steps
      SEM_SEAM=$pm timeout -k 10 200 python bench.py --no-cpu-baseline --steps $steps --geometry $geo > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
      python -c "import json; d=json.load(open('$O/$tag.json')); c=d['config']; print('%-20s' % '$tag', round(d['ms_per_step'],4), 'kern', round(c['kernel_ms_avg'],4), 'min', round(c['kernel_ms_min'],4), 'frac', round(d['roofline']['frac'],3))"
    done
  done
done
