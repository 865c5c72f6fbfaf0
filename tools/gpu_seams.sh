# one-launch seam-atomic plan (SEM_PLAN=3) vs the coloured chains
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/seams
i=0
for pass in 1 2; do
  for spec in "8 1024" "16 198" "4 790" "12 263"; do
    set -- $spec
    for pm in -1 3; do
      i=$((i+1))
      SEM_PLAN=$pm timeout -k 10 300 python bench.py --no-cpu-baseline --p $1 --nex $2 --ney $2 --steps 30 > gpurun_out/seams/$i.json 2> gpurun_out/seams/$i.err || { echo "p$1 plan $pm failed"; tail -5 gpurun_out/seams/$i.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/seams/$i.json')); c=d['config']; print('p=%-3s plan=%-3s' % ('$1', '$pm'), round(c['kernel_ms_avg'],4), 'min', round(c['kernel_ms_min'],4), 'frac', round(d['roofline']['frac'],3), 'colours', c['scatter_plan']['colours'], 'zero', c['scatter_plan']['zero_list'], 'parity', d['parity']['rel_l2'])"
    done
  done
done
