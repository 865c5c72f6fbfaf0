# final build: the bench's multi-rank flow rehearsed on one GPU (2 ranks,
# torch transport), the PCG leg, and p = 8 1024^2 seams vs colours again
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2o
mkdir -p $O
timeout -k 10 300 python bench.py --rehearse-one-gpu --gpus 2 --no-cpu-baseline --steps 20 > $O/rehearse2.json 2> $O/rehearse2.err || { tail -10 $O/rehearse2.err; exit 1; }
cat $O/rehearse2.json
timeout -k 10 300 python bench.py --op pcg --no-cpu-baseline --steps 20 > $O/pcg.json 2> $O/pcg.err || { tail -10 $O/pcg.err; exit 1; }
cat $O/pcg.json
for pm in 0 1; do
  SEM_SEAM=$pm timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > $O/p8_seam$pm.json 2> $O/p8_seam$pm.err || { tail -5 $O/p8_seam$pm.err; exit 1; }
  python -c "import json; d=json.load(open('$O/p8_seam$pm.json')); c=d['config']; print('seam=$pm', round(c['kernel_ms_avg'],4), 'min', round(c['kernel_ms_min'],4), c['scatter_plan']['plan'])"
done
