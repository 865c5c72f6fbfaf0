# axisymmetric seams: tests, cfg5 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2p
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_seams.py tests/test_gpu_one_launch.py tests/test_gpu_multirank.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for pm in 0 1; do
  for spec in "6 512" "6 128"; do
    set -- $spec
    SEM_SEAM=$pm timeout -k 10 200 python bench.py --op axisym_stokes --no-cpu-baseline --steps 30 --p $1 --nex $2 --ney $2 > $O/axi$1_$2_seam$pm.json 2> $O/axi$1_$2_seam$pm.err || { tail -5 $O/axi$1_$2_seam$pm.err; exit 1; }
    python -c "import json; d=json.load(open('$O/axi$1_$2_seam$pm.json')); c=d['config']; print('axi p=$1 $2^2 seam=$pm', round(c['kernel_ms_avg'],4), 'min', round(c['kernel_ms_min'],4), 'frac', round(d['roofline']['frac'],3), c['scatter_plan']['plan'])"
  done
done
