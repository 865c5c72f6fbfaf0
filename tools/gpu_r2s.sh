# PMC HBM traffic of the headline on the final build (separate passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2s
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex k_poisson_apply --output-format csv -d $O/pmc_$c -o run -- python3 bench.py --no-cpu-baseline --no-check --steps 4 --warmup 1 > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $O/pmc_$c.log; exit 1; }
done
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['traffic'], d['roofline']['traffic_source'])"
