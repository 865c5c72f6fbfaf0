set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2g
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_facade.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2g/tests.log 2>&1 || { echo "tests failed"; grep -v "^    \|^  File" gpurun_out/r2g/tests.log | tail -40; exit 1; }
tail -1 gpurun_out/r2g/tests.log
for e in 0 1; do
SEM_PCG_ENERGY=$e timeout -k 10 200 python bench.py --op pcg --steps 200 --warmup 5 > gpurun_out/r2g/pcg_e$e.json 2> gpurun_out/r2g/pcg_e$e.err || { echo "pcg bench failed"; tail -5 gpurun_out/r2g/pcg_e$e.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r2g/pcg_e$e.json')); print('energy=$e', round(d['ms_per_step'],4), 'ms/it', d['pcg']['final_relres'])"
SEM_PCG_ENERGY=$e timeout -k 10 200 python bench.py --op pcg --pcg-rtol 1e-10 --nex 128 --ney 128 > gpurun_out/r2g/pcgs_e$e.json 2> gpurun_out/r2g/pcgs_e$e.err || { echo "pcg solve failed"; tail -5 gpurun_out/r2g/pcgs_e$e.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r2g/pcgs_e$e.json')); print('solve energy=$e', d['pcg']['iterations'], round(d['pcg']['seconds'],4), d['pcg']['rel_l2_error_vs_manufactured'])"
done
