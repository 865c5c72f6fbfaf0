# round 2: multi-rank path (ranks on one GPU), device PCG, strong-scaling bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2b
O=gpurun_out/r2b
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 200 --timeout-method thread > $O/multirank.log 2>&1 || { echo "multirank tests failed"; tail -40 $O/multirank.log; exit 1; }
tail -3 $O/multirank.log
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python bench.py --steps 20 > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
timeout -k 10 200 python bench.py --gpus 2 --rehearse-one-gpu --steps 5 --warmup 2 --nex 256 --ney 256 > $O/bench_rehearse2.json 2> $O/bench_rehearse2.err || { echo "rehearse failed"; tail -20 $O/bench_rehearse2.err; exit 1; }
cat $O/bench_rehearse2.json
timeout -k 10 200 python bench.py --op pcg --steps 200 --warmup 5 > $O/bench_pcg_cfg3.json 2> $O/bench_pcg_cfg3.err || { echo "pcg bench failed"; tail -20 $O/bench_pcg_cfg3.err; exit 1; }
cat $O/bench_pcg_cfg3.json
timeout -k 10 200 python bench.py --op pcg --pcg-rtol 1e-10 --nex 128 --ney 128 > $O/bench_pcg_solve128.json 2> $O/bench_pcg_solve128.err || { echo "pcg solve failed"; tail -20 $O/bench_pcg_solve128.err; exit 1; }
cat $O/bench_pcg_solve128.json
