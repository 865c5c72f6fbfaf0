set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench_r1.json 2> gpurun_out/bench_r1.err || { echo "bench failed"; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_r1 -o run -- python bench.py --no-cpu-baseline --steps 20 > gpurun_out/prof_r1.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
