set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2d
timeout -k 10 300 python -u -m pytest tests/test_gpu_facade.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2d/facade.log 2>&1 || { echo "facade tests failed"; tail -40 gpurun_out/r2d/facade.log; exit 1; }
tail -2 gpurun_out/r2d/facade.log
timeout -k 10 60 python examples/poisson.py > gpurun_out/r2d/example.log 2>&1 || { echo "example failed"; tail -20 gpurun_out/r2d/example.log; exit 1; }
tail -1 gpurun_out/r2d/example.log
V9="$V9" V17="$V17" bash tools/gpu_var2.sh
