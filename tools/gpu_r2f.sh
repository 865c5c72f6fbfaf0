set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2f
timeout -k 10 500 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_unstructured.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2f/tests.log 2>&1 || { echo "tests failed"; grep -v "^    \|^  File" gpurun_out/r2f/tests.log | tail -40; exit 1; }
tail -2 gpurun_out/r2f/tests.log
