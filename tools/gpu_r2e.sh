set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2e
timeout -k 10 400 python -u -m pytest tests/test_gpu_unstructured.py tests/test_gpu_multirank.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2e/tests.log 2>&1 || { echo "tests failed"; grep -v "^    \|^  File" gpurun_out/r2e/tests.log | tail -40; exit 1; }
tail -2 gpurun_out/r2e/tests.log
timeout -k 10 300 python tools/unstructured_bench.py > gpurun_out/r2e/unstructured.log 2>&1 || { echo "ubench failed"; tail -20 gpurun_out/r2e/unstructured.log; exit 1; }
cat gpurun_out/r2e/unstructured.log | grep kind
