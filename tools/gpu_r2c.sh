set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2c
O=gpurun_out/r2c
timeout -k 10 200 python tools/dd_stress.py base > $O/stress.log 2>&1 || { echo "stress failed"; tail -20 $O/stress.log; exit 1; }
grep check= $O/stress.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread > $O/scale.log 2>&1 || { echo "scale tests failed"; tail -40 $O/scale.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/scale.log
