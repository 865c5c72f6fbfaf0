# GPU parity tests on one library variant, then the headline bench per variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TEST_VARIANT:-np4}
SEM_LIB_PATH=$PWD/build_variants/lib_$T.so timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests_$T.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$T.log
bash tools/gpu_variants.sh
