set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TEST_VARIANT=pre1 VARIANTS="np4ns pre1 pre2 pre1nn" bash tools/gpu_occ.sh || exit 1
BENCH_ARGS="--geometry stored" VARIANTS="np4ns pre1" bash tools/gpu_variants.sh || exit 1
