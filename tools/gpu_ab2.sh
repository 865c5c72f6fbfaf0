set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
BENCH_ARGS="--op axisym_stokes --p 6 --nex 512 --ney 512" VARIANTS="head base head base" bash tools/gpu_variants.sh || exit 1
BENCH_ARGS="--p 12 --nex 263 --ney 263" VARIANTS="head base" bash tools/gpu_variants.sh || exit 1
VARIANTS="head base" bash tools/gpu_variants.sh || exit 1
