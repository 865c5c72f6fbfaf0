# shader clock per colour launch over a sustained headline run: GRBM_GUI_ACTIVE
# (GPU-busy cycles) per dispatch next to its kernel-trace duration
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/clock
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --kernel-include-regex k_poisson_apply --output-format csv -d $O/pmc -o run -- python3 bench.py --no-cpu-baseline --no-check --steps 50 > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc.log; exit 1; }
ls $O/pmc
