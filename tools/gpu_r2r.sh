# final default bench line (sustained defaults) and its rocprofv3 kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2r
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline > $O/trace_bench.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
head -4 $O/trace/run_kernel_stats.csv
