# final build check: full GPU suite, smoke(), p = 16 under rocprofv3, default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2n
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace_p16_198 -o run -- python3 bench.py --no-cpu-baseline --steps 20 --p 16 --nex 198 --ney 198 > $O/trace_p16_198.json 2> $O/trace_p16_198.err || { tail -5 $O/trace_p16_198.err; exit 1; }
head -4 $O/trace_p16_198/run_kernel_stats.csv
timeout -k 10 300 python bench.py --p 16 --nex 198 --ney 198 --no-cpu-baseline > $O/bench_p16.json 2> $O/bench_p16.err || { tail -5 $O/bench_p16.err; exit 1; }
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
cat $O/bench_p16.json
cat $O/bench_default.json
