# Round 2 (final): GPU suite, MFMA vs column+seams at p = 13..15, default
# bench line, rocprofv3 kernel-trace stats (csv) of the headline and of the
# seam-plan configurations, PMC traffic of p = 16.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash tools/gpu_mfma_vs_seams.sh || exit 1
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
prof() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/$tag -o run -- python3 bench.py --no-cpu-baseline --steps 20 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; return 1; }
}
prof trace_p8_1024 || exit 1
prof trace_p16_198 --p 16 --nex 198 --ney 198 || exit 1
prof trace_p8_256 --p 8 --nex 256 --ney 256 || exit 1
prof trace_p12_263 --p 12 --nex 263 --ney 263 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex 'k_poisson_apply|k_seam_sum' --output-format csv -d $O/pmc16_$c -o run -- python3 bench.py --no-cpu-baseline --no-check --steps 4 --warmup 1 --p 16 --nex 198 --ney 198 > $O/pmc16_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $O/pmc16_$c.log; exit 1; }
done
find $O -name '*kernel_stats*' | head
