#!/bin/bash
# Round 3, call M: the n = 17 MFMA kernel (k_poisson_mfma17): parity tests,
# then p = 16 198^2 MFMA against the column kernel, alternating on one box.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03m
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "mfma" > $O/pytest_mfma.log 2>&1; rc=$?; echo "pytest mfma rc=$rc"; tail -3 $O/pytest_mfma.log
fatal $rc pytest
[ $rc = 0 ] || exit $rc
for rep in 1 2; do
  for k in mfma column; do
    timeout -k 10 180 python bench.py --no-cpu-baseline --p 16 --nex 198 --ney 198 --geometry stored --kernel $k > $O/p16_${k}_$rep.json 2> $O/p16_${k}_$rep.log; rc=$?
    echo "p16 $k $rep rc=$rc $(python -c "import json;d=json.load(open('$O/p16_${k}_$rep.json'));c=d['config'];print(round(d['ms_per_step'],4), [round(x,4) for x in c['kernel_ms_quartiles']], d['roofline']['frac'], d.get('parity',{}).get('rel_l2'))" 2>/dev/null)"
    fatal $rc bench
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/p16_trace -o run -- python bench.py --no-cpu-baseline --p 16 --nex 198 --ney 198 --geometry stored --kernel mfma > $O/p16_trace.log 2>&1; rc=$?; echo "trace rc=$rc"
fatal $rc trace
head -5 $O/p16_trace/run_kernel_stats.csv | cut -c1-150
