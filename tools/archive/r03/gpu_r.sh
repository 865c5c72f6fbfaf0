#!/bin/bash
# Round 3, call R: persistent pipelined k_poisson_mfma17p (next triple's map
# and u read while the current one computes): parity, then p = 16 198^2
# against the one-pair-per-triple form, the element seam plan and the column
# kernel, alternating on one box.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_seams.py tests/test_gpu_scale.py -m gpu -q -s --timeout 170 --timeout-method thread -p no:cacheprovider -k "mfma" > $O/pytest_mfma.log 2>&1; rc=$?; echo "pytest mfma rc=$rc"; grep -E "extended|passed|failed" $O/pytest_mfma.log | tail -4
fatal $rc pytest
grep -q " passed" $O/pytest_mfma.log || exit 1
for rep in 1 2; do
  for v in persist np seams column; do
    k=mfma; unset SEM_LIB_PATH SEM_SEAM
    [ $v = column ] && k=column
    [ $v = np ] && export SEM_LIB_PATH=$PWD/build_variants/libsem_np.so
    [ $v = seams ] && export SEM_SEAM=1
    timeout -k 10 180 python bench.py --no-cpu-baseline --p 16 --nex 198 --ney 198 --geometry stored --kernel $k > $O/p16_${v}_$rep.json 2> $O/p16_${v}_$rep.log; rc=$?
    echo "p16 $v $rep rc=$rc $(python -c "import json;d=json.load(open('$O/p16_${v}_$rep.json'));c=d['config'];print(round(d['ms_per_step'],4), [round(x,4) for x in c['kernel_ms_quartiles']], d['roofline']['frac'], d.get('parity',{}).get('rel_l2'), c['scatter_plan']['plan'])" 2>/dev/null)"
    fatal $rc bench
  done
done
unset SEM_LIB_PATH SEM_SEAM
timeout -k 10 180 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/p16_trace -o run -- python bench.py --no-cpu-baseline --p 16 --nex 198 --ney 198 --geometry stored --kernel mfma > $O/p16_trace.log 2>&1; rc=$?; echo "trace rc=$rc"
fatal $rc trace
head -3 $O/p16_trace/run_kernel_stats.csv | cut -c1-150
