#!/bin/bash
# Round 3, call P: k_poisson_mfma17 at full cfg4 size (parity vs the oracle
# and vs extended precision), builds A/B at p = 16 198^2 (default colour
# launches, factors read early at 3 / 2 waves, 4 waves) against the column
# kernel, and the MFMA-utilisation and traffic counters of the default.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_seams.py tests/test_gpu_scale.py -m gpu -q -s --timeout 170 --timeout-method thread -p no:cacheprovider -k "mfma" > $O/pytest_mfma.log 2>&1; rc=$?; echo "pytest mfma rc=$rc"; grep -E "extended|passed|failed" $O/pytest_mfma.log | tail -6
fatal $rc pytest
grep -q " passed" $O/pytest_mfma.log || exit 1
for rep in 1 2; do
  for v in main gpre3 gpre2 mf4 column; do
    k=mfma; unset SEM_LIB_PATH
    [ $v = column ] && k=column
    [ $v != main ] && [ $v != column ] && export SEM_LIB_PATH=$PWD/build_variants/libsem_$v.so
    timeout -k 10 180 python bench.py --no-cpu-baseline --p 16 --nex 198 --ney 198 --geometry stored --kernel $k > $O/p16_${v}_$rep.json 2> $O/p16_${v}_$rep.log; rc=$?
    echo "p16 $v $rep rc=$rc $(python -c "import json;d=json.load(open('$O/p16_${v}_$rep.json'));c=d['config'];print(round(d['ms_per_step'],4), [round(x,4) for x in c['kernel_ms_quartiles']], d['roofline']['frac'], d.get('parity',{}).get('rel_l2'), c['scatter_plan']['plan'])" 2>/dev/null)"
    fatal $rc bench
  done
done
unset SEM_LIB_PATH
timeout -k 10 180 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/p16_trace -o run -- python bench.py --no-cpu-baseline --p 16 --nex 198 --ney 198 --geometry stored --kernel mfma > $O/p16_trace.log 2>&1; rc=$?; echo "trace rc=$rc"
fatal $rc trace
head -4 $O/p16_trace/run_kernel_stats.csv | cut -c1-150
for set in "SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU" "GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "k_poisson_mfma17" --output-format csv -d $O/pmc_$tag -o run -- python bench.py --no-cpu-baseline --no-check --p 16 --nex 198 --ney 198 --geometry stored --kernel mfma --steps 8 --warmup 2 > $O/pmc_$tag.log 2>&1; rc=$?; echo "pmc $tag rc=$rc"
  fatal $rc pmc
done
python tools/pmc_traffic.py $O/pmc_FETCH_SIZE/run_counter_collection.csv $O/pmc_WRITE_SIZE/run_counter_collection.csv $O/traffic.json --kernel k_poisson_mfma17 --launches-per-action 4 > /dev/null 2>&1; head -c 600 $O/traffic.json
