#!/bin/bash
# Round 3, call B: parity numbers at p > 10, captured-step test, the 8-rank
# rehearsal, a 2-rank kernel trace (overlap), PMC passes of the headline.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -k "extended" tests/test_gpu_multirank.py::test_captured_step_equals_eager -s -q --timeout 170 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "extended|enqueue|passed|failed" $O/pytest.log
fatal $rc pytest
# 8 ranks of the cfg3 strong-scaling flow on one device (torch transport)
timeout -k 10 300 python bench.py --rehearse-one-gpu --gpus 8 --steps 20 --warmup 5 --deadline 280 > $O/rehearse8.json 2> $O/rehearse8.log; rc=$?; echo "rehearse8 rc=$rc"; tail -c 600 $O/rehearse8.json
fatal $rc rehearse8
# 2 ranks, each under its own kernel trace (same device clock: overlap check)
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 \
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace2_r$r -o run -- python bench.py --rehearse-one-gpu --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline --deadline 250 > $O/trace2_r$r.json 2> $O/trace2_r$r.log &
done
wait; echo "trace2 done"; tail -c 300 $O/trace2_r0.json
# PMC passes, headline workload, default plan
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" "GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "k_poisson_apply|k_seam_sum" --output-format csv -d $O/pmc_$tag -o run -- python bench.py --no-cpu-baseline --no-check --steps 8 --warmup 2 > $O/pmc_$tag.log 2>&1; rc=$?; echo "pmc $tag rc=$rc"
  fatal $rc pmc
done
python tools/pmc_traffic.py $O/pmc_FETCH_SIZE/run_counter_collection.csv $O/pmc_WRITE_SIZE/run_counter_collection.csv $O/traffic.json --kernel k_poisson_apply --launches-per-action 1 > /dev/null 2>&1; cat $O/traffic.json | head -20
# geometry A/B on the block-seam plan
for g in nodal stored; do
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --geometry $g > $O/bench_$g.json 2> $O/bench_$g.log; rc=$?
  echo "bench $g rc=$rc $(python -c "import json;d=json.load(open('$O/bench_$g.json'));c=d['config'];print(round(d['ms_per_step'],4), c['kernel_ms_quartiles'], c['scatter_plan']['plan'])" 2>/dev/null)"
  fatal $rc bench
done
