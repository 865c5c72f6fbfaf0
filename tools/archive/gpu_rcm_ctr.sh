#!/bin/bash
# PMC passes (HBM bytes, L2 hit rate, wait) of the 2-D element kernel under
# lexicographic vs RCM (reference default) node numbering.
#   tools/gpu_rcm_ctr.sh NEX
set -o pipefail
NE=${1:-256}
for nb in lex rcm; do
  TAG=rcm_$nb SETS="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAVES" \
    BENCH_ARGS="--nex $NE --ney $NE --numbering $nb --no-check" bash tools/gpu_counters.sh || exit 1
done
