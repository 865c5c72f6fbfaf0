# Extra PMC passes (one rocprofv3 run per counter set) on the element kernel.
#   TAG=name SETS="A B;C D" KERNEL=regex BENCH_ARGS="..." bash tools/gpu_counters.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ctr_${TAG:-x}
mkdir -p $OUT
DEFAULT_SETS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR;TCC_HIT_sum TCC_MISS_sum;TCC_EA0_RDREQ_DRAM_sum;TCC_EA0_WRREQ_DRAM_sum;TCC_EA0_RDREQ_32B_sum;TCC_EA0_RDREQ_sum;TCC_EA0_WRREQ_64B_sum;TCC_EA0_WRREQ_sum;TA_BUSY_avr;GRBM_GUI_ACTIVE"
IFS=';' read -ra SETLIST <<< "${SETS:-$DEFAULT_SETS}"
i=0
for set in "${SETLIST[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex ${KERNEL:-k_poisson_apply} --output-format csv -d $OUT/p$i -o run -- python bench.py --no-cpu-baseline --steps 4 --warmup 1 ${BENCH_ARGS} > $OUT/p$i.log 2>&1 || { echo "pass $i ($set) failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo done
