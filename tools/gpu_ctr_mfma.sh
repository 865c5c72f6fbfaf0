set -o pipefail
cd $GRAFT_REPO_ROOT
S1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY"
S2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE TA_BUSY_avr"
S3="SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64"
for k in mfma column; do
  TAG=p12_$k SETS="$S1;$S2" KERNEL=k_poisson BENCH_ARGS="--p 12 --nex 263 --ney 263 --kernel $k --geometry stored" bash tools/gpu_counters.sh || exit 1
done
TAG=p12_mfma_f64 SETS="$S3" KERNEL=k_poisson BENCH_ARGS="--p 12 --nex 263 --ney 263 --kernel mfma" bash tools/gpu_counters.sh || echo "f64 mfma counters unavailable"
for d in gpurun_out/ctr_p12_*; do echo == $d; python tools/ctr_summary.py $d; done
