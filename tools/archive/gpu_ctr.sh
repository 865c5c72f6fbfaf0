#!/bin/bash
# SQ counters of one kernel (three passes, one counter set each), averaged
# per dispatch:   tools/gpu_ctr.sh OUT KERNEL_REGEX [env ...] -- bench args...
set -o pipefail
export TMPDIR=/tmp
O=$1; K=$2; shift 2
E=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do E+=("$1"); shift; done
shift
mkdir -p $O
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
           "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  env "${E[@]}" timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "$K" --output-format csv -d $O/p$i -o run -- python3 bench.py --no-cpu-baseline --no-check --steps 4 --warmup 1 "$@" > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 tools/ctr_summary.py $O > $O/summary.txt
python3 - $O/summary.txt <<'PY'
import sys
v = {l.split()[0]: float(l.split()[1]) for l in open(sys.argv[1]) if l.strip()}
wc = v["SQ_WAVE_CYCLES"]
print("waves %d  wait_any %.1f %%  issuing %.1f %%  valu/wave-cycle %.1f %%  lds bank-conflict/lds-active %.1f %%" % (
    v["SQ_WAVES"], 100 * v["SQ_WAIT_ANY"] / wc, 100 * v["SQ_ACTIVE_INST_ANY"] / wc,
    100 * v["SQ_ACTIVE_INST_VALU"] / wc, 100 * v["SQ_LDS_BANK_CONFLICT"] / max(1, v["SQ_LDS_IDX_ACTIVE"])))
PY
