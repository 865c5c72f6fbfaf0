# nodal vs stored geometry (column kernel) at ~1e7 DOF for p = 2..8, and the
# column kernel vs MFMA at p = 12..15 (stored) -- the AUTO choices
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/geosweep
mkdir -p $OUT
for cfg in "2 1581" "3 1054" "4 790" "5 632" "6 527" "7 452" "8 395"; do
  set -- $cfg
  for g in nodal stored; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --p $1 --nex $2 --ney $2 --steps 30 --geometry $g --kernel column > $OUT/p$1_$g.json 2> $OUT/p$1_$g.err || { echo "p$1 $g failed"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/p$1_$g.json')); print('p$1 $g', round(d['config']['kernel_ms_avg'],4), '%.3g' % d['value'])"
  done
done
for cfg in "12 263" "13 243" "14 225" "15 211" "16 198"; do
  set -- $cfg
  for k in column mfma; do
    [ $1 = 16 ] && [ $k = mfma ] && continue
    timeout -k 10 120 python bench.py --no-cpu-baseline --p $1 --nex $2 --ney $2 --steps 30 --geometry stored --kernel $k > $OUT/p$1_$k.json 2> $OUT/p$1_$k.err || { echo "p$1 $k failed"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/p$1_$k.json')); print('p$1 $k', round(d['config']['kernel_ms_avg'],4), '%.3g' % d['value'])"
  done
done
