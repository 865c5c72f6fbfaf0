#!/bin/bash
# Block-layout rounds per chain (SEM_BLOCK_ROUNDS) on the driver command,
# alternating:   tools/gpu_block_rounds.sh OUT R...
set -o pipefail
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
for k in 1 2; do
  for R in "$@"; do
    SEM_BLOCK_ROUNDS=$R timeout -k 10 300 python bench.py --no-cpu-baseline > $O/R${R}_r$k.json 2> $O/R${R}_r$k.err || { echo "R=$R failed"; tail -5 $O/R${R}_r$k.err; exit 1; }
    python3 -c "
import json; r = json.load(open('$O/R${R}_r$k.json')); c = r['config']; s = c['scatter_plan']
ch = sum(s['chains_per_colour'])
print('R=%s r$k chains %5d gens %.2f seams %d ms/step %.4f kernel %.4f q50 %.4f frac %.3f parity %.1e' % ('$R', ch, ch / 1024.0, s['seam_nodes'], r['ms_per_step'], c['kernel_ms_avg'], c['kernel_ms_quartiles'][1], r['roofline']['frac'], r['parity']['rel_l2']))"
  done
done
