#!/bin/bash
# Reference default (RCM) node numbering vs lexicographic, one GPU:  tools/gpu_rcm.sh OUT NEX [extra]
export TMPDIR=/tmp
O=$1; NE=$2; shift 2
mkdir -p $O
for nb in lex rcm; do
  timeout -k 10 900 python -u bench.py --nex $NE --ney $NE --numbering $nb --no-cpu-baseline "$@" > $O/bench_${nb}_$NE.json 2> $O/bench_${nb}_$NE.err || { echo "$nb failed"; tail -5 $O/bench_${nb}_$NE.err; exit 1; }
  python3 -c "
import json; r = json.load(open('$O/bench_${nb}_$NE.json'))
c = r['config']; print('$nb', '$NE', 'ms/step %.4f' % r['ms_per_step'], 'kernel %.4f' % c['kernel_ms_avg'], 'frac %.3f' % r['roofline']['frac'], c['scatter_plan'], 'map bytes', c['map_entry_bytes'], r.get('parity'))
"
done
