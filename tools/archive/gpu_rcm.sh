#!/bin/bash
# Reference default (RCM) node numbering vs lexicographic on one GPU:
#   tools/gpu_rcm.sh OUT
# cfg2 action + PCG (solver numbering auto / off) and the cfg3-size mesh.
set -o pipefail
export TMPDIR=/tmp
O=$1; mkdir -p $O
run() {  # name, args...
  local nm=$1; shift
  timeout -k 10 900 python -u bench.py --no-cpu-baseline "$@" > $O/$nm.json 2> $O/$nm.err || { echo "$nm failed"; tail -5 $O/$nm.err; return 1; }
  python3 -c "
import json; r = json.load(open('$O/$nm.json')); c = r['config']
x = r.get('pcg') or {}
print('%-22s ms/step %.4f' % ('$nm', r['ms_per_step']), 'kernel %.4f frac %.3f' % (c['kernel_ms_avg'], r['roofline']['frac']) if 'roofline' in r else 'its %s relres %.2e err %.2e %s' % (x.get('iterations'), x.get('final_relres', 0), x.get('rel_l2_error_vs_manufactured', 0), x.get('solver_numbering')), r.get('parity', ''))
"
}
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -k "rcm" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for nb in lex rcm; do run action_${nb}_256 --nex 256 --ney 256 --numbering $nb || exit 1; done
run pcg_lex_256 --op pcg --nex 256 --ney 256 --steps 300 --warmup 20 || exit 1
run pcg_rcm_256 --op pcg --nex 256 --ney 256 --steps 300 --warmup 20 --numbering rcm || exit 1
run pcg_rcm_off_256 --op pcg --nex 256 --ney 256 --steps 300 --warmup 20 --numbering rcm --renumber off || exit 1
run solve_lex_256 --op pcg --nex 256 --ney 256 --pcg-rtol 1e-10 || exit 1
run solve_rcm_256 --op pcg --nex 256 --ney 256 --pcg-rtol 1e-10 --numbering rcm || exit 1
for nb in lex rcm; do run action_${nb}_1024 --nex 1024 --ney 1024 --numbering $nb || exit 1; done
