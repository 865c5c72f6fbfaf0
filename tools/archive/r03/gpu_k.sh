#!/bin/bash
# Round 3, call K: DPP wave_shl:1 for the in-group merge (SEM_DPP_SHIFT) and
# the second per-round barrier only where a chain revisits a node
# (round_sync): main = both, sync = DPP with the barrier always, old =
# neither (build_variants/); parity tests, then cfg3 and cfg5 alternating.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03k
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
line() { python -c "import json;d=json.load(open('$1'));c=d['config'];r=d['roofline'];print(round(d['ms_per_step'],4), round(c['kernel_ms_avg'],4), [round(x,4) for x in c['kernel_ms_quartiles']], round(r['frac'],3), d.get('parity',{}).get('rel_l2'))" 2>/dev/null; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_blocks.py tests/test_gpu_seams.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
fatal $rc pytest
[ $rc = 0 ] || exit 1
for rep in 1 2 3; do
  for v in main sync old; do
    if [ $v = main ]; then unset SEM_LIB_PATH; else export SEM_LIB_PATH=$PWD/build_variants/libsem_$v.so; fi
    timeout -k 10 180 python bench.py --no-cpu-baseline > $O/cfg3_${v}_$rep.json 2> $O/cfg3_${v}_$rep.log; rc=$?
    echo "cfg3 $v $rep rc=$rc $(line $O/cfg3_${v}_$rep.json)"
    fatal $rc cfg3
    timeout -k 10 180 python bench.py --no-cpu-baseline --op axisym_stokes --p 6 --nex 512 --ney 512 > $O/cfg5_${v}_$rep.json 2> $O/cfg5_${v}_$rep.log; rc=$?
    echo "cfg5 $v $rep rc=$rc $(line $O/cfg5_${v}_$rep.json)"
    fatal $rc cfg5
  done
done
