#!/bin/bash
# Round 3, call C: full GPU suite on the seams-on-blocks AUTO, PCG after the
# vector-kernel rework, p-sweep / cfg2 / cfg5 block layout vs round-2 plans.
set -u
cd "$(dirname "$0")/../.."
O=gpurun_out/r03c
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 170 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest.log
fatal $rc pytest
timeout -k 10 300 python bench.py --op pcg --steps 100 --warmup 5 > $O/pcg.json 2> $O/pcg.log; rc=$?
echo "pcg rc=$rc $(python -c "import json;d=json.load(open('$O/pcg.json'));print(d['ms_per_step'], d['pcg'])" 2>/dev/null)"
fatal $rc pcg
run() {  # tag, env, args
  tag=$1; shift; envs=$1; shift
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --warmup 5 "$@" > $O/$tag.json 2> $O/$tag.log; rc=$?
  echo "$tag rc=$rc $(python -c "import json;d=json.load(open('$O/$tag.json'));c=d['config'];print(round(d['ms_per_step'],4), round(c['kernel_ms_avg'],4), [round(x,4) for x in c['kernel_ms_quartiles']], c['scatter_plan']['plan'], c['geometry'], round(d['roofline']['frac'],3), d.get('parity',{}).get('rel_l2'))" 2>/dev/null)"
  fatal $rc $tag
}
for cfg in "2 1581" "4 790" "6 527" "8 395" "12 263" "16 198"; do
  set -- $cfg
  run p$1_r02plan SEM_BLOCK_ROUNDS=0 --p $1 --nex $2 --ney $2 --steps 50
  run p$1_blocks SEM_X=1 --p $1 --nex $2 --ney $2 --steps 50
done
run cfg2_r02plan SEM_BLOCK_ROUNDS=0 --nex 256 --ney 256 --steps 100
run cfg2_blocks SEM_X=1 --nex 256 --ney 256 --steps 100
run cfg5_r02plan SEM_BLOCK_ROUNDS=0 --op axisym_stokes --p 6 --nex 512 --ney 512 --steps 50
run cfg5_blocks SEM_X=1 --op axisym_stokes --p 6 --nex 512 --ney 512 --steps 50
run cfg5_blocks_colours SEM_SEAM=0 --op axisym_stokes --p 6 --nex 512 --ney 512 --steps 50
run cfg5_blocks_seams SEM_SEAM=1 --op axisym_stokes --p 6 --nex 512 --ney 512 --steps 50
