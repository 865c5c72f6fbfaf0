#!/bin/bash
# Round 3, call L: calibrate FETCH_SIZE / WRITE_SIZE per access width on
# gfx950 (tools/r03/pmc_calib.cpp), one counter per rocprofv3 pass.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03l
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/calib_$c -o run -- ./tools/r03/pmc_calib.bin > $O/calib_$c.log 2>&1; rc=$?
  echo "calib $c rc=$rc"; fatal $rc calib
  python - "$O/calib_$c" "$c" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if r["Counter_Name"] == sys.argv[2]:
        print("%-60s %s %.4e bytes" % (r["Kernel_Name"][:60], sys.argv[2], float(r["Counter_Value"]) * 1024))
PY
done
