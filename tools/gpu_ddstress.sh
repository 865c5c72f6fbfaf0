set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/dd_stress.py base 2>&1 | grep check=
