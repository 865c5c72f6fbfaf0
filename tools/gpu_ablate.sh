set -o pipefail
cd $GRAFT_REPO_ROOT
for a in 0 1 2 3; do
  SEM_ABLATE=$a timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/abl_$a.json 2>/dev/null || exit 1
done
echo done
