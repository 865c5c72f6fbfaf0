# Resource usage of one kernel instantiation for a set of -D flags:
#   bash tools/kres.sh 'k_poisson_applyILi9ELb1' -DSEM_X=1 ...
K=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics --cuda-device-only \
  -c "$(dirname "$0")/../spectralelementmethod_amd/csrc/sem_device.hip" -o /tmp/kres_$$.o "$@" \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "error|$K" -A12 |
  grep -E "VGPRs:|Scratch|Occupancy|VGPRs Spill|error|LDS S" | sed 's/.*remark: *//;s/ \[-R.*//' | tr '\n' ' '
echo " <= $*"
rm -f /tmp/kres_$$.o
