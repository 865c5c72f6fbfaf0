export TMPDIR=/tmp
mkdir -p gpurun_out/hex5
timeout -k 10 600 python -u -m pytest tests/test_gpu_hex.py -x -q --timeout 300 --timeout-method thread > gpurun_out/hex5/tests.log 2>&1 || { tail -30 gpurun_out/hex5/tests.log; exit 1; }
tail -1 gpurun_out/hex5/tests.log
for v in base hex_nog hex_nogather hex_nostore; do
  if [ $v = base ]; then L=""; else L="SEM_LIB_PATH=build_variants/$v/libsem_hip.so"; fi
  env $L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hex5/$v -o run -- python3 bench.py --dim 3 --no-cpu-baseline --no-check > gpurun_out/hex5/$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/hex5/$v.log; exit 1; }
done
echo ok
