python tools/gpu_steps.py gpurun_out/r06e \
 "hextests|600|python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_hex.py" \
 "hex_p8|200|python -u bench.py --dim 3 --steps 20 --warmup 5 --no-cpu-baseline" \
 "hex_p12|300|python -u bench.py --dim 3 --p 12 --hex-ne 17 --steps 20 --warmup 5 --no-cpu-baseline" \
 "hex_p14|300|python -u bench.py --dim 3 --p 14 --hex-ne 15 --steps 20 --warmup 5 --no-cpu-baseline" \
 "hex_p16|300|python -u bench.py --dim 3 --p 16 --hex-ne 13 --steps 20 --warmup 5 --no-cpu-baseline" \
 "hexmr|300|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_hex_multirank.py"
