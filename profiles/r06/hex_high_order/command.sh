python tools/gpu_steps.py gpurun_out/r06h \
 "diag|300|python -u tools/hex_geom_diag.py 12 14 16" \
 "hextests|600|python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_hex.py" \
 "scale2d|900|python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_const_d.py" \
 "hex_p12|300|python -u bench.py --dim 3 --p 12 --hex-ne 17 --steps 20 --warmup 5 --no-cpu-baseline" \
 "hex_p14|300|python -u bench.py --dim 3 --p 14 --hex-ne 15 --steps 20 --warmup 5 --no-cpu-baseline" \
 "hex_p16|300|python -u bench.py --dim 3 --p 16 --hex-ne 13 --steps 20 --warmup 5 --no-cpu-baseline"
