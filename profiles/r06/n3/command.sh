python tools/gpu_steps.py gpurun_out/r06a \
 "hexmr|420|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_hex_multirank.py" \
 "seams|300|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_seams.py -k 'fence or hex_slab'" \
 "hexforms|300|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_hex.py -k 'kernel_forms or accumulate_diag'" \
 "bench_hex|240|python -u bench.py --dim 3 --steps 20 --warmup 5" \
 "hex_rehearse2|240|python -u bench.py --dim 3 --gpus 2 --rehearse-one-gpu --hex-ne 12 --steps 5 --warmup 2" \
 "hex_tr3_strong|240|python -u bench.py --dim 3 --gpus 8 --time-rank 3 --steps 200 --warmup 20" \
 "hex_tr3_weak|300|python -u bench.py --dim 3 --gpus 8 --time-rank 3 --scaling weak --steps 200 --warmup 20"
