python tools/gpu_steps.py gpurun_out/r06d \
 "api_cost|120|tools/hip_api_cost" \
 "tr3_2d|240|python -u bench.py --gpus 8 --time-rank 3 --steps 200 --warmup 20" \
 "bench_hex|200|python -u bench.py --dim 3 --steps 20 --warmup 5 --no-cpu-baseline"
