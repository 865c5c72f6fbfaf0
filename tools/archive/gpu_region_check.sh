set -o pipefail
O=gpurun_out/region_check; mkdir -p $O
for k in 1 2; do timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$k.json 2> $O/bench_$k.err || exit 1; python3 -c "import json; r=json.load(open('$O/bench_$k.json')); print('default', r['value'], r['ms_per_step'], r['config']['kernel_ms_avg'], r['config']['kernel_ms_quartiles'], r['roofline']['frac'], r['parity']['rel_l2'], r['config']['step_events'])"; done
timeout -k 10 300 python bench.py --dim 3 --no-cpu-baseline > $O/hex.json 2> $O/hex.err || exit 1
python3 -c "import json; r=json.load(open('$O/hex.json')); print('hex', r['ms_per_step'], r['config']['kernel_ms_avg'], r['config']['kernel_ms_quartiles'], r['roofline']['frac'], r['parity']['rel_l2'])"
timeout -k 10 300 python bench.py --gpus 8 --time-rank 3 --steps 200 --warmup 20 > $O/tr3.json 2> $O/tr3.err || exit 1
python3 -c "import json; r=json.load(open('$O/tr3.json')); s=r['single_gpu_whole_mesh']['wall_ms_per_step']; print('tr3', r['step']['wall_ms_per_step'], s, s/r['step']['wall_ms_per_step'], r.get('projected_speedup'))"
