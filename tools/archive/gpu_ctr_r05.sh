#!/bin/bash
# Round-5 counter passes: 2-D p = 8 / 14 / 16 and the hex row form against the
# three-block kernel at p = 4 / 8.   bash tools/gpu_ctr_r05.sh
bash tools/gpu_ctr.sh gpurun_out/ctr/p16 k_poisson_apply -- --p 16 --nex 198 --ney 198 && \
bash tools/gpu_ctr.sh gpurun_out/ctr/p14 k_poisson_apply -- --p 14 --nex 227 --ney 227 && \
bash tools/gpu_ctr.sh gpurun_out/ctr/p8 k_poisson_apply -- --p 8 --nex 395 --ney 395 && \
bash tools/gpu_ctr.sh gpurun_out/ctr/hex4_rows "k_hex_(rows|poisson)" SEM_HEX_ROWS=1 -- --dim 3 --p 4 --hex-ne 54 && \
bash tools/gpu_ctr.sh gpurun_out/ctr/hex4_old "k_hex_(rows|poisson)" SEM_HEX_ROWS=0 -- --dim 3 --p 4 --hex-ne 54 && \
bash tools/gpu_ctr.sh gpurun_out/ctr/hex8_rows "k_hex_(rows|poisson)" SEM_HEX_ROWS=1 -- --dim 3 --p 8 && \
bash tools/gpu_ctr.sh gpurun_out/ctr/hex8_old "k_hex_(rows|poisson)" SEM_HEX_ROWS=0 -- --dim 3 --p 8
