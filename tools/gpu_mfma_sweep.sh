set -o pipefail
TESTK=all_orders_mfma CFGS="12 263 263;9 351 351;10 316 316;11 287 287;13 243 243;14 226 226;15 211 211;8 1024 1024" VARIANTS="${VARIANTS:-column base mw6 mw7}" bash tools/gpu_mfma_ab.sh
