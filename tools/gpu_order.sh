set -o pipefail
cd $GRAFT_REPO_ROOT
for pass in 1 2; do
SEM_CHAIN_ROUNDS=1 timeout -k 10 120 python tools/order_ab.py 1 || exit 1
SEM_CHAIN_ROUNDS=2 timeout -k 10 120 python tools/order_ab.py 2 || exit 1
SEM_CHAIN_ROUNDS=4 timeout -k 10 120 python tools/order_ab.py 4 || exit 1
SEM_SERPENTINE=1 SEM_CHAIN_ROUNDS=1 timeout -k 10 120 python tools/order_ab.py 1 || exit 1
done
