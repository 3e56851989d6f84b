set -u
O=gpurun_out/stress2
mkdir -p $O
timeout -k 10 500 python -u scripts/peer_stress.py --P 4 --iters 1500 > $O/p4.log 2>&1 || { echo "p4 rc=$?"; exit 1; }
timeout -k 10 500 python -u scripts/peer_stress.py --P 8 --iters 800 --blocks 32 > $O/p8.log 2>&1 || { echo "p8 rc=$?"; exit 1; }
timeout -k 10 500 python -u scripts/peer_stress.py --P 2 --iters 1500 --n 4000037 --blocks 256 > $O/p2.log 2>&1 || { echo "p2 rc=$?"; exit 1; }
