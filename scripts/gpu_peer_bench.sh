set -u
O=gpurun_out/peerb4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_peer.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; exit 1; }
timeout -k 10 200 python -u scripts/peer_bench.py --P 2 --blocks 256 > $O/p2.log 2>&1 || { echo "p2 rc=$?"; exit 1; }
timeout -k 10 200 python -u scripts/peer_bench.py --P 4 --blocks 128 --n 65536 16777216 > $O/p4.log 2>&1 || { echo "p4 rc=$?"; exit 1; }
timeout -k 10 200 python -u scripts/peer_bench.py --P 8 --blocks 64 --n 65536 16777216 > $O/p8.log 2>&1 || { echo "p8 rc=$?"; exit 1; }
