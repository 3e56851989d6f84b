set -u
O=gpurun_out/peerb5
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_peer.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; exit 1; }
timeout -k 10 300 python -u bench.py --force-dist --steps 10 --warmup 2 --elements 16777216 > $O/forcedist.log 2>&1 || { echo "forcedist rc=$?"; exit 1; }
