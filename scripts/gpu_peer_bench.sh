set -u
O=gpurun_out/peerb6
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_peer.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 scripts/peer_bench.py --P 2 --blocks 256 --n 16777216 > $O/prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
