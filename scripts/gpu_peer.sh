set -u
mkdir -p gpurun_out/peer1
timeout -k 10 600 python -u -m pytest tests/test_gpu_peer.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/peer1/pytest.log 2>&1
echo "rc=$?" >> gpurun_out/peer1/pytest.log
