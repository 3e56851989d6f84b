set -u
mkdir -p gpurun_out/wait
timeout -k 10 300 python -u -m pytest tests/test_gpu_xgmi.py -x -v -k "comm_wait or graph_replay" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/wait/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --force-dist --steps 10 --warmup 2 --elements 16777216 > gpurun_out/wait/forcedist.log 2>&1 || exit 1
