set -u
O=gpurun_out/quick
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d $O/mt -o run -- python3 bench.py --force-dist --steps 5 --warmup 1 --elements 4194304 --no-config5 > $O/mt.log 2>&1 || { echo "mt rc=$?"; exit 1; }
