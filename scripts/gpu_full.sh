set -u
O=gpurun_out/full1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest rc=$?" >> $O/pytest.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; exit 1; }
