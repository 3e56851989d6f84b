#!/bin/bash
# rocprofv3 kernel trace + separate FETCH_SIZE / WRITE_SIZE passes of the P-way fold kernel.
set -u
O=$PWD/gpurun_out/${1:-fold_pmc}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 scripts/fold_pmc.py > $O/kt.log 2>&1 || { echo "kt rc=$?"; tail $O/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 scripts/fold_pmc.py > $O/fetch.log 2>&1 || { echo "fetch rc=$?"; tail $O/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 scripts/fold_pmc.py > $O/write.log 2>&1 || { echo "write rc=$?"; tail $O/write.log; exit 1; }
find $O -name "*.csv" | head -20
