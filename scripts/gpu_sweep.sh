set -u
O=gpurun_out/sweep
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --sweep --steps 50 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 bench.py --sweep --steps 20 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
