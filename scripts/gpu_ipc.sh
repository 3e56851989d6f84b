#!/bin/bash
# peer_algo with buckets allocated once per process (no free + re-register), repeated.
set -u
O=gpurun_out/ipc5
mkdir -p $O
fails=0
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 120 tests/cpp/peer_algo 2 1000003 $(mktemp -d) > $O/algo_$i.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "run $i rc=$rc"; cat $O/algo_$i.log; fails=$((fails+1)); }
  case $rc in 124|134|137|139) exit 1;; esac
done
for i in 1 2 3 4; do
  timeout -k 10 120 tests/cpp/peer_algo 4 262147 $(mktemp -d) > $O/algo4_$i.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "P=4 run $i rc=$rc"; cat $O/algo4_$i.log; fails=$((fails+1)); }
  case $rc in 124|134|137|139) exit 1;; esac
done
echo "peer_algo failures: $fails/14"
