"""HipAllreduceRing / HipAllreduceRingChunked over pointers on several GPUs of one process
(CudaAllreduceRing's shape, cuda_allreduce_ring.cc:34-42, 147-174): the per-pointer
device bookkeeping -- the local reduce tree / chain, which steps read a peer device and which
stage, the ring's pointer -- checked on the CPU (tests/cpp/local_steps.cc).  One GPU cannot run
the cross-device branches; every single-device case runs the same code on the GPU
(tests/test_gpu_host.py)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_local_reduce_bookkeeping(tmp_path):
    exe = tmp_path / "local_steps"
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    "-o", str(exe), os.path.join(ROOT, "tests", "cpp", "local_steps.cc")],
                   check=True, capture_output=True, text=True, timeout=120)
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0 and "local steps ok" in p.stdout, p.stderr
