"""Host-runtime race and memory checks (the reference's SANITIZE=thread CI job,
gloo/CMakeLists.txt:66-71, .circleci/config.yml:117-121): tests/cpp/host_ring_sanitize.cc
built against hydra_amd/csrc/host/{transport,allreduce,reduce}.cpp with ThreadSanitizer and with
AddressSanitizer + UBSan, run on loopback TCP thread-ranks."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = [os.path.join(ROOT, "tests", "cpp", "host_ring_sanitize.cc"),
        os.path.join(ROOT, "hydra_amd", "csrc", "host", "transport.cpp"),
        os.path.join(ROOT, "hydra_amd", "csrc", "host", "allreduce.cpp"),
        os.path.join(ROOT, "hydra_amd", "csrc", "host", "reduce.cpp")]


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_host_runtime_sanitized(tmp_path, san):
    exe = tmp_path / f"host_ring_{san.split(',')[0]}"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-pthread", f"-fsanitize={san}",
           "-fno-omit-frame-pointer", "-I", os.path.join(ROOT, "include"), *SRCS, "-o", str(exe)]
    subprocess.check_call(cmd)
    # the environment is passed through unchanged; an inherited preload list is tolerated
    # (verify_asan_link_order=0) rather than edited
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0 and "OK" in p.stdout, (p.stdout[-2000:], p.stderr[-4000:])
    assert "ThreadSanitizer" not in p.stderr and "AddressSanitizer" not in p.stderr
    assert "runtime error" not in p.stderr


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_copy_pool_sanitized(tmp_path, san):
    """The staging copy fan-out (hydra_amd/csrc/copy_pool.cpp): concurrent callers sharing the
    helper threads, every byte and the guard bytes checked, under TSan and ASan + UBSan."""
    exe = tmp_path / f"copy_pool_{san.split(',')[0]}"
    srcs = [os.path.join(ROOT, "tests", "cpp", "copy_pool_stress.cc"),
            os.path.join(ROOT, "hydra_amd", "csrc", "copy_pool.cpp"),
            os.path.join(ROOT, "hydra_amd", "csrc", "options.cpp")]
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-pthread", f"-fsanitize={san}",
                           "-fno-omit-frame-pointer", *srcs, "-o", str(exe)])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1",
               ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0 and "OK" in p.stdout, (p.stdout[-2000:], p.stderr[-4000:])
    assert "ThreadSanitizer" not in p.stderr and "AddressSanitizer" not in p.stderr
    assert "runtime error" not in p.stderr
