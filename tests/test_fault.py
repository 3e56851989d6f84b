"""Process-per-rank fault tests of the host runtime's ring (the reference's
TransportMultiProcTest.IoErrors / IoTimeouts, gloo/gloo/test/transport_test.cc:44-152, on
MultiProcTest, gloo/gloo/test/multiproc_test.{h,cc}): P processes (tests/cpp/host_fault_ranks.cc)
loop gloo-style allreduces over a FileStore + loopback TCP mesh; rank 0 is then SIGKILLed or
SIGSTOPped.  Every other rank must leave with kExitWithIoException (10):
* after SIGKILL, within half the timeout (transport_test.cc:86-91): the dead peer's sockets
  close, the survivors' pending operations fail at once and the failure cascades along the
  ring as each survivor exits;
* after SIGSTOP, by the per-operation timeout (the stopped rank keeps its sockets open).
The library must not let SIGPIPE kill a survivor that writes to the dead rank (the binary keeps
SIGPIPE's default action)."""
import os
import signal
import subprocess
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = [os.path.join(ROOT, "tests", "cpp", "host_fault_ranks.cc"),
        os.path.join(ROOT, "hydra_amd", "csrc", "host", "transport.cpp"),
        os.path.join(ROOT, "hydra_amd", "csrc", "host", "allreduce.cpp"),
        os.path.join(ROOT, "hydra_amd", "csrc", "host", "reduce.cpp")]
K_EXIT_WITH_IO_EXCEPTION = 10  # gloo/gloo/test/multiproc_test.h:26


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = tmp_path_factory.mktemp("fault") / "host_fault_ranks"
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-pthread", "-I",
                           os.path.join(ROOT, "include"), *SRCS, "-o", str(out)])
    return str(out)


def _spawn(exe, tmp_path, P, n, timeout_ms, *extra):
    store = tmp_path / "store"
    store.mkdir()
    procs = [subprocess.Popen([exe, str(r), str(P), str(store), str(n), str(timeout_ms), *extra],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for r in range(P)]
    try:
        for p in procs:  # every rank finished one correct allreduce
            line = p.stdout.readline()
            assert line.strip() == "ready", (line, p.poll())
    except BaseException:
        for p in procs:
            p.kill()
            p.wait()
        raise
    return procs


def _finish(procs, deadline_s):
    """Wait for ranks 1.. (bounded); return their exit codes and stderr."""
    codes, errs = [], []
    for p in procs[1:]:
        try:
            p.wait(timeout=deadline_s)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
                q.wait()
            raise AssertionError("a surviving rank did not leave")
        codes.append(p.returncode)
        errs.append(p.stderr.read())
    return codes, errs


@pytest.mark.parametrize("P", [2, 3, 4])
@pytest.mark.parametrize("n", [1, 1000, 1 << 18])
@pytest.mark.parametrize("sleep_ms", [0, 50])
def test_io_errors_after_sigkill(exe, tmp_path, P, n, sleep_ms):
    timeout_ms = 2000
    procs = _spawn(exe, tmp_path, P, n, timeout_ms)
    time.sleep(sleep_ms / 1000)
    t0 = time.monotonic()
    procs[0].send_signal(signal.SIGKILL)
    codes, errs = _finish(procs, 30)
    dt = time.monotonic() - t0
    procs[0].wait()
    assert codes == [K_EXIT_WITH_IO_EXCEPTION] * (P - 1), (codes, errs)
    assert dt < timeout_ms / 2 / 1000, dt  # transport_test.cc:91
    assert all("IoException" in e for e in errs), errs


@pytest.mark.parametrize("P", [2, 3])
def test_io_timeouts_after_sigstop(exe, tmp_path, P):
    timeout_ms = 500  # kMultiProcTimeout, multiproc_test.h:27
    procs = _spawn(exe, tmp_path, P, 1000, timeout_ms)
    t0 = time.monotonic()
    procs[0].send_signal(signal.SIGSTOP)
    try:
        codes, errs = _finish(procs, 30)
        dt = time.monotonic() - t0
    finally:
        procs[0].send_signal(signal.SIGKILL)
        procs[0].wait()
    assert codes == [K_EXIT_WITH_IO_EXCEPTION] * (P - 1), (codes, errs)
    assert dt >= timeout_ms / 1000 * 0.9, dt
    assert any("Timed out" in e for e in errs), errs


def test_blocked_write_to_a_killed_rank_raises_not_sigpipe(exe, tmp_path):
    """Rank 1's writer is blocked inside a 256 MiB send that rank 0 never reads (far past the
    4 MiB socket buffers) when rank 0 is SIGKILLed: the write fails with EPIPE / ECONNRESET.
    With SIGPIPE at its default action (the binary does not ignore it) the library must report
    that as IoException (sendmsg + MSG_NOSIGNAL), not let the signal kill rank 1 (-13)."""
    procs = _spawn(exe, tmp_path, 2, 64 << 20, 20000, "bigsend")
    time.sleep(0.3)  # rank 1's writer fills the socket buffers and blocks
    assert procs[1].poll() is None
    procs[0].send_signal(signal.SIGKILL)
    codes, errs = _finish(procs, 30)
    procs[0].wait()
    assert codes == [K_EXIT_WITH_IO_EXCEPTION], (codes, errs)
    assert "Connection closed by peer 0" in errs[0], errs


GPU_EXE = os.path.join(ROOT, "tests", "cpp", "host_fault_ranks_gpu")


@pytest.mark.gpu
@pytest.mark.parametrize("P", [2, 3])
def test_io_errors_after_sigkill_gpu_reducer(tmp_path, P):
    """The same SIGKILL test with the drop-in GPU Func (gloo_compat::hostSum<float>, the gfx950
    chunk-sum) as the reducer and pinned receive slots, P processes sharing the GPU: every
    survivor still leaves with IoException (10) within half the timeout -- a rank blocked in the
    ring, with kernels, pinned memory and streams in use, is not wedged by a dead peer."""
    if not os.path.exists(GPU_EXE):
        pytest.fail(f"{GPU_EXE} missing: build() (hydra_amd/csrc/Makefile) makes it")
    timeout_ms = 4000
    procs = _spawn(GPU_EXE, tmp_path, P, 1 << 20, timeout_ms, "gpu")
    time.sleep(0.05)
    t0 = time.monotonic()
    procs[0].send_signal(signal.SIGKILL)
    codes, errs = _finish(procs, 60)
    dt = time.monotonic() - t0
    procs[0].wait()
    assert codes == [K_EXIT_WITH_IO_EXCEPTION] * (P - 1), (codes, errs)
    assert dt < timeout_ms / 2 / 1000, dt
