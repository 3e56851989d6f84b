"""C-ABI boundary checks that need no GPU: the library loads, exports exactly what
include/hydra_hip.h declares, validates arguments before touching HIP, and computes the ring
geometry of allreduce.cc:199-221 identically to the oracle."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from hydra_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(ROOT, "include", "hydra_hip.h")).read()
    return sorted(set(re.findall(r"\b(hydra_[a-z0-9_]+)\s*\(", txt)))


def test_header_symbols_exported():
    declared = header_functions()
    assert set(declared) == set(_lib.EXPORTS), set(declared) ^ set(_lib.EXPORTS)
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH], text=True)
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = [f for f in declared if f not in exported]
    assert not missing, missing
    L = _lib.lib()
    for f in declared:
        assert hasattr(L, f)
    assert L.hydra_abi_version() == 2


def test_measurement_symbols_only_in_the_measurement_build():
    """the product library exports no measurement entry point (the A/B
    variants and phase clocks are built into libhydra_measure.so only), and the measurement
    build exports the whole product ABI plus include/hydra_measure.h."""
    def exported(path):
        out = subprocess.check_output(["nm", "-D", "--defined-only", path], text=True)
        return {ln.split()[-1] for ln in out.splitlines() if " T " in ln}

    prod, meas = exported(_lib.LIB_PATH), exported(_lib.MEASURE_LIB_PATH)
    assert not [f for f in _lib.MEASURE_EXPORTS if f in prod]
    txt = open(os.path.join(ROOT, "include", "hydra_measure.h")).read()
    declared = set(re.findall(r"\b(hydra_[a-z0-9_]+)\s*\(", re.sub(r"/\*.*?\*/", "", txt, flags=re.S)))
    assert declared == set(_lib.MEASURE_EXPORTS)
    assert set(_lib.EXPORTS) | declared <= meas


def test_library_reads_no_environment():
    """every tunable is a documented option on the C-ABI (hydra_set_option
    / hydra_ctx_set_option), never an environment variable: no getenv in the library's sources,
    and getenv is not among the product library's undefined symbols."""
    csrc = os.path.join(ROOT, "hydra_amd", "csrc")
    hits = []
    for dp, _, fs in os.walk(csrc):
        if "build" in dp:
            continue
        for f in fs:
            if f.endswith((".cpp", ".h", ".hip")):
                if "getenv" in open(os.path.join(dp, f), errors="replace").read():
                    hits.append(f)
    assert not hits, hits
    und = subprocess.check_output(["nm", "-D", "--undefined-only", _lib.LIB_PATH], text=True)
    assert not [ln for ln in und.splitlines() if ln.split()[-1].startswith("getenv")]


def test_options_validate_and_round_trip():
    """hydra_set_option / hydra_get_option: defaults, range checks, unknown keys; per-context
    keys only through hydra_ctx_set_option (its null-context check needs no GPU)."""
    L = _lib.lib()
    assert _lib.get_option(_lib.OPT_STAGE_SPLIT) == 4
    assert _lib.get_option(_lib.OPT_RESIDENT_IDLE_US) == 2000
    assert L.hydra_set_option(99, 1) == _lib.ERR_INVALID
    assert L.hydra_set_option(_lib.OPT_STAGE_SPLIT, 0) == _lib.ERR_INVALID  # 1..64
    assert b"outside" in L.hydra_last_error()
    _lib.set_option(_lib.OPT_STAGE_SPLIT, 8)
    try:
        assert _lib.get_option(_lib.OPT_STAGE_SPLIT) == 8
    finally:
        _lib.set_option(_lib.OPT_STAGE_SPLIT, 4)
    assert L.hydra_ctx_set_option(None, _lib.OPT_STAGE_SPLIT, 2) == _lib.ERR_INVALID


def test_no_hip_types_in_abi():
    """Plain C at the boundary: no HIP/torch headers or types outside comments."""
    txt = open(os.path.join(ROOT, "include", "hydra_hip.h")).read()
    code = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    assert not re.search(r"#include\s*<(hip|torch|c10|ATen)", code)
    assert not re.search(r"\bhip[A-Z]\w*", code)


@pytest.mark.parametrize("op,dtype,rc", [(9, 6, 1), (0, 42, 1), (-1, 6, 1)])
def test_invalid_args_rejected_before_hip(op, dtype, rc):
    L = _lib.lib()
    a = np.zeros(8, np.float32)
    assert L.hydra_reduce(op, dtype, a.ctypes.data, a.ctypes.data, a.ctypes.data, 8, None) == rc
    assert L.hydra_last_error()


def test_alignment_and_overlap_rejected():
    L = _lib.lib()
    buf = np.zeros(64, np.float32)
    p = buf.ctypes.data
    assert L.hydra_reduce(0, 6, p + 2, p + 2, p + 2, 4, None) == 1  # not 4-B aligned
    assert b"aligned" in L.hydra_last_error()
    assert L.hydra_reduce(0, 6, p + 4, p, p + 128, 8, None) == 1    # c partially overlaps a
    assert b"overlap" in L.hydra_last_error()
    assert L.hydra_reduce(0, 6, p, p, p, 0, None) == 0               # n == 0: no-op, no HIP


@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 7, 8, 16])
def test_ring_plan_matches_oracle(O, P):
    rng = np.random.default_rng(P)
    for n in list(rng.integers(1, 1 << 27, 40)) + [1, 2, 3, 100, 262144, 1 << 26, (1 << 28) + 3]:
        for es in (1, 2, 4, 8):
            for ms in (128, 1000, 1 << 20):
                assert _lib.ring_plan(P, int(n), es, ms) == O.ring_plan(P, int(n), es, ms)


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    """No silent fallback: a missing .so raises HydraError."""
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.HydraError):
        _lib.lib()


def test_split_elements_shared_with_host_runtime():
    """The device library's split (hydra_split_elements) and the host runtime's
    calculateElements are the same table (split_table.h), incl. the band edges."""
    from hydra_amd import host, ring

    for table in (0, 1):
        for P in (2, 3, 4, 5, 6, 8):
            for n in (0, 1, 6144, 6145, 65535, 65536, 65537, 131072, 524288, 524289, 828344,
                      1048577, 1500000, 2097152, 4000001, 16777217, 67108864, 67108865):
                assert ring.split_elements(table, P, n) == host.calculate_elements(table, P, n)


def test_split_elements_vs_reference_fixture(golden_split):
    """hydra_split_elements (split_table.h, the device rail split) and the host runtime's
    calculateElements equal the reference's own compiled calculateElements_AA / _AG
    (pipeallreduce-a.h:137-376; tests/golden/golden_split.json) on every fixture row."""
    from hydra_amd import host, ring

    bad = []
    for table, P, n, e1, e2 in golden_split:
        if ring.split_elements(table, P, n) != (e1, e2):
            bad.append(("device", table, P, n))
        if host.calculate_elements(table, P, n) != (e1, e2):
            bad.append(("host", table, P, n))
    assert not bad, bad[:5]


def test_peer_args_rejected_before_hip():
    """hydra_peer_*: bad arguments fail with HYDRA_ERR_INVALID before any HIP call (no GPU)."""
    import ctypes

    L = _lib.lib()
    h = ctypes.c_void_p()
    sig = ctypes.create_string_buffer(_lib.PEER_HANDLE_BYTES)
    assert L.hydra_peer_create(9, 0, 0, ctypes.byref(h), sig) == 1  # > 8 ranks
    assert L.hydra_peer_create(2, 2, 0, ctypes.byref(h), sig) == 1  # rank out of range
    assert L.hydra_peer_create(2, 0, 0, None, sig) == 1
    assert L.hydra_peer_allreduce(None, 1, 0, _lib.FLOAT32, 0, None, 4, 0, None) == 1
    assert L.hydra_peer_connect(None, sig) == 1
    assert L.hydra_peer_set_option(None, 1, 5) == 1
    assert L.hydra_peer_destroy(None) == 0


def test_examples_and_headers_compile(tmp_path):
    """The INTEGRATION.md examples build against the shipped headers and libraries: the Gloo
    shim example links and runs (no GPU here: it reports that and exits 0), and every C++
    header a Gloo-side caller includes compiles on its own."""
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    inc = os.path.join(root, "include")
    lib = os.path.join(root, "hydra_amd")
    exe = str(tmp_path / "gloo_shim_example")
    subprocess.check_call(["g++", "-std=c++14", "-I" + inc,
                           os.path.join(root, "examples", "gloo_shim_example.cc"), "-o", exe,
                           "-L" + lib, "-lhydra_hip", "-Wl,-rpath," + lib])
    r = subprocess.run([exe], capture_output=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    for h in ("hydra_hip.h", "hydra_host.h", "hydra/allreduce.h", "hydra/gloo_reduce.h",
              "hydra/hip_allreduce_ring.h", "hydra/peer_allreduce.h"):
        src = tmp_path / "h.cc"
        src.write_text(f'#include "{h}"\nint main() {{ return 0; }}\n')
        subprocess.check_call(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-I" + inc,
                               str(src)])


def test_fault_lookup_names_the_mapping():
    """hydra_fault_lookup (the body of the GPU-fault report) without a GPU: a host
    array's address is inside a /proc/self/maps mapping, the zero page is not, and hydra's ledger
    holds no range for either."""
    from hydra_amd import _lib

    x = np.zeros(1 << 16, np.float32)
    r = _lib.fault_lookup(x.ctypes.data)
    assert "mapped by:" in r and "no block, registration or per-call pin" in r, r
    r0 = _lib.fault_lookup(8)
    assert "not mapped" in r0, r0


def test_struct_layouts_match_the_header():
    """The ctypes mirrors of the round-4 measurement structs match include/hydra_hip.h (sizes
    computed by the C compiler from the header itself)."""
    import subprocess
    import tempfile

    src = ('#include <stdio.h>\n#include "hydra_hip.h"\n#include <stddef.h>\nint main(void){'
           'printf("%zu %zu %zu %zu\\n", sizeof(hydra_host_call_t), sizeof(hydra_comm_phases_t),'
           ' offsetof(hydra_host_call_t, total_us), offsetof(hydra_comm_phases_t, peers));'
           'return 0;}\n')
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "s.c")
        with open(c, "w") as f:
            f.write(src)
        subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), "-o",
                        os.path.join(d, "s"), c], check=True, capture_output=True)
        got = [int(v) for v in subprocess.run([os.path.join(d, "s")], check=True,
                                              capture_output=True, text=True).stdout.split()]
    assert got == [ctypes.sizeof(_lib.HostCall), ctypes.sizeof(_lib.CommPhases),
                   _lib.HostCall.total_us.offset, _lib.CommPhases.peers.offset], got
