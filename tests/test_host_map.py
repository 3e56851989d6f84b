"""CPU checks of the host-mapping rules (hydra_amd/csrc/host_map.h): hydra never registers a page
that holds memory outside the operand it was given.

hydra_page_interior is the one place the pages of a registration are chosen (hydra_host_register
and the per-call pins of hydra_reduce_host both register exactly its result); it is pure
arithmetic, so it runs without a GPU.  The GPU side (tests/test_gpu_host_map.py) checks that the
live registrations are those pages."""
import os

import pytest
from hypothesis import given, settings, strategies as st

from hydra_amd import _lib

PAGE = os.sysconf("SC_PAGESIZE")


def _lib_or_skip():
    try:
        return _lib.lib()
    except (_lib.HydraError, OSError) as e:
        pytest.skip(f"libhydra_hip.so not loadable here: {e}")


@settings(max_examples=3000, deadline=None)
@given(st.integers(min_value=1, max_value=1 << 47), st.integers(min_value=0, max_value=1 << 30))
def test_registration_never_leaves_the_operand_pages(ptr, nbytes):
    """For every operand [ptr, ptr + nbytes): the registered range is whole pages, lies inside
    the operand (so no page of it holds a neighbour's bytes), and is the largest such range (every
    page of the operand not registered is a ragged edge page, staged instead)."""
    _lib_or_skip()
    lo, hi = _lib.page_interior(ptr, nbytes)
    end = ptr + nbytes
    if lo == hi:
        # nothing to register: no whole page fits inside
        first = -(-ptr // PAGE) * PAGE
        assert first + PAGE > end
        return
    assert lo % PAGE == 0 and hi % PAGE == 0
    assert ptr <= lo < hi <= end
    assert lo - ptr < PAGE and end - hi < PAGE  # maximal: only the ragged edges are left out


@pytest.mark.parametrize("ptr,nbytes,exp", [
    (0x10000, 0x3000, (0x10000, 0x13000)),  # page-aligned: all of it
    (0x10064, 0x3000, (0x11000, 0x13000)),  # misaligned start: the first page is an edge
    (0x10000, 0x2fff, (0x10000, 0x12000)),  # ragged end
    (0x10001, 0xffe, (0, 0)),               # inside one page: nothing
    (0x10fff, 0x1002, (0x11000, 0x12000)),  # one whole page between two edges
    (0x10000, 0, (0, 0)),
])
def test_page_interior_cases(ptr, nbytes, exp):
    _lib_or_skip()
    if PAGE != 4096:
        pytest.skip("cases written for 4 KiB pages")
    assert _lib.page_interior(ptr, nbytes) == exp
