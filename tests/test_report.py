"""benchkit.report: the reference benchmark's table (runner.cc:563-649, timer.h:68-102)."""
import numpy as np

from benchkit import report

# The header line of the reference's published tables (README.md:61, :98).
REF_HEADER = ("   elements   min (us)   p50 (us)   p99 (us)  p995 (us)   max (us)   avg (us)"
              "   avg (GB/s)    samples")


def test_header_matches_the_reference_tables():
    h = report.header("new_allreduce_ring", 2).splitlines()
    assert h[-1] == REF_HEADER
    assert h[1] == "Algorithm:   new_allreduce_ring"
    assert h[2] == "Options:     processes=2, inputs=1, threads=1"


def test_row_arithmetic():
    # 1000 samples 1..1000 us: percentile index = int(p * size) into the sorted samples,
    # microseconds by integer division, GiB/s from bytes x samples / summed ns
    s = (np.arange(1, 1001) * 1000).astype(np.int64)[::-1]  # unsorted on purpose
    r = report.row(67108864, 4, s)
    cols = r.split()
    assert cols[:7] == ["67108864", "1", "501", "991", "996", "1000", "500"]
    gib = 67108864 * 4 * 1000 / (s.sum() * 1e-9) / 2**30
    assert abs(float(cols[7]) - gib) < 1e-3 * gib
    assert cols[8] == "1000"
    assert len(r) == 11 * 7 + 13 + 11


def test_row_reproduces_a_published_bandwidth():
    # README.md:89: 67108864 fp32 elements, avg 325034 us over 1000 samples -> 0.769 "GB/s"
    s = np.full(1000, 325034 * 1000, dtype=np.int64)
    assert report.row(67108864, 4, s).split()[7] == "0.769"
