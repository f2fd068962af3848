"""the bench line's committed counters (profiles/pmc_traffic.json: HBM traffic and
VALU counts per config) are tied to the machine code they were measured on.  tools/traffic_update.py
and valu_update.py record sha256 of the measured kernels' code (jeromq_amd.build.kernel_code_sha256);
bench.py recomputes it from the loaded library and marks traffic / valu stale when it differs."""
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "jeromq_amd", "libcurvezmq_mi355x.so")
pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")


def test_kernel_code_sha_is_per_kernel_and_deterministic():
    from jeromq_amd.build import kernel_code_sha256
    a = kernel_code_sha256(LIB, ["k_seal_uniform<1, true, 0>"])
    assert a and a == kernel_code_sha256(LIB, ["k_seal_uniform<1, true, 0>"])
    assert a != kernel_code_sha256(LIB, ["k_open_uniform<1, true, 16>"])
    assert kernel_code_sha256(LIB, ["k_seal_combine", "k_seal_segments"]) == \
        kernel_code_sha256(LIB, ["k_seal_segments", "k_seal_combine"])       # order-free
    assert kernel_code_sha256(LIB, ["no_such_kernel"]) is None


def test_bench_marks_counters_of_other_code_stale():
    import bench
    from jeromq_amd.build import kernel_code_sha256
    fresh = kernel_code_sha256(LIB, ["k_seal_uniform<1, true, 0>"])
    entry = {"kernels": ["k_seal_uniform<1, true, 0>"], "hbm_bytes_per_launch": 1,
             "traffic_kernel_sha256": fresh, "valu_kernel_sha256": "0" * 64}
    f = bench.pmc_freshness(entry, LIB)
    assert f["traffic_stale"] is False and f["valu_stale"] is True
    assert f["traffic_kernel_sha256_loaded"] == fresh
    assert bench.pmc_freshness({"kernels": ["k_seal_uniform<1, true, 0>"]}, LIB)["traffic_stale"] is None
    assert bench.pmc_freshness({}, LIB) == {"traffic_stale": None, "traffic_kernel_sha256_loaded": None,
                                            "valu_stale": None, "valu_kernel_sha256_loaded": None}


def test_committed_headline_counters_match_the_shipped_kernel():
    """the headline's counters in profiles/pmc_traffic.json were measured on the shipped k_seal_uniform"""
    import bench
    f = bench.pmc_freshness(bench.load_pmc("4k"), LIB)
    if f["traffic_stale"] is None:
        pytest.skip("counters recorded before kernel sha256s were kept")
    assert f["traffic_stale"] is False and f["valu_stale"] is False
