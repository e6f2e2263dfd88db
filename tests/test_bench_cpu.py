"""CPU checks of bench.py's measurement helpers: the algorithmic AES count of
SURVEY.md 8(d), the proto Value flattening the tuple CPU baselines feed to the
oracle, and the lookup of committed rocprofv3 summaries by kernel name (the
octet kernel's name carries an anonymous-namespace qualifier in rocprofv3
traces)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.fixture(scope="module")
def bench():
    argv = sys.argv
    sys.argv = ["bench.py"]
    try:
        import bench as b
    finally:
        sys.argv = argv
    return b


def test_tree_aes_per_launch_matches_survey(bench):
    # config 2 = 2 (2^29 - 1) + 2^29 AES blocks.
    assert bench.tree_aes_per_launch(29) == 1610612734
    assert bench.tree_aes_per_launch(19) == 1572862          # config 1
    assert bench.tree_aes_per_launch(3, 2) == 2 * 7 + 2 * 8  # two value blocks per leaf


def test_leaf_ints_flattens_tuples(bench):
    from distributed_point_functions_amd import dpf as D
    el = D.int_mod_n_type(32, 4294967291)
    v = D.to_value(D.tuple_type(el, el), (123456789, 4000000000))
    assert bench._leaf_ints(v) == [123456789, 4000000000]
    v = D.to_value(D.tuple_type(D.integer_type(32), D.integer_type(128)), (7, (1 << 100) + 3))
    assert bench._leaf_ints(v) == [7, (1 << 100) + 3]
    assert bench._leaf_ints(D.to_value(D.integer_type(64), 42)) == [42]


def test_profiled_traffic_ignores_namespace_qualifier(bench, tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    summary = {"kernel": "void (anonymous namespace)::expand_octet_kernel<(anonymous namespace)::"
                         "FastIntLeaf<64, false> >((anonymous namespace)::ExpandParams, "
                         "(anonymous namespace)::FastIntLeaf<64, false>)",
               "leaves_per_launch": 1 << 30, "hbm_traffic_bytes": 12.0e9, "avg_ns": 17.5e6}
    (prof / "r99_summary.json").write_text(json.dumps(summary))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    tr = bench.profiled_traffic(bench.KERNEL, 1 << 30)
    assert tr is not None and tr[0] == 12.0e9 and tr[1] == os.path.join("profiles",
                                                                        "r99_summary.json")
    # Queries written with the qualifier match too; other sizes do not.
    assert bench.profiled_traffic("expand_octet_kernel<(anonymous namespace)::FastIntLeaf<64, "
                                  "false> >", 1 << 30) is not None
    assert bench.profiled_traffic(bench.KERNEL, 1 << 29) is None


def test_committed_profile_backs_the_headline(bench):
    # The newest committed summary of the headline kernel at config 2's size.
    tr = bench.profiled_traffic(bench.KERNEL, 1 << 30)
    assert tr is not None
    assert 8.5e9 < tr[0] < 30e9      # >= the 8 GiB written, well below HBM-bound
