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


def _run_bench(args, env_extra=None, timeout=120):
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT,
                          env=env, capture_output=True, text=True, timeout=timeout)


def test_gpus_flag_never_falls_back_to_one_rank():
    # No GPU here: `--gpus 2` without a launcher must refuse (exit non-zero)
    # before it would start ranks, never run one rank and report n_gpus 1.
    r = _run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr and not r.stdout.strip()


def test_gpus_flag_must_match_launcher_world_size():
    r = _run_bench(["--gpus", "2"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr
    r = _run_bench(["--gpus", "2", "--workload", "synthetic_direct"])
    assert r.returncode != 0 and "one GPU" in r.stderr


def test_launcher_cmd_relaunches_same_arguments(bench):
    cmd = bench.launcher_cmd(["--gpus", "8", "--steps", "5"], 8, 29511)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29511"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"]
    assert os.path.basename(cmd[-5]) == "bench.py"


def _parse(bench, argv):
    old = sys.argv
    sys.argv = ["bench.py", *argv]
    try:
        return bench.parse()
    finally:
        sys.argv = old


def test_default_line_is_the_metric_configuration(bench):
    # BASELINE metric: ONE 2^30 uint64 domain at 1/2/4/8 GPUs -> strong
    # scaling by default; the drop-in API rate (api_level) on by default.
    a = _parse(bench, [])
    assert a.workload == "full_domain" and a.log_domain == 30
    assert a.scaling == "strong" and a.host_output
    assert _parse(bench, ["--gpus", "8"]).scaling == "strong"
    assert not _parse(bench, ["--no-host-output"]).host_output
    assert _parse(bench, ["--scaling", "weak"]).scaling == "weak"
    # config 3 (2^34 uint128 over 8 GPUs = 2^31 per GPU): weak by default.
    assert _parse(bench, ["--workload", "full_domain_u128"]).scaling == "weak"
    with pytest.raises(SystemExit):
        _parse(bench, ["--gpus", "2", "--rehearse-world", "8"])
    assert _parse(bench, ["--rehearse-world", "8"]).rehearse_world == 8


def test_line_keys_pinned_in_source(bench):
    # The keys the driver's line carries beside `value` (bench.py builds them
    # only on a GPU; pinned here by source so a refactor cannot drop them).
    src = open(os.path.join(ROOT, "bench.py")).read()
    for key in ('"scaling": args.scaling', "sustained_clock_ghz=", "clk_per_aes_per_cu=",
                '"step_overhead"', 'res["api_level"]', "H.clock_probe(True)"):
        assert key in src, key
