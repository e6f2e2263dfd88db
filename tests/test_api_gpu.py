"""The DistributedPointFunction API (host C++ -> C ABI -> gfx950 kernels) on an
MI355X: the reference's own correctness grids and error paths
(dpf/distributed_point_function_test.cc), and bit-exact parity with the CPU
oracle on identical keys."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle as O
import dpf_checks as C
import ref_grids as G
from distributed_point_functions_amd import dpf as D
from distributed_point_functions_amd import proto as pb
from test_host_api_cpu import params, vt_from_oracle, leaves_value, _fixture_context

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


class GpuEngine:
    """The product API behind the dpf_checks engine interface."""

    def params(self, levels):
        dpf = D.DistributedPointFunction.create_incremental(params(levels))
        for _, vt, _ in levels:
            dpf.register_value_type(vt_from_oracle(vt))
        dpf._levels = levels
        return dpf

    def generate_keys(self, P, alpha, betas, seeds):
        vals = [leaves_value(vt, b) for (_, vt, _), b in zip(P._levels, betas)]
        return P.generate_keys_incremental(alpha, vals, seeds=seeds)

    def context(self, P, key):
        return P.create_evaluation_context(key)

    def evaluate_until(self, P, h, prefixes, ctx):
        return P.evaluate_until(h, prefixes, ctx, packed=True)

    def evaluate_at(self, P, key, h, points, ctx=None):
        if ctx is None:
            return P.evaluate_at(key, h, points, packed=True)
        return P.evaluate_at(h, points, ctx=ctx, packed=True)


E = GpuEngine()


@pytest.mark.parametrize("case", G.ONE_LEVEL_ELEMENT_SIZES + G.ONE_LEVEL_DOMAIN_SIZES,
                         ids=lambda c: str(c[0]))
@pytest.mark.parametrize("single_point", [False, True])
def test_two_party_one_level(case, single_point):
    levels, alphas, betas, steps = case
    for alpha in alphas:
        if alpha >= (1 << levels[-1][0]):
            continue
        for beta in betas:
            C.incremental_correctness(E, levels, alpha, beta, steps[0], single_point, seed=alpha)


@pytest.mark.parametrize("case", G.TWO_LEVELS + G.THREE_LEVELS, ids=lambda c: str(c[0]))
@pytest.mark.parametrize("single_point", [False, True])
def test_two_party_multi_level(case, single_point):
    levels, alphas, betas, steps = case
    for alpha in alphas:
        if alpha >= (1 << levels[-1][0]):
            continue
        for step in steps:
            C.incremental_correctness(E, levels, alpha, betas[-1], step, single_point,
                                      seed=alpha + step, num_points=300)


@pytest.mark.parametrize("step", [1, 2, 3, 5, 7])
@pytest.mark.parametrize("single_point", [False, True])
def test_two_party_max_domain(step, single_point):
    levels, alphas, betas, _ = G.MAX_DOMAIN
    C.incremental_correctness(E, levels, alphas[0], betas[0], step, single_point, num_points=200)


@pytest.mark.parametrize("vt", G.EVALUATION_TYPES, ids=str)
def test_typed_regular_dpf(vt):
    C.typed_regular(E, vt)


@pytest.mark.parametrize("vt", G.EVALUATION_TYPES, ids=str)
def test_typed_batch_single_point(vt):
    C.typed_batch_single_point(E, vt)


# ------------------------------------------------------------------ oracle parity
PARITY_CASES = [
    [(20, ("int", 64), 0)],
    [(14, ("int", 8), 0)],
    [(13, ("int", 128), 0)],
    [(12, ("xor", 128), 48.0)],
    [(11, ("tuple", [("intmodn", 32, G.M32)] * 2), 48.0)],
    [(10, ("tuple", [("int", 32), ("int", 64)]), 48.0)],
    [(5, ("int", 8), 0), (10, ("int", 16), 0), (15, ("int", 32), 0)],
    [(4, ("int", 64), 0), (9, ("int", 64), 0), (16, ("int", 64), 0)],
]


@pytest.mark.parametrize("levels", PARITY_CASES, ids=str)
def test_bit_exact_vs_oracle_incremental(levels):
    P = O.OracleParams(levels)
    alpha = (1 << levels[-1][0]) // 3
    betas = [[7 + i] * len(O.leaves(vt)) for i, (_, vt, _) in enumerate(levels)]
    ok0, ok1 = O.generate_keys(P, alpha, betas, 0x1234, 0x5678)
    dpf = E.params(levels)
    k0, k1 = E.generate_keys(dpf, alpha, betas, (0x1234, 0x5678))
    rng = np.random.default_rng(len(levels))
    # Prefixes of each call must extend those of the previous call (h:262-300).
    plan, prev_set = [], None
    for h in range(len(levels)):
        if h == 0:
            plan.append([])
            continue
        lp = levels[h - 1][0]
        a_pref = alpha >> (levels[-1][0] - lp)
        if prev_set is None:
            cur = sorted(set(int(x) for x in rng.integers(0, 1 << lp, size=6)) | {a_pref})
        else:
            shift = lp - levels[h - 2][0]
            cur = sorted({(p << shift) | int(rng.integers(0, 1 << shift)) for p in prev_set} | {a_pref})
        plan.append(cur)
        prev_set = cur
    for okey, key in ((ok0, k0), (ok1, k1)):
        octx, ctx = O.create_context(P, okey), dpf.create_evaluation_context(key)
        for h in range(len(levels)):
            want = O.evaluate_until(P, h, plan[h], octx)
            got = dpf.evaluate_until(h, plan[h], ctx, packed=True)
            np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("levels", PARITY_CASES, ids=str)
def test_bit_exact_vs_oracle_evaluate_at(levels):
    P = O.OracleParams(levels)
    h = len(levels) - 1
    alpha = (1 << levels[-1][0]) // 5
    betas = [[9] * len(O.leaves(vt)) for (_, vt, _) in levels]
    ok0, _ = O.generate_keys(P, alpha, betas, 0x99, 0x98)
    dpf = E.params(levels)
    k0, _ = E.generate_keys(dpf, alpha, betas, (0x99, 0x98))
    rng = np.random.default_rng(3)
    pts = [int(x) for x in rng.integers(0, 1 << levels[h][0], size=500)] + [alpha]
    np.testing.assert_array_equal(dpf.evaluate_at(k0, h, pts, packed=True),
                                  O.evaluate_at(P, ok0, h, pts))


# Small calls move no data by DMA by default: argument images of <= 128 KiB
# are read by the kernels from page-locked memory and results of <= 1 MiB are
# written there (PackedUploads / PinnedOut).  Every combination of those two
# and the copying paths they replace stays bit-exact against the oracle.
@pytest.mark.parametrize("upload", ["1", "0"])
@pytest.mark.parametrize("output", ["1", "0"])
@pytest.mark.parametrize("levels", [PARITY_CASES[0], PARITY_CASES[-1]], ids=str)
def test_small_call_copy_modes(levels, upload, output, monkeypatch):
    monkeypatch.setenv("DPF_UPLOAD_ZERO_COPY", upload)
    monkeypatch.setenv("DPF_OUTPUT_ZERO_COPY", output)
    test_bit_exact_vs_oracle_incremental(levels)
    test_bit_exact_vs_oracle_evaluate_at(levels)


def test_golden_full_domain_fixtures():
    g = json.load(open(os.path.join(GOLDEN, "full_domain.json")))
    for case in g["cases"]:
        vt = _vt_from_json(json.loads(case["value_type"]))
        levels = [(case["log_domain_size"], vt, case["security_parameter"])]
        dpf = E.params(levels)
        k0, k1 = E.generate_keys(dpf, int(case["alpha"], 16), [[int(b, 16) for b in case["beta"]]],
                                 (int(case["seed0"], 16), int(case["seed1"], 16)))
        assert [hex((c.seed.high << 64) | c.seed.low) for c in k0.correction_words] == case["cw_seeds"]
        for key, digest in ((k0, case["party0_sha256"]), (k1, case["party1_sha256"])):
            out = dpf.evaluate_until(0, [], dpf.create_evaluation_context(key), packed=True)
            assert hashlib.sha256(np.ascontiguousarray(out).tobytes()).hexdigest() == digest


def _vt_from_json(v):
    if v[0] == "tuple":
        return ("tuple", [_vt_from_json(e) for e in v[1]])
    return tuple(v)


# ------------------------------------------------------------------ reference error paths on ctx
def _three_level_128():
    dpf = D.DistributedPointFunction.create_incremental(
        params([(5, ("int", 128), 0), (10, ("int", 128), 0), (15, ("int", 128), 0)]))
    a, _ = dpf.generate_keys_incremental(1, [1, 2, 3])
    return dpf, dpf.create_evaluation_context(a)


def test_fails_if_prefix_not_present_in_ctx():
    # test.cc:470-491
    dpf, ctx = _three_level_128()
    dpf.evaluate_next([], ctx)
    dpf.evaluate_next([0, 1], ctx)
    del ctx.partial_evaluations[0]
    with pytest.raises(D.DpfStatusError) as e:
        dpf.evaluate_next([0], ctx)
    assert e.value.message == "Prefix not present in ctx.partial_evaluations at hierarchy level 1"


def test_fails_if_duplicate_prefix_in_ctx():
    # test.cc:493-519
    dpf, ctx = _three_level_128()
    dpf.evaluate_next([], ctx)
    dpf.evaluate_next([0, 1], ctx)
    dup = ctx.partial_evaluations.add()
    dup.CopyFrom(ctx.partial_evaluations[0])
    dup.seed.low = (dup.seed.low + 1) & ((1 << 64) - 1)
    with pytest.raises(D.DpfStatusError) as e:
        dpf.evaluate_next([0], ctx)
    assert e.value.message == ("Duplicate prefix in `ctx.partial_evaluations()` with mismatching "
                               "seed or control bit")


def test_fails_if_level_already_evaluated():
    dpf, ctx = _three_level_128()
    dpf.evaluate_until(0, [], ctx)
    with pytest.raises(D.DpfStatusError) as e:
        dpf.evaluate_until(0, [], ctx)
    assert e.value.message == "`hierarchy_level` must be greater than `ctx.previous_hierarchy_level`"


def test_fails_if_prefix_out_of_range():
    dpf, ctx = _three_level_128()
    dpf.evaluate_until(0, [], ctx)
    with pytest.raises(D.DpfStatusError) as e:
        dpf.evaluate_until(1, [1 << 5], ctx)
    assert e.value.message == "Index 32 out of range for hierarchy level 0"


def test_fully_evaluated_context_rejected():
    dpf, ctx = _three_level_128()
    dpf.evaluate_until(0, [], ctx)
    dpf.evaluate_until(1, [0], ctx)
    dpf.evaluate_until(2, [0], ctx)
    with pytest.raises(D.DpfStatusError) as e:
        dpf.evaluate_until(2, [0], ctx)
    assert e.value.message == "This context has already been fully evaluated"


def test_single_point_partial_evaluation():
    # test.cc:157-202: EvaluateAt on a 2^108 level through ctx, then a full
    # 2^20 expansion below that prefix.
    dpf = D.DistributedPointFunction.create_incremental(
        params([(108, ("int", 32), 0), (128, ("int", 32), 0)]))
    prefix, suffix, beta = 0xDEADBEEF, 23, 42
    alpha = (prefix << 20) + suffix
    ka, kb = dpf.generate_keys_incremental(alpha, [beta, beta])
    ca, cb = dpf.create_evaluation_context(ka), dpf.create_evaluation_context(kb)
    ra = dpf.evaluate_at(0, [prefix], ctx=ca)
    rb = dpf.evaluate_at(0, [prefix], ctx=cb)
    assert (int(ra[0]) + int(rb[0])) & 0xFFFFFFFF == beta
    ra = dpf.evaluate_until(1, [prefix], ca)
    rb = dpf.evaluate_until(1, [prefix], cb)
    assert ra.size == 1 << 20
    s = (ra.astype(np.uint64) + rb.astype(np.uint64)) & 0xFFFFFFFF
    assert s[suffix] == beta
    assert np.count_nonzero(s) == 1


def test_fixture_context_value_correction_error_on_gpu():
    ctx = _fixture_context()
    dpf = D.DistributedPointFunction.create_incremental(list(ctx.parameters))
    with pytest.raises(D.DpfStatusError) as e:
        dpf.evaluate_until(0, [], ctx)
    assert e.value.message == "values.size() (= 1) does not match ElementsPerBlock<T>() (= 4)"


# ------------------------------------------------------------------ extensions
def test_evaluate_until_to_device_matches_host():
    import torch
    dpf = E.params([(22, ("int", 64), 0)])
    k0, _ = E.generate_keys(dpf, 12345, [[42]], (1, 2))
    host_out = dpf.evaluate_until(0, [], dpf.create_evaluation_context(k0))
    dev = torch.empty((1 << 22) * 8, dtype=torch.uint8, device="cuda")
    n = dpf.evaluate_until_to_device(0, [], dpf.create_evaluation_context(k0), dev)
    torch.cuda.synchronize()
    assert n == 1 << 22
    np.testing.assert_array_equal(dev.cpu().numpy().view(np.uint64), host_out)


def test_evaluate_until_to_device_with_prefix_gather():
    import torch
    levels = [(6, ("int", 16), 0), (14, ("int", 16), 0)]
    dpf = E.params(levels)
    k0, _ = E.generate_keys(dpf, 999, [[1], [2]], (3, 4))
    prefixes = [5, 3, 5, 60]
    c1 = dpf.create_evaluation_context(k0)
    dpf.evaluate_until(0, [], c1)
    want = dpf.evaluate_until(1, prefixes, c1, packed=True)
    c2 = dpf.create_evaluation_context(k0)
    dpf.evaluate_until(0, [], c2)
    dev = torch.zeros(want.size, dtype=torch.uint8, device="cuda")
    n = dpf.evaluate_until_to_device(1, prefixes, c2, dev)
    torch.cuda.synchronize()
    assert n == len(prefixes) << 8
    np.testing.assert_array_equal(dev.cpu().numpy().reshape(want.shape), want)
    assert c1 == c2


@pytest.mark.parametrize("vt", [("int", 64), ("xor", 128), ("tuple", [("intmodn", 32, G.M32)] * 2)],
                         ids=str)
def test_evaluate_at_batch_matches_per_key(vt):
    levels = [(40, vt, 48.0)]
    dpf = E.params(levels)
    rng = np.random.default_rng(5)
    keys = []
    for k in range(9):
        a, b = E.generate_keys(dpf, int(rng.integers(0, 1 << 40)), [[k + 1] * len(O.leaves(vt))],
                               (100 + k, 200 + k))
        keys.append(a if k % 2 == 0 else b)
    ppk = 70
    pts = [int(x) for x in rng.integers(0, 1 << 40, size=9 * ppk)]
    got = dpf.evaluate_at_batch(keys, 0, pts, ppk, packed=True)
    want = np.concatenate([dpf.evaluate_at(keys[k], 0, pts[k * ppk:(k + 1) * ppk], packed=True)
                           for k in range(9)])
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("levels,num_shards", [
    ([(20, ("int", 64), 0)], 4),
    ([(20, ("int", 64), 0)], 1),
    ([(17, ("int", 32), 0)], 8),
    ([(12, ("xor", 128), 0)], 16),
    ([(10, ("tuple", [("int", 32), ("intmodn", 64, G.M64)]), 0)], 2),
    ([(6, ("int", 16), 0), (15, ("int", 64), 0)], 4),
], ids=str)
def test_evaluate_shard_to_device_concatenates_to_full_domain(levels, num_shards):
    """Weak-scaling shards (subtree prefixes of the top log2(N) tree levels)
    concatenate to EvaluateUntil(h, {}) on a fresh context -- the multi-GPU
    partition bench.py uses."""
    import torch
    dpf = E.params(levels)
    k0, k1 = E.generate_keys(dpf, 0x5a5a % (1 << levels[0][0]),
                             [[7] * len(O.leaves(l[1])) for l in levels], (11, 12))
    h = len(levels) - 1
    for key in (k0, k1):
        # a fresh context evaluated straight to level h gives its full domain
        want = dpf.evaluate_until(h, [], dpf.create_evaluation_context(key), packed=True)
        per = want.size // num_shards
        dev = torch.zeros(want.size, dtype=torch.uint8, device="cuda")
        for s in range(num_shards):
            ctx = dpf.create_evaluation_context(key)
            n = dpf.evaluate_shard_to_device(h, s, num_shards, ctx, dev[s * per:(s + 1) * per])
            assert n * want.shape[1] == per
            assert ctx.previous_hierarchy_level == h
        torch.cuda.synchronize()
        np.testing.assert_array_equal(dev.cpu().numpy().reshape(want.shape), want)


def test_evaluate_shard_to_device_errors():
    import torch
    dpf = E.params([(10, ("int", 64), 0)])
    k0, _ = E.generate_keys(dpf, 3, [[1]], (1, 2))
    dev = torch.zeros(1 << 13, dtype=torch.uint8, device="cuda")
    for shard, num in [(0, 3), (4, 4), (-1, 2), (0, 0)]:
        with pytest.raises(D.DpfStatusError) as e:
            dpf.evaluate_shard_to_device(0, shard, num, dpf.create_evaluation_context(k0), dev)
        assert e.value.code == 3
    with pytest.raises(D.DpfStatusError, match="too small"):
        dpf.evaluate_shard_to_device(0, 0, 1, dpf.create_evaluation_context(k0), dev[:100])
    ctx = dpf.create_evaluation_context(k0)
    dpf.evaluate_until(0, [], ctx)
    with pytest.raises(D.DpfStatusError, match="fully evaluated"):
        dpf.evaluate_shard_to_device(0, 0, 2, ctx, dev)
    dpf2 = E.params([(5, ("int", 64), 0), (10, ("int", 64), 0)])
    a, _ = E.generate_keys(dpf2, 3, [[1], [2]], (1, 2))
    ctx = dpf2.create_evaluation_context(a)
    dpf2.evaluate_until(0, [], ctx)
    with pytest.raises(D.DpfStatusError, match="first call"):
        dpf2.evaluate_shard_to_device(1, 0, 2, ctx, dev)


@pytest.mark.parametrize("log,vt", [(26, ("int", 64)), (25, ("int", 128)), (22, ("int", 64)),
                                    (24, ("tuple", [("int", 32), ("int", 64)]))], ids=str)
def test_large_host_output_matches_device(log, vt):
    """Host outputs of >= 512 MiB (DPF_HIP_REGISTER_MIN_BYTES) take
    dpf_hip_memcpy_d2h_staged: the fresh vector is mapped and registered piece
    by piece and value-initialised chunk by chunk while the previous 64 MiB
    chunk's DMA runs; smaller ones arrive through the 16 MiB page-locked staging buffers
    chunk by chunk (dpf_hip_memcpy_d2h_chunked).  Every byte equals the device
    output, and the two parties' host outputs reconstruct the point function."""
    import torch
    dpf = E.params([(log, vt, 0)])
    alpha = (1 << log) - 12345
    beta = [[7]] if vt[0] == "int" else [[3, 9]]
    k0, k1 = E.generate_keys(dpf, alpha, beta, (11, 12))
    host0 = dpf.evaluate_until(0, [], dpf.create_evaluation_context(k0), packed=True)
    host1 = dpf.evaluate_until(0, [], dpf.create_evaluation_context(k1), packed=True)
    dev = torch.empty(host0.size, dtype=torch.uint8, device="cuda")
    n = dpf.evaluate_until_to_device(0, [], dpf.create_evaluation_context(k0), dev)
    torch.cuda.synchronize()
    assert n == 1 << log
    np.testing.assert_array_equal(dev.cpu().numpy().reshape(host0.shape), host0)
    total = O.add_packed(vt, host0.reshape(1 << log, -1), host1.reshape(1 << log, -1))
    nz = np.flatnonzero(total.reshape(1 << log, -1).any(axis=1))
    assert nz.tolist() == [alpha]


@pytest.mark.parametrize("env", [{}, {"DPF_HIP_D2H_REGISTER_PIECES": "1"},
                                 {"DPF_HIP_D2H_REGISTER_PIECES": "0"},
                                 {"DPF_HIP_D2H_PIPELINE": "0"}, {"DPF_EVAL_SPLIT": "0"},
                                 {"DPF_EVAL_SPLIT": "0", "DPF_HIP_D2H_PIPELINE": "0"}], ids=str)
def test_pipelined_host_output_and_its_fallbacks(env, monkeypatch):
    """A fresh host output of >= 512 MiB is mapped and registered in 256 MiB
    pieces by a helper thread while the DMA fills the pieces already
    registered (dpf_kernels.hip: pipelined_d2h).  A 1 GiB output (five pieces:
    the vector starts off a 2 MiB boundary) equals the device output byte for
    byte by default, when the registration of piece 1 or 0 and every later one
    is refused (the rest of the range through the bounce buffers), and with
    the pipeline off (map and register the whole range first).  By default
    the expansion itself runs as 8 subtree launches whose events the copy
    waits for part by part (DPF_EVAL_SPLIT=0: one launch).  The hooks are
    read per call."""
    import torch
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    log = 27
    dpf = E.params([(log, ("int", 64), 0)])
    k0, _ = E.generate_keys(dpf, (1 << log) - 777, [[5]], (31, 32))
    host = dpf.evaluate_until(0, [], dpf.create_evaluation_context(k0), packed=True)
    dev = torch.empty(host.size, dtype=torch.uint8, device="cuda")
    dpf.evaluate_until_to_device(0, [], dpf.create_evaluation_context(k0), dev)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dev.cpu().numpy().reshape(host.shape), host)


def test_split_first_call_then_next_level():
    """A first call whose >= 512 MiB host output is expanded as 8 subtree
    launches leaves the context as one launch does: the next level's call
    (from its prefixes) equals the device path's, and both levels reconstruct
    the point function with the other party's key."""
    import torch
    dpf = E.params([(26, ("int", 64), 0), (27, ("int", 64), 0)])
    alpha = (1 << 27) - 4321
    k0, k1 = E.generate_keys(dpf, alpha, [[3], [4]], (71, 72))
    prefixes = [alpha >> 1, 17, (1 << 26) - 1]
    got = []
    for key in (k0, k1):
        ctx = dpf.create_evaluation_context(key)
        h0 = dpf.evaluate_until(0, [], ctx, packed=True)
        h1 = dpf.evaluate_until(1, prefixes, ctx, packed=True)
        ctx_d = dpf.create_evaluation_context(key)
        dev = torch.empty(h0.size, dtype=torch.uint8, device="cuda")
        dpf.evaluate_until_to_device(0, [], ctx_d, dev)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(dev.cpu().numpy().reshape(h0.shape), h0)
        del dev
        np.testing.assert_array_equal(h1, dpf.evaluate_until(1, prefixes, ctx_d, packed=True))
        got.append((h0, h1))
    vt = ("int", 64)
    t0 = O.add_packed(vt, got[0][0], got[1][0])
    assert np.flatnonzero(t0.any(axis=1)).tolist() == [alpha >> 1]
    t1 = O.add_packed(vt, got[0][1], got[1][1])
    assert np.flatnonzero(t1.any(axis=1)).tolist() == [2 * 0 + (alpha & 1)]


def test_concurrent_pipelined_host_outputs():
    """Two threads evaluate 512 MiB host outputs at once (two pipelined
    copies, each with its own helper thread and registrations): each equals
    the same key's sequential result."""
    from concurrent.futures import ThreadPoolExecutor
    dpf = E.params([(26, ("int", 64), 0)])
    keys = [E.generate_keys(dpf, 999 + 5 * i, [[i + 2]], (50 + i, 60 + i))[i % 2] for i in range(2)]
    want = [dpf.evaluate_until(0, [], dpf.create_evaluation_context(k), packed=True) for k in keys]
    with ThreadPoolExecutor(2) as ex:
        got = list(ex.map(lambda k: dpf.evaluate_until(0, [], dpf.create_evaluation_context(k),
                                                         packed=True), keys))
    for i, g in enumerate(got):
        np.testing.assert_array_equal(g, want[i])
    del got, want


def test_concurrent_large_host_outputs():
    """Four threads evaluate different keys into fresh host vectors at once
    (the registered-DMA path of >= 32 MiB outputs runs concurrently, GIL
    released): every result equals the same key's sequential result."""
    from concurrent.futures import ThreadPoolExecutor
    dpf = E.params([(24, ("int", 64), 0)])
    keys = [E.generate_keys(dpf, 1000 + 7 * i, [[i + 1]], (20 + i, 40 + i))[i % 2] for i in range(4)]
    want = [dpf.evaluate_until(0, [], dpf.create_evaluation_context(k), packed=True) for k in keys]
    with ThreadPoolExecutor(4) as ex:
        got = list(ex.map(lambda k: dpf.evaluate_until(0, [], dpf.create_evaluation_context(k),
                                                         packed=True), keys * 2))
    for i, g in enumerate(got):
        np.testing.assert_array_equal(g, want[i % 4])
