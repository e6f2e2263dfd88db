"""DCF evaluation on an MI355X (dpf_hip_dcf_eval_batch): bit-exact against the
oracle's restatement of Evaluate (dcf/distributed_comparison_function.h:83-105)
on the same keys, the reference's GenEval and large-domain properties
(distributed_comparison_function_test.cc:96-177), and batches of keys."""
import numpy as np
import pytest

import oracle as O
import ref_grids as G
from distributed_point_functions_amd import dpf as D
from test_dcf_cpu import TYPES, make
from test_host_api_cpu import leaves_value

pytestmark = pytest.mark.gpu

MORE = [(("int", 8), 5), (("int", 16), 6), (("int", 64), 7), (("xor", 64), 4),
        (("intmodn", 64, G.M64), 5), (("tuple", [("int", 16), ("intmodn", 128, G.M80)]), 4),
        (("tuple", [("int", 8)] * 5), 3)]


@pytest.mark.parametrize("vt,n", TYPES + MORE, ids=str)
def test_dcf_all_points_bit_exact(vt, n):
    dcf = make(vt, n)
    P = O.dcf_params(n, vt)
    beta = [42] * len(O.leaves(vt))
    xs = list(range(1 << n))
    for alpha in range(1 << n):
        keys = dcf.generate_keys(alpha, leaves_value(vt, beta), seed_0=alpha + 3, seed_1=alpha + 77)
        okeys = O.dcf_generate_keys(P, alpha, beta, alpha + 3, alpha + 77)
        shares = []
        for k, ok in zip(keys, okeys):
            got = dcf.evaluate_packed(k, xs)
            want = np.concatenate([O.dcf_evaluate(P, ok, x) for x in xs])
            np.testing.assert_array_equal(got, want, err_msg=f"alpha={alpha}")
            shares.append(got)
        if vt[0] != "xor":  # SetToZero leaves XorWrapper betas unchanged (cc:21-32)
            total = O.unpack_elements(vt, O.add_packed(vt, shares[0], shares[1]))
            for x in xs:
                assert total[x] == (beta if x < alpha else [0] * len(beta)), (alpha, x)


@pytest.mark.parametrize("upload,output", [("1", "1"), ("0", "0"), ("1", "0"), ("0", "1")])
def test_dcf_uint64_large_domain(upload, output, monkeypatch):
    # test.cc:125-177; with and without the small-call zero-copy paths
    # (DPF_UPLOAD_ZERO_COPY / DPF_OUTPUT_ZERO_COPY).
    monkeypatch.setenv("DPF_UPLOAD_ZERO_COPY", upload)
    monkeypatch.setenv("DPF_OUTPUT_ZERO_COPY", output)
    dcf = make(("int", 64), 64)
    P = O.dcf_params(64, ("int", 64))
    alpha = 50
    k0, k1 = dcf.generate_keys(alpha, 42, seed_0=11, seed_1=12)
    o0, o1 = O.dcf_generate_keys(P, alpha, [42], 11, 12)
    rng = np.random.default_rng(5)
    xs = list(range(alpha)) + [int(x) for x in rng.integers(0, 2**63, size=99)] + [2**64 - 1]
    a = dcf.evaluate_packed(k0, xs).view(np.uint64).reshape(-1)
    b = dcf.evaluate_packed(k1, xs).view(np.uint64).reshape(-1)
    for i, x in enumerate(xs):
        assert int(a[i]) + int(b[i]) & (2**64 - 1) == (42 if x < alpha else 0), x
    for i in (0, 49, 50, len(xs) - 1):
        assert int(a[i]) == int(O.dcf_evaluate(P, o0, xs[i]).view(np.uint64)[0, 0])


def test_dcf_domain_128_prefix_quirk():
    # h:88-92: with log_domain_size == 128 every level is evaluated at prefix 0.
    dcf = make(("int", 32), 128)
    P = O.dcf_params(128, ("int", 32))
    k0, _ = dcf.generate_keys(2**127 + 5, 9, seed_0=1, seed_1=2)
    o0, _ = O.dcf_generate_keys(P, 2**127 + 5, [9], 1, 2)
    xs = [0, 1, 2**127 + 4, 2**128 - 1, 12345678901234567890123456789]
    got = dcf.evaluate_packed(k0, xs)
    want = np.concatenate([O.dcf_evaluate(P, o0, x) for x in xs])
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("vt,n,shared", [(("int", 64), 20, False), (("int", 64), 20, True),
                                         (("tuple", [("intmodn", 32, G.M32)] * 2), 16, False),
                                         (("int", 128), 33, True)], ids=str)
def test_dcf_batch_to_device(vt, n, shared):
    import torch
    dcf = make(vt, n)
    P = O.dcf_params(n, vt)
    rng = np.random.default_rng(n)
    nk, ppk = 37, 65
    beta = [int(b) for b in rng.integers(1, 1000, size=len(O.leaves(vt)))]
    keys, okeys = [], []
    for k in range(nk):
        alpha = int(rng.integers(0, 1 << n))
        ks = dcf.generate_keys(alpha, leaves_value(vt, beta), seed_0=k + 1, seed_1=k + 500)
        oks = O.dcf_generate_keys(P, alpha, beta, k + 1, k + 500)
        keys.append(ks[k % 2])
        okeys.append(oks[k % 2])
    npts = ppk if shared else nk * ppk
    pts = [int(x) for x in rng.integers(0, 1 << n, size=npts)]
    batch = dcf.make_key_batch(keys)
    dev = dcf.upload_key_batch(batch)
    dpts = torch.from_numpy(D.u128_array(pts).view(np.int64)).cuda()
    size = dcf.packed_size()
    out = torch.empty(nk * ppk * size, dtype=torch.uint8, device="cuda")
    assert dcf.evaluate_batch_to_device(dev, dpts, ppk, out, shared_points=shared) == nk * ppk
    got = out.cpu().numpy().reshape(nk, ppk, size)
    for k in (0, 1, nk // 2, nk - 1):
        kp = pts if shared else pts[k * ppk:(k + 1) * ppk]
        want = np.concatenate([O.dcf_evaluate(P, okeys[k], x) for x in kp])
        np.testing.assert_array_equal(got[k], want, err_msg=f"key {k}")


def test_dcf_errors_match_reference():
    dcf = make(("int", 32), 6)
    k0, _ = dcf.generate_keys(3, 1)
    with pytest.raises(D.DpfStatusError,
                       match="`evaluation_points\\[0\\]` larger than the domain size at hierarchy level 0"):
        dcf.evaluate_packed(k0, [64])
    with pytest.raises(D.DpfStatusError, match="Value type T doesn't match"):
        dcf.evaluate(k0, 3, D.integer_type(64))


def _batch_case(vt, n, nk, ppk, shared, seed):
    import torch
    dcf = make(vt, n)
    P = O.dcf_params(n, vt)
    rng = np.random.default_rng(seed)
    beta = [int(b) for b in rng.integers(1, 100, size=len(O.leaves(vt)))]
    alphas = [int(a) for a in rng.integers(0, 1 << min(n, 63), size=nk)]
    keys = [dcf.generate_keys(a, leaves_value(vt, beta), seed_0=2 * k + 1, seed_1=2 * k + 2)[k % 2]
            for k, a in enumerate(alphas)]
    npts = ppk if shared else nk * ppk
    hi = 1 << min(n, 127)
    pts = [int(x) for x in rng.integers(0, min(hi, 2**63), size=npts)]
    # Points near each key's alpha as well, so both comparison outcomes occur.
    if not shared:
        for k in range(nk):
            pts[k * ppk] = alphas[k]
            pts[k * ppk + 1] = max(alphas[k] - 1, 0)
    dev = dcf.upload_key_batch(dcf.make_key_batch(keys))
    dpts = torch.from_numpy(D.u128_array(pts).view(np.int64)).cuda()
    size = dcf.packed_size()

    def run():
        out = torch.empty(nk * ppk * size, dtype=torch.uint8, device="cuda")
        assert dcf.evaluate_batch_to_device(dev, dpts, ppk, out, shared_points=shared) == nk * ppk
        return out.cpu().numpy().reshape(nk, ppk, size)

    return dcf, P, beta, alphas, pts, run


FAST_TYPES = [("int", 8), ("int", 16), ("int", 32), ("int", 64), ("int", 128), ("xor", 32),
              ("xor", 64)]


@pytest.mark.parametrize("quad", ["1", "0"])
@pytest.mark.parametrize("vt", FAST_TYPES, ids=str)
@pytest.mark.parametrize("n,shared", [(17, False), (64, True), (128, False)], ids=str)
def test_dcf_fast_kernel_uniform_keys(vt, n, shared, quad, monkeypatch):
    """dcf_fast_kernel with wave-uniform keys (points_per_key % 64 == 0) is
    bit-exact against the general kernel on every output and against the
    oracle on sampled rows -- in latency mode (a launch this small runs one
    (key, x) per lane quad, dcf_fast_quad_kernel) and, with DPF_DCF_QUAD=0,
    one per lane."""
    monkeypatch.setenv("DPF_DCF_QUAD", quad)
    nk, ppk = 24, 128
    dcf, P, beta, alphas, pts, run = _batch_case(vt, n, nk, ppk, shared, seed=n * 7 + len(vt))
    got = run()
    monkeypatch.setenv("DPF_DCF_GENERAL", "1")
    general = run()
    np.testing.assert_array_equal(got, general)
    rng = np.random.default_rng(3)
    for k in (0, nk - 1):
        okeys = O.dcf_generate_keys(P, alphas[k], beta, 2 * k + 1, 2 * k + 2)
        for j in [0, 1] + [int(q) for q in rng.integers(0, ppk, size=6)]:
            x = pts[j] if shared else pts[k * ppk + j]
            np.testing.assert_array_equal(got[k, j], O.dcf_evaluate(P, okeys[k % 2], x).reshape(-1),
                                          err_msg=f"key {k} point {j}")


@pytest.mark.parametrize("vt", [("int", 64), ("xor", 32), ("int", 8)], ids=str)
def test_dcf_fast_kernel_full_launch(vt, monkeypatch):
    """A launch that fills the chip twice over (512 keys x 1024 points):
    bit-exact against the general kernel on every output and against the
    oracle on sampled rows."""
    nk, ppk, n = 512, 1024, 64
    dcf, P, beta, alphas, pts, run = _batch_case(vt, n, nk, ppk, False, seed=99)
    got = run()
    monkeypatch.setenv("DPF_DCF_GENERAL", "1")
    general = run()
    np.testing.assert_array_equal(got, general)
    for k in (0, 1, nk - 1):
        okeys = O.dcf_generate_keys(P, alphas[k], beta, 2 * k + 1, 2 * k + 2)
        for j in (0, 1, 2, 700, ppk - 1):
            np.testing.assert_array_equal(got[k, j],
                                          O.dcf_evaluate(P, okeys[k % 2], pts[k * ppk + j]).reshape(-1))
