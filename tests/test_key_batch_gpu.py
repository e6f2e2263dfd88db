"""Batched EvaluateAt over a device key batch (SURVEY.md config 4 and its
aggregation variant) on an MI355X, bit-exact against the CPU oracle's
EvaluateAtImpl (distributed_point_function.h:839-1010) run key by key on the
same keys (oracle keygen with the same root seeds)."""
import numpy as np
import pytest

import oracle as O
import ref_grids as G
from distributed_point_functions_amd import dpf as D
from test_host_api_cpu import vt_from_oracle, leaves_value
from test_key_batch_cpu import make

pytestmark = pytest.mark.gpu
MASK64 = (1 << 64) - 1


def _rand_u128(rng, n, log):
    out = []
    for _ in range(n):
        x = (int(rng.integers(0, 1 << 63)) << 65) ^ int(rng.integers(0, 1 << 63)) ^ int(rng.integers(0, 4))
        out.append(x & ((1 << log) - 1) if log < 128 else x & ((1 << 128) - 1))
    return out


def _dev_points(pts):
    import torch
    return torch.from_numpy(D.u128_array(pts).view(np.int64)).cuda()


def _setup(levels, n_keys, seed, party_mix=True):
    dpf = make(levels)
    P = O.OracleParams(levels)
    rng = np.random.default_rng(seed)
    top = levels[-1][0]
    alphas = _rand_u128(rng, n_keys, top)
    seeds = rng.integers(1, 1 << 62, size=(2 * n_keys, 2), dtype=np.uint64)
    beta_leaves = [[(7 * h + 3) % 200 + 1] * len(O.leaves(vt)) for h, (_, vt, _) in enumerate(levels)]
    beta = [leaves_value(vt, b) for (_, vt, _), b in zip(levels, beta_leaves)]
    b0, b1 = dpf.generate_key_batch(alphas, beta, root_seeds=seeds, threads=4)
    okeys = []
    for k in range(n_keys):
        s0 = int(seeds[2 * k, 0]) | int(seeds[2 * k, 1]) << 64
        s1 = int(seeds[2 * k + 1, 0]) | int(seeds[2 * k + 1, 1]) << 64
        okeys.append(O.generate_keys(P, alphas[k], beta_leaves, s0, s1))
    # Mixed-party batch: even keys party 0, odd keys party 1.
    keys = [dpf.key_from_batch(b0 if (k % 2 == 0 or not party_mix) else b1, k) for k in range(n_keys)]
    mixed = dpf.make_key_batch(keys)
    oks = [okeys[k][0 if (k % 2 == 0 or not party_mix) else 1] for k in range(n_keys)]
    return dpf, P, rng, mixed, oks, alphas, okeys, (b0, b1)


CASES = [
    # (levels, hierarchy level, keys, points per key)
    ([(128, ("int", 64), 0)], 0, 6, 256),      # uniform-key waves (128 points per half)
    ([(128, ("int", 64), 0)], 0, 5, 7),        # odd points per key, ragged pairs
    ([(40, ("int", 128), 0)], 0, 9, 130),
    ([(30, ("int", 8), 0)], 0, 4, 200),        # 16 elements per block
    ([(64, ("xor", 128), 0)], 0, 3, 64),
    ([(20, ("xor", 16), 0)], 0, 3, 129),
    ([(24, ("tuple", [("intmodn", 32, G.M32)] * 2), 64.0)], 0, 5, 128),
    ([(10, ("int", 16), 0), (50, ("int", 64), 0)], 0, 4, 100),
    ([(10, ("int", 16), 0), (50, ("int", 64), 0)], 1, 4, 100),
    ([(12, ("tuple", [("int", 32), ("intmodn", 64, G.M64)]), 48.0)], 0, 3, 1),
]


@pytest.mark.parametrize("levels,h,n_keys,ppk", CASES, ids=str)
def test_evaluate_at_batch_per_key_points(levels, h, n_keys, ppk):
    import torch
    dpf, P, rng, batch, oks, _, _, _ = _setup(levels, n_keys, seed=n_keys * 31 + ppk)
    log = levels[h][0]
    pts = _rand_u128(rng, n_keys * ppk, log)
    dev_batch = dpf.upload_key_batch(batch)
    size = dpf.packed_size(h)
    out = torch.empty(n_keys * ppk * size, dtype=torch.uint8, device="cuda")
    n = dpf.evaluate_at_batch_to_device(dev_batch, h, _dev_points(pts), ppk, out)
    torch.cuda.synchronize()
    assert n == n_keys * ppk
    got = out.cpu().numpy().reshape(n_keys * ppk, size)
    for k in range(n_keys):
        want = O.evaluate_at(P, oks[k], h, pts[k * ppk:(k + 1) * ppk])
        np.testing.assert_array_equal(got[k * ppk:(k + 1) * ppk], want, err_msg=f"key {k}")


@pytest.mark.parametrize("levels,h,n_keys,ppk", CASES[:4] + CASES[6:7], ids=str)
def test_evaluate_at_batch_shared_points(levels, h, n_keys, ppk):
    import torch
    dpf, P, rng, batch, oks, _, _, _ = _setup(levels, n_keys, seed=ppk)
    pts = _rand_u128(rng, ppk, levels[h][0])
    dev_batch = dpf.upload_key_batch(batch)
    size = dpf.packed_size(h)
    out = torch.empty(n_keys * ppk * size, dtype=torch.uint8, device="cuda")
    dpf.evaluate_at_batch_to_device(dev_batch, h, _dev_points(pts), ppk, out, shared_points=True)
    got = out.cpu().numpy().reshape(n_keys, ppk, size)
    for k in range(n_keys):
        np.testing.assert_array_equal(got[k], O.evaluate_at(P, oks[k], h, pts))


SUM_CASES = [
    ([(128, ("int", 64), 0)], 0, 64, 256),
    ([(128, ("int", 64), 0)], 0, 7, 5),
    ([(40, ("int", 128), 0)], 0, 33, 130),
    ([(30, ("int", 8), 0)], 0, 20, 64),
    ([(64, ("xor", 128), 0)], 0, 9, 128),
    ([(24, ("tuple", [("intmodn", 32, G.M32)] * 2), 64.0)], 0, 17, 128),
    ([(12, ("tuple", [("int", 16), ("intmodn", 128, G.M80)]), 48.0)], 0, 6, 10),
    ([(20, ("intmodn", 64, G.M64), 48.0)], 0, 40, 20),
]


@pytest.mark.parametrize("levels,h,n_keys,npts", SUM_CASES, ids=str)
def test_evaluate_at_batch_sum(levels, h, n_keys, npts):
    import torch
    dpf, P, rng, batch, oks, _, _, _ = _setup(levels, n_keys, seed=n_keys + npts)
    vt = levels[h][1]
    pts = _rand_u128(rng, npts, levels[h][0])
    dev_batch = dpf.upload_key_batch(batch)
    size = dpf.packed_size(h)
    out = torch.empty(npts * size, dtype=torch.uint8, device="cuda")
    dpf.evaluate_at_batch_sum_to_device(dev_batch, h, _dev_points(pts), out)
    got = out.cpu().numpy().reshape(npts, size)
    want = O.evaluate_at(P, oks[0], h, pts)
    for k in range(1, n_keys):
        want = O.add_packed(vt, want, O.evaluate_at(P, oks[k], h, pts))
    np.testing.assert_array_equal(got, want)


def test_two_server_reconstruction_through_batch_sums():
    """Heavy-hitters style aggregation: the two servers' batch sums add up to
    the number of clients whose alpha equals each point (beta = 1)."""
    import torch
    levels = [(32, ("int", 64), 0)]
    dpf = make(levels)
    rng = np.random.default_rng(9)
    n = 512
    hot = [5, 77, 1 << 31]
    alphas = [hot[i % 3] if i % 4 else int(rng.integers(0, 1 << 32)) for i in range(n)]
    b0, b1 = dpf.generate_key_batch(alphas, [D.to_value(D.integer_type(64), 1)], threads=4)
    pts = hot + [6, 0, (1 << 32) - 1]
    sums = []
    for b in (b0, b1):
        out = torch.empty(len(pts) * 8, dtype=torch.uint8, device="cuda")
        dpf.evaluate_at_batch_sum_to_device(dpf.upload_key_batch(b), 0, _dev_points(pts), out)
        sums.append(out.cpu().numpy().view(np.uint64))
    total = (sums[0] + sums[1]).tolist()
    want = [sum(1 for a in alphas if a == p) for p in pts]
    assert total == want


def test_batch_range_upload_and_errors():
    import torch
    levels = [(20, ("int", 32), 0)]
    dpf, P, rng, batch, oks, _, _, _ = _setup(levels, 10, seed=1)
    pts = _rand_u128(rng, 8, 20)
    part = dpf.upload_key_batch(batch, 3, 7)
    assert (part.num_keys, part.first_key) == (4, 3)
    out = torch.empty(4 * 8 * 4, dtype=torch.uint8, device="cuda")
    dpf.evaluate_at_batch_to_device(part, 0, _dev_points(pts), 8, out, shared_points=True)
    got = out.cpu().numpy().reshape(4, 8, 4)
    for i in range(4):
        np.testing.assert_array_equal(got[i], O.evaluate_at(P, oks[3 + i], 0, pts))
    with pytest.raises(D.DpfStatusError) as e:
        dpf.evaluate_at_batch_to_device(part, 0, _dev_points([1 << 20]), 1, out, shared_points=True)
    assert e.value.code_name == "INVALID_ARGUMENT"
    with pytest.raises(D.DpfStatusError):
        dpf.evaluate_at_batch_to_device(part, 1, _dev_points(pts), 8, out)
    small = torch.empty(3, dtype=torch.uint8, device="cuda")
    with pytest.raises(D.DpfStatusError) as e:
        dpf.evaluate_at_batch_to_device(part, 0, _dev_points(pts), 8, small)
    assert e.value.message == "device output buffer too small"
    other = make([(21, ("int", 32), 0)])
    with pytest.raises(D.DpfStatusError) as e:
        other.evaluate_at_batch_to_device(part, 0, _dev_points(pts), 8, out)
    assert e.value.message == "key batch does not match this DistributedPointFunction"


ILP_CASES = [
    # (levels, keys, points per key): a quarter of the points a whole number of waves
    ([(128, ("int", 64), 0)], 6, 256),
    ([(40, ("int", 128), 0)], 3, 512),
    ([(64, ("xor", 128), 0)], 3, 256),
    ([(30, ("int", 8), 0)], 4, 256),                 # 16 elements per block
    ([(10, ("int", 16), 0), (50, ("int", 64), 0)], 4, 256),
    ([(7, ("int", 64), 0)], 2, 256),                 # 6 tree levels: all shared
    ([(6, ("int", 64), 0)], 2, 256),                 # 5: no shared top
]


@pytest.mark.parametrize("ilp", ["4", "4/full-walk", "4/shared-top", "2"])
@pytest.mark.parametrize("levels,n_keys,ppk", ILP_CASES, ids=str)
def test_points_kernel_chains_per_lane(levels, n_keys, ppk, ilp, monkeypatch):
    """Integer point evaluation with four path chains per lane
    (eval_points4_kernel, the default for launches that fill the chip; its top
    6 levels walked once per wave by default in the key sum, forced on or off
    for both forms with DPF_POINTS_SHARED_TOP=1|0) and with two (eval_points_kernel), forced through DPF_POINTS_ILP:
    per-key points, shared points and the key sum all equal the oracle, and the
    dispatch diagnostic names the kernel that ran."""
    import torch
    from distributed_point_functions_amd import hip_abi as H
    if "/" in ilp:
        ilp, walk = ilp.split("/")
        monkeypatch.setenv("DPF_POINTS_SHARED_TOP", "1" if walk == "shared-top" else "0")
    monkeypatch.setenv("DPF_POINTS_ILP", ilp)
    h = len(levels) - 1
    dpf, P, rng, batch, oks, _, _, _ = _setup(levels, n_keys, seed=ppk + int(ilp))
    vt, log = levels[h][1], levels[h][0]
    dev_batch = dpf.upload_key_batch(batch)
    size = dpf.packed_size(h)
    pts = _rand_u128(rng, n_keys * ppk, log)
    out = torch.empty(n_keys * ppk * size, dtype=torch.uint8, device="cuda")
    dpf.evaluate_at_batch_to_device(dev_batch, h, _dev_points(pts), ppk, out)
    torch.cuda.synchronize()
    assert H.last_points_kernel() == f"points/ilp{ilp}"
    got = out.cpu().numpy().reshape(n_keys * ppk, size)
    for k in range(n_keys):
        np.testing.assert_array_equal(got[k * ppk:(k + 1) * ppk],
                                      O.evaluate_at(P, oks[k], h, pts[k * ppk:(k + 1) * ppk]),
                                      err_msg=f"key {k}")
    shared = pts[:ppk]
    dpf.evaluate_at_batch_to_device(dev_batch, h, _dev_points(shared), ppk, out, shared_points=True)
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(n_keys, ppk, size)
    want = [O.evaluate_at(P, oks[k], h, shared) for k in range(n_keys)]
    for k in range(n_keys):
        np.testing.assert_array_equal(got[k], want[k])
    sums = torch.empty(ppk * size, dtype=torch.uint8, device="cuda")
    dpf.evaluate_at_batch_sum_to_device(dev_batch, h, _dev_points(shared), sums)
    torch.cuda.synchronize()
    assert H.last_points_kernel() == f"points/ilp{ilp}"
    total = want[0]
    for k in range(1, n_keys):
        total = O.add_packed(vt, total, want[k])
    np.testing.assert_array_equal(sums.cpu().numpy().reshape(ppk, size), total)


def test_points_kernel_default_dispatch():
    """Without the hook, a launch that fills every CU with 1024-thread
    workgroups takes four chains per lane; a smaller one takes two; one of at
    most num_cus x 256 points runs one lane quad per point."""
    import torch
    from distributed_point_functions_amd import hip_abi as H
    levels = [(64, ("int", 64), 0)]
    dpf, P, rng, batch, oks, _, _, _ = _setup(levels, 1024, seed=5)
    dev_batch = dpf.upload_key_batch(batch)
    pts = _rand_u128(rng, 1024, 64)
    out = torch.empty(1024 * 1024 * 8, dtype=torch.uint8, device="cuda")
    dpf.evaluate_at_batch_to_device(dev_batch, 0, _dev_points(pts), 1024, out, shared_points=True)
    torch.cuda.synchronize()
    assert H.last_points_kernel() == "points/ilp4"
    got = out.cpu().numpy().reshape(1024, 1024, 8)
    for k in (0, 1, 511, 1023):
        np.testing.assert_array_equal(got[k], O.evaluate_at(P, oks[k], 0, pts), err_msg=f"key {k}")
    # 512 keys x 256 points: more than one pass of lane quads over the chip
    # (num_cus x 256 points), less than a full chip of four-chain lanes.
    mid = torch.empty(512 * 256 * 8, dtype=torch.uint8, device="cuda")
    sub = dpf.upload_key_batch(batch, 0, 512)
    dpf.evaluate_at_batch_to_device(sub, 0, _dev_points(pts[:256]), 256, mid, shared_points=True)
    torch.cuda.synchronize()
    assert H.last_points_kernel() == "points/ilp2"
    got = mid.cpu().numpy().reshape(512, 256, 8)
    for k in (0, 511):
        np.testing.assert_array_equal(got[k], O.evaluate_at(P, oks[k], 0, pts[:256]), err_msg=f"key {k}")
    # 128 keys x 256 points: within one pass of quads, latency mode.
    small = torch.empty(128 * 256 * 8, dtype=torch.uint8, device="cuda")
    sub = dpf.upload_key_batch(batch, 0, 128)
    dpf.evaluate_at_batch_to_device(sub, 0, _dev_points(pts[:256]), 256, small, shared_points=True)
    torch.cuda.synchronize()
    assert H.last_points_kernel() == "points/quad"
    got = small.cpu().numpy().reshape(128, 256, 8)
    for k in (0, 127):
        np.testing.assert_array_equal(got[k], O.evaluate_at(P, oks[k], 0, pts[:256]), err_msg=f"key {k}")


QUAD_CASES = [
    ([(128, ("int", 64), 0)], 3, 100),
    ([(56, ("xor", 128), 0)], 2, 333),
    ([(40, ("int", 128), 0)], 5, 64),
    ([(30, ("int", 8), 0)], 4, 77),                  # 16 elements per block
    ([(10, ("int", 16), 0), (50, ("int", 32), 0)], 3, 50),
    ([(20, ("int", 64), 0)], 1, 1),
]


@pytest.mark.parametrize("quad", ["1", "0"])
@pytest.mark.parametrize("levels,n_keys,ppk", QUAD_CASES, ids=str)
def test_points_latency_mode(levels, n_keys, ppk, quad, monkeypatch):
    """Small integer point evaluations (at most num_cus x 256 points) run
    one (key, point) per lane quad, lane c computing AES column c
    (eval_points_quad_kernel); DPF_POINTS_QUAD=0 keeps one chain per lane.
    Per-key and shared points equal the oracle either way."""
    import torch
    from distributed_point_functions_amd import hip_abi as H
    monkeypatch.setenv("DPF_POINTS_QUAD", quad)
    h = len(levels) - 1
    dpf, P, rng, batch, oks, _, _, _ = _setup(levels, n_keys, seed=ppk + 17)
    dev_batch = dpf.upload_key_batch(batch)
    size = dpf.packed_size(h)
    pts = _rand_u128(rng, n_keys * ppk, levels[h][0])
    out = torch.empty(n_keys * ppk * size, dtype=torch.uint8, device="cuda")
    dpf.evaluate_at_batch_to_device(dev_batch, h, _dev_points(pts), ppk, out)
    torch.cuda.synchronize()
    assert H.last_points_kernel() == ("points/quad" if quad == "1" else "points/single")
    got = out.cpu().numpy().reshape(n_keys * ppk, size)
    for k in range(n_keys):
        np.testing.assert_array_equal(got[k * ppk:(k + 1) * ppk],
                                      O.evaluate_at(P, oks[k], h, pts[k * ppk:(k + 1) * ppk]),
                                      err_msg=f"key {k}")
    shared = pts[:ppk]
    dpf.evaluate_at_batch_to_device(dev_batch, h, _dev_points(shared), ppk, out, shared_points=True)
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(n_keys, ppk, size)
    for k in range(n_keys):
        np.testing.assert_array_equal(got[k], O.evaluate_at(P, oks[k], h, shared))
