"""BASELINE.json's full-size configurations on one MI355X, checked through
size-independent properties (the oracle cannot produce 2^30+
outputs in a test's time):

* configs 2 and 3: both parties' full-domain outputs (2^30 uint64; one of the
  eight 2^31-output uint128 shards of the 2^34 domain) add up to beta exactly
  at alpha and to 0 everywhere else (distributed_point_function_test.cc's
  two-party property at full size), and sampled 2^12-output windows are
  bit-exact against the oracle's ExpandSeeds + HashExpandedSeeds;
* config 4: 2^20 keys x 2^10 shared points, summed over keys on the device for
  both parties: the shares reconstruct the number of keys hitting each point;
  and per key (2^30 outputs): planted hits reconstruct to beta, every other
  output to 0, four keys' rows bit-exact against the oracle;
* config 5b: one full heavy-hitters pass (2^20 clients, 61 levels, both
  servers) reconstructs the plaintext prefix histogram at every level.
"""
import numpy as np
import pytest

import oracle as O
from distributed_point_functions_amd import dpf as D
from distributed_point_functions_amd import proto as pb

pytestmark = pytest.mark.gpu
SIGN = -(1 << 63)


def _params(log, bits):
    p = pb.DpfParameters()
    p.log_domain_size = log
    p.value_type.CopyFrom(D.integer_type(bits))
    return p


def _oracle_key(key):
    return {"seed": D.u128_from_block(key.seed), "party": key.party,
            "cws": [(D.u128_from_block(c.seed), int(c.control_left), int(c.control_right), None)
                    for c in key.correction_words],
            "last_vc": [[D.from_value(D.integer_type(128), v)]
                        for v in key.last_level_value_correction]}


def _oracle_window(P, okey, start_leaf_block, depth_below, bits):
    """Outputs of the subtree of 2^depth_below leaf blocks starting at leaf block
    `start_leaf_block` (oracle EvaluateSeeds to its root, then expansion)."""
    T = P.hierarchy_to_tree[0]
    top = T - depth_below
    root = start_leaf_block >> depth_below
    s, c = O.evaluate_seeds(O.blocks_from_ints([okey["seed"]]), np.array([okey["party"]], np.uint8),
                            O.blocks_from_ints([root]), *O._cw_arrays(okey, 0, top))
    es, ec = O.expand_seeds(s, c, *O._cw_arrays(okey, top, T))
    vcw = O._value_correction(P, okey, 0)
    return O.hash_correct(("int", bits), es, ec, 1, P.cepb(0), vcw, okey["party"])


@pytest.mark.parametrize("log,bits,shard,num_shards", [(30, 64, 0, 1), (34, 128, 5, 8)],
                         ids=["config2_2^30_u64", "config3_shard5of8_2^34_u128"])
def test_full_domain_two_party_reconstruction(log, bits, shard, num_shards):
    import torch
    dpf = D.DistributedPointFunction.create(_params(log, bits))
    n = (1 << log) // num_shards
    lo = shard * n
    alpha = lo + 0x2B5E_9F31 % n          # inside this shard
    beta = (0xC0FFEE << 64 | 0x1234_5678_9ABC) if bits == 128 else 0xDEADBEEF12345
    k0, k1 = dpf.generate_keys_incremental(alpha, [D.to_value(D.integer_type(bits), beta)],
                                           seeds=(0x5EED0 + log, 0x5EED1 + log))
    words = bits // 64
    outs = []
    for k in (k0, k1):
        out = torch.empty(n * words, dtype=torch.int64, device="cuda")
        ctx = dpf.create_evaluation_context(k)
        assert dpf.evaluate_shard_to_device(0, shard, num_shards, ctx, out) == n
        outs.append(out.view(n, words))
    torch.cuda.synchronize()
    a, b = outs
    # (a + b) mod 2^bits, chunked: word 0 with carry into word 1 for uint128.
    hits = []
    chunk = 1 << 26
    for s in range(0, n, chunk):
        x, y = a[s:s + chunk], b[s:s + chunk]
        lo_sum = x[:, 0] + y[:, 0]
        nz = lo_sum != 0
        if words == 2:
            carry = ((lo_sum ^ SIGN) < (x[:, 0] ^ SIGN)).to(torch.int64)
            nz |= (x[:, 1] + y[:, 1] + carry) != 0
        idx = torch.nonzero(nz).flatten()
        hits += (idx + s).tolist()
    assert hits == [alpha - lo]
    i = alpha - lo
    got_lo = (int(a[i, 0]) + int(b[i, 0])) & ((1 << 64) - 1)
    if words == 2:
        tot = ((int(a[i, 1]) << 64 | (int(a[i, 0]) & ((1 << 64) - 1))) +
               (int(b[i, 1]) << 64 | (int(b[i, 0]) & ((1 << 64) - 1)))) & ((1 << 128) - 1)
        assert tot == beta
    else:
        assert got_lo == beta
    # Bit-exact windows against the oracle: shard start, alpha's window, shard end.
    P = O.OracleParams([(log, ("int", bits), 0)])
    cepb = P.cepb(0)
    okey = _oracle_key(k0)
    for start in (lo, (alpha // 4096) * 4096, lo + n - 4096):
        want = _oracle_window(P, okey, start // cepb, 12 - (cepb.bit_length() - 1), bits)
        got = a[start - lo:start - lo + 4096].cpu().numpy().view(np.uint8).reshape(4096, bits // 8)
        np.testing.assert_array_equal(got, want, err_msg=f"window at {start}")


def test_config4_batched_points_reconstruct_hit_counts():
    import torch
    dpf = D.DistributedPointFunction.create(_params(128, 64))
    n_keys, n_pts = 1 << 20, 1 << 10
    rng = np.random.default_rng(44)
    alphas = rng.integers(0, 2**64, size=(n_keys, 2), dtype=np.uint64)
    seeds = rng.integers(0, 2**64, size=(2 * n_keys, 2), dtype=np.uint64)
    pts = rng.integers(0, 2**64, size=(n_pts, 2), dtype=np.uint64)
    # Plant hits: point j < 16 equals the alpha of keys {j, j + 16, ...} for
    # j-dependent multiplicities.
    hits = np.zeros(n_pts, np.int64)
    for j in range(16):
        pts[j] = alphas[j]
        for r in range(j):
            alphas[1000 + 16 * r + j] = alphas[j]
        hits[j] = j + 1
    beta = D.to_value(D.integer_type(64), 3)
    b0, b1 = dpf.generate_key_batch(alphas, [beta], root_seeds=seeds, threads=16)
    dev_pts = torch.from_numpy(pts.view(np.int64)).cuda()
    sums = []
    for b in (b0, b1):
        out = torch.empty(n_pts * 8, dtype=torch.uint8, device="cuda")
        dpf.evaluate_at_batch_sum_to_device(dpf.upload_key_batch(b), 0, dev_pts, out)
        sums.append(out.cpu().numpy().view(np.uint64).astype(object))
    rec = [(int(x) + int(y)) % (1 << 64) for x, y in zip(*sums)]
    assert rec == [3 * int(h) for h in hits]


def test_config4_per_key_outputs_full_size():
    """Config 4 at full size, per-key outputs (EvaluateAtBatchToDevice): 2^20
    keys x 2^10 independent points each on the 2^128 domain.  Every key's
    alpha is planted at point slot k % 1024, so the two parties' 2^30 outputs
    add up to beta at exactly those 2^20 slots and to 0 at every other slot;
    four keys' 1024-point rows are bit-exact against the oracle's EvaluateAt."""
    import torch
    dpf = D.DistributedPointFunction.create(_params(128, 64))
    n_keys, ppk = 1 << 20, 1 << 10
    rng = np.random.default_rng(4444)
    alphas = rng.integers(0, 2**64, size=(n_keys, 2), dtype=np.uint64)
    seeds = rng.integers(0, 2**64, size=(2 * n_keys, 2), dtype=np.uint64)
    beta = 0x0123_4567_89AB_CDEF
    b0, b1 = dpf.generate_key_batch(alphas, [D.to_value(D.integer_type(64), beta)],
                                    root_seeds=seeds, threads=16)
    g = torch.Generator(device="cuda")
    g.manual_seed(4444)
    pts = torch.randint(-2**63, 2**63 - 1, (n_keys * ppk, 2), dtype=torch.int64, device="cuda",
                        generator=g)
    keys_idx = torch.arange(n_keys, device="cuda")
    slot = keys_idx * ppk + (keys_idx % ppk)
    pts[slot] = torch.from_numpy(alphas.view(np.int64)).cuda()
    outs = []
    for b in (b0, b1):
        out = torch.empty(n_keys * ppk, dtype=torch.int64, device="cuda")
        dpf.evaluate_at_batch_to_device(dpf.upload_key_batch(b), 0, pts, ppk, out)
        outs.append(out)
    torch.cuda.synchronize()
    s = outs[0] + outs[1]                  # mod 2^64 in int64
    assert int((s != 0).sum()) == n_keys
    assert bool((s[slot] == beta).all())
    host_pts = pts.view(n_keys, ppk, 2)
    for k in (0, 1, 123457, n_keys - 1):
        okey = _oracle_key(dpf.key_from_batch(b0, k))
        row = host_pts[k].cpu().numpy().view(np.uint64)
        want = O.evaluate_at(O.OracleParams([(128, ("int", 64), 0)]), okey, 0,
                             [int(a) | int(h) << 64 for a, h in row])
        got = outs[0][k * ppk:(k + 1) * ppk].cpu().numpy().view(np.uint8).reshape(ppk, 8)
        np.testing.assert_array_equal(got, want, err_msg=f"key {k}")


def test_config5b_heavy_hitters_full_size():
    """Config 5b at full size: 2^20 clients, the 61-level 128-bit hierarchy,
    Tuple<IntModN32 x 2>, top-1024 candidates per level, both servers, one
    full pass; at every level the two servers' key sums reconstruct the
    plaintext prefix histogram exactly (HH.verify)."""
    import torch
    from distributed_point_functions_amd import heavy_hitters as HH
    logs = HH.hierarchy()
    dpf = HH.create_dpf(logs)
    n_keys, top_k = 1 << 20, 1024
    values, idx, alphas = HH.client_values(n_keys, seed=0x5B)
    seeds = np.random.default_rng(0x5B5B).integers(0, 2**64, size=(2 * n_keys, 2), dtype=np.uint64)
    beta = D.to_value(HH.value_type(), HH.BETA)
    b0, b1 = dpf.generate_key_batch(alphas, [beta] * len(logs), root_seeds=seeds, threads=16)
    max_out = max(4 * top_k, 1 << logs[0])
    servers = [HH.Server(dpf, dpf.upload_key_batch(b), max_out, torch.device("cuda"))
               for b in (b0, b1)]
    rec = []
    final = HH.run(dpf, servers, logs, top_k=top_k, record=rec)
    assert len(rec) == len(logs) == 61
    HH.verify(rec, logs, values, idx)
    ref = HH.plaintext_prefix_counts(values, idx, 128)
    head = sorted(ref, key=lambda v: (-ref[v], v))[:8]
    assert set(head) <= set(final)
