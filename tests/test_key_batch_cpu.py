"""Key batches on the host (no GPU): SoA ingestion of DpfKeys, batched
multi-threaded key generation and the host-side share sum.  Row k of a
generated batch must be exactly the DpfKey the single-key keygen
(GenerateKeysIncrementalWithSeeds, distributed_point_function.cc:619-687)
produces for the same alpha and root seeds, which test_host_api_cpu pins to
the oracle."""
import numpy as np
import pytest

import oracle as O
import ref_grids as G
from distributed_point_functions_amd import dpf as D
from test_host_api_cpu import params, vt_from_oracle, leaves_value

MASK64 = (1 << 64) - 1

GRID = [
    [(128, ("int", 64), 0)],
    [(20, ("int", 8), 0)],
    [(16, ("xor", 128), 0)],
    [(5, ("int", 16), 0), (12, ("int", 64), 0), (40, ("int", 128), 0)],
    [(8, ("tuple", [("intmodn", 32, 4294967291)] * 2), 64.0),
     (16, ("tuple", [("intmodn", 32, 4294967291)] * 2), 64.0)],
    [(12, ("tuple", [("int", 32), ("intmodn", 64, G.M64)]), 48.0)],
]


def make(levels):
    dpf = D.DistributedPointFunction.create_incremental(params(levels))
    for _, vt, _ in levels:
        dpf.register_value_type(vt_from_oracle(vt))
    return dpf


def seeds_array(rng, n):
    return rng.integers(0, 1 << 63, size=(2 * n, 2), dtype=np.uint64)


def betas_for(levels, k=0):
    return [leaves_value(vt, [(k + 7 * h + 1) % 251 + 1] * len(O.leaves(vt)))
            for h, (_, vt, _) in enumerate(levels)]


@pytest.mark.parametrize("levels", GRID, ids=str)
def test_generate_key_batch_rows_equal_single_keygen(levels):
    dpf = make(levels)
    rng = np.random.default_rng(len(levels) * 7 + levels[-1][0])
    n = 37
    top = levels[-1][0]
    alphas = [int(rng.integers(0, 1 << 62)) % (1 << top) if top < 128 else
              (int(rng.integers(0, 1 << 62)) << 66) | int(rng.integers(0, 1 << 62)) for _ in range(n)]
    seeds = seeds_array(rng, n)
    beta = betas_for(levels)
    b0, b1 = dpf.generate_key_batch(alphas, beta, root_seeds=seeds, threads=3)
    assert b0.num_keys == n and b1.num_keys == n
    assert b0.num_levels == dpf.tree_levels_needed() - 1
    np.testing.assert_array_equal(b0.party(), np.zeros(n, np.uint8))
    np.testing.assert_array_equal(b1.party(), np.ones(n, np.uint8))
    for k in range(n):
        s0 = int(seeds[2 * k, 0]) | int(seeds[2 * k, 1]) << 64
        s1 = int(seeds[2 * k + 1, 0]) | int(seeds[2 * k + 1, 1]) << 64
        k0, k1 = dpf.generate_keys_incremental(alphas[k], beta, seeds=(s0, s1))
        assert dpf.key_from_batch(b0, k).SerializeToString() == k0.SerializeToString()
        assert dpf.key_from_batch(b1, k).SerializeToString() == k1.SerializeToString()


def test_generate_key_batch_thread_count_invariant():
    levels = GRID[3]
    dpf = make(levels)
    rng = np.random.default_rng(3)
    n = 1000
    alphas = [int(x) for x in rng.integers(0, 1 << 40, size=n)]
    seeds = seeds_array(rng, n)
    beta = betas_for(levels)
    ref = dpf.generate_key_batch(alphas, beta, root_seeds=seeds, threads=1)
    for t in (2, 7, 0):
        got = dpf.generate_key_batch(alphas, beta, root_seeds=seeds, threads=t)
        for a, b in zip(ref, got):
            np.testing.assert_array_equal(a.seeds(), b.seeds())
            for k in (0, 499, 999):
                assert (dpf.key_from_batch(a, k).SerializeToString() ==
                        dpf.key_from_batch(b, k).SerializeToString())


def test_generate_key_batch_random_seeds_differ():
    dpf = make(GRID[1])
    b0, b1 = dpf.generate_key_batch([1, 1], betas_for(GRID[1]))
    s = np.concatenate([b0.seeds(), b1.seeds()])
    assert len({tuple(r) for r in s.tolist()}) == 4


@pytest.mark.parametrize("levels", GRID, ids=str)
def test_make_key_batch_roundtrip(levels):
    dpf = make(levels)
    keys = []
    for k in range(5):
        a, b = dpf.generate_keys_incremental(k * 3 + 1, betas_for(levels, k), seeds=(10 + k, 20 + k))
        keys += [a, b]
    batch = dpf.make_key_batch(keys)
    assert batch.num_keys == len(keys)
    for k, key in enumerate(keys):
        assert dpf.key_from_batch(batch, k).SerializeToString() == key.SerializeToString()


def test_key_batch_errors():
    levels = GRID[1]
    dpf = make(levels)
    beta = betas_for(levels)
    with pytest.raises(D.DpfStatusError) as e:
        dpf.generate_key_batch([1 << 20], beta)
    assert e.value.message == "`alpha` must be smaller than the output domain size"
    with pytest.raises(D.DpfStatusError) as e:
        dpf.generate_key_batch([1, 2], beta, root_seeds=np.zeros((3, 2), np.uint64))
    assert e.value.code_name == "INVALID_ARGUMENT"
    with pytest.raises(D.DpfStatusError) as e:
        dpf.generate_key_batch([1], beta + beta)
    assert e.value.message == "`beta` has to have the same size as `parameters` passed at construction"
    batch, _ = dpf.generate_key_batch([1, 2], beta)
    with pytest.raises(D.DpfStatusError):
        dpf.key_from_batch(batch, 2)
    other = make(GRID[0])
    with pytest.raises(D.DpfStatusError) as e:
        other.key_from_batch(batch, 0)
    assert e.value.message == "key batch does not match this DistributedPointFunction"
    bad = dpf.generate_keys_incremental(1, beta)[0]
    del bad.correction_words[-1]
    with pytest.raises(D.DpfStatusError):
        dpf.make_key_batch([bad])


@pytest.mark.parametrize("vt", [("int", 64), ("int", 8), ("xor", 128),
                                ("tuple", [("intmodn", 32, 4294967291)] * 2),
                                ("tuple", [("int", 16), ("intmodn", 128, G.M80)])], ids=str)
def test_sum_packed_shares_matches_oracle_group_sum(vt):
    levels = [(10, vt, 48.0)]
    dpf = make(levels)
    rng = np.random.default_rng(11)
    size = O.packed_size(vt)
    num_shares, count = 5, 33
    # Valid group elements: reduce IntModN leaves below their modulus.
    vals = []
    for _ in range(num_shares * count):
        leaves = []
        for kind, bits, mod in O.leaves(vt):
            x = int(rng.integers(0, 1 << 62)) << 66 | int(rng.integers(0, 1 << 62))
            x &= (1 << bits) - 1
            if kind == "intmodn":
                x %= mod
            leaves.append(x)
        vals.append(O.pack_element(vt, leaves))
    shares = np.frombuffer(b"".join(vals), np.uint8).reshape(num_shares, count, size)
    got = dpf.sum_packed_shares(0, shares, num_shares, count).reshape(count, size)
    want = shares[0]
    for r in range(1, num_shares):
        want = O.add_packed(vt, want, shares[r])
    np.testing.assert_array_equal(got, want)


def test_parse_key_batch_matches_make_key_batch():
    # Batched ingestion of serialized keys == MakeKeyBatch of
    # the parsed protos, on several threads; the first bad key is reported.
    levels = [(10, ("int", 16), 0), (40, ("tuple", [("int", 32), ("intmodn", 64, G.M64)]), 48.0)]
    dpf = make(levels)
    rng = np.random.default_rng(4)
    alphas = [int(a) for a in rng.integers(0, 1 << 40, size=3000)]
    b0, _ = dpf.generate_key_batch(alphas, betas_for(levels), root_seeds=seeds_array(rng, 3000),
                                   threads=4)
    keys = [dpf.key_from_batch(b0, k) for k in range(3000)]
    parsed = dpf.parse_key_batch([k.SerializeToString() for k in keys], threads=4)
    made = dpf.make_key_batch(keys)
    assert np.array_equal(parsed.seeds(), made.seeds())
    for k in (0, 1234, 2999):
        assert dpf.key_from_batch(parsed, k) == keys[k]
    bad = [k.SerializeToString() for k in keys[:2500]]
    bad[1700] = b"\xff\xff\xff"
    with pytest.raises(D.DpfStatusError, match="Failed to parse DpfKey 1700"):
        dpf.parse_key_batch(bad, threads=4)


def test_serialize_key_batch_roundtrip():
    # SerializeKeyBatch (threaded egress) is byte-identical to serializing each
    # KeyFromBatch proto, and ParseKeyBatch of it restores the batch.
    levels = [(10, ("int", 16), 0), (40, ("tuple", [("int", 32), ("intmodn", 64, G.M64)]), 48.0)]
    dpf = make(levels)
    rng = np.random.default_rng(5)
    alphas = [int(a) for a in rng.integers(0, 1 << 40, size=2000)]
    b0, b1 = dpf.generate_key_batch(alphas, betas_for(levels), root_seeds=seeds_array(rng, 2000),
                                    threads=4)
    for b in (b0, b1):
        ser = dpf.serialize_key_batch(b, threads=4)
        assert len(ser) == 2000
        for k in (0, 999, 1999):
            assert ser[k] == dpf.key_from_batch(b, k).SerializeToString()
        back = dpf.parse_key_batch(ser, threads=4)
        assert np.array_equal(back.seeds(), b.seeds())
        assert dpf.serialize_key_batch(back, threads=1) == ser


def _varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _len_field(num, payload):
    return _varint(num << 3 | 2) + _varint(len(payload)) + payload


def _key_batch_fixture():
    levels = [(10, ("int", 16), 0)]
    dpf = make(levels)
    rng = np.random.default_rng(6)
    b0, _ = dpf.generate_key_batch([5, 77], betas_for(levels), root_seeds=seeds_array(rng, 2),
                                   threads=1)
    return dpf, [dpf.key_from_batch(b0, k) for k in range(2)]


def test_parse_rejects_deep_nesting():
    # A Value nested ~100k deep through tuples (a few hundred KB from an
    # untrusted client) is a clean parse error, not a stack overflow: the
    # parser stops at protobuf's default recursion limit of 100.
    dpf, keys = _key_batch_fixture()
    v = b""
    for _ in range(100_000):
        v = _len_field(2, _len_field(1, v))          # Value.tuple { elements: v }
    deep = keys[1].SerializeToString() + _len_field(5, v)
    with pytest.raises(D.DpfStatusError, match="Failed to parse DpfKey 1"):
        dpf.parse_key_batch([keys[0].SerializeToString(), deep], threads=1)
    # 60 levels of nesting (120 message levels) is past the limit as well,
    # while a shallow nested tuple still parses (then fails validation only).
    v = b""
    for _ in range(60):
        v = _len_field(2, _len_field(1, v))
    with pytest.raises(D.DpfStatusError, match="Failed to parse DpfKey 0"):
        dpf.parse_key_batch([keys[0].SerializeToString() + _len_field(5, v)], threads=1)


def test_parse_merges_repeated_singular_message():
    # A singular message field that occurs twice on the wire is merged, as
    # protobuf does: a second `seed` carrying only `low` keeps the first's `high`.
    from distributed_point_functions_amd import proto as pb
    dpf, keys = _key_batch_fixture()
    raw = keys[0].SerializeToString() + _len_field(1, _varint(2 << 3 | 0) + _varint(12345))
    want = pb.DpfKey()
    want.ParseFromString(raw)
    assert want.seed.low == 12345 and want.seed.high == keys[0].seed.high
    got = dpf.key_from_batch(dpf.parse_key_batch([raw], threads=1), 0)
    assert got == want
