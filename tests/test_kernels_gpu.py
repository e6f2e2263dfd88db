"""Parity of the gfx950 kernels (through the C ABI) against the CPU oracle.

Every comparison is bit-exact.  Inputs are seeded; sizes are small enough for
the oracle to finish in seconds.
"""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

KEY0 = 0
KEY1 = O.make_uint128(0x1111111111111111, 0x1111111111111111)
SEED0 = O.make_uint128(0x0123012301230123, 0x0123012301230123)
SEED1 = O.make_uint128(0x4567456745674567, 0x4567456745674567)


@pytest.fixture(scope="module")
def hip():
    import torch
    from distributed_point_functions_amd import hip_abi
    hip_abi.load(require_gpu=True)
    assert torch.cuda.is_available()
    return hip_abi


def _rand_blocks(rng, n):
    return rng.integers(0, 2**64, size=(n, 2), dtype=np.uint64)


def test_hash_known_answer(hip):
    # dpf/aes_128_fixed_key_hash_test.cc:114-135
    x = hip.to_device_blocks(O.blocks_from_ints([SEED0, SEED1]))
    out0 = O.ints_from_blocks(hip.blocks_to_numpy(hip.hash_blocks(x, KEY0)))
    out1 = O.ints_from_blocks(hip.blocks_to_numpy(hip.hash_blocks(x, KEY1)))
    assert out0 == [O.make_uint128(0x73C2DC14812BE4EF, 0xEAC64D09C8ADF8ED),
                    O.make_uint128(0xB8F33653A53A8436, 0xAEDF39B62DE91D95)]
    assert out1 == [O.make_uint128(0x934704AFF58FA233, 0xD3C20D1B9CC18D8F),
                    O.make_uint128(0x530098817046D284, 0x43E61D3273A04F7C)]


@pytest.mark.parametrize("n", [1, 63, 64, 1000, 300_001])
@pytest.mark.parametrize("key", [O.PRG_KEY_LEFT, O.PRG_KEY_RIGHT, O.PRG_KEY_VALUE])
def test_hash_random(hip, n, key):
    rng = np.random.default_rng(n)
    x = _rand_blocks(rng, n)
    got = hip.blocks_to_numpy(hip.hash_blocks(hip.to_device_blocks(x), key))
    np.testing.assert_array_equal(got, O.aes_hash(key, x))


def test_hash_in_place(hip):
    rng = np.random.default_rng(7)
    x = _rand_blocks(rng, 4097)
    d = hip.to_device_blocks(x)
    hip.hash_blocks(d, O.PRG_KEY_VALUE, out=d)
    np.testing.assert_array_equal(hip.blocks_to_numpy(d), O.aes_hash(O.PRG_KEY_VALUE, x))


def _hwy_test_inputs(num_seeds, num_levels):
    """Deterministic inputs of dpf/internal/evaluate_prg_hwy_test.cc:55-86."""
    seeds = O.blocks_from_ints([O.make_uint128(i, i + 1) for i in range(num_seeds)])
    paths = O.blocks_from_ints([O.make_uint128(23 * i + 42, 42 * i + 23) for i in range(num_seeds)])
    ctrl = np.array([1 if i % 7 == 0 else 0 for i in range(num_seeds)], np.uint8)
    cws = O.blocks_from_ints([O.make_uint128(i + 1, i) for i in range(num_levels)])
    cl = np.array([1 if i % 23 == 0 else 0 for i in range(num_levels)], np.uint8)
    cr = np.array([1 if i % 42 != 0 else 0 for i in range(num_levels)], np.uint8)
    return seeds, ctrl, paths, cws, cl, cr


@pytest.mark.parametrize("num_seeds", [1, 2, 101, 128, 1000])
@pytest.mark.parametrize("num_levels", [0, 1, 2, 32, 63, 64, 127])
def test_eval_paths_matches_reference_grid(hip, num_seeds, num_levels):
    seeds, ctrl, paths, cws, cl, cr = _hwy_test_inputs(num_seeds, num_levels)
    want_s, want_c = O.evaluate_seeds(seeds, ctrl, paths, cws, cl, cr, KEY0, KEY1)
    d = [hip.to_device_blocks(seeds), hip.to_device_u8(ctrl), hip.to_device_blocks(paths),
         hip.to_device_blocks(cws if len(cws) else np.zeros((1, 2), np.uint64)),
         hip.to_device_u8(cl if len(cl) else np.zeros(1, np.uint8)),
         hip.to_device_u8(cr if len(cr) else np.zeros(1, np.uint8))]
    import torch
    cl_t = d[4][:num_levels]
    cr_t = d[5][:num_levels]
    s, c = hip.eval_paths(d[0], d[1], d[2], d[3], cl_t, cr_t, KEY0, KEY1)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(hip.blocks_to_numpy(s), want_s)
    np.testing.assert_array_equal(c.cpu().numpy(), want_c)


@pytest.mark.parametrize("dynamic", ["1", "0"])
def test_hash_and_paths_full_launch(hip, dynamic, monkeypatch):
    """Launches large enough for dynamic 64-item chunks per wave (2^21 + a
    ragged tail) and, with DPF_HASH_DYNAMIC=0 / DPF_PATHS_DYNAMIC=0, the fixed
    grid-stride share: sampled rows (first, last, random) equal the oracle and
    the two distributions agree on every row."""
    import torch
    rng = np.random.default_rng(21)
    n = (1 << 21) + 5
    x = _rand_blocks(rng, n)
    d = hip.to_device_blocks(x)
    rows = np.unique(np.concatenate([[0, 63, 64, n - 1], rng.integers(0, n, size=512)]))
    got = {}
    for dyn in (dynamic, "1" if dynamic == "0" else "0"):
        monkeypatch.setenv("DPF_HASH_DYNAMIC", dyn)
        got[dyn] = hip.blocks_to_numpy(hip.hash_blocks(d, O.PRG_KEY_LEFT))
    np.testing.assert_array_equal(got["1"], got["0"])
    np.testing.assert_array_equal(got[dynamic][rows], O.aes_hash(O.PRG_KEY_LEFT, x[rows]))
    levels = 20
    paths = _rand_blocks(rng, n)
    ctrl = rng.integers(0, 2, size=n, dtype=np.uint8)
    cws = _rand_blocks(rng, levels)
    cl = rng.integers(0, 2, size=levels, dtype=np.uint8)
    cr = rng.integers(0, 2, size=levels, dtype=np.uint8)
    dev = [hip.to_device_blocks(x), hip.to_device_u8(ctrl), hip.to_device_blocks(paths),
           hip.to_device_blocks(cws), hip.to_device_u8(cl), hip.to_device_u8(cr)]
    res = {}
    for dyn in ("1", "0"):
        monkeypatch.setenv("DPF_PATHS_DYNAMIC", dyn)
        s, c = hip.eval_paths(*dev, KEY0, KEY1)
        torch.cuda.synchronize()
        res[dyn] = (hip.blocks_to_numpy(s), c.cpu().numpy())
    np.testing.assert_array_equal(res["1"][0], res["0"][0])
    np.testing.assert_array_equal(res["1"][1], res["0"][1])
    want_s, want_c = O.evaluate_seeds(x[rows[:64]], ctrl[rows[:64]], paths[rows[:64]], cws, cl, cr,
                                      KEY0, KEY1)
    np.testing.assert_array_equal(res[dynamic][0][rows[:64]], want_s)
    np.testing.assert_array_equal(res[dynamic][1][rows[:64]], want_c)


def _desc(hip, vt, b):
    return hip.value_desc(O.leaves(vt), O.is_direct(vt), O.elements_per_block(vt), b)


def _rand_value(rng, vt):
    out = []
    for kind, bits, mod in O.leaves(vt):
        if kind == O.LEAF_INTMODN:
            out.append(int(rng.integers(0, 2**62)) % mod)
        else:
            out.append(int.from_bytes(rng.bytes(bits // 8), "little"))
    return out


FAST_TYPES = [("int", 8), ("int", 16), ("int", 32), ("int", 64), ("int", 128),
              ("xor", 8), ("xor", 32), ("xor", 64), ("xor", 128)]
M32 = 4294967291
M64 = 18446744073709551557
M80 = O.make_uint128(65535, 18446744073709551551)
GENERIC_TYPES = [
    ("tuple", [("int", 32), ("int", 64)]),
    ("tuple", [("int", 8), ("int", 16), ("int", 32), ("int", 64)]),
    ("tuple", [("int", 32), ("tuple", [("int", 32), ("int", 32)]), ("int", 32)]),
    ("tuple", [("int", 32), ("int", 128)]),
    ("tuple", [("int", 32), ("int", 32)]),
    ("tuple", [("int", 8)]),
    ("intmodn", 32, M32),
    ("tuple", [("intmodn", 32, M32), ("intmodn", 32, M32)]),
    ("tuple", [("int", 32), ("intmodn", 32, M32)]),
    ("tuple", [("int", 128), ("intmodn", 32, M32)]),
    ("tuple", [("intmodn", 64, M64)] * 5),
    ("tuple", [("intmodn", 128, M80), ("intmodn", 128, M80)]),
    ("tuple", [("xor", 32), ("int", 128)]),
]


def _expand_case(hip, rng, vt, n0, levels, party, sec=48.0, cepb=None):
    b = (O.bits_needed(vt, sec) + 127) // 128
    E = O.elements_per_block(vt)
    cepb = cepb or E
    seeds = _rand_blocks(rng, n0)
    ctrl = rng.integers(0, 2, size=n0, dtype=np.uint8)
    cws = _rand_blocks(rng, max(levels, 1))
    cl = rng.integers(0, 2, size=max(levels, 1), dtype=np.uint8)
    cr = rng.integers(0, 2, size=max(levels, 1), dtype=np.uint8)
    vcw = [_rand_value(rng, vt) for _ in range(E)]
    es, ec = O.expand_seeds(seeds, ctrl, cws[:levels], cl[:levels], cr[:levels])
    want = O.hash_correct(vt, es, ec, b, cepb, vcw, party)
    import torch
    got = hip.expand(hip.to_device_blocks(seeds), hip.to_device_u8(ctrl),
                     hip.to_device_blocks(cws), hip.to_device_u8(cl)[:levels],
                     hip.to_device_u8(cr)[:levels],
                     (O.PRG_KEY_LEFT, O.PRG_KEY_RIGHT, O.PRG_KEY_VALUE), _desc(hip, vt, b), cepb,
                     hip.to_device_blocks(O._leaf_array(vcw)), party)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy().reshape(want.shape), want)


@pytest.mark.parametrize("vt", FAST_TYPES, ids=str)
@pytest.mark.parametrize("levels,n0", [(0, 1), (1, 1), (3, 2), (9, 1), (14, 1), (6, 37)])
@pytest.mark.parametrize("party", [0, 1])
def test_expand_fast_types(hip, vt, levels, n0, party):
    rng = np.random.default_rng(hash((str(vt), levels, n0, party)) & 0xFFFFFFFF)
    _expand_case(hip, rng, vt, n0, levels, party)


# The specialised full-domain leaves (dpf_hip_expand dispatch): uniform direct
# tuples as FastIntLeaf lanes, mixed-width direct tuples (incl. XorWrapper
# lanes) as SwarLeaf, tuples of IntModN32 as Mod32Leaf (Moller-Granlund
# sampling from 1 or 2 blocks, blocks_needed >= the blocks read) -- at a size
# where every lane runs whole subtrees, both parties.
SPECIALISED_TYPES = [
    ("tuple", [("int", 32), ("int", 32)]),
    ("tuple", [("int", 16), ("int", 16), ("int", 16)]),
    ("tuple", [("int", 32), ("int", 64)]),
    ("tuple", [("int", 8), ("int", 16), ("int", 32), ("int", 64)]),
    ("tuple", [("xor", 32), ("int", 32)]),
    ("tuple", [("int", 8), ("xor", 8)]),
    ("tuple", [("int", 64), ("xor", 64)]),
    ("intmodn", 32, M32),
    ("tuple", [("intmodn", 32, M32), ("intmodn", 32, M32)]),
    ("tuple", [("intmodn", 32, 65537)] * 3),
    ("tuple", [("intmodn", 32, 4294967295)] * 2),
    ("tuple", [("intmodn", 32, M32)] * 4),
    # Moduli below 2^31 (normalisation shifts in the Moller-Granlund division)
    # and 2^31 itself, on the octet kernel's Mod32Leaf<2> and the single leaf.
    ("tuple", [("intmodn", 32, 2147483647)] * 2),
    ("intmodn", 32, 3),
    ("tuple", [("intmodn", 32, 2147483648)] * 2),
    # Five IntModN32 leaves: the most that two hashed blocks can sample.
    ("tuple", [("intmodn", 32, M32)] * 5),
]


@pytest.mark.parametrize("vt", SPECIALISED_TYPES, ids=str)
@pytest.mark.parametrize("party", [0, 1])
@pytest.mark.parametrize("sec", [40.0, 64.0])
def test_expand_specialised_leaves(hip, vt, party, sec):
    rng = np.random.default_rng(hash((str(vt), party, sec)) & 0xFFFFFFFF)
    _expand_case(hip, rng, vt, 3, 17, party, sec=sec)


# The same types at octet-sized shapes: subtrees of >= 8 leaves per lane, so
# dpf_hip_expand dispatches expand_octet_kernel<Leaf> (FastIntLeaf lanes,
# SwarLeaf, Mod32Leaf<2>); both that launch and the pair kernel
# (DPF_EXPAND_NO_OCTET=1) must match the oracle, and the dispatch is checked.
# Expected launch per type: Tuple<uint16_t x3> stores 12-byte leaves and 3 or
# 4 (or 5) IntModN32 leaves use Mod32Leaf<5>, both on the pair kernel.
EXPECTED_KERNEL = ["octet/fast", "pair/fast", "octet/swar", "octet/swar", "octet/swar",
                   "octet/swar", "octet/swar", "octet/mod32", "octet/mod32", "pair/mod32",
                   "octet/mod32", "pair/mod32", "octet/mod32", "octet/mod32", "octet/mod32",
                   "pair/mod32"]


@pytest.mark.parametrize("i", range(len(SPECIALISED_TYPES)),
                         ids=[str(v) for v in SPECIALISED_TYPES])
@pytest.mark.parametrize("party", [0, 1])
@pytest.mark.parametrize("levels,n0", [(21, 1), (18, 5)])
def test_expand_specialised_leaves_octet(hip, i, party, levels, n0, monkeypatch):
    vt = SPECIALISED_TYPES[i]
    seed = hash((str(vt), party, levels, n0, "octet")) & 0xFFFFFFFF
    _expand_case(hip, np.random.default_rng(seed), vt, n0, levels, party, sec=40.0)
    name, depth = hip.last_expand_kernel()
    want = EXPECTED_KERNEL[i]
    assert name == want and depth >= 3, (name, depth)
    if want.startswith("octet/"):
        monkeypatch.setenv("DPF_EXPAND_NO_OCTET", "1")
        _expand_case(hip, np.random.default_rng(seed), vt, n0, levels, party, sec=40.0)
        assert hip.last_expand_kernel()[0] == "pair/" + want[6:]


# Small trees (<= one workgroup per CU, <= 11 levels below the workgroups'
# subtree roots) run expand_small_kernel: wave 0 walks to the subtree root
# in quads, the levels are expanded breadth-first through LDS (quads while a
# level has <= 256 parents, lanes above), the last level's two leaves per
# parent hashed side by side.  Every shape -- config 1's (one start, 19
# levels: 256 workgroups of 11 levels), one workgroup, several starts, leaves
# narrower than a block -- matches the oracle, reports "small/fast", and
# equals the general launch (DPF_EXPAND_SMALL=0) byte for byte.
@pytest.mark.parametrize("vt,levels,n0,cepb", [
    (("int", 64), 19, 1, None), (("xor", 128), 19, 1, None), (("int", 64), 11, 1, None),
    (("int", 32), 12, 3, None), (("int", 128), 8, 256, None), (("int", 8), 10, 2, 4),
    (("xor", 16), 1, 1, None), (("int", 64), 9, 200, 1)], ids=str)
@pytest.mark.parametrize("party", [0, 1])
def test_expand_small_trees(hip, vt, levels, n0, cepb, party, monkeypatch):
    seed = hash((str(vt), levels, n0, cepb, party, "small")) & 0xFFFFFFFF
    _expand_case(hip, np.random.default_rng(seed), vt, n0, levels, party, cepb=cepb)
    name, depth = hip.last_expand_kernel()
    assert name == "small/fast" and 1 <= depth <= 11, (name, depth)
    monkeypatch.setenv("DPF_EXPAND_SMALL", "0")
    _expand_case(hip, np.random.default_rng(seed), vt, n0, levels, party, cepb=cepb)
    assert not hip.last_expand_kernel()[0].startswith("small/")


# The small-tree launch takes the other leaf policies too (Leaf::emit2 for
# the last level): SwarLeaf, Mod32Leaf<2>, Mod32Leaf<5>.  GenericLeaf is not
# dispatched to it (spills there; measured no faster): "pair/generic".
@pytest.mark.parametrize("vt,want", [
    (("tuple", [("int", 8), ("xor", 8)]), "small/swar"),
    (("tuple", [("intmodn", 32, M32), ("intmodn", 32, M32)]), "small/mod32"),
    (("tuple", [("intmodn", 32, M32)] * 4), "small/mod32"),
    (("tuple", [("intmodn", 32, M32)] * 5), "small/mod32"),
    (("tuple", [("int", 32), ("int", 128)]), "pair/generic"),
    (("tuple", [("intmodn", 64, M64)] * 5), "pair/generic")], ids=str)
@pytest.mark.parametrize("levels,n0", [(12, 1), (9, 3)])
@pytest.mark.parametrize("party", [0, 1])
def test_expand_small_trees_all_leaves(hip, vt, want, levels, n0, party, monkeypatch):
    seed = hash((str(vt), levels, n0, party, "small-leaves")) & 0xFFFFFFFF
    _expand_case(hip, np.random.default_rng(seed), vt, n0, levels, party, sec=40.0)
    assert hip.last_expand_kernel()[0] == want
    monkeypatch.setenv("DPF_EXPAND_SMALL", "0")
    _expand_case(hip, np.random.default_rng(seed), vt, n0, levels, party, sec=40.0)
    assert not hip.last_expand_kernel()[0].startswith("small/")


# Start counts that are not powers of two: dpf_hip_expand picks the subtree
# depth by the per-thread critical path (5 starts x 2^21: depth 4, 5 * 2^17
# subtrees in 3 even rounds, where "fill the launch" gave depth 5 in 2 rounds).
@pytest.mark.parametrize("vt", [("int", 64), ("xor", 128), ("int", 32)], ids=str)
@pytest.mark.parametrize("levels,n0", [(21, 5), (19, 11)])
@pytest.mark.parametrize("party", [0, 1])
def test_expand_uneven_starts(hip, vt, levels, n0, party):
    rng = np.random.default_rng(hash((str(vt), levels, n0, party, "uneven")) & 0xFFFFFFFF)
    _expand_case(hip, rng, vt, n0, levels, party)


@pytest.mark.parametrize("vt,cepb", [(("int", 8), 1), (("int", 8), 4), (("int", 16), 2),
                                     (("int", 32), 1), (("int", 64), 1)], ids=str)
def test_expand_partial_blocks(hip, vt, cepb):
    # Small domains: fewer corrected elements than ElementsPerBlock (h:785-791).
    _expand_case(hip, np.random.default_rng(cepb), vt, 1, 5, 1, cepb=cepb)


@pytest.mark.parametrize("vt", GENERIC_TYPES, ids=str)
@pytest.mark.parametrize("party", [0, 1])
def test_expand_generic_types(hip, vt, party):
    rng = np.random.default_rng(len(str(vt)) * 7 + party)
    _expand_case(hip, rng, vt, 2, 7, party)


def _points_case(hip, rng, vt, num_keys, ppk, levels, sec=48.0, from_partials=False):
    b = (O.bits_needed(vt, sec) + 127) // 128
    E = O.elements_per_block(vt)
    n = num_keys * ppk
    key_seed = _rand_blocks(rng, num_keys)
    party = rng.integers(0, 2, size=num_keys, dtype=np.uint8)
    cws = _rand_blocks(rng, max(num_keys * levels, 1))
    cl = rng.integers(0, 2, size=max(num_keys * levels, 1), dtype=np.uint8)
    cr = rng.integers(0, 2, size=max(num_keys * levels, 1), dtype=np.uint8)
    tree = _rand_blocks(rng, n)
    if levels < 128:
        ints = [x & ((1 << levels) - 1) for x in O.ints_from_blocks(tree)]
        tree = O.blocks_from_ints(ints)
    bi = rng.integers(0, E, size=n, dtype=np.int32)
    vcws = [[_rand_value(rng, vt) for _ in range(E)] for _ in range(num_keys)]
    seeds_in = _rand_blocks(rng, n) if from_partials else None
    ctrl_in = rng.integers(0, 2, size=n, dtype=np.uint8) if from_partials else None
    want = []
    for k in range(num_keys):
        sl = slice(k * ppk, (k + 1) * ppk)
        if from_partials:
            s0, c0 = seeds_in[sl], ctrl_in[sl]
        else:
            s0 = np.repeat(key_seed[k:k + 1], ppk, axis=0)
            c0 = np.full(ppk, party[k], np.uint8)
        s, c = O.evaluate_seeds(s0, c0, tree[sl], cws[k * levels:(k + 1) * levels],
                                cl[k * levels:(k + 1) * levels], cr[k * levels:(k + 1) * levels])
        want.append(O.hash_select_correct(vt, s, c, b, bi[sl], vcws[k], int(party[k])))
    want = np.concatenate(want)
    import torch
    flat_vcw = O._leaf_array([e for v in vcws for e in v])
    got = hip.eval_points(n, ppk, levels, hip.to_device_blocks(key_seed), hip.to_device_u8(party),
                          hip.to_device_blocks(tree), torch.from_numpy(bi).cuda(),
                          hip.to_device_blocks(cws), hip.to_device_u8(cl), hip.to_device_u8(cr),
                          (O.PRG_KEY_LEFT, O.PRG_KEY_RIGHT, O.PRG_KEY_VALUE), _desc(hip, vt, b),
                          hip.to_device_blocks(flat_vcw),
                          seeds_in=hip.to_device_blocks(seeds_in) if from_partials else None,
                          ctrl_in=hip.to_device_u8(ctrl_in) if from_partials else None)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy()[: want.size].reshape(want.shape), want)


@pytest.mark.parametrize("vt", FAST_TYPES + GENERIC_TYPES[:4] + GENERIC_TYPES[6:9], ids=str)
def test_eval_points_single_key(hip, vt):
    _points_case(hip, np.random.default_rng(3), vt, 1, 777, 20)


@pytest.mark.parametrize("levels", [0, 1, 63, 64, 127])
def test_eval_points_many_keys(hip, levels):
    _points_case(hip, np.random.default_rng(levels), ("int", 64), 37, 64, levels)


def test_eval_points_from_partials(hip):
    _points_case(hip, np.random.default_rng(11), ("xor", 128), 5, 100, 12, from_partials=True)


# Either side of the launcher's pairing threshold (paired items < one wave per
# CU run unpaired; 256 CUs -> 16384 items = 32768 points of one key).
@pytest.mark.parametrize("vt,ppk", [(("int", 64), 32765), (("int", 64), 32767),
                                    (("xor", 128), 40001), (GENERIC_TYPES[0], 33001)], ids=str)
def test_eval_points_pairing_threshold(hip, vt, ppk):
    _points_case(hip, np.random.default_rng(ppk), vt, 1, ppk, 20)


# Ragged and wave-uniform point counts (P % 4 != 0, P < 4, P = 256, 1024),
# with and without partial-evaluation starts.
@pytest.mark.parametrize("vt,num_keys,ppk,levels,partials", [
    (("int", 64), 1, 777, 20, False), (("int", 64), 37, 64, 63, False),
    (("int", 64), 9, 256, 1, False), (("int", 32), 3, 1024, 30, False),
    (("int", 128), 5, 6, 127, False), (("xor", 128), 5, 100, 12, True),
    (("int", 8), 4, 5, 0, False), (("int", 16), 2, 3, 9, False),
    (("xor", 64), 11, 13, 40, True)], ids=str)
def test_eval_points_shapes(hip, vt, num_keys, ppk, levels, partials):
    _points_case(hip, np.random.default_rng(ppk * 31 + levels), vt, num_keys, ppk, levels,
                 from_partials=partials)


# Dynamic distribution in the octet kernel (dpf_kernels.hip octet_shape):
# launches with >= 4 items per thread of the chip take 2 or 4 levels off the
# subtrees and let each wave take 64 items at a time from its workgroup's
# counter.  At 2^26 leaves both shapes apply; every shape must give the
# static one-item-per-thread launch's bytes (DPF_OCTET_DYNAMIC=0), which the
# tests above and the full-size tests tie to the oracle.
@pytest.mark.parametrize("vt", [("int", 64), ("tuple", [("intmodn", 32, M32)] * 2),
                                ("tuple", [("int", 32), ("int", 64)])], ids=str)
def test_expand_octet_dynamic_shapes(hip, vt, monkeypatch):
    import torch
    rng = np.random.default_rng(hash((str(vt), "dyn")) & 0xFFFFFFFF)
    levels, party = 26, 1
    b = (O.bits_needed(vt, 40.0) + 127) // 128
    E = O.elements_per_block(vt)
    args = (hip.to_device_blocks(_rand_blocks(rng, 1)),
            hip.to_device_u8(rng.integers(0, 2, size=1, dtype=np.uint8)),
            hip.to_device_blocks(_rand_blocks(rng, levels)),
            hip.to_device_u8(rng.integers(0, 2, size=levels, dtype=np.uint8)),
            hip.to_device_u8(rng.integers(0, 2, size=levels, dtype=np.uint8)),
            (O.PRG_KEY_LEFT, O.PRG_KEY_RIGHT, O.PRG_KEY_VALUE), _desc(hip, vt, b), E,
            hip.to_device_blocks(O._leaf_array([_rand_value(rng, vt) for _ in range(E)])), party)
    monkeypatch.setenv("DPF_OCTET_DYNAMIC", "0")
    want = hip.expand(*args)
    assert hip.last_expand_kernel()[0].startswith("octet/")
    for mode in ("2", "4", ""):
        monkeypatch.setenv("DPF_OCTET_DYNAMIC", mode)
        got = hip.expand(*args)
        torch.cuda.synchronize()
        assert torch.equal(got, want), mode
        del got


# The pair-leaf kernel (expand_kernel: GenericLeaf types and DPF_EXPAND_NO_OCTET)
# takes the same dynamic shape (tree-top pass, 64-item chunks per wave); at
# 2^24 leaves every mode equals the static launch byte for byte.
@pytest.mark.parametrize("vt", [("int", 64), ("tuple", [("intmodn", 64, M64)] * 2)], ids=str)
def test_expand_pair_dynamic_shapes(hip, vt, monkeypatch):
    import torch
    rng = np.random.default_rng(hash((str(vt), "pairdyn")) & 0xFFFFFFFF)
    levels, party = 24, 0
    b = (O.bits_needed(vt, 40.0) + 127) // 128
    E = O.elements_per_block(vt)
    args = (hip.to_device_blocks(_rand_blocks(rng, 1)),
            hip.to_device_u8(rng.integers(0, 2, size=1, dtype=np.uint8)),
            hip.to_device_blocks(_rand_blocks(rng, levels)),
            hip.to_device_u8(rng.integers(0, 2, size=levels, dtype=np.uint8)),
            hip.to_device_u8(rng.integers(0, 2, size=levels, dtype=np.uint8)),
            (O.PRG_KEY_LEFT, O.PRG_KEY_RIGHT, O.PRG_KEY_VALUE), _desc(hip, vt, b), E,
            hip.to_device_blocks(O._leaf_array([_rand_value(rng, vt) for _ in range(E)])), party)
    monkeypatch.setenv("DPF_EXPAND_NO_OCTET", "1")
    monkeypatch.setenv("DPF_OCTET_DYNAMIC", "0")
    monkeypatch.setenv("DPF_EXPAND_TOP", "0")
    want = hip.expand(*args)
    assert hip.last_expand_kernel()[0].startswith("pair/")
    monkeypatch.delenv("DPF_EXPAND_TOP")
    for mode in ("0", "2", "4", ""):
        monkeypatch.setenv("DPF_OCTET_DYNAMIC", mode)
        got = hip.expand(*args)
        torch.cuda.synchronize()
        assert torch.equal(got, want), mode
        del got
