"""CPU parity oracle -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg import this module.  The product package
(``distributed_point_functions_amd``) never imports it and has no CPU fallback.

Two layers:

* ``liboracle_dpf.so`` (``dpf_oracle.c``): the arithmetic hot loops restated in
  plain C on top of OpenSSL EVP AES-128-ECB (the reference drives the same EVP
  interface through BoringSSL, ``dpf/aes_128_fixed_key_hash.cc:38-40``).
* this file: the creation-time tree mapping and the incremental evaluation
  orchestration, restated in Python.  Each function cites the reference
  file:line it follows (paths relative to the reference repository root).

Pinning: the AES MMO hash is checked against the reference's known-answer
test (``dpf/aes_128_fixed_key_hash_test.cc:114-135``); conversions against the
reference's FromBytes examples; the full DPF against the reference's two-party
reconstruction property over its own parameter grids.  See ``tests/test_oracle.py``.

Value types are plain tuples:
  ("int", bits) | ("xor", bits) | ("intmodn", base_bits, modulus) | ("tuple", [vt, ...])
A 128-bit block is a Python int; arrays of blocks are numpy uint64 (n, 2)
arrays holding the absl::uint128 memory image {low, high}.
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import List, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

MAX_LEAVES = 64
LEAF_INT, LEAF_INTMODN, LEAF_XOR = 0, 1, 2
MASK64 = (1 << 64) - 1
MASK128 = (1 << 128) - 1


def make_uint128(high: int, low: int) -> int:
    return ((high & MASK64) << 64) | (low & MASK64)


# PRG keys, dpf/distributed_point_function.cc:37-42.
PRG_KEY_LEFT = make_uint128(0x5BE037CCF6A03DE5, 0x935F08D0A5B6A2FD)
PRG_KEY_RIGHT = make_uint128(0xEF94B6AEDEBB026C, 0xE2EA1FE0F66F4D0B)
PRG_KEY_VALUE = make_uint128(0x05A5D1588C5423E3, 0x46A31101B21D1C98)


def key_bytes(k: int) -> bytes:
    """Memory image of an absl::uint128 key (aes_128_fixed_key_hash.cc:38-40)."""
    return (k & MASK128).to_bytes(16, "little")


class _VType(ctypes.Structure):
    _fields_ = [
        ("num_leaves", ctypes.c_int32),
        ("direct", ctypes.c_int32),
        ("kind", ctypes.c_int32 * MAX_LEAVES),
        ("bits", ctypes.c_int32 * MAX_LEAVES),
        ("mod_lo", ctypes.c_uint64 * MAX_LEAVES),
        ("mod_hi", ctypes.c_uint64 * MAX_LEAVES),
    ]


class _Params(ctypes.Structure):
    _fields_ = [
        ("num_levels", ctypes.c_int32),
        ("tree_levels_needed", ctypes.c_int32),
        ("last_log_domain_size", ctypes.c_int32),
        ("log_domain_size", ctypes.c_int32 * 130),
        ("hierarchy_to_tree", ctypes.c_int32 * 130),
        ("blocks_needed", ctypes.c_int32 * 130),
    ]


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle_dpf.so")
        if not os.path.exists(path):
            raise RuntimeError(f"oracle not built: {path} (run `make -C oracle`)")
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        L.oracle_aes_hash.argtypes = [P, ctypes.c_int64, P, P]
        L.oracle_expand_seeds.argtypes = [P, P, ctypes.c_int64, P, P, ctypes.c_int, P, P, P, P, P]
        L.oracle_evaluate_seeds.argtypes = [P, P, ctypes.c_int64, ctypes.c_int, P, P, P, P, P, P, P, P]
        L.oracle_hash_correct.argtypes = [P, P, ctypes.c_int64, ctypes.c_int, ctypes.c_int, P, P, P,
                                          ctypes.c_int, P]
        L.oracle_hash_select_correct.argtypes = [P, P, ctypes.c_int64, ctypes.c_int, P, P, P, P,
                                                 ctypes.c_int, P]
        L.oracle_add_packed.argtypes = [P, ctypes.c_int64, P, P, P]
        L.oracle_convert_bytes.argtypes = [P, P, P]
        L.oracle_elements_per_block.argtypes = [P]
        L.oracle_packed_element_size.argtypes = [P]
        U = ctypes.c_uint64
        L.oracle_generate_keys.argtypes = [P, P, P, P, P, U, U, P, U, U, U, U, P, P, P, P]
        I64 = ctypes.c_int64
        L.baseline_evaluate_at_u64.argtypes = [P, P, P, I64, I64, ctypes.c_int, ctypes.c_int, P, P,
                                               P, P, P, I64, P, P, P]
        _LIB = L
    return _LIB


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _u128_args(x: int):
    return (x & MASK64, (x >> 64) & MASK64)


def blocks_from_ints(xs: Sequence[int]) -> np.ndarray:
    a = np.zeros((len(xs), 2), dtype=np.uint64)
    for i, x in enumerate(xs):
        a[i, 0] = x & MASK64
        a[i, 1] = (x >> 64) & MASK64
    return a


def ints_from_blocks(a: np.ndarray) -> List[int]:
    return [int(lo) | (int(hi) << 64) for lo, hi in a]


def baseline_evaluate_at_u64(L: int, bib: int, key_seed: np.ndarray, party: np.ndarray,
                             cw_seed: np.ndarray, cw_left: np.ndarray, cw_right: np.ndarray,
                             vcw: np.ndarray, points: np.ndarray) -> np.ndarray:
    """bench.py's CPU baseline for batched EvaluateAt<uint64_t> (cpu_baseline.c:
    the reference's one-AES-per-level path walk on AES-NI, 8 points
    interleaved).  key_seed (K, 2) u64 blocks, party (K,) u8, cw_* (K, L) rows,
    vcw (K, 2, 2) u64 blocks (two elements), points (K, P, 2) u64 blocks.
    Releases the GIL (ctypes), so host threads run it in parallel."""
    K, Pn = points.shape[0], points.shape[1]
    out = np.empty((K, Pn), np.uint64)
    args = [np.ascontiguousarray(a) for a in (key_seed, party, cw_seed, cw_left, cw_right, vcw,
                                               points)]
    lib().baseline_evaluate_at_u64(key_bytes(PRG_KEY_LEFT), key_bytes(PRG_KEY_RIGHT),
                                   key_bytes(PRG_KEY_VALUE), K, Pn, L, bib,
                                   *[_ptr(a) for a in args[:5]], cw_seed.shape[1],
                                   _ptr(args[5]), _ptr(args[6]), _ptr(out))
    return out


# --------------------------------------------------------------------------
# Value types (dpf/internal/value_type_helpers.{h,cc}, dpf/int_mod_n.cc)
# --------------------------------------------------------------------------

def leaves(vt) -> List[tuple]:
    """Flatten a value type into (kind, bits, modulus) leaves in order."""
    k = vt[0]
    if k == "int":
        return [(LEAF_INT, vt[1], 0)]
    if k == "xor":
        return [(LEAF_XOR, vt[1], 0)]
    if k == "intmodn":
        return [(LEAF_INTMODN, vt[1], vt[2])]
    if k == "tuple":
        out = []
        for e in vt[1]:
            out += leaves(e)
        return out
    raise ValueError(vt)


def is_direct(vt) -> bool:
    return all(l[0] != LEAF_INTMODN for l in leaves(vt))


def total_bits(vt) -> int:
    return sum(l[1] for l in leaves(vt))


def elements_per_block(vt) -> int:
    """ElementsPerBlock<T>() (value_type_helpers.h:508-520)."""
    if not is_direct(vt):
        return 1
    tb = total_bits(vt)
    return 128 // tb if tb <= 128 else 1


def packed_size(vt) -> int:
    return sum(l[1] // 8 for l in leaves(vt))


def to_cvtype(vt) -> _VType:
    ls = leaves(vt)
    if len(ls) > MAX_LEAVES:
        raise ValueError("too many leaves")
    c = _VType()
    c.num_leaves = len(ls)
    c.direct = 1 if is_direct(vt) else 0
    for i, (kind, bits, mod) in enumerate(ls):
        c.kind[i] = kind
        c.bits[i] = bits
        c.mod_lo[i] = mod & MASK64
        c.mod_hi[i] = (mod >> 64) & MASK64
    return c


def _security_level(num_samples: int, modulus: int) -> float:
    # IntModNBase::GetSecurityLevel (dpf/int_mod_n.cc:21-26)
    return 128 + 3 - (math.log2(float(modulus)) + math.log2(float(num_samples)) +
                      math.log2(float(num_samples + 1)))


def _num_bytes_required(num_samples: int, base_bits: int, modulus: int, sec: float) -> int:
    # IntModNBase::CheckParameters + GetNumBytesRequired (dpf/int_mod_n.cc:28-78)
    if num_samples <= 0 or base_bits <= 0 or base_bits > 128:
        raise ValueError("invalid IntModN parameters")
    if base_bits < 128 and (1 << base_bits) < modulus:
        raise ValueError("modulus out of range")
    sigma = _security_level(num_samples, modulus)
    if sec > sigma:
        raise ValueError(f"insufficient statistical security: {sigma}")
    return 16 + ((base_bits + 7) // 8) * (num_samples - 1)


def bits_needed(vt, sec: float) -> int:
    """BitsNeeded (value_type_helpers.cc:60-130), including its quirk of
    recursing into the *first* num_other tuple elements (:94-103)."""
    k = vt[0]
    if k in ("int", "xor"):
        return vt[1]
    if k == "intmodn":
        return 8 * _num_bytes_required(1, vt[1], vt[2], sec)
    if k == "tuple":
        els = vt[1]
        mods = [e for e in els if e[0] == "intmodn"]
        num_other = len(els) - len(mods)
        if mods and any((m[1], m[2]) != (mods[0][1], mods[0][2]) for m in mods):
            raise NotImplementedError("All elements of type IntModN in a tuple must be the same")
        bits_other = 0
        for i in range(num_other):
            bits_other += bits_needed(els[i], sec + math.log2(float(num_other)))
        bits_mod = 0
        if mods:
            bits_mod = 8 * _num_bytes_required(len(mods), mods[0][1], mods[0][2], sec)
        return bits_mod + bits_other
    raise ValueError(vt)


# --------------------------------------------------------------------------
# Parameters / tree mapping (dpf/internal/proto_validator.cc:97-142)
# --------------------------------------------------------------------------

class OracleParams:
    def __init__(self, params: Sequence[Tuple[int, tuple, float]]):
        """params: [(log_domain_size, value_type, security_parameter or 0)]."""
        self.log_domain = [p[0] for p in params]
        self.vtypes = [p[1] for p in params]
        # default security parameter 40 + log_domain (proto_validator.cc:27-30, 104-109)
        self.sec = [(p[2] if p[2] else 40.0 + p[0]) for p in params]
        self.hierarchy_to_tree = []
        tln = 0
        for i in range(len(params)):
            bn = bits_needed(self.vtypes[i], self.sec[i])
            lb = int(math.ceil(math.log2(bn)))
            tl = max(tln, self.log_domain[i] - 7 + min(lb, 7))
            self.hierarchy_to_tree.append(tl)
            tln = max(tln, tl + 1)
        self.tree_levels_needed = tln
        # blocks_needed (distributed_point_function.cc:578-587)
        self.blocks_needed = [(bits_needed(self.vtypes[i], self.sec[i]) + 127) // 128
                              for i in range(len(params))]
        self.cvtypes = [to_cvtype(v) for v in self.vtypes]

    def cparams(self) -> _Params:
        c = _Params()
        c.num_levels = len(self.log_domain)
        c.tree_levels_needed = self.tree_levels_needed
        c.last_log_domain_size = self.log_domain[-1]
        for i in range(len(self.log_domain)):
            c.log_domain_size[i] = self.log_domain[i]
            c.hierarchy_to_tree[i] = self.hierarchy_to_tree[i]
            c.blocks_needed[i] = self.blocks_needed[i]
        return c

    def cepb(self, h: int) -> int:
        # corrected_elements_per_block (distributed_point_function.h:785-787)
        return 1 << (self.log_domain[h] - self.hierarchy_to_tree[h])


# --------------------------------------------------------------------------
# Thin wrappers over the C restatement
# --------------------------------------------------------------------------

def aes_hash(key: int, blocks: np.ndarray) -> np.ndarray:
    blocks = np.ascontiguousarray(blocks, dtype=np.uint64).reshape(-1, 2)
    out = np.zeros_like(blocks)
    kb = key_bytes(key)
    st = lib().oracle_aes_hash(kb, len(blocks), _ptr(blocks), _ptr(out))
    assert st == 0
    return out


def expand_seeds(seeds: np.ndarray, ctrl: np.ndarray, cw_seeds: np.ndarray,
                 cw_cl: np.ndarray, cw_cr: np.ndarray,
                 key_left: int = PRG_KEY_LEFT, key_right: int = PRG_KEY_RIGHT):
    seeds = np.ascontiguousarray(seeds, dtype=np.uint64).reshape(-1, 2)
    ctrl = np.ascontiguousarray(ctrl, dtype=np.uint8)
    L = len(cw_cl)
    n0 = len(seeds)
    so = np.zeros((n0 << L, 2), dtype=np.uint64)
    co = np.zeros(n0 << L, dtype=np.uint8)
    cws = np.ascontiguousarray(cw_seeds, dtype=np.uint64).reshape(-1, 2)
    cl = np.ascontiguousarray(cw_cl, dtype=np.uint8)
    cr = np.ascontiguousarray(cw_cr, dtype=np.uint8)
    st = lib().oracle_expand_seeds(key_bytes(key_left), key_bytes(key_right), n0, _ptr(seeds),
                                   _ptr(ctrl), L, _ptr(cws), _ptr(cl), _ptr(cr), _ptr(so), _ptr(co))
    assert st == 0
    return so, co


def evaluate_seeds(seeds: np.ndarray, ctrl: np.ndarray, paths: np.ndarray,
                   cw_seeds: np.ndarray, cw_cl: np.ndarray, cw_cr: np.ndarray,
                   key_left: int = PRG_KEY_LEFT, key_right: int = PRG_KEY_RIGHT):
    seeds = np.ascontiguousarray(seeds, dtype=np.uint64).reshape(-1, 2)
    ctrl = np.ascontiguousarray(ctrl, dtype=np.uint8)
    paths = np.ascontiguousarray(paths, dtype=np.uint64).reshape(-1, 2)
    n = len(seeds)
    L = len(cw_cl)
    so = np.zeros((n, 2), dtype=np.uint64)
    co = np.zeros(n, dtype=np.uint8)
    cws = np.ascontiguousarray(cw_seeds, dtype=np.uint64).reshape(-1, 2)
    if cws.size == 0:
        cws = np.zeros((1, 2), dtype=np.uint64)
    cl = np.ascontiguousarray(cw_cl, dtype=np.uint8)
    cr = np.ascontiguousarray(cw_cr, dtype=np.uint8)
    if cl.size == 0:
        cl = np.zeros(1, np.uint8)
        cr = np.zeros(1, np.uint8)
    st = lib().oracle_evaluate_seeds(key_bytes(key_left), key_bytes(key_right), n, L, _ptr(seeds),
                                     _ptr(ctrl), _ptr(paths), _ptr(cws), _ptr(cl), _ptr(cr),
                                     _ptr(so), _ptr(co))
    assert st == 0
    return so, co


def _leaf_array(values: Sequence[Sequence[int]]) -> np.ndarray:
    flat = [x for el in values for x in el]
    return blocks_from_ints(flat) if flat else np.zeros((1, 2), np.uint64)


def hash_correct(vt, seeds: np.ndarray, ctrl: np.ndarray, b: int, cepb: int,
                 cw_elems: Sequence[Sequence[int]], party: int) -> np.ndarray:
    """HashExpandedSeeds + correction loop; returns packed bytes (n*cepb, size)."""
    cv = to_cvtype(vt)
    seeds = np.ascontiguousarray(seeds, dtype=np.uint64).reshape(-1, 2)
    ctrl = np.ascontiguousarray(ctrl, dtype=np.uint8)
    n = len(seeds)
    ps = packed_size(vt)
    out = np.zeros(max(n * cepb * ps, 1), dtype=np.uint8)
    cw = _leaf_array(cw_elems)
    st = lib().oracle_hash_correct(key_bytes(PRG_KEY_VALUE), ctypes.byref(cv), n, b, cepb,
                                   _ptr(seeds), _ptr(ctrl), _ptr(cw), party, _ptr(out))
    assert st == 0
    return out[: n * cepb * ps].reshape(n * cepb, ps)


def hash_select_correct(vt, seeds: np.ndarray, ctrl: np.ndarray, b: int,
                        block_index: Sequence[int], cw_elems, party: int) -> np.ndarray:
    cv = to_cvtype(vt)
    seeds = np.ascontiguousarray(seeds, dtype=np.uint64).reshape(-1, 2)
    ctrl = np.ascontiguousarray(ctrl, dtype=np.uint8)
    n = len(seeds)
    ps = packed_size(vt)
    out = np.zeros(max(n * ps, 1), dtype=np.uint8)
    bi = np.ascontiguousarray(block_index, dtype=np.int32)
    if bi.size == 0:
        bi = np.zeros(1, np.int32)
    cw = _leaf_array(cw_elems)
    st = lib().oracle_hash_select_correct(key_bytes(PRG_KEY_VALUE), ctypes.byref(cv), n, b,
                                          _ptr(seeds), _ptr(ctrl), _ptr(bi), _ptr(cw), party,
                                          _ptr(out))
    assert st == 0
    return out[: n * ps].reshape(n, ps)


def add_packed(vt, a: np.ndarray, b: np.ndarray) -> np.ndarray:
    cv = to_cvtype(vt)
    a = np.ascontiguousarray(a, dtype=np.uint8)
    b = np.ascontiguousarray(b, dtype=np.uint8)
    ps = packed_size(vt)
    n = a.size // ps
    out = np.zeros(max(a.size, 1), dtype=np.uint8)
    lib().oracle_add_packed(ctypes.byref(cv), n, _ptr(a), _ptr(b), _ptr(out))
    return out[: a.size].reshape(n, ps)


def convert_bytes(vt, data: bytes) -> List[List[int]]:
    """ConvertBytesToArrayOf<T> on raw bytes (value_type_helpers.h:569-589)."""
    cv = to_cvtype(vt)
    E = elements_per_block(vt)
    nl = len(leaves(vt))
    buf = np.zeros(max(len(data), 16 * 16), dtype=np.uint8)
    buf[: len(data)] = np.frombuffer(data, dtype=np.uint8)
    out = np.zeros((E * nl, 2), dtype=np.uint64)
    lib().oracle_convert_bytes(ctypes.byref(cv), _ptr(buf), _ptr(out))
    ints = ints_from_blocks(out)
    return [ints[i * nl:(i + 1) * nl] for i in range(E)]


def pack_element(vt, leaves_vals: Sequence[int]) -> bytes:
    out = b""
    for (kind, bits, _), v in zip(leaves(vt), leaves_vals):
        out += (v & ((1 << bits) - 1)).to_bytes(bits // 8, "little")
    return out


def unpack_elements(vt, packed: np.ndarray) -> List[List[int]]:
    ls = leaves(vt)
    res = []
    for row in np.asarray(packed, dtype=np.uint8).reshape(-1, packed_size(vt)):
        off = 0
        el = []
        raw = row.tobytes()
        for (_, bits, _) in ls:
            w = bits // 8
            el.append(int.from_bytes(raw[off:off + w], "little"))
            off += w
        res.append(el)
    return res


# --------------------------------------------------------------------------
# Keys and evaluation contexts as plain dicts
# --------------------------------------------------------------------------

def generate_keys(P: OracleParams, alpha: int, betas: Sequence[Sequence[int]],
                  seed0: int, seed1: int):
    """GenerateKeysIncremental (distributed_point_function.cc:619-687) with
    injected root seeds.  betas[h] = leaves of beta at hierarchy level h.
    Returns two key dicts {seed, party, cws=[(seed, cl, cr, vc or None)], last_vc}."""
    T = P.tree_levels_needed
    H = len(P.log_domain)
    ncw = max(T - 1, 1)
    cws = np.zeros((ncw, 2), dtype=np.uint64)
    cl = np.zeros(ncw, dtype=np.uint8)
    cr = np.zeros(ncw, dtype=np.uint8)
    nvc = sum(elements_per_block(P.vtypes[h]) * len(leaves(P.vtypes[h])) for h in range(H))
    vc = np.zeros((nvc, 2), dtype=np.uint64)
    flat_beta = [x for b in betas for x in b]
    ba = blocks_from_ints(flat_beta) if flat_beta else np.zeros((1, 2), np.uint64)
    cvt = (_VType * H)(*P.cvtypes)
    cp = P.cparams()
    st = lib().oracle_generate_keys(key_bytes(PRG_KEY_LEFT), key_bytes(PRG_KEY_RIGHT),
                                    key_bytes(PRG_KEY_VALUE), ctypes.byref(cp), cvt,
                                    *_u128_args(alpha), _ptr(ba), *_u128_args(seed0),
                                    *_u128_args(seed1), _ptr(cws), _ptr(cl), _ptr(cr), _ptr(vc))
    assert st == 0, st
    vc_ints = ints_from_blocks(vc)
    vcs = []
    off = 0
    for h in range(H):
        E = elements_per_block(P.vtypes[h])
        nl = len(leaves(P.vtypes[h]))
        vcs.append([vc_ints[off + i * nl: off + (i + 1) * nl] for i in range(E)])
        off += E * nl
    cw_list = []
    cw_seed_ints = ints_from_blocks(cws)
    for i in range(T - 1):
        v = None
        for h in range(H - 1):
            if P.hierarchy_to_tree[h] == i:
                v = vcs[h]
        cw_list.append((cw_seed_ints[i], int(cl[i]), int(cr[i]), v))
    keys = []
    for party, seed in ((0, seed0), (1, seed1)):
        keys.append({"seed": seed, "party": party, "cws": cw_list, "last_vc": vcs[H - 1]})
    return keys[0], keys[1]


def _cw_arrays(key, start: int, stop: int):
    cws = key["cws"][start:stop]
    s = blocks_from_ints([c[0] for c in cws]) if cws else np.zeros((0, 2), np.uint64)
    return s, np.array([c[1] for c in cws], np.uint8), np.array([c[2] for c in cws], np.uint8)


def _value_correction(P: OracleParams, key, h: int):
    # distributed_point_function.h:763-780
    if h < len(P.log_domain) - 1:
        v = key["cws"][P.hierarchy_to_tree[h]][3]
    else:
        v = key["last_vc"]
    if v is None or len(v) != elements_per_block(P.vtypes[h]):
        raise ValueError("value correction size does not match ElementsPerBlock")
    return v


def create_context(P: OracleParams, key):
    # CreateEvaluationContext (distributed_point_function.cc:689-704)
    return {"key": key, "prev": -1, "partials": [], "partials_level": 0}


def _compute_partial_evaluations(P, prefixes, h, update_ctx, ctx):
    """ComputePartialEvaluations (distributed_point_function.cc:351-453)."""
    key = ctx["key"]
    start = P.hierarchy_to_tree[ctx["partials_level"]]
    stop = P.hierarchy_to_tree[h]
    n = len(prefixes)
    if ctx["partials"] and start <= stop:
        prev = {}
        for (pfx, seed, c) in ctx["partials"]:
            if pfx in prev and prev[pfx] != (seed, c):
                raise ValueError("Duplicate prefix in `ctx.partial_evaluations()` with "
                                 "mismatching seed or control bit")
            prev.setdefault(pfx, (seed, c))
        seeds, ctrl = [], []
        for p in prefixes:
            pp = p >> (stop - start) if stop - start < 128 else 0
            if pp not in prev:
                raise ValueError("Prefix not present in ctx.partial_evaluations at "
                                 f"hierarchy level {h}")
            seeds.append(prev[pp][0])
            ctrl.append(prev[pp][1])
    else:
        seeds = [key["seed"]] * n
        ctrl = [key["party"]] * n
        start = 0
    s_arr, c_arr = evaluate_seeds(blocks_from_ints(seeds), np.array(ctrl, np.uint8),
                                  blocks_from_ints(list(prefixes)), *_cw_arrays(key, start, stop))
    ctx["partials"] = []
    if update_ctx:
        sl = ints_from_blocks(s_arr)
        ctx["partials"] = [(prefixes[i], sl[i], int(c_arr[i])) for i in range(n)]
    ctx["partials_level"] = h
    return s_arr, c_arr


def evaluate_until(P: OracleParams, h: int, prefixes: Sequence[int], ctx) -> np.ndarray:
    """EvaluateUntil<T> (distributed_point_function.h:641-837) on the oracle.
    Returns packed elements (num_outputs, packed_size)."""
    key = ctx["key"]
    H = len(P.log_domain)
    if h < 0 or h >= H:
        raise ValueError("`hierarchy_level` must be non-negative and less than parameters_.size()")
    if h <= ctx["prev"]:
        raise ValueError("`hierarchy_level` must be greater than `ctx.previous_hierarchy_level`")
    if (ctx["prev"] < 0) != (len(prefixes) == 0):
        raise ValueError("`prefixes` must be empty if and only if this is the first call with `ctx`.")
    prev_h = ctx["prev"]
    prev_log = 0
    if prefixes:
        prev_log = P.log_domain[prev_h]
        for p in prefixes:
            if prev_log < 128 and p >= (1 << prev_log):
                raise ValueError(f"Index {p} out of range for hierarchy level {prev_h}")
    log = P.log_domain[h]
    if log - prev_log > 62:
        raise ValueError("Output size would be larger than 2**62. Please evaluate fewer "
                         "hierarchy levels at once.")
    # prefix dedup (h:718-742)
    tree_indices, inverse, prefix_map = [], {}, []
    for p in prefixes:
        bib = P.log_domain[prev_h] - P.hierarchy_to_tree[prev_h]
        ti, bi = p >> bib, p & ((1 << bib) - 1)
        if ti not in inverse:
            inverse[ti] = len(tree_indices)
            tree_indices.append(ti)
        prefix_map.append((inverse[ti], bi))
    vc = _value_correction(P, key, h)
    # ExpandAndUpdateContext (cc:455-498)
    if not tree_indices:
        seeds = blocks_from_ints([key["seed"]])
        ctrl = np.array([key["party"]], np.uint8)
        start = 0
    else:
        update = h < H - 1
        seeds, ctrl = _compute_partial_evaluations(P, tree_indices, prev_h, update, ctx)
        start = P.hierarchy_to_tree[prev_h]
    stop = P.hierarchy_to_tree[h]
    es, ec = expand_seeds(seeds, ctrl, *_cw_arrays(key, start, stop))
    ctx["prev"] = h
    cepb = P.cepb(h)
    corrected = hash_correct(P.vtypes[h], es, ec, P.blocks_needed[h], cepb, vc, key["party"])
    opp = 1 << (log - prev_log)
    if not prefixes:
        return corrected
    bptp = len(ec) // len(tree_indices)
    res = np.zeros((len(prefixes) * opp, corrected.shape[1]), np.uint8)
    for i, (ti, bi) in enumerate(prefix_map):
        s = ti * bptp * cepb + bi * opp
        res[i * opp:(i + 1) * opp] = corrected[s:s + opp]
    return res


def evaluate_at(P: OracleParams, key, h: int, points: Sequence[int], ctx=None) -> np.ndarray:
    """EvaluateAtImpl<T> (distributed_point_function.h:839-1010)."""
    log = P.log_domain[h]
    maxp = MASK128 if log >= 128 else (1 << log) - 1
    for i, p in enumerate(points):
        if p > maxp:
            raise ValueError(f"`evaluation_points[{i}]` larger than the domain size at "
                             f"hierarchy level {h}")
    if not points:
        return np.zeros((0, packed_size(P.vtypes[h])), np.uint8)
    vc = _value_correction(P, key, h)
    bib = log - P.hierarchy_to_tree[h]
    E = elements_per_block(P.vtypes[h])
    tree_idx = [p >> bib for p in points] if E > 1 else list(points)
    if ctx is None:
        seeds = blocks_from_ints([key["seed"]] * len(points))
        ctrl = np.full(len(points), key["party"], np.uint8)
        start = 0
    else:
        seeds, ctrl = _compute_partial_evaluations(P, tree_idx, h, True, ctx)
        start = P.hierarchy_to_tree[h]
    stop = P.hierarchy_to_tree[h]
    s, c = evaluate_seeds(seeds, ctrl, blocks_from_ints(tree_idx), *_cw_arrays(key, start, stop))
    bi = [(p & ((1 << bib) - 1)) if E > 1 else 0 for p in points]
    out = hash_select_correct(P.vtypes[h], s, c, P.blocks_needed[h], bi, vc, key["party"])
    if ctx is not None:
        ctx["prev"] = h
    return out


# --------------------------------------------------------------------------
# Distributed comparison function (dcf/distributed_comparison_function.{h,cc})
# --------------------------------------------------------------------------

def dcf_params(n: int, vt, sec: float = 0.0) -> OracleParams:
    """The DCF's incremental DPF: level i has log domain i (cc:57-63)."""
    return OracleParams([(i, vt, sec) for i in range(n)])


def dcf_zero_like(vt, beta_leaves: Sequence[int]) -> List[int]:
    """SetToZero (cc:21-32): integer and IntModN leaves (also inside tuples)
    become 0; XorWrapper values are left unchanged, as in the reference."""
    return [b if kind == LEAF_XOR else 0 for (kind, _, _), b in zip(leaves(vt), beta_leaves)]


def dcf_generate_keys(P: OracleParams, alpha: int, beta_leaves: Sequence[int],
                      seed0: int, seed1: int):
    """GenerateKeys (cc:79-101): level i's value is beta if bit (n-1-i) of alpha
    is set, else SetToZero(beta); the DPF point is alpha >> 1."""
    n = len(P.log_domain)
    vt = P.vtypes[0]
    betas = [list(beta_leaves) if (alpha >> (n - i - 1)) & 1 else dcf_zero_like(vt, beta_leaves)
             for i in range(n)]
    return generate_keys(P, alpha >> 1, betas, seed0, seed1)


def dcf_evaluate(P: OracleParams, key, x: int) -> np.ndarray:
    """Evaluate<T> (h:83-105): the sum over levels i with bit (n-1-i) of x clear
    of EvaluateAt(key, i, {x >> (n - i)}) (prefix 0 when n == 128).  Returns one
    packed element (1, packed_size)."""
    n = len(P.log_domain)
    vt = P.vtypes[0]
    acc = np.zeros((1, packed_size(vt)), np.uint8)
    for i in range(n):
        prefix = x >> (n - i) if n < 128 else 0
        e = evaluate_at(P, key, i, [prefix])
        if not (x >> (n - i - 1)) & 1:
            acc = add_packed(vt, acc, e)
    return acc
