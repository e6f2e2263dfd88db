"""Incremental evaluation of a key batch with a device-resident context
(config 5b's heavy-hitters pattern) on an MI355X.

Every key of a batch is evaluated level by level at the same prefixes; per-key
outputs must equal the CPU oracle's EvaluateUntil
(distributed_point_function.h:641-837) run key by key with its own context,
the summed variant must equal the group sum of those outputs, and the exported
per-key context must equal the oracle's context after the same calls.
"""
import os

import numpy as np
import pytest

import oracle as O
import ref_grids as G
from distributed_point_functions_amd import dpf as D
from test_key_batch_gpu import _setup

pytestmark = pytest.mark.gpu


def _prefix_plan(P, plan, rng, first_prefix_count=6):
    """[(hierarchy level, prefixes)] following `plan` (list of levels); each
    later level's prefixes extend the previous call's prefixes, with a shuffle
    and a duplicate when there are several."""
    out, prev_pre, prev_h = [], [], None
    for i, h in enumerate(plan):
        if i == 0:
            out.append((h, []))
        else:
            log_prev = P.log_domain[prev_h]
            if i == 1:
                cand = sorted({int(x) for x in rng.integers(0, 1 << min(log_prev, 62),
                                                            size=first_prefix_count)})
                cand = [c & ((1 << log_prev) - 1) for c in cand]
            else:
                step = log_prev - P.log_domain[plan[i - 2]]
                cand = []
                for p in prev_pre:
                    for r in rng.choice(1 << min(step, 16), size=min(2, 1 << step), replace=False).tolist():
                        cand.append((p << step) | int(r))
                cand = sorted(set(cand))
                if len(cand) > 8:
                    idx = rng.choice(len(cand), size=8, replace=False)
                    cand = sorted(cand[int(i)] for i in idx)
            if len(cand) > 3 and i % 2 == 0:
                rng.shuffle(cand)
                cand.append(cand[0])  # duplicate prefix: its outputs repeat
            out.append((h, cand))
            prev_pre = sorted(set(cand))
        prev_h = h
    return out


def _check_export(dpf, bctx, batch, octx, k):
    """Lazy export of the device context == the oracle's per-key context."""
    ctx = dpf.export_evaluation_context(bctx, batch, k)
    assert ctx.previous_hierarchy_level == octx[k]["prev"]
    got = [(D.u128_from_block(e.prefix), D.u128_from_block(e.seed), int(e.control_bit))
           for e in ctx.partial_evaluations]
    assert sorted(got) == sorted(set(octx[k]["partials"]))
    if octx[k]["partials"]:
        assert ctx.partial_evaluations_level == octx[k]["partials_level"]


def _run(levels, plan, n_keys, sum_mode, seed, party_mix=True):
    import torch
    dpf, P, rng, batch, oks, _, _, _ = _setup(levels, n_keys, seed=seed, party_mix=party_mix)
    dev = dpf.upload_key_batch(batch)
    bctx = dpf.create_batch_evaluation_context(dev)
    octx = [O.create_context(P, k) for k in oks]
    cache_on = os.environ.get("DPF_BATCH_NO_CACHE") != "1"
    for h, prefixes in _prefix_plan(P, plan, rng):
        size = dpf.packed_size(h)
        vt = levels[h][1]
        n_out = dpf.output_elements(h, len(prefixes), bctx.previous_hierarchy_level)
        rows = 1 if sum_mode else n_keys
        out = torch.full((rows * n_out * size,), 0xAB, dtype=torch.uint8, device="cuda")
        n = dpf.evaluate_until_batch_to_device(h, prefixes, bctx, out, sum_over_keys=sum_mode)
        torch.cuda.synchronize()
        assert n == n_out
        got = out.cpu().numpy().reshape(rows, n_out, size)
        want = [O.evaluate_until(P, h, prefixes, c) for c in octx]
        if sum_mode:
            acc = want[0]
            for w in want[1:]:
                acc = O.add_packed(vt, acc, w)
            np.testing.assert_array_equal(got[0], acc, err_msg=f"level {h}")
        else:
            for k in range(n_keys):
                np.testing.assert_array_equal(got[k], want[k], err_msg=f"level {h} key {k}")
        assert bctx.previous_hierarchy_level == h
        # The expansion cache is written by every call but the last level's
        # (and not when the level's leaves are the root: tree depth 0).
        writes = cache_on and h < len(levels) - 1 and dpf.hierarchy_to_tree()[h] > 0
        assert bctx.expansion_cache_level == (h if writes else -1)
        _check_export(dpf, bctx, batch, octx, n_keys - 1)
    for k in (0, n_keys - 1):
        _check_export(dpf, bctx, batch, octx, k)
    return dpf, bctx


HH = ("tuple", [("intmodn", 32, G.M32)] * 2)
CASES = [
    # heavy-hitters shape: Tuple<IntModN32 x2>, 2-bit steps, security 64
    ([(4, HH, 64.0), (6, HH, 64.0), (8, HH, 64.0), (10, HH, 64.0), (12, HH, 64.0)],
     [0, 1, 2, 3, 4]),
    # uint32 hierarchy with several elements per block and block-index bits
    ([(5, ("int", 32), 0), (9, ("int", 32), 0), (14, ("int", 32), 0), (20, ("int", 32), 0)],
     [0, 1, 2, 3]),
    # deep jumps: expansions split into walked start nodes; a skipped level
    ([(3, ("int", 64), 0), (12, ("int", 64), 0), (13, ("int", 64), 0), (24, ("int", 64), 0)],
     [0, 1, 3]),
    ([(6, ("xor", 128), 0), (8, ("xor", 128), 0), (20, ("xor", 128), 0)], [0, 1, 2]),
    # the full 128-bit domain in 4-bit steps
    ([(b, ("int", 64), 0) for b in range(4, 129, 4)], list(range(32))),
    ([(2, ("int", 8), 0), (5, ("int", 8), 0), (7, ("int", 8), 0), (11, ("int", 8), 0)],
     [0, 1, 2, 3]),
    ([(8, ("int", 128), 0), (10, ("int", 128), 0), (16, ("int", 128), 0)], [0, 1, 2]),
    # generic conversion (no in-kernel key sum): per-key rows + row sum
    ([(6, ("tuple", [("int", 32), ("intmodn", 64, G.M64)]), 48.0),
      (8, ("tuple", [("int", 32), ("intmodn", 64, G.M64)]), 48.0),
      (11, ("tuple", [("int", 32), ("intmodn", 64, G.M64)]), 48.0)], [0, 1, 2]),
    ([(7, ("intmodn", 64, G.M64), 48.0), (9, ("intmodn", 64, G.M64), 48.0)], [0, 1]),
    ([(4, ("intmodn", 32, G.M32), 48.0), (6, ("intmodn", 32, G.M32), 48.0),
      (8, ("intmodn", 32, G.M32), 48.0)], [0, 1, 2]),
    # Moduli below 2^31: the Moller-Granlund division's normalisation shifts.
    ([(5, ("tuple", [("intmodn", 32, 1000003)] * 2), 48.0),
      (7, ("tuple", [("intmodn", 32, 1000003)] * 2), 48.0),
      (9, ("tuple", [("intmodn", 32, 1000003)] * 2), 48.0)], [0, 1, 2]),
    ([(4, ("intmodn", 32, 251), 48.0), (6, ("intmodn", 32, 251), 48.0)], [0, 1]),
]


@pytest.mark.parametrize("levels,plan", CASES, ids=lambda x: str(x)[:60])
@pytest.mark.parametrize("n_keys", [1, 70])
def test_batch_incremental_per_key(levels, plan, n_keys):
    _run(levels, plan, n_keys, False, seed=n_keys * 7 + len(levels))


@pytest.mark.parametrize("levels,plan", CASES, ids=lambda x: str(x)[:60])
@pytest.mark.parametrize("n_keys", [3, 130])
def test_batch_incremental_sum(levels, plan, n_keys):
    _run(levels, plan, n_keys, True, seed=n_keys * 5 + len(levels))


@pytest.mark.parametrize("levels,plan", CASES[:4] + CASES[-3:], ids=lambda x: str(x)[:60])
@pytest.mark.parametrize("sum_mode", [False, True])
def test_batch_incremental_without_expansion_cache(levels, plan, sum_mode, monkeypatch):
    """DPF_BATCH_NO_CACHE=1: every call re-derives its tree nodes by the path
    walk from the partial evaluations (the reference's ComputePartialEvaluations,
    distributed_point_function.cc:351-453) -- same outputs and contexts."""
    monkeypatch.setenv("DPF_BATCH_NO_CACHE", "1")
    _run(levels, plan, 37, sum_mode, seed=len(levels) + 11)


@pytest.mark.parametrize("levels,plan", CASES[:4] + CASES[-3:], ids=lambda x: str(x)[:60])
@pytest.mark.parametrize("sum_mode", [False, True])
def test_batch_incremental_cache_in_place(levels, plan, sum_mode, monkeypatch):
    """DPF_BATCH_CACHE_IN_PLACE=1: the fallback for when no spare cache buffer
    fits -- the start seeds are gathered out of the cache, which the kernel
    then rewrites in place.  Same outputs and contexts."""
    monkeypatch.setenv("DPF_BATCH_CACHE_IN_PLACE", "1")
    _run(levels, plan, 37, sum_mode, seed=len(levels) + 13)


def test_batch_many_prefixes_one_key():
    """Config-5a shape: one key, thousands of prefixes per level."""
    import torch
    levels = [(12, ("int", 32), 0), (14, ("int", 32), 0), (16, ("int", 32), 0),
              (18, ("int", 32), 0)]
    dpf, P, rng, batch, oks, _, _, _ = _setup(levels, 1, seed=3, party_mix=False)
    bctx = dpf.create_batch_evaluation_context(dpf.upload_key_batch(batch))
    octx = O.create_context(P, oks[0])
    prefixes = []
    for h in range(len(levels)):
        size = dpf.packed_size(h)
        n_out = dpf.output_elements(h, len(prefixes), bctx.previous_hierarchy_level)
        out = torch.empty(n_out * size, dtype=torch.uint8, device="cuda")
        dpf.evaluate_until_batch_to_device(h, prefixes, bctx, out)
        want = O.evaluate_until(P, h, prefixes, octx)
        np.testing.assert_array_equal(out.cpu().numpy().reshape(n_out, size), want)
        # next prefixes: ~3000 of this call's outputs (extensions of its prefixes)
        if not prefixes:
            cand = np.arange(1 << levels[h][0])
        else:
            step = levels[h][0] - levels[h - 1][0]
            cand = (np.array(prefixes)[:, None] << step | np.arange(1 << step)[None, :]).ravel()
        prefixes = sorted(int(x) for x in rng.choice(cand, size=min(3000, cand.size), replace=False))


def test_batch_errors_match_reference():
    import torch
    levels = [(4, ("int", 32), 0), (8, ("int", 32), 0), (12, ("int", 32), 0)]
    dpf, P, rng, batch, oks, _, _, _ = _setup(levels, 4, seed=11)
    bctx = dpf.create_batch_evaluation_context(dpf.upload_key_batch(batch))
    out = torch.empty(1 << 16, dtype=torch.uint8, device="cuda")
    with pytest.raises(D.DpfStatusError, match="must be empty if and only if"):
        dpf.evaluate_until_batch_to_device(1, [1], bctx, out)
    dpf.evaluate_until_batch_to_device(0, [], bctx, out)
    with pytest.raises(D.DpfStatusError, match="must be greater than"):
        dpf.evaluate_until_batch_to_device(0, [1], bctx, out)
    with pytest.raises(D.DpfStatusError, match="out of range for hierarchy level 0"):
        dpf.evaluate_until_batch_to_device(1, [16], bctx, out)
    dpf.evaluate_until_batch_to_device(1, [3, 5], bctx, out)
    with pytest.raises(D.DpfStatusError,
                       match="Prefix not present in ctx.partial_evaluations at hierarchy level 1"):
        dpf.evaluate_until_batch_to_device(2, [200], bctx, out)
    with pytest.raises(D.DpfStatusError, match="device output buffer too small"):
        dpf.evaluate_until_batch_to_device(2, [3 << 4], bctx, out[:10])
