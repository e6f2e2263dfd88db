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


@pytest.mark.parametrize("levels,plan", CASES[:4] + CASES[-3:], ids=lambda x: str(x)[:60])
@pytest.mark.parametrize("sum_mode", [False, True])
def test_batch_incremental_cache_permuted(levels, plan, sum_mode, monkeypatch):
    """DPF_BATCH_CACHE_MODE=permute: no spare; the kernel rewrites the cache
    in place through a slot table (each start node's leaf 0 into the slot it
    read, the other leaves into slots no start node reads; several start
    nodes per tree index leave their shared slot alone).  Same outputs and
    contexts, and no gather once the cache stride has stopped growing."""
    monkeypatch.setenv("DPF_BATCH_CACHE_MODE", "permute")
    _, bctx = _run(levels, plan, 37, sum_mode, seed=len(levels) + 17)
    ev = bctx.cache_events
    assert ev["evicted_spare"] == 0 and ev["evicted_cache"] == 0, ev
    if levels is HH5[0]:
        assert ev["permuted"] >= 1, ev


def test_permuted_cache_hh_shape_reads_and_writes_one_buffer(monkeypatch):
    """Heavy-hitters shape (Tuple<IntModN32 x2>, 2-bit steps, all candidates
    kept): every cached level after the stride stops growing is a permuted
    in-place rewrite, and the context never holds a second cache buffer."""
    levels, plan = HH5
    bctx0, _, held0 = _pressure_run(levels, plan, 40, True, seed=97)
    assert bctx0.cache_events["permuted"] == 0      # default: a spare fits
    monkeypatch.setenv("DPF_BATCH_CACHE_MODE", "permute")
    bctx, failed, held = _pressure_run(levels, plan, 40, True, seed=97)
    ev = bctx.cache_events
    assert failed == [] and ev["permuted"] >= 1 and ev["spare_refused"] == 0, ev
    assert max(held) < max(held0)          # the spare run holds two cache buffers


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


# ---------------------------------------------------------------------------
# The expansion cache under memory pressure (batch_context.cc: the spare and
# cache allocations, the per-call buffers' eviction-and-retry).  Whatever the
# cache does, outputs and exported contexts must equal the oracle's; a call
# that cannot get its per-call buffers fails with the reference's
# RESOURCE_EXHAUSTED "Memory allocation error" (distributed_point_function.cc:
# 289-291) and leaves the context usable: the same call retried succeeds.
# ---------------------------------------------------------------------------

def _pressure_run(levels, plan, n_keys, sum_mode, seed, arm=None, limit=None, monkeypatch=None):
    """Like _run; arm(i, bctx) is called before call i (it may arm the
    fail-next-allocations hook).  With `limit`, DPF_BATCH_ALLOC_LIMIT is set
    for every call.  A call failing with RESOURCE_EXHAUSTED is retried once
    with the hooks off.  Returns (bctx, indices of calls that failed,
    device_bytes after each call)."""
    import torch
    dpf, P, rng, batch, oks, _, _, _ = _setup(levels, n_keys, seed=seed, party_mix=True)
    bctx = dpf.create_batch_evaluation_context(dpf.upload_key_batch(batch))
    octx = [O.create_context(P, k) for k in oks]
    failed, held = [], []
    for i, (h, prefixes) in enumerate(_prefix_plan(P, plan, rng)):
        size = dpf.packed_size(h)
        n_out = dpf.output_elements(h, len(prefixes), bctx.previous_hierarchy_level)
        rows = 1 if sum_mode else n_keys
        out = torch.full((rows * n_out * size,), 0xAB, dtype=torch.uint8, device="cuda")
        if arm:
            arm(i, bctx)
        if limit is not None:
            monkeypatch.setenv("DPF_BATCH_ALLOC_LIMIT", str(limit))
        try:
            n = dpf.evaluate_until_batch_to_device(h, prefixes, bctx, out, sum_over_keys=sum_mode)
        except D.DpfStatusError as e:
            assert "RESOURCE_EXHAUSTED" in str(e) and "Memory allocation error" in str(e), str(e)
            failed.append(i)
            bctx.fail_next_allocations_for_testing(0)
            if limit is not None:
                monkeypatch.delenv("DPF_BATCH_ALLOC_LIMIT")
            assert bctx.previous_hierarchy_level != h   # the failed call left ctx as it was
            n = dpf.evaluate_until_batch_to_device(h, prefixes, bctx, out, sum_over_keys=sum_mode)
        finally:
            if limit is not None:
                monkeypatch.delenv("DPF_BATCH_ALLOC_LIMIT", raising=False)
        torch.cuda.synchronize()
        assert n == n_out
        got = out.cpu().numpy().reshape(rows, n_out, size)
        want = [O.evaluate_until(P, h, prefixes, c) for c in octx]
        if sum_mode:
            acc = want[0]
            for w in want[1:]:
                acc = O.add_packed(levels[h][1], acc, w)
            np.testing.assert_array_equal(got[0], acc, err_msg=f"call {i} level {h}")
        else:
            for k in range(n_keys):
                np.testing.assert_array_equal(got[k], want[k], err_msg=f"call {i} level {h} key {k}")
        held.append(bctx.device_bytes)
        _check_export(dpf, bctx, batch, octx, n_keys - 1)
    return bctx, failed, held


HH5 = CASES[0]   # Tuple<IntModN32 x2>, five levels, 2-bit steps


@pytest.mark.parametrize("sum_mode", [False, True])
def test_cache_spare_evicted_for_per_call_buffer(sum_mode):
    """Call 2 reads the cache and would write the spare; its first per-call
    allocation fails once, so the spare is freed, the call writes no cache,
    and call 3 walks down from the partial evaluations and rebuilds it."""
    levels, plan = HH5
    arm = lambda i, c: c.fail_next_allocations_for_testing(1) if i == 2 else None
    bctx, failed, held = _pressure_run(levels, plan, 33, sum_mode, seed=91, arm=arm)
    ev = bctx.cache_events
    assert failed == [] and ev["evicted_spare"] == 1 and ev["evicted_cache"] == 0, ev
    assert ev["alloc_failures"] == 1, ev
    # After the last level nothing reads the cache; an explicit release gives
    # its memory back.
    assert bctx.expansion_cache_level == -1
    before = bctx.device_bytes
    bctx.release_expansion_cache()
    assert bctx.device_bytes < before


@pytest.mark.parametrize("sum_mode", [False, True])
def test_cache_in_use_cannot_be_evicted_call_fails_and_retries(sum_mode):
    """Call 3 reads the cache; two allocation failures free the spare and then
    find only the cache the call is reading: RESOURCE_EXHAUSTED.  The same
    call retried reads the still-valid cache and succeeds."""
    levels, plan = HH5
    arm = lambda i, c: c.fail_next_allocations_for_testing(2) if i == 3 else None
    bctx, failed, _ = _pressure_run(levels, plan, 21, sum_mode, seed=92, arm=arm)
    ev = bctx.cache_events
    assert failed == [3] and ev["evicted_spare"] == 1 and ev["evicted_cache"] == 0, ev


def test_cache_evicted_after_in_place_gather(monkeypatch):
    """No spare (the in-place path): once call 2 has gathered its start seeds
    the cache is only the write target, so a per-call allocation failure after
    the gather frees it -- the call writes no cache, call 3 walks down from
    the partial evaluations and rebuilds it."""
    monkeypatch.setenv("DPF_BATCH_CACHE_IN_PLACE", "1")
    levels, plan = HH5
    # Four per-call buffers precede the gather (the start-node table image,
    # the next partial evaluations' seeds and control bits, the cache slots).
    arm = lambda i, c: c.fail_next_allocations_for_testing(1, skip=4) if i == 2 else None
    bctx, failed, _ = _pressure_run(levels, plan, 17, True, seed=93, arm=arm)
    ev = bctx.cache_events
    assert failed == [] and ev["evicted_cache"] == 1 and ev["evicted_spare"] == 0, ev
    assert ev["in_place"] >= 2, ev


@pytest.mark.parametrize("frac", [0.9, 0.7, 0.5, 0.35])
def test_cache_under_device_memory_limit(frac, monkeypatch):
    """DPF_BATCH_ALLOC_LIMIT models a device with less memory: below the
    unlimited run's peak the spare (quarter-of-device headroom) and then the
    cache (an eighth) are refused or evicted; calls that cannot get their
    per-call buffers fail with RESOURCE_EXHAUSTED and succeed on retry."""
    levels, plan = HH5
    bctx0, _, held0 = _pressure_run(levels, plan, 64, True, seed=94)
    limit = int(max(held0) * frac)
    bctx, failed, _ = _pressure_run(levels, plan, 64, True, seed=94, limit=limit,
                                    monkeypatch=monkeypatch)
    ev = bctx.cache_events
    assert ev["spare_refused"] + ev["cache_refused"] + ev["evicted_spare"] + ev["evicted_cache"] \
        + len(failed) > 0, ev


def test_allocation_limit_too_small_is_resource_exhausted(monkeypatch):
    """A limit below the first call's per-call buffers (one byte): the
    reference's RESOURCE_EXHAUSTED message, and the context is untouched."""
    import torch
    levels, plan = HH5
    dpf, P, rng, batch, oks, _, _, _ = _setup(levels, 8, seed=95)
    bctx = dpf.create_batch_evaluation_context(dpf.upload_key_batch(batch))
    out = torch.empty(1 << 16, dtype=torch.uint8, device="cuda")
    monkeypatch.setenv("DPF_BATCH_ALLOC_LIMIT", "1")
    with pytest.raises(D.DpfStatusError, match="Memory allocation error"):
        dpf.evaluate_until_batch_to_device(0, [], bctx, out)
    assert bctx.previous_hierarchy_level == -1
    monkeypatch.delenv("DPF_BATCH_ALLOC_LIMIT")
    dpf.evaluate_until_batch_to_device(0, [], bctx, out)
    assert bctx.previous_hierarchy_level == 0


def test_reset_releases_expansion_cache():
    """Reset(release_expansion_cache=True) gives the expansion cache's memory
    back; plain Reset() keeps it for the next pass."""
    import torch
    levels, plan = HH5
    dpf, P, rng, batch, oks, _, _, _ = _setup(levels, 40, seed=96)
    bctx = dpf.create_batch_evaluation_context(dpf.upload_key_batch(batch))
    out = torch.empty(40 * (1 << 12) * 8, dtype=torch.uint8, device="cuda")
    dpf.evaluate_until_batch_to_device(0, [], bctx, out)
    dpf.evaluate_until_batch_to_device(1, [0, 1, 5], bctx, out)
    torch.cuda.synchronize()
    assert bctx.expansion_cache_level == 1
    before = bctx.device_bytes
    bctx.reset()
    assert bctx.expansion_cache_level == -1 and bctx.device_bytes == before
    dpf.evaluate_until_batch_to_device(0, [], bctx, out)
    dpf.evaluate_until_batch_to_device(1, [0, 1, 5], bctx, out)
    torch.cuda.synchronize()
    assert bctx.expansion_cache_level == 1
    bctx.reset(release_expansion_cache=True)
    assert bctx.expansion_cache_level == -1 and bctx.device_bytes < before
    dpf.evaluate_until_batch_to_device(0, [], bctx, out)
    assert bctx.expansion_cache_level == 0


def test_heavy_hitters_levels_run_the_lean_kernel(monkeypatch):
    """Cached heavy-hitters levels (start seeds from the expansion cache, two
    expanded levels, Tuple<IntModN32 x2> sums) run hh_keys_kernel (lanes =
    keys, index-major tables; dpf_batch_hh.hip); DPF_BATCH_KEY_MAJOR=1 runs
    r15's hh_level_kernel (lanes = start nodes, key-major tables) and
    DPF_BATCH_NO_LEAN=1 the general kernel.  All equal the oracle (checked by
    _pressure_run), and each other."""
    from distributed_point_functions_amd import hip_abi as H
    levels, plan = HH5
    seen = []

    def arm(i, c):
        if i > 0:
            seen.append(H.last_batch_kernel())
    _pressure_run(levels, plan, 45, True, seed=97, arm=arm)
    seen.append(H.last_batch_kernel())
    assert seen[-1] == "hh_keys", seen   # the last (cached) level
    monkeypatch.setenv("DPF_BATCH_KEY_MAJOR", "1")
    _pressure_run(levels, plan, 45, True, seed=97)
    assert H.last_batch_kernel() == "hh_level"
    monkeypatch.delenv("DPF_BATCH_KEY_MAJOR")
    monkeypatch.setenv("DPF_BATCH_NO_LEAN", "1")
    _pressure_run(levels, plan, 45, True, seed=97)
    assert H.last_batch_kernel() == "batch_level/mod32"


@pytest.mark.parametrize("levels,plan", CASES[:4] + CASES[-3:], ids=lambda x: str(x)[:60])
@pytest.mark.parametrize("mode", ["default", "permute", "gather"])
def test_batch_key_major_layout(levels, plan, mode, monkeypatch):
    """DPF_BATCH_KEY_MAJOR=1: the r15 key-major context tables ([key][slot])
    with every cache mode -- same outputs and exported contexts as the
    index-major default."""
    monkeypatch.setenv("DPF_BATCH_KEY_MAJOR", "1")
    if mode != "default":
        monkeypatch.setenv("DPF_BATCH_CACHE_MODE", mode)
    _run(levels, plan, 37, True, seed=len(levels) + 19)


@pytest.mark.parametrize("n_keys", [63, 64, 65, 1000])
@pytest.mark.parametrize("mode", ["default", "permute", "gather"])
def test_hh_keys_kernel_key_groups(n_keys, mode, monkeypatch):
    """Lanes = keys: ragged last 64-key group, one group, and enough groups
    that each wave takes a range of start nodes -- sums and exported contexts
    equal the oracle in every cache mode."""
    if mode != "default":
        monkeypatch.setenv("DPF_BATCH_CACHE_MODE", mode)
    levels, plan = HH5
    _pressure_run(levels, plan, n_keys, True, seed=n_keys + 3)


def test_permuted_cache_slot_tables_pass_the_contract_check(monkeypatch):
    """DPF_HIP_CHECK_SLOTS=1: every slot table the context builds for an
    in-place rewrite satisfies the contract of
    dpf_hip_eval_prefix_batch_cached_slots (checked on the host before each
    launch) -- in both table layouts."""
    monkeypatch.setenv("DPF_HIP_CHECK_SLOTS", "1")
    monkeypatch.setenv("DPF_BATCH_CACHE_MODE", "permute")
    levels, plan = HH5
    bctx, failed, _ = _pressure_run(levels, plan, 40, True, seed=98)
    assert failed == [] and bctx.cache_events["permuted"] >= 1
    monkeypatch.setenv("DPF_BATCH_KEY_MAJOR", "1")
    bctx, failed, _ = _pressure_run(levels, plan, 40, True, seed=98)
    assert failed == [] and bctx.cache_events["permuted"] >= 1


@pytest.mark.parametrize("bad", ["out_of_range", "twice", "overwrites_other_reader"])
def test_broken_slot_table_is_rejected(bad, monkeypatch):
    """A slot table breaking the contract is INVALID_ARGUMENT under
    DPF_HIP_CHECK_SLOTS=1, before anything is launched."""
    import ctypes
    import torch
    from distributed_point_functions_amd import hip_abi as H
    monkeypatch.setenv("DPF_HIP_CHECK_SLOTS", "1")
    L = H.load(require_gpu=True)
    K, U, E, stride = 4, 2, 2, 8
    dev = "cuda"
    blocks = lambda n: torch.zeros((n, 2), dtype=torch.int64, device=dev)
    key_seed, cw_seed, vcw = blocks(K), blocks(K * 2), blocks(K * 2)
    party = torch.zeros(K, dtype=torch.uint8, device=dev)
    cw_l = torch.zeros(K * 2, dtype=torch.uint8, device=dev)
    cw_r = torch.zeros(K * 2, dtype=torch.uint8, device=dev)
    cache = blocks(K * stride)
    parent = torch.tensor([0, 1], dtype=torch.int32, device=dev)
    slots = {"out_of_range": [0, 2, 3, 8, 1, 4, 5, 6],
             "twice": [0, 2, 3, 4, 1, 4, 5, 6],
             "overwrites_other_reader": [0, 1, 3, 4, 2, 5, 6, 7]}[bad]
    leaf_slot = torch.tensor(slots, dtype=torch.int32, device=dev)
    out = torch.zeros(K * (U << E) * 8, dtype=torch.uint8, device=dev)
    desc = H.value_desc([(H.LEAF_INT, 64, 0)], True, 2, 1)
    kl, kr, kv = H.aes_key(1), H.aes_key(2), H.aes_key(3)
    P, I64, I = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    f = L.dpf_hip_eval_prefix_batch_layout
    f.argtypes = [I64, I64, I, I, I, I, I, P, P, P, P, I64, P, P, P, P, P, I64, P, P, P, P, P, P,
                  P, I, P, I, P, P, P, I64, P, I, P]
    for index_major in (0, 1):
        rc = f(K, U, 0, -1, E, 0, 2, key_seed.data_ptr(), party.data_ptr(), cache.data_ptr(), None,
               stride, parent.data_ptr(), None, None, None, None, 0, cw_seed.data_ptr(),
               cw_l.data_ptr(), cw_r.data_ptr(), ctypes.byref(kl), ctypes.byref(kr),
               ctypes.byref(kv), ctypes.byref(desc), 2, vcw.data_ptr(), 0, None, out.data_ptr(),
               cache.data_ptr(), stride, leaf_slot.data_ptr(), index_major,
               H._stream(None))
        assert rc == 3, (bad, rc)
        assert "slot table" in L.dpf_hip_last_error().decode()
    torch.cuda.synchronize()
