"""The reference's two-party correctness checks, restated once and run against
any engine (the CPU oracle in test_oracle.py, the HIP-backed API in
test_api_gpu.py).

An engine provides:
  params(list of (log_domain, vt, sec)) -> handle P
  generate_keys(P, alpha, betas_leaves, seeds) -> (key0, key1)
  context(P, key) -> ctx
  evaluate_until(P, level, prefixes, ctx) -> packed uint8 (n, size)
  evaluate_at(P, key, level, points, ctx=None) -> packed uint8 (n, size)
"""
import numpy as np

import oracle as O


def _sum_ok(vt, a, b, expect_leaves_fn):
    tot = O.unpack_elements(vt, O.add_packed(vt, a, b))
    for i, el in enumerate(tot):
        exp = expect_leaves_fn(i)
        if el != exp:
            return i, el, exp
    return None


def prefix_for_level(log_domains, h, x):
    """GetPrefixForLevel (distributed_point_function_test.cc:317-325)."""
    shift = log_domains[-1] - log_domains[h]
    return x >> shift if shift < 128 else 0


def incremental_correctness(engine, levels, alpha, betas, level_step, single_point, seed=0,
                            num_points=1000):
    """IncrementalDpfTest::TestCorrectness (test.cc:619-663, 335-452).
    levels = [(log_domain, bits)], betas = one int per level."""
    params = [(ld, ("int", bits), 0) for ld, bits in levels]
    vts = [p[1] for p in params]
    logs = [ld for ld, _ in levels]
    P = engine.params(params)
    k0, k1 = engine.generate_keys(P, alpha, [[b] for b in betas], seeds=(seed * 2 + 11, seed * 2 + 13))
    rng = np.random.default_rng(seed)
    pts = []
    for _ in range(num_points - 1):
        x = int.from_bytes(rng.bytes(16), "little")
        if logs[-1] < 128:
            x %= 1 << logs[-1]
        pts.append(x)
    pts.append(alpha)
    c0, c1 = engine.context(P, k0), engine.context(P, k1)
    prev = -1
    for h in range(level_step - 1, len(levels), level_step):
        vt = vts[h]
        mask = (1 << levels[h][1]) - 1
        beta = betas[h] & mask
        cur_alpha = prefix_for_level(logs, h, alpha)
        if single_point:
            prefixes = [prefix_for_level(logs, h, x) for x in pts]
            r0 = engine.evaluate_at(P, k0, h, prefixes, c0)
            r1 = engine.evaluate_at(P, k1, h, prefixes, c1)
            bad = _sum_ok(vt, r0, r1, lambda i: [beta] if prefixes[i] == cur_alpha else [0])
        else:
            first = prev < 0
            prefixes = [] if first else [prefix_for_level(logs, prev, x) for x in pts]
            r0 = engine.evaluate_until(P, h, prefixes, c0)
            r1 = engine.evaluate_until(P, h, prefixes, c1)
            prev_log = 0 if first else logs[prev]
            opp = 1 << (logs[h] - prev_log)
            n_exp = 1 if first else len(prefixes)
            assert r0.shape[0] == n_exp * opp
            prev_alpha = 0 if first else prefix_for_level(logs, prev, alpha)

            def exp(i):
                pi, pe = divmod(i, opp)
                on = (first or prefixes[pi] == prev_alpha) and pe == cur_alpha % opp
                return [beta] if on else [0]
            bad = _sum_ok(vt, r0, r1, exp)
        assert bad is None, (h, bad)
        prev = h


def typed_regular(engine, vt, log_domain=10, alpha=23, sec=48.0):
    """DpfEvaluationTest::TestRegularDpf (test.cc:902-993)."""
    P = engine.params([(log_domain, vt, sec)])
    beta = [42] * len(O.leaves(vt))
    k0, k1 = engine.generate_keys(P, alpha, [beta], seeds=(77, 78))
    r0 = engine.evaluate_until(P, 0, [], engine.context(P, k0))
    r1 = engine.evaluate_until(P, 0, [], engine.context(P, k1))
    assert r0.shape[0] == 1 << log_domain
    zero = [0] * len(beta)
    bad = _sum_ok(vt, r0, r1, lambda i: beta if i == alpha else zero)
    assert bad is None, bad
    return r0, r1


def typed_batch_single_point(engine, vt, sec=48.0):
    """DpfEvaluationTest::TestBatchSinglePointEvaluation (test.cc:995-1030)."""
    beta = [42] * len(O.leaves(vt))
    zero = [0] * len(beta)
    for log_domain in (0, 1, 2, 32, 128):
        maxp = (1 << 128) - 1 if log_domain >= 128 else (1 << log_domain) - 1
        alpha = 23 & maxp
        P = engine.params([(log_domain, vt, sec)])
        k0, k1 = engine.generate_keys(P, alpha, [beta], seeds=(5 + log_domain, 9 + log_domain))
        for n in (0, 1, 2, 100, 1000):
            pts = [i & maxp for i in range(n)]
            r0 = engine.evaluate_at(P, k0, 0, pts)
            r1 = engine.evaluate_at(P, k1, 0, pts)
            assert r0.shape[0] == n
            if n:
                bad = _sum_ok(vt, r0, r1, lambda i: beta if pts[i] == alpha else zero)
                assert bad is None, (log_domain, n, bad)


class OracleEngine:
    """Adapter of the CPU oracle to the engine interface."""

    def params(self, params):
        return O.OracleParams(params)

    def generate_keys(self, P, alpha, betas, seeds):
        return O.generate_keys(P, alpha, betas, seeds[0], seeds[1])

    def context(self, P, key):
        return O.create_context(P, key)

    def evaluate_until(self, P, h, prefixes, ctx):
        return O.evaluate_until(P, h, prefixes, ctx)

    def evaluate_at(self, P, key, h, points, ctx=None):
        return O.evaluate_at(P, key, h, points, ctx)
