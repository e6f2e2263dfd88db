"""Host C++ API checks that need no GPU: key generation (stays on the CPU),
the proto wire codec, parameter/key/context validation and the error contract
of the reference's tests (dpf/distributed_point_function_test.cc,
dpf/internal/proto_validator_test.cc)."""
import json
import os

import numpy as np
import pytest

import oracle as O
import ref_grids as G
from distributed_point_functions_amd import dpf as D
from distributed_point_functions_amd import proto as pb

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def vt_from_oracle(vt):
    k = vt[0]
    if k == "int":
        return D.integer_type(vt[1])
    if k == "xor":
        return D.xor_wrapper_type(vt[1])
    if k == "intmodn":
        return D.int_mod_n_type(vt[1], vt[2])
    return D.tuple_type(*[vt_from_oracle(e) for e in vt[1]])


def params(levels):
    out = []
    for ld, vt, sec in levels:
        p = pb.DpfParameters()
        p.log_domain_size = ld
        p.value_type.CopyFrom(vt_from_oracle(vt) if isinstance(vt, tuple) else vt)
        if sec:
            p.security_parameter = sec
        out.append(p)
    return out


def leaves_value(vt, leaves):
    it = iter(leaves)

    def build(t):
        if t[0] == "tuple":
            return tuple(build(e) for e in t[1])
        return next(it)
    return D.to_value(vt_from_oracle(vt), build(vt))


# ------------------------------------------------------------------ creation
def test_create_all_domains_and_bitsizes():
    # test.cc:36-52
    for log in range(0, 129, 4):
        for bits in (1, 2, 4, 8, 16, 32, 64, 128):
            p = pb.DpfParameters(log_domain_size=log)
            p.value_type.integer.bitsize = bits
            D.DistributedPointFunction.create(p)


def test_create_incremental_large_domain():
    D.DistributedPointFunction.create_incremental(params([(10, ("int", 128), 0), (100, ("int", 128), 0)]))


def test_create_fails_for_tuple_with_different_intmodn():
    # test.cc:67-77
    p = params([(10, ("tuple", [("intmodn", 32, 3), ("intmodn", 64, 4)]), 0)])
    with pytest.raises(D.DpfStatusError) as e:
        D.DistributedPointFunction.create(p[0])
    assert e.value.code_name == "UNIMPLEMENTED"
    assert e.value.message == "All elements of type IntModN in a tuple must be the same"


def test_create_fails_for_missing_value_type():
    p = pb.DpfParameters(log_domain_size=10)
    with pytest.raises(D.DpfStatusError) as e:
        D.DistributedPointFunction.create(p)
    assert (e.value.code_name, e.value.message) == ("INVALID_ARGUMENT", "`value_type` is required")


def test_create_fails_for_invalid_value_type():
    p = pb.DpfParameters(log_domain_size=10)
    p.value_type.SetInParent()
    with pytest.raises(D.DpfStatusError) as e:
        D.DistributedPointFunction.create(p)
    assert e.value.message.startswith("ValidateValueType: Unsupported ValueType")


@pytest.mark.parametrize("bad,msg", [
    (dict(log_domain_size=-1), "`log_domain_size` must be non-negative"),
    (dict(log_domain_size=129), "`log_domain_size` must be <= 128"),
    (dict(security_parameter=float("nan")), "`security_parameter` must not be NaN"),
    (dict(security_parameter=-1.0), "`security_parameter` must be in [0, 128]"),
    (dict(security_parameter=129.0), "`security_parameter` must be in [0, 128]"),
])
def test_parameter_validation(bad, msg):
    p = pb.DpfParameters(log_domain_size=10)
    p.value_type.integer.bitsize = 32
    for k, v in bad.items():
        setattr(p, k, v)
    with pytest.raises(D.DpfStatusError) as e:
        D.DistributedPointFunction.create(p)
    assert e.value.message == msg


def test_parameters_must_ascend():
    with pytest.raises(D.DpfStatusError) as e:
        D.DistributedPointFunction.create_incremental(params([(10, ("int", 32), 0), (10, ("int", 32), 0)]))
    assert "ascending order" in e.value.message


@pytest.mark.parametrize("bits,msg", [(0, "`bitsize` must be positive"),
                                      (256, "`bitsize` must be less than or equal to 128"),
                                      (24, "`bitsize` must be a power of 2")])
def test_integer_type_validation(bits, msg):
    p = pb.DpfParameters(log_domain_size=4)
    p.value_type.integer.bitsize = bits
    with pytest.raises(D.DpfStatusError) as e:
        D.DistributedPointFunction.create(p)
    assert e.value.message == msg


# ------------------------------------------------------------------ key generation
@pytest.mark.parametrize("levels,alpha,betas", [
    ([(10, ("int", 64), 0)], 23, [[42]]),
    ([(20, ("int", 64), 0)], 0xABCDE, [[7]]),
    ([(5, ("int", 8), 0), (10, ("int", 16), 0), (15, ("int", 32), 0)], 12345, [[1], [2], [3]]),
    ([(0, ("int", 8), 0), (10, ("int", 128), 0)], 100, [[80], [90]]),
    ([(128, ("int", 64), 0)], O.make_uint128(23, 42), [[1234567]]),
    ([(10, ("tuple", [("intmodn", 32, G.M32)] * 5), 48.0)], 23, [[42] * 5]),
    ([(10, ("tuple", [("int", 32), ("tuple", [("int", 32), ("int", 32)]), ("int", 32)]), 48.0)], 23,
     [[42] * 4]),
    ([(10, ("xor", 128), 48.0)], 23, [[42]]),
    ([(12, ("tuple", [("intmodn", 128, G.M80)] * 2), 48.0)], 77, [[42, 43]]),
])
def test_keygen_matches_oracle(levels, alpha, betas):
    P = O.OracleParams(levels)
    ok0, ok1 = O.generate_keys(P, alpha, betas, 0xAAAA, 0xBBBB)
    dpf = D.DistributedPointFunction.create_incremental(params(levels))
    for _, vt, _ in levels:
        dpf.register_value_type(vt_from_oracle(vt))
    bvals = [leaves_value(vt, b) for (_, vt, _), b in zip(levels, betas)]
    k0, k1 = dpf.generate_keys_incremental(alpha, bvals, seeds=(0xAAAA, 0xBBBB))
    assert dpf.hierarchy_to_tree() == P.hierarchy_to_tree
    for key, okey, party in ((k0, ok0, 0), (k1, ok1, 1)):
        assert key.party == party
        assert ((key.seed.high << 64) | key.seed.low) == okey["seed"]
        assert len(key.correction_words) == len(okey["cws"])
        for cw, (s, cl, cr, vc) in zip(key.correction_words, okey["cws"]):
            assert ((cw.seed.high << 64) | cw.seed.low) == s
            assert (int(cw.control_left), int(cw.control_right)) == (cl, cr)
            if vc is None:
                assert len(cw.value_correction) == 0
            else:
                got = [O.leaves(()) if False else None for _ in []]
                assert len(cw.value_correction) == len(vc)
        # last level correction, leaf by leaf
        vt_last = levels[-1][1]
        got = [_leaves_of_value(v) for v in key.last_level_value_correction]
        assert got == okey["last_vc"]


def _leaves_of_value(v):
    which = v.WhichOneof("value")
    if which == "tuple":
        out = []
        for e in v.tuple.elements:
            out += _leaves_of_value(e)
        return out
    return [D._get_integer(getattr(v, which))]


def test_key_has_correct_format():
    # test.cc:226-236
    for log in (0, 1, 7, 32, 62):
        for bits in (8, 16, 32, 64, 128):
            p = pb.DpfParameters(log_domain_size=log)
            p.value_type.integer.bitsize = bits
            dpf = D.DistributedPointFunction.create(p)
            a, b = dpf.generate_keys(0, 0)
            assert (a.party, b.party) == (0, 1)
            dpf.create_evaluation_context(a)  # validates the key


def test_keygen_errors():
    p = pb.DpfParameters(log_domain_size=10)
    p.value_type.integer.bitsize = 16
    dpf = D.DistributedPointFunction.create(p)
    with pytest.raises(D.DpfStatusError) as e:
        dpf.generate_keys_incremental(0, [1, 2])
    assert e.value.message == "`beta` has to have the same size as `parameters` passed at construction"
    with pytest.raises(D.DpfStatusError) as e:
        dpf.generate_keys(1 << 10, 1)
    assert e.value.message == "`alpha` must be smaller than the output domain size"
    with pytest.raises(D.DpfStatusError) as e:
        dpf.generate_keys(0, 1 << 16)
    assert e.value.code_name == "INVALID_ARGUMENT"


def test_keygen_fails_if_value_type_not_registered():
    # test.cc:115-134
    p = pb.DpfParameters(log_domain_size=10)
    p.value_type.tuple.elements.add().integer.bitsize = 32
    dpf = D.DistributedPointFunction.create(p)
    beta = pb.Value()
    beta.tuple.elements.add().integer.value_uint64 = 42
    with pytest.raises(D.DpfStatusError) as e:
        dpf.generate_keys(23, beta)
    assert e.value.code_name == "FAILED_PRECONDITION"
    assert e.value.message.startswith("No value correction function known")


def test_random_keys_differ():
    p = pb.DpfParameters(log_domain_size=20)
    p.value_type.integer.bitsize = 64
    dpf = D.DistributedPointFunction.create(p)
    a, _ = dpf.generate_keys(5, 6)
    c, _ = dpf.generate_keys(5, 6)
    assert a.seed != c.seed


# ------------------------------------------------------------------ wire format
def _fixture_context():
    g = json.load(open(os.path.join(GOLDEN, "validator_context.json")))
    ctx = pb.EvaluationContext()
    for p in g["parameters"]:
        q = ctx.parameters.add(log_domain_size=p["log_domain_size"],
                               security_parameter=p["security_parameter"])
        q.value_type.integer.bitsize = p["bitsize"]
    k = g["key"]
    ctx.key.seed.high, ctx.key.seed.low = k["seed_high"], k["seed_low"]
    for cw in k["correction_words"]:
        c = ctx.key.correction_words.add(control_left=cw["control_left"],
                                         control_right=cw["control_right"])
        c.seed.high, c.seed.low = cw["seed_high"], cw["seed_low"]
        for v in cw["value_correction"]:
            c.value_correction.add().integer.value_uint64 = v
    for v in k["last_level_value_correction"]:
        ctx.key.last_level_value_correction.add().integer.value_uint64 = v
    ctx.previous_hierarchy_level = g["previous_hierarchy_level"]
    return ctx


def test_wire_roundtrip_fixture_context():
    ctx = _fixture_context()
    b = ctx.SerializeToString()
    assert D.host().roundtrip("EvaluationContext", b) == b
    assert D.host().roundtrip("DpfKey", ctx.key.SerializeToString()) == ctx.key.SerializeToString()


def test_wire_roundtrip_generated_keys():
    dpf = D.DistributedPointFunction.create_incremental(
        params([(5, ("int", 8), 0), (10, ("tuple", [("int", 32), ("int", 64)]), 48.0)]))
    dpf.register_value_type(vt_from_oracle(("tuple", [("int", 32), ("int", 64)])))
    vt = vt_from_oracle(("tuple", [("int", 32), ("int", 64)]))
    a, b = dpf.generate_keys_incremental(23, [5, D.to_value(vt, (1, 2))])
    for k in (a, b):
        raw = k.SerializeToString()
        assert D.host().roundtrip("DpfKey", raw) == raw
        k2 = pb.DpfKey()
        k2.ParseFromString(raw)
        assert k2 == k


@pytest.mark.parametrize("v", [0, 1, 2**64 - 1, 2**64, 2**128 - 1])
def test_wire_value_integer(v):
    val = D.to_value(D.integer_type(128), v)
    assert D.host().roundtrip("Value", val.SerializeToString()) == val.SerializeToString()


def test_wire_partial_evaluations_and_negative_level():
    ctx = _fixture_context()
    for i in range(5):
        pe = ctx.partial_evaluations.add(control_bit=bool(i & 1))
        pe.prefix.low = i
        pe.seed.high, pe.seed.low = 2**63 + i, 7 * i
    ctx.partial_evaluations_level = 1
    ctx.previous_hierarchy_level = -1
    b = ctx.SerializeToString()
    assert D.host().roundtrip("EvaluationContext", b) == b


def test_validator_accepts_fixture_context_and_rejects_mismatch():
    ctx = _fixture_context()
    D._call(D.host().validate_context, [p.SerializeToString() for p in ctx.parameters],
            ctx.SerializeToString())
    bad = pb.EvaluationContext()
    bad.CopyFrom(ctx)
    bad.parameters[1].log_domain_size = 7
    with pytest.raises(D.DpfStatusError) as e:
        D._call(D.host().validate_context, [p.SerializeToString() for p in ctx.parameters],
                bad.SerializeToString())
    assert e.value.message == "Parameter 1 in `ctx` doesn't match"
    bad.CopyFrom(ctx)
    del bad.key.correction_words[0]
    with pytest.raises(D.DpfStatusError) as e:
        D._call(D.host().validate_context, [p.SerializeToString() for p in ctx.parameters],
                bad.SerializeToString())
    assert e.value.message == "Malformed DpfKey: expected 6 correction words, but got 5"
    bad.CopyFrom(ctx)
    bad.ClearField("key")
    with pytest.raises(D.DpfStatusError) as e:
        D._call(D.host().validate_context, [p.SerializeToString() for p in ctx.parameters],
                bad.SerializeToString())
    assert e.value.message == "ctx.key must be present"


# ------------------------------------------------------------------ evaluation errors before GPU work
def _ctx128(levels=((5, 128), (10, 128), (15, 128))):
    dpf = D.DistributedPointFunction.create_incremental(
        params([(l, ("int", b), 0) for l, b in levels]))
    a, _ = dpf.generate_keys_incremental(1, [1, 2, 3][: len(levels)])
    return dpf, dpf.create_evaluation_context(a)


def test_evaluation_fails_on_empty_context():
    dpf, _ = _ctx128()
    with pytest.raises(D.DpfStatusError) as e:
        dpf.evaluate_next([], pb.EvaluationContext())
    assert e.value.code_name == "INVALID_ARGUMENT"


@pytest.mark.parametrize("level", [-1, 3])
def test_evaluation_fails_if_level_out_of_range(level):
    dpf, ctx = _ctx128()
    with pytest.raises(D.DpfStatusError) as e:
        dpf.evaluate_until(level, [], ctx)
    assert e.value.message == "`hierarchy_level` must be non-negative and less than parameters_.size()"


def test_evaluation_fails_if_value_type_doesnt_match():
    dpf, ctx = _ctx128()
    strange = D.tuple_type(D.integer_type(8), D.integer_type(32), D.integer_type(8),
                           D.integer_type(16), D.integer_type(8))
    with pytest.raises(D.DpfStatusError) as e:
        dpf.evaluate_until(0, [], ctx, value_type=strange)
    assert e.value.message == "Value type T doesn't match parameters at `hierarchy_level`"


def test_evaluation_fails_if_prefixes_not_empty_on_first_call():
    dpf, ctx = _ctx128()
    with pytest.raises(D.DpfStatusError) as e:
        dpf.evaluate_until(0, [0], ctx)
    assert e.value.message == ("`prefixes` must be empty if and only if this is the first call "
                               "with `ctx`.")


def test_evaluation_fails_if_output_too_large():
    # test.cc:136-155
    dpf = D.DistributedPointFunction.create_incremental(
        params([(10, ("int", 128), 0), (100, ("int", 128), 0)]))
    a, _ = dpf.generate_keys_incremental(123, [456, 789])
    ctx = dpf.create_evaluation_context(a)
    with pytest.raises(D.DpfStatusError) as e:
        dpf.evaluate_until(1, [], ctx)
    assert e.value.message == ("Output size would be larger than 2**62. Please evaluate fewer "
                               "hierarchy levels at once.")


def test_evaluate_at_errors():
    dpf, ctx = _ctx128()
    a = ctx.key
    with pytest.raises(D.DpfStatusError) as e:
        dpf.evaluate_at(a, -1, [0])
    assert e.value.message == "`hierarchy_level` must be non-negative"
    with pytest.raises(D.DpfStatusError) as e:
        dpf.evaluate_at(a, 3, [0])
    assert e.value.message == ("`hierarchy_level` must be less than the number of parameters "
                               "passed at construction")
    with pytest.raises(D.DpfStatusError) as e:
        dpf.evaluate_at(a, 0, [0, 1 << 5])
    assert e.value.message == "`evaluation_points[1]` larger than the domain size at hierarchy level 0"
    assert dpf.evaluate_at(a, 0, []).size == 0


def test_fixture_context_value_correction_size_error():
    # proto_validator_test.textproto's key carries one value-correction entry
    # where uint32 packing needs four: EvaluateUntil reports ValuesToArray's error
    # (value_type_helpers.h:547-551) -- before any tree expansion result is used.
    ctx = _fixture_context()
    dpf = D.DistributedPointFunction.create_incremental(list(ctx.parameters))
    with pytest.raises(D.DpfStatusError) as e:
        try:
            dpf.evaluate_until(0, [], ctx)
        except D.DpfStatusError as err:
            if err.code_name == "INTERNAL":  # no GPU in this container
                pytest.skip("needs a GPU to reach the value-correction check")
            raise
    assert e.value.message == "values.size() (= 1) does not match ElementsPerBlock<T>() (= 4)"


def test_evaluate_shard_argument_validation_before_device():
    """EvaluateShardToDevice rejects bad shard arguments on the host, before
    any device work (so these run without a GPU)."""
    import torch
    dpf = D.DistributedPointFunction.create(params([(10, ("int", 64), 0)])[0])
    k0, _ = dpf.generate_keys_incremental(3, [D.to_value(D.integer_type(64), 1)], seeds=(1, 2))
    buf = torch.zeros(1 << 13, dtype=torch.uint8)
    for shard, num in [(0, 3), (4, 4), (-1, 2), (0, 0), (0, 1 << 10)]:
        with pytest.raises(D.DpfStatusError) as e:
            dpf.evaluate_shard_to_device(0, shard, num, dpf.create_evaluation_context(k0), buf,
                                         stream=_NullStream())
        assert e.value.code == 3, (shard, num, e.value.message)
    with pytest.raises(D.DpfStatusError, match="too small"):
        dpf.evaluate_shard_to_device(0, 0, 1, dpf.create_evaluation_context(k0), buf[:100],
                                     stream=_NullStream())
    with pytest.raises(D.DpfStatusError, match="hierarchy_level"):
        dpf.evaluate_shard_to_device(1, 0, 1, dpf.create_evaluation_context(k0), buf,
                                     stream=_NullStream())


class _NullStream:
    cuda_stream = 0
