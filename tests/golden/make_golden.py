#!/usr/bin/env python3
"""Generates the committed golden fixtures under tests/golden/.

* aes_kat.json            -- the reference's AES MMO known-answer vectors
                              (dpf/aes_128_fixed_key_hash_test.cc:29-41, 114-135), verbatim.
* validator_context.json  -- the reference's embedded EvaluationContext fixture
                              (dpf/internal/proto_validator_test.textproto) as JSON data.
* eval_paths_grid.json    -- oracle outputs (sha256) for the reference's Hwy-vs-scalar
                              differential inputs (dpf/internal/evaluate_prg_hwy_test.cc:55-86).
* full_domain.json        -- oracle keys (injected root seeds) and full-domain output
                              digests for several value types.

Run in the build container (it reads /root/reference only to transcribe the
textproto fixture):  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle as O  # noqa: E402

REF_TEXTPROTO = "/root/reference/dpf/internal/proto_validator_test.textproto"


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1)
        f.write("\n")


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def aes_kat():
    mk = O.make_uint128
    s0, s1 = mk(0x0123012301230123, 0x0123012301230123), mk(0x4567456745674567, 0x4567456745674567)
    return {"source": "dpf/aes_128_fixed_key_hash_test.cc:29-41,114-135",
            "cases": [
                {"key": hex(0), "in": [hex(s0), hex(s1)],
                 "out": [hex(mk(0x73C2DC14812BE4EF, 0xEAC64D09C8ADF8ED)),
                         hex(mk(0xB8F33653A53A8436, 0xAEDF39B62DE91D95))]},
                {"key": hex(mk(0x1111111111111111, 0x1111111111111111)), "in": [hex(s0), hex(s1)],
                 "out": [hex(mk(0x934704AFF58FA233, 0xD3C20D1B9CC18D8F)),
                         hex(mk(0x530098817046D284, 0x43E61D3273A04F7C))]}]}


def validator_context():
    txt = open(REF_TEXTPROTO).read()
    params = []
    for m in re.finditer(r"parameters \{\s*log_domain_size: (\d+)\s*value_type \{\s*integer \{\s*"
                         r"bitsize: (\d+)\s*\}\s*\}\s*security_parameter: ([\d.]+)", txt):
        params.append({"log_domain_size": int(m.group(1)), "bitsize": int(m.group(2)),
                       "security_parameter": float(m.group(3))})
    key_txt = txt[txt.index("key {"):]
    seed = re.search(r"seed \{\s*high: (\d+)\s*low: (\d+)", key_txt)
    cws = []
    for m in re.finditer(r"correction_words \{(.*?)\n  \}", key_txt, re.S):
        body = m.group(1)
        s = re.search(r"seed \{\s*high: (\d+)\s*low: (\d+)", body)
        vc = [int(v) for v in re.findall(r"value_uint64: (\d+)", body)]
        cws.append({"seed_high": int(s.group(1)), "seed_low": int(s.group(2)),
                    "control_left": "control_left: true" in body,
                    "control_right": "control_right: true" in body,
                    "value_correction": vc})
    last = re.search(r"last_level_value_correction: \{\s*integer: \{\s*value_uint64: (\d+)", key_txt)
    return {"source": "dpf/internal/proto_validator_test.textproto",
            "parameters": params,
            "key": {"seed_high": int(seed.group(1)), "seed_low": int(seed.group(2)),
                    "correction_words": cws,
                    "last_level_value_correction": [int(last.group(1))]},
            "previous_hierarchy_level": -1}


def hwy_inputs(num_seeds, num_levels):
    seeds = O.blocks_from_ints([O.make_uint128(i, i + 1) for i in range(num_seeds)])
    paths = O.blocks_from_ints([O.make_uint128(23 * i + 42, 42 * i + 23) for i in range(num_seeds)])
    ctrl = np.array([1 if i % 7 == 0 else 0 for i in range(num_seeds)], np.uint8)
    cws = O.blocks_from_ints([O.make_uint128(i + 1, i) for i in range(num_levels)])
    cl = np.array([1 if i % 23 == 0 else 0 for i in range(num_levels)], np.uint8)
    cr = np.array([1 if i % 42 != 0 else 0 for i in range(num_levels)], np.uint8)
    return seeds, ctrl, paths, cws, cl, cr


def eval_paths_grid():
    k1 = O.make_uint128(0x1111111111111111, 0x1111111111111111)
    cases = []
    for n in (1, 2, 101, 128, 1000):
        for L in (0, 1, 2, 32, 63, 64, 127):
            s, c = O.evaluate_seeds(*hwy_inputs(n, L), key_left=0, key_right=k1)
            cases.append({"num_seeds": n, "num_levels": L, "seeds_sha256": digest(s),
                          "ctrl_sha256": digest(c), "first_seed": hex(O.ints_from_blocks(s[:1])[0])})
    return {"source": "inputs of dpf/internal/evaluate_prg_hwy_test.cc:55-86, keys 0 / 0x11..11",
            "key_right": hex(k1), "cases": cases}


def vt_json(vt):
    if vt[0] == "tuple":
        return ["tuple", [vt_json(e) for e in vt[1]]]
    return list(vt)


def full_domain():
    cases = []
    spec = [
        (("int", 64), 12, 0.0, 1234, [42]),
        (("int", 8), 10, 0.0, 1023, [255]),
        (("int", 128), 9, 0.0, 0, [O.make_uint128(5, 6)]),
        (("xor", 128), 9, 48.0, 23, [42]),
        (("tuple", [("int", 32), ("int", 64)]), 8, 48.0, 100, [42, 43]),
        (("tuple", [("intmodn", 32, 4294967291)] * 2), 8, 48.0, 7, [42, 43]),
    ]
    for i, (vt, log, sec, alpha, beta) in enumerate(spec):
        P = O.OracleParams([(log, vt, sec)])
        s0, s1 = 0x1000 + i, 0x2000 + i
        k0, k1 = O.generate_keys(P, alpha, [beta], s0, s1)
        r0 = O.evaluate_until(P, 0, [], O.create_context(P, k0))
        r1 = O.evaluate_until(P, 0, [], O.create_context(P, k1))
        cases.append({"value_type": json.dumps(vt_json(vt)), "log_domain_size": log,
                      "security_parameter": sec, "alpha": hex(alpha),
                      "beta": [hex(b) for b in beta], "seed0": hex(s0), "seed1": hex(s1),
                      "cw_seeds": [hex(c[0]) for c in k0["cws"]],
                      "party0_sha256": digest(r0), "party1_sha256": digest(r1)})
    return {"source": "oracle (dpf_oracle.c) with injected root seeds", "cases": cases}


if __name__ == "__main__":
    dump("aes_kat.json", aes_kat())
    dump("validator_context.json", validator_context())
    dump("eval_paths_grid.json", eval_paths_grid())
    dump("full_domain.json", full_domain())
    print("golden fixtures written to", HERE)
