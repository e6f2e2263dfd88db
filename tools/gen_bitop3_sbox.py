"""Maps the Boyar-Peralta AES S-box circuit onto gfx950 3-input LUT gates
(v_bitop3_b32) and emits the C++ body used by tools/bs_aes.h.

The BP circuit ("A depth-16 circuit for the AES S-box", Boyar and Peralta 2011:
32 AND, 77 XOR, 4 XNOR) is covered with 3-feasible cuts; an exact ILP
(scipy.optimize.milp / HiGHS) picks the cover with the fewest gates.  Every
gate becomes one VALU instruction: v_bitop3_b32 for 3-input functions,
v_xor/v_and/v_or (via bitop3 with a repeated operand) for 2-input ones.

Usage: python tools/gen_bitop3_sbox.py > /dev/null   (prints stats to stderr,
the generated header fragment to stdout)
"""
from __future__ import annotations

import itertools
import sys

import numpy as np
from scipy.optimize import LinearConstraint, milp

# Inputs U0 (MSB) .. U7 (LSB); outputs S0 (MSB) .. S7 (LSB).
NETLIST = """
T1 = U0 ^ U3
T2 = U0 ^ U5
T3 = U0 ^ U6
T4 = U3 ^ U5
T5 = U4 ^ U6
T6 = T1 ^ T5
T7 = U1 ^ U2
T8 = U7 ^ T6
T9 = U7 ^ T7
T10 = T6 ^ T7
T11 = U1 ^ U5
T12 = U2 ^ U5
T13 = T3 ^ T4
T14 = T6 ^ T11
T15 = T5 ^ T11
T16 = T5 ^ T12
T17 = T9 ^ T16
T18 = U3 ^ U7
T19 = T7 ^ T18
T20 = T1 ^ T19
T21 = U6 ^ U7
T22 = T7 ^ T21
T23 = T2 ^ T22
T24 = T2 ^ T10
T25 = T20 ^ T17
T26 = T3 ^ T16
T27 = T1 ^ T12
M1 = T13 & T6
M2 = T23 & T8
M3 = T14 ^ M1
M4 = T19 & U7
M5 = M4 ^ M1
M6 = T3 & T16
M7 = T22 & T9
M8 = T26 ^ M6
M9 = T20 & T17
M10 = M9 ^ M6
M11 = T1 & T15
M12 = T4 & T27
M13 = M12 ^ M11
M14 = T2 & T10
M15 = M14 ^ M11
M16 = M3 ^ M2
M17 = M5 ^ T24
M18 = M8 ^ M7
M19 = M10 ^ M15
M20 = M16 ^ M13
M21 = M17 ^ M15
M22 = M18 ^ M13
M23 = M19 ^ T25
M24 = M22 ^ M23
M25 = M22 & M20
M26 = M21 ^ M25
M27 = M20 ^ M21
M28 = M23 ^ M25
M29 = M28 & M27
M30 = M26 & M24
M31 = M20 & M23
M32 = M27 & M31
M33 = M27 ^ M25
M34 = M21 & M22
M35 = M24 & M34
M36 = M24 ^ M25
M37 = M21 ^ M29
M38 = M32 ^ M33
M39 = M23 ^ M30
M40 = M35 ^ M36
M41 = M38 ^ M40
M42 = M37 ^ M39
M43 = M37 ^ M38
M44 = M39 ^ M40
M45 = M42 ^ M41
M46 = M44 & T6
M47 = M40 & T8
M48 = M39 & U7
M49 = M43 & T16
M50 = M38 & T9
M51 = M37 & T17
M52 = M42 & T15
M53 = M45 & T27
M54 = M41 & T10
M55 = M44 & T13
M56 = M40 & T23
M57 = M39 & T19
M58 = M43 & T3
M59 = M38 & T22
M60 = M37 & T20
M61 = M42 & T1
M62 = M45 & T4
M63 = M41 & T2
L0 = M61 ^ M62
L1 = M50 ^ M56
L2 = M46 ^ M48
L3 = M47 ^ M55
L4 = M54 ^ M58
L5 = M49 ^ M61
L6 = M62 ^ L5
L7 = M46 ^ L3
L8 = M51 ^ M59
L9 = M52 ^ M53
L10 = M53 ^ L4
L11 = M60 ^ L2
L12 = M48 ^ M51
L13 = M50 ^ L0
L14 = M52 ^ M61
L15 = M55 ^ L1
L16 = M56 ^ L0
L17 = M57 ^ L1
L18 = M58 ^ L8
L19 = M63 ^ L4
L20 = L0 ^ L1
L21 = L1 ^ L7
L22 = L3 ^ L12
L23 = L18 ^ L2
L24 = L15 ^ L9
L25 = L6 ^ L10
L26 = L7 ^ L9
L27 = L8 ^ L10
L28 = L11 ^ L14
L29 = L11 ^ L17
S0 = L6 ^ L24
S1 = L16 ~^ L26
S2 = L19 ~^ L28
S3 = L6 ^ L21
S4 = L20 ^ L22
S5 = L25 ^ L29
S6 = L13 ~^ L27
S7 = L6 ~^ L23
"""

INPUTS = [f"U{i}" for i in range(8)]
OUTPUTS = [f"S{i}" for i in range(8)]


def parse():
    gates = {}
    order = []
    for line in NETLIST.strip().splitlines():
        lhs, rhs = [s.strip() for s in line.split("=")]
        for op in ("~^", "^", "&"):
            if op in rhs:
                a, b = [s.strip() for s in rhs.split(op)]
                gates[lhs] = (op, a, b)
                order.append(lhs)
                break
    return gates, order


def truth(gates, node, leaves):
    """Truth table (bitop3 convention: index = S0*4 + S1*2 + S2, missing
    operands repeat the last one) of `node` over `leaves`."""
    k = len(leaves)
    lv = list(leaves) + [leaves[-1]] * (3 - k)
    tt = 0
    for idx in range(8):
        env = {lv[0]: (idx >> 2) & 1}
        env.setdefault(lv[1], (idx >> 1) & 1)
        env.setdefault(lv[2], idx & 1)
        # Consistency for repeated operands.
        if (lv[1] == lv[0] and ((idx >> 1) & 1) != ((idx >> 2) & 1)) or \
           (lv[2] == lv[1] and (idx & 1) != ((idx >> 1) & 1)):
            continue
        memo = {}

        def ev(n):
            if n in env:
                return env[n]
            if n in memo:
                return memo[n]
            op, a, b = gates[n]
            x, y = ev(a), ev(b)
            r = x ^ y if op == "^" else (1 - (x ^ y) if op == "~^" else x & y)
            memo[n] = r
            return r

        if ev(node):
            tt |= 1 << idx
    # Fill don't-care rows of repeated operands with the canonical value.
    return tt


def main():
    gates, order = parse()
    cuts = {u: [frozenset([u])] for u in INPUTS}
    for n in order:
        _, a, b = gates[n]
        cs = set()
        for ca in cuts[a]:
            for cb in cuts[b]:
                u = ca | cb
                if len(u) <= 3:
                    cs.add(u)
        cs = sorted(cs, key=lambda s: (len(s), sorted(s)))
        cuts[n] = cs + [frozenset([n])]
    # ILP: x[n, c] = node n is materialised as one gate over cut c.
    var = []
    for n in order:
        for c in cuts[n][:-1]:
            var.append((n, c))
    index = {v: i for i, v in enumerate(var)}
    nv = len(var)
    rows, lo, hi = [], [], []
    for o in OUTPUTS:
        r = np.zeros(nv)
        for c in cuts[o][:-1]:
            r[index[(o, c)]] = 1
        rows.append(r); lo.append(1); hi.append(1)
    for (n, c), i in index.items():
        for leaf in c:
            if leaf in INPUTS:
                continue
            r = np.zeros(nv)
            r[i] = -1
            for c2 in cuts[leaf][:-1]:
                r[index[(leaf, c2)]] = 1
            rows.append(r); lo.append(0); hi.append(np.inf)
    for n in order:
        r = np.zeros(nv)
        for c in cuts[n][:-1]:
            r[index[(n, c)]] = 1
        rows.append(r); lo.append(0); hi.append(1)
    res = milp(c=np.ones(nv), constraints=LinearConstraint(np.array(rows), lo, hi),
               integrality=np.ones(nv), bounds=(0, 1), options={"time_limit": 600})
    chosen = {var[i][0]: var[i][1] for i in range(nv) if res.x[i] > 0.5}
    print(f"gates: {len(chosen)} (BP: {len(order)}), status {res.message}", file=sys.stderr)
    # Emit in topological order.
    topo = [n for n in order if n in chosen]
    outname = {f"S{i}": None for i in range(8)}
    lines = []
    for n in topo:
        leaves = sorted(chosen[n], key=lambda s: (s[0], int(s[1:])))
        tt = truth(gates, n, leaves)
        args = list(leaves) + [leaves[-1]] * (3 - len(leaves))
        lines.append((n, args, tt))
    return lines


SIMPLE = {0x18: "{0} ^ {1}", 0x80: "{0} & {1}", 0x98: "{0} | {1}", 0x60: None}


def emit(lines):
    out = ["// Generated by tools/gen_bitop3_sbox.py -- do not edit.",
           "// AES S-box as %d gfx950 3-input LUT gates (v_bitop3_b32), an exact" % len(lines),
           "// 3-feasible-cut cover of the Boyar-Peralta circuit.  x7 = most significant",
           "// bit plane, x0 = least; in place.",
           "BS_HD void sbox_planes(uint32_t& x7, uint32_t& x6, uint32_t& x5, uint32_t& x4,",
           "                       uint32_t& x3, uint32_t& x2, uint32_t& x1, uint32_t& x0) {"]
    names = {f"U{k}": f"x{7 - k}" for k in range(8)}
    for k in range(8):
        out.append(f"  const uint32_t U{k} = x{7 - k};")
    for n, args, tt in lines:
        two = args[1] == args[2]
        if two and tt in (0x18, 0x80, 0x98):
            expr = SIMPLE[tt].format(args[0], args[1])
        else:
            expr = f"BS3({args[0]}, {args[1]}, {args[2]}, 0x{tt:02x})"
        out.append(f"  const uint32_t {n} = {expr};")
    for k in range(8):
        out.append(f"  x{7 - k} = S{k};")
    out.append("}")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    sys.stdout.write(emit(main()))
