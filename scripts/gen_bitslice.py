#!/usr/bin/env python3
"""Generate talos_amd/csrc/bs_sbox.h: a bitsliced AES S-box for gfx950.

Starts from the Boyar-Peralta depth-16 S-box circuit (113 XOR/AND/XNOR gates;
J. Boyar, R. Peralta, "A depth-16 circuit for the AES S-box", 2011), merges
single-fan-out gates into 3-input nodes (each becomes one v_bitop3_b32 with a
computed truth table), verifies the merged circuit on all 256 inputs against the
S-box derived from GF(2^8) inversion, and emits straight-line HIP code.
"""
import os
import re
import sys

CIRCUIT = """
y14 = x3 ^ x5
y13 = x0 ^ x6
y9 = x0 ^ x3
y8 = x0 ^ x5
t0 = x1 ^ x2
y1 = t0 ^ x7
y4 = y1 ^ x3
y12 = y13 ^ y14
y2 = y1 ^ x0
y5 = y1 ^ x6
y3 = y5 ^ y8
t1 = x4 ^ y12
y15 = t1 ^ x5
y20 = t1 ^ x1
y6 = y15 ^ x7
y10 = y15 ^ t0
y11 = y20 ^ y9
y7 = x7 ^ y11
y17 = y10 ^ y11
y19 = y10 ^ y8
y16 = t0 ^ y11
y21 = y13 ^ y16
y18 = x0 ^ y16
t2 = y12 & y15
t3 = y3 & y6
t4 = t3 ^ t2
t5 = y4 & x7
t6 = t5 ^ t2
t7 = y13 & y16
t8 = y5 & y1
t9 = t8 ^ t7
t10 = y2 & y7
t11 = t10 ^ t7
t12 = y9 & y11
t13 = y14 & y17
t14 = t13 ^ t12
t15 = y8 & y10
t16 = t15 ^ t12
t17 = t4 ^ t14
t18 = t6 ^ t16
t19 = t9 ^ t14
t20 = t11 ^ t16
t21 = t17 ^ y20
t22 = t18 ^ y19
t23 = t19 ^ y21
t24 = t20 ^ y18
t25 = t21 ^ t22
t26 = t21 & t23
t27 = t24 ^ t26
t28 = t25 & t27
t29 = t28 ^ t22
t30 = t23 ^ t24
t31 = t22 ^ t26
t32 = t31 & t30
t33 = t32 ^ t24
t34 = t23 ^ t33
t35 = t27 ^ t33
t36 = t24 & t35
t37 = t36 ^ t34
t38 = t27 ^ t36
t39 = t29 & t38
t40 = t25 ^ t39
t41 = t40 ^ t37
t42 = t29 ^ t33
t43 = t29 ^ t40
t44 = t33 ^ t37
t45 = t42 ^ t41
z0 = t44 & y15
z1 = t37 & y6
z2 = t33 & x7
z3 = t43 & y16
z4 = t40 & y1
z5 = t29 & y7
z6 = t42 & y11
z7 = t45 & y17
z8 = t41 & y10
z9 = t44 & y12
z10 = t37 & y3
z11 = t33 & y4
z12 = t43 & y13
z13 = t40 & y5
z14 = t29 & y2
z15 = t42 & y9
z16 = t45 & y14
z17 = t41 & y8
t46 = z15 ^ z16
t47 = z10 ^ z11
t48 = z5 ^ z13
t49 = z9 ^ z10
t50 = z2 ^ z12
t51 = z2 ^ z5
t52 = z7 ^ z8
t53 = z0 ^ z3
t54 = z6 ^ z7
t55 = z16 ^ z17
t56 = z12 ^ t48
t57 = t50 ^ t53
t58 = z4 ^ t46
t59 = z3 ^ t54
t60 = t46 ^ t57
t61 = z14 ^ t57
t62 = t52 ^ t58
t63 = t49 ^ t58
t64 = z4 ^ t59
t65 = t61 ^ t62
t66 = z1 ^ t63
s0 = t59 ^ t63
s6 = t56 ^ ~t62
s7 = t48 ^ ~t60
t67 = t64 ^ t65
s3 = t53 ^ t66
s4 = t51 ^ t66
s5 = t47 ^ t65
s1 = t64 ^ ~s3
s2 = t55 ^ ~t67
"""

OUTS = [f"s{i}" for i in range(8)]


def sbox_table():
    def xt(a):
        return ((a << 1) ^ (0x1B if a & 0x80 else 0)) & 0xFF

    def gm(a, b):
        p = 0
        while b:
            if b & 1:
                p ^= a
            a = xt(a)
            b >>= 1
        return p
    sb = []
    for x in range(256):
        inv = next((y for y in range(1, 256) if gm(x, y) == 1), 0)
        s = inv
        for k in range(1, 5):
            s ^= ((inv << k) | (inv >> (8 - k))) & 0xFF
        sb.append(s ^ 0x63)
    return sb


def parse():
    nodes = {}   # name -> (inputs tuple, truth table over inputs as int bitmask)
    order = []
    for line in CIRCUIT.strip().splitlines():
        lhs, rhs = [s.strip() for s in line.split("=")]
        m = re.match(r"(\w+) (\^ ~|\^|&) ?(\w+)", rhs)
        a, op, b = m.group(1), m.group(2), m.group(3)
        # truth table index: bit i of index = value of input i
        tt = 0
        for idx in range(4):
            va, vb = idx & 1, (idx >> 1) & 1
            v = (va ^ vb) if op == "^" else (va & vb) if op == "&" else (va ^ (1 - vb))
            tt |= v << idx
        nodes[lhs] = ((a, b), tt)
        order.append(lhs)
    return nodes, order


def compose(nodes, g, p):
    """Inline node p into node g; return new (inputs, tt) or None if > 3 inputs."""
    gin, gtt = nodes[g]
    pin, ptt = nodes[p]
    new_in = []
    for x in list(pin) + [x for x in gin if x != p]:
        if x not in new_in:
            new_in.append(x)
    if len(new_in) > 3:
        return None
    tt = 0
    for idx in range(1 << len(new_in)):
        val = {x: (idx >> i) & 1 for i, x in enumerate(new_in)}
        pv = (ptt >> sum(val[x] << i for i, x in enumerate(pin))) & 1
        gval = {**val, p: pv}
        gv = (gtt >> sum(gval[x] << i for i, x in enumerate(gin))) & 1
        tt |= gv << idx
    return tuple(new_in), tt


def merge(nodes, order):
    changed = True
    while changed:
        changed = False
        uses = {n: 0 for n in nodes}
        for n in order:
            for x in nodes[n][0]:
                if x in uses:
                    uses[x] += 1
        for g in order:
            for p in nodes[g][0]:
                if p in nodes and uses[p] == 1 and p not in OUTS:
                    r = compose(nodes, g, p)
                    if r is not None:
                        nodes[g] = r
                        order.remove(p)
                        del nodes[p]
                        changed = True
                        break
            if changed:
                break
    return nodes, order


def evaluate(nodes, order, xin):
    env = dict(xin)
    for n in order:
        ins, tt = nodes[n]
        idx = sum(env[x] << i for i, x in enumerate(ins))
        env[n] = (tt >> idx) & 1
    return env


def to_bitop3(ins, tt):
    """v_bitop3_b32 D, S0, S1, S2 with table bit (S0<<2 | S1<<1 | S2)."""
    ins = list(ins)
    while len(ins) < 3:
        ins.append(ins[-1])
    k = len(set(ins))
    imm = 0
    for s0 in (0, 1):
        for s1 in (0, 1):
            for s2 in (0, 1):
                vals = {}
                # our tt index uses input position i (bit i); map S0=ins[0], S1=ins[1], S2=ins[2]
                v = [s0, s1, s2]
                assign = {}
                okv = True
                for name, bit in zip(ins, v):
                    if name in assign and assign[name] != bit:
                        okv = False
                    assign[name] = bit
                if not okv:
                    continue
                uniq = []
                for x in ins:
                    if x not in uniq:
                        uniq.append(x)
                idx = sum(assign[x] << i for i, x in enumerate(uniq))
                imm |= ((tt >> idx) & 1) << ((s0 << 2) | (s1 << 1) | s2)
    del k, vals
    return ins, imm


def c_expr(args, imm):
    """Plain C for two-input nodes (the compiler then picks VOP2 encodings and
    may fold them); v_bitop3_b32 for true three-input nodes."""
    if args[1] == args[2] and args[0] != args[1]:
        # 2-input table over (a, b): bits at S-index (a<<2)|(b<<1)|b
        t = [(imm >> ((a << 2) | (b << 1) | b)) & 1 for a in (0, 1) for b in (0, 1)]
        ops = {(0, 1, 1, 0): "({0} ^ {1})", (0, 0, 0, 1): "({0} & {1})",
               (0, 1, 1, 1): "({0} | {1})", (1, 0, 0, 1): "~({0} ^ {1})"}
        if tuple(t) in ops:
            return ops[tuple(t)].format(args[0], args[1])
    return f"bop3({args[0]}, {args[1]}, {args[2]}, 0x{imm:02X})"


def main():
    sb = sbox_table()
    nodes, order = parse()
    base = len(order)
    nodes, order = merge(nodes, order)
    for x in range(256):
        env = evaluate(nodes, order, {f"x{7 - b}": (x >> b) & 1 for b in range(8)})
        out = sum(env[f"s{7 - b}"] << b for b in range(8))
        assert out == sb[x], (x, out, sb[x])
    lines = []
    for n in order:
        ins, tt = nodes[n]
        if len(set(ins)) == 1 and len(ins) == 1:
            raise RuntimeError
        args, imm = to_bitop3(ins, tt)
        # original tt is over unique inputs; to_bitop3 needs tt over `ins` uniques order
        lines.append(f"  const uint32_t {n} = {c_expr(args, imm)};")
    hdr = f"""// bs_sbox.h — GENERATED by scripts/gen_bitslice.py; do not edit.
// Bitsliced AES S-box: {base} Boyar-Peralta gates merged into {len(order)}
// v_bitop3_b32 nodes, verified on all 256 inputs at generation time.
// x0 = bit 7 (MSB) ... x7 = bit 0 of the input byte planes; s0 = bit 7 ... s7 = bit 0.
#pragma once
#define TG_BS_SBOX(x0, x1, x2, x3, x4, x5, x6, x7, s0, s1, s2, s3, s4, s5, s6, s7) \\
  do {{ \\
"""
    # re-verify the emitted bitop3 form: D bit = imm[(S0 << 2) | (S1 << 1) | S2]
    emitted = []
    for n in order:
        args, imm = to_bitop3(*nodes[n])
        emitted.append((n, args, imm))
    for x in range(256):
        env = {f"x{7 - b}": (x >> b) & 1 for b in range(8)}
        for n, args, imm in emitted:
            env[n] = (imm >> ((env[args[0]] << 2) | (env[args[1]] << 1) | env[args[2]])) & 1
        assert sum(env[f"s{7 - b}"] << b for b in range(8)) == sb[x], x
    body = " \\\n".join(l.replace("  const uint32_t s", "  s").replace("const uint32_t s", "s")
                        if re.match(r"\s*const uint32_t s\d =", l) else l for l in lines)
    tail = " \\\n  } while (0)\n"
    out = hdr + body + tail
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "talos_amd", "csrc", "bs_sbox.h")
    open(path, "w").write(out)
    print(f"{base} gates -> {len(order)} bitop3 nodes; wrote {path}")


if __name__ == "__main__":
    main()
