"""Generate tools/bitsliced/sbox_bs.h: the AES S-box as a bitsliced circuit mapped onto
gfx950 3-input LUT instructions (v_bitop3_b32).

Source circuit: Boyar & Peralta's 128-gate AES S-box (XOR/XNOR/AND), checked exhaustively
against the FIPS-197 table below before emission. Mapping: gates whose output feeds exactly
one other gate are folded into that consumer while the merged cone has at most 3 leaves; every
remaining node becomes one v_bitop3_b32 (truth table computed here) or, for 2-input nodes,
one 2-input op. Run: python tools/gen_sbox_bitop3.py  (writes the header, prints op counts).
"""
import itertools
import os
import re

CIRCUIT = """
T1=U0^U3 T2=U0^U5 T3=U0^U6 T4=U3^U5 T5=U4^U6 T6=T1^T5 T7=U1^U2 T8=U7^T6 T9=U7^T7 T10=T6^T7
T11=U1^U5 T12=U2^U5 T13=T3^T4 T14=T6^T11 T15=T5^T11 T16=T5^T12 T17=T9^T16 T18=U3^U7 T19=T7^T18
T20=T1^T19 T21=U6^U7 T22=T7^T21 T23=T2^T22 T24=T2^T10 T25=T20^T17 T26=T3^T16 T27=T1^T12
M1=T13&T6 M2=T23&T8 M3=T14^M1 M4=T19&U7 M5=M4^M1 M6=T3&T16 M7=T22&T9 M8=T26^M6 M9=T20&T17
M10=M9^M6 M11=T1&T15 M12=T4&T27 M13=M12^M11 M14=T2&T10 M15=M14^M11 M16=M3^M2 M17=M5^T24
M18=M8^M7 M19=M10^M15 M20=M16^M13 M21=M17^M15 M22=M18^M13 M23=M19^T25 M24=M22^M23 M25=M22&M20
M26=M21^M25 M27=M20^M21 M28=M23^M25 M29=M28&M27 M30=M26&M24 M31=M20&M23 M32=M27&M31 M33=M27^M25
M34=M21&M22 M35=M24&M34 M36=M24^M25 M37=M21^M29 M38=M32^M33 M39=M23^M30 M40=M35^M36 M41=M38^M40
M42=M37^M39 M43=M37^M38 M44=M39^M40 M45=M42^M41 M46=M44&T6 M47=M40&T8 M48=M39&U7 M49=M43&T16
M50=M38&T9 M51=M37&T17 M52=M42&T15 M53=M45&T27 M54=M41&T10 M55=M44&T13 M56=M40&T23 M57=M39&T19
M58=M43&T3 M59=M38&T22 M60=M37&T20 M61=M42&T1 M62=M45&T4 M63=M41&T2
L0=M61^M62 L1=M50^M56 L2=M46^M48 L3=M47^M55 L4=M54^M58 L5=M49^M61 L6=M62^L5 L7=M46^L3 L8=M51^M59
L9=M52^M53 L10=M53^L4 L11=M60^L2 L12=M48^M51 L13=M50^L0 L14=M52^M61 L15=M55^L1 L16=M56^L0
L17=M57^L1 L18=M58^L8 L19=M63^L4 L20=L0^L1 L21=L1^L7 L22=L3^L12 L23=L18^L2 L24=L15^L9
L25=L6^L10 L26=L7^L9 L27=L8^L10 L28=L11^L14 L29=L11^L17
S0=L6^L24 S1=L16~L26 S2=L19~L28 S3=L6^L21 S4=L20^L22 S5=L25^L29 S6=L13~L27 S7=L6~L23
"""
SBOX = bytes.fromhex(
    "637c777bf26b6fc53001672bfed7ab76ca82c97dfa5947f0add4a2af9ca472c0b7fd9326363ff7cc34a5e5f171d8311504c723c31896059a071280e2eb27b275"
    "09832c1a1b6e5aa0523bd6b329e32f8453d100ed20fcb15b6acbbe394a4c58cfd0efaafb434d338545f9027f503c9fa851a3408f929d38f5bcb6da2110fff3d2"
    "cd0c13ec5f974417c4a77e3d645d197360814fdc222a908846eeb814de5e0bdbe0323a0a4906245cc2d3ac629195e479e7c8376d8dd54ea96c56f4ea657aae08"
    "ba78252e1ca6b4c6e8dd741f4bbd8b8a703eb5664803f60e613557b986c11d9ee1f8981169d98e949b1e87e9ce5528df8ca1890dbfe6426841992d0fb054bb16")

OPS = {"^": lambda a, b: a ^ b, "&": lambda a, b: a & b, "~": lambda a, b: 1 ^ a ^ b}


def parse():
    gates = []
    for tok in CIRCUIT.split():
        m = re.match(r"(\w+)=(\w+)([\^&~])(\w+)$", tok)
        gates.append((m.group(1), m.group(3), m.group(2), m.group(4)))
    return gates


def evaluate(gates, x):
    env = {f"U{i}": (x >> (7 - i)) & 1 for i in range(8)}
    for out, op, a, b in gates:
        env[out] = OPS[op](env[a], env[b])
    return sum(env[f"S{i}"] << (7 - i) for i in range(8))


def lut_map(gates):
    """Fold single-fanout gates into their consumer while the cone has <= 3 leaves."""
    fan = {}
    for _, _, a, b in gates:
        fan[a] = fan.get(a, 0) + 1
        fan[b] = fan.get(b, 0) + 1
    cone = {}  # name -> (leaves tuple, function over leaves as python callable via gate list)
    gdef = {out: (op, a, b) for out, op, a, b in gates}
    outputs = {f"S{i}" for i in range(8)}

    def leaves_of(sig):
        return cone[sig][0] if sig in cone else (sig,)

    absorbed = set()
    for out, op, a, b in gates:
        la, lb = (a,), (b,)
        # candidate absorption of a and/or b (fanout 1, internal)
        best = None
        for take_a in (True, False):
            for take_b in (True, False):
                L = []
                for sig, take in ((a, take_a), (b, take_b)):
                    if take:
                        if sig not in cone or fan.get(sig, 0) != 1 or sig in outputs:
                            break
                        L.extend(cone[sig][0])
                    else:
                        L.append(sig)
                else:
                    L = tuple(dict.fromkeys(L))
                    if len(L) <= 3:
                        score = int(take_a) + int(take_b)
                        if best is None or score > best[0]:
                            best = (score, take_a, take_b, L)
        _, take_a, take_b, L = best
        if take_a:
            absorbed.add(a)
        if take_b:
            absorbed.add(b)
        cone[out] = (L, (op, a if not take_a else ("cone", a), b if not take_b else ("cone", b)))
    nodes = [out for out, _, _, _ in gates if out not in absorbed]
    return cone, nodes

    
def cone_eval(cone, name, env):
    L, (op, a, b) = cone[name]
    va = cone_eval(cone, a[1], env) if isinstance(a, tuple) else env[a]
    vb = cone_eval(cone, b[1], env) if isinstance(b, tuple) else env[b]
    return OPS[op](va, vb)


def truth_table(cone, name):
    L = cone[name][0]
    tt = 0
    for idx in range(8):
        bits = [(idx >> 2) & 1, (idx >> 1) & 1, idx & 1][: len(L)] if len(L) == 3 else None
        env = {}
        if len(L) == 3:
            env = {L[0]: (idx >> 2) & 1, L[1]: (idx >> 1) & 1, L[2]: idx & 1}
        elif len(L) == 2:
            env = {L[0]: (idx >> 1) & 1, L[1]: idx & 1}
        else:
            env = {L[0]: idx & 1}
        tt |= cone_eval(cone, name, env) << idx
    return tt


def emit(cone, nodes):
    lines = []
    for n in nodes:
        L = cone[n][0]
        op, a, b = cone[n][1]
        simple = not isinstance(a, tuple) and not isinstance(b, tuple)
        if len(L) == 3 or not simple or op == "~":
            if len(L) == 3:
                tt = truth_table(cone, n)
                lines.append(f"  const uint32_t {n} = __builtin_amdgcn_bitop3_b32({L[0]}, {L[1]}, {L[2]}, 0x{tt:02x});")
            else:  # 2 leaves: pad with a repeated leaf
                L3 = (L[0], L[1], L[1]) if len(L) == 2 else (L[0], L[0], L[0])
                tt = 0
                for idx in range(8):
                    env = {L3[0]: (idx >> 2) & 1, L3[1]: (idx >> 1) & 1}
                    if len(L) == 1:
                        env = {L3[0]: (idx >> 2) & 1}
                    tt |= cone_eval(cone, n, env) << idx
                lines.append(f"  const uint32_t {n} = __builtin_amdgcn_bitop3_b32({L3[0]}, {L3[1]}, {L3[2]}, 0x{tt:02x});")
        else:
            c = {"^": "^", "&": "&"}[op]
            lines.append(f"  const uint32_t {n} = {a} {c} {b};")
    return lines


def main():
    gates = parse()
    assert all(evaluate(gates, x) == SBOX[x] for x in range(256)), "circuit != S-box"
    cone, nodes = lut_map(gates)
    # verify the mapped form
    for x in range(256):
        env = {f"U{i}": (x >> (7 - i)) & 1 for i in range(8)}
        for n in nodes:
            L = cone[n][0]
            env[n] = cone_eval(cone, n, env)
        assert sum(env[f"S{i}"] << (7 - i) for i in range(8)) == SBOX[x]
    body = emit(cone, nodes)
    hdr = os.path.join(os.path.dirname(__file__), "sbox_bs.h")
    with open(hdr, "w") as f:
        f.write("// GENERATED by tools/bitsliced/gen_sbox_bitop3.py -- do not edit.\n")
        f.write("// Bitsliced AES S-box (Boyar-Peralta 128-gate circuit, LUT3-mapped onto v_bitop3_b32:\n")
        f.write(f"// {len(nodes)} instructions for 32 byte-instances). U0 = input MSB ... U7 = LSB; S0 = output MSB.\n")
        f.write("#pragma once\n#include <stdint.h>\n\n")
        f.write("// x[0] = input MSB plane ... x[7] = LSB plane; results replace x (MSB first).\n")
        f.write("__device__ __forceinline__ void sbox_bs(uint32_t (&x)[8]) {\n")
        f.write("  const uint32_t U0 = x[0], U1 = x[1], U2 = x[2], U3 = x[3], U4 = x[4], U5 = x[5], U6 = x[6], U7 = x[7];\n")
        for l in body:
            f.write(l + "\n")
        f.write("  x[0] = S0; x[1] = S1; x[2] = S2; x[3] = S3; x[4] = S4; x[5] = S5; x[6] = S6; x[7] = S7;\n}\n")
    print(f"gates={len(gates)} mapped_nodes={len(nodes)}")


if __name__ == "__main__":
    main()
