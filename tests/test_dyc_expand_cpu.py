"""CPU specification of the compact-record expansion used by the conv backward kernels.

fc_bwd writes one record per (image, pooled position): 64 bf16 pooled gradients + 64 argmax codes
(0..3, the 2x2 window pixel that won the max).  The conv kernels expand a 16-B chunk (8 channels) into
the dense chunk of window pixel q: channel j keeps its value iff its code == q.

Two device formulations exist (csrc/kernels/conv_bwd.hip):
  * ``dyc_expand`` / ``dyc_expand_rep``: SWAR zero-byte test of (codes ^ q*0x01010101), then
    v_perm_b32 byte selectors double each 0xFF byte into a 16-bit lane mask;
  * ``dyc_expand_q`` (conv2_dgrad): the codes shifted so each channel's code bits sit at bit 15 / 31
    of two words, one bit-op pair per window pixel, and v_perm_b32's sign selectors (8..11 = 0xFF iff
    bit 15 / 31 / 47 / 63 of {src0, src1} is set) turn the match flag into the lane mask.

This test emulates v_perm_b32 per the ISA (LLVM AMDGPU: selector >= 13 -> 0xFF, 12 -> 0x00,
8..11 -> sign of bit 15 / 31 / 47 / 63 of {S0, S1}, else byte sel of {S0, S1}) and checks that both
formulations equal the definition on random chunks, and that window code 4 (used by the lean wgrad to
zero rows past a chunk) selects nothing.
"""
import random

M32 = 0xFFFFFFFF


def perm(s0, s1, sel):
    comb = (s0 << 32) | s1
    out = 0
    for i in range(4):
        b = (sel >> (8 * i)) & 0xFF
        if b >= 13:
            v = 0xFF
        elif b == 12:
            v = 0
        elif b >= 8:
            v = 0xFF if (comb >> [15, 31, 47, 63][b - 8]) & 1 else 0
        else:
            v = (comb >> (8 * b)) & 0xFF
        out |= v << (8 * i)
    return out


def expand_swar(g, routes, q):
    rep = (q * 0x01010101) & M32
    keep = []
    for r in routes:
        x = r ^ rep
        nz = (((x & 0x7F7F7F7F) + 0x7F7F7F7F) | x) & 0x80808080
        keep.append((~((nz >> 7) * 0xFF)) & M32)
    return [g[0] & perm(0, keep[0], 0x01010000), g[1] & perm(0, keep[0], 0x03030202),
            g[2] & perm(0, keep[1], 0x01010000), g[3] & perm(0, keep[1], 0x03030202)]


def expand_sign_select(g, routes, q):
    out = []
    for w, r in enumerate(routes):
        e0, e1, o0, o1 = (r << 15) & M32, (r << 14) & M32, (r << 7) & M32, (r << 6) & M32
        me = (e0 if q & 1 else ~e0 & M32) & (e1 if q & 2 else ~e1 & M32)
        mo = (o0 if q & 1 else ~o0 & M32) & (o1 if q & 2 else ~o1 & M32)
        out += [g[2 * w] & perm(me, mo, 0x08080A0A), g[2 * w + 1] & perm(me, mo, 0x09090B0B)]
    return out


def expand_definition(g, routes, q):
    out = []
    for w in range(4):
        v = 0
        for h in range(2):
            ch = 2 * w + h                                  # channel within the chunk
            code = (routes[ch // 4] >> (8 * (ch % 4))) & 0xFF
            if code == q:
                v |= g[w] & (0xFFFF << (16 * h))
        out.append(v)
    return out


def test_record_expansion_formulations_agree():
    rng = random.Random(1234)
    for _ in range(4000):
        g = [rng.getrandbits(32) for _ in range(4)]
        routes = [sum(rng.randrange(4) << (8 * i) for i in range(4)) for _ in range(2)]
        for q in range(4):
            ref = expand_definition(g, routes, q)
            assert expand_swar(g, routes, q) == ref
            assert expand_sign_select(g, routes, q) == ref
        assert expand_swar(g, routes, 4) == [0, 0, 0, 0]     # window code 4: rows past the chunk
