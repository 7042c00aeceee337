"""CPU specification of the compact-record expansion used by the conv backward kernels.

fc_bwd writes one record per (image, pooled position): 64 bf16 pooled gradients + the 64 argmax codes
(0..3, the 2x2 window pixel that won the max) as bit planes - per 8-channel chunk two bytes, bit j of
the first = code bit 0 of channel j, of the second = code bit 1 (csrc/include/kernels.h DYC_ROUTE).
The conv kernels expand a 16-B chunk (8 channels) into the dense chunk of window pixel q: channel j
keeps its value iff its code == q.

Device formulation (csrc/kernels/conv_bwd.hip ``dyc_expand_flags``): rr = r16 | (r16 >> 1) << 16 puts
both channels of output word k next to each other 16 bits apart; rr << (15 - 2k) and rr << (7 - 2k)
bring their bit-0 / bit-1 flags to bits 15 / 31, ANDed (each operand inverted where the pixel's code
bit is 0), and v_perm_b32's sign selectors 8 / 9 (0xFF iff bit 15 / 31 of src1) turn the flags into
16-bit lane masks.  Window code 4 (the lean wgrad's rows past a chunk) selects nothing.

The producer side (fc_bwd role B) builds the planes from two wave ballots: bit 16 kg + m of a ballot
= channel 16 nt + m of row 4 kg + r, so the row's 16-bit slice holds chunks 2 nt / 2 nt + 1, and one
v_perm_b32 (selector 0x05010400) interleaves the two planes' bytes.  Both are emulated here per the
ISA (LLVM AMDGPU: selector >= 13 -> 0xFF, 12 -> 0x00, 8..11 -> sign of bit 15 / 31 / 47 / 63 of
{S0, S1}, else byte sel of {S0, S1}).
"""
import random

import torch

from pytorch_mnist_ddp_amd.ops.functional import route_codes

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


def planes_of(codes):
    """8 codes -> r16 (plane 0 in the low byte, plane 1 in the high byte)."""
    p0 = sum((c & 1) << j for j, c in enumerate(codes))
    p1 = sum(((c >> 1) & 1) << j for j, c in enumerate(codes))
    return p0 | (p1 << 8)


def expand_device(g, r16, q):
    rr = (r16 | ((r16 >> 1) << 16)) & M32
    none = M32 if q < 4 else 0
    bx = (rr if q & 1 else ~rr & M32) & none
    by = rr if q & 2 else ~rr & M32
    out = []
    for k in range(4):
        f = ((bx << (15 - 2 * k)) & M32) & ((by << (7 - 2 * k)) & M32)
        out.append(g[k] & perm(0, f, 0x09090808))
    return out


def expand_definition(g, codes, q):
    out = []
    for w in range(4):
        v = 0
        for h in range(2):
            if codes[2 * w + h] == q:
                v |= g[w] & (0xFFFF << (16 * h))
        out.append(v)
    return out


def test_record_expansion_matches_definition():
    rng = random.Random(1234)
    for _ in range(4000):
        g = [rng.getrandbits(32) for _ in range(4)]
        codes = [rng.randrange(4) for _ in range(8)]
        r16 = planes_of(codes)
        for q in range(4):
            assert expand_device(g, r16, q) == expand_definition(g, codes, q)
        assert expand_device(g, r16, 4) == [0, 0, 0, 0]     # window code 4: rows past the chunk


def test_ballot_producer_writes_the_planes():
    """fc_bwd role B: per (nt, r) two 64-lane ballots (lane 16 kg + m = channel 16 nt + m of row
    4 kg + r); the lane m == 0 of group kg writes route dword nt of its row's record."""
    rng = random.Random(7)
    for _ in range(200):
        codes = [[rng.randrange(4) for _ in range(64)] for _ in range(16)]   # [row bl][channel]
        route = [[0] * 4 for _ in range(16)]                                    # [row][dword nt]
        for nt in range(4):
            for r in range(4):
                p0 = p1 = 0
                for lane in range(64):
                    kg, m = lane >> 4, lane & 15
                    c = codes[4 * kg + r][16 * nt + m]
                    p0 |= (c & 1) << lane
                    p1 |= ((c >> 1) & 1) << lane
                for kg in range(4):
                    w0, w1 = (p0 >> (16 * kg)) & M32, (p1 >> (16 * kg)) & M32
                    route[4 * kg + r][nt] = perm(w1, w0, 0x05010400)
        for bl in range(16):
            block = b"".join(d.to_bytes(4, "little") for d in route[bl])     # the record's 16 code bytes
            for c8 in range(8):
                assert block[2 * c8] | (block[2 * c8 + 1] << 8) == planes_of(codes[bl][8 * c8:8 * c8 + 8])
            got = route_codes(torch.tensor(list(block), dtype=torch.uint8))
            assert got.tolist() == codes[bl]
