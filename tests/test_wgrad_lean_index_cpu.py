"""CPU specification of the lean conv2_wgrad kernels' index arithmetic (csrc/kernels/conv_bwd.hip).

The original kernel computed, per k-step and lane, the a1 tile pixel under dy pixel p of a chunk that
starts at global dy row c0 as

    blo_px = (a1_row_of(c0 + p // 24) - a1_row_of(c0)) * 26 + p % 24,   a1_row_of(R) = R + 2 (R // 24)

(a1 rows are 26 per image, dy rows 24).  The lean kernels precompute tb = p + 2 (p // 24) per
(k-step, lane) once and add 52 when the lane's dy row crossed the chunk's image boundary, tested as
c >= 24 bnd - 32 ks with bnd = 24 - c0 % 24 (a scalar per k-step).  The staging plan packs the
record offset, the 2x2-window code ((r0 + row) & 1, x & 1) and the chunk row into one register.
"""

H1, H2, HP, DYC_REC = 26, 24, 12, 144


def a1_row_of(r):
    return r + 2 * (r // H2)


def test_b_row_offsets_match_the_original_formula():
    for c0 in range(0, 3 * H2):                       # every chunk start phase within an image
        bnd = H2 - c0 % H2
        for ks in range(6):
            for gq in range(4):
                for q in range(4):
                    for h in range(2):
                        c = 4 * gq + q + 16 * h        # lo / hi pixel of the lane inside the k-step
                        p = 32 * ks + c
                        orig = (a1_row_of(c0 + p // H2) - a1_row_of(c0)) * H1 + (p - (p // H2) * H2)
                        lean = p + 2 * (p // H2) + (52 if c >= H2 * bnd - 32 * ks else 0)
                        assert orig == lean, (c0, ks, c)


def test_k_to_pixel_map_gives_8_consecutive_pixels_per_half_wave():
    # lane = 16 gq + 4 q + pp; the "lo" read of lanes 0-31 covers gq 0, 1 -> pixels 4 gq + q
    for h in range(2):
        for half in range(2):
            pix = sorted({4 * gq + q + 16 * h for gq in (2 * half, 2 * half + 1) for q in range(4)})
            assert pix == list(range(pix[0], pix[0] + 8)) and pix[0] % 8 == 0


def test_staging_plan_packing_roundtrips():
    for nth in (256, 512):
        for tid in range(nth):
            c8 = tid & 7
            for r0 in (0, 1, 7, 24, 4799):
                for i in range(24576 // 16 // nth):
                    pix = (tid >> 3) + (nth // 8) * i
                    pr, x = pix // H2, pix % H2
                    code = (((r0 + pr) & 1) << 1) | (x & 1)
                    rec = (x >> 1) * DYC_REC + c8 * 16 + (code << 12) + (pr << 16)
                    assert (x >> 1) * DYC_REC + c8 * 16 < 4096
                    assert rec & 0xFFF == (x >> 1) * DYC_REC + c8 * 16
                    assert (rec >> 12) & 3 == code and rec >> 16 == pr
