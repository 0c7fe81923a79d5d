"""Host-side checks of the padded K-outer LDS image used by gemmt_kk_kernel
(csrc/kernels/gemmt.hip): the LDS-DMA lane -> element map covers every
element of a half image exactly once, the fragment addresses formed as
"lane base + compile-time immediate" equal the logical ones, and every
32-lane group of a ds_read_b64_tr_b16 touches 64 distinct banks
(bank = (byte / 4) mod 64, MI355X_MICROARCH.md LDS table)."""
PITCH, HALF_ROWS, PIECES = 288, 64, 18


def swap23(r):
    return (r & ~12) | ((r & 4) << 1) | ((r & 8) >> 1)


def phys(r, col):
    return swap23(r) * PITCH + col * 2


def test_dma_covers_half_image_once():
    seen = {}
    for q in range(PIECES):
        for lane in range(64):
            b = q * 1024 + lane * 16
            prow, w = divmod(b, PITCH)
            if w >= 256:
                continue   # pad slot
            r = swap23(prow)
            assert phys(r, w // 2) == b
            key = (r, w // 16)
            assert key not in seen
            seen[key] = b
    assert len(seen) == HALF_ROWS * 16


def _lane_base(lane):
    g, i = lane >> 4, lane & 15
    return swap23(8 * g + (i >> 2)) * PITCH + 8 * (i & 3)


def test_fragment_offsets_are_immediates():
    for ks in range(2):
        for mb in range(8):
            imm = ks * 32 * PITCH + mb * 32
            assert imm + 8 * PITCH < 65536
            for lane in range(64):
                g, i = lane >> 4, lane & 15
                col = mb * 16 + 4 * (i & 3)
                r = ks * 32 + 8 * g + (i >> 2)
                assert _lane_base(lane) + imm == phys(r, col)
                assert _lane_base(lane) + imm + 8 * PITCH == phys(r + 4, col)


def test_transposed_reads_bank_conflict_free():
    for ks in range(2):
        for mb in range(8):
            for second in (0, 8 * PITCH):
                for grp in range(2):
                    banks = set()
                    for lane in range(32 * grp, 32 * grp + 32):
                        a = _lane_base(lane) + ks * 32 * PITCH + mb * 32 + second
                        banks.update({(a // 4) % 64, (a // 4 + 1) % 64})
                    assert len(banks) == 64


def test_lds_budget_and_max_immediate():
    pt = 2 * HALF_ROWS * PITCH             # one operand tile
    assert 4 * pt <= 160 * 1024            # [A0][A1][B0][B1]
    # B reads: base holds 2 * A tile + half; immediates add buffer + k-step + block + 4 rows
    assert pt + 32 * PITCH + 7 * 32 + 8 * PITCH < 65536


def _slot128(r, c):
    return c ^ ((r >> 1) & 7)


def test_k_contiguous_reads_are_immediates():
    """K-contiguous operand (gemmt's 128-B-row image): row16's offset for
    16-row block mb equals the k-step's lane base (block 0) + mb * 2048, the
    immediate of gemmt_kk_kernel's asm ds_read_b128."""
    for w in range(2):
        for ks in range(2):
            for lane in range(64):
                r0 = lane & 15
                base = (w * 128 + r0) * 128 + (_slot128(r0, ks * 4 + (lane >> 4)) << 4)
                for mb in range(8):
                    r = w * 128 + mb * 16 + (lane & 15)
                    assert r * 128 + (_slot128(r, ks * 4 + (lane >> 4)) << 4) == base + mb * 2048
