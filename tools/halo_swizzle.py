"""Bank-conflict check of conv3x3_gn_p4_kernel's halo B reads (ds_read_b128) under a row swizzle, for every
row offset a tap can give, both operand forms (CPU only; measurement aid, never part of the product).

Halo row h (128 B = 64 bf16 channels) holds its eight 16-B units XOR-permuted: unit u at u ^ f(h). ds_read_b128
serves a wave in four 16-lane groups over 64 banks (MI355X_MICROARCH.md, LDS table); a group is conflict-free when
its 16 lanes hit 16 distinct 16-B slots of a 256-B bank line: slot = (h & 1) * 8 + (u ^ f(h)).
  16x16x32 (p4's M16 form): lane = pixel m (lane & 15) x k-group kg (lane >> 4), unit kg (^ 4 for the second half-step)
  32x32x16 (p4's other forms, p5): lane = pixel (lane & 31) x half hh (lane >> 5), unit 2 kk + hh
    python tools/halo_swizzle.py          (p4's 256-pixel halo: rows contiguous per 16-pixel block)
    python tools/halo_swizzle.py --p5     (conv3x3_gn_p5_kernel's 128-pixel tiles: a 32-pixel block spans image rows /
                                           whole 4x4 images, so a group's rows are not contiguous; slot = (hx & 1, f))
"""
import sys
GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[l + 32 for l in g] for g in GROUPS]


def conflicts(f, lane, unit, offsets):
    """Lanes that repeat a slot, summed over row offsets, groups and unit variants."""
    bad = 0
    for r0 in offsets:
        for v in unit:
            for g in GROUPS:
                seen = set()
                for l in g:
                    row, k = lane(l)
                    h = r0 + row
                    slot = ((h & 1) << 3) | (v(k) ^ f(h))
                    bad += slot in seen
                    seen.add(slot)
    return bad


def main():
    m16 = (lambda l: (l & 15, l >> 4), [lambda k: k, lambda k: k ^ 4])
    m32 = (lambda l: (l & 31, l >> 5), [lambda h, kk=kk: 2 * kk + h for kk in range(4)])
    for name, f in (("(h >> 1) & 7", lambda h: (h >> 1) & 7), ("h & 6", lambda h: h & 6)):
        print(f"{name:14s} 16x16x32: {conflicts(f, *m16, range(64)):5d} conflicting lanes   "
              f"32x32x16: {conflicts(f, *m32, range(64)):5d}")


def p5_conflicts(W, f):
    """conv3x3_gn_p5_kernel<W>'s 32x32x16 B reads: pixel block j (32 px) of a 128-pixel tile of whole images (W <= 8,
    halo rows (seg, y + 1 + ...)) or of 128 / W rows of one image (W >= 16); f(hy, hx, h) -> unit XOR."""
    rows_mode = W * W > 128
    th = 128 // W if rows_mode else W
    w2 = W + 2
    hs, spx = (th + 2) * w2, th * W
    bad = 0
    for j in range(4):
        for g in GROUPS[:2]:  # (lanes + 32: the other half hh, a uniform XOR: the same count)
            for ky in range(3):
                for kx in range(3):
                    seen = set()
                    for rl in g:
                        pl = 32 * j + rl
                        seg, rem = divmod(pl, spx)
                        y, x = divmod(rem, W)
                        hy, hx = y + ky, x + kx
                        h = seg * hs + hy * w2 + hx
                        slot = ((h & 1) << 3) | f(hy, hx, h)
                        bad += slot in seen
                        seen.add(slot)
    return bad


def main_p5():
    shipped = {4: lambda hy, hx, h: (hy + 2 * hx) & 7, 8: lambda hy, hx, h: (hy + 2 * hx) & 7,
               16: lambda hy, hx, h: (hy + hx) & 7, 32: lambda hy, hx, h: (h >> 1) & 7, 64: lambda hy, hx, h: (h >> 1) & 7}
    for W, f in shipped.items():
        print(f"p5<{W:2d}>  (h >> 1) & 7: {p5_conflicts(W, lambda hy, hx, h: (h >> 1) & 7):4d} conflicting lanes   "
              f"shipped swz: {p5_conflicts(W, f):4d}")


if __name__ == "__main__":
    main_p5() if "--p5" in sys.argv else main()
