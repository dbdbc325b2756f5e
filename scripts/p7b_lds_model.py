"""LDS bank model of the fused CNN's conv2-dgrad A reads (cnn_fused.hip P7b).

Each wave runs one M-tile (16 r1 cells, lane lr = cell) over 19 k-steps; lane group lg reads the 16-byte co
group (g % 3) of tap g / 3 (g = 4 ks + lg) at source position (Y - ky, X - kx) of the 8x8 conv2-output
gradient, or a shared zero block when that position is outside.  A ds_read_b128 is serviced in 4 lane groups
of 16 (MI355X_MICROARCH.md LDS table), one LDS cycle per distinct dword address on the busiest bank; 4 cycles
per wave-instruction is conflict-free.

Prints the mean cycles per A read for the plain [pos][40] channel-last rows and searches linear layouts
offset(Y, X, cg) = Y RP + X P + cg Q (bytes, 16-byte slots that never overlap).  The kernel uses
P = 48, RP = 528, Q = 256 (d2n_ofs).
"""
from __future__ import annotations

import argparse

GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[lane + 32 for lane in g] for g in GROUPS]
CG, NGD, KSD = 3, 75, 19
ZERO = -16  # the zero block: one address shared by every out-of-range lane


def tiles_linear():
    return [[((t * 16 + lr) // 12, (t * 16 + lr) % 12) for lr in range(16)] for t in range(9)]


def cycles(tiles, addr) -> float:
    tot = n = 0
    for cells in tiles:
        for ks in range(KSD):
            a = []
            for lane in range(64):
                lr, lg = lane & 15, lane >> 4
                ty, tx = cells[lr]
                g = ks * 4 + lg
                v = ZERO
                if g < NGD:
                    tap, cg = divmod(g, CG)
                    ky, kx = divmod(tap, 5)
                    y, x = ty - ky, tx - kx
                    if 0 <= y < 8 and 0 <= x < 8:
                        v = addr(y, x, cg)
                a.append(v)
            c = 0
            for grp in GROUPS:
                banks: dict[int, set[int]] = {}
                for lane in grp:
                    for d in range(4):
                        dw = a[lane] // 4 + d
                        banks.setdefault(dw % 64, set()).add(dw)
                c += max(len(s) for s in banks.values())
            tot += c
            n += 1
    return tot / n


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--search", action="store_true", help="search (P, RP, Q) layouts (slow)")
    args = ap.parse_args()
    tl = tiles_linear()
    print("plain [pos][40] rows:", round(cycles(tl, lambda y, x, c: (y * 8 + x) * 80 + c * 16), 2))
    print("kernel layout (48, 528, 256):", round(cycles(tl, lambda y, x, c: y * 528 + x * 48 + c * 256), 2))
    if not args.search:
        return
    res = []
    for p in (16, 32, 48, 80, 112):
        for rpm in range(8, 13):
            rp = rpm * p
            for q in range(16, 1100, 16):
                offs = sorted(y * rp + x * p + c * q for y in range(8) for x in range(8) for c in range(3))
                if any(b - a < 16 for a, b in zip(offs, offs[1:])) or offs[-1] + 16 > 6144:
                    continue
                res.append((round(cycles(tl, lambda y, x, c, p=p, rp=rp, q=q: y * rp + x * p + c * q), 2),
                            p, rp, q, offs[-1] + 16))
    for r in sorted(res)[:10]:
        print("cycles %.2f  P %d  RP %d  Q %d  bytes/image %d" % r)


if __name__ == "__main__":
    main()
