"""LDS bank-conflict model of the attention kernels' image reads (not a test).

Bank rule (cdna_hip_programming.md §2, MI355X_MICROARCH.md §LDS): 64 banks of 4 bytes; ds_read_b128 is serviced
in four 16-lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32), ds_read_b64_tr_b16 in two 32-lane halves; each
extra distinct dword on one bank inside a group costs one LDS cycle.  For a [rows][D] bf16 image whose 16-byte
chunk ch of row r is stored at ch ^ f(r), prints the LDS cycles of the 32x32x16 operand reads the kernels issue:
  row reads: lane (r, h) reads row r, chunk 2s + h (lds_row_frag / DualOffs::rowf);
  transposed reads: lane 16G + 4q + p reads row 16s + 4h + q (+8), columns col0 + 16(G & 1) + 4p (tr_frag).
and searches every f that XORs the row's bits into the chunk index for the cheapest layout serving both.

usage: python tools/lds_bank_model.py
"""
import itertools

G128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
        list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
G128 += [[x + 32 for x in g] for g in G128]
G64 = [list(range(32)), list(range(32, 64))]


def cycles(addrs, groups, width):
    tot = 0
    for g in groups:
        banks = {}
        for lane in g:
            a = addrs[lane]
            for w in range(width // 4):
                banks.setdefault((a // 4 + w) % 64, set()).add(a // 4 + w)
        tot += max(len(v) for v in banks.values())
    return tot


def row_cost(off, D, rows=32):
    c = 0
    for base in range(0, rows, 32):
        for s in range(D // 16):
            c += cycles([off(base + (lane & 31), 2 * s + (lane >> 5)) for lane in range(64)], G128, 16)
    return c


def tr_cost(off, D, rows=32):
    c = 0
    for row0 in range(0, rows, 32):
        for s in range(2):
            for col0 in range(0, D, 32):
                for add in (0, 8):
                    ad = []
                    for lane in range(64):
                        G, i, h = lane >> 4, lane & 15, lane >> 5
                        q, p = i >> 2, i & 3
                        r = row0 + 16 * s + 4 * h + q + add
                        col = col0 + 16 * (G & 1) + 4 * p
                        ad.append(off(r, col // 8) + 8 * (p & 1))
                    c += cycles(ad, G64, 8)
    return c


def xor_layout(D, f):
    return lambda r, ch: r * 2 * D + 16 * (ch ^ f(r))


def parity_fn(masks):
    return lambda r: sum(((bin(r & m).count("1") & 1) << k) for k, m in enumerate(masks))


def main():
    for D in (64, 128):
        nch = D // 8
        ideal_row, ideal_tr = 4 * (D // 16), 2 * 4 * (D // 32)
        print(f"D = {D}: conflict-free costs row {ideal_row}, transposed {ideal_tr}")
        print("  row-only swizzle (ch ^ (r & 7)):", row_cost(xor_layout(D, lambda r: r & 7), D),
              tr_cost(xor_layout(D, lambda r: r & 7), D))
        if D == 64:
            f = lambda r: ((r >> 1) & 1) | (((r >> 2) & 1) << 1) | ((((r >> 1) ^ (r >> 3)) & 1) << 2)
        else:
            f = lambda r: ((r & 3) << 2) | ((r >> 2) & 3)
        print("  dual (dsw):", row_cost(xor_layout(D, f), D), tr_cost(xor_layout(D, f), D))
        if D == 64:   # exhaustive search over XORs of row bits 0..4 into the 3 chunk bits
            best = min((row_cost(xor_layout(D, parity_fn(m)), D) + tr_cost(xor_layout(D, parity_fn(m)), D), m)
                       for m in itertools.product(range(32), repeat=(nch - 1).bit_length()))
            print("  best XOR layout found: cost", best[0], "masks", best[1])


if __name__ == "__main__":
    main()
