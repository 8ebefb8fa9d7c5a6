"""Exhaustive check of the LDS granule swizzle of spconv_bf16.hip k_gemm_pipe (pswz): for every row
width G (16-B granules per row: 4, 8, 16) and K-step, every ds_read_b128 lane group of an MFMA A / B
fragment read (lane -> row lane & 15, granule ks*4 + lane >> 4) hits 16 distinct 16-B bank slots.
Lane groups from /opt/skills/guides/MI355X_MICROARCH.md (LDS table)."""
G1 = [0, 1, 2, 3, 12, 13, 14, 15] + list(range(20, 28))
G2 = [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19] + list(range(28, 32))
GROUPS = [G1, G2, [l + 32 for l in G1], [l + 32 for l in G2]]


def pswz(G, row):
    return row & 15 if G == 16 else (row >> 1) & (G - 1)


def conflict_free(G):
    for ks in range(G // 4):
        for base in (0, 16, 48, 112):          # B rows n*16 + r: the swizzle depends on r only
            for grp in GROUPS:
                slots = {((base + (l & 15)) * G + ((ks * 4 + (l >> 4)) ^ pswz(G, base + (l & 15)))) % 16 for l in grp}
                if len(slots) != 16:
                    return False
    return True


if __name__ == "__main__":
    for G in (4, 8, 16):
        print(G, conflict_free(G))
        assert conflict_free(G)
