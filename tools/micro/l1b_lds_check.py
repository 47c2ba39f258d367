"""Host-side check of the layer-1 backward's LDS x tiles (convnet_fused.hip).

``main``: the opt-in level-pair layout (LV_RS / LV_OB): emulates the staging writes (bf16 pairs in
copies E and O, 16-bit stores for O's split pairs) and every lane's B-operand read of every K-step,
and checks (a) each read returns the packed pair (column c0, c0 + 1) of the right row, (b) no
ds_read_b32 lane half (lanes 0-31, 32-63) touches two different addresses in one bank.  Prints
'mismatches 0 conflicted 0' when both hold.

``word_layout``: the default word layout (LM_XS = 137, ones block at LM_ONES): every data lane's
read returns its tap's word, the sum-dz lanes (n = 25) read 1.0, and no lane half touches two
addresses in one bank.  At the old stride 80 (constants at columns 72..75, absolute) the same
emulation with the old constants counts 1280 extra bank cycles over the 1024 half-wave reads of a tile."""
import numpy as np

LB_XR, LV_RS, LV_OB = 20, 41, 837


def bf(level):
    return int(np.float32(level).view(np.uint32)) >> 16


def main():
    tile = np.random.default_rng(0).integers(0, 256, (LB_XR, 72))
    mem = np.zeros(LV_OB + LB_XR * LV_RS, dtype=np.int64)
    for rr in range(LB_XR):
        for cv in range(18):
            f = [bf(tile[rr, 4 * cv + k]) for k in range(4)]
            e, o = rr * LV_RS + 2 * cv, LV_OB + rr * LV_RS + 2 * cv
            mem[e], mem[e + 1], mem[o] = f[0] | f[1] << 16, f[2] | f[3] << 16, f[1] | f[2] << 16
            mem[o + 1] = (mem[o + 1] & 0xFFFF0000) | f[3]
            if cv > 0:
                mem[o - 1] = (mem[o - 1] & 0xFFFF) | f[0] << 16
    bad = conflicted = 0
    for rp in range(8):
        for sg in range(4):
            for blk in range(2):
                for j in range(4):
                    wi, dr2 = j >> 1, j & 1
                    banks = {}
                    for g in range(4):
                        for li in range(16):
                            n = 16 * blk + li
                            t = min(n, 24)  # constant columns read tap 24's address (broadcast)
                            ky, kx = t // 5, t % 5
                            lof = LV_OB + ky * LV_RS + (kx + 1 + 4 * g) // 2 if kx & 1 else ky * LV_RS + (kx + 2 + 4 * g) // 2
                            a = lof + 2 * rp * LV_RS + 8 * sg + dr2 * LV_RS + wi
                            if n < 25:
                                r, c0 = 2 * rp + ky + dr2, kx + 2 + 4 * g + 16 * sg + 2 * wi
                                bad += int(mem[a]) != (bf(tile[r, c0]) | bf(tile[r, c0 + 1]) << 16)
                            banks.setdefault((g // 2, a % 32), set()).add(a)
                    conflicted += any(len(s) > 1 for s in banks.values())
    print("mismatches", bad, "conflicted", conflicted)
    return bad == 0 and conflicted == 0


LM_XS, LM_ONES = 137, 137 + 80
ONE = 0x3F800000


def word_layout(xs=LM_XS, ones=LM_ONES):
    tile = np.random.default_rng(1).integers(0, 256, (LB_XR, 72))
    mem = np.zeros(LB_XR * xs, dtype=np.int64)
    for rr in range(LB_XR):
        mem[rr * xs:rr * xs + 72] = [int(np.float32(v).view(np.uint32)) for v in tile[rr]]
        mem[rr * xs + 72:(rr + 1) * xs] = ONE
    bad = extra = 0
    for rp in range(8):
        for sg in range(4):
            base = 2 * rp * xs + 16 * sg
            for blk in range(2):
                for j in range(8):
                    wi, dr2, dc = j >> 2, (j >> 1) & 1, j & 1
                    for half in range(2):
                        banks = {}
                        for g in (2 * half, 2 * half + 1):
                            for li in range(16):
                                n = 16 * blk + li
                                t = min(n, 24)
                                off = ones if n == 25 else (t // 5) * xs + t % 5 + 2 + 4 * g
                                a = base + off + dr2 * xs + 2 * wi + dc
                                if n < 25:
                                    r, c = 2 * rp + t // 5 + dr2, t % 5 + 2 + 4 * g + 16 * sg + 2 * wi + dc
                                    bad += int(mem[a]) != int(np.float32(tile[r, c]).view(np.uint32))
                                elif n == 25:
                                    bad += int(mem[a]) != ONE
                                banks.setdefault(a % 32, set()).add(a)
                        extra += max(len(v) for v in banks.values()) - 1
    print("word layout: mismatches", bad, "extra bank cycles", extra)
    return bad == 0 and extra == 0


if __name__ == "__main__":
    raise SystemExit(0 if main() and word_layout() else 1)
