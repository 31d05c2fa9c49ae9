#!/usr/bin/env python3
"""Offline LDS bank-conflict model of the MNIST step's hot LDS accesses.

Banking rules are the CDNA4 table in /opt/skills/guides/MI355X_MICROARCH.md
(section LDS): per instruction, a wave64 access is serviced in fixed lane
groups; within a group, identical dword addresses broadcast and each extra
distinct address on a bank costs one LDS cycle.  Validated against
tools/probes/lds_patterns.hip on the GPU (profiles/lds_conflicts_r3.md).

Each pattern is a function lane -> byte address for one wave-instruction;
`extra(kind, addrs)` is the number of conflict cycles it adds.
Usage: python tools/lds_bank_model.py
"""
from __future__ import annotations

from collections import defaultdict

B128_GROUPS = [
    [*range(0, 4), *range(12, 16), *range(20, 28)],
    [*range(4, 12), *range(16, 20), *range(28, 32)],
    [*range(32, 36), *range(44, 48), *range(52, 60)],
    [*range(36, 44), *range(48, 52), *range(60, 64)],
]
HALVES = [list(range(32)), list(range(32, 64))]
QUARTERS = [list(range(16 * i, 16 * i + 16)) for i in range(4)]
EIGHTHS = [list(range(8 * i, 8 * i + 8)) for i in range(8)]

# kind -> (lane groups, dwords per lane, banks)
KINDS = {
    "read_b32": (HALVES, 1, 32),
    "read_b64": (HALVES, 2, 64),
    "read_b128": (B128_GROUPS, 4, 64),
    "write_b32": (HALVES, 1, 32),
    "write_b64": (QUARTERS, 2, 32),
    "write_b128": (EIGHTHS, 4, 32),
}


def extra(kind: str, addrs, active=None) -> int:
    """Conflict cycles of one wave-instruction; addrs[lane] = byte address
    (None or lanes outside `active` = exec-masked)."""
    if kind == "read2_b32":  # two ds_read_b32 at addr and addr + 4
        a0 = [None if a is None else a for a in addrs]
        a1 = [None if a is None else a + 4 for a in addrs]
        return extra("read_b32", a0, active) + extra("read_b32", a1, active)
    groups, nd, nb = KINDS[kind]
    total = 0
    for grp in groups:
        per_bank = defaultdict(set)
        for ln in grp:
            a = addrs[ln]
            if a is None or (active is not None and ln not in active):
                continue
            d0 = a // 4
            for k in range(nd):
                per_bank[(d0 + k) % nb].add(d0 + k)
        if per_bank:
            total += max(len(v) for v in per_bank.values()) - 1
    return total


def f(dw):  # dword offset -> byte address
    return 4 * dw


# ---------------------------------------------------------------- probes
def probe_rules():
    kh = lambda c: c // 5  # noqa: E731
    modes = {
        "consecutive": lambda l: l,
        "one address": lambda l: 0,
        "lane&15": lambda l: l & 15,
        "lane>>2": lambda l: l >> 2,
        "wgrad patch": lambda l: kh(l & 15) * 12 + (l & 15) % 5 + 2 * (l >> 4),
        "patch w/o 2g": lambda l: kh(l & 15) * 12 + (l & 15) % 5,
        "stride 2": lambda l: 2 * l,
        "one bank": lambda l: 64 * l,
    }
    print("probe rules (model; GPU measured b32/read2/b64: 0 0 0 0 2 2 2 62 | 0 0 0 0 4 4 4 124 | 0 0 0 0 2 2 2 62)")
    for name, fn in modes.items():
        a = [f(fn(l) & 4095) for l in range(64)]
        b64 = [f(2 * (fn(l) & 4095)) for l in range(64)]
        print(f"  {name:14s} b32 {extra('read_b32', a):3d}  read2 {extra('read2_b32', a):3d}  "
              f"b64 {extra('read_b64', b64):3d}")


# ---------------------------------------------------------------- F12
def f12(xs_ld=28):
    """conv1 patch reads (ds_read_b64 of xs rows) and conv2 A/B operand reads."""
    out = {}
    tot = 0
    for task_half in (0, 1):
        for r in range(6):
            for c in (0, 2, 4):
                addrs = []
                for l in range(64):
                    pix = task_half * 64 + l
                    if pix >= 144:
                        addrs.append(None)
                        continue
                    ph, pw = divmod(pix, 12)
                    addrs.append(f((2 * ph + r) * xs_ld + 2 * pw + c))
                tot += extra("read_b64", addrs)
    out["conv1 xs reads per 2 full tasks"] = tot
    # conv2 A reads: il + ic*144 + kh*12 + j, lane map i = lane&15, g = lane>>4
    tot = 0
    for t in range(4):
        for G in range(25):
            for j in range(5):
                addrs = []
                for l in range(64):
                    i, g = l & 15, l >> 4
                    pw, dy, dx = i >> 2, (i >> 1) & 1, i & 1
                    R = 4 * G + g
                    ic, kh = divmod(R, 5)
                    addrs.append(f((2 * t + dy) * 12 + 2 * pw + dx + ic * 144 + kh * 12 + j))
                tot += extra("read_b32", addrs)
    out["conv2 A reads, all 4 t x 25 G x 5 (b32)"] = tot
    return out


def main():
    probe_rules()
    for ld in (28, 44):
        print(f"F12 xs stride {ld}:", f12(ld))


if __name__ == "__main__":
    main()


# ---------------------------------------------------------------- wgrad
def wgrad_patch(rs=12, ps=144, ntw=1):
    """conv2 wgrad MFMA loop: per sample and pooled row G, the read2_b32 pairs
    (ap[0], ap[1]) and (ap[rs], ap[rs+1]) of every lane, all 32 column tiles.
    as plane layout: row stride rs, channel stride ps (dwords)."""
    tot = 0
    for nt in range(32):
        col0 = nt * 16
        ic0 = col0 // 25
        koff = []
        for c in range(16):
            kk = col0 + c
            if kk < 500:
                ic, r25 = divmod(kk, 25)
                kh, kw = divmod(r25, 5)
                koff.append((ic - ic0) * ps + kh * rs + kw)
            else:
                koff.append(0)
        for G in range(4):
            for j in (0, rs):
                addrs = [f(koff[l & 15] + 2 * rs * G + 2 * (l >> 4) + j) for l in range(64)]
                tot += extra("read2_b32", addrs)
    return tot


def search_wgrad():
    best = []
    for rs in range(12, 33, 4):
        for pres in range(0, 32, 2):
            ps = 12 * rs + ((pres - 12 * rs) % 32)
            best.append((wgrad_patch(rs, ps), rs, ps))
    best.sort()
    print("wgrad patch conflicts per sample (all 32 tiles), current rs=12 ps=144:", wgrad_patch())
    print("  best (conflicts, row stride, plane stride):", best[:6])


# ---------------------------------------------------------------- conv1 wgrad gather (dgrad blocks)
def conv1_gather(xld=28, seed=0, trials=8):
    """c2_dgrad_block's conv1 weight grad: lane = pooled pixel (72 per wave),
    25 code-dependent b32 reads xs[(2py+dy+kh)*xld + 2px+dx+kw]; mean conflict
    cycles per wave over random argmax codes."""
    import random

    rnd = random.Random(seed)
    tot = 0
    for _ in range(trials):
        for p0 in (0, 72):
            codes = [rnd.randrange(4) for _ in range(72)]
            for it in (0, 1):
                for kh in range(5):
                    for kw in range(5):
                        addrs = []
                        for l in range(64):
                            pl = l + 64 * it
                            if pl >= 72:
                                addrs.append(None)
                                continue
                            pix = p0 + pl
                            py, px = divmod(pix, 12)
                            cd = codes[pl]
                            addrs.append(f((2 * py + (cd >> 1) + kh) * xld + 2 * px + (cd & 1) + kw))
                        tot += extra("read_b32", addrs)
    return tot / (trials * 2)
