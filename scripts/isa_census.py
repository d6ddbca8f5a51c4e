"""Instruction census of one kernel in an llvm-objdump listing: per basic block (split at
branch targets and branches), the count of MFMA / VALU / transcendental / SALU / LDS /
global-memory / wait instructions, so the issue budget of a loop body can be read off the
ISA (docs/performance.md, attention issue budget).

    python scripts/isa_census.py fa.s flash_bwd_dq2_kernelILb0E [--min-mfma 4]
"""
import argparse
import re
import sys

CATS = [
    ("mfma", re.compile(r"^v_mfma")),
    ("trans", re.compile(r"^v_(exp|log|rcp|rsq|sqrt|sin|cos)_")),
    ("valu", re.compile(r"^v_")),
    ("lds", re.compile(r"^ds_")),
    ("vmem", re.compile(r"^(global|buffer|flat|scratch)_")),
    ("wait", re.compile(r"^s_(waitcnt|barrier|nop|sleep)")),
    ("salu", re.compile(r"^s_")),
]


def census(lines):
    out = {k: 0 for k, _ in CATS}
    for op in lines:
        for k, rx in CATS:
            if rx.match(op):
                out[k] += 1
                break
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("listing")
    ap.add_argument("kernel", help="substring of the mangled kernel name")
    ap.add_argument("--min-mfma", type=int, default=1)
    a = ap.parse_args()
    text = open(a.listing).read().splitlines()
    start = None
    for i, l in enumerate(text):
        if l.endswith(">:") and a.kernel in l:
            start = i
            break
    if start is None:
        sys.exit(f"kernel {a.kernel} not found")
    body = []
    for l in text[start + 1:]:
        if l.endswith(">:"):
            break
        m = re.match(r"\s+(\w+)(.*?)//\s*([0-9A-Fa-f]+):", l)
        if m:
            body.append((int(m.group(3), 16), m.group(1), m.group(2).strip()))
    targets = set()
    for addr, op, args in body:
        if op.startswith("s_cbranch") or op == "s_branch":
            t = re.search(r"<[^>]*\+0x([0-9a-f]+)>", args)
            if t:
                targets.add(int(t.group(1), 16))
    base = body[0][0] if body else 0
    # objdump prints targets relative to the symbol: normalise to absolute addresses
    targets = {base + t - (body[0][0] - base) if False else t for t in targets}
    blocks, cur, cur_start = [], [], None
    fn_off = base
    for addr, op, args in body:
        rel = addr - fn_off
        if (rel in targets or addr in targets) and cur:
            blocks.append((cur_start, cur))
            cur, cur_start = [], None
        if cur_start is None:
            cur_start = rel
        cur.append(op)
        if op.startswith("s_cbranch") or op == "s_branch":
            blocks.append((cur_start, cur))
            cur, cur_start = [], None
    if cur:
        blocks.append((cur_start, cur))
    tot = census([op for _, b in blocks for op in b])
    print(f"{a.kernel}: {len(body)} instructions, {len(blocks)} blocks; whole kernel {tot}")
    for s, b in blocks:
        c = census(b)
        if c["mfma"] >= a.min_mfma:
            v = c["valu"] + c["trans"]
            print(f"  block +0x{s:x}: {len(b):5d} instr | " + " ".join(f"{k}={c[k]}" for k, _ in CATS)
                  + f" | VALU/MFMA={v / max(c['mfma'], 1):.2f} SALU/MFMA={c['salu'] / max(c['mfma'], 1):.2f}")


if __name__ == "__main__":
    main()
