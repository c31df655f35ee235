"""Instruction mix of a kernel's basic blocks from a hipcc -S listing (gfx950).

    python3 tools/isa_mix.py FILE.s KERNEL_SUBSTRING [--top N]

Prints, for the N blocks with the most v_mad_u64_u32 (the comb loop bodies), the count of each
mnemonic class; and the kernel's totals.  Used to attribute k_verify's non-MAD issue."""
import collections
import re
import sys


def blocks(lines, kernel):
    start = None
    for i, l in enumerate(lines):
        if l.startswith(kernel + ":"):
            start = i
            break
    if start is None:
        raise SystemExit("kernel not found")
    cur, name = [], "entry"
    out = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            out.append((name, cur))
            name, cur = m.group(1), []
            continue
        t = l.strip()
        if not t or t.startswith(";") or t.startswith("."):
            continue
        cur.append(t.split()[0])
    out.append((name, cur))
    return out


def main():
    path, kern = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 4
    lines = open(path).read().splitlines()
    bl = blocks(lines, kern)
    tot = collections.Counter()
    for _, ins in bl:
        tot.update(ins)
    ranked = sorted(bl, key=lambda b: -sum(1 for x in b[1] if x == "v_mad_u64_u32"))[:top]
    for name, ins in ranked:
        c = collections.Counter(ins)
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        print("== %s: %d instrs, %d VALU, %d v_mad_u64_u32, %d s_nop" % (name, len(ins), valu, c["v_mad_u64_u32"],
                                                                          c["s_nop"]))
        for k, v in c.most_common(40):
            print("   %-28s %5d" % (k, v))
    valu = sum(v for k, v in tot.items() if k.startswith("v_"))
    print("== kernel total: %d instrs, %d VALU, %d v_mad_u64_u32" % (sum(tot.values()), valu, tot["v_mad_u64_u32"]))


if __name__ == "__main__":
    main()
