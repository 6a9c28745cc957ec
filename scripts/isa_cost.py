"""Estimated VALU issue cost of the hot loop of a kernel in a hipcc -S listing.

usage: python scripts/isa_cost.py file.s kernel_substring pixels_per_iteration [min_block_len]

Costs are cycles per wave64 instruction on gfx950 as measured by
scripts/ubench/valu_rate.hip (profiles/ubench_valu_rates_*.txt): the plain
32-bit add/sub/logic/right-shift ops and the 16-bit VOP2 ops issue at ~2
cycles, everything else (VOPC, v_cndmask, v_dot4, mad24/mul24, bfe, perm,
3-operand ops, packed ops, SDWA/DPP forms, v_lshlrev_b32) at ~4, and
v_mad_u16 / v_med3_*16 / v_max3_i16 at ~8.  The largest basic block with at
least min_block_len instructions is taken as the loop body.
"""
import collections
import re
import sys

FULL = {
    "v_mov_b32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_not_b32", "v_add_u32", "v_sub_u32",
    "v_subrev_u32", "v_lshrrev_b32", "v_ashrrev_i32", "v_add_u16", "v_sub_u16", "v_subrev_u16",
    "v_mul_lo_u16", "v_lshlrev_b16", "v_lshrrev_b16", "v_ashrrev_i16", "v_max_u16", "v_min_u16",
    "v_max_i16", "v_min_i16",
}
QUARTER = {"v_mad_u16", "v_mad_i16", "v_med3_i16", "v_med3_u16", "v_max3_i16", "v_max3_u16",
           "v_min3_i16", "v_min3_u16", "v_mad_u64_u32", "v_mad_i64_i32"}


def cost(op, line):
    if not op.startswith("v_"):
        return 0.0
    base = op.replace("_e32", "").replace("_e64", "").replace("_sdwa", "").replace("_dpp", "")
    if "sdwa" in op or "dpp" in op or "row_" in line or "_sel:" in line:
        return 4.0
    if base in QUARTER:
        return 8.0
    if base in FULL and "_e64" not in op:
        return 2.0
    if base in FULL:  # VOP3 encoding of a VOP2 op (modifiers/sgpr operands); assume full rate
        return 2.0
    return 4.0


def main():
    path, name, ppi = sys.argv[1], sys.argv[2], float(sys.argv[3])
    minlen = int(sys.argv[4]) if len(sys.argv) > 4 and sys.argv[4].isdigit() else 100
    s = open(path).read()
    st = [m.start() for m in re.finditer(r"^(_Z\S*" + re.escape(name) + r"\S*):", s, re.M)][0]
    body = s[st:s.index(".Lfunc_end", st)].split("\n")
    print(body[0])
    blocks, cur = [], None
    for line in body[1:]:
        t = line.strip()
        if re.match(r"^(\.LBB\S+|;\s*%bb\.\d+):", t) or t.startswith("; %bb."):
            cur = [t.split()[0] if not t.startswith(";") else t, []]
            blocks.append(cur)
            continue
        if not t or t.startswith((".", ";")) or cur is None:
            continue
        cur[1].append((t.split()[0], t))
    big = max((b for b in blocks if len(b[1]) >= minlen), key=lambda b: len(b[1]), default=None)
    if big is None:
        sys.exit("no block")
    # whole innermost loop: every block whose header comment names the same loop
    hdr = None
    for line in body:
        if big[0] in line and "Loop: Header=" in line:
            hdr = line.split("Loop: Header=")[1].split()[0]
            depth = line.split("Depth=")[1].split()[0]
    if hdr is not None and "--loop" in sys.argv:
        loop_blocks = [b for b in blocks if any(hdr in l and f"Depth={depth}" in l for l in body
                                                if l.strip().startswith(b[0]))]
        merged = [big[0] + "..", [x for lb in loop_blocks for x in lb[1]]]
        print(f"loop {hdr} depth {depth}: {len(loop_blocks)} blocks")
        big = merged
    c = collections.Counter()
    cyc = collections.Counter()
    for op, line in big[1]:
        c[op] += 1
        cyc[op] += cost(op, line)
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    total = sum(cyc.values())
    lds = sum(v for k, v in c.items() if k.startswith("ds_"))
    print(f"block {big[0]}: {len(big[1])} instr, {valu} VALU, {lds} LDS; est {total:.0f} VALU cycles "
          f"= {total / ppi:.1f} cycles/px, {valu / ppi:.1f} VALU instr/px")
    for op, v in sorted(cyc.items(), key=lambda kv: -kv[1])[:30]:
        print(f"  {op:28s} n={c[op]:4d}  cyc={v:6.0f}  per_px={v / ppi:5.2f}")


if __name__ == "__main__":
    main()
