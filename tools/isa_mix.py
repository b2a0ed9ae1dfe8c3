#!/usr/bin/env python3
"""Instruction mix of one kernel in a gfx950 .s file (from `make isa`): totals per mnemonic,
and per basic block so the hot loops can be read off.  Usage: isa_mix.py FILE.s KERNEL_SUBSTR [BLOCK]

With BLOCK (a label such as .LBB4_52, the Straus loop body), that block is broken into classes
and weighted by the measured issue cost per instruction at 2 waves/SIMD
(profiles/r02/micro/issue_probe.jsonl; unmeasured VOP3 ops take the VOP3 median 4.5 cycles,
VOP2 (_e32) ops 2.5), so the share of issue cycles left to non-mad work can be read off."""
import collections
import re
import sys

# cycles per wave instruction at 2 waves/SIMD (issue_probe.jsonl, cyc_per_instr_2w)
CYC = {"v_mad_i64_i32": 5.25, "v_mad_u64_u32": 5.57, "v_add_u32_e32": 2.96, "v_add_u32": 2.96,
       "v_mul_lo_u32": 5.06, "v_ashrrev_i64": 4.97, "v_lshl_add_u64": 4.73, "v_lshl_add_u32": 4.98,
       "v_and_b32_e32": 2.57, "v_alignbit_b32": 4.71, "v_add3_u32": 4.82, "v_lshlrev_b32_e32": 4.24,
       "v_mad_i32_i24": 4.65, "v_sub_u32_e32": 2.50, "v_bfe_u32": 4.52}
CLASS = [("mad (v_mad_i64_i32)", ("v_mad_i64_i32",)),
         ("operand pre-multiplies x19/x38 (v_mul_lo_u32)", ("v_mul_lo_u32",)),
         ("carry: 64-bit shifts", ("v_ashrrev_i64", "v_lshrrev_b64", "v_lshlrev_b64")),
         ("carry: 64-bit adds", ("v_lshl_add_u64",)),
         ("limb masks (v_and)", ("v_and_b32_e32",)),
         ("32-bit add/sub (x2 copies, fe_add/fe_sub, limb bias)", ("v_add_u32_e32", "v_add_u32", "v_sub_u32_e32",
                                                                  "v_add3_u32", "v_sub_u32_sdwa", "v_add_u32_sdwa")),
         ("table unpack / sign select", ("v_alignbit_b32", "v_cndmask_b32_e32", "v_cndmask_b32_e64", "v_or_b32_e32",
                                        "v_lshlrev_b32_e32", "v_lshrrev_b32_e32", "v_perm_b32", "v_bfe_u32",
                                        "v_ashrrev_i32_e32"))]


def cost(op):
    if op in CYC:
        return CYC[op]
    if op.startswith("s_") or op.startswith("global_") or op.startswith("flat_") or op.startswith("ds_") \
            or op.startswith("buffer_"):
        return 0.0  # not VALU issue
    return 2.5 if op.endswith("_e32") else 4.5


def block_report(c):
    n = sum(c.values())
    mads = c.get("v_mad_i64_i32", 0)
    tot_cyc = sum(cost(op) * k for op, k in c.items())
    print("\nblock: %d instructions, %d v_mad_i64_i32 (%.2f instructions per mad), %.0f issue cycles"
          % (n, mads, n / max(mads, 1), tot_cyc))
    seen = set()
    print("%-58s %7s %9s %8s %7s" % ("class", "instr", "per 100 mad", "cycles", "share"))
    for name, ops in CLASS:
        k = sum(c.get(o, 0) for o in ops)
        cy = sum(cost(o) * c.get(o, 0) for o in ops)
        seen.update(ops)
        print("%-58s %7d %9.1f %8.0f %6.1f%%" % (name, k, 100.0 * k / max(mads, 1), cy, 100 * cy / tot_cyc))
    rest = {o: k for o, k in c.items() if o not in seen}
    k = sum(rest.values())
    cy = sum(cost(o) * v for o, v in rest.items())
    print("%-58s %7d %9.1f %8.0f %6.1f%%" % ("other (loads, scalar, moves, compares)", k, 100.0 * k / max(mads, 1), cy,
                                             100 * cy / tot_cyc))


def main():
    path, name = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^[_A-Za-z0-9]+:\s*(;.*)?$", l) and name in l and not l.startswith(".L"):
            start = i
            break
    if start is None:
        sys.exit("kernel not found")
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    body = lines[start:end]
    tot = collections.Counter()
    blocks = []
    cur = ("entry", collections.Counter())
    for l in body:
        s = l.strip()
        if s.startswith(".LBB"):
            blocks.append(cur)
            cur = (s.split(":")[0], collections.Counter())
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        op = s.split()[0]
        tot[op] += 1
        cur[1][op] += 1
    blocks.append(cur)
    print("total instructions", sum(tot.values()))
    for op, c in tot.most_common(40):
        print("%6d %s" % (c, op))
    if len(sys.argv) > 3:
        for lab, c in blocks:
            if lab == sys.argv[3]:
                block_report(c)
        return
    print("\nblocks (size >= 200):")
    for lab, c in blocks:
        n = sum(c.values())
        if n >= 200:
            top = ", ".join("%s %d" % kv for kv in c.most_common(8))
            print("%s  %d : %s" % (lab, n, top))


if __name__ == "__main__":
    main()
