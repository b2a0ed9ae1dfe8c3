#!/usr/bin/env python3
"""Generates tendermint-fork_amd/csrc/fe_cols.h: the column accumulation of the GF(2^255-19) field
multiplication and squaring (fe25519.h) as explicit v_mad_i64_i32 schedules.

Why: written in C++, LLVM re-associates every column sum and adds the carry-rounding bias with a
separate 64-bit v_lshl_add_u64 at the end (10 per square, ~7 per multiplication; see
tools/micro/fe_micro.hip), and pinning the partial sums instead serialises the columns.  Here each
column starts with ONE mad whose 64-bit addend is the bias, and the mads are issued round-robin
over the ten columns, so consecutive mads never depend on each other (the nearest dependency is
>= 5 instructions away: no hazard wait states are needed inside the block).

The same schedule is emitted as plain C++ for the host build (tests/native/hostsim.cpp), so the
CPU test-suite checks exactly the operand choice the device code uses.

Usage: python3 tools/gen_fe_asm.py   (rewrites the header; commit the result)
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tendermint-fork_amd", "csrc", "fe_cols.h")

MULT = ["", "2", "4", "19", "38"]  # x[m][i] = f_i * {1, 2, 4, 19, 38}[m]


def mul_products():
    """(column, a, b) with a/b = (array, index): f*g schedule of fe_mul (radix 2^25.5)."""
    cols = {k: [] for k in range(10)}
    for i in range(10):
        for j in range(10):
            k = i + j
            a = ("f2", i) if (i & 1 and j & 1) else ("f", i)
            b = ("g19", j) if k >= 10 else ("g", j)
            cols[k % 10].append((a, b))
    return cols


def sq_products(D):
    """(column, a, b) of D * f^2: the operand split of fe_sq_acc (fe25519.h)."""
    cols = {k: [] for k in range(10)}
    for i in range(10):
        for j in range(i, 10):
            k = i + j
            wrap = k >= 10
            oo = (i & 1) and (j & 1)
            off = i < j
            c2 = (1 if off else 0) + (1 if oo else 0) + (1 if D == 2 else 0)
            if not wrap:
                ma, mb = {0: (0, 0), 1: (1, 0), 2: (1, 1), 3: (2, 1)}[c2]
            else:
                on_b = (j & 1) or not (i & 1)
                idx19 = j if on_b else i
                rest, m19 = c2, 3
                if (idx19 & 1) and rest > 0:
                    m19, rest = 4, rest - 1
                mo = rest
                ma, mb = (mo, m19) if on_b else (m19, mo)
            cols[k % 10].append((("x%s" % MULT[ma], i), ("x%s" % MULT[mb], j)))
    return cols


def schedule(cols):
    order = []
    r = 0
    while any(len(c) > r for c in cols.values()):
        for k in range(10):
            if len(cols[k]) > r:
                order.append((k, r, cols[k][r]))
        r += 1
    return order


def check_distance(order):
    last = {}
    for pos, (k, r, _) in enumerate(order):
        if k in last:
            assert pos - last[k] >= 2, "dependent mads too close"
        last[k] = pos


def cname(op):
    arr, i = op
    if arr in ("f", "g"):
        return "%s[%d]" % (arr, i)
    return "%s[%d]" % (arr, i)


def emit(fn_sig, order, inputs, doc):
    idx = {}
    operands_out = ['"=&v"(acc[%d])' % k for k in range(10)]
    operands_in = []
    for op in inputs:
        idx[op] = 10 + len(operands_in)
        operands_in.append('"v"(%s)' % cname(op))
    ib_e = 10 + len(operands_in)
    operands_in.append('"s"(be)')
    ib_o = ib_e + 1
    operands_in.append('"s"(bo)')
    lines = []
    for k, r, (a, b) in order:
        addend = ("%%%d" % (ib_e if k % 2 == 0 else ib_o)) if r == 0 else "%%%d" % k
        lines.append("v_mad_i64_i32 %%%d, vcc, %%%d, %%%d, %s" % (k, idx[a], idx[b], addend))
    host = []
    for k, r, (a, b) in order:
        prod = "(int64_t)%s * (int64_t)%s" % (cname(a), cname(b))
        if r == 0:
            host.append("  acc[%d] = %s + %s;" % (k, "be" if k % 2 == 0 else "bo", prod))
        else:
            host.append("  acc[%d] += %s;" % (k, prod))
    asm = "\n".join('      "%s\\n"' % l for l in lines)
    return """%s
%s {
  const int64_t be = (int64_t)1 << 25, bo = (int64_t)1 << 24;  // column biases (fe_bias)
#if defined(__HIP_DEVICE_COMPILE__)
  asm(
%s
      : %s
      : %s
      : "vcc");
#else
%s
#endif
}
""" % (doc, fn_sig, asm, ",\n        ".join(", ".join(operands_out[i:i + 5]) for i in range(0, 10, 5)),
       ",\n        ".join(", ".join(operands_in[i:i + 6]) for i in range(0, len(operands_in), 6)),
       "\n".join(host))


# ---------------------------------------------------------------- fused column sums + carries
# The chain (fe25519.h "Fused carry"): even columns are rounded (centered limbs), odd columns are
# floored (limbs in [0, 2^25)).  Column 0 starts from its bias 2^25, columns 1, 3, 5, 7 from the
# constant 2^50 (= the next even column's bias shifted by 25), column 9 from 0; each even column
# 2, 4, 6, 8 starts from the carry of the odd column below it (its first mad's addend: the carry
# costs no add), and each odd column takes the carry of the even column below it with one 64-bit
# add.  The wrap (column 9 -> 0, x19) and the last small carry 0 -> 1 follow in C++ (fe_fused_fin).
S = [26 if k % 2 == 0 else 25 for k in range(10)]
CARRIED = [2**25 if k % 2 == 0 else 2**25 + 2**16 for k in range(10)]  # |limb| bound of the carried form
MULT_V = {"": 1, "2": 2, "4": 4, "19": 19, "38": 38}


def sq_products_fused(D, nsum):
    """(column, a, b) of D * f^2 for inputs that are nsum-sums of carried values: for a wrapped
    pair (i <= j) the 19 goes on f_j (x19, or x38 when that still fits int32), the remaining
    powers of two on f_i; a non-wrapped pair splits its power of two over both operands."""
    def fits(idx, m):
        return MULT_V[m] * nsum * CARRIED[idx] < 2**31
    cols = {k: [] for k in range(10)}
    need = set()
    pend = []
    for i in range(10):
        for j in range(i, 10):
            k = i + j
            c2 = (1 if i < j else 0) + (1 if (i & 1 and j & 1) else 0) + (1 if D == 2 else 0)
            if k >= 10:
                if c2 >= 1 and fits(j, "38"):
                    a, b = ("x%s" % ["", "2", "4"][c2 - 1], i), ("x38", j)
                else:
                    a, b = ("x%s" % ["", "2", "4"][c2], i), ("x19", j)
                assert fits(a[1], a[0][1:]) and fits(b[1], b[0][1:]), (D, i, j)
                cols[k % 10].append((a, b))
                need.update(x for x in (a, b) if x[0] != "x")
            else:
                pend.append((i, j, k, c2))
    for i, j, k, c2 in pend:
        best = None
        for ma in range(3):
            mb = c2 - ma
            if not 0 <= mb <= 2:
                continue
            a, b = ("x%s" % ["", "2", "4"][ma], i), ("x%s" % ["", "2", "4"][mb], j)
            if not (fits(i, a[0][1:]) and fits(j, b[0][1:])):
                continue
            extra = sum(1 for x in (a, b) if x[0] != "x" and x not in need)
            key = (extra, -ma)
            if best is None or key < best[0]:
                best = (key, a, b)
        _, a, b = best
        cols[k].append((a, b))
        need.update(x for x in (a, b) if x[0] != "x")
    return cols


def check_bounds(cols, nsum_a, nsum_b):
    """Every pre-multiplied operand inside int32 and every column (with the column constant and
    the incoming carry) inside int64, for operands that are nsum-sums of carried values."""
    worst = 0
    for k in range(10):
        tot = 2**50 + 2**40
        for a, b in cols[k]:
            va = MULT_V[a[0][1:]] * nsum_a * CARRIED[a[1]]
            vb = MULT_V[b[0][1:]] * nsum_b * CARRIED[b[1]]
            assert va < 2**31 and vb < 2**31, (a, b)
            tot += va * vb
        worst = max(worst, tot)
    assert worst < 2**62.5, worst
    return worst


def fused_nodes(cols):
    """Instruction DAG of the fused sum: mads ('m', k, r), carries ('c', k) = H_k >> s_k for
    k = 0..8, adds ('a', k) H_k += c_{k-1} for odd k."""
    nodes, deps = [], {}
    for k in range(10):
        for r in range(len(cols[k])):
            n = ("m", k, r)
            nodes.append(n)
            d = []
            if r > 0:
                d.append(("m", k, r - 1))
            elif k % 2 == 0 and k > 0:
                d.append(("c", k - 1))
            deps[n] = d
    for k in range(10):
        last = ("m", k, len(cols[k]) - 1)
        if k % 2 == 1:
            nodes.append(("a", k))
            deps[("a", k)] = [last, ("c", k - 1)]
        if k < 9:
            nodes.append(("c", k))
            deps[("c", k)] = [("a", k)] if k % 2 == 1 else [last]
    return nodes, deps


def list_schedule(nodes, deps, min_dist=2):
    """Greedy list schedule: critical path first, among instructions whose inputs were issued at
    least min_dist slots earlier; if none is, the one whose inputs are oldest."""
    succ = {n: [] for n in nodes}
    for n, d in deps.items():
        for x in d:
            succ[x].append(n)
    crit = {}
    def cp(n):
        if n not in crit:
            crit[n] = 1 + max((cp(s) for s in succ[n]), default=0)
        return crit[n]
    for n in nodes:
        cp(n)
    issued, order = {}, []
    left = set(nodes)
    while left:
        slot = len(order)
        ready = [n for n in left if all(x in issued for x in deps[n])]
        def dist(n):
            return min((slot - issued[x] for x in deps[n]), default=99)
        strict = [n for n in ready if dist(n) >= min_dist]
        pick = max(strict, key=lambda n: (crit[n], -nodes.index(n))) if strict else \
            max(ready, key=lambda n: (dist(n), crit[n]))
        issued[pick] = slot
        order.append(pick)
        left.remove(pick)
    return order


def emit_fused(fn_sig, cols, inputs, doc):
    nodes, deps = fused_nodes(cols)
    order = list_schedule(nodes, deps)
    idx = {}
    outs = ['"=&v"(H[%d])' % k for k in range(10)] + ['"=&v"(t0)', '"=&v"(t1)']
    ins = []
    for op in inputs:
        idx[op] = 12 + len(ins)
        ins.append('"v"(%s[%d])' % op)
    i_b0 = 12 + len(ins); ins.append('"s"(b0)')
    i_b50 = 12 + len(ins); ins.append('"s"(b50)')
    tmp = lambda k: "%%%d" % (10 + (k % 2))
    lines, host = [], []
    for n in order:
        if n[0] == "m":
            _, k, r = n
            a, b = cols[k][r]
            if r > 0:
                add, hadd = "%%%d" % k, "H[%d]" % k
            elif k == 0:
                add, hadd = "%%%d" % i_b0, "b0"
            elif k % 2 == 1:
                add, hadd = ("%%%d" % i_b50, "b50") if k < 9 else ("0", "0")
            else:
                add, hadd = tmp(k - 1), "t%d" % ((k - 1) % 2)
            lines.append("v_mad_i64_i32 %%%d, vcc, %%%d, %%%d, %s" % (k, idx[a], idx[b], add))
            host.append("  H[%d] = %s + (int64_t)%s[%d] * (int64_t)%s[%d];" % (k, hadd, a[0], a[1], b[0], b[1]))
        elif n[0] == "c":
            k = n[1]
            lines.append("v_ashrrev_i64 %s, %d, %%%d" % (tmp(k), S[k], k))
            host.append("  t%d = H[%d] >> %d;" % (k % 2, k, S[k]))
        else:
            k = n[1]
            lines.append("v_lshl_add_u64 %%%d, %s, 0, %%%d" % (k, tmp(k - 1), k))
            host.append("  H[%d] += t%d;" % (k, (k - 1) % 2))
    asm = "\n".join('      "%s\\n"' % l for l in lines)
    return """%s
%s {
  const int64_t b0 = (int64_t)1 << 25, b50 = (int64_t)1 << 50;  // column constants (fe_fused_fin)
  int64_t t0, t1;
#if defined(__HIP_DEVICE_COMPILE__)
  asm(
%s
      : %s
      : %s
      : "vcc");
#else
%s
#endif
}
""" % (doc, fn_sig, asm, ",\n        ".join(", ".join(outs[i:i + 6]) for i in range(0, len(outs), 6)),
       ",\n        ".join(", ".join(ins[i:i + 6]) for i in range(0, len(ins), 6)), "\n".join(host))


def emit_fused_multi(fn_sig, ops, doc, min_dist=3):
    """Several independent fused sums in ONE schedule (ops: [(cols, inputs, prefix)]): with two
    chains interleaved every dependent pair of instructions is >= 3 slots apart (the
    dependent-mad probe: distance <= 2 costs ~5 % per mad, >= 3 nothing)."""
    nodes, deps = [], {}
    for o, (cols, _, _) in enumerate(ops):
        n1, d1 = fused_nodes(cols)
        tag = lambda n: (o,) + n
        nodes += [tag(n) for n in n1]
        for n, d in d1.items():
            deps[tag(n)] = [tag(x) for x in d]
    order = list_schedule(nodes, deps, min_dist)
    outs, ins, idx = [], [], {}
    for o, (cols, inputs, pre) in enumerate(ops):
        outs += ['"=&v"(H%d[%d])' % (o, k) for k in range(10)] + ['"=&v"(t%d_0)' % o, '"=&v"(t%d_1)' % o]
    nout = len(outs)
    for o, (cols, inputs, pre) in enumerate(ops):
        for op in inputs:
            idx[(o, op)] = nout + len(ins)
            ins.append('"v"(%s%s[%d])' % (pre, op[0], op[1]))
    i_b0 = nout + len(ins); ins.append('"s"(b0)')
    i_b50 = nout + len(ins); ins.append('"s"(b50)')
    H = lambda o, k: "%%%d" % (12 * o + k)
    T = lambda o, k: "%%%d" % (12 * o + 10 + (k % 2))
    lines, host = [], []
    for n in order:
        o, kind = n[0], n[1]
        cols, inputs, pre = ops[o]
        if kind == "m":
            k, r = n[2], n[3]
            a, b = cols[k][r]
            if r > 0:
                add, hadd = H(o, k), "H%d[%d]" % (o, k)
            elif k == 0:
                add, hadd = "%%%d" % i_b0, "b0"
            elif k % 2 == 1:
                add, hadd = ("%%%d" % i_b50, "b50") if k < 9 else ("0", "0")
            else:
                add, hadd = T(o, k - 1), "t%d_%d" % (o, (k - 1) % 2)
            lines.append("v_mad_i64_i32 %s, vcc, %%%d, %%%d, %s" % (H(o, k), idx[(o, a)], idx[(o, b)], add))
            host.append("  H%d[%d] = %s + (int64_t)%s%s[%d] * (int64_t)%s%s[%d];"
                        % (o, k, hadd, pre, a[0], a[1], pre, b[0], b[1]))
        elif kind == "c":
            k = n[2]
            lines.append("v_ashrrev_i64 %s, %d, %s" % (T(o, k), S[k], H(o, k)))
            host.append("  t%d_%d = H%d[%d] >> %d;" % (o, k % 2, o, k, S[k]))
        else:
            k = n[2]
            lines.append("v_lshl_add_u64 %s, %s, 0, %s" % (H(o, k), T(o, k - 1), H(o, k)))
            host.append("  H%d[%d] += t%d_%d;" % (o, k, o, (k - 1) % 2))
    asm = "\n".join('      "%s\\n"' % l for l in lines)
    temps = ", ".join("t%d_0, t%d_1" % (o, o) for o in range(len(ops)))
    return """%s
%s {
  const int64_t b0 = (int64_t)1 << 25, b50 = (int64_t)1 << 50;  // column constants (fe_fused_fin)
  int64_t %s;
#if defined(__HIP_DEVICE_COMPILE__)
  asm(
%s
      : %s
      : %s
      : "vcc");
#else
%s
#endif
}
""" % (doc, fn_sig, temps, asm, ",\n        ".join(", ".join(outs[i:i + 6]) for i in range(0, len(outs), 6)),
       ",\n        ".join(", ".join(ins[i:i + 6]) for i in range(0, len(ins), 6)), "\n".join(host))


def used_inputs(cols, sortkey):
    used = []
    for k in range(10):
        for a, b in cols[k]:
            for op in (a, b):
                if op not in used:
                    used.append(op)
    used.sort(key=sortkey)
    return used


def main():
    parts = ["""// fe_cols.h — GENERATED by tools/gen_fe_asm.py (do not edit): the column sums of the field
// multiplication and squaring of fe25519.h as explicit v_mad_i64_i32 schedules (gfx950).
//
// Each column k of the 64-bit accumulators starts with one mad whose addend is the rounding
// bias of fe_carry64 (2^25 even / 2^24 odd column), then takes the column's remaining products;
// the mads go round-robin over the ten columns, so no mad depends on one of the previous four.
// LLVM, given the same sums in C++, adds the bias with an extra 64-bit v_lshl_add_u64 per
// column (re-association; tools/micro/fe_micro.hip).  The host build compiles the identical
// schedule as C++ (the CPU test-suite's simulation of the kernels).
#pragma once
"""]
    order = schedule(mul_products())
    check_distance(order)
    ins = [("f", i) for i in range(10)] + [("f2", i) for i in (1, 3, 5, 7, 9)] + \
          [("g", j) for j in range(10)] + [("g19", j) for j in range(1, 10)]
    parts.append(emit("TMED_HD void fe_mul_cols(int64_t acc[10], const int32_t f[10], const int32_t f2[10], "
                      "const int32_t g[10], const int32_t g19[10])", order, ins,
                      "// acc[k] = bias_k + sum_{i+j = k mod 10} f_i g_j (x2 odd-odd, x19 wrapped): 100 mads"))
    for D in (1, 2):
        cols = sq_products(D)
        order = schedule(cols)
        check_distance(order)
        used = []
        for k, r, (a, b) in order:
            for op in (a, b):
                if op not in used:
                    used.append(op)
        used.sort(key=lambda o: (MULT.index(o[0][1:]), o[1]))
        parts.append(emit("TMED_HD void fe_sq%d_cols(int64_t acc[10], const int32_t x[10], const int32_t x2[10], "
                          "const int32_t x4[10], const int32_t x19[10], const int32_t x38[10])" % D, order, used,
                          "// acc[k] = bias_k + the column sums of %s: 55 mads" % ("f^2" if D == 1 else "2 f^2")))
    parts.append('''
// ---- fused forms (the default; fe25519.h "Fused carry"): the column sums AND the carry chain up
// to column 9 in one schedule.  H[0] is column 0 before the wrap, H[1..9] are final; fe_fused_fin
// does the x19 wrap and extracts the limbs.''')
    check_bounds({k: [(("x" + a[0][1:], a[1]), ("x" + b[0][1:], b[1])) for a, b in v]
                  for k, v in mul_products().items()}, 3, 3)
    cols = mul_products()
    ins = [("f", i) for i in range(10)] + [("f2", i) for i in (1, 3, 5, 7, 9)] + \
          [("g", j) for j in range(10)] + [("g19", j) for j in range(1, 10)]
    parts.append(emit_fused("TMED_HD void fe_mul_fused(int64_t H[10], const int32_t f[10], const int32_t f2[10], "
                            "const int32_t g[10], const int32_t g19[10])", cols, ins,
                            "// f * g: 100 mads, 9 carries, 5 adds"))
    for D, nsum in ((1, 3), (2, 1)):
        cols = sq_products_fused(D, nsum)
        check_bounds(cols, nsum, nsum)
        used = used_inputs(cols, lambda o: (["x", "x2", "x4", "x19", "x38"].index(o[0]), o[1]))
        parts.append(emit_fused("TMED_HD void fe_sq%d_fused(int64_t H[10], const int32_t x[10], const int32_t x2[10], "
                                "const int32_t x4[10], const int32_t x19[10], const int32_t x38[10])" % D, cols, used,
                                "// %s (inputs up to %d-sums of carried values): 55 mads, 9 carries, 5 adds; premuls used: %s"
                                % ("f^2" if D == 1 else "2 f^2", nsum,
                                   " ".join("%s[%d]" % o for o in used if o[0] != "x"))))
    parts.append('''
// ---- pairs of independent fused sums in one schedule (the point formulas' independent
// multiplications and squarings): dependent instructions >= 3 slots apart.''')
    mcols = mul_products()
    mins = [("f", i) for i in range(10)] + [("f2", i) for i in (1, 3, 5, 7, 9)] + \
           [("g", j) for j in range(10)] + [("g19", j) for j in range(1, 10)]
    parts.append(emit_fused_multi(
        "TMED_HD void fe_mul_fused_x2(int64_t H0[10], int64_t H1[10], const int32_t a_f[10], const int32_t a_f2[10], "
        "const int32_t a_g[10], const int32_t a_g19[10], const int32_t b_f[10], const int32_t b_f2[10], "
        "const int32_t b_g[10], const int32_t b_g19[10])", [(mcols, mins, "a_"), (mcols, mins, "b_")],
        "// two independent products f * g"))
    sortk = lambda o: (["x", "x2", "x4", "x19", "x38"].index(o[0]), o[1])
    s1 = sq_products_fused(1, 3)
    s2 = sq_products_fused(2, 1)
    psig = "const int32_t %s_x[10], const int32_t %s_x2[10], const int32_t %s_x4[10], const int32_t %s_x19[10], " \
           "const int32_t %s_x38[10]"
    parts.append(emit_fused_multi(
        "TMED_HD void fe_sq1_fused_x2(int64_t H0[10], int64_t H1[10], %s, %s)" % (psig % (("a",) * 5), psig % (("b",) * 5)),
        [(s1, used_inputs(s1, sortk), "a_"), (s1, used_inputs(s1, sortk), "b_")], "// two independent squares"))
    parts.append(emit_fused_multi(
        "TMED_HD void fe_sq2_sq1_fused(int64_t H0[10], int64_t H1[10], %s, %s)" % (psig % (("a",) * 5), psig % (("b",) * 5)),
        [(s2, used_inputs(s2, sortk), "a_"), (s1, used_inputs(s1, sortk), "b_")], "// 2 a^2 (a carried) and b^2"))
    parts.append('''
// ---- squares of CARRIED inputs (one carried value, not a sum: every squaring chain of the
// exponentiations and the X^2, Y^2 of a doubling): with inputs half the size of a 2-sum the 19
// and the factors 2 fit on fewer premultiplied copies — x2 of limbs 0, 1, 2, 3, 5, 7, x19 of 6, 8
// and x38 of 5..9 (13 copies, 5 of them v_mul_lo_u32, against 19 for up-to-3-sum inputs).''')
    s1c = sq_products_fused(1, 1)
    check_bounds(s1c, 1, 1)
    csig = "const int32_t %s_x[10], const int32_t %s_x2[10], const int32_t %s_x19[10], const int32_t %s_x38[10]"
    used_c = used_inputs(s1c, sortk)
    assert all(o[0] in ("x", "x2", "x19", "x38") for o in used_c), used_c
    parts.append(emit_fused("TMED_HD void fe_sq1c_fused(int64_t H[10], const int32_t x[10], const int32_t x2[10], "
                            "const int32_t x19[10], const int32_t x38[10])", s1c, used_c,
                            "// f^2, f carried: 55 mads, 9 carries, 5 adds; premuls used: %s"
                            % " ".join("%s[%d]" % o for o in used_c if o[0] != "x")))
    parts.append(emit_fused_multi(
        "TMED_HD void fe_sq1c_fused_x2(int64_t H0[10], int64_t H1[10], %s, %s)" % (csig % (("a",) * 4), csig % (("b",) * 4)),
        [(s1c, used_c, "a_"), (s1c, used_c, "b_")], "// two independent squares of carried values"))
    with open(OUT, "w") as fh:
        fh.write("\n".join(parts))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
