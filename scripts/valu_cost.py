"""Issue cycles per wave on one SIMD of a basic block in a `hipcc -S` listing, with the gfx950
issue costs measured by scripts/ubench_issue.hip (4 waves per SIMD, independent chains):
2 cycles for FP32 add/mul/fma/fmac/fmamk and v_and/v_add_u32/v_sub_u32/v_cmp/v_mov, 4 for packed FP32,
floor/fract/cvt, perm, shifts, 3-operand integer ops and 64-bit mads, 8 for transcendentals.
usage: valu_cost.py file.s kernel-prefix label [label ...]"""
import collections
import re
import sys

TWO = re.compile(r"v_(add|sub|mul|fma|fmac|fmamk|fmaak|max|min)_f32|v_(and|or|xor|add|sub)_(b32|u32|co_u32)|v_cmp|v_mov_b32|v_cndmask")
EIGHT = re.compile(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)_f32")


def cost(op):
    if EIGHT.match(op):
        return 8
    if TWO.match(op) and not op.startswith("v_pk"):
        return 2
    return 4


def block(lines, kernel, label):
    out, on, inside = [], False, False
    for l in lines:
        if l.startswith(kernel) and ":" in l:
            inside = True
        if inside and l.startswith(label + ":"):
            on = True
            continue
        if on:
            s = l.strip()
            if s.startswith(".LBB") or s.startswith("s_cbranch"):
                break
            if s and not s.startswith((";", ".")):
                out.append(s.split()[0])
    return out


lines = open(sys.argv[1]).read().split("\n")
for lab in sys.argv[3:]:
    ins = block(lines, sys.argv[2], lab)
    v = [o for o in ins if o.startswith("v_")]
    c = collections.Counter(cost(o) for o in v)
    print(f"{lab}: {len(v)} VALU, issue cycles {sum(cost(o) for o in v)} (2-cycle {c[2]}, 4-cycle {c[4]}, 8-cycle {c[8]}); "
          f"LDS {sum(1 for o in ins if o.startswith('ds_'))}")
    print("   4-cycle ops:", dict(collections.Counter(o for o in v if cost(o) == 4)))
