#!/usr/bin/env python3
"""Issue cost of each loop of a kernel in a `hipcc -S` listing, split into its octave bodies (blocks
with >= 4 ds_read_b128: the noise lattice) and the rest, using the gfx950 issue costs of
profiles/r02/ubench_cost_model.md (2.3 cycles full-rate FP32/int, 4.3 packed / conversions / perm /
64-bit, 8 transcendental).  Loop membership from LLVM's `; in Loop: Header=...` annotations; a loop's
own numbers exclude its inner loops.  Static counts: every block once (both sides of each branch).

  hipcc --offload-arch=gfx950 -O3 ... --cuda-device-only -S rt_kernels.hip -o k.s
  python3 scripts/loop_costs.py k.s _ZN12_GLOBAL__N_17k_traceILi0ELb0EE"""
import collections
import re
import sys

TWO = re.compile(r"v_(add|sub|mul|fma|fmac|fmamk|fmaak|max|min)_f32|v_(and|or|xor|add|sub)_(b32|u32|co_u32)|v_cmp|"
                 r"v_mov_b32|v_cndmask")
EIGHT = re.compile(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)_f32")


def cost(op):
    if EIGHT.match(op):
        return 8.0
    if TWO.match(op) and not op.startswith("v_pk"):
        return 2.3
    return 4.3


def main(path, prefix):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(prefix) and l.rstrip().endswith(":") or
                 (l.startswith(prefix) and ": ;" in l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur = [], None
    for l in lines[start:end]:
        m = re.match(r"^(\.LBB\w+|; %bb\.\d+):(.*)$", l)
        if m:
            cur = {"name": m.group(1), "ann": m.group(2), "ins": []}
            blocks.append(cur)
            continue
        if cur is None:
            continue
        st = l.strip()
        if st.startswith(";") and "Loop" in st:
            cur["ann"] += " " + st
        elif l.startswith("\t") and st and not st.startswith((".", ";")):
            cur["ins"].append(st.split()[0])
    parent, agg = {}, collections.defaultdict(lambda: collections.Counter())
    for b in blocks:
        a = b["ann"]
        if "Loop Header" in a:
            loop = b["name"].replace(".LBB", "")
            ps = re.findall(r"Parent Loop BB(\d+_\d+)", a)
            parent[loop] = ps[-1] if ps else None
        else:
            m = re.search(r"in Loop: Header=BB(\d+_\d+)", a)
            loop = m.group(1) if m else "-"
        v = [i for i in b["ins"] if i.startswith("v_")]
        body = sum(1 for i in b["ins"] if i == "ds_read_b128") >= 4
        key = "octave body" if body else "rest"
        agg[loop][key + " VALU"] += len(v)
        agg[loop][key + " cycles"] += sum(cost(i) for i in v)
        agg[loop]["blocks"] += 1
        for i in b["ins"]:
            if i.startswith("s_setprio"):
                agg[loop]["setprio"] += 1
            if i.startswith("ds_bpermute"):
                agg[loop]["bpermute"] += 1
            if i.startswith("v_exp_f32") or i.startswith("v_log_f32"):
                agg[loop]["exp/log"] += 1
    for loop in sorted(agg, key=lambda x: (x == "-", x)):
        c = agg[loop]
        print(f"loop {loop:8s} parent {str(parent.get(loop)):8s} blocks {c['blocks']:4d}  rest {c['rest VALU']:5d} VALU "
              f"{c['rest cycles']:7.0f} cyc  octave bodies {c['octave body VALU']:4d} VALU {c['octave body cycles']:6.0f} cyc"
              f"  setprio {c['setprio']} bpermute {c['bpermute']} exp/log {c['exp/log']}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
