"""Per-basic-block instruction mix of one kernel in a `hipcc -S` listing: blocks that read the
noise tables (ds_read_b128) are the noise3d bodies.  usage: isa_blocks.py file.s kernel-prefix"""
import collections
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(sys.argv[2]) and l.rstrip().endswith(tuple(":;@")) or
             (l.startswith(sys.argv[2]) and ": ;" in l))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
blocks, cur = [], None
for l in lines[start:end]:
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        cur = [m.group(1), []]
        blocks.append(cur)
        continue
    s = l.strip()
    if cur is not None and l.startswith("\t") and s and not s.startswith((".", ";")):
        cur[1].append(s.split()[0])
tot = collections.Counter()
for name, ins in blocks:
    c = collections.Counter(ins)
    tot.update(c)
    if c["ds_read_b128"] >= 4:
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        trans = sum(c[k] for k in c if re.match(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)_f32", k))
        print(f"{name}: {len(ins)} instrs, VALU {valu} (pk {sum(v for k, v in c.items() if k.startswith('v_pk_'))}, "
              f"mov {c['v_mov_b32'] + c['v_mov_b64']}, trans {trans}), ds_read {sum(v for k, v in c.items() if k.startswith('ds_read'))}, "
              f"scratch {sum(v for k, v in c.items() if k.startswith('scratch_'))}, salu {sum(v for k, v in c.items() if k.startswith('s_'))}")
print("kernel total", sum(tot.values()), "scratch ops", sum(v for k, v in tot.items() if k.startswith("scratch_")))
