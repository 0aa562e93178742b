#!/bin/bash
# Same-box A/B of compile-time knobs on the headline bench line: `rounds` alternating passes over the builds named
# on the command line ("default" = the product build; others = librt_hip_<name>.so from `make variant`), each a
# `bench.py --steps 20 --warmup 5` C3 line without companions, CPU baseline or PMC passes.  One line per run in
# gpurun_out/<out>/ab.txt: build, Mray/s, ms per frame, roofline frac.
#   gpurun -- bash scripts/ab_knobs.sh <out> <rounds> <build> [<build> ...]
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$1; rounds=$2; shift 2
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    lv=$v; [ "$v" = default ] && lv=
    RT_LIB_VARIANT=$lv timeout -k 10 120 python3 scripts/with_variant.py bench.py --steps 20 --warmup 5 \
      --no-companions --no-cpu-baseline --traffic off > "$out/$v.$r.json" 2> "$out/$v.$r.err" || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'])" \
      "$out/$v.$r.json" "$v" >> "$out/ab.txt" || exit 1
  done
done
cat "$out/ab.txt"
