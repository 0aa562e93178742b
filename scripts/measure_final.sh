#!/bin/bash
# One GPU call: the default build's bench lines for BASELINE.md's table: C1, C2, C5 (their own
# configs), the driver's command (--steps 20 --warmup 5) and 96 frames, under gpurun_out/final_cfg/.
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/final_cfg; mkdir -p $O
run() { local name=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -20 $O/$name.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'], d['roofline']['frac'])"
}
run c1 --config c1 && run c2 --config c2 && run c5 --config c5 --cpu-row-step 16 && \
run driver --steps 20 --warmup 5 && run f96 --steps 96 --warmup 12 --no-companions --no-cpu-baseline
