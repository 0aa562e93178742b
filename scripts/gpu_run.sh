#!/bin/bash
# One gpurun call, parametrised (replaces round 4's single-use r4_check*.sh wrappers):
#   gpurun -- bash scripts/gpu_run.sh <name> <step> [<step> ...]
# Output goes to gpurun_out/<name>/; the call stops at the first failing step (each step has its own
# time limit; a GPU step that fails, faults or times out ends the call).
#   tests[=<pytest -k expr>]     python -m pytest tests -m gpu -x (optionally -k); testsall: without -x
#   bench[=<bench.py args>]      one bench.py line -> bench<i>.json (default args: the driver's default)
#   r4bench[=<args>]             the same command on the round-4 snapshot in _ab/r4 (same-box A/B)
#   ab=<args>                    bench.py --no-cpu-baseline --traffic off --no-companions <args>: one line
#   r4ab=<args>                  the same on the round-4 snapshot
#   vtests=<variant>:<-k expr>  the GPU tests (-k) against an A/B build
#   vbench=<variant>:<args>      bench.py against the A/B build _build/librt_hip_<variant>.so
#   gbench=<args>                bench.py with RT_BENCH_GATED=1 (the gated launch: the prepass inside k_trace)
#   sim=<batch_shard_sim args>   scripts/batch_shard_sim.py
#   prof=<bench.py args>         rocprofv3 --kernel-trace --stats over bench.py -> prof<i>/
#   smoke                        __graft_entry__.smoke()
#   py=<script and args>         any python script of the repo (diagnostics)
#   pyprof=<script and args>     the same under rocprofv3 --kernel-trace -> prof<i>/
#   vpy=<variant>:<script args>  the same against an A/B build _build/librt_hip_<variant>.so
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
name=$1; shift
out=gpurun_out/$name; mkdir -p "$out"
i=0
summ() {  # one summary line of a bench json
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r, c = d["roofline"], d["config"]
sf = c.get("single_frame", {}); ss = c.get("single_frame_serial", {}); sd = c.get("single_frame_deferred", {}); s2 = c.get("single_frame_deferred2", {})
print("== %-40s %8.2f Mray/s %.4f ms/frame frac %.4f kernel %.3f ms  hbm x%s  sf %s  serial p+s %s  deferred p+s %s / %s" % (
    sys.argv[1][:40], d["value"], d["ms_per_step"], r["frac"], r["kernel_avg_ms"], r.get("traffic_per_frame_vs_rgba8"),
    sf.get("primary_plus_shadow_mrays"), ss.get("primary_plus_shadow_mrays"), sd.get("primary_plus_shadow_mrays"), s2.get("primary_plus_shadow_mrays")))
PY
}
for step in "$@"; do
  i=$((i+1)); kind=${step%%=*}; arg=""; [ "$kind" != "$step" ] && arg=${step#*=}
  echo "[$i] $step"
  case $kind in
    tests|testsall)  # testsall: no -x (every failure of the suite in one call)
      k=(); [ -n "$arg" ] && k=(-k "$arg")
      x=-x; [ $kind = testsall ] && x=
      timeout -k 10 900 python3 -u -m pytest tests -m gpu $x -v --timeout 300 --timeout-method thread "${k[@]}" \
        > "$out/tests$i.log" 2>&1 || { tail -40 "$out/tests$i.log"; exit 1; }
      tail -1 "$out/tests$i.log";;
    vtests|vtestsc)  # vtests=<variant>:<pytest -k expr>: the GPU tests against an A/B build (vtestsc: a test
                     # failure does not end the call; a timeout or crash still does)
      v=${arg%%:*}; k=${arg#*:}
      RT_LIB_VARIANT=$v timeout -k 10 900 python3 -u scripts/with_variant.py -m pytest tests -m gpu -x -v --timeout 300 \
        --timeout-method thread -k "$k" > "$out/tests$i.log" 2>&1; rc=$?
      tail -1 "$out/tests$i.log"
      if [ $rc -ne 0 ] && { [ $kind = vtests ] || [ $rc -ne 1 ]; }; then tail -40 "$out/tests$i.log"; exit 1; fi;;
    bench|r4bench|ab|r4ab)
      dir=.; [ "${kind:0:2}" = r4 ] && dir=_ab/r4
      extra=""; [ "${kind#r4}" = ab ] && extra="--no-cpu-baseline --traffic off --no-companions"
      (cd $dir && timeout -k 10 600 python3 bench.py $extra $arg) > "$out/bench$i.json" 2> "$out/bench$i.err" \
        || { tail -20 "$out/bench$i.err"; exit 1; }
      summ "$step" "$out/bench$i.json";;
    vbench|gbench)  # vbench=<variant>:<bench args> (an A/B build); gbench=<args>: RT_BENCH_GATED=1
      if [ $kind = vbench ]; then v=${arg%%:*}; rest=${arg#*:}; else v=; rest=$arg; fi
      gt=0; [ $kind = gbench ] && gt=1
      RT_BENCH_GATED=$gt RT_LIB_VARIANT=$v timeout -k 10 600 python3 scripts/with_variant.py bench.py $rest \
        > "$out/bench$i.json" 2> "$out/bench$i.err" || { tail -20 "$out/bench$i.err"; exit 1; }
      summ "$step" "$out/bench$i.json";;
    sim)
      timeout -k 10 600 python3 scripts/batch_shard_sim.py $arg > "$out/sim$i.log" 2>&1 || { tail -20 "$out/sim$i.log"; exit 1; }
      tail -5 "$out/sim$i.log";;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$out/prof$i" \
        -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --traffic off --no-companions $arg) \
        > "$out/prof$i.log" 2>&1 || { tail -20 "$out/prof$i.log"; exit 1; }
      tail -1 "$out/prof$i.log";;
    pyprof)  # pyprof=<script and args>: rocprofv3 --kernel-trace over a python script of the repo -> prof<i>/
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$out/prof$i" \
        -o run -- python3 $GRAFT_REPO_ROOT/$arg) > "$out/prof$i.log" 2>&1 || { tail -20 "$out/prof$i.log"; exit 1; }
      tail -3 "$out/prof$i.log";;
    py)
      timeout -k 10 600 python3 $arg > "$out/py$i.log" 2>&1 || { tail -20 "$out/py$i.log"; exit 1; }
      tail -5 "$out/py$i.log";;
    vpy)  # vpy=<variant>:<script and args>: the script against _build/librt_hip_<variant>.so (with_variant.py)
      v=${arg%%:*}; rest=${arg#*:}
      RT_LIB_VARIANT=$v timeout -k 10 600 python3 scripts/with_variant.py $rest > "$out/py$i.log" 2>&1 \
        || { tail -20 "$out/py$i.log"; exit 1; }
      tail -5 "$out/py$i.log";;
    smoke)  # __graft_entry__.smoke() (the driver's round-end smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke$i.log" 2>&1 \
        || { tail -20 "$out/smoke$i.log"; exit 1; }
      tail -2 "$out/smoke$i.log";;
    *) echo "unknown step $step"; exit 2;;
  esac
done
