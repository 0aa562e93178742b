cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c22
for c in WRITE_SIZE FETCH_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r4c22/$c -o run -- ./scripts/_build/ubench_atomic > gpurun_out/r4c22/$c.log 2>&1 || { tail -5 gpurun_out/r4c22/$c.log; exit 1; }
  python3 - gpurun_out/r4c22/$c <<'PY'
import csv, glob, sys, collections
v = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_op" in r["Kernel_Name"]:
            v[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
for i, d in enumerate(sorted(v)):
    print(sys.argv[1].split("/")[-1], "launch", i, "%.2f MiB" % (v[d] / 1024.0))
PY
done
cat gpurun_out/r4c22/WRITE_SIZE.log | grep launch
