# round-3: instruction-cache behaviour of the codec kernels (config 2, 131,072 pieces)
export TMPDIR=/tmp
mkdir -p gpurun_out/r3z_ic
timeout -k 10 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQ_IFETCH SQ_WAVES -d gpurun_out/r3z_ic/p1 -o p1 --output-format csv -- python3 tools/prof_run.py 2 131072 2 > gpurun_out/r3z_ic/p1.log 2>&1 && \
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/r3z_ic/p1/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-30:]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    if m.get("SQ_WAVES", 0) < 100: continue
    print(k, {c: "%.4g" % v for c, v in sorted(m.items())},
          "miss rate %.2f %%" % (100 * m.get("SQC_ICACHE_MISSES", 0) / max(m.get("SQC_ICACHE_REQ", 1), 1)))
PY
