#!/bin/bash
# Two SQ counter passes (instruction mix, LDS) over a command, one directory
# per tag, then the per-kernel averages (GPU box):
#   tools/pmc_sq.sh TAG KERNEL_SUBSTRING -- python3 script.py args...
TAG=$1; KSUB=$2; shift 2
[ "$1" = "--" ] && shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  -d $OUT/sq1 -o sq1 --output-format csv -- "$@" > $OUT/sq1.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES \
  -d $OUT/sq2 -o sq2 --output-format csv -- "$@" > $OUT/sq2.log 2>&1 || exit $?
python3 - "$OUT" "$KSUB" <<'PY'
import csv, collections, glob, sys
out, ksub = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(float); cnt = collections.Counter()
for f in glob.glob(out + "/sq*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if ksub not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
print(out, {c: "%.4g" % (v / cnt[c]) for c, v in sorted(agg.items())})
PY
