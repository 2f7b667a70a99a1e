#!/bin/bash
# rocprofv3 passes over a command (GPU box): kernel trace + stats, then PMC
# passes, one counter group per run (MI355X_MICROARCH.md: FETCH_SIZE and
# WRITE_SIZE cannot share a pass).
# usage: tools/profile.sh TAG [sq] -- python3 script.py args...
TAG=$1; shift
SQ=0
if [ "$1" = "sq" ]; then SQ=1; shift; fi
[ "$1" = "--" ] && shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, seconds, rocprofv3 args...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 $secs rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- "${CMD[@]}" > $OUT/$name.log 2>&1
  local rc=$?
  tail -2 $OUT/$name.log
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; exit $rc; fi
}
CMD=("$@")
run trace 300 --kernel-trace --stats
run fetch 300 --pmc FETCH_SIZE
run write 300 --pmc WRITE_SIZE
if [ $SQ = 1 ]; then
  run sq1 300 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
  run sq2 300 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES
  # (the effective clock: GRBM_GUI_ACTIVE / 8 XCDs / kernel time, MI355X_MICROARCH.md DVFS)
  run sq3 300 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES
fi
echo "profile done"
