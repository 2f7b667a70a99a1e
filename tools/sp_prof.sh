#!/bin/bash
# SQ counter passes of the encoders on 65,536 config-2 pieces (GPU box):
#   tools/sp_prof.sh TAG lib.so@0 [lib.so@4 ...]
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
export QB_N=${QB_N:-65536} QB_CFG=${QB_CFG:-2}
run() {
  local name=$1; shift
  timeout -k 10 120 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 tools/quick_bench.py "${LIBS[@]}" > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -5 $OUT/$name.log; exit 1; }
}
LIBS=("$@")
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
run sq2 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES
python3 tools/pmc_summary.py $OUT
