#!/bin/bash
# Collect PMC counters for tools/opbench.py cases, one rocprofv3 invocation per counter pass.
# usage: tools/pmc_passes.sh OUTDIR <tools/opbench.py arguments, e.g. --only conv3_l0_320 --plans auto>
set -e
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $line --kernel-trace --output-format csv -d "$OUT/p$i" -o pmc \
    -- python3 tools/opbench.py --iters 3 "$@" > "$OUT/p$i.log" 2>&1
done <<'PASSES'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU
SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum
TA_BUSY_avr TA_BUFFER_LOAD_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
FETCH_SIZE
WRITE_SIZE
PASSES
