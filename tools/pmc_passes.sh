#!/bin/bash
# PMC passes over one census forward (each pass its own rocprofv3 run; no tracing domains
# mixed with --pmc). Usage (on the GPU box): bash tools/pmc_passes.sh OUTDIR [census args]
OUT=${1:-gpurun_out/pmc}; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum TCC_MISS_sum"
P4="FETCH_SIZE"
P5="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- python3 tools/census.py --reps 1 "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo pmc_done
