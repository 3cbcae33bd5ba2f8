#!/bin/bash
# round 5: SQ counter passes over the LP = 512 split Gram and split panel product (tools/wide_lab)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r5o
mkdir -p $out
cd /tmp
for what in gsplit psplit; do
  LAB_LP=512 timeout -k 10 60 $R/tools/wide_lab $what > $out/$what.txt 2>&1 || { cat $out/$what.txt; exit 1; }
  cat $out/$what.txt
  LAB_LP=512 timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out/${what}_p1 -o run -- $R/tools/wide_lab $what > $out/${what}_p1.log 2>&1 || { tail -5 $out/${what}_p1.log; exit 1; }
  LAB_LP=512 timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_MFMA --output-format csv -d $out/${what}_p2 -o run -- $R/tools/wide_lab $what > $out/${what}_p2.log 2>&1 || { tail -5 $out/${what}_p2.log; exit 1; }
  python3 $R/tools/pmc_summary.py $out/${what}_p1 > $out/${what}_pmc.txt && python3 $R/tools/pmc_summary.py $out/${what}_p2 >> $out/${what}_pmc.txt
  cat $out/${what}_pmc.txt
done
