#!/bin/bash
# SQ stall breakdown of the narrow-engine kernels (kernel_lab, C2 shapes): one rocprofv3 --pmc pass.
set -o pipefail
mkdir -p gpurun_out/pmc_lab
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM --output-format csv -d gpurun_out/pmc_lab -o pmc -- tools/kernel_lab 4096 4096 64 > gpurun_out/pmc_lab/lab.log 2>&1
