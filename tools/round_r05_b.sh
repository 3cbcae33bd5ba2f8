#!/bin/bash
# Round-5 PMC evidence: FETCH_SIZE and WRITE_SIZE passes (separate runs: they cannot share one) and
# an MFMA-busy pass for C4, C5, C3, with RSVD_COOP=0 (plain launches of the persistent kernels: the
# projection and QR kernels these files describe launch the same way on either path, and the
# process then exits cleanly, so the passes can share one call).  The C4 MFMA pass on the
# cooperative path runs last: the process exits 139 after the counters are written.
# Usage: tools/round_r05_b.sh <tag>
set -o pipefail
tag=${1:-r05_v2}
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in c4 c5 c3; do
  out=$R/gpurun_out/prof_${tag}_$c
  mkdir -p $out
  for pass in fetch write mfma; do
    case $pass in
      fetch) ctr="FETCH_SIZE"; st=3 ;;
      write) ctr="WRITE_SIZE"; st=3 ;;
      mfma) ctr="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; st=1 ;;
    esac
    (cd /tmp && RSVD_COOP=0 timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $out/$pass -o run -- python3 $R/bench.py --config $c --steps $st --warmup 1 --cpu-budget 0 > $out/$pass.log 2>&1) || { echo "$c $pass failed"; tail -5 $out/$pass.log; exit 1; }
    echo "$c $pass ok"
  done
done
out=$R/gpurun_out/prof_${tag}_c4coop
mkdir -p $out
cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $out/mfma -o run -- python3 $R/bench.py --config c4 --steps 1 --warmup 1 --cpu-budget 0 > $out/mfma.log 2>&1
echo "c4 MFMA pass, cooperative path: rc=$? (139 = the known exit-time fault after the counters are written)"
ls $out/mfma
