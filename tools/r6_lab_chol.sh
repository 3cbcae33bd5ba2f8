#!/bin/bash
# round 6: the Cholesky lab (tools/wide_lab_cprof, built by tools/build_cprof.sh): the 16 x 16 diagonal
# factor's cycles (DPP / v2 / pipelined v3, bit-identity against the DPP form) and the leaf timings.
set -o pipefail
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6lab}
mkdir -p $out
timeout -k 10 120 $GRAFT_REPO_ROOT/tools/wide_lab_cprof chol > $out/chol.txt 2>&1 || { tail -20 $out/chol.txt; exit 1; }
grep -v "^$" $out/chol.txt | head -20
