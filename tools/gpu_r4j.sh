set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4j
for v in 1 3; do
  RSVD_GSPLIT_LG=$v timeout -k 10 120 tools/wide_lab gsplit > gpurun_out/r4j/gsplit_$v.txt 2>&1 || { cat gpurun_out/r4j/gsplit_$v.txt; exit 1; }
  echo "LG=$v"; grep "LP=128" gpurun_out/r4j/gsplit_$v.txt
done
CFGS="c3" STEPS=20 tools/ab_round.sh r4j "" "RSVD_GSPLIT_LG=3" "RSVD_GSPLIT_LG=1" "RSVD_GSPLIT_LG=3"
