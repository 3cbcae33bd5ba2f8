#!/bin/bash
# tools/wide_lab_cprof: tools/wide_lab with the Cholesky phase timers and the 16 x 16 diagonal-factor
# bench (RSVD_CHOL_PROF) compiled in.  Run after `make -C rsvd_kamaneh_raganato_terrana_amd/csrc all`.
set -e
cd "$(dirname "$0")/../rsvd_kamaneh_raganato_terrana_amd/csrc"
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-result -DRSVD_CHOL_PROF -DRSVD_LAB"
T=$(mktemp -d)
/opt/rocm/bin/hipcc $F -c wide_qr.hip -o $T/wide_qr.o
/opt/rocm/bin/hipcc $F -I. -c ../../tools/wide_lab.cpp -o $T/wide_lab.o
O=../../build/obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -o ../../tools/wide_lab_cprof $T/wide_lab.o $T/wide_qr.o $O/util.o $O/proj.o \
  $O/qr.o $O/jacobi.o $O/wide_proj.o $O/wide_svd.o $O/wide_eig.o $O/dense.o $O/gemm.o
rm -rf $T
